#!/bin/bash
# A/B of liborbamd variants (tools/build_variant.sh) on the GPU box: parity tests of the extraction
# per variant, then interleaved bench runs (4 graphs x 256 frames) and a serial one-graph run whose
# stage timings are the kernels alone. usage: [AB_ARGS="--config c4"] tools/ab.sh "<test selector>" v1 v2 ...
sel=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  ORBAMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $sel \
    > gpurun_out/ab_test_$v.log 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -n 1 gpurun_out/ab_test_$v.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi  # a variant with broken parity is not timed
done
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match")))'
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in "$@"; do
    out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 120 python bench.py --sustain 0 --no-cpu --steps 30 ${AB_ARGS} | python -c "$summ") || exit $?
    echo "r$r $v overlapped: $out"
  done
done
for v in "$@"; do
  out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 120 python bench.py --sustain 0 --no-cpu --steps 30 ${AB_ARGS} --pipes 1 --batch 256 --serial-stages | python -c "$summ") || exit $?
  echo "$v serial-1graph: $out"
done
