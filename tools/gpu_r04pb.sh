#!/bin/bash
# round 4: the batch pyramid in row bands (2 / 4 / 8 bands of 1024 threads per frame) against whole-frame
# workgroups (pb1, shipped): parity of pb4 on the batch tests, then tools/ab.sh-style interleaved bench rounds
export TMPDIR=/tmp
T=r04pb
tools/gpu_run.sh \
  "400 ${T}_tests env ORBAMD_LIB_VARIANT=pb4 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_schedule.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match")))'
for r in 1 2; do
  for v in pb1 pb2 pb4 pb8; do
    out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 180 python bench.py --sustain 0 --no-cpu | python -c "$summ") || exit $?
    echo "r$r $v $out" | tee -a gpurun_out/${T}_ab.log
  done
done
for v in pb1 pb4; do
  out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 180 python bench.py --sustain 0 --no-cpu --pipes 1 --batch 256 --serial-stages | python -c "$summ") || exit $?
  echo "$v serial-1graph $out" | tee -a gpurun_out/${T}_ab.log
done
