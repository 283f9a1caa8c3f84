#!/bin/bash
# A/B of runtime switches of one build: parity tests under each variant's environment, then interleaved
# bench runs. usage: [AB_ARGS="--config c4"] [AB_TESTS="tests/test_gpu_extract.py"] tools/ab_env.sh "ENV=a" "ENV=b" ...
mkdir -p gpurun_out
tests=${AB_TESTS:-"tests/test_gpu_extract.py tests/test_gpu_schedule.py"}
for v in "$@"; do
  tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
  env $v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $tests \
    > gpurun_out/abenv_test_$tag.log 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -n 1 gpurun_out/abenv_test_$tag.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi  # a variant with broken parity is not timed
done
summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], "bit_exact=%s" % d["bit_exact"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match")))'
for r in 1 2 3; do
  for v in "$@"; do
    out=$(env $v timeout -k 10 120 python bench.py --sustain 0 --no-cpu --ingest-steps 0 ${AB_ARGS} | python -c "$summ") || exit $?
    echo "r$r $v: $out"
  done
done
