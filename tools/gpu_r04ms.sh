#!/bin/bash
# round 4: C2 bench with the matcher contexts' HIP streams created at their first host call (new) against HEAD's library
# (cold: created at orbm_create, one per graph), interleaved on one box: default arguments (three rounds), driver arguments (two)
export TMPDIR=/tmp
T=r04ms
tools/gpu_run.sh \
  "500 ${T}_tests python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_cache.py tests/test_gpu_projection.py tests/test_gpu_stereo.py tests/test_gpu_exchange.py tests/test_cpp_dropin.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s.get("exchange", 0.0), "sustained=%.0f" % (d.get("sustained") or {}).get("frames_per_s", 0))'
for r in 1 2 3; do
  for v in new cold; do
    if [ $v = new ]; then unset ORBAMD_LIB_VARIANT; else export ORBAMD_LIB_VARIANT=$v; fi
    out=$(timeout -k 10 180 python bench.py --no-cpu 2>/dev/null | python -c "$summ") || exit $?
    echo "r$r default $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
for r in 1 2; do
  for v in new cold; do
    if [ $v = new ]; then unset ORBAMD_LIB_VARIANT; else export ORBAMD_LIB_VARIANT=$v; fi
    out=$(timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu 2>/dev/null | python -c "$summ") || exit $?
    echo "r$r driver-args $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
