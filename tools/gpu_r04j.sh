#!/bin/bash
# round 4: the one-frame call as two queue lists (l0new) vs the previous three-list order (l0old), the hardware
# queue count's effect on the one-frame call and on the batch bench (GPU_MAX_HW_QUEUES, HIP's default 4)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04j
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_cpp_dropin.py" \
  "300 ${T}_latency_kt rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_latency_kt -o run -- tests/cpp/build/bench_latency 200" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
for v in l0old l0new; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
for r in 1 2; do
  for v in l0old l0new; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v q4 /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
  GPU_MAX_HW_QUEUES=8 LD_LIBRARY_PATH=$R/gpurun_out/var_l0new timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r l0new q8 /" >> gpurun_out/${T}_latency_ab.log || exit $?
done
cat gpurun_out/${T}_latency_ab.log
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], "ms/step %.4f" % d["ms_per_step"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match","exchange")))'
for r in 1 2; do
  for q in 4 8 16; do
    out=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python bench.py --sustain 0 --no-cpu | python -c "$summ") || exit $?
    echo "r$r queues=$q $out" | tee -a gpurun_out/${T}_queues_ab.log
  done
done
