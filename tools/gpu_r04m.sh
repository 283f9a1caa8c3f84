#!/bin/bash
# round 4: one-frame call A/B -- prev (two queue lists, previous commit), cur (levels 0-1 branch + 14-row blur),
# sq (one queue: pyramid, FAST and octree of every level, 14-row blur, describe), sqr (sq + wave-aggregated octree
# counts in the roots and first rounds); parity of sq / sqr, the sq kernel trace, the octree phase trace with aggregation
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04m
for v in prev cur sq sqr; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
tools/gpu_run.sh \
  "300 ${T}_tests_sq env LD_LIBRARY_PATH=$R/gpurun_out/var_sq ORBAMD_LIB_VARIANT=sq python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_cpp_dropin.py" \
  "300 ${T}_tests_sqr env LD_LIBRARY_PATH=$R/gpurun_out/var_sqr ORBAMD_LIB_VARIANT=sqr python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_schedule.py" \
  "120 ${T}_oct_trace2 env ORBAMD_LIB_VARIANT=octtrace2 python tools/oct_trace.py" \
  "300 ${T}_latency_kt env LD_LIBRARY_PATH=$R/gpurun_out/var_sq rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_latency_kt -o run -- tests/cpp/build/bench_latency 200" || exit $?
for t in sq sqr; do grep -q "passed" gpurun_out/${T}_tests_$t.log && ! grep -q "failed" gpurun_out/${T}_tests_$t.log || exit 1; done
grep -v amdgpu gpurun_out/${T}_oct_trace2.log
for r in 1 2 3; do
  for v in prev cur sq sqr; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
done
cut -c1-140 gpurun_out/${T}_latency_ab.log
