#!/bin/bash
# round 4: the one-frame call with the chain on one queue (levels 0-1 branch only) and 14-row blur chunks (cur)
# against the previous commit's two-list form (prev): parity, an interleaved latency A/B, the kernel trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04l
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_cpp_dropin.py tests/test_gpu_stereo.py" \
  "300 ${T}_latency_kt rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_latency_kt -o run -- tests/cpp/build/bench_latency 200" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
for v in prev cur; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
for r in 1 2 3; do
  for v in prev cur; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
done
cat gpurun_out/${T}_latency_ab.log
