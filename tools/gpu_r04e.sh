#!/bin/bash
# round 4: the one-frame host path (level-0 side branch, results written into pinned memory by the kernels)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "600 r04e_tests python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_cpp_dropin.py tests/test_gpu_schedule.py -m gpu -x -v --timeout 240 --timeout-method thread" \
  "300 r04e_latency tests/cpp/build/bench_latency 2000" \
  "300 r04e_latency_kt rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04e_latency_kt -o run -- tests/cpp/build/bench_latency 200"
