#!/bin/bash
# round 4: full GPU suite on the head, the per-call C++ latency rows, a kernel trace of the one-frame call
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "600 r04d_tests python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread" \
  "300 r04d_latency tests/cpp/build/bench_latency 2000" \
  "300 r04d_latency_kt rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04d_latency_kt -o run -- tests/cpp/build/bench_latency 200"
