#!/bin/bash
# round 4: octree workgroup size for small batches (the one-frame call's octree is on its critical path):
# o256 / o512 / o1024 (shipped); parity of each on the extraction tests, an interleaved latency A/B
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04r
for v in o256 o512 o1024; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
tools/gpu_run.sh \
  "300 ${T}_tests_o256 env ORBAMD_LIB_VARIANT=o256 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py" \
  "300 ${T}_tests_o512 env ORBAMD_LIB_VARIANT=o512 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py" || exit $?
for t in o256 o512; do grep -q "passed" gpurun_out/${T}_tests_$t.log && ! grep -q "failed" gpurun_out/${T}_tests_$t.log || exit 1; done
for r in 1 2 3; do
  for v in o256 o512 o1024; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
done
cut -c1-150 gpurun_out/${T}_latency_ab.log
