#!/bin/bash
# round 4: the octree's count pass keeps each cell's key offset / slot for the gather (one load round and one scan
# fewer), phase 2's children counts in one scan, wave-aggregated root counts (oct2) against the previous head
# (oct1): parity, the per-phase trace, an interleaved latency A/B
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04s
for v in oct1 oct2; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_cpp_dropin.py tests/test_gpu_stereo.py tests/test_gpu_schedule.py" \
  "120 ${T}_oct_trace env ORBAMD_LIB_VARIANT=octtrace python tools/oct_trace.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
grep -v amdgpu gpurun_out/${T}_oct_trace.log
for r in 1 2 3; do
  for v in oct1 oct2; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
done
cut -c1-150 gpurun_out/${T}_latency_ab.log
