#!/bin/bash
# round 4: the one-frame call with the done word written by describe's last workgroup (cur4) against k_call_done (cur2):
# parity (extraction, drop-ins, stereo, schedule), an interleaved latency A/B, the cur4 kernel trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04q
for v in cur2 cur4; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_cpp_dropin.py tests/test_gpu_stereo.py tests/test_gpu_schedule.py" \
  "300 ${T}_latency_kt rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_latency_kt -o run -- tests/cpp/build/bench_latency 200" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
for r in 1 2 3; do
  for v in cur2 cur4; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
done
cut -c1-150 gpurun_out/${T}_latency_ab.log
