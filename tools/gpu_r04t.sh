#!/bin/bash
# round 4: the octree's phase-2 rounds with one thread per node (oct3) against the previous head (oct2):
export TMPDIR=/tmp
# parity (extraction, drop-ins, stereo, schedule, matchers), the per-phase trace, an interleaved latency A/B
R=$GRAFT_REPO_ROOT
T=r04t
for v in oct2 oct3; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_cpp_dropin.py tests/test_gpu_stereo.py tests/test_gpu_schedule.py tests/test_gpu_match.py" \
  "120 ${T}_oct_trace env ORBAMD_LIB_VARIANT=octtrace python tools/oct_trace.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
grep -v amdgpu gpurun_out/${T}_oct_trace.log
for r in 1 2 3; do
  for v in oct2 oct3; do
    LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_latency_ab.log || exit $?
  done
done
cut -c1-150 gpurun_out/${T}_latency_ab.log
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match","exchange")))'
for r in 1 2; do
  for v in oct2 oct3; do
    out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 180 python bench.py --sustain 0 --no-cpu | python -c "$summ") || exit $?
    echo "r$r $v bench $out" | tee -a gpurun_out/${T}_bench_ab.log
  done
done
