#!/bin/bash
# round 4: the vocabulary's HIP stream created at its first host transform instead of at orbv_create: parity of the
# host and device transforms, the exchange-object / no-exchange-object step rates (tools/exp_host_issue.py), and C2
# bench lines with and without the exchange
export TMPDIR=/tmp
T=r04vs
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_vocabulary.py tests/test_gpu_cache.py tests/test_gpu_schedule.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
for c in A B; do
  XCFG=$c timeout -k 10 200 python -u tools/exp_host_issue.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${T}_host_issue.log || exit $?
done
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s.get("exchange", 0.0), "sustained=%.0f" % (d.get("sustained") or {}).get("frames_per_s", 0))'
for r in 1 2; do
  for v in full none; do
    a=""; [ $v = none ] && a="--no-exchange"
    out=$(timeout -k 10 180 python bench.py --no-cpu $a 2>/dev/null | python -c "$summ") || exit $?
    echo "r$r $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
out=$(timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu 2>/dev/null | python -c "$summ") || exit $?
echo "driver-args full $out" | tee -a gpurun_out/${T}_bench.log
