#!/bin/bash
# round 4: k_voc_bow with 128-key register blocks in the bitonic sorts and a pipelined normalisation chain:
# parity (vocabulary incl. every sort-block boundary, exchange, schedule, BoW matchers), the phase trace, and
# interleaved C2 bench lines against the previous kernel (variant old)
export TMPDIR=/tmp
T=r04bs2
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_vocabulary.py" \
  "120 ${T}_bow_trace env ORBAMD_LIB_VARIANT=bowtrace python tools/bow_trace.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
grep -v amdgpu gpurun_out/${T}_bow_trace.log
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], "ms/step %.4f" % d["ms_per_step"], "exchange=%.3f" % s["exchange"])'
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export ORBAMD_LIB_VARIANT=old; else unset ORBAMD_LIB_VARIANT; fi
    out=$(timeout -k 10 180 python bench.py --sustain 0 --no-cpu | python -c "$summ") || exit $?
    echo "r$r $v $out" | tee -a gpurun_out/${T}_bench.log
  done
done
