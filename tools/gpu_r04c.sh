#!/bin/bash
# round 4: tests of the changed paths, the BF matcher A/B (pre-expanded operands vs per-workgroup LDS expansion),
# then the L2-residency bound experiment
export TMPDIR=/tmp
tools/gpu_run.sh \
  "600 r04c_tests python -u -m pytest tests/test_gpu_match.py tests/test_gpu_exchange.py tests/test_gpu_schedule.py tests/test_gpu_cache.py tests/test_cpp_dropin.py -m gpu -x -v --timeout 240 --timeout-method thread" || exit $?
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f frames/s" % d["value"], "match-only %.0f pairs/s" % d["match_only_pairs_per_s_per_gpu"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match")))'
for r in 1 2 3; do
  for v in 0 1; do
    out=$(ORBX_BF_PRE=$v timeout -k 10 120 python3 bench.py --no-cpu --sustain 0 --ingest-steps 0 --steps 100 --warmup 10 | python3 -c "$summ") || exit $?
    echo "r$r BF_PRE=$v: $out"
  done
done 2>&1 | tee gpurun_out/r04c_ab_bf_pre.log
tools/exp_l2_bound.sh 2>&1 | tee gpurun_out/r04c_l2_bound.log
