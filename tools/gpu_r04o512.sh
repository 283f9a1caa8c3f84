#!/bin/bash
# round 4: the batch octree at 512 threads for geometries whose levels reach > 256 live nodes (C4), so every round
# takes the node-per-thread path (o512) against the previous head (pre512): parity, C4 and C2 bench A/B; then the
# 8-rank gloo rehearsal and the self-launching 2-rank bench
export TMPDIR=/tmp
T=r04o512
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_schedule.py tests/test_cpp_dropin.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], d["bit_exact"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match","exchange")))'
for r in 1 2; do
  for c in c4 c2; do
    for v in pre512 o512; do
      out=$(ORBAMD_LIB_VARIANT=$v timeout -k 10 180 python bench.py --sustain 0 --no-cpu --config $c | python -c "$summ") || exit $?
      echo "r$r $c $v $out" | tee -a gpurun_out/${T}_bench_ab.log
    done
  done
done
tools/gpu_run.sh \
  "400 r04_rehearse_8ranks_gloo tools/rehearse_ranks.sh 8" \
  "300 r04_bench_gpus2_gloo env ORBAMD_DIST_BACKEND=gloo ORBAMD_BENCH_DEVICE=0 python3 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu --batch 512 --pipes 2 --sustain 0" || exit $?
