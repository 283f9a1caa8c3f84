#!/bin/bash
# round 4 final evidence on the shipped head (after the BoW register-block sorts): the whole GPU suite + smoke; the kernel trace + PMC passes of the
# bench (tools/prof_round.sh) whose traffic file the bench lines then read; the bench at the driver's arguments
# and at its defaults (C2), C3 and C4 lines; the one-frame / per-call latency rows; the timed region's per-kernel
# averages and the exchange kernels
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04fin
tools/gpu_run.sh \
  "700 ${T}_tests python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread" \
  "200 ${T}_smoke python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q " failed" gpurun_out/${T}_tests.log || exit 1
grep -q "SMOKE OK" gpurun_out/${T}_smoke.log || exit 1
tools/prof_round.sh $T || exit $?
kt=$(find gpurun_out/${T}_kt -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_segments.py "$kt" 10 2 > gpurun_out/${T}_timed_region_kernels.txt || exit $?
python3 - "$kt" > gpurun_out/${T}_exchange_kernels.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    if any(k in n for k in ("k_voc", "k_pack_slot", "k_tri_slots", "k_bow_slots", "k_rot_slots")):
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items()):
    v.sort()
    print("%-60s %5d launches, mean %.1f us, median %.1f us, max %.1f us" % (n, len(v), sum(v) / len(v), v[len(v) // 2], max(v)))
PY
tools/prof_reduce.sh $T
cp gpurun_out/${T}_pmc_traffic.json profiles/pmc_traffic.json || exit 1
tools/gpu_run.sh \
  "300 ${T}_bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_bench python3 bench.py" \
  "300 ${T}_bench_c3 python3 bench.py --config c3 --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_bench_c4 python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_latency tests/cpp/build/bench_latency 2000" || exit $?
