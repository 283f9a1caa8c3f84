#!/bin/bash
# round 4: the exchange kernels' duration distributions in the bench (kernel trace), k_voc_bow with register-block
# sorts (new) against the previous kernel (old): medians and tails, two runs each, interleaved
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04bd
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export ORBAMD_LIB_VARIANT=old; else unset ORBAMD_LIB_VARIANT; fi
    d=$R/gpurun_out/${T}_${v}_$r
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu --sustain 0 > gpurun_out/${T}_${v}_$r.log 2>&1 || exit $?
    kt=$(find $d -name '*kernel_trace.csv' | head -n 1)
    python3 - "$kt" "$v r$r" <<'PY' | tee -a gpurun_out/${T}.log
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("orbamd::", "")
    if any(k in n for k in ("k_voc", "k_pack_slot", "k_tri_slots", "k_bow_slots", "k_rot_slots")):
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items()):
    v.sort()
    q = lambda p: v[min(len(v) - 1, int(p * len(v)))]
    print("%s %-16s n=%4d median %6.1f p90 %6.1f p99 %7.1f max %7.1f mean %6.1f" % (sys.argv[2], n, len(v), q(.5), q(.9), q(.99), v[-1], sum(v) / len(v)))
PY
    rm -rf $d
  done
done
