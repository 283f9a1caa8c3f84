#!/bin/bash
# round 4: k_voc_bow in 256-thread workgroups (new) against the 1024-thread kernel of HEAD~1 (old): parity, the
# one-keyframe phase trace, the exchange kernels duration distributions in the bench, and bench lines
# (mid: HEAD, 1024 threads with the register-block sorts)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04bt
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_vocabulary.py tests/test_gpu_exchange.py tests/test_gpu_schedule.py" \
  "120 ${T}_bow_trace env ORBAMD_LIB_VARIANT=bowtrace python tools/bow_trace.py" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
grep -v amdgpu gpurun_out/${T}_bow_trace.log
for r in 1 2; do
  for v in new mid old; do
    if [ $v = new ]; then unset ORBAMD_LIB_VARIANT; else export ORBAMD_LIB_VARIANT=$v; fi
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
    grep '^{' gpurun_out/${T}_${v}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print(sys.argv[1], "%.0f" % d["value"], d["bit_exact"], "exchange=%.3f" % d["stage_ms_per_step"]["exchange"])' "$v r$r" | tee -a gpurun_out/${T}.log
  done
done
