#!/bin/bash
# round 4: the one-frame capture order (chain first), the chained pyramid (k_pyramid_chain), the vocabulary in child-slot order, k_voc_bow at 1024
# threads, the LDS-staged slot SearchByBoW -- parity (BoW, exchange, extraction), the one-frame latency rows,
# a bench line and its exchange kernels
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04i
tools/gpu_run.sh \
  "400 ${T}_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_vocabulary.py tests/test_gpu_exchange.py tests/test_gpu_extract.py tests/test_gpu_cache.py tests/test_cpp_dropin.py" \
  "300 ${T}_latency tests/cpp/build/bench_latency 2000" \
  "300 ${T}_latency_kt rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_latency_kt -o run -- tests/cpp/build/bench_latency 200" \
  "300 ${T}_bench python bench.py --sustain 0 --no-cpu" \
  "300 ${T}_bench_kt rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_bench_kt -o run -- python bench.py --sustain 0 --no-cpu --steps 20" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q "failed" gpurun_out/${T}_tests.log || exit 1
kt=$(find gpurun_out/${T}_bench_kt -name '*kernel_trace.csv' | head -n 1)
python3 - "$kt" > gpurun_out/${T}_exchange_kernels.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    if any(k in n for k in ("k_voc", "k_pack_slot", "k_tri_slots", "k_bow_slots", "k_rot_slots", "fillBuffer")):
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items()):
    v.sort()
    print("%-60s %5d launches, mean %.1f us, median %.1f us, max %.1f us" % (n, len(v), sum(v) / len(v), v[len(v) // 2], max(v)))
PY
cat gpurun_out/${T}_exchange_kernels.txt; grep '^{' gpurun_out/${T}_bench.log | head -c 600
# one-frame call A/B: levels [0, 2) on the side branch + the chained pyramid (br2, shipped), levels [0, 3) (br3),
# per-level resize launches (nochain)
for v in br2 br3 nochain; do mkdir -p gpurun_out/var_$v && ln -sf $R/cooperative-orb-slam_amd/lib/liborbamd_$v.so gpurun_out/var_$v/liborbamd.so; done
for r in 1 2; do for v in br2 br3 nochain; do
  LD_LIBRARY_PATH=$R/gpurun_out/var_$v timeout -k 10 200 tests/cpp/build/bench_latency 1000 2>/dev/null | grep '"extract"' | sed "s/^/r$r $v /" >> gpurun_out/${T}_branch_ab.log || exit $?
done; done
cat gpurun_out/${T}_branch_ab.log
