set -o pipefail
T0=$(date +%s); timeout -k 10 300 python bench.py > gpurun_out/bench_sus.log 2> gpurun_out/bench_sus.err || { tail -5 gpurun_out/bench_sus.err; exit 1; }
python -c 'import json; d=json.loads(open("gpurun_out/bench_sus.log").read().strip().splitlines()[-1]); print(d["value"], d["bit_exact"], d["sustained"], d["cpu_baseline"]["value"])'
echo "wall $(( $(date +%s) - T0 )) s"
timeout -k 10 300 tools/rehearse_ranks.sh 2 > gpurun_out/rehearse.log 2>&1 || { tail -5 gpurun_out/rehearse.log; exit 1; }
grep '^{' gpurun_out/rehearse.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("N=2 rehearsal", d["value"], d["bit_exact"], d["sustained"])'
