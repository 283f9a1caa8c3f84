#!/bin/bash
# round 4: the one-frame host path (level-0 side branch, results written into pinned memory by the kernels),
# then the exchange-stream A/B at N = 1 with the heavier exchange (BoW + two slot matchers), then the bench line
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "600 r04f_tests python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_cpp_dropin.py tests/test_gpu_schedule.py -m gpu -x -v --timeout 240 --timeout-method thread" \
  "300 r04f_latency tests/cpp/build/bench_latency 2000" \
  "300 r04f_latency_kt rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04f_latency_kt -o run -- tests/cpp/build/bench_latency 200" || exit $?
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f frames/s" % d["value"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match","exchange")))'
for r in 1 2 3; do
  for x in graph0 own; do
    out=$(timeout -k 10 120 python3 bench.py --no-cpu --sustain 0 --ingest-steps 0 --exchange-stream $x | python3 -c "$summ") || exit $?
    echo "r$r exchange-stream $x: $out"
  done
done 2>&1 | tee gpurun_out/r04f_ab_exchange_stream.log
timeout -k 10 300 python3 bench.py > gpurun_out/r04f_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04f_bench_driver.log 2>&1
