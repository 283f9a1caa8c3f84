#!/bin/bash
# One parameterised GPU recipe for the evidence of a head (replaces the per-session gpu_rNN*.sh files):
#   tools/gpu_round.sh <tag> <step> [<step> ...]
# steps, run in the order given, each under its own time limit (tools/gpu_run.sh stops at the first step that
# faults, aborts, times out or segfaults):
#   tests         the whole GPU suite (pytest -m gpu)            -> gpurun_out/<tag>_tests.log
#   smoke         __graft_entry__.smoke()                          -> <tag>_smoke.log
#   prof          kernel trace + PMC passes (tools/prof_round.sh), the timed region's per-kernel averages and the
#                 exchange kernels, reduced to <tag>_pmc_traffic.json / _pmc_summary.txt / _timed_region_kernels.txt
#   prof_cfg      the counter passes of C3 and C4 (tools/pmc_config.sh) -> profiles/pmc_traffic_c3.json, _c4.json
#   bench_driver  bench.py at the driver's arguments (C2)          -> <tag>_bench_driver.log
#   bench         bench.py at its defaults (C2)                    -> <tag>_bench.log
#   c3 / c4       bench.py --config c3 / c4 at the driver's arguments
#   latency       the one-frame / per-call C++ latency rows (tests/cpp/build/bench_latency 2000)
#   dropin        the drop-in ORBextractor's eager operator() and a two-thread stereo pair (bench_dropin_latency)
# A failing test or smoke step ends the recipe before any bench runs.
export TMPDIR=/tmp
T=$1
shift
[ -n "$T" ] || { echo "usage: tools/gpu_round.sh <tag> <step>..."; exit 2; }
for step in "$@"; do
  case $step in
    tests)
      tools/gpu_run.sh "600 ${T}_tests python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread" || exit $?
      grep -q " passed" gpurun_out/${T}_tests.log && ! grep -q " failed" gpurun_out/${T}_tests.log || exit 1 ;;
    smoke)
      tools/gpu_run.sh "200 ${T}_smoke python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" || exit $?
      grep -q "SMOKE OK" gpurun_out/${T}_smoke.log || exit 1 ;;
    prof)
      tools/prof_round.sh $T || exit $?
      kt=$(find gpurun_out/${T}_kt -name '*kernel_trace.csv' | head -n 1)
      read sub pipes < <(python3 bench.py --launch-frames)
      python3 tools/trace_segments.py "$kt" 10 2 $pipes 7 > gpurun_out/${T}_timed_region_kernels.txt || exit $?
      python3 tools/exchange_kernels.py "$kt" > gpurun_out/${T}_exchange_kernels.txt || exit $?
      python3 tools/queue_map.py "$kt" > gpurun_out/${T}_queue_map.txt || exit $?
      tools/prof_reduce.sh $T $sub
      cp gpurun_out/${T}_pmc_traffic.json profiles/pmc_traffic.json ;;  # the bench steps that follow read it
    prof_cfg) for c in c3 c4; do tools/pmc_config.sh $c || exit $?; done ;;
    bench_driver) tools/gpu_run.sh "300 ${T}_bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5" || exit $? ;;
    bench) tools/gpu_run.sh "300 ${T}_bench python3 bench.py" || exit $? ;;
    c3) tools/gpu_run.sh "300 ${T}_bench_c3 python3 bench.py --config c3 --gpus 1 --steps 20 --warmup 5" || exit $? ;;
    c4) tools/gpu_run.sh "300 ${T}_bench_c4 python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5" || exit $? ;;
    latency) tools/gpu_run.sh "300 ${T}_latency tests/cpp/build/bench_latency 2000" || exit $? ;;
    dropin) tools/gpu_run.sh "300 ${T}_dropin_latency tests/cpp/build/bench_dropin_latency 2000" || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
