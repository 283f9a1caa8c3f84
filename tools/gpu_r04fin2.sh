#!/bin/bash
# round 4 final evidence on the shipped head (after the lazy vocabulary stream; kernels unchanged since r04fin, so no PMC passes): the whole GPU suite + smoke; the kernel trace + PMC passes of the
# bench (tools/prof_round.sh) whose traffic file the bench lines then read; the bench at the driver's arguments
# and at its defaults (C2), C3 and C4 lines; the one-frame / per-call latency rows; the timed region's per-kernel
# averages and the exchange kernels
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=r04fin2
tools/gpu_run.sh \
  "700 ${T}_tests python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread" \
  "200 ${T}_smoke python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q " failed" gpurun_out/${T}_tests.log || exit 1
grep -q "SMOKE OK" gpurun_out/${T}_smoke.log || exit 1
tools/gpu_run.sh \
  "300 ${T}_bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_bench python3 bench.py" \
  "300 ${T}_bench_c3 python3 bench.py --config c3 --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_bench_c4 python3 bench.py --config c4 --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_latency tests/cpp/build/bench_latency 2000" || exit $?
