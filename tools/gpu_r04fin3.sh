#!/bin/bash
# round 4 final head (matcher contexts' streams lazy): the whole GPU suite + smoke + the driver-argument bench line
export TMPDIR=/tmp
T=r04fin3
tools/gpu_run.sh \
  "700 ${T}_tests python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread" \
  "200 ${T}_smoke python3 -c 'import __graft_entry__ as g; g.smoke(); print(\"SMOKE OK\")'" || exit $?
grep -q "passed" gpurun_out/${T}_tests.log && ! grep -q " failed" gpurun_out/${T}_tests.log || exit 1
grep -q "SMOKE OK" gpurun_out/${T}_smoke.log || exit 1
tools/gpu_run.sh \
  "300 ${T}_bench_driver python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "300 ${T}_bench python3 bench.py" \
  "300 ${T}_latency tests/cpp/build/bench_latency 2000" || exit $?
