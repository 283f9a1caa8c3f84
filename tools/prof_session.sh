#!/bin/bash
# Full evidence session on the GPU box: the default bench line (with the CPU baseline), the kernel
# trace + PMC passes of tools/prof_round.sh, the stage-serial isolated trace and the
# row benchmarks under a kernel trace. Outputs under gpurun_out/<tag>_*. usage: tools/prof_session.sh <tag>
export TMPDIR=/tmp
T=${1:-r01}
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh "300 ${T}_bench python3 bench.py" || exit $?
cp gpurun_out/${T}_bench.log gpurun_out/${T}_bench.json
tools/prof_round.sh "$T" || exit $?
tools/gpu_run.sh \
  "300 ${T}_iso rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_iso -o run -- python3 bench.py --pipes 1 --batch 256 --serial-stages --no-cpu --steps 10 --sustain 0" || exit $?
tools/gpu_run.sh \
  "300 ${T}_rows rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_rows -o run -- python3 tools/bench_rows.py"
