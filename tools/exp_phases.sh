#!/bin/bash
# Phase costs of one extraction stage (timing only): serial one-graph stage times of variants built with a
# phase-cut macro (tools/build_variant.sh <tag> -DORBX_<STAGE>_STOP=<k>); their outputs are invalid, so the
# bench runs with --no-check. usage: [PH_ARGS="--config c4"] tools/exp_phases.sh <stage key> v1 v2 ... (e.g. octree os1 os2 os3 head)
st=$1; shift
for v in "$@"; do
  out=$(ORBAMD_LIB_VARIANT=$v ORBX_SCHED=serial timeout -k 10 120 python bench.py --sustain 0 --no-cpu --no-check --steps 30 --pipes 1 --batch 256 ${PH_ARGS} | \
    python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$st=%.4f' % d['stage_ms_per_step']['$st'])") || exit $?
  echo "$v $out"
done
