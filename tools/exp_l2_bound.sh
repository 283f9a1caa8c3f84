#!/bin/bash
# The L2-residency bound: the bench schedule as is against the same
# schedule with orbx_debug_alias_frames (every frame of a graph is its frame 0 and shares one pyramid /
# blur buffer, so every stage's reads hit data the launch keeps in L2), overlapped (4 graphs) and stage-serial
# (one graph, each kernel alone), 3 interleaved rounds; then FETCH_SIZE per launch of each stage for both.
export TMPDIR=/tmp
mkdir -p gpurun_out
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); s=d["stage_ms_per_step"]; print("%.0f frames/s" % d["value"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match")))'
B="python3 bench.py --no-cpu --sustain 0 --ingest-steps 0 --steps 100 --warmup 10"
for r in 1 2 3; do
  for m in "" "--alias-frames"; do
    out=$(timeout -k 10 120 $B $m | python3 -c "$summ") || exit $?
    echo "r$r overlapped ${m:-normal}: $out"
  done
done
for m in "" "--alias-frames"; do
  out=$(timeout -k 10 120 $B --pipes 1 --batch 256 --serial-stages $m | python3 -c "$summ") || exit $?
  echo "serial-1graph ${m:-normal}: $out"
done
R=$GRAFT_REPO_ROOT
P="python3 bench.py --no-cpu --sustain 0 --ingest-steps 0 --steps 2 --warmup 1 --no-check"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/l2b_fetch_normal -o run -- $P > gpurun_out/l2b_fetch_normal.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/l2b_fetch_alias -o run -- $P --alias-frames > gpurun_out/l2b_fetch_alias.log 2>&1 || exit $?
echo "pmc done"
