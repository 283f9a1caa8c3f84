#!/bin/bash
# HBM traffic + VALU counters of one bench configuration (separate --pmc passes, reduced on the box):
# writes gpurun_out/pmc_traffic_<cfg>.json (tools/pmc_traffic.py), which bench.py --config <cfg> reads for
# roofline.traffic and the VALU roofline. usage: tools/pmc_config.sh c3|c4
export TMPDIR=/tmp
C=$1
R=$GRAFT_REPO_ROOT
B="python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu --sustain 0"
tools/gpu_run.sh \
  "300 pmc_${C}_a rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_${C}_a -o run -- $B" \
  "300 pmc_${C}_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_${C}_fetch -o run -- $B" \
  "300 pmc_${C}_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_${C}_write -o run -- $B" || exit $?
one() { find "$1" -name "$2" 2>/dev/null | head -n 1; }
O=gpurun_out
read sub pipes < <(python3 bench.py --config $C --launch-frames)
python3 tools/pmc_traffic.py "$(one $O/pmc_${C}_fetch '*counter_collection.csv')" "$(one $O/pmc_${C}_write '*counter_collection.csv')" \
  $O/pmc_traffic_${C}.json "$(one $O/pmc_${C}_a '*counter_collection.csv')" $sub || exit $?
cp $O/pmc_traffic_${C}.json profiles/pmc_traffic_${C}.json  # the bench lines that follow on this box read it
python3 tools/pmc_summary.py "$(one $O/pmc_${C}_a '*counter_collection.csv')" > $O/pmc_summary_${C}.txt
rm -rf $O/pmc_${C}_a $O/pmc_${C}_fetch $O/pmc_${C}_write
