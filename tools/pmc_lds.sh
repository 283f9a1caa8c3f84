#!/bin/bash
# LDS bank-conflict pass of the bench (one --pmc run, SQ block only): per-kernel conflict cycles per LDS
# instruction -> gpurun_out/pmc_lds_<tag>.txt. usage: tools/pmc_lds.sh <tag> [bench args]
export TMPDIR=/tmp
T=$1; shift
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES \
  --output-format csv -d $R/gpurun_out/pmc_lds_$T -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --sustain 0 \
  --ingest-steps 0 "$@" > gpurun_out/pmc_lds_$T.log 2>&1 || exit $?
f=$(find gpurun_out/pmc_lds_$T -name '*counter_collection.csv' | head -n 1)
python3 tools/pmc_summary.py "$f" > gpurun_out/pmc_lds_$T.txt
rm -rf gpurun_out/pmc_lds_$T
cat gpurun_out/pmc_lds_$T.txt
