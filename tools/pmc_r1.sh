#!/bin/bash
# PMC passes (counters only with --kernel-trace-free collection; separate runs per counter group).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu"
tools/gpu_run.sh \
  "300 pmc_a rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_a -o run -- $B" \
  "300 pmc_b rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM --output-format csv -d $R/gpurun_out/pmc_b -o run -- $B" \
  "300 pmc_c rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --output-format csv -d $R/gpurun_out/pmc_c -o run -- $B"
