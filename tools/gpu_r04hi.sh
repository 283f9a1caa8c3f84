#!/bin/bash
# round 4 diagnostic: what in the exchange-enabled schedule object slows the step (tools/exp_host_issue.py, one
# configuration per process, two rounds)
export TMPDIR=/tmp
for r in 1 2; do
  for c in A A0 B C D; do
    XCFG=$c timeout -k 10 200 python -u tools/exp_host_issue.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r04hi3_host_issue.log || exit $?
  done
done
