#!/bin/bash
# round 4: where k_voc_bow's time goes for one keyframe (per-phase trace, diagnostic build bowtrace)
export TMPDIR=/tmp
ORBAMD_LIB_VARIANT=bowtrace timeout -k 10 300 python tools/bow_trace.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04x_bow_trace.log
