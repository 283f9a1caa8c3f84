#!/bin/bash
# round 4: where the one-frame call's octree time goes (per-phase s_memrealtime trace, A/B build octtrace)
export TMPDIR=/tmp
ORBAMD_LIB_VARIANT=octtrace timeout -k 10 300 python tools/oct_trace.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04k_oct_trace.log
