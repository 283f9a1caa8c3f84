#!/bin/bash
# round 4: the r04g evidence run, then the matcher A/B (query tiles per wave: base = 8 waves x 1 tile,
# q2w4 = 4 waves x 2 tiles at 3 waves/SIMD, q2w4s = the same held to 4 waves/SIMD)
tools/gpu_r04g.sh || exit $?
AB_ROUNDS=2 tools/ab.sh tests/test_gpu_match.py base q2w4 q2w4s > gpurun_out/r04h_ab_match_qt.log 2>&1
rc=$?; cat gpurun_out/r04h_ab_match_qt.log; exit $rc
