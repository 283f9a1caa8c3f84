"""Per-phase wall-clock trace of k_octree for the one-frame call (A/B build with -DORBX_OCT_TRACE=1:
tools/build_variant.sh octtrace -DORBX_OCT_TRACE=1; run with ORBAMD_LIB_VARIANT=octtrace). Slots written by thread 0
of frame 0's workgroup of each level: 0 start, 1 key count, 2 keys gathered, 3 roots, 4+i division round i,
34 rounds done, 35 end; 36 = rounds | n << 16 | phase << 40 | size << 48. s_memrealtime ticks = 10 ns."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))
import orbamd  # noqa: E402

lib = orbamd.load()
frames = orbamd.synth_frames(0, 0, 8, 640, 480)
ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7, device=0)
buf = np.zeros((16, 40), dtype=np.uint64)
rows = []
for it in range(40):
    ext(frames[it % 8])
    assert lib.orbx_debug_octree_trace(buf.ctypes.data_as(C.c_void_p)) == 0
    if it >= 8:
        rows.append(buf.copy())
for l in range(8):
    tr = [r[l] for r in rows]
    info = int(tr[-1][36])
    iters, n, phase, size = info & 0xFFFF, (info >> 16) & 0xFFFFFF, (info >> 40) & 0xFF, info >> 48

    def med(a, b):
        return float(np.median([(int(t[b]) - int(t[a])) * 0.01 for t in tr]))

    rounds = " ".join("%.2f" % med(4 + i, 5 + i if i + 1 < iters else 34) for i in range(min(iters, 29)))
    print("level %d: n=%d rounds=%d phase=%d size=%d | count %.2f gather %.2f roots %.2f | rounds [%s] | select %.2f"
          " | total %.2f us" % (l, n, iters, phase, size, med(0, 1), med(1, 2), med(2, 3), rounds, med(34, 35),
                                 med(0, 35)))
