"""Per-phase wall-clock trace of k_voc_bow for one keyframe (A/B build with -DORBX_BOW_TRACE=1:
tools/build_variant.sh bowtrace -DORBX_BOW_TRACE=1; run with ORBAMD_LIB_VARIANT=bowtrace). Stamps by thread 0 of
workgroup 0: 0 start, 1 FeatureVector keys, 2 sorted, 3 FeatureVector written, 4 BowVector keys, 5 sorted,
6 word values, 7 normalised. s_memrealtime ticks = 10 ns."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cooperative-orb-slam_amd"))
import orbamd  # noqa: E402
from orbamd.vocabulary import L1_NORM, TF_IDF, ORBVocabulary, synth_vocabulary_full  # noqa: E402

lib = orbamd.load()
k, L, par, leaf, vdesc, w = synth_vocabulary_full(seed=7)
voc = ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, par, leaf, vdesc, w, device=0)
ext = orbamd.ORBextractor(1000, 1.2, 8, 20, 7, device=0)
frames = orbamd.synth_frames(0, 0, 4, 640, 480)
descs = [ext(f)[1] for f in frames]
buf = np.zeros(16, dtype=np.uint64)
rows = []
for it in range(24):
    voc.transform(descs[it % 4], 4)
    assert lib.orbx_debug_bow_trace(buf.ctypes.data_as(C.c_void_p)) == 0
    if it >= 4:
        rows.append(buf.copy())
names = ["fv keys", "fv sort", "fv write", "bow keys", "bow sort", "values", "normalise"]
med = lambda a, b: float(np.median([(int(r[b]) - int(r[a])) * 0.01 for r in rows]))  # noqa: E731
print("n=%d: " % len(descs[0]) + " | ".join("%s %.2f" % (nm, med(i, i + 1)) for i, nm in enumerate(names)) +
      " | total %.2f us" % med(0, 7))
