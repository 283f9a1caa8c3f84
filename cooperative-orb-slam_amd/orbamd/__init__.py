"""orbamd -- MI355X-native ORB front-end + Hamming matcher (Python host binding).

Mirrors the reference's two C++ class surfaces so tests and tools read like ORB-SLAM2:

* :class:`ORBextractor` -- ``ORB_SLAM2::ORBextractor`` (ORBextractor.h:45-111)
* :class:`ORBmatcher`   -- ``ORB_SLAM2::ORBmatcher`` (ORBmatcher.h:37-102)

All compute runs in liborbamd.so (HIP kernels for gfx950) through the C ABI declared in
include/orbslam_amd.h. There is no CPU fallback: without the library or a GPU the
compute calls raise.
"""
from ._lib import LIB_PATH, KP_FIELDS, load  # noqa: F401
from .extractor import ORBextractor, synth_frames, kp_dtype  # noqa: F401
from .matcher import ORBmatcher, KeyFrameView, KeyFrameCache, epipole, compute_f12  # noqa: F401
from . import device, frame, projection  # noqa: F401
from .projection import FrameView, MapPoints  # noqa: F401
from .vocabulary import ORBVocabulary  # noqa: F401
from .frame import compute_stereo_matches  # noqa: F401
