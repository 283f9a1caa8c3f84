"""ctypes binding of include/orbslam_amd.h (the C ABI of liborbamd.so).

The library is built in-tree (``make -C cooperative-orb-slam_amd``) and loaded from
``cooperative-orb-slam_amd/lib/liborbamd.so``. There is no fallback: if the library is
missing, importing the compute API raises.
"""
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ORBAMD_LIB_VARIANT=<tag> loads lib/liborbamd_<tag>.so instead: A/B builds of one source tree for the
# tools/ab_*.sh experiments (same ABI, different kernel variants)
_VARIANT = os.environ.get("ORBAMD_LIB_VARIANT", "")
LIB_PATH = os.path.join(PKG_DIR, "lib", "liborbamd%s.so" % ("_" + _VARIANT if _VARIANT else ""))

ORBX_OK = 0
ORBX_EARG = -1
ORBX_EDEVICE = -2
ORBX_ECAPACITY = -3


class OrbxParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class OrbxKp(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32)]


class OrbmKfView(C.Structure):
    _fields_ = [("n", C.c_int32), ("desc", C.c_void_p), ("x", C.c_void_p), ("y", C.c_void_p),
                ("angle", C.c_void_p), ("octave", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("mp_bad", C.c_void_p), ("n_nodes", C.c_int32),
                ("node_id", C.c_void_p), ("node_off", C.c_void_p), ("node_feat", C.c_void_p),
                ("nlevels", C.c_int32), ("scale_factors", C.c_void_p), ("level_sigma2", C.c_void_p)]


# numpy dtype matching orbx_kp (24 bytes)
KP_FIELDS = [("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
             ("octave", "<i4")]

# every entry point declared in include/orbslam_amd.h: name -> (restype, argtypes)
_P = C.c_void_p
_I = C.c_int
_F = C.c_float
_SZ = C.c_size_t
SIGNATURES = {
    "orbx_create": (_I, [C.POINTER(OrbxParams), _I, _I, _I, _I, C.POINTER(_P)]),
    "orbx_destroy": (None, [_P]),
    "orbx_max_keypoints": (_I, [_P, _I, _I]),
    "orbx_extract": (_I, [_P, _P, _I, _I, _SZ, _P, _P, _I, C.POINTER(_I)]),
    "orbx_extract_batch_device": (_I, [_P, _I, _P, _SZ, _I, _I, _SZ, _P, _P, _P, _I, _P]),
    "orbx_pyramid_level": (_I, [_P, _I, _I, _P, _SZ, C.POINTER(_I), C.POINTER(_I)]),
    "orbx_get_levels": (_I, [_P]),
    "orbx_get_scale_factor": (_F, [_P]),
    "orbx_get_scale_tables": (_I, [_P, _P, _P, _P, _P]),
    "orbx_get_feature_split": (_I, [_P, _P, _P]),
    "orbm_create": (_I, [_I, C.POINTER(_P)]),
    "orbm_destroy": (None, [_P]),
    "orbm_descriptor_distance": (_I, [_P, _P]),
    "orbm_search_for_triangulation": (_I, [_P, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _P, _F, _F, _I, _I,
                                           _P, C.POINTER(_I)]),
    "orbm_search_by_bow_kf_f": (_I, [_P, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _F, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_bow_kf_kf": (_I, [_P, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _F, _I, _P, C.POINTER(_I)]),
    "orbm_triangulation_bf_batch_device": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _P, _F, _F, _I, _P, _P, _I, _P, _P,
                                                _P]),
    "orbm_triangulation_bf_packed_device": (_I, [_P, _P, _P, _P, _I, _P, _SZ, _P, _F, _F, _I, _P, _P, _P, _I, _P,
                                                 _P]),
    "orbm_triangulation_nodes_batch_device": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _P, _F, _F,
                                                   _I, _P, _P, _I, _P, _P, _P]),
    "orbm_search_by_bow_batch_device": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _F, _I, _P,
                                             _P, _P]),
    "orbm_epipole": (None, [_P, _P, _P, _F, _F, _F, _F, C.POINTER(_F), C.POINTER(_F)]),
    "orbx_slot_bytes": (_SZ, [_I]),
    "orbx_pack_keyframe_device": (_I, [_P, _P, _P, _I, _P, _P]),
    "orbx_synth_frame": (_I, [_I, _I, _I, _I, _P]),
    "orbx_synth_frames": (_I, [_I, _I, _I, _I, _I, _P]),
    "orbx_synth_frames_shifted": (_I, [_I, _I, _I, _I, _I, _I, _P]),
    "orbx_compute_stereo_matches": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _P, _P, C.POINTER(_I)]),
    "orbx_stereo_matches_batch_device": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _P, _P, _P,
                                              _P]),
    "orbx_check_error": (_I, [_P, _P]),
    "orbm_search_by_projection_local": (_I, [_P, _P, _P, _F, _F, _P, C.POINTER(_I)]),
    "orbm_search_by_projection_last_frame": (_I, [_P, _P, _P, _P, _P, _F, _I, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_projection_keyframe": (_I, [_P, _P, _P, _P, _F, _I, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_projection_sim3": (_I, [_P, _P, _P, _P, _I, _P, C.POINTER(_I)]),
    "orbm_compute_distinctive_descriptors": (_I, [_P, _I, _P, _P, _P, _P]),
    "orbv_load_text": (_I, [C.c_char_p, _I, C.POINTER(_P)]),
    "orbv_create": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _I, C.POINTER(_P)]),
    "orbv_destroy": (None, [_P]),
    "orbv_info": (_I, [_P, C.POINTER(_I), C.POINTER(_I), C.POINTER(_I), C.POINTER(_I)]),
    "orbv_transform": (_I, [_P, _P, _I, _I, _P, _P, C.POINTER(_I), _P, _P, _P, C.POINTER(_I)]),
    "orbv_transform_batch_device": (_I, [_P, _I, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "orbm_compute_distinctive_descriptors_device": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "orbx_selftest_sincosf": (_I, [_P, _P, _P, _I, _P]),
    "orbx_profile_enable": (_I, [_P, _I]),
    "orbx_profile_read": (_I, [_P, C.POINTER(C.c_double), C.POINTER(_I)]),
    "orbx_version": (C.c_char_p, []),
    "orbx_device_count": (_I, []),
}

_lib = None


def _bind_runtime():
    """One HIP runtime per process: if torch is importable, import it first so liborbamd.so's
    DT_NEEDED `libamdhip64.so` binds to the runtime torch loaded (device pointers and streams
    from torch are then valid in our kernels); otherwise RUNPATH picks /opt/rocm/lib's."""
    if os.environ.get("ORBAMD_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def runtime_path():
    """Path of the libamdhip64 this process uses (for diagnostics/tests)."""
    for line in open("/proc/self/maps"):
        if "libamdhip64" in line:
            return line.split()[-1]
    return None


def load():
    """Load liborbamd.so (raises OSError when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("liborbamd.so not built: run `make -C cooperative-orb-slam_amd` "
                          "(or __graft_entry__.build()); expected at %s" % LIB_PATH)
        _bind_runtime()
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc, what):
    if rc != ORBX_OK:
        names = {ORBX_EARG: "ORBX_EARG", ORBX_EDEVICE: "ORBX_EDEVICE", ORBX_ECAPACITY: "ORBX_ECAPACITY"}
        raise RuntimeError("%s failed: %s (%d)" % (what, names.get(rc, "?"), rc))
    return rc
