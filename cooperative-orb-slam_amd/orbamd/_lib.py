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


SLOT_NSECTIONS = 12
SLOT_SECTIONS = ("KPS", "KUN", "URIGHT", "DEPTH", "DESC", "MPFLAGS", "MPPOS", "BOWWORD", "BOWVALUE", "FVNODE", "FVOFF",
                 "FVFEAT")
SLOT_MAGIC = 0x4B42524F
SLOT_VERSION = 2
SLOT_F_KUN, SLOT_F_STEREO, SLOT_F_MP, SLOT_F_BOW, SLOT_F_FV = 1, 2, 4, 8, 16


class OrbxSlotHeader(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("version", C.c_uint32), ("n", C.c_int32), ("cap", C.c_int32),
                ("nbow", C.c_int32), ("nfv", C.c_int32), ("flags", C.c_uint32), ("bytes", C.c_uint32),
                ("off", C.c_uint32 * SLOT_NSECTIONS), ("reserved", C.c_uint32 * 12)]


_META_I64 = ["nNextId", "mnId", "mnFrameId", "mnGridCols", "mnGridRows", "mnTrackReferenceForFrame",
             "mnFuseTargetForKF", "mnBALocalForKF", "mnBAFixedForKF", "mnLoopQuery", "mnLoopWords", "mnRelocQuery",
             "mnRelocWords", "mnBAGlobalForKF", "mnMinX", "mnMinY", "mnMaxX", "mnMaxY"]
_META_F32 = ["mfGridElementWidthInv", "mfGridElementHeightInv", "mLoopScore", "mRelocScore", "fx", "fy", "cx", "cy",
             "invfx", "invfy", "mbf", "mb", "mThDepth", "mfScaleFactor", "mfLogScaleFactor"]


class OrbxKfMeta(C.Structure):
    """orbx_kf_meta: the scalar / matrix fields of lcmKeyFrameInfo (lcmKeyFrameInfo.hpp:24-100)."""
    _fields_ = ([(k, C.c_int64) for k in _META_I64] + [("mTimeStamp", C.c_double), ("agent", C.c_int32),
                                                       ("mnScaleLevels", C.c_int32)] +
                [(k, C.c_float) for k in _META_F32] +
                [("mvScaleFactors", C.c_float * 16), ("mvLevelSigma2", C.c_float * 16),
                 ("mvInvLevelSigma2", C.c_float * 16), ("mK", C.c_float * 9), ("mTcw", C.c_float * 16),
                 ("mTcwGBA", C.c_float * 16), ("mTcwBefGBA", C.c_float * 16), ("mTcp", C.c_float * 16)])


class OrbxKfSource(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("kps", "desc", "count", "kun", "uright", "depth", "mp_flags", "mp_pos",
                                          "bow_word", "bow_value", "nbow", "fv_node", "fv_off", "fv_feat", "nfv")]


class OrbxSlotView(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("hdr", "meta", "kps", "kun", "uright", "depth", "desc", "mp_flags",
                                          "mp_pos", "bow_word", "bow_value", "fv_node", "fv_off", "fv_feat")]


class OrbmSlotGeom(C.Structure):
    _fields_ = [("F12", C.c_float * 9), ("ex", C.c_float), ("ey", C.c_float)]


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
    "orbx_set_host_pyramid": (_I, [_P, _I]),
    "orbx_host_pyramid_level": (_I, [_P, _I, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_I), C.POINTER(_I)]),
    "orbx_host_pyramid_bytes": (_I, [_P, _I, _I, C.POINTER(_SZ)]),
    "orbx_host_register": (_I, [_P, _SZ]),
    "orbx_host_unregister": (_I, [_P]),
    "orbx_set_host_pyramid_target": (_I, [_P, _P, _SZ]),
    "orbx_get_levels": (_I, [_P]),
    "orbx_get_scale_factor": (_F, [_P]),
    "orbx_get_scale_tables": (_I, [_P, _P, _P, _P, _P]),
    "orbx_get_feature_split": (_I, [_P, _P, _P]),
    "orbx_compute_scale_tables": (_I, [C.POINTER(OrbxParams), _P, _P, _P, _P]),
    "orbx_set_pyramid_event": (_I, [_P, _P]),
    "orbx_set_stage_event": (_I, [_P, _I, _P]),
    "orbx_debug_skip_stages": (_I, [_P, _I]),
    "orbx_debug_hip_failure": (_I, []),
    "orbx_comm_unique_id": (_I, [_P]),
    "orbx_comm_create": (_I, [_P, _I, _I, _I, _P]),
    "orbx_comm_allgather": (_I, [_P, _P, _P, _SZ, _P]),
    "orbx_comm_destroy": (None, [_P]),
    "orbx_describe_blur_fused": (_I, [_P, _SZ, _SZ]),
    "orbx_debug_serial": (_I, [_P, _I]),
    "orbx_debug_alias_frames": (_I, [_P, _I]),
    "orbx_debug_raise_error": (_I, [_P, _I, _P]),
    "orbm_create": (_I, [_I, C.POINTER(_P)]),
    "orbm_destroy": (None, [_P]),
    "orbm_descriptor_distance": (_I, [_P, _P]),
    "orbm_search_for_triangulation": (_I, [_P, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _P, _F, _F, _I, _I,
                                           _P, C.POINTER(_I)]),
    "orbm_search_by_bow_kf_f": (_I, [_P, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _F, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_bow_kf_kf": (_I, [_P, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _F, _I, _P, C.POINTER(_I)]),
    "orbm_triangulation_bf_batch_device": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _P, _F, _F, _I, _P, _P, _I, _P, _P,
                                                _P]),
    "orbm_triangulation_bf_stereo_batch_device": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _I, _P, _F, _F, _I, _P, _P, _I,
                                                       _I, _P, _P, _P]),
    "orbm_search_for_triangulation_slots_device": (_I, [_P, C.POINTER(OrbxKfSource), _I, _I, _P, _SZ,
                                                        C.POINTER(OrbmSlotGeom), _I, _I, _P, _P, _P]),
    "orbm_search_by_bow_slots_device": (_I, [_P, C.POINTER(OrbxKfSource), _I, _I, _P, _SZ, _F, _I, _I, _P, _P, _P]),
    "orbm_check_error": (_I, [_P, _P]),
    "orbm_triangulation_nodes_batch_device": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _I, _P, _F, _F,
                                                   _I, _P, _P, _I, _P, _P, _P]),
    "orbm_search_by_bow_batch_device": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _F, _I, _P,
                                             _P, _P]),
    "orbm_epipole": (None, [_P, _P, _P, _F, _F, _F, _F, C.POINTER(_F), C.POINTER(_F)]),
    "orbx_slot_bytes": (_SZ, [_I]),
    "orbx_slot_layout": (_I, [_I, C.POINTER(OrbxSlotHeader)]),
    "orbx_pack_keyframe_device": (_I, [C.POINTER(OrbxKfSource), C.POINTER(OrbxKfMeta), _I, _P, _P, _P]),
    "orbx_pack_keyframe_host": (_I, [C.POINTER(OrbxKfSource), C.POINTER(OrbxKfMeta), _I, _P, _SZ]),
    "orbx_slot_parse": (_I, [_P, _SZ, C.POINTER(OrbxSlotView)]),
    "orbx_synth_frame": (_I, [_I, _I, _I, _I, _P]),
    "orbx_synth_frames": (_I, [_I, _I, _I, _I, _I, _P]),
    "orbx_synth_frames_shifted": (_I, [_I, _I, _I, _I, _I, _I, _P]),
    "orbx_synth_scene_frames": (_I, [_I, _I, _I, _I, _I, _I, _I, _P]),
    "orbx_compute_stereo_matches": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _F, _F, _P, _P, C.POINTER(_I)]),
    "orbx_stereo_matches_batch_device": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _P, _P, _P,
                                              _P]),
    "orbx_check_error": (_I, [_P, _P]),
    "orbm_search_by_projection_local": (_I, [_P, _P, _P, _F, _F, _P, C.POINTER(_I)]),
    "orbm_search_by_projection_last_frame": (_I, [_P, _P, _P, _P, _P, _F, _I, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_projection_keyframe": (_I, [_P, _P, _P, _P, _F, _I, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_projection_sim3": (_I, [_P, _P, _P, _P, _I, _P, C.POINTER(_I)]),
    "orbm_fuse": (_I, [_P, _P, _P, _P, _P, _F, _P, _P, C.POINTER(_I)]),
    "orbm_fuse_sim3": (_I, [_P, _P, _P, _P, _F, _P, C.POINTER(_I)]),
    "orbm_search_for_initialization": (_I, [_P, _P, _P, _P, _I, _F, _I, _P, C.POINTER(_I)]),
    "orbm_kf_cache_create": (_I, [_I, _SZ, C.POINTER(_P)]),
    "orbm_kf_cache_destroy": (None, [_P]),
    "orbm_kf_cache_erase": (_I, [_P, C.c_uint64]),
    "orbm_kf_cache_stats": (_I, [_P, C.POINTER(_I), C.POINTER(_SZ), C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "orbm_search_for_triangulation_cached": (_I, [_P, _P, C.c_uint64, C.POINTER(OrbmKfView), C.c_uint64,
                                                  C.POINTER(OrbmKfView), _P, _F, _F, _I, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_bow_kf_kf_cached": (_I, [_P, _P, C.c_uint64, C.POINTER(OrbmKfView), C.c_uint64,
                                             C.POINTER(OrbmKfView), _F, _I, _P, C.POINTER(_I)]),
    "orbm_search_by_bow_kf_f_cached": (_I, [_P, _P, C.c_uint64, C.POINTER(OrbmKfView), C.POINTER(OrbmKfView), _F,
                                            _I, _P, C.POINTER(_I)]),
    "orbm_fuse_cached": (_I, [_P, _P, C.c_uint64, _P, _P, _P, _P, _F, _P, _P, C.POINTER(_I)]),
    "orbm_search_by_sim3": (_I, [_P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _F, _P, C.POINTER(_I)]),
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
