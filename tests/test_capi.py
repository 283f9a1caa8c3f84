"""The C ABI library loads without a GPU, exports every symbol include/orbslam_amd.h
declares, and its host-only entry points behave; compute entry points fail loudly
(ORBX_EDEVICE) instead of falling back to the CPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import orbamd
from orbamd._lib import SIGNATURES, OrbxParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "orbslam_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b((?:orbx|orbm)_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported_and_bound():
    lib = orbamd.load()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in SIGNATURES, "python binding misses " + s


def test_single_hip_runtime_in_process():
    from orbamd._lib import runtime_path
    orbamd.load()
    libs = {l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}
    assert len(libs) == 1 and runtime_path() in libs


def test_synth_frames_deterministic():
    a = orbamd.synth_frames(0, 0, 3, 640, 480)
    b = orbamd.synth_frames(0, 1, 2, 640, 480)
    assert np.array_equal(a[1:], b)
    c = orbamd.synth_frames(1, 0, 1, 640, 480)
    assert not np.array_equal(a[0], c[0])
    assert 60 < a.mean() < 190 and a.std() > 20


def test_synth_scene_views_overlap():
    """Shared-scene mode: view 0 of scene s is agent s's own stream; view v is the same texture with the crop
    12*v px further along the pan, so two agents' frames at one time step overlap by all but 12*|dv| columns."""
    W, H = 640, 480
    a0 = orbamd.synth_frames(0, 4, 2, W, H)
    assert np.array_equal(orbamd.synth_frames(0, 4, 2, W, H, scene=0), a0)
    v2 = orbamd.synth_frames(2, 4, 2, W, H, scene=0)
    assert not np.array_equal(v2, a0)
    assert np.array_equal(v2[:, :, :W - 24], a0[:, :, 24:])  # view 2 starts 24 px to the right
    assert np.array_equal(orbamd.synth_frames(3, 4, 1, W, H, dx=5, scene=0)[0, :, :W - 5],
                          orbamd.synth_frames(3, 4, 1, W, H, scene=0)[0, :, 5:])


def test_descriptor_distance_host():
    rng = np.random.default_rng(0)
    for _ in range(100):
        x = rng.integers(0, 256, 32, dtype=np.uint8)
        y = rng.integers(0, 256, 32, dtype=np.uint8)
        assert orbamd.ORBmatcher.DescriptorDistance(x, y) == int(np.unpackbits(x ^ y).sum())


def test_epipole_helper():
    R = np.eye(3, dtype=np.float32)
    t = np.array([0.05, 0.0, 0.01], np.float32)
    ex, ey = orbamd.epipole(R, t, np.zeros(3, np.float32), 715.092024, 719.025258, 334.298489, 256.326097)
    assert abs(ex - (715.092024 * 5 + 334.298489)) < 1e-2 and abs(ey - 256.326097) < 1e-3


def test_no_cpu_fallback_without_gpu():
    lib = orbamd.load()
    if lib.orbx_device_count() > 0:
        pytest.skip("a GPU is present")
    p = OrbxParams(1000, 1.2, 8, 20, 7)
    h = C.c_void_p()
    assert lib.orbx_create(C.byref(p), 0, 640, 480, 1, C.byref(h)) == -2  # ORBX_EDEVICE
    assert lib.orbm_create(0, C.byref(h)) == -2


def test_bad_arguments():
    lib = orbamd.load()
    h = C.c_void_p()
    assert lib.orbx_create(None, 0, 640, 480, 1, C.byref(h)) == -1
    p = OrbxParams(1000, 1.2, 99, 20, 7)
    assert lib.orbx_create(C.byref(p), 0, 640, 480, 1, C.byref(h)) == -1


def test_host_pyramid_target_arguments():
    """the caller-owned eager-pyramid storage (orbx_host_register / orbx_set_host_pyramid_target, the drop-in's
    refcounted mvImagePyramid): argument checks, and no GPU means ORBX_EDEVICE, never a silent success"""
    lib = orbamd.load()
    nb = C.c_size_t(7)
    assert lib.orbx_host_pyramid_bytes(None, 640, 480, C.byref(nb)) == -1
    assert lib.orbx_set_host_pyramid_target(None, None, 0) == -1
    assert lib.orbx_host_register(None, 4096) == -1
    assert lib.orbx_host_unregister(None) == -1
    buf = np.zeros(8192, np.uint8)
    assert lib.orbx_host_register(buf.ctypes.data, 0) == -1
    if lib.orbx_device_count() == 0:
        assert lib.orbx_host_register(buf.ctypes.data, 4096) == -2  # ORBX_EDEVICE
