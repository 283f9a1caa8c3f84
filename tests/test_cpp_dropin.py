"""The C++ drop-in classes (host/ORBextractor.*, host/ORBmatcher*) build with g++ against
the C ABI, and (GPU) reproduce the oracle bit-exactly when called like ORB-SLAM2 does."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_dropin")


def _build():
    subprocess.check_call([os.path.join(ROOT, "tests", "cpp", "build.sh")])


def test_dropin_builds():
    _build()
    assert os.path.exists(BIN)


@pytest.mark.gpu
@pytest.mark.parametrize("kf_cache_mb", [None, "0"])
def test_dropin_bit_exact_on_gpu(kf_cache_mb):
    """with the device keyframe cache (the default; test_dropin checks the matcher threads shared it) and
    without it (ORBAMD_KF_CACHE_MB=0: every call uploads its keyframes)"""
    _build()
    env = dict(os.environ)
    env.pop("ORBAMD_KF_CACHE_MB", None)
    if kf_cache_mb is not None:
        env["ORBAMD_KF_CACHE_MB"] = kf_cache_mb
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and "ALL PASS" in r.stdout


@pytest.mark.gpu
def test_stock_pyramid_reader_sees_current_frame():
    """ORBextractor built without the drop-in Frame::ComputeStereoMatches and no ORBAMD_HOST_PYRAMID: a stock
    reader of mvImagePyramid straight after operator() (A1 Frame.cc:474-581) gets this frame's levels, bit-exact
    (ORBextractor.cc:1107-1132), with no SyncImagePyramid() call"""
    _build()
    env = dict(os.environ)
    env.pop("ORBAMD_HOST_PYRAMID", None)
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", "test_pyramid_reader")], capture_output=True,
                       text=True, timeout=300, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and "ALL PASS" in r.stdout


def test_dropins_do_not_throw_without_device():
    """ORBX_EDEVICE from every C ABI call (ORBAMD_DEVICE=99 is out of range on any box): each drop-in returns
    the reference's "nothing found" result and logs the status instead of throwing into the caller's thread"""
    _build()
    env = dict(os.environ, ORBAMD_DEVICE="99")
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", "test_nodevice")], capture_output=True,
                       text=True, timeout=120, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and "ALL PASS" in r.stdout
    assert "orbslam_amd: orbx_create failed (status -2, device)" in r.stderr


def test_slot_codec_roundtrip_cpp():
    """host/KeyFrameSlot_amd.*: receiveKeyframeInfo -> slot -> receiveKeyframeInfo, field for field (CPU)"""
    _build()
    env = dict(os.environ, ORBAMD_NO_TORCH="1")
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", "test_slot")], capture_output=True, text=True,
                       timeout=120, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and "ALL PASS" in r.stdout
