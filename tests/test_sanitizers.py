"""Host-side sanitizer runs (GPU sanitizers are not available on the pool): the CPU
oracle + synthetic generator under AddressSanitizer/UBSan (tests/cpp/test_oracle_asan.c), the
C++ keyframe-slot codec (host/KeyFrameSlot_amd.*) under the same sanitizers, and the concurrent host code under
ThreadSanitizer: the keyframe cache's books (csrc/kf_cache.h) from the three matcher threads and the C++ drop-ins
from 2 extractor + 3 matcher threads on their device-less path (tests/cpp/test_kf_cache_tsan.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "cpp", "build")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def _run(cmd, env=None):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-3000:], r.stderr[-3000:])
    return r


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_oracle_under_asan_ubsan():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "test_oracle_asan")
    srcs = [os.path.join(ROOT, "tests", "cpp", "test_oracle_asan.c")] + [
        os.path.join(ROOT, "oracle", f) for f in ("orb_oracle.c", "orb_oracle_frame.c", "orb_oracle_voc.c")] + [
        os.path.join(ROOT, "cooperative-orb-slam_amd", "csrc", "synth.c")]
    r = _run(["gcc", "-std=c11", "-ffp-contract=off", *SAN, "-I", os.path.join(ROOT, "oracle"), "-I",
              os.path.join(ROOT, "include"), *srcs, "-lm", "-o", exe])
    assert r.returncode == 0, "build failed"
    r = _run([exe], env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert r.returncode == 0 and "ALL PASS" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_slot_codec_under_asan_ubsan():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "test_slot_asan")
    lib = os.path.join(ROOT, "cooperative-orb-slam_amd", "lib")
    r = _run(["g++", "-std=c++14", *SAN, "-I", os.path.join(ROOT, "tests", "cpp", "cvmin"), "-I",
              os.path.join(ROOT, "tests", "cpp", "mock"), "-I", os.path.join(ROOT, "cooperative-orb-slam_amd", "host"),
              "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "test_slot.cpp"),
              os.path.join(ROOT, "cooperative-orb-slam_amd", "host", "KeyFrameSlot_amd.cc"), "-L", lib, "-lorbamd",
              "-Wl,-rpath," + lib, "-Wl,-rpath,/opt/rocm/lib", "-o", exe])
    assert r.returncode == 0, "build failed"
    # the HIP runtime is not instrumented (and leaks by design at exit): leak checking off
    r = _run([exe], env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", ORBAMD_NO_TORCH="1"))
    assert r.returncode == 0 and "ALL PASS" in r.stdout


def _tsan_build(exe, extra):
    R = ROOT
    H = os.path.join(R, "cooperative-orb-slam_amd", "host")
    lib = os.path.join(R, "cooperative-orb-slam_amd", "lib")
    srcs = [os.path.join(R, "tests", "cpp", "test_kf_cache_tsan.cpp")]
    if "-DWITH_DROPINS" in extra:
        srcs += [os.path.join(H, f) for f in ("ORBextractor.cc", "ORBmatcher_amd.cc", "ORBmatcher_base_amd.cc",
                                              "ORBmatcher_projection_amd.cc", "Frame_stereo_amd.cc",
                                              "MapPoint_distinctive_amd.cc", "Frame_bow_amd.cc", "orbamd_status.cc")]
    return _run(["g++", "-std=c++14", "-O1", "-g", "-fsanitize=thread", "-pthread", *extra, "-I",
                 os.path.join(R, "tests", "cpp", "cvmin"), "-I", os.path.join(R, "tests", "cpp", "mock"), "-I", H, "-I",
                 os.path.join(R, "include"), "-I", os.path.join(R, "cooperative-orb-slam_amd", "csrc"), *srcs, "-L", lib,
                 "-lorbamd", "-Wl,-rpath," + lib, "-Wl,-rpath,/opt/rocm/lib", "-o", exe])


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_concurrent_host_code_under_tsan():
    """ThreadSanitizer over the keyframe cache's LRU books (the product header, three matcher threads racing on
    lookups / inserts / evictions / ForgetKeyFrame) and the C++ drop-ins' shared state from 2 extractor + 3 matcher
    threads (Tracking.cc:767, LocalMapping.cc:268, LoopClosing.cc:267); a canary build with a planted race shows the
    sanitizer reports what it should"""
    os.makedirs(OUT, exist_ok=True)
    canary = os.path.join(OUT, "tsan_canary")
    assert _tsan_build(canary, ["-DTSAN_CANARY"]).returncode == 0, "canary build failed"
    r = _run([canary], env=dict(os.environ, TSAN_OPTIONS="exitcode=0"))
    assert "WARNING: ThreadSanitizer: data race" in r.stderr, "ThreadSanitizer missed the planted race"
    exe = os.path.join(OUT, "test_kf_cache_tsan")
    assert _tsan_build(exe, ["-DWITH_DROPINS"]).returncode == 0, "build failed"
    # ORBAMD_DEVICE=99: every C ABI call fails with ORBX_EDEVICE (no GPU touched, on any machine)
    r = _run([exe], env=dict(os.environ, ORBAMD_DEVICE="99", ORBAMD_NO_TORCH="1", TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "ALL PASS" in r.stdout
    assert "ThreadSanitizer" not in r.stderr
