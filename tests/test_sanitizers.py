"""Host-side sanitizer runs (GPU sanitizers are not available on the pool): the CPU
oracle + synthetic generator under AddressSanitizer/UBSan (tests/cpp/test_oracle_asan.c), and the
C++ keyframe-slot codec (host/KeyFrameSlot_amd.*) under the same sanitizers."""
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
