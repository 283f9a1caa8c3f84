"""Shared test setup: import paths, the `gpu` marker, lazy builds of the native libraries."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cooperative-orb-slam_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "liborbamd.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", PKG, "-j8"])
    olib = os.path.join(ROOT, "oracle", "build", "liborb_oracle.so")
    if not os.path.exists(olib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import orbamd
    return orbamd.load().orbx_device_count() > 0
