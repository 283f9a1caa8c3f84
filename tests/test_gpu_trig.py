"""GPU: the device restatement of glibc sinf/cosf (orb_math.h) equals the host libm on a large
sample of [0, 2*pi] -- every 64th float bit pattern (17M values) plus dense windows around
the quadrant-reduction and small-argument thresholds. (The exhaustive CPU proof of the same
algorithm is tools/check_trig.c.)"""
import numpy as np
import pytest

import oracle_py
import orbamd

pytestmark = pytest.mark.gpu


def test_device_sincos_equals_host_libm():
    torch = pytest.importorskip("torch")
    hi = np.float32(360.0) * np.float32(np.pi / 180.0)
    top = int(np.array([hi], np.float32).view(np.uint32)[0])
    bits = [np.arange(0, top + 1, 64, dtype=np.uint32)]
    for centre in (np.pi / 4, 3 * np.pi / 4, 5 * np.pi / 4, 7 * np.pi / 4, np.pi / 2, np.pi, 1.5 * np.pi, 2 * np.pi,
                   2.0 ** -12, 0.75, 0.8125):
        c = int(np.array([centre], np.float32).view(np.uint32)[0])
        bits.append(np.arange(c - 50000, c + 50000, dtype=np.uint32))
    x = np.unique(np.concatenate(bits)).view(np.float32)
    x = x[(x >= 0) & (x <= hi)]
    hs, hc = oracle_py.sincosf(x)
    dx = torch.from_numpy(x).cuda()
    ds = torch.empty_like(dx)
    dc = torch.empty_like(dx)
    lib = orbamd.load()
    assert lib.orbx_selftest_sincosf(dx.data_ptr(), ds.data_ptr(), dc.data_ptr(), x.size, 0) == 0
    torch.cuda.synchronize()
    gs, gc = ds.cpu().numpy(), dc.cpu().numpy()
    bad_s = np.nonzero(gs.view(np.uint32) != hs.view(np.uint32))[0]
    bad_c = np.nonzero(gc.view(np.uint32) != hc.view(np.uint32))[0]
    assert bad_s.size == 0, (x.size, x[bad_s[:5]])
    assert bad_c.size == 0, (x.size, x[bad_c[:5]])
