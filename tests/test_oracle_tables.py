"""Oracle constant tables vs values derived from the reference source (no GPU).

The reference has no tests; these known answers come from executing the
reference's constructor logic by hand / from its source text:
  umax                 ORBextractor.cc:454-469
  mnFeaturesPerLevel   ORBextractor.cc:435-446
  bit_pattern_31_      ORBextractor.cc:150-408 (FNV-1a of the 1024 int8 values, tools/gen_pattern.py)
  level sizes          ORBextractor.cc:1111-1112
"""
import os
import re

import numpy as np
import pytest

import oracle_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_umax():
    t = oracle_py.OracleExtractor().tables()
    assert list(t["umax"]) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


@pytest.mark.parametrize("nf,expect", [
    (1000, [217, 181, 151, 126, 105, 87, 73, 60]),
    (2000, [434, 362, 302, 251, 209, 175, 145, 122]),
    (1200, [261, 217, 181, 151, 126, 105, 87, 72]),
])
def test_features_per_level(nf, expect):
    assert list(oracle_py.OracleExtractor(nf).tables()["nfeat"]) == expect


def test_scale_tables_double_member():
    # mvScaleFactor[i] = mvScaleFactor[i-1]*scaleFactor with scaleFactor a double member (ORBextractor.h:100)
    t = oracle_py.OracleExtractor().tables()
    s = [np.float32(1)]
    for _ in range(7):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(1.2))))
    assert np.array_equal(t["scale"], np.array(s, np.float32))
    assert np.array_equal(t["sigma2"], (np.array(s, np.float32) * np.array(s, np.float32)).astype(np.float32))


def _decode_header(path, name):
    txt = open(path).read()
    body = txt[txt.index(name):]
    body = body[body.index("{") + 1: body.index("}")]
    vals = [int(v, 16) for v in re.findall(r"0x[0-9a-f]{2}", body)]
    return np.array(vals, np.uint8).astype(np.int8)


def test_pattern_tables_match_reference_hash():
    aos = _decode_header(os.path.join(ROOT, "oracle", "orb_pattern_data.h"), "orb_oracle_pattern_u8")
    soa = _decode_header(os.path.join(ROOT, "cooperative-orb-slam_amd", "csrc", "orb_pattern.h"), "orbx_pattern_soa_u8")
    assert aos.size == soa.size == 1024
    assert np.array_equal(aos.reshape(256, 4).T.reshape(-1), soa)
    h = 0xCBF29CE484222325
    for v in aos.astype(np.int64):
        h ^= int(v) & 0xFF
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    assert h == 0x1F34D6CD6D716873 and int(aos.astype(np.int64).sum()) == -406
    # first/last pairs as printed in ORBextractor.cc:152,407
    assert list(aos[:4]) == [8, -3, 9, 5] and list(aos[-4:]) == [-1, -6, 0, -11]


def test_gaussian_kernel_q8():
    k, s = oracle_py.gauss_kernel_q8()
    assert list(k) == [18, 34, 49, 55, 49, 34, 18] and s == 257


@pytest.mark.parametrize("W,H,sizes", [
    (640, 480, [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)]),
    (752, 480, [(752, 480), (627, 400), (522, 333), (435, 278), (363, 231), (302, 193), (252, 161), (210, 134)]),
    (1241, 376, [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151), (416, 126), (346, 105)]),
])
def test_level_sizes(W, H, sizes):
    orc = oracle_py.OracleExtractor()
    orc(np.zeros((H, W), np.uint8))
    assert [orc.level_size(l) for l in range(8)] == sizes
