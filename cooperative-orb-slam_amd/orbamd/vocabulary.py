"""ORBVocabulary -- the DBoW2 vocabulary transform behind Frame::ComputeBoW (Frame.cc:400-407)
over the C ABI (orbv_*). DBoW2 is not vendored in the reference: the ORB-SLAM2 fork's published
algorithm is restated (parity unpinned).
"""
import ctypes as C

import numpy as np

from ._lib import check, load

# DBoW2 enums
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)
TF_IDF, TF, IDF, BINARY = range(4)


class ORBVocabulary:
    """TemplatedVocabulary<FORB::TDescriptor, FORB> on the device.

    ORBVocabulary(path) loads ORBvoc.txt-format text (loadFromTextFile); ORBVocabulary.from_arrays
    takes the node lines directly."""

    def __init__(self, path=None, device=0, _handle=None):
        self._lib = load()
        if _handle is not None:
            self._h = _handle
        else:
            h = C.c_void_p()
            check(self._lib.orbv_load_text(str(path).encode(), device, C.byref(h)), "orbv_load_text")
            self._h = h

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight, device=0):
        lib = load()
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        check(lib.orbv_create(k, L, scoring, weighting, len(parent), parent.ctypes.data, is_leaf.ctypes.data,
                              desc.ctypes.data, weight.ctypes.data, device, C.byref(h)), "orbv_create")
        return cls(_handle=h)

    def info(self):
        k, L, n, w = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        check(self._lib.orbv_info(self._h, C.byref(k), C.byref(L), C.byref(n), C.byref(w)), "orbv_info")
        return {"k": k.value, "L": L.value, "nodes": n.value, "words": w.value}

    def transform(self, descriptors, levelsup=4):
        """Returns (BowVector as (word ids uint32, values float64), FeatureVector as dict node -> feature list)."""
        d = np.ascontiguousarray(descriptors if descriptors is not None else np.zeros((0, 32)), np.uint8)
        n = len(d)
        bw = np.empty(max(n, 1), np.uint32)
        bv = np.empty(max(n, 1), np.float64)
        fn = np.empty(max(n, 1), np.uint32)
        fo = np.empty(n + 1, np.int32)
        ff = np.empty(max(n, 1), np.int32)
        nb, nf = C.c_int(), C.c_int()
        check(self._lib.orbv_transform(self._h, d.ctypes.data, n, levelsup, bw.ctypes.data, bv.ctypes.data,
                                       C.byref(nb), fn.ctypes.data, fo.ctypes.data, ff.ctypes.data, C.byref(nf)),
              "orbv_transform")
        fv = {int(fn[i]): ff[fo[i]:fo[i + 1]].tolist() for i in range(nf.value)}
        return (bw[:nb.value].copy(), bv[:nb.value].copy()), fv

    def close(self):
        if getattr(self, "_h", None):
            self._lib.orbv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_vocabulary(k=10, L=4, seed=0, flip_bits=40, zero_weight_frac=0.02, ragged=False):
    """A deterministic synthetic vocabulary in loadFromTextFile's node order (breadth first; ORBvoc.txt is
    absent here): children = parent descriptor with random bit flips, leaves flagged, idf-like weights
    (a few zero: 'stopped' words). ragged=True varies the child counts and stops some branches early.
    Returns (k, L, parent, is_leaf, desc, weight) for ORBVocabulary.from_arrays / to_text."""
    rng = np.random.default_rng(seed)
    parent, leaf, desc, weight = [], [], [], []
    root_desc = rng.integers(0, 256, 32, dtype=np.uint8)
    frontier = [(0, root_desc, 0)]  # (node id, descriptor, depth)
    nid = 0
    while frontier:
        nxt = []
        for pid, pd, depth in frontier:
            if depth >= L:
                continue
            nc = int(rng.integers(2, k + 1)) if ragged else k
            if ragged and depth > 0 and rng.random() < 0.1:
                continue  # this node stays childless (a leaf by Node::isLeaf)
            for _ in range(nc):
                d = pd.copy() if depth else rng.integers(0, 256, 32, dtype=np.uint8)
                if depth:
                    for p in rng.choice(256, flip_bits, replace=False):
                        d[p >> 3] ^= np.uint8(1 << (p & 7))
                nid += 1
                is_leaf = depth + 1 == L
                parent.append(pid)
                leaf.append(1 if is_leaf else 0)
                desc.append(d)
                w = 0.0 if (is_leaf and rng.random() < zero_weight_frac) else float(rng.uniform(0.1, 8.0))
                weight.append(w)
                nxt.append((nid, d, depth + 1))
        frontier = nxt
    return k, L, np.array(parent, np.int32), np.array(leaf, np.uint8), np.array(desc, np.uint8), \
        np.array(weight, np.float64)


def synth_vocabulary_full(k=10, L=6, seed=0):
    """A full k-ary synthetic vocabulary of depth L (ORBvoc.txt's shape is k=10, L=6: 1,111,110 nodes),
    vectorised: children = parent descriptor XOR (r1 & r2 & r3) (about 32 flipped bits), breadth-first
    node order, idf-like weights on every node. For benchmarks; same return layout as synth_vocabulary."""
    rng = np.random.default_rng(seed)
    parents, leaves, descs, weights = [], [], [], []
    level_desc = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    level_ids = np.arange(1, k + 1)
    parents.append(np.zeros(k, np.int32))
    next_id = k + 1
    for depth in range(1, L + 1):
        n = len(level_ids)
        leaves.append(np.full(n, 1 if depth == L else 0, np.uint8))
        descs.append(level_desc)
        weights.append(rng.uniform(0.1, 8.0, n))
        if depth == L:
            break
        child_desc = np.repeat(level_desc, k, axis=0)
        m = rng.integers(0, 256, child_desc.shape, dtype=np.uint8)
        m &= rng.integers(0, 256, child_desc.shape, dtype=np.uint8)
        m &= rng.integers(0, 256, child_desc.shape, dtype=np.uint8)
        child_desc ^= m
        child_ids = np.arange(next_id, next_id + n * k)
        parents.append(np.repeat(level_ids, k).astype(np.int32))
        next_id += n * k
        level_desc, level_ids = child_desc, child_ids
    return k, L, np.concatenate(parents), np.concatenate(leaves), np.concatenate(descs), np.concatenate(weights)


def to_text(path, k, L, parent, is_leaf, desc, weight, scoring=L1_NORM, weighting=TF_IDF):
    """Writes the ORBvoc.txt text format (saveToTextFile of the ORB-SLAM2 DBoW2 fork)."""
    with open(path, "w") as f:
        f.write("%d %d %d %d\n" % (k, L, scoring, weighting))
        for p, lf, d, w in zip(parent, is_leaf, desc, weight):
            f.write("%d %d %s %s\n" % (p, lf, " ".join(str(int(x)) for x in d), repr(float(w))))
