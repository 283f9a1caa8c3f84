"""Device-resident batch pipeline (torch tensors as HBM buffers, HIP stream from torch).

One "step" of the hot path over a batch of B frames already in HBM:
  orbx_extract_batch_device  -> keypoints/descriptors/counts per frame
  orbm_triangulation_bf_batch_device -> SearchForTriangulation(frame b, frame b-1 mod B)
torch is plumbing only (allocation, streams, torch.distributed); all compute is in
liborbamd.so.
"""
import ctypes as C

import numpy as np

from ._lib import check, load
from .extractor import ORBextractor

# camera of the reference config (ORB_SLAM2/my.yaml:8-11)
FX, FY, CX, CY = 715.092024, 719.025258, 334.298489, 256.326097

# stereo rigs of the BASELINE stereo configs: Camera.bf and the baseline mb = mbf / fx (Frame.cc:501-503, Tracking.cc
# reads Camera.bf). EuRoC (EuRoC.yaml: fx 435.2047, bf 47.90639384423901) and KITTI 00-02 (KITTI00-02.yaml: fx 718.856,
# bf 386.1448)
STEREO_RIGS = {"euroc": (47.90639384423901, 47.90639384423901 / 435.2046959714599),
               "kitti": (386.1448, 386.1448 / 718.856)}


def default_geometry():
    """KF2 pose relative to KF1: R = I, t = (0.05, 0, 0.01); returns (F12, ex, ey)."""
    from .matcher import compute_f12, epipole
    K = np.array([[FX, 0, CX], [0, FY, CY], [0, 0, 1]], np.float32)
    R1 = np.eye(3, dtype=np.float32)
    t1 = np.zeros(3, np.float32)
    R2 = np.eye(3, dtype=np.float32)
    t2 = np.array([0.05, 0.0, 0.01], np.float32)
    F12 = compute_f12(R1, t1, R2, t2, K, K)
    Cw = -R1.T @ t1  # KF1 camera centre
    ex, ey = epipole(R2, t2, Cw, FX, FY, CX, CY)
    return F12, ex, ey


class BatchPipeline:
    """Extract + match over batches of frames on one GPU.

    stereo=(mbf, mb): every frame is a rectified stereo pair (the stereo Frame constructor, ORB_SLAM2.1/src/Frame.cc:
    80-98): the extraction batch holds the B left images (images 0..B-1) and then the B right images (B..2B-1),
    one orbx_extract_batch_device over all 2B (the two ORBextractor instances share the parameters,
    Tracking.cc:119-125); Frame::ComputeStereoMatches gives every left keypoint its mvuRight / mvDepth
    (orbx_stereo_matches_batch_device), and SearchForTriangulation of frame b against b-1 takes the stereo branch
    (orbm_triangulation_bf_stereo_batch_device)."""

    def __init__(self, torch, width=640, height=480, batch=64, nfeatures=1000, scale=1.2, nlevels=8, ini=20, mini=7,
                 device=0, check_ori=False, stereo=None):
        self.torch = torch
        self.W, self.H, self.B = width, height, batch
        self.stereo = stereo
        self.nimg = 2 * batch if stereo else batch
        nimg = self.nimg
        self.ext = ORBextractor(nfeatures, scale, nlevels, ini, mini, device=device, max_width=width,
                                max_height=height, max_batch=nimg)
        self.lib = load()
        self.stride = self.ext.max_keypoints(width, height)
        dev = torch.device("cuda", device)
        self.dev = dev
        self.kps = torch.empty((nimg, self.stride, 6), dtype=torch.float32, device=dev)
        self.desc = torch.empty((nimg, self.stride, 32), dtype=torch.uint8, device=dev)
        self.counts = torch.zeros(nimg, dtype=torch.int32, device=dev)
        self.match = torch.empty((batch, self.stride), dtype=torch.int32, device=dev)
        self.nmatch = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.q1 = torch.arange(batch, dtype=torch.int32, device=dev)
        self.q2 = ((self.q1 + batch - 1) % batch).to(torch.int32)
        if stereo:
            self.uright = torch.empty((batch, self.stride), dtype=torch.float32, device=dev)
            self.depth = torch.empty((batch, self.stride), dtype=torch.float32, device=dev)
            self.nstereo = torch.zeros(batch, dtype=torch.int32, device=dev)
            self.fr = (self.q1 + batch).to(torch.int32)
        h = C.c_void_p()
        check(self.lib.orbm_create(device, C.byref(h)), "orbm_create")
        self.mh = h
        self.F12, self.ex, self.ey = default_geometry()
        self.scale = self.ext.GetScaleFactors()
        self.sigma2 = self.ext.GetScaleSigmaSquares()
        self.check_ori = int(check_ori)

    def stream_ptr(self):
        return self.torch.cuda.current_stream(self.dev).cuda_stream

    def extract(self, frames, stream=None, stereo=True):
        """frames: [nimg, H, W] device images (stereo: the B left images, then the B right ones); a stereo pipeline
        then runs ComputeStereoMatches for every pair on the same stream (stereo=False: the caller does)"""
        st = self.stream_ptr() if stream is None else stream
        self.ext.extract_batch_device(frames, self.kps, self.desc, self.counts, st)
        if self.stereo and stereo:
            self.stereo_matches(st)

    def stereo_matches(self, stream=None):
        """Frame::ComputeStereoMatches of every pair (left image b, right image B + b) on the device"""
        st = self.stream_ptr() if stream is None else stream
        mbf, mb = self.stereo
        check(self.lib.orbx_stereo_matches_batch_device(
            self.ext._h, self.ext._h, self.B, self.q1.data_ptr(), self.fr.data_ptr(), self.kps.data_ptr(),
            self.desc.data_ptr(), self.counts.data_ptr(), self.kps.data_ptr(), self.desc.data_ptr(),
            self.counts.data_ptr(), self.stride, float(mbf), float(mb), self.uright.data_ptr(), self.depth.data_ptr(),
            self.nstereo.data_ptr(), st), "orbx_stereo_matches_batch_device")

    def check_error(self, stream=None):
        st = self.stream_ptr() if stream is None else stream
        check(self.lib.orbx_check_error(self.ext._h, st), "orbx_check_error")

    def match_pairs(self, stream=None):
        st = self.stream_ptr() if stream is None else stream
        F = np.ascontiguousarray(self.F12.reshape(9))
        if self.stereo:
            check(self.lib.orbm_triangulation_bf_stereo_batch_device(
                self.mh, self.B, self.q1.data_ptr(), self.q2.data_ptr(), self.kps.data_ptr(), self.desc.data_ptr(),
                self.counts.data_ptr(), self.uright.data_ptr(), self.stride, F.ctypes.data, self.ex, self.ey,
                len(self.scale), self.scale.ctypes.data, self.sigma2.ctypes.data, 0, self.check_ori,
                self.match.data_ptr(), self.nmatch.data_ptr(), st), "orbm_triangulation_bf_stereo_batch_device")
            return
        check(self.lib.orbm_triangulation_bf_batch_device(
            self.mh, self.B, self.q1.data_ptr(), self.q2.data_ptr(), self.kps.data_ptr(), self.desc.data_ptr(),
            self.counts.data_ptr(), self.stride, F.ctypes.data, self.ex, self.ey, len(self.scale),
            self.scale.ctypes.data, self.sigma2.ctypes.data, self.check_ori, self.match.data_ptr(),
            self.nmatch.data_ptr(), st), "orbm_triangulation_bf_batch_device")

    def bow(self, vocabulary, levelsup=4, stream=None):
        """Frame::ComputeBoW of every extracted frame on the device (orbv_transform_batch_device); the
        FeatureVectors stay in self.fv_node / fv_off / fv_feat / nfv for match_pairs_nodes."""
        torch, dev, B, S = self.torch, self.dev, self.B, self.stride
        if getattr(self, "_bow_bufs", None) is None:
            z = lambda *sh, dt=torch.int32: torch.zeros(*sh, dtype=dt, device=dev)  # noqa: E731
            self.word, self.word_w, self.word_nid = z(B, S), z(B, S, dt=torch.float64), z(B, S)
            self.bow_word, self.bow_val, self.nbow = z(B, S), z(B, S, dt=torch.float64), z(B)
            self.fv_node, self.fv_off, self.fv_feat, self.nfv = z(B, S), z(B, S + 1), z(B, S), z(B)
            self._bow_bufs = True
        st = self.stream_ptr() if stream is None else stream
        check(self.lib.orbv_transform_batch_device(
            vocabulary._h, B, self.desc.data_ptr(), self.counts.data_ptr(), S, levelsup, self.word.data_ptr(),
            self.word_w.data_ptr(), self.word_nid.data_ptr(), self.bow_word.data_ptr(), self.bow_val.data_ptr(),
            self.nbow.data_ptr(), self.fv_node.data_ptr(), self.fv_off.data_ptr(), self.fv_feat.data_ptr(),
            self.nfv.data_ptr(), st), "orbv_transform_batch_device")
        info = vocabulary.info()
        self.max_nodes = int(min(S, info["k"] ** max(info["L"] - levelsup, 0)))

    def match_pairs_nodes(self, stream=None):
        """SearchForTriangulation over the common BoW nodes of each pair (after bow())."""
        st = self.stream_ptr() if stream is None else stream
        F = np.ascontiguousarray(self.F12.reshape(9))
        check(self.lib.orbm_triangulation_nodes_batch_device(
            self.mh, self.B, self.q1.data_ptr(), self.q2.data_ptr(), self.kps.data_ptr(), self.desc.data_ptr(),
            self.counts.data_ptr(), self.stride, self.fv_node.data_ptr(), self.fv_off.data_ptr(),
            self.fv_feat.data_ptr(), self.nfv.data_ptr(), self.max_nodes, F.ctypes.data, self.ex, self.ey,
            len(self.scale), self.scale.ctypes.data, self.sigma2.ctypes.data, self.check_ori, self.match.data_ptr(),
            self.nmatch.data_ptr(), st), "orbm_triangulation_nodes_batch_device")

    def search_by_bow_pairs(self, mode, qf, cf, mp_flags, nnratio, check_ori, out, nmatches, stream=None):
        """SearchByBoW over the device FeatureVectors of bow(): mode 1 = (KF,KF), 0 = (KF,F); qf / cf int32
        cuda [npairs]; mp_flags uint8 cuda [B, stride] (bit 0 MapPoint, bit 1 bad); out int32 [npairs, stride]."""
        st = self.stream_ptr() if stream is None else stream
        check(self.lib.orbm_search_by_bow_batch_device(
            self.mh, int(qf.numel()), int(mode), qf.data_ptr(), cf.data_ptr(), self.kps.data_ptr(), self.desc.data_ptr(),
            self.counts.data_ptr(), self.stride, mp_flags.data_ptr(), self.fv_node.data_ptr(), self.fv_off.data_ptr(),
            self.fv_feat.data_ptr(), self.nfv.data_ptr(), self.max_nodes, float(nnratio), int(check_ori),
            out.data_ptr(), nmatches.data_ptr(), st), "orbm_search_by_bow_batch_device")

    def step(self, frames, stream=None):
        self.extract(frames, stream)
        self.match_pairs(stream)

    # ---- cross-agent exchange (include/orbslam_amd.h "Cross-agent keyframe slot") ----
    def slot_bytes(self):
        return int(self.lib.orbx_slot_bytes(self.stride))

    def meta(self, frame_idx=0, agent=0):
        """orbx_kf_meta of frame frame_idx as a keyframe of agent `agent` (camera of my.yaml, the
        extractor's scale tables, identity pose)."""
        from .exchange import make_meta
        inv = self.ext.GetInverseScaleSigmaSquares()
        K = np.array([[FX, 0, CX], [0, FY, CY], [0, 0, 1]], np.float32)
        return make_meta(agent=agent, mnId=frame_idx, nlevels=len(self.scale), scale=self.scale, sigma2=self.sigma2,
                         inv_sigma2=inv, scale_factor=self.ext.GetScaleFactor(), K=K, width=self.W, height=self.H)

    def kf_source(self, frame_idx, with_bow=False, uright=None, depth=None, mp_flags=None, mp_pos=None):
        """orbx_kf_source of frame frame_idx's device arrays (its BoW / FeatureVector from bow() with
        with_bow; optional per-keypoint uright/depth/MapPoint device tensors)."""
        from .exchange import kf_source
        f, S = frame_idx, self.stride
        if self.stereo and uright is None:  # a stereo keyframe carries its mvuRight / mvDepth
            uright, depth = self.uright[f], self.depth[f]
        kw = {}
        if with_bow:
            kw = dict(bow_word=self.bow_word[f], bow_value=self.bow_val[f], nbow=self.nbow[f:f + 1],
                      fv_node=self.fv_node[f], fv_off=self.fv_off[f], fv_feat=self.fv_feat[f], nfv=self.nfv[f:f + 1])
        return kf_source(self.kps[f], self.desc[f], self.counts[f:f + 1], uright=uright, depth=depth,
                         mp_flags=mp_flags, mp_pos=mp_pos, **kw)

    def pack(self, frame_idx, slot, meta, stream=None, with_bow=False, err=None, src=None):
        """orbx_pack_keyframe_device of frame frame_idx into the device slot."""
        from .exchange import pack_device
        st = self.stream_ptr() if stream is None else stream
        src = self.kf_source(frame_idx, with_bow) if src is None else src
        pack_device(src, meta, self.stride, slot, err, st)

    def match_slots(self, frame_idx, slots, nref, out_match, out_n, stream=None, use_bow=False, geoms=None,
                    query=None):
        """Cross-agent SearchForTriangulation of frame frame_idx against nref received slots
        (orbm_search_for_triangulation_slots_device); geoms = per-slot (F12, ex, ey), default the bench
        geometry for every slot."""
        from .exchange import match_slots_device, slot_geoms
        st = self.stream_ptr() if stream is None else stream
        if geoms is None:
            if getattr(self, "_geo_cache", (None, None))[0] != nref:
                self._geo_cache = (nref, slot_geoms([(self.F12, self.ex, self.ey)] * nref))
            geoms = self._geo_cache[1]
        q = self.kf_source(frame_idx, use_bow) if query is None else query
        match_slots_device(self.mh, q, self.stride, nref, slots, self.slot_bytes(), geoms, out_match, out_n,
                           use_bow=use_bow, max_nodes=getattr(self, "max_nodes", 0) if use_bow else 0, stream=st)

    def check_match_error(self, stream=None):
        st = self.stream_ptr() if stream is None else stream
        check(self.lib.orbm_check_error(self.mh, st), "orbm_check_error")

    def host_results(self, b):
        """(keypoints structured array, descriptors uint8 [n,32], match12 int32 [n]) of frame b (stereo: its left
        image)."""
        k, d = self.host_keypoints(b)
        m = self.match[b, :len(k)].cpu().numpy()
        return k, d, m

    def host_keypoints(self, i):
        """(keypoints, descriptors) of extraction image i (stereo: i >= B is the right image of frame i - B)"""
        from .extractor import kp_dtype
        n = int(self.counts[i].item())
        k = self.kps[i, :n].cpu().numpy().copy().view(np.uint8).view(kp_dtype).reshape(n)
        d = self.desc[i, :n].cpu().numpy()
        return k, d

    def host_stereo(self, b):
        """(mvuRight float32 [n], mvDepth float32 [n], stereo matches kept) of stereo frame b"""
        n = int(self.counts[b].item())
        return (self.uright[b, :n].cpu().numpy(), self.depth[b, :n].cpu().numpy(), int(self.nstereo[b].item()))

    def close(self):
        if getattr(self, "mh", None):
            self.lib.orbm_destroy(self.mh)
            self.mh = None
        self.ext.close()
