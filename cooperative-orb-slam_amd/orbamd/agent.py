"""One agent's per-step work on one GPU: the schedule bench.py times and tests/test_gpu_schedule.py
checks.

A step = B frames already resident in HBM, split over P concurrent extraction+match graphs (own
orbx handle, matcher ctx and HIP stream each):
  * ORBextractor::operator() on every frame (orbx_extract_batch_device);
  * SearchForTriangulation of frame b against frame b-1 of the same graph (one node holding every
    feature, mono, no MapPoints: the BASELINE "BF" configuration);
  * the cooperative exchange: graph 0's frame 0 is this agent's keyframe; its BoW / FeatureVector is
    computed on the device (orbv_transform_batch_device), it is packed into a keyframe slot with its
    MapPoint records (orbx_pack_keyframe_device), all-gathered across the agents (RCCL over xGMI at
    N > 1, a local copy at N = 1), and matched against every agent's slot straight from the receive
    buffer: SearchForTriangulation (orbm_search_for_triangulation_slots_device, LocalMapping) and the
    loop-candidate SearchByBoW(KF,KF) (orbm_search_by_bow_slots_device, LoopClosing).
Stereo (stereo=(mbf, mb), BASELINE configs 3 and 4): every frame is a rectified stereo pair, as the stereo Frame
constructor builds it (ORB_SLAM2.1/src/Frame.cc:80-98): both images extracted (one batch per graph: its left
images, then its right ones), Frame::ComputeStereoMatches on the device-resident pyramids (mvuRight / mvDepth), and
SearchForTriangulation's stereo branch against the previous frame (ORBmatcher.cc:703-749); the keyframe slot carries
mvuRight / mvDepth, so the cross-agent triangulation takes the stereo branch too.
Graphs are staggered: in a staggered step graph p starts extracting once graph p-1 has finished extracting
it, so one graph's FAST overlaps another's latency-bound tail (octree, describe, matcher); the offset is
imposed in the first step of a pass and every 8th step after it (DEFAULT_STAGGER) and persists in between.
The frames live in a pool of `pool` resident batches and consecutive steps process consecutive
batches, so no step's correct output equals the previous step's: a stage that stopped launching
leaves stale results that the self-check (oracle/check_schedule.py) sees.
torch is plumbing only (HBM buffers, streams, torch.distributed); every kernel is liborbamd.so's.
"""
from .device import BatchPipeline

# Graph stagger of the bench schedule: the first step of a pass and every 8th step after it
# (profiles/r03_exp_stagger.log: at the driver's 20 timed steps +1.5 % over staggering every step, whose last
# step drains as a 4-graph chain, and +1.0 % over it in the ~2000-step sustained pass, where a stagger imposed
# only once lets the graphs' phases drift)
DEFAULT_STAGGER = "every8"
SYNTH_VOC_SEED = 7    # the exchange's synthetic vocabulary (ORBvoc.txt's shape; ORBvoc.txt is absent)
KF_LEVELSUP = 4       # KeyFrame::ComputeBoW's levelsup (Frame.cc:400-407)
LOOP_NNRATIO = 0.75   # LoopClosing::ComputeSim3's ORBmatcher(0.75, true) (LoopClosing.cc:239)


def kf_mp_flags(n):
    """Synthetic MapPoint records of the bench keyframe (the slot's MPFLAGS: bit 0 = mvpMapPoints[i] != NULL,
    bit 1 = isBad()): about half of the features carry a MapPoint (the loop-candidate SearchByBoW matches those),
    about 5 % of them bad; the other half are what SearchForTriangulation may triangulate. A fixed hash of the
    feature index, so the oracle check rebuilds them."""
    import numpy as np
    h = (np.arange(n, dtype=np.uint64) * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)
    mp = ((h >> np.uint64(8)) % np.uint64(10)) < np.uint64(5)
    bad = mp & (((h >> np.uint64(20)) % np.uint64(20)) == np.uint64(0))
    return (mp.astype(np.uint8) | (bad.astype(np.uint8) << 1)).astype(np.uint8)


class AgentSchedule:
    def __init__(self, torch, frames_np, width, height, pipes, device=0, rank=0, world=1, allgather=None,
                 stagger=DEFAULT_STAGGER, exchange=True, priorities=None, nfeatures=1000, pool=1,
                 async_exchange=False, stereo=None):
        """frames_np: uint8 [pool*B, H, W] host frames of this agent (copied to HBM once), batch r = frames
        [r*B, (r+1)*B); with stereo=(mbf, mb) uint8 [pool*B, 2, H, W] (left, right image of each frame);
        allgather(out, inp): all-gather of equal-sized device byte tensors across agents (None: no collective,
        only possible at world 1, where the slot is packed in place)."""
        assert len(frames_np) % pool == 0
        assert (frames_np.ndim == 4 and frames_np.shape[1] == 2) == bool(stereo), "stereo frames are [N, 2, H, W]"
        self.stereo = stereo
        self.images_per_frame = 2 if stereo else 1
        B = len(frames_np) // pool
        assert B % pipes == 0, "frames per step must be a multiple of the graph count"
        assert allgather is not None or world == 1
        self.torch, self.W, self.H, self.B, self.P = torch, width, height, B, pipes
        self.sub = B // pipes
        self.pool, self.cursor, self.last_batch = pool, 0, None
        self.rank, self.world, self.allgather = rank, world, allgather
        # stagger: "each" step, "once" (the first step of a pass only) or "everyK" (the first step of a pass and
        # every K-th step after it: the graphs' phase offset is re-imposed periodically, and the other steps carry
        # no cross-graph wait)
        # a "pyr_" / "fast_" prefix staggers graph p behind graph p-1's pyramid / FAST instead of its whole extraction
        self.stagger_stage = 0 if stagger.startswith("pyr_") else 1 if stagger.startswith("fast_") else None
        self.stagger_pyr = self.stagger_stage is not None  # graph p waits for an event inside graph p-1's extraction
        mode = stagger.split("_", 1)[1] if self.stagger_pyr else stagger
        assert mode in ("each", "once", "none") or (mode.startswith("every") and int(mode[5:]) > 0)
        self.stagger, self.exchange_on = mode, exchange
        self.stagger_every = int(mode[5:]) if mode.startswith("every") else 0
        self.pass_step = 0
        dev = torch.device("cuda", device)
        self.dev = dev
        sub = self.sub
        # frames live in a pitched HBM buffer: rows padded to 64 bytes when the width is not a multiple of 4
        # (C4's 1241), so every row starts 4-aligned and the whole-frame pyramid kernel applies
        pitch = width if width % 4 == 0 else (width + 63) // 64 * 64
        self.pitch = pitch
        self.frames = []  # [batch r][graph p] -> device view [sub * images_per_frame, H, W]
        per = self.images_per_frame
        for r in range(pool):
            row = []
            for p in range(pipes):
                buf = torch.zeros((per * sub, height, pitch), dtype=torch.uint8, device=dev)
                view = buf[:, :, :width]
                view.copy_(torch.from_numpy(self.graph_images(frames_np, r, p)).to(dev))
                row.append(view)
            self.frames.append(row)
        self.nfeatures = nfeatures
        self.pipes = [BatchPipeline(torch, width, height, sub, nfeatures=nfeatures, device=device, stereo=stereo)
                      for _ in range(pipes)]
        prio = priorities or [0] * pipes
        self.streams = [torch.cuda.Stream(dev, priority=prio[p]) for p in range(pipes)]
        self.done = [torch.cuda.Event() for _ in range(pipes)]
        self.pyr_done = None
        if self.stagger_pyr:
            from ._lib import load
            lib = load()
            self.pyr_done = [torch.cuda.Event() for _ in range(pipes)]
            for p in range(pipes):
                self.pyr_done[p].record(self.streams[p])  # materialise the HIP event
                assert lib.orbx_set_stage_event(self.pipes[p].ext._h, self.stagger_stage, self.pyr_done[p].cuda_event) == 0
        p0 = self.pipes[0]
        self.slot_bytes = p0.slot_bytes()
        # without a collective (N = 1) the keyframe is packed straight into the receive buffer (no copy);
        # with one (N > 1, or N = 1 under torch.distributed: bench.py --dist) into its own send buffer for
        # an out-of-place all-gather
        self.collective = allgather is not None
        self.all_slots = torch.zeros(world * self.slot_bytes, dtype=torch.uint8, device=dev)
        self.my_slot = (torch.zeros(self.slot_bytes, dtype=torch.uint8, device=dev) if self.collective else
                        self.all_slots)
        S = p0.stride
        self.xmatch = torch.empty((world, S), dtype=torch.int32, device=dev)
        self.xn = torch.zeros(world, dtype=torch.int32, device=dev)
        self.xbow = torch.empty((world, S), dtype=torch.int32, device=dev)
        self.xbn = torch.zeros(world, dtype=torch.int32, device=dev)
        self.pack_err = torch.zeros(16, dtype=torch.int32, device=dev)
        self.meta = p0.meta(0, agent=rank)
        self.ag_events = []
        # async_exchange: the exchange runs on its own stream once graph 0 has extracted the keyframe; it first
        # copies the keyframe's arrays, and only that copy (not the BoW transform, the pack, the all-gather, whose
        # latency at N > 1 includes waiting for the other agents, nor the slot matchers) holds graph 0's next
        # extraction, which overwrites them. Without it the exchange runs in order on graph 0's stream (bench.py:
        # own stream when a collective runs, graph 0's at N = 1, where it measured 0.9 % faster).
        self.xstream = None
        kps, desc, count = p0.kps[0], p0.desc[0], p0.counts[0:1]
        if async_exchange and exchange:
            self.xstream = torch.cuda.Stream(dev)
            self.q_kps = torch.empty_like(p0.kps[0])
            self.q_desc = torch.empty_like(p0.desc[0])
            self.q_count = torch.empty_like(p0.counts[0:1])
            kps, desc, count = self.q_kps, self.q_desc, self.q_count
            self.kf_released = torch.cuda.Event()
            self.kf_pending = False
        self.kf_stereo = (None, None)
        if stereo:
            self.kf_stereo = (p0.uright[0], p0.depth[0])
            if self.xstream is not None:
                self.q_uright, self.q_depth = torch.empty_like(p0.uright[0]), torch.empty_like(p0.depth[0])
                self.kf_stereo = (self.q_uright, self.q_depth)
        self.kf_arrays = (kps, desc, count)
        # the keyframe as a KeyFrame of the map: Frame::ComputeBoW on the device against the vocabulary (a
        # deterministic synthetic one of ORBvoc.txt's shape, k = 10, L = 6: ORBvoc.txt is absent; levelsup 4,
        # KeyFrame::ComputeBoW) and the synthetic MapPoint flags of kf_mp_flags, so the slot carries mBowVec /
        # mFeatVec / the MapPoint records and the receiving agents' loop-candidate SearchByBoW(KF,KF) has work
        if exchange:
            from .exchange import kf_source
            from .vocabulary import L1_NORM, TF_IDF, ORBVocabulary, synth_vocabulary_full
            self.voc_arrays = synth_vocabulary_full(seed=SYNTH_VOC_SEED)
            k, L, par, leaf, vdesc, w = self.voc_arrays
            self.voc = ORBVocabulary.from_arrays(k, L, L1_NORM, TF_IDF, par, leaf, vdesc, w, device=device)
            z = lambda *sh, dt=torch.int32: torch.zeros(*sh, dtype=dt, device=dev)  # noqa: E731
            self.kf_word, self.kf_word_w, self.kf_word_nid = z(S), z(S, dt=torch.float64), z(S)
            self.kf_bow_word, self.kf_bow_val, self.kf_nbow = z(S), z(S, dt=torch.float64), z(1)
            self.kf_fv_node, self.kf_fv_off, self.kf_fv_feat, self.kf_nfv = z(S), z(S + 1), z(S), z(1)
            self.kf_mpf = torch.from_numpy(kf_mp_flags(S)).to(dev)
            self.bow_max_nodes = int(min(S, k ** max(L - KF_LEVELSUP, 0)))
            self.kf_src = kf_source(kps, desc, count, uright=self.kf_stereo[0], depth=self.kf_stereo[1],
                                    mp_flags=self.kf_mpf, bow_word=self.kf_bow_word,
                                    bow_value=self.kf_bow_val, nbow=self.kf_nbow, fv_node=self.kf_fv_node,
                                    fv_off=self.kf_fv_off, fv_feat=self.kf_fv_feat, nfv=self.kf_nfv)

    # ------------------------------------------------------------------------------------------
    def graph_images(self, frames_np, r, p):
        """host images of graph p in pool batch r, in the device batch's order (stereo: the graph's left images,
        then its right ones)"""
        lo = r * self.B + p * self.sub
        f = frames_np[lo:lo + self.sub]
        if not self.stereo:
            return f
        import numpy as np
        return np.ascontiguousarray(np.concatenate([f[:, 0], f[:, 1]]))

    def host_batch(self, frames_np, r):
        """every graph's images of pool batch r back to back (graph order; the ingest leg's pinned source)"""
        import numpy as np
        if not self.stereo:
            return frames_np[r * self.B:(r + 1) * self.B]
        return np.ascontiguousarray(np.concatenate([self.graph_images(frames_np, r, p) for p in range(self.P)]))

    def device_images(self, r, p):
        """the device images graph p extracts in pool batch r ([sub * images_per_frame, H, W] view)"""
        return self.frames[r][p]

    def exchange_stream(self):
        """the stream the exchange runs on"""
        return self.xstream if self.xstream is not None else self.streams[0]

    def exchange(self, ag=None):
        """this agent's keyframe -> BoW -> slot -> all-gather -> cross-agent SearchForTriangulation (LocalMapping's
        CreateNewMapPoints on a received keyframe) and SearchByBoW(KF,KF) (LoopClosing's loop-candidate match,
        ORBmatcher(0.75, true): LoopClosing.cc:239-265) against every agent's slot"""
        from ._lib import check, load
        from .exchange import bow_slots_device, pack_device
        torch = self.torch
        p0 = self.pipes[0]
        st = self.exchange_stream()
        kps, desc, count = self.kf_arrays
        if self.xstream is not None:
            self.xstream.wait_event(self.done[0])  # graph 0 has extracted this step's keyframe (frame 0)
        with torch.cuda.stream(st):
            if self.xstream is not None:
                kps.copy_(p0.kps[0])
                desc.copy_(p0.desc[0])
                count.copy_(p0.counts[0:1])
                if self.stereo:
                    self.q_uright.copy_(p0.uright[0])
                    self.q_depth.copy_(p0.depth[0])
                self.kf_released.record(st)  # graph 0 may overwrite its buffers from here on
                self.kf_pending = True
            S = p0.stride
            check(load().orbv_transform_batch_device(
                self.voc._h, 1, desc.data_ptr(), count.data_ptr(), S, KF_LEVELSUP, self.kf_word.data_ptr(),
                self.kf_word_w.data_ptr(), self.kf_word_nid.data_ptr(), self.kf_bow_word.data_ptr(),
                self.kf_bow_val.data_ptr(), self.kf_nbow.data_ptr(), self.kf_fv_node.data_ptr(),
                self.kf_fv_off.data_ptr(), self.kf_fv_feat.data_ptr(), self.kf_nfv.data_ptr(), st.cuda_stream),
                "orbv_transform_batch_device")
            pack_device(self.kf_src, self.meta, S, self.my_slot, self.pack_err, st.cuda_stream)
            if ag is not None:
                ag[0].record(st)
            if self.collective:
                self.allgather(self.all_slots, self.my_slot)
            if ag is not None:
                ag[1].record(st)
            p0.match_slots(0, self.all_slots, self.world, self.xmatch, self.xn, st.cuda_stream, query=self.kf_src)
            bow_slots_device(p0.mh, self.kf_src, S, self.world, self.all_slots, self.slot_bytes, self.xbow, self.xbn,
                             LOOP_NNRATIO, True, self.bow_max_nodes, st.cuda_stream)

    def step(self, ev=None, xev=None, extract=True, match=True, xchg=True, first=True, batch=None, wait=None, sev=None):
        """enqueue one step over the next pool batch (or `batch`); ev[p] = (start, end) events around graph
        p's matcher, xev around the exchange, sev[p] around graph p's ComputeStereoMatches (stereo); wait: an event
        every graph waits for before extracting, or per graph an event or a list of events (the ingest leg's
        uploads of that graph's frames)"""
        torch = self.torch
        r = self.cursor % self.pool if batch is None else batch
        self.cursor += 1
        self.last_batch = r
        if first:
            self.pass_step = 0
        stagger_now = (self.stagger == "each" or (self.stagger == "once" and first) or
                       (self.stagger_every > 0 and self.pass_step % self.stagger_every == 0))
        self.pass_step += 1
        for p in range(self.P):
            st = self.streams[p].cuda_stream
            if extract:
                if wait is not None:
                    w = wait[p] if isinstance(wait, (list, tuple)) else wait
                    for e in (w if isinstance(w, (list, tuple)) else (w,)):
                        self.streams[p].wait_event(e)
                if p > 0 and stagger_now:
                    self.streams[p].wait_event(self.pyr_done[p - 1] if self.stagger_pyr else self.done[p - 1])
                if p == 0 and self.xstream is not None and self.kf_pending:
                    self.streams[0].wait_event(self.kf_released)  # the previous exchange has copied the keyframe
                self.pipes[p].extract(self.frames[r][p], st, stereo=False)
                if self.stereo:  # Frame::ComputeStereoMatches of the graph's pairs (Frame.cc:92)
                    if sev is not None:
                        sev[p][0].record(self.streams[p])
                    self.pipes[p].stereo_matches(st)
                    if sev is not None:
                        sev[p][1].record(self.streams[p])
                self.done[p].record(self.streams[p])
            if match:
                if ev is not None:
                    ev[p][0].record(self.streams[p])
                self.pipes[p].match_pairs(st)
                if ev is not None:
                    ev[p][1].record(self.streams[p])
        if xchg and self.exchange_on:
            if self.xstream is not None:
                self.xstream.wait_event(self.done[0])  # before xev[0]: the exchange's time excludes this wait
            if xev is not None:
                xev[0].record(self.exchange_stream())
            ag = None
            if xev is not None:
                ag = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                self.ag_events.append(ag)
            self.exchange(ag)
            if xev is not None:
                xev[1].record(self.exchange_stream())

    # ------------------------------------------------------------------------------------------
    def check_errors(self):
        """Device-side consistency flags of every graph (extraction: octree capacity / root index;
        matcher: slot validation) and of the keyframe pack; raises RuntimeError on any."""
        for p, pp in enumerate(self.pipes):
            st = self.streams[p].cuda_stream
            pp.check_error(st)
            pp.check_match_error(st)
        self.torch.cuda.synchronize(self.dev)
        if int(self.pack_err.max().item()) != 0:
            raise RuntimeError("keyframe pack clamped a count (slot capacity)")

    def frame_index(self, p, b):
        """index into the host frames (frames_np) of frame b of graph p in the last step's batch"""
        return (self.last_batch or 0) * self.B + p * self.sub + b

    def frame_results(self, p, b):
        """(keypoints, descriptors, match12 vs frame b-1 of the same graph) of frame b of graph p (stereo: its left
        image)"""
        return self.pipes[p].host_results(b)

    def stereo_results(self, p, b):
        """stereo: ((right keypoints, right descriptors), (mvuRight, mvDepth, kept)) of frame b of graph p"""
        pp = self.pipes[p]
        return pp.host_keypoints(self.sub + b), pp.host_stereo(b)

    def exchange_results(self):
        """(triangulation rows [world, n], counts [world], SearchByBoW rows [world, n], counts [world]) of this agent's
        keyframe against every agent's slot"""
        n = int(self.pipes[0].counts[0].item())
        return (self.xmatch[:, :n].cpu().numpy(), self.xn.cpu().numpy(), self.xbow[:, :n].cpu().numpy(),
                self.xbn.cpu().numpy())

    def close(self):
        if self.pyr_done is not None:
            from ._lib import load
            for pp in self.pipes:
                load().orbx_set_stage_event(pp.ext._h, self.stagger_stage, None)
        for pp in self.pipes:
            pp.close()
        if getattr(self, "voc", None) is not None:
            self.voc.close()
            self.voc = None
