"""GPU: the exact schedule bench.py times (orbamd.agent.AgentSchedule) checked against the oracle.

The headline configuration: 3072 frames per step as 3 staggered 1024-frame graphs on 3 streams (bench.py's
default; the round-4 shape, 4 x 256 frames, beside it), with the keyframe-slot exchange; every graph's device
error flags, then EVERY frame's keypoints and
descriptors (raw bits), every frame's SearchForTriangulation row against its predecessor, and the
cross-agent match row are compared with the oracle (ORBextractor.cc:1043-1105,
ORBmatcher.cc:657-823). The BASELINE configs C3 (752x480, 1200 features) and C4 (1241x376, 2000
features) run the same schedule on smaller batches, and as the stereo frames those configs name."""
import pytest

import orbamd
from check_schedule import check_schedule

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,nf,B,P,stagger,async_x", [(640, 480, 1000, 3072, 3, "every8", False),
                                                         (640, 480, 1000, 1024, 4, "every8", False),
                                                         (640, 480, 1000, 1024, 4, "each", False),
                                                         (640, 480, 1000, 1024, 4, "every8", True),
                                                         (752, 480, 1200, 128, 2, "every8", False),
                                                         (1241, 376, 2000, 128, 2, "every8", False)])
def test_bench_schedule_bit_exact(W, H, nf, B, P, stagger, async_x):
    torch = pytest.importorskip("torch")
    from orbamd.agent import AgentSchedule, DEFAULT_STAGGER
    assert DEFAULT_STAGGER == "every8"  # bench.py's default (--stagger)
    frames = orbamd.synth_frames(0, 0, B, W, H)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, nfeatures=nf, stagger=stagger, async_exchange=async_x)
    sched.step()                   # warmup (the first step also builds the geometry tables; staggered)
    sched.step(first=False)        # free-running under every8, staggered under each
    sched.step(first=False)        # the checked step (with async_x graph 0 first waits for the previous exchange's copy)
    torch.cuda.synchronize()
    sched.check_errors()
    sub = B // P
    samples = [(p, b) for p in range(P) for b in range(sub)]  # every frame
    res = check_schedule(sched, frames, samples=samples, nfeatures=nf)
    assert res["bit_exact"], res["mismatches"]
    assert res["checked_frames"] == B and res["checked_slots"] == 1
    assert res["slot_bow_matches"][0] > 100  # SearchByBoW(KF,KF) of the keyframe against its own slot
    assert all(int(pp.nmatch.min().item()) > 0 for pp in sched.pipes)
    sched.close()


@pytest.mark.parametrize("cfg,B,P,async_x", [("c3", 256, 2, False), ("c4", 128, 2, False), ("c3", 192, 3, True)])
def test_stereo_schedule_bit_exact(cfg, B, P, async_x):
    """BASELINE configs 3 and 4 as stereo frames (bench.py --config c3 / c4): every frame's left and right
    keypoints / descriptors, mvuRight / mvDepth (raw bits) and kept count of ComputeStereoMatches (Frame.cc:471-645),
    the stereo SearchForTriangulation row against its predecessor (ORBmatcher.cc:703-749) and the cross-agent rows of
    the stereo keyframe slot, against the oracle"""
    torch = pytest.importorskip("torch")
    import numpy as np
    import bench
    from orbamd.agent import AgentSchedule
    from orbamd.device import STEREO_RIGS
    c = bench.CONFIGS[cfg]
    W, H, nf, rig = c["W"], c["H"], c["nfeatures"], STEREO_RIGS[c["stereo"]]
    frames = np.stack([orbamd.synth_frames(0, 0, B, W, H, scene=0),
                       orbamd.synth_frames(0, 0, B, W, H, dx=c["dx"], scene=0)], axis=1)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, nfeatures=nf, async_exchange=async_x, stereo=rig)
    for i in range(3):
        sched.step(first=i == 0)
    torch.cuda.synchronize()
    sched.check_errors()
    samples = [(p, b) for p in range(P) for b in range(B // P)]  # every frame
    res = check_schedule(sched, frames, samples=samples, nfeatures=nf)
    assert res["bit_exact"], res["mismatches"]
    assert res["checked_frames"] == B and res["checked_slots"] == 1
    for pp in sched.pipes:  # the stereo branch has work: most left keypoints find their right partner
        assert int(pp.nstereo.min().item()) > int(pp.counts[:pp.B].min().item()) // 4
        assert int(pp.nmatch.min().item()) > 0
    sched.close()


@pytest.mark.parametrize("stage", [2, 16])  # fast_cells, describe (orbx_debug_skip_stages bits)
def test_skipped_stage_fails_the_self_check(stage):
    """The bench's stale-output guard: with a 2-batch frame pool a stage that stops launching leaves the
    previous step's (different) outputs and the oracle check fails; with one repeated batch it would not."""
    torch = pytest.importorskip("torch")
    from orbamd.agent import AgentSchedule
    W, H, B, P = 640, 480, 64, 2
    lib = orbamd.load()
    for pool in (2, 1):
        frames = orbamd.synth_frames(0, 0, pool * B, W, H)
        sched = AgentSchedule(torch, frames, W, H, P, device=0, nfeatures=1000, pool=pool)
        sched.step()
        sched.step(first=False)
        torch.cuda.synchronize()
        assert check_schedule(sched, frames)["bit_exact"]
        for pp in sched.pipes:
            assert lib.orbx_debug_skip_stages(pp.ext._h, stage) == 0
        sched.step(first=False)  # the stage does not launch in this step
        torch.cuda.synchronize()
        res = check_schedule(sched, frames)
        for pp in sched.pipes:
            lib.orbx_debug_skip_stages(pp.ext._h, 0)
        if pool == 2:
            assert not res["bit_exact"] and res["mismatches"], "a skipped stage must fail the check"
        else:
            assert res["bit_exact"]  # repeated frames hide it: why bench.py uses --pool 2
        sched.close()


def test_serial_measurement_hook_bit_exact():
    """orbx_debug_serial (the measurement hook that runs every stage in order on one stream, so a kernel
    trace times each kernel alone) changes no output: the bench schedule with it on, every frame checked"""
    torch = pytest.importorskip("torch")
    from orbamd.agent import AgentSchedule
    W, H, B, P = 640, 480, 512, 2
    lib = orbamd.load()
    frames = orbamd.synth_frames(0, 0, 2 * B, W, H)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, pool=2)
    for pp in sched.pipes:
        assert lib.orbx_debug_serial(pp.ext._h, 1) == 0
    for i in range(3):
        sched.step(first=i == 0)
    torch.cuda.synchronize()
    sched.check_errors()
    res = check_schedule(sched, frames, samples=[(p, b) for p in range(P) for b in range(B // P)])
    assert res["bit_exact"], res["mismatches"]
    assert res["checked_frames"] == B
    sched.close()


def test_alias_frames_measurement_hook():
    """orbx_debug_alias_frames (the L2-residency bound of DESIGN.md 6.0): every frame of a batch then yields
    frame 0's keypoints and descriptors, equal to the oracle's on frame 0"""
    torch = pytest.importorskip("torch")
    import numpy as np
    import oracle_py
    from orbamd.device import BatchPipeline
    W, H, B = 640, 480, 64
    frames = orbamd.synth_frames(0, 0, B, W, H)
    pp = BatchPipeline(torch, W, H, B)
    assert orbamd.load().orbx_debug_alias_frames(pp.ext._h, 1) == 0
    pp.extract(torch.from_numpy(frames).cuda())
    torch.cuda.synchronize()
    ko, do = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)(frames[0])
    for b in (0, 1, 33, B - 1):
        kg, dg, _ = pp.host_results(b)
        assert kg.tobytes() == ko.tobytes() and np.array_equal(dg, do), b
    pp.close()
