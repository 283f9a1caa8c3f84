"""GPU: the exact schedule bench.py times (orbamd.agent.AgentSchedule) checked against the oracle.

The headline configuration: 1024 frames per step as 4 staggered 256-frame graphs on 4 streams, with
the keyframe-slot exchange; every graph's device error flags, then EVERY frame's keypoints and
descriptors (raw bits), every frame's SearchForTriangulation row against its predecessor, and the
cross-agent match row are compared with the oracle (ORBextractor.cc:1043-1105,
ORBmatcher.cc:657-823). The BASELINE configs C3 (752x480, 1200 features) and C4 (1241x376, 2000
features) run the same schedule on smaller batches."""
import pytest

import orbamd
from check_schedule import check_schedule

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,nf,B,P", [(640, 480, 1000, 1024, 4), (752, 480, 1200, 128, 2),
                                         (1241, 376, 2000, 128, 2)])
def test_bench_schedule_bit_exact(W, H, nf, B, P):
    torch = pytest.importorskip("torch")
    from orbamd.agent import AgentSchedule
    frames = orbamd.synth_frames(0, 0, B, W, H)
    sched = AgentSchedule(torch, frames, W, H, P, device=0, nfeatures=nf)
    sched.step()                   # warmup (the first step also builds the geometry tables)
    sched.step(first=False)        # the checked step, staggered exactly as in bench.py
    torch.cuda.synchronize()
    sched.check_errors()
    sub = B // P
    samples = [(p, b) for p in range(P) for b in range(sub)]  # every frame
    res = check_schedule(sched, frames, samples=samples, nfeatures=nf)
    assert res["bit_exact"], res["mismatches"]
    assert res["checked_frames"] == B and res["checked_slots"] == 1
    assert all(int(pp.nmatch.min().item()) > 0 for pp in sched.pipes)
    sched.close()
