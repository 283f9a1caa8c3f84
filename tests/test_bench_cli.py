"""CPU: bench.py's launcher contract (no GPU needed).

`bench.py --gpus N` called directly with N > 1 starts N ranks itself under torch.distributed.run; with the
product backend (RCCL) it refuses, before any rank starts, when fewer than N devices are visible (here: none).
A rank whose WORLD_SIZE disagrees with --gpus refuses too.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ORBAMD_DIST_BACKEND", "ORBAMD_BENCH_DEVICE")}
    env.update(kw)
    return env


def test_gpus_n_without_devices_fails_cleanly():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=_env())
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 2 visible GPUs" in r.stderr
    assert not r.stdout.strip()


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "--gpus 4 but WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]


def test_launch_frames_query():
    """tools/gpu_round.sh reads the stage-launch size and the graph count of the default step from the bench
    itself (the PMC traffic file is tagged with it, and bench.py prices only launches of that size)"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch-frames"], capture_output=True,
                       text=True, timeout=120, cwd=ROOT, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    sub, pipes = (int(v) for v in r.stdout.split())
    assert sub * pipes > 0 and sub >= 64


def test_describe_touched_bytes_is_the_patch_union():
    """describe's algorithmic bytes (bench.describe_touched_bytes): per level the union of the windows its patches
    read, at most every level pixel once, plus 56 B per keypoint; the fused form (the 43x43 unblurred source window)
    touches fewer bytes than the separate form's unblurred 31x31 + blurred 37x37 windows"""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cooperative-orb-slam_amd"), os.path.join(ROOT, "oracle")]
    import bench
    import oracle_py
    import orbamd
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    imgs = orbamd.synth_frames(0, 0, 2, 640, 480)

    class Sched:
        P, sub = 1, 2

        def frame_results(self, p, b):
            return orc(imgs[b])[0], None, None
    px = sum(w * h for w, h in bench.level_sizes(640, 480))
    nkp = len(orc(imgs[0])[0])
    fused = bench.describe_touched_bytes(Sched(), 640, 480, True)
    sep = bench.describe_touched_bytes(Sched(), 640, 480, False)
    assert 56 * nkp < fused <= px + 56 * nkp
    assert fused < sep <= 2 * px + 56 * nkp
