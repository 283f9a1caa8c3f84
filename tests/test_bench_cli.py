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
