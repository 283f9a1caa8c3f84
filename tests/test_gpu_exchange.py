"""GPU: the cross-agent keyframe exchange on the product path.

* orbx_pack_keyframe_device writes the same bytes as the host packer (every field the receiving
  agent consumes: mvKeys/mvKeysUn/mvuRight/mvDepth/descriptors/MapPoints/BowVector/FeatureVector +
  the lcmKeyFrameInfo scalars), clamps an over-capacity count and flags it;
* orbm_search_for_triangulation_slots_device (brute force and over common BoW nodes, stereo and
  MapPoint flags on both sides, a different geometry per slot) equals the oracle's
  SearchForTriangulation (ORBmatcher.cc:657-823) on the decoded slots; a corrupt slot yields no
  matches and raises the matcher's error flag while the others stay exact;
* two agents in two processes on cuda:0: device extract -> device pack -> all-gather -> slot match,
  against the oracle (the agents exchange over gloo here; the product run uses RCCL over xGMI).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle_py
import orbamd
from orbamd import exchange
from orbamd.matcher import KeyFrameView

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cuda(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _extract(agent, t, n=1, W=640, H=480, nf=1000):
    orc = oracle_py.OracleExtractor(nf, 1.2, 8, 20, 7)
    return [orc(img) for img in orbamd.synth_frames(agent, t, n, W, H)], orc.tables()


def _extras(rng, k, with_fv=True):
    n = len(k)
    ur = np.where(rng.random(n) < 0.4, k["x"] - rng.random(n, dtype=np.float32) * 40, -1).astype(np.float32)
    kun = (np.stack([k["x"], k["y"]], 1) + (rng.random((n, 2), dtype=np.float32) - 0.5)).astype(np.float32)
    e = dict(kun=kun, uright=ur, depth=np.where(ur >= 0, np.float32(3.5), np.float32(-1)).astype(np.float32),
             mp_flags=((rng.random(n) < 0.25).astype(np.uint8) | ((rng.random(n) < 0.1).astype(np.uint8) << 1)),
             mp_pos=rng.standard_normal((n, 3)).astype(np.float32))
    if with_fv:
        nodes = np.sort(rng.choice(3000, 48, replace=False)).astype(np.uint32)
        assign = rng.integers(0, len(nodes), n)
        feats = [np.nonzero(assign == i)[0] for i in range(len(nodes))]
        keep = [i for i in range(len(nodes)) if len(feats[i])]
        nodes = nodes[keep]
        feats = [feats[i] for i in keep]
        off = np.concatenate([[0], np.cumsum([len(f) for f in feats])]).astype(np.int32)
        e["fv"] = (nodes, off, np.concatenate(feats).astype(np.int32))
        words = np.sort(rng.choice(10 ** 6, 200, replace=False)).astype(np.uint32)
        e["bow"] = (words, rng.random(200))
    return e


def _device_source(torch, k, d, e):
    n = len(k)
    t = {"kps": _cuda(torch, np.ascontiguousarray(k, exchange.KP_DTYPE).view(np.uint8)), "desc": _cuda(torch, d),
         "count": _cuda(torch, np.array([n], np.int32))}
    for key in ("kun", "uright", "depth", "mp_flags", "mp_pos"):
        if key in e:
            t[key] = _cuda(torch, e[key])
    if "bow" in e:
        t.update(bow_word=_cuda(torch, e["bow"][0]), bow_value=_cuda(torch, e["bow"][1]),
                 nbow=_cuda(torch, np.array([len(e["bow"][0])], np.int32)))
    if "fv" in e:
        t.update(fv_node=_cuda(torch, e["fv"][0]), fv_off=_cuda(torch, e["fv"][1]), fv_feat=_cuda(torch, e["fv"][2]),
                 nfv=_cuda(torch, np.array([len(e["fv"][0])], np.int32)))
    return exchange.kf_source(**t), t


def _meta(agent, tabs):
    return exchange.make_meta(agent=agent, mnId=7 + agent, scale=tabs["scale"], sigma2=tabs["sigma2"],
                              inv_sigma2=tabs["inv_sigma2"], bf=40.0, b=0.11, th_depth=35.0)


@pytest.mark.parametrize("full", [True, False])
def test_device_pack_equals_host_pack(full):
    torch = pytest.importorskip("torch")
    (res,), tabs = _extract(0, 3)
    k, d = res
    rng = np.random.default_rng(1)
    e = _extras(rng, k) if full else {}
    meta = _meta(0, tabs)
    cap = 1100
    src, keep = _device_source(torch, k, d, e)
    slot = torch.full((exchange.slot_bytes(cap),), 0xAB, dtype=torch.uint8, device="cuda")  # dirty buffer
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    exchange.pack_device(src, meta, cap, slot, err)
    torch.cuda.synchronize()
    host = exchange.pack_host(meta, k, d, cap, **e)
    got = slot.cpu().numpy()
    assert got.tobytes() == host.tobytes()
    assert int(err[0].item()) == 0
    dec = exchange.parse(got)
    assert dec["kps"].tobytes() == k.tobytes() and np.array_equal(dec["desc"], d)
    if full:
        for key in ("kun", "uright", "depth", "mp_flags", "mp_pos"):
            assert np.array_equal(dec[key], e[key]), key
        assert np.array_equal(dec["fv_feat"], e["fv"][2]) and np.array_equal(dec["bow_value"], e["bow"][1])


def test_device_pack_clamps_and_flags_overflow():
    torch = pytest.importorskip("torch")
    (res,), tabs = _extract(0, 5)
    k, d = res
    cap = 600
    assert len(k) > cap
    src, keep = _device_source(torch, k, d, {})
    slot = torch.zeros(exchange.slot_bytes(cap), dtype=torch.uint8, device="cuda")
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    exchange.pack_device(src, _meta(0, tabs), cap, slot, err)
    torch.cuda.synchronize()
    assert int(err[0].item()) & 1
    dec = exchange.parse(slot.cpu().numpy())
    assert dec["n"] == cap and dec["kps"].tobytes() == k[:cap].tobytes()


def _oracle_slot_match(kq, dq, eq, dec, geo, use_bow):
    """oracle SearchForTriangulation(query KF, slot KF) with mvKeysUn / mvuRight / MapPoints from both sides"""
    F12, ex, ey = geo
    m = dec["meta"]
    nl = m.mnScaleLevels
    scale = np.array(m.mvScaleFactors[:nl], np.float32)
    sig = np.array(m.mvLevelSigma2[:nl], np.float32)

    def view(k, d, e, fvd, sc, sg):
        kk = k.copy()
        if e.get("kun") is not None:
            kk["x"], kk["y"] = e["kun"][:, 0], e["kun"][:, 1]
        fv = None
        if use_bow:
            node, off, feat = fvd
            fv = {int(node[i]): list(feat[off[i]:off[i + 1]]) for i in range(len(node))}
        has_mp = None if e.get("mp_flags") is None else (e["mp_flags"] & 1).astype(bool)
        return KeyFrameView(kk, d, sc, sg, feat_vec=fv, uright=e.get("uright"), has_mp=has_mp)

    vq = view(kq, dq, eq, eq.get("fv"), scale, sig)
    ds = {"kun": dec["kun"], "uright": dec["uright"], "mp_flags": dec["mp_flags"]}
    vs = view(dec["kps"], dec["desc"], ds, (dec["fv_node"], dec["fv_off"], dec["fv_feat"]), scale, sig)
    return oracle_py.search_for_triangulation(vq, vs, F12, ex, ey, False, False)


@pytest.mark.parametrize("use_bow", [False, True])
def test_slot_match_equals_oracle(use_bow):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(17)
    frames, tabs = _extract(1, 0, n=4)
    cap = 1100
    nref = 3
    # query = frame 0 (stereo + MapPoints + FeatureVector); slots = frames 1..3 of agents 0..2
    kq, dq = frames[0]
    eq = _extras(rng, kq)
    eq["fv"] = _desc_fv(dq)
    srcq, keepq = _device_source(torch, kq, dq, eq)
    slots = torch.zeros(nref * exchange.slot_bytes(cap), dtype=torch.uint8, device="cuda")
    decs = []
    for r in range(nref):
        k, d = frames[1 + r]
        e = _extras(rng, k) if r != 1 else ({"fv": _extras(rng, k)["fv"]} if use_bow else {})  # slot 1 mono
        if "fv" in e:
            e["fv"] = _desc_fv(d)  # node ids shared with the query's (common nodes to match over)
        host = exchange.pack_host(_meta(r, tabs), k, d, cap, **e)
        slots[r * host.size:(r + 1) * host.size].copy_(torch.from_numpy(host))
        decs.append(exchange.parse(host))
    R = [np.eye(3, dtype=np.float32), np.array([[0.9998, -0.02, 0], [0.02, 0.9998, 0], [0, 0, 1]], np.float32),
         np.eye(3, dtype=np.float32)]
    t = [np.array([0.05, 0, 0.01], np.float32), np.array([-0.1, 0.02, 0.0], np.float32),
         np.array([0.0, 0.08, -0.02], np.float32)]
    K = np.array([[orbamd.device.FX, 0, orbamd.device.CX], [0, orbamd.device.FY, orbamd.device.CY], [0, 0, 1]],
                 np.float32)
    geos = []
    for r in range(nref):
        F12 = orbamd.matcher.compute_f12(np.eye(3), np.zeros(3), R[r], t[r], K, K)
        ex, ey = orbamd.epipole(R[r], t[r], np.zeros(3, np.float32), orbamd.device.FX, orbamd.device.FY,
                                orbamd.device.CX, orbamd.device.CY)
        geos.append((F12, ex, ey))
    mh = orbamd.ORBmatcher(0.6, False)
    out = torch.empty((nref, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(nref, dtype=torch.int32, device="cuda")
    exchange.match_slots_device(mh._h, srcq, cap, nref, slots, exchange.slot_bytes(cap), geos, out, nm,
                                use_bow=use_bow, max_nodes=len(eq["fv"][0]))
    torch.cuda.synchronize()
    assert orbamd.load().orbm_check_error(mh._h, None) == 0
    total = 0
    for r in range(nref):
        no, mo = _oracle_slot_match(kq, dq, eq, decs[r], geos[r], use_bow)
        np.testing.assert_array_equal(out[r, :len(kq)].cpu().numpy(), mo)
        assert int(nm[r].item()) == no
        assert np.all(out[r, len(kq):].cpu().numpy() == -1)
        total += no
    assert total > 0
    # a corrupt slot (foreign version) in the middle: no matches, error flag, the others unchanged
    bad = slots.clone()
    sb = exchange.slot_bytes(cap)
    bad[sb + 4:sb + 8] = torch.tensor([1, 0, 0, 0], dtype=torch.uint8)
    out2 = torch.empty_like(out)
    exchange.match_slots_device(mh._h, srcq, cap, nref, bad, sb, geos, out2, nm, use_bow=use_bow,
                                max_nodes=len(eq["fv"][0]))
    torch.cuda.synchronize()
    assert orbamd.load().orbm_check_error(mh._h, None) == -2
    assert orbamd.load().orbm_check_error(mh._h, None) == 0  # cleared by the read
    assert np.all(out2[1].cpu().numpy() == -1) and int(nm[1].item()) == 0
    assert torch.equal(out2[0], out[0]) and torch.equal(out2[2], out[2])
    mh.close()


def _rot(ax, ay, az):
    cx, cy, cz, sx, sy, sz = np.cos(ax), np.cos(ay), np.cos(az), np.sin(ax), np.sin(ay), np.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return (Rz @ Ry @ Rx).astype(np.float32)


def _desc_fv(d):
    """a FeatureVector that, like a vocabulary, tends to put similar descriptors in the same node: node =
    100 + the top 4 bits of descriptor byte 0 (CSR: ascending node ids, ascending features in a node)"""
    node = 100 + (d[:, 0] >> 4).astype(np.int64)
    ids = np.unique(node)
    feats = [np.nonzero(node == i)[0] for i in ids]
    off = np.concatenate([[0], np.cumsum([len(f) for f in feats])]).astype(np.int32)
    return ids.astype(np.uint32), off, np.concatenate(feats).astype(np.int32)


@pytest.mark.parametrize("use_bow", [False, True])
def test_eight_agent_slots_equal_oracle(use_bow):
    """C5 at 8 agents on one GPU: 8 slots packed from 8 agents' keyframes, the agents viewing one environment
    (shared-scene views 1..8 of scene 9, as A1 and A2 map one place), each slot with its own pose (F12 / epipole: a
    mostly lateral baseline, as the views' crop offsets are), mixing stereo, mono, MapPoints and BoW
    FeatureVectors; the product slot matcher over all 8 (one launch) equals the oracle's
    SearchForTriangulation (ORBmatcher.cc:657-823) row by row, BF and over common BoW nodes, and every row
    holds real cross-agent matches."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(88)
    nref, cap = 8, 1100
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    tabs = orc.tables()
    kq, dq = orc(orbamd.synth_frames(0, 3, 1, 640, 480, scene=9)[0])   # the querying agent's keyframe
    eq = _extras(rng, kq)
    eq["fv"] = _desc_fv(dq)
    srcq, keepq = _device_source(torch, kq, dq, eq)
    sb = exchange.slot_bytes(cap)
    slots = torch.zeros(nref * sb, dtype=torch.uint8, device="cuda")
    decs = []
    for r in range(nref):
        k, d = orc(orbamd.synth_frames(r + 1, 3, 1, 640, 480, scene=9)[0])  # agent r+1's view of the scene
        kind = r % 4  # 0 full (stereo + MapPoints + BoW), 1 mono + BoW only, 2 stereo without MapPoints, 3 mono bare
        e = _extras(rng, k)
        e["fv"] = _desc_fv(d)
        if kind == 1:
            e = {"fv": e["fv"], "bow": e["bow"]}
        elif kind == 2:
            e.pop("mp_flags"), e.pop("mp_pos")
        elif kind == 3:
            e = {"fv": e["fv"]} if use_bow else {}
        host = exchange.pack_host(_meta(r, tabs), k, d, cap, **e)
        slots[r * sb:(r + 1) * sb].copy_(torch.from_numpy(host))
        decs.append(exchange.parse(host))
    K = np.array([[orbamd.device.FX, 0, orbamd.device.CX], [0, orbamd.device.FY, orbamd.device.CY], [0, 0, 1]],
                 np.float32)
    geos = []
    for r in range(nref):
        R = _rot(*(rng.standard_normal(3) * 0.001))
        t = np.array([(0.03 + 0.01 * r) * (1 if r % 2 == 0 else -1), rng.standard_normal() * 0.002, 0.01], np.float32)
        F12 = orbamd.matcher.compute_f12(np.eye(3, dtype=np.float32), np.zeros(3, np.float32), R, t, K, K)
        ex, ey = orbamd.epipole(R, t, np.zeros(3, np.float32), orbamd.device.FX, orbamd.device.FY,
                                orbamd.device.CX, orbamd.device.CY)
        geos.append((F12, ex, ey))
    mh = orbamd.ORBmatcher(0.6, False)
    out = torch.empty((nref, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(nref, dtype=torch.int32, device="cuda")
    exchange.match_slots_device(mh._h, srcq, cap, nref, slots, sb, geos, out, nm, use_bow=use_bow,
                                max_nodes=len(eq["fv"][0]))
    torch.cuda.synchronize()
    assert orbamd.load().orbm_check_error(mh._h, None) == 0
    got, gn = out.cpu().numpy(), nm.cpu().numpy()
    nonzero = 0
    for r in range(nref):
        no, mo = _oracle_slot_match(kq, dq, eq, decs[r], geos[r], use_bow)
        np.testing.assert_array_equal(got[r, :len(kq)], mo, err_msg="slot %d" % r)
        assert int(gn[r]) == no, (r, int(gn[r]), no)
        assert np.all(got[r, len(kq):] == -1)
        nonzero += no > 100
    assert nonzero == nref, "every agent's view of the scene should give cross-agent matches"
    mh.close()


@pytest.mark.parametrize("collective", ["rccl", "torch"])
def test_bench_rccl_world1(collective):
    """bench.py under torch.distributed.run with one rank and --dist, as at N>1: the keyframe slot's out-of-place RCCL
    all-gather (rccl: liborbamd's communicator, ncclAllGather on graph 0's stream, gloo control plane; torch: the
    ProcessGroupNCCL all_gather_into_tensor on the exchange's own stream) and the cross-agent match from the receive
    buffer; the run's self-check must be bit-exact."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--dist", "--steps", "4",
           "--warmup", "2", "--batch", "256", "--pipes", "2", "--no-cpu", "--sustain", "0", "--ingest-steps", "4",
           "--collective", collective]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    print(r.stdout[-3000:], r.stderr[-3000:])
    assert r.returncode == 0
    import json
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["collective"].startswith("rccl"), res["collective"]
    assert ("liborbamd" in res["collective"]) == (collective == "rccl"), res["collective"]
    assert res["bit_exact"] is True and res["checked_slots"] == 1 and res["device_errors"] is None
    assert res["ingest"]["bit_exact"] is True
    assert res["stage_ms_per_step"]["allgather"] > 0


def test_bench_gpus2_launches_ranks():
    """`bench.py --gpus 2` called directly (as the driver calls it) starts two ranks itself under
    torch.distributed.run; here both share cuda:0 and exchange over gloo (ORBAMD_DIST_BACKEND /
    ORBAMD_BENCH_DEVICE, the one-GPU rehearsal hooks): n_gpus 2, both agents' slots checked, bit-exact."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2",
           "--batch", "256", "--pipes", "2", "--no-cpu", "--sustain", "0", "--ingest-steps", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(ORBAMD_DIST_BACKEND="gloo", ORBAMD_BENCH_DEVICE="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    print(r.stdout[-3000:], r.stderr[-3000:])
    assert r.returncode == 0
    import json
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, "rank 0 alone prints the JSON line"
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["checked_slots"] == 2 and res["bit_exact"] is True
    assert res["collective"].startswith("gloo")


def test_bench_gpus2_nccl_needs_two_devices():
    """with the product backend (RCCL) `--gpus 2` on a one-GPU box fails cleanly before any rank starts"""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one visible GPU")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "ORBAMD_DIST_BACKEND", "ORBAMD_BENCH_DEVICE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 2 and "needs 2 visible GPUs" in r.stderr, r.stderr[-2000:]
    assert not r.stdout.strip()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_agents_exchange_on_device():
    """two agent processes (fresh children, both on cuda:0): AgentSchedule step with the device pack ->
    all-gather -> slot match, every rank checked against the oracle by oracle/check_schedule.py"""
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    script = os.path.join(ROOT, "tests", "agent_child.py")
    procs = [subprocess.Popen([sys.executable, script], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append(o)
    for r, (p, o) in enumerate(zip(procs, outs)):
        print(o[-3000:])
        assert p.returncode == 0, "rank %d failed" % r
        assert "AGENT OK" in o


def _oracle_slot_bow(kq, dq, eq, dec, nnratio, check_ori):
    """oracle SearchByBoW(query KF, slot KF) (ORBmatcher.cc:522-655) on the decoded slot"""
    def view(k, d, mpf, fvd):
        node, off, feat = fvd
        fv = {int(node[i]): list(feat[off[i]:off[i + 1]]) for i in range(len(node))}
        has_mp = None if mpf is None else (mpf & 1).astype(bool)
        bad = None if mpf is None else ((mpf >> 1) & 1).astype(bool)
        return KeyFrameView(k, d, np.ones(8, np.float32), np.ones(8, np.float32), feat_vec=fv, has_mp=has_mp,
                            mp_bad=bad)
    vq = view(kq, dq, eq.get("mp_flags"), eq["fv"])
    vs = view(dec["kps"], dec["desc"], dec["mp_flags"], (dec["fv_node"], dec["fv_off"], dec["fv_feat"]))
    return oracle_py.search_by_bow(vq, vs, nnratio, check_ori, other_is_keyframe=True)


@pytest.mark.parametrize("check_ori", [True, False])
def test_eight_agent_slots_search_by_bow_equals_oracle(check_ori):
    """The loop-candidate match of the exchange (LoopClosing::ComputeSim3's SearchByBoW(KF,KF), ORBmatcher(0.75,
    true), LoopClosing.cc:239-265) of the querying agent's keyframe against 8 slots straight from the receive
    buffer: the query itself, a shifted view of it and six other agents' views of the same scene, MapPoints (some
    bad) on both sides, one slot without MapPoints, one malformed. Row by row the oracle's SearchByBoW
    (ORBmatcher.cc:522-655), every other agent's row holding real matches."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    nref, cap = 8, 1100
    orc = oracle_py.OracleExtractor(1000, 1.2, 8, 20, 7)
    tabs = orc.tables()
    img_q = orbamd.synth_frames(0, 3, 1, 640, 480, scene=9)[0]
    kq, dq = orc(img_q)

    def mp(n):
        return ((rng.random(n) < 0.8).astype(np.uint8) | ((rng.random(n) < 0.05).astype(np.uint8) << 1))
    eq = {"mp_flags": mp(len(kq)), "fv": _desc_fv(dq)}
    srcq, keepq = _device_source(torch, kq, dq, eq)
    sb = exchange.slot_bytes(cap)
    slots = torch.zeros(nref * sb, dtype=torch.uint8, device="cuda")
    decs = []
    for r in range(nref):
        if r == 0:
            k, d = kq, dq
        elif r == 1:
            k, d = orc(orbamd.synth_frames(0, 3, 1, 640, 480, dx=3, scene=9)[0])
        else:
            k, d = orc(orbamd.synth_frames(r, 3 + r, 1, 640, 480, scene=9)[0])
        e = {"fv": _desc_fv(d)}
        if r != 5:
            e["mp_flags"] = mp(len(k))
        host = exchange.pack_host(_meta(r, tabs), k, d, cap, **e)
        slots[r * sb:(r + 1) * sb].copy_(torch.from_numpy(host))
        decs.append(exchange.parse(host))
    mh = orbamd.ORBmatcher(0.75, True)
    out = torch.empty((nref, cap), dtype=torch.int32, device="cuda")
    nm = torch.zeros(nref, dtype=torch.int32, device="cuda")
    exchange.bow_slots_device(mh._h, srcq, cap, nref, slots, sb, out, nm, 0.75, check_ori, max_nodes=len(eq["fv"][0]))
    torch.cuda.synchronize()
    assert orbamd.load().orbm_check_error(mh._h, None) == 0
    got, gn = out.cpu().numpy(), nm.cpu().numpy()
    counts = []
    for r in range(nref):
        no, mo = _oracle_slot_bow(kq, dq, eq, decs[r], 0.75, check_ori)
        np.testing.assert_array_equal(got[r, :len(kq)], mo, err_msg="slot %d" % r)
        assert int(gn[r]) == no, (r, int(gn[r]), no)
        assert np.all(got[r, len(kq):] == -1)
        counts.append(no)
    assert counts[0] > 300 and counts[1] > 50 and counts[5] == 0, counts
    assert all(counts[r] > 100 for r in (2, 3, 4, 6, 7)), counts  # the other agents' views of the scene
    # a malformed slot (foreign version): no matches, the error flag, the other rows unchanged
    bad = slots.clone()
    bad[2 * sb + 4:2 * sb + 8] = torch.tensor([1, 0, 0, 0], dtype=torch.uint8)
    out2 = torch.empty_like(out)
    exchange.bow_slots_device(mh._h, srcq, cap, nref, bad, sb, out2, nm, 0.75, check_ori, max_nodes=len(eq["fv"][0]))
    torch.cuda.synchronize()
    assert orbamd.load().orbm_check_error(mh._h, None) == -2
    assert np.all(out2[2].cpu().numpy() == -1) and int(nm[2].item()) == 0
    assert torch.equal(out2[0], out[0]) and torch.equal(out2[7], out[7])
    mh.close()
