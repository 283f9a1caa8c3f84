"""One agent of tests/test_gpu_exchange.py::test_two_agents_exchange_on_device (run as a fresh child
process; RANK / WORLD_SIZE / MASTER_* from the environment). Runs the bench schedule
(orbamd.agent.AgentSchedule: device extract + BF match + device keyframe pack + all-gather + slot
match) for one step on cuda:0 and checks it against the oracle (oracle/check_schedule.py).
The agents exchange over gloo (both share one GPU here; the product run is one GPU per agent over
RCCL): the all-gather stages the slot through host memory."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cooperative-orb-slam_amd"), os.path.join(ROOT, "oracle")]


def main():
    import torch
    import torch.distributed as dist
    import orbamd
    from orbamd.agent import AgentSchedule
    from check_schedule import check_schedule

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    W, H, B, P = 640, 480, 64, 2

    def allgather(out, inp):
        o = torch.empty(out.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(o, inp.cpu().clone())
        out.copy_(o.to(out.device))

    # both agents view one synthetic environment (shared scene, crops 12 px apart), as A1 and A2 do
    frames = orbamd.synth_frames(rank, 0, B, W, H, scene=0)
    # the exchange on its own stream, as bench.py runs it whenever a collective does
    sched = AgentSchedule(torch, frames, W, H, P, device=0, rank=rank, world=world, allgather=allgather,
                          async_exchange=True)
    sched.step()
    sched.step(first=False)
    torch.cuda.synchronize()
    sched.check_errors()
    res = check_schedule(sched, frames, agent_frames=lambda r, t: orbamd.synth_frames(r, t, 1, W, H, scene=0)[0])
    xm, xn, xb, xbn = sched.exchange_results()
    print("rank", rank, res, "cross-agent matches", list(xn), "SearchByBoW", list(xbn), flush=True)
    assert res["bit_exact"], res["mismatches"]
    # every slot checked bit-exact above; every agent's keyframe (a view of the same scene) gives both matchers work
    assert res["checked_slots"] == world
    assert all(int(v) > 0 for v in xn) and all(int(v) > 0 for v in xbn), (list(xn), list(xbn))
    sched.close()
    dist.barrier()
    dist.destroy_process_group()
    print("AGENT OK", flush=True)


if __name__ == "__main__":
    main()
