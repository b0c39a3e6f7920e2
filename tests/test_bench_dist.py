"""bench.py's timed-region plumbing (DistPlumbing) on the CPU, world 2 over gloo: with host_ctl (the RCCL default:
the communicator is left for the first gather after the clock) the barriers and the max over ranks of the step
times go over a second, gloo group; without it over the default group.  Both must give every rank the max."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, host_ctl, out_q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from bench import DistPlumbing
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    pg = DistPlumbing("gloo", torch.device("cpu"), host_ctl=host_ctl)
    pg.init()
    pg.barrier()
    got = pg.max_over_ranks([float(rank), 10.0 - rank, 0.5 * rank])
    pg.barrier()
    out_q.put((rank, got, pg.ctl is not None))
    dist.destroy_process_group()


@pytest.mark.parametrize("host_ctl", [True, False])
def test_barrier_and_max_over_ranks(host_ctl):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, host_ctl, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got, has_ctl in res:
        assert got == [1.0, 10.0, 0.5], (rank, got)
        assert has_ctl == host_ctl
