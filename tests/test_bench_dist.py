"""bench.py's multi-rank plumbing on the CPU over gloo, at world 2 and world 8: the barriers and the
job span on the node's shared clock (max(t1) - min(t0) over ranks), the communicator-size check (an all_reduce of ones
must sum to the world), the rank-identity check (distinct devices and PCI addresses, else exit 3), and the content check
of the rollout-end gather (every rank's checksums of what it sent against its shard of the gathered tensors; a corrupted
gathered element must fail it on every rank)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TOTAL = 1003   # uneven shards at both world sizes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_q):
    import time
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from bench import DistPlumbing, clock, comm_report
    from walker_gym_amd.distributed import gather_rollout, shard_bounds, verify_gathered
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    pg = DistPlumbing("gloo", torch.device("cpu"))
    pg.init()
    ident = {"rank": rank, "device": 0 if mode == "shared" else rank,
             "pci": "0000:05:00" if mode == "shared" else f"0000:{rank + 5:02x}:00"}
    rep = comm_report(pg, world, ident, strict=True)   # (mode "shared": every rank exits 3 here)
    pg.barrier()
    t0 = clock()
    time.sleep(0.02 * (rank % 3))
    t1 = clock()
    job, slowest = pg.span(t0, t1)
    mx = pg.max_over_ranks([float(rank), 10.0 - rank])
    a, b = shard_bounds(N_TOTAL, world, rank)
    g = torch.Generator().manual_seed(100 + rank)
    sent = {"obs": torch.randn((b - a, 7), generator=g), "reward": torch.randn((5, b - a), generator=g),
            "done": (torch.rand((5, b - a), generator=g) > 0.5).to(torch.uint8)}
    got = {"obs": gather_rollout(sent["obs"], n_total=N_TOTAL), "reward": gather_rollout(sent["reward"], n_total=N_TOTAL, dim=1),
           "done": gather_rollout(sent["done"], n_total=N_TOTAL, dim=1)}
    if mode == "corrupt" and rank == world - 1:
        got["reward"][3, 2] = got["reward"][3, 2] + 1.0   # rank 0's shard as this rank received it
    res = verify_gathered(sent, got, {"obs": 0, "reward": 1, "done": 1}, N_TOTAL, pg.host_group)
    out_q.put((rank, rep, job, slowest, mx, res))
    dist.destroy_process_group()


def _run(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [] if mode == "shared" else [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
    return res, [p.exitcode for p in procs]


@pytest.mark.parametrize("world", [2, 8])
def test_plumbing_and_checks(world):
    res, codes = _run(world, "ok")
    assert codes == [0] * world
    for rank, rep, job, slowest, mx, res_ in res:
        assert rep["communicator_size"] == world and rep["ok"] and rep["distinct_devices"]
        assert [r["rank"] for r in rep["ranks"]] == list(range(world))
        assert mx == [world - 1.0, 10.0]
        # the span from the first start to the last end covers the slowest rank's own time (start skew included)
        assert job >= slowest >= 0.02 * min(2, world - 1) - 1e-3, (job, slowest)
        assert res_["ok"] and not res_["mismatches"] and res_["checked"] == 3 * world, res_


@pytest.mark.parametrize("world", [2, 8])
def test_gather_content_check_catches_corruption(world):
    res, codes = _run(world, "corrupt")
    assert codes == [0] * world
    for rank, rep, job, slowest, mx, res_ in res:
        assert not res_["ok"]                                   # every rank learns of it (AND over ranks)
        if rank == world - 1:
            assert res_["mismatches"] == [[0, "reward"]], res_


def test_shared_device_exits_3():
    """Two ranks reporting the same device and PCI address: comm_report refuses the run (exit 3) on every rank."""
    _, codes = _run(2, "shared")
    assert codes == [3, 3]


def test_check_distinct():
    from walker_gym_amd.distributed import check_distinct
    assert check_distinct([{"device": 0, "pci": "0000:05:00"}, {"device": 1, "pci": "0000:06:00"}]) == (True, "")
    # per-rank device visibility: every rank's GPU is its index 0, the PCI addresses still tell them apart
    assert check_distinct([{"device": 0, "pci": "0000:05:00"}, {"device": 0, "pci": "0000:06:00"}])[0]
    assert not check_distinct([{"device": 0, "pci": "0000:05:00"}, {"device": 1, "pci": "0000:05:00"}])[0]


def test_rollout_checksum_is_order_sensitive():
    import torch
    from walker_gym_amd.distributed import rollout_checksum
    x = torch.randn(100, 5)
    assert rollout_checksum(x) == rollout_checksum(x.clone())
    assert rollout_checksum(x) != rollout_checksum(x.flip(0))
    y = x.clone()
    y[17, 3] = torch.nextafter(y[17, 3], torch.tensor(1e9))
    assert rollout_checksum(x) != rollout_checksum(y)
    d = torch.tensor([0, 1, 1, 0], dtype=torch.uint8)
    assert rollout_checksum(d) == rollout_checksum(d.bool())
