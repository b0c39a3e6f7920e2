"""Multi-GPU data parallelism for the walker batch.

Walkers are independent (no inter-walker force on the env path), so a node-wide batch shards into
contiguous walker blocks, one per rank (one process per GPU, torch.distributed over RCCL/xGMI).
Stepping needs no communication at all; the only collective is the observation gather at the end
of a rollout (``gather_rollout``: one all_gather_into_tensor on RCCL, all_gather on gloo; uneven
shards are padded to the longest and trimmed).  The gathered rollout is SURVEY §8(e)'s tuple: the final
observations [N, D] and every step's reward and done flags [T, N] (``dim=1``: walkers on the second axis).
``gather_rollout_async`` issues a gather without waiting, so an actor loop can overlap the gather of rollout i with
the steps of rollout i + 1 (bench.py ``--gather pipelined``, opt-in: on one MI355X the concurrent RCCL kernel
stalled the steps, DESIGN §8, so bench.py's default is ``--gather serial``).
Results of shard g are bit-identical to the same walkers stepped on one GPU (tested).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous walker range [start, stop) of ``rank`` (the first n_total % world ranks get one more)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_spec(spec: dict, start: int, stop: int) -> dict:
    """Restrict a flat CSR walker spec to walkers [start, stop) (offsets rebased)."""
    import numpy as np
    mo, eo = np.asarray(spec["mass_off"]), np.asarray(spec["edge_off"])
    nm = np.asarray(spec["n_muscles"])
    uo = np.concatenate([[0], np.cumsum(nm)])
    p0, p1, e0, e1, u0, u1 = mo[start], mo[stop], eo[start], eo[stop], uo[start], uo[stop]
    out = {}
    for k in ("m", "pos", "vel", "acc", "pinned", "charge", "radius", "bounce_set"):
        if k in spec:
            out[k] = np.asarray(spec[k])[p0:p1]
    for k in ("ei", "ej", "rest", "k", "c", "flags"):
        out[k] = np.asarray(spec[k])[e0:e1]
    for k in ("minl", "maxl", "stride", "mx"):
        if k in spec:
            out[k] = np.asarray(spec[k])[u0:u1]
    out["mass_off"] = (mo[start:stop + 1] - p0).astype(np.int32)
    out["edge_off"] = (eo[start:stop + 1] - e0).astype(np.int32)
    out["n_muscles"] = nm[start:stop].astype(np.int32)
    return out


class GatherHandle:
    """An issued rollout-end gather (gather_rollout_async): wait() makes the calling stream wait for the collective
    and returns the gathered [n_total, ...] tensor.  The buffers stay referenced until then."""

    def __init__(self, work, out, sizes, nmax, world, dim=0):
        self._work, self._out, self._sizes, self._nmax, self._world = work, out, sizes, nmax, world
        self._dim = dim

    def wait(self) -> Optional[torch.Tensor]:
        if self._work is not None:
            self._work.wait()
            self._work = None
        out, sizes, nmax, world = self._out, self._sizes, self._nmax, self._world
        if out is None:      # a gather to another rank: nothing lands here
            return None
        if self._dim == 1:   # [world * T, nmax, ...] rank blocks -> [T, sum(sizes), ...] (one device copy)
            T = out.shape[0] // world
            blk = out.view((world, T) + tuple(out.shape[1:]))
            if all(sz == nmax for sz in sizes):
                return blk.transpose(0, 1).reshape((T, world * nmax) + tuple(out.shape[2:]))
            return torch.cat([blk[r, :, :sizes[r]] for r in range(world)], 1)
        if all(sz == nmax for sz in sizes):
            return out
        return torch.cat([out[r * nmax:r * nmax + sizes[r]] for r in range(world)], 0)


def gather_rollout_async(local: torch.Tensor, group: Optional[dist.ProcessGroup] = None,
                         n_total: Optional[int] = None, dim: int = 0, dst: Optional[int] = None) -> GatherHandle:
    """Issue the rollout-end gather (every rank's [n_r, ...] block concatenated along dim 0 in rank order) without
    waiting for it: on RCCL the collective runs on the process group's own stream, ordered after the work already
    queued on the calling stream, so steps issued afterwards overlap it (an actor loop gathers rollout i while
    stepping rollout i + 1).  `local` must not be written until wait().

    Blocks may differ in length (shard_bounds gives the first n_total % world ranks one walker more): each block is
    padded to the longest, gathered with one collective (all_gather_into_tensor on RCCL, all_gather on gloo) and
    trimmed.  The lengths come from shard_bounds when ``n_total`` is given, otherwise from a small (synchronous)
    all_gather of every rank's length.

    dim = 1: `local` is a per-step record [T, n_r, ...] (rewards, done flags); the rank blocks are gathered whole
    (each rank's [T, nmax, ...] is one contiguous send buffer, no transpose copy) and returned as [T, N, ...].

    dst = None: every rank receives the whole rollout (all_gather).  dst = r: only rank r — the learner of an
    actor / learner split — receives it (dist.gather: every other rank sends its block straight to r, over its own xGMI
    link on an 8-GPU node, instead of relaying the other ranks' blocks around a ring); the others' wait() returns
    None."""
    if dim not in (0, 1):
        raise ValueError("dim must be 0 (walker rows) or 1 ([T, walkers, ...] records)")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = int(local.shape[dim])
    if n_total is not None:
        sizes = [b - a for a, b in (shard_bounds(n_total, world, r) for r in range(world))]
        if sizes[rank] != n:
            raise ValueError(f"rank {rank} holds {n} rows, shard_bounds({n_total}, {world}) gives {sizes[rank]}")
    else:
        t = torch.tensor([n], dtype=torch.int64, device=local.device)
        all_n = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(all_n, t, group=group)
        sizes = [int(x.item()) for x in all_n]
    nmax = max(sizes)
    block = local.contiguous()
    if n < nmax:
        pad = list(local.shape)
        pad[dim] = nmax - n
        block = torch.cat([block, block.new_zeros(pad)], dim)
    lead = block.shape[0]
    if dst is not None:
        if not 0 <= dst < world:
            raise ValueError(f"dst {dst} is not a rank of this group (world {world})")
        g_dst = dist.get_global_rank(group, dst) if group is not None else dst
        out = (torch.empty((world * lead,) + tuple(block.shape[1:]), dtype=local.dtype, device=local.device)
               if rank == dst else None)
        work = dist.gather(block, list(out.chunk(world, 0)) if out is not None else None, dst=g_dst, group=group,
                           async_op=True)
        h = GatherHandle(work, out, sizes, nmax, world, dim)
        h._block = block
        return h
    out = torch.empty((world * lead,) + tuple(block.shape[1:]), dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        work = dist.all_gather_into_tensor(out, block, group=group, async_op=True)
    else:
        work = dist.all_gather(list(out.chunk(world, 0)), block, group=group, async_op=True)
    h = GatherHandle(work, out, sizes, nmax, world, dim)
    h._block = block   # (the padded copy, if any, lives until wait)
    return h


def gather_rollout(local: torch.Tensor, group: Optional[dist.ProcessGroup] = None,
                   n_total: Optional[int] = None, dim: int = 0, dst: Optional[int] = None) -> Optional[torch.Tensor]:
    """Concatenate every rank's block along the walker axis `dim`, in rank order — the rollout-end gather
    (gather_rollout_async, waited for at once); with dst, on rank dst only (None elsewhere)."""
    return gather_rollout_async(local, group, n_total, dim, dst).wait()


# ---------------------------------------------------------------- self-checks of a multi-GPU run
def rollout_checksum(t: torch.Tensor) -> int:
    """A position-weighted checksum of a tensor's bits, computed where the tensor lives: the elements' bit patterns
    (float32 -> int32, bytes -> int) times (flat index mod 1009) + 1, summed in int64 with wrap-around (two's-complement
    addition is associative, so the value does not depend on the reduction order).  Equal tensors give equal sums; a
    changed, dropped or reordered element changes the sum (barring a 2^-64 collision)."""
    x = t.contiguous().reshape(-1)
    if x.dtype == torch.float32:
        x = x.view(torch.int32)
    elif x.dtype == torch.bool:
        x = x.view(torch.uint8)
    x = x.to(torch.int64)
    w = torch.arange(x.numel(), dtype=torch.int64, device=x.device).remainder_(1009).add_(1)
    return int((x * w).sum().item())


def verify_gathered(sent: dict, gathered: dict, dims: dict, n_total: int, host_group=None) -> dict:
    """Check that a rollout-end gather delivered every rank's own results: each rank checksums what it sent
    (rollout_checksum per tensor), the checksums are all-gathered over `host_group` (a gloo group: CPU tensors), and
    every rank that received the gathered tensors compares rank r's shard of each (shard_bounds rows, along dims[k]) with
    rank r's own checksum.  Returns {"ok", "checked", "mismatches": [[rank, tensor], ...]}, the same on every rank ("ok"
    is the AND over ranks)."""
    keys = sorted(sent)
    world = dist.get_world_size(host_group)
    mine = torch.tensor([rollout_checksum(sent[k]) for k in keys], dtype=torch.int64)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine, group=host_group)
    bad, checked = [], 0
    for r in range(world):
        a, b = shard_bounds(n_total, world, r)
        for i, k in enumerate(keys):
            g = gathered.get(k)
            if g is None:            # a gather to another rank: nothing landed here
                continue
            blk = g[a:b] if dims.get(k, 0) == 0 else g[:, a:b]
            checked += 1
            if rollout_checksum(blk) != int(every[r][i]):
                bad.append([r, k])
    flag = torch.tensor([0 if bad else 1], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=host_group)
    return {"ok": bool(flag.item()), "checked": checked, "mismatches": bad, "tensors": keys}


def rank_identity(dev: torch.device) -> dict:
    """This rank's device: index and PCI address (domain:bus:device) of the GPU it steps on."""
    p = torch.cuda.get_device_properties(dev)
    return {"device": int(dev.index), "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"}


def check_distinct(identities: list) -> Tuple[bool, str]:
    """Every rank on a GPU of its own: PCI addresses pairwise distinct (the physical device; a rank's device INDEX may
    repeat when each rank is shown only its own GPU, e.g. per-rank HIP_VISIBLE_DEVICES, so it decides nothing alone)."""
    pcis = [i["pci"] for i in identities]
    if len(set(pcis)) != len(pcis):
        return False, f"ranks share a GPU (PCI addresses {pcis}, device indices {[i['device'] for i in identities]})"
    return True, ""
