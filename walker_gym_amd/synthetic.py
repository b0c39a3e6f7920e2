"""Seeded synthetic walker batches in the flat CSR layout.

Every builder returns a dict of numpy arrays:
  m [P] f32, pos/vel/acc [P,3] f32, mass_off [N+1] i32,
  ei/ej [E] i32 (walker-local mass indices), rest/k/c [E] f32, flags [E] u8 (bit0 = string),
  edge_off [N+1] i32, n_muscles [N] i32 (muscles are the first n_muscles edges of each walker),
  minl/maxl/stride [U] f32 per muscle.
Rest lengths are the initial distances computed exactly as ``np.linalg.norm`` does for a float32
3-vector (float32 products summed in double, rounded to float32, then float32 sqrt — the OpenBLAS
sdot path the reference hits at gym/optimized_walker.py:23-25 / gym/engine.py:86), vectorised.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def norm3_f32(d: np.ndarray) -> np.ndarray:
    """``np.linalg.norm`` of float32 3-vectors, bit-exact, vectorised over the leading axes."""
    d = np.asarray(d, dtype=np.float32)
    sq = d * d                                          # float32 products
    s = (np.float64(0.0) + sq[..., 0].astype(np.float64)) + sq[..., 1].astype(np.float64)
    s = s + sq[..., 2].astype(np.float64)
    return np.sqrt(s.astype(np.float32))


_LATTICE_CACHE = {}


def _lattice(side: int):
    if side not in _LATTICE_CACHE:
        edges = []
        for r in range(side):
            for c in range(side - 1):
                edges.append((r * side + c, r * side + c + 1))
        for r in range(side - 1):
            for c in range(side):
                edges.append((r * side + c, (r + 1) * side + c))
        M = side * side
        lat = set(edges)
        others = [(i, j) for i in range(M) for j in range(i + 1, M) if (i, j) not in lat]
        _LATTICE_CACHE[side] = (np.array(edges, np.int32), np.array(others, np.int32))
    return _LATTICE_CACHE[side]


def canonical_walkers(N: int, seed: int = 0, M: int = 16, K: int = 40, A: int = 8):
    """The canonical synthetic walker of SURVEY §8(d): M=16 (4x4 jittered lattice, spacing 10,
    y in [0, 40]), m ~ U(1,5), v = 0, 24 lattice edges + (K-24) random distinct non-lattice pairs,
    the first A edges are muscles, rest = initial length, k = 1000, c = 20."""
    side = int(round(M ** 0.5))
    assert side * side == M, "canonical walker needs a square lattice"
    lat, others = _lattice(side)
    n_rand = K - len(lat)
    assert 0 <= n_rand <= len(others)
    rng = np.random.default_rng(seed)
    m = rng.uniform(1.0, 5.0, (N, M)).astype(f32)
    cols = np.tile(np.arange(side), side).astype(np.float32)
    rows = np.repeat(np.arange(side), side).astype(np.float32)
    base = np.stack([10.0 * cols - 15.0, 10.0 * rows + 5.0, np.zeros(M)], axis=1).astype(f32)
    pos = (base[None] + rng.uniform(-1.0, 1.0, (N, M, 3))).astype(f32)
    # per-walker random distinct non-lattice pairs
    keys = rng.random((N, len(others)))
    pick = np.argsort(keys, axis=1)[:, :n_rand]
    rand_pairs = others[pick]                                    # [N, n_rand, 2]
    pairs = np.concatenate([np.broadcast_to(lat, (N,) + lat.shape), rand_pairs], axis=1)  # [N,K,2]
    ei = pairs[..., 0].astype(np.int32)
    ej = pairs[..., 1].astype(np.int32)
    wi = np.arange(N)[:, None]
    rest = norm3_f32(pos[wi, ei] - pos[wi, ej])
    P = N * M
    return dict(
        m=m.reshape(P), pos=pos.reshape(P, 3), vel=np.zeros((P, 3), f32), acc=np.zeros((P, 3), f32),
        mass_off=(np.arange(N + 1) * M).astype(np.int32),
        ei=ei.reshape(-1), ej=ej.reshape(-1), rest=rest.reshape(-1).astype(f32),
        k=np.full(N * K, 1000.0, f32), c=np.full(N * K, 20.0, f32), flags=np.zeros(N * K, np.uint8),
        edge_off=(np.arange(N + 1) * K).astype(np.int32), n_muscles=np.full(N, A, np.int32),
        minl=np.full(N * A, 0.1, f32), maxl=np.full(N * A, 1.5, f32), stride=np.full(N * A, 2.0, f32),
    )


def ragged_walkers(N: int, seed: int = 0, mmin: int = 4, mmax: int = 32, string_frac: float = 0.0):
    """Mixed-topology batch: M ~ U{mmin..mmax}, K ~ U{M..2M}, A = K // 5.
    Edges are random pairs (i != j; repeats allowed once distinct pairs run out), rest = initial
    length x U(0.9, 1.1), k ~ U(200, 1500), c ~ U(0, 30)."""
    rng = np.random.default_rng(seed)
    Ms = rng.integers(mmin, mmax + 1, N)
    Ks = np.array([rng.integers(M, 2 * M + 1) for M in Ms])
    As = Ks // 5
    m, pos, ei, ej = [], [], [], []
    for M, K in zip(Ms, Ks):
        m.append(rng.uniform(1.0, 5.0, M))
        p = np.stack([rng.uniform(-30, 30, M), rng.uniform(0, 40, M), rng.uniform(-5, 5, M)], 1)
        pos.append(p)
        allp = [(i, j) for i in range(M) for j in range(i + 1, M)]
        order = rng.permutation(len(allp))
        prs = [allp[o] for o in order[:K]]
        while len(prs) < K:
            i, j = rng.choice(M, 2, replace=False)
            prs.append((int(i), int(j)))
        sw = rng.random(K) < 0.5
        for (i, j), s in zip(prs, sw):
            ei.append(j if s else i); ej.append(i if s else j)
    m = np.concatenate(m).astype(f32)
    pos = np.concatenate(pos).astype(f32)
    mass_off = np.concatenate([[0], np.cumsum(Ms)]).astype(np.int32)
    edge_off = np.concatenate([[0], np.cumsum(Ks)]).astype(np.int32)
    ei = np.array(ei, np.int32); ej = np.array(ej, np.int32)
    wid = np.repeat(np.arange(N), Ks)
    gi = mass_off[wid] + ei; gj = mass_off[wid] + ej
    rest = (norm3_f32(pos[gi] - pos[gj]) * rng.uniform(0.9, 1.1, len(ei)).astype(f32)).astype(f32)
    E = len(ei)
    flags = np.zeros(E, np.uint8)
    if string_frac > 0:
        local = np.arange(E) - edge_off[wid]
        is_sk = local >= As[wid]
        flags[(rng.random(E) < string_frac) & is_sk] = 1
    U = int(As.sum())
    return dict(
        m=m, pos=pos, vel=np.zeros_like(pos), acc=np.zeros_like(pos), mass_off=mass_off,
        ei=ei, ej=ej, rest=rest, k=rng.uniform(200, 1500, E).astype(f32),
        c=rng.uniform(0, 30, E).astype(f32), flags=flags, edge_off=edge_off,
        n_muscles=As.astype(np.int32), minl=np.full(U, 0.1, f32), maxl=np.full(U, 1.5, f32),
        stride=np.full(U, 2.0, f32),
    )


def chain_walkers(N: int, n_points: int = 100, seed: int = 0):
    """performance_demo's chain (gym/performance_demo.py:18-47) as N independent walkers: n_points masses of
    m = 1 at U(-100, 100)^3 with velocities U(-10, 10)^3, linked in order by Skeleton(k=50) springs (rest = the
    initial distance, damping c = 20, the Skeleton default), no muscles.  The demo steps it with
    Point.gravity() over the walker's points (pair_mode 1)."""
    rng = np.random.default_rng(seed)
    P, K = N * n_points, N * (n_points - 1)
    pos = rng.uniform(-100, 100, (P, 3)).astype(f32)
    vel = rng.uniform(-10, 10, (P, 3)).astype(f32)
    ei = np.tile(np.arange(n_points - 1, dtype=np.int32), N)
    ej = ei + 1
    base = np.repeat(np.arange(N) * n_points, n_points - 1)
    rest = norm3_f32(pos[base + ei] - pos[base + ej]).astype(f32)
    return dict(m=np.ones(P, f32), pos=pos, vel=vel, acc=np.zeros_like(pos),
                mass_off=(np.arange(N + 1) * n_points).astype(np.int32), ei=ei, ej=ej.astype(np.int32), rest=rest,
                k=np.full(K, 50.0, f32), c=np.full(K, 20.0, f32), flags=np.zeros(K, np.uint8),
                edge_off=(np.arange(N + 1) * (n_points - 1)).astype(np.int32), n_muscles=np.zeros(N, np.int32),
                minl=np.zeros(0, f32), maxl=np.zeros(0, f32), stride=np.zeros(0, f32))
