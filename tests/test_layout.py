"""Host packing: incidence lists reproduce the reference accumulation order; encodings; byte model."""
import numpy as np
import pytest

from walker_gym_amd.layout import algorithmic_bytes_per_walker_step, incidence, pack
from walker_gym_amd.synthetic import canonical_walkers, norm3_f32, ragged_walkers
from walker_gym_amd.walker import balance_spec, create_balance_creature, creatures_to_spec


def brute_incidence(ei, ej, M):
    lists = [[] for _ in range(M)]
    for e, (i, j) in enumerate(zip(ei, ej)):
        lists[i].append((e << 1) | 0)
        lists[j].append((e << 1) | 1)
    return lists


def test_incidence_matches_reference_order():
    spec = ragged_walkers(40, seed=2, mmin=2, mmax=20)
    inc, inc_off = incidence(spec["ei"], spec["ej"], spec["mass_off"], spec["edge_off"])
    mo, eo = spec["mass_off"], spec["edge_off"]
    for w in range(40):
        M = mo[w + 1] - mo[w]
        ref = brute_incidence(spec["ei"][eo[w]:eo[w + 1]], spec["ej"][eo[w]:eo[w + 1]], M)
        offs = inc_off[mo[w] + w: mo[w + 1] + w + 1]
        lst = inc[2 * eo[w]: 2 * eo[w + 1]]
        for q in range(M):
            assert list(lst[offs[q]:offs[q + 1]]) == ref[q]
        assert offs[-1] == 2 * (eo[w + 1] - eo[w])


def test_pack_uniform_and_ragged():
    u = pack(canonical_walkers(8, seed=0))
    assert not u.ragged and (u.M, u.K, u.A) == (16, 40, 8)
    assert u.edges.shape == (320, 4) and u.muscle_bounds.shape == (64, 2)
    r = pack(ragged_walkers(8, seed=0))
    assert r.ragged


def test_edge_encoding_and_bounds():
    spec = balance_spec(2)
    spec["flags"][3] = 1
    h = pack(spec)
    ij = h.edges[:, 0]
    assert np.array_equal(ij & 0x7fff, spec["ei"]) and np.array_equal((ij >> 16) & 0x7fff, spec["ej"])
    assert ((ij >> 31) == spec["flags"]).all()
    assert np.array_equal(h.edges[:, 1].view(np.float32), spec["rest"])
    x0 = spec["rest"][[0, 1, 5, 6]]
    assert np.array_equal(h.muscle_bounds[:, 0], (x0 * np.float32(0.1)).astype(np.float32))
    assert np.array_equal(h.muscle_bounds[:, 1], (x0 * np.float32(1.5)).astype(np.float32))


def test_builder_rest_lengths_are_numpy_norms():
    cr = create_balance_creature()
    spec = creatures_to_spec([cr])
    for e, el in enumerate(list(cr.muscles) + list(cr.skeletons)):
        assert spec["rest"][e] == np.linalg.norm(el.p1.pos - el.p2.pos)
    d = np.random.default_rng(0).standard_normal((1000, 3)).astype(np.float32) * 30
    assert np.array_equal(norm3_f32(d), np.array([np.linalg.norm(x) for x in d]))


def test_algorithmic_bytes_canonical():
    # canonical M=16, K=40, A=8, 3-D obs (152 floats) -> 2,440 B per walker-step
    assert algorithmic_bytes_per_walker_step(16, 40, 8, 152) == 2440
    assert algorithmic_bytes_per_walker_step(4, 5, 2, 38) == 536


def test_pair_and_g3_host_plumbing():
    """Point.e / Point.r reach the packed layout (float64, the reference's Python floats); the G3 and pair
    parameters reach the C struct; a malformed per-mass array is refused."""
    import ctypes as C

    import pytest

    from walker_gym_amd.batched_env import EnvParams
    from walker_gym_amd.distributed import shard_spec
    from walker_gym_amd.layout import default_radius
    cr = create_balance_creature()
    cr.phys[1].e = 2.5
    spec = creatures_to_spec([cr])
    h = pack(spec)
    assert h.charge.dtype == np.float64 and h.charge[1] == 2.5 and h.charge[0] == 16e-20
    assert np.array_equal(h.radius, np.array([float(p.m) ** 0.3 for p in cr.phys]))
    assert np.array_equal(default_radius(h.mass), h.radius)
    two = creatures_to_spec([create_balance_creature(), cr])
    sh = shard_spec(two, 1, 2)
    assert np.array_equal(sh["charge"], spec["charge"]) and np.array_equal(sh["radius"], spec["radius"])
    bad = dict(spec)
    bad["charge"] = spec["charge"][:2]
    with pytest.raises(ValueError):
        pack(bad)
    s = EnvParams(spring_mode=2, g3_gravity=(1.0, -98.0, 0.5), g3_ground=0, pair_mode=6, bounce_k=40.0).to_struct()
    assert tuple(s.g3_gravity) == (1.0, -98.0, 0.5) and s.g3_ground == 0 and s.spring_mode == 2
    assert s.pair_mode == 6 and s.bounce_k == 40.0 and s.pair_k == 8.99e9 and s.pair_e == 16e-20
    assert C.sizeof(s) > 0
    with pytest.raises(ValueError):
        EnvParams(g3_gravity=(0.0, 1.0)).to_struct()


def test_concat_specs_matches_creatures_to_spec():
    from walker_gym_amd.walker import concat_specs, create_box_creature, replicate_spec
    a, b = create_balance_creature(), create_box_creature()
    joined = concat_specs([replicate_spec(creatures_to_spec([a]), 3), replicate_spec(creatures_to_spec([b]), 2)])
    ref = creatures_to_spec([a, a, a, b, b])
    assert set(joined) == set(ref)
    for k in ref:
        assert np.array_equal(joined[k], ref[k]), k
    h = pack(joined)
    assert h.N == 5 and h.ragged   # Box-v0 has 4 muscles, Balance-v0 2: a ragged batch


def test_wave_edge_passes_matches_library():
    """layout.wave_edge_passes restates walker_hip.hip wave_passes (wg_wave_edge_passes)."""
    import ctypes as C
    from walker_gym_amd import _lib
    from walker_gym_amd.layout import wave_edge_passes
    L = _lib.load()
    for M in (0, 1, 2, 4, 13, 32, 64, 65):
        for K in (0, 1, 5, 63, 64, 65, 128, 200, 300, 512, 513, 600):
            assert wave_edge_passes(M, K) == L.wg_wave_edge_passes(C.c_int32(M), C.c_int32(K)), (M, K)


def test_wave_tile_order_fills_tiles_and_planner_reproduces_them():
    """Ragged batches whose walkers fit one wave are stored in best-fit-decreasing wave-tile order: every tile within
    the wave caps, wg_plan_waves' greedy contiguous packing of that order yields exactly those tiles, and far fewer
    of them than size-sorted neighbours (config 5's distribution)."""
    import ctypes as C
    from walker_gym_amd import _lib
    from walker_gym_amd.layout import WAVE_LANES, size_order, wave_edge_passes
    spec = ragged_walkers(3000, seed=5)
    lay = pack(spec)
    assert lay.row is not None and sorted(lay.row.tolist()) == list(range(3000))
    assert np.array_equal(size_order(spec), lay.row)
    L = _lib.load()

    def plan(mo, eo, uo):
        N = len(mo) - 1
        out = np.zeros(N + 1, np.int32)
        mo, eo, uo = (np.ascontiguousarray(x, np.int32) for x in (mo, eo, uo))
        nb = L.wg_plan_waves(mo.ctypes.data_as(C.c_void_p), eo.ctypes.data_as(C.c_void_p),
                             uo.ctypes.data_as(C.c_void_p), N, out.ctypes.data_as(C.c_void_p), N + 1)
        assert nb > 0
        return out[:nb + 1]
    p = plan(lay.mass_off, lay.edge_off, lay.muscle_off)
    Ms, Ks, As = np.diff(lay.mass_off), np.diff(lay.edge_off), np.diff(lay.muscle_off)
    ne = wave_edge_passes(int(Ms.max()), int(Ks.max()))
    for t in range(len(p) - 1):
        a, b = p[t], p[t + 1]
        assert Ms[a:b].sum() <= WAVE_LANES and Ks[a:b].sum() <= 64 * ne and As[a:b].sum() <= WAVE_LANES
    # size-sorted neighbours (the previous order) for comparison
    srt = np.lexsort((np.arange(3000), np.asarray(spec["n_muscles"]), np.diff(spec["edge_off"]),
                      np.diff(spec["mass_off"])))
    M0, K0, A0 = np.diff(spec["mass_off"])[srt], np.diff(spec["edge_off"])[srt], np.asarray(spec["n_muscles"])[srt]
    p0 = plan(np.concatenate([[0], np.cumsum(M0)]), np.concatenate([[0], np.cumsum(K0)]),
              np.concatenate([[0], np.cumsum(A0)]))
    assert len(p) < 0.92 * len(p0), (len(p), len(p0))
    assert Ms.sum() / (len(p) - 1) > 62.0


def test_wave_tile_order_caps_and_reproduction_edge_cases():
    """Best-fit wave tiles under each cap in turn (the walker-count cap with 1-mass walkers, the spring cap with
    spring-dense walkers, the muscle cap), and wg_plan_waves' greedy pass over the order reproduces them."""
    import ctypes as C
    from walker_gym_amd import _lib
    from walker_gym_amd.layout import wave_edge_passes, wave_tile_order
    L = _lib.load()
    rng = np.random.default_rng(11)
    cases = [(np.ones(100, np.int64), np.zeros(100, np.int64), np.zeros(100, np.int64)),             # 32 walkers/tile
             (rng.integers(4, 9, 300), rng.integers(20, 64, 300), np.zeros(300, np.int64)),           # springs bind
             (rng.integers(2, 12, 300), rng.integers(0, 10, 300), rng.integers(0, 40, 300)),          # muscles bind
             (rng.integers(1, 65, 500), rng.integers(0, 65, 500), rng.integers(0, 13, 500))]
    for Ms, Ks, As in cases:
        ne = wave_edge_passes(int(Ms.max()), int(Ks.max()))
        order = wave_tile_order(Ms, Ks, As, ne)
        assert sorted(order.tolist()) == list(range(len(Ms)))
        mo, eo, uo = (np.concatenate([[0], np.cumsum(x[order])]).astype(np.int32) for x in (Ms, Ks, As))
        plan = np.zeros(len(Ms) + 1, np.int32)
        nb = L.wg_plan_waves(mo.ctypes.data_as(C.c_void_p), eo.ctypes.data_as(C.c_void_p),
                             uo.ctypes.data_as(C.c_void_p), len(Ms), plan.ctypes.data_as(C.c_void_p), len(Ms) + 1)
        assert nb > 0
        for t in range(nb):
            a, b = plan[t], plan[t + 1]
            assert mo[b] - mo[a] <= 64 and eo[b] - eo[a] <= 64 * ne and uo[b] - uo[a] <= 64 and b - a <= 32
        # the lower bound on tiles from masses alone is met within a tile or two where masses bind
        if Ks.max() == 0:
            assert nb == -(-len(Ms) // 32)


def test_wave_tile_order_windows_keep_caller_locality():
    """Windowed best-fit packing (layout.wave_tile_order, WG_TILE_WINDOW): each window of W consecutive caller
    walkers occupies W consecutive stored positions (so its wave tiles are consecutive and, under the kernel's
    XCD-aware workgroup order, share one L2), at almost the tile count of one global packing."""
    from walker_gym_amd.layout import wave_edge_passes, wave_tile_order
    spec = ragged_walkers(5000, seed=17, mmin=4, mmax=32)
    M, K = np.diff(spec["mass_off"]), np.diff(spec["edge_off"])
    A = np.asarray(spec["n_muscles"])
    ne = wave_edge_passes(int(M.max()), int(K.max()))

    def ntiles(order):
        n, P, E, U, c = 1, 0, 0, 0, 0
        for w in order:
            if c and (P + M[w] > 64 or E + K[w] > 64 * ne or U + A[w] > 64 or c + 1 > 32):
                n, P, E, U, c = n + 1, 0, 0, 0, 0
            P, E, U, c = P + M[w], E + K[w], U + A[w], c + 1
        return n
    glob, win = wave_tile_order(M, K, A, ne, window=0), wave_tile_order(M, K, A, ne, window=512)
    for s in range(0, 5000, 512):
        assert sorted(win[s:s + 512].tolist()) == list(range(s, min(s + 512, 5000)))
    assert ntiles(win) <= 1.01 * ntiles(glob), (ntiles(win), ntiles(glob))


def test_bounce_set_packing():
    """ABI 12: Point.bounce(k, other=<list>) per point as bit 0 (calls) | bit 1 (in the list); all 3 (other="*") is
    stored as None, entries outside 0..3 and a wrong length are refused; a ragged batch's copy follows its walkers
    into stored order."""
    from walker_gym_amd.layout import pack
    from walker_gym_amd.synthetic import canonical_walkers, ragged_walkers
    spec = canonical_walkers(5, seed=1)
    P = int(spec["mass_off"][-1])
    assert pack(spec).bounce_set is None
    assert pack(dict(spec, bounce_set=np.full(P, 3, np.uint8))).bounce_set is None
    bs = np.random.default_rng(0).integers(0, 4, P).astype(np.uint8)
    assert np.array_equal(pack(dict(spec, bounce_set=bs)).bounce_set, bs)
    with pytest.raises(ValueError):
        pack(dict(spec, bounce_set=np.full(P, 4, np.uint8)))
    with pytest.raises(ValueError):
        pack(dict(spec, bounce_set=bs[:-1]))
    rg = ragged_walkers(300, seed=3, mmin=3, mmax=40)
    Pr = int(rg["mass_off"][-1])
    bsr = np.random.default_rng(1).integers(0, 4, Pr).astype(np.uint8)
    lay = pack(dict(rg, bounce_set=bsr))
    assert np.array_equal(lay.bounce_set[lay.mass_perm], bsr) if lay.mass_perm is not None else \
        np.array_equal(lay.bounce_set, bsr)


def test_bounce_set_from_lists():
    """The converter from the reference's calls (`for p in callers: p.bounce(k, other=L)`) to bounce_set bytes: callers
    and one shared list, both in registry order; lists the two bits cannot express (another order, repeats, bad
    indices) are refused rather than silently reordered."""
    from walker_gym_amd.layout import bounce_set_from_lists
    assert bounce_set_from_lists(5, [0, 2, 4]).tolist() == [3, 2, 3, 2, 3]
    assert bounce_set_from_lists(5, [1, 3], [0, 1, 4]).tolist() == [2, 3, 0, 1, 2]
    assert bounce_set_from_lists(4, [], []).tolist() == [0, 0, 0, 0]
    for callers, other in (([2, 1], "*"), ([0], [3, 1]), ([0], [1, 1]), ([0, 0], "*"), ([5], "*"), ([0], "all")):
        with pytest.raises(ValueError):
            bounce_set_from_lists(5, callers, other)
