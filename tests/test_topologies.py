"""Topology import: the G1 / G3 builders of walker_gym_amd.topologies reproduce the
reference builders' creatures exactly.  Pinned by fixtures made from the reference's own builder code
(tests/golden/make_golden.py scenarios M and N): g1_builders.npz (gym/walker.py, run with its missing
``Phy(m, v, p)`` supplied; its physics and G1 getstat steps are checked by the golden tests like every
other fixture) and topology/g3_builders.npz (gym/optimized_walker/walker.py through the reference
env's own add_point / add_ding_point / add_spring)."""
import os

import numpy as np
import pytest

from walker_gym_amd.topologies import G1_BUILDERS, G3_BUILDERS, build_creature, mixed_spec, topology_spec
from walker_gym_amd.walker import creatures_to_spec

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_g1_builders_match_reference():
    z = np.load(os.path.join(GOLDEN, "g1_builders.npz"))
    names = [str(n) for n in z["g1_names"]]
    assert sorted(names) == sorted(G1_BUILDERS)
    spec = mixed_spec([(n, 1) for n in names], generation=1)
    for key in ("m", "pos", "vel", "mass_off", "ei", "ej", "rest", "k", "c", "flags", "edge_off", "n_muscles",
                "minl", "maxl", "stride"):
        got, ref = np.asarray(spec[key]), z["in_" + key]
        assert got.shape == ref.shape, key
        assert np.array_equal(got.astype(ref.dtype), ref), key
    assert np.array_equal(spec["pinned"], z["in_pinned"])   # balance3's DingPoint


@pytest.mark.parametrize("name", sorted(set(G3_BUILDERS) | {"insect8"}))
def test_g3_builders_match_reference(name):
    z = np.load(os.path.join(GOLDEN, "topology", "g3_builders.npz"))
    kw = {"legs": 8} if name == "insect8" else {}
    cr = build_creature("insect" if name == "insect8" else name, generation=3, **kw)
    spec = creatures_to_spec([cr])
    assert np.array_equal(spec["m"], z[name + "_m"].astype(np.float32))
    assert np.array_equal(spec["pos"], z[name + "_pos"])
    assert np.array_equal(spec["pinned"], z[name + "_ding"])
    A = len(cr.muscles)
    mus, spr = z[name + "_muscles"], z[name + "_springs"]
    assert A == len(mus) and len(spec["ei"]) == A + len(spr)
    # muscles first (Creature.run order), then the springs, each in call order
    assert np.array_equal(np.stack([spec["ei"][:A], spec["ej"][:A]], 1).reshape(-1, 2), mus)
    assert np.array_equal(np.stack([spec["ei"][A:], spec["ej"][A:]], 1).reshape(-1, 2), spr)
    assert np.array_equal(spec["rest"][:A], z[name + "_muscle_x"])
    assert np.array_equal(spec["rest"][A:], z[name + "_spring_x"])
    assert np.array_equal(spec["k"][:A], z[name + "_muscle_power"].astype(np.float32))
    assert np.array_equal(spec["k"][A:], z[name + "_spring_k"].astype(np.float32))
    assert np.array_equal(spec["flags"][A:], z[name + "_spring_string"])


def test_topology_batches_step_on_the_oracle():
    """Every imported topology packs into a batch the stepper accepts (uniform and ragged)."""
    from oracle.oracle import Oracle
    for g, table in ((1, G1_BUILDERS), (3, G3_BUILDERS)):
        for name in table:
            spec = topology_spec(name, 3, generation=g)
            o = Oracle(spec, dict(in3d=1, midform=2 if g == 1 else 1))
            A = int(spec["n_muscles"][0])
            for _ in range(3):
                o.step(np.zeros((3, A), np.float32) if A else None)
    spec = mixed_spec([(n, 2) for n in G3_BUILDERS], generation=3)
    assert len(spec["mass_off"]) == 2 * len(G3_BUILDERS) + 1


def test_unknown_topology():
    for g in (1, 2, 3):
        with pytest.raises(ValueError):
            build_creature("nope", generation=g)
