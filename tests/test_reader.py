"""The driver-surface .inp reader (C++ in libhakai_hip.so) against the reference decks and an
independent pure-Python restatement of the parts of readInpFile the solver consumes."""
import os

import numpy as np
import pytest

import hakai
from hakai import mesh

HERE = os.path.dirname(os.path.abspath(__file__))
TENSILE = "/root/reference/HAKAI-v0.0.0/input/Tensile5e.inp"   # read in place, never copied
REF_DIR = "/root/reference/HAKAI-v0.0.2/input"


@pytest.mark.skipif(not os.path.exists(TENSILE), reason="reference decks not present")
def test_tensile5e_reader_matches_code_model():
    a = hakai.read_inp(TENSILE)
    b = mesh.tensile5e_model()
    assert a.nNode == 24 and a.nElement == 5
    assert np.array_equal(a.coordmat, b.coordmat)
    assert np.array_equal(a.elementmat, b.elementmat)
    assert np.array_equal(a.element_material, b.element_material)
    assert (a.d_time, a.end_time, a.mass_scaling, a.contact_flag) == (5e-7, 0.01, 1.0, 0)
    assert a.n_steps == 20000
    assert len(a.materials) == 3
    for x, y in zip(a.materials, b.materials):
        assert (x.density, x.young, x.poisson) == (y.density, y.young, y.poisson)
        assert np.array_equal(x.plastic, y.plastic) and np.array_equal(x.ductile, y.ductile)
    assert len(a.bc) == len(b.bc) == 2
    for g, h in zip(a.bc, b.bc):
        assert len(g.entries) == len(h.entries)
        for (d1, v1), (d2, v2) in zip(g.entries, h.entries):
            assert np.array_equal(d1, d2) and v1 == v2
    assert np.array_equal(a.bc[1].amp_time, [0., 0.01]) and np.array_equal(a.bc[1].amp_value, [0., 1.])


def _py_nodes_elems(path):
    """Independent minimal restatement: *Part/*Node/*Element blocks and *Instance offsets."""
    lines = open(path).read().split("\n")
    parts, insts = {}, []
    i = 0
    while i < len(lines):
        l = lines[i]
        if "*Part, name=" in l:
            name = l.replace(" ", "").split(",")[1].split("name=")[1]
            j = i + 1
            while "*Node" not in lines[j]:
                j += 1
            nodes = []
            j += 1
            while "*" not in lines[j]:
                nodes.append([float(x) for x in lines[j].replace(" ", "").split(",") if x][1:4])
                j += 1
            while "*Element" not in lines[j]:
                j += 1
            els = []
            j += 1
            while "*" not in lines[j]:
                els.append([int(x) for x in lines[j].replace(" ", "").split(",") if x][1:9])
                j += 1
            parts[name] = (np.array(nodes), np.array(els, np.int64))
        if "*Instance" in l:
            s = l.replace(" ", "").split(",")
            insts.append((s[2].split("part=")[1], [t.replace(" ", "") for t in
                                                    lines[i + 1:lines.index("*End Instance", i)]]))
        i += 1
    return parts, insts


@pytest.mark.skipif(not os.path.isdir(REF_DIR), reason="reference decks not present")
@pytest.mark.parametrize("deck", ["car-crash-N2k.inp", "car-wall-N2k.inp", "carx2-crash-N43k.inp",
                                  "../../HAKAI-v0.0.1/input/projectile-impact-d1mm.inp"])
def test_multi_instance_decks(deck):
    """Multi-instance decks: translations and rotations of *Instance (v2/readInpFile_j.jl:566-620)."""
    path = os.path.join(REF_DIR, deck)
    m = hakai.read_inp(path)
    parts, insts = _py_nodes_elems(path)
    coords, elems, off = [], [], 0
    for pname, tr in insts:
        c, e = parts[pname]
        c = c.copy()
        for t in reversed(tr):
            s = [x for x in t.split(",") if x]
            if len(s) == 3:
                c = c + np.array([float(x) for x in s])
            elif len(s) == 7:  # rotation about the axis (p1 -> p2) by s[6] degrees (readInpFile_j.jl:590-604)
                v = [float(x) for x in s]
                n = np.array(v[3:6]) - np.array(v[0:3])
                n = n / np.linalg.norm(n)
                d = v[6] / 180.0 * np.pi
                K = np.array([[0, -n[2], n[1]], [n[2], 0, -n[0]], [-n[1], n[0], 0]])
                T = np.cos(d) * np.eye(3) + (1 - np.cos(d)) * np.outer(n, n) + np.sin(d) * K
                c = c @ T.T
        coords.append(c)
        elems.append(e + off)
        off += c.shape[0]
    assert np.allclose(m.coordmat, np.vstack(coords), rtol=0, atol=1e-9)
    assert np.array_equal(m.elementmat, np.vstack(elems))
    assert m.contact_flag >= 1
    assert m.mass_scaling == {"carx2-crash-N43k.inp": 60.0, "../../HAKAI-v0.0.1/input/projectile-impact-d1mm.inp": 1.0}.get(deck, 100.0)
    assert len(m.ic_dofs) > 0 and np.all(m.ic_dofs >= 1)
    diag, vol = m.lumped_mass()
    assert np.all(diag > 0)


def _dof_map(groups):
    out = {}
    for g in groups:
        for d, v in g.entries:
            for x in np.asarray(d):
                out[int(x)] = float(v)
    return out


@pytest.mark.parametrize("which", ["tensile5e", "two_body", "two_body_self", "two_body_cp", "bar_ic"])
def test_written_decks_round_trip(tmp_path, which):
    """Decks written from code (tests/inp_writer.py) read back by the C++ reader to the same model:
    the path the GPU-box driver tests use, since the box has no reference decks."""
    from inp_writer import write_inp
    m = {"tensile5e": mesh.tensile5e_model,
         "two_body": lambda: mesh.two_body_model(perturb=0.05, seed=3),
         "two_body_self": lambda: mesh.two_body_model(contact_flag=2),
         "two_body_cp": lambda: mesh.two_body_model(surfaces=True),
         "bar_ic": lambda: mesh.bar_model(2, 3, 4, mesh.steel_ductile(), lambda z, L: 1e4 * z / L, perturb=0.02)}[which]()
    path = write_inp(str(tmp_path / "deck.inp"), m)
    a = hakai.read_inp(path)
    assert np.array_equal(a.coordmat, m.coordmat) and np.array_equal(a.elementmat, m.elementmat)
    assert np.array_equal(a.element_material, m.element_material)
    assert (a.d_time, a.end_time, a.mass_scaling, a.contact_flag) == (m.d_time, m.end_time, m.mass_scaling,
                                                                      m.contact_flag)
    assert _dof_map(a.bc) == _dof_map(m.bc)
    assert dict(zip(a.ic_dofs.tolist(), a.ic_values.tolist())) == dict(zip(m.ic_dofs.tolist(), m.ic_values.tolist()))
    if m.element_instance is not None:
        assert np.array_equal(a.element_instance, m.element_instance)
    for x, y in zip(a.materials, m.materials):
        assert (x.density, x.young, x.poisson) == (y.density, y.young, y.poisson)
        assert np.array_equal(x.plastic, np.asarray(y.plastic).reshape(-1, 2))
    assert (a.contact_pairs is None) == (m.contact_pairs is None)
    for p, q in zip(a.contact_pairs or [], m.contact_pairs or []):
        for (ia, ea), (ib, eb) in zip(p, q):
            assert ia == ib and np.array_equal(ea, eb)


@pytest.mark.skipif(not os.path.isdir(REF_DIR), reason="reference decks not present")
def test_every_reference_deck_parses():
    """readInpFile on every deck the reference ships (v0.0.0-v0.0.2): sizes, positive lumped mass."""
    import glob
    decks = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(REF_DIR)), "..", "**", "*.inp"),
                             recursive=True))
    assert len(decks) >= 20
    for d in decks:
        m = hakai.read_inp(d)
        assert m.nNode > 0 and m.nElement > 0 and m.elementmat.min() >= 1 and m.elementmat.max() <= m.nNode
        diag, _ = m.lumped_mass()
        assert np.all(diag > 0), d


@pytest.mark.skipif(not os.path.isdir(REF_DIR), reason="reference decks not present")
def test_deck_fixtures_round_trip():
    """tests/golden/deck_*.npz hold exactly what readInpFile makes of the shipped decks."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
    from deck_fixtures import model_from_arrays, model_to_arrays
    from make_deck_golden import DECKS, REF
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    for deck, steps, _ in DECKS:
        name = os.path.splitext(os.path.basename(deck))[0].replace("-", "_")
        z = np.load(os.path.join(gold, f"deck_{name}.npz"))
        m = hakai.read_inp(os.path.join(REF, deck))
        assert int(z["steps"]) == (steps or m.n_steps)
        a = model_to_arrays(m)
        for k, v in a.items():
            assert np.array_equal(np.asarray(v), z[k]), (deck, k)
        b = model_to_arrays(model_from_arrays(z))
        assert sorted(b) == sorted(a)
