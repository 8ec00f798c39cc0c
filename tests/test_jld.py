"""JLD output: ``save("model.jld", "model", models)``
(main_inversion.jl:18) written with the reference file's own HDF5 layout.

The reference's 100 saved models (tests/golden/model_jld_kat.npz, decoded
from its model.jld) are written by jld.save: the file's structure must equal
the reference file's (tests/golden/model_jld_structure.json: user block,
every object and its storage layout, types with member offsets, the
committed Model type, every attribute), and reading it back must return the
same numbers bit for bit.  Needs an interpreter with h5py (the image's
/opt/conda/bin/python3.9); skipped without one."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def jld(tt):
    import importlib
    m = importlib.import_module(tt.__name__ + ".jld")
    if not m.available():
        pytest.skip("no interpreter with h5py")
    return m


def kat_models(tt, kat):
    """The reference's saved models, with its aliasing (a position saving the
    same Model object as an earlier one holds that object)."""
    off, chains, same = kat["cell_off"], kat["chain"], kat["same_as"]
    models, objs = [[], []], []
    for j in range(len(kat["phi"])):
        if same[j] != j:
            objs.append(objs[int(same[j])])
            models[int(chains[j]) - 1].append(objs[-1])
            continue
        sl = slice(int(off[j]), int(off[j + 1]))
        m = tt.Model(float(kat["nCells"][j]), kat["xCell"][sl].copy(), kat["yCell"][sl].copy(),
                     kat["zCell"][sl].copy(), kat["zeta"][sl].copy(), float(kat["phi"][j]), kat["ptS"][j].copy(),
                     kat["tS"].copy(), float(kat["likelihood"][j]), int(kat["action"][j]), int(kat["accept"][j]),
                     float(kat["zeta_xz"][j]), float(kat["zeta_xy"][j]))
        objs.append(m)
        models[int(chains[j]) - 1].append(m)
    return models


def test_reference_models_reproduce_reference_layout(tt, kat, jld, tmp_path):
    path = tmp_path / "model.jld"
    jld.save(path, kat_models(tt, kat))
    with open(os.path.join(GOLDEN, "model_jld_structure.json")) as fh:
        want = json.load(fh)
    got = jld.fingerprint(path)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g == w, (g, w)


def test_round_trip_bit_exact(tt, kat, jld, tmp_path):
    models = kat_models(tt, kat)
    path = tmp_path / "model.jld"
    jld.save(path, models)
    back = jld.load(path)
    assert [len(c) for c in back] == [len(c) for c in models]
    assert back[1][4] is back[1][5] and back[0][0] is not back[0][1]  # the reference's one alias
    for ca, cb in zip(models, back):
        for a, b in zip(ca, cb):
            for k in ("xCell", "yCell", "zCell", "zeta", "ptS", "tS"):
                assert np.array_equal(getattr(a, k), getattr(b, k)), k
            for k in ("nCells", "phi", "likelihood", "action", "accept", "zeta_xz", "zeta_xy"):
                assert getattr(a, k) == getattr(b, k), k


def test_own_models_and_large_arrays(tt, jld, tmp_path):
    """Models of this build (5000 cells: arrays past HDF5's compact limit are
    stored contiguous), three chains of different lengths, one empty."""
    rng = np.random.default_rng(3)
    chains = []
    for c, k in enumerate((3, 0, 2)):
        chain = []
        for j in range(k):
            m = tt.random_model(5000 if j == 0 else 17, 10 * c + j)
            m.phi, m.likelihood, m.action, m.accept = float(rng.random()), -3.5, j % 4 + 1, j % 2
            m.ptS, m.tS = rng.random(381), rng.random(381)
            chain.append(m)
        chains.append(chain)
    path = tmp_path / "own.jld"
    jld.save(path, chains)
    back = jld.load(path)
    assert [len(c) for c in back] == [3, 0, 2]
    for ca, cb in zip(chains, back):
        for a, b in zip(ca, cb):
            assert np.array_equal(a.xCell, b.xCell) and np.array_equal(a.zeta, b.zeta)
            assert np.array_equal(a.ptS, b.ptS) and a.phi == b.phi and a.action == b.action


def test_checkpoint_round_trip(tt, ds, jld, tmp_path):
    """A chain checkpoint (TD_inversion_function.jl:285 burn-in / :292 before):
    the model, model_hist (aliasing kept), iter, saved_#, model_num, burnin and
    the DataStruct arrays come back bit for bit."""
    rng = np.random.default_rng(4)
    hist = []
    for k in range(4):
        m = tt.random_model(int(rng.integers(5, 40)), k)
        m.phi, m.ptS, m.tS, m.likelihood = float(rng.uniform(10, 99)), rng.random(len(ds.tS)), ds.tS, 3.25
        m.action, m.accept = int(rng.integers(1, 5)), int(rng.integers(0, 2))
        hist.append(m)
    hist.append(hist[-1])  # the reference pushes the same object when nothing was accepted in between
    path = tmp_path / "chain3_iter777_77.7%.jld"
    jld.save_checkpoint(path, hist[-1], ds, 777.0, True, hist, saved=5, model_num=100)
    c = jld.load_checkpoint(path)
    assert c["burnin"] and c["iter"] == 777.0 and c["saved"] == 5 and c["model_num"] == 100
    assert len(c["model_hist"]) == 5 and c["model_hist"][3] is c["model_hist"][4] is c["model"]
    for a, b in zip(c["model_hist"], hist):
        for f in ("xCell", "yCell", "zCell", "zeta", "ptS", "tS"):
            assert np.array_equal(getattr(a, f), getattr(b, f))
        assert (a.phi, a.likelihood, a.action, a.accept, a.nCells) == (b.phi, b.likelihood, b.action, b.accept,
                                                                      b.nCells)
    for f in ("tS", "allSig", "rayX", "rayY", "rayZ", "rayL", "rayU", "U"):
        assert np.array_equal(c["ds"][f], getattr(ds, f), equal_nan=True), f
    assert list(c["ds"]["xVec_range"]) == [ds.xVec[0], ds.xVec[1] - ds.xVec[0], len(ds.xVec)]
    pre = tmp_path / "chain3_iter100_10%.jld"
    jld.save_checkpoint(pre, hist[0], ds, 100, False)
    p = jld.load_checkpoint(pre)
    assert not p["burnin"] and p["iter_is_int"] and p["iter"] == 100 and p["model_hist"] == []
    assert "saved" not in p
    fp = jld.fingerprint(path)
    assert fp[0] == ["userblock", "Julia data file (HDF5), version 0.1.3"]
    top = {e[0] for e in fp if "/" not in e[0]}
    assert {"model", "dataStruct", "iter", "saved_#", "model_num", "model_hist", "burnin"} <= top
