"""The drop-in path's one-point Interpolation on the host (csrc/host_nn.h, tdt_host_nn_query) against the
C oracle's v_nearest (MCsub.jl:247-263): value and winning Julia position, on the committed model after
births / deaths / changes / moves and on that model plus one pending edit of each kind -- ties,
duplicate sites, flat axes, points far outside the cells' box and the 1e9 sentinel.  CPU only: the
hook builds and queries the host grid without touching the GPU."""
import numpy as np
import pytest

from conftest import ROOT  # noqa: F401  (sys.path)


def _p(a):
    return None if a is None else a.ctypes.data


def host_query(tt, cells, edits, pending, Q):
    L = tt.lib()
    x, y, z, v = (np.ascontiguousarray(a, dtype=np.float64) for a in cells)
    ed = np.ascontiguousarray(np.asarray(edits, dtype=np.float64).reshape(-1, 6))
    pe = None if pending is None else np.ascontiguousarray(np.asarray(pending, dtype=np.float64))
    qx, qy, qz = (np.ascontiguousarray(Q[:, a], dtype=np.float64) for a in range(3))
    val = np.empty(len(Q))
    pos = np.empty(len(Q), dtype=np.int64)
    rc = L.tdt_host_nn_query(_p(x), _p(y), _p(z), _p(v), len(x), _p(ed) if len(ed) else None,
                             len(ed), _p(pe), _p(qx), _p(qy), _p(qz), len(Q), _p(val),
                             _p(pos))
    assert rc == 0
    return val, pos


def apply(cells, e):
    x, y, z, v = (list(a) for a in cells)
    a, k = int(e[0]), int(e[1])
    if a == 1:
        x.append(e[2]), y.append(e[3]), z.append(e[4]), v.append(e[5])
    elif a == 2:
        for arr in (x, y, z, v):
            del arr[k]
    elif a == 3:
        v[k] = e[5]
    else:
        x[k], y[k], z[k] = e[2], e[3], e[4]
    return [np.array(t, dtype=np.float64) for t in (x, y, z, v)]


def check(tt, orc, cells, edits, pending, Q):
    val, pos = host_query(tt, cells, edits, pending, Q)
    model = [np.asarray(a, dtype=np.float64) for a in cells]
    for e in edits:
        model = apply(model, e)
    if pending is not None:
        model = apply(model, pending)
    for k, q in enumerate(Q):
        ov, oi = orc.v_nearest(q[0], q[1], q[2], *model)
        assert (val[k] == ov or (np.isnan(val[k]) and np.isnan(ov))) and pos[k] == oi, (k, q, val[k], ov, pos[k], oi)


def random_edit(rng, n, box):
    a = int(rng.integers(1, 5)) if n > 1 else 1
    k = int(rng.integers(0, n)) if a != 1 else n
    p = rng.uniform(box[0], box[1], 3)
    return [a, k, p[0], p[1], p[2], rng.normal()]


@pytest.mark.parametrize("n", [1, 2, 50, 700, 5000])
def test_random_models_and_edits(tt, orc, n):
    rng = np.random.default_rng(n)
    box = (-100.0, 300.0)
    cells = [rng.uniform(*box, n), rng.uniform(*box, n), rng.uniform(0, 600, n), rng.normal(size=n)]
    edits, m = [], n
    for _ in range(60):
        e = random_edit(rng, m, box)
        edits.append(e)
        m += 1 if e[0] == 1 else -1 if e[0] == 2 else 0
    Q = np.concatenate([rng.uniform(-150, 350, (40, 3)),  # inside and just around the box
                        rng.uniform(-5000, 5000, (8, 3)),  # far outside
                        np.stack([cells[0][:5], cells[1][:5], cells[2][:5]], 1)])  # on cells (distance 0)
    for a in (None, 1, 2, 3, 4):
        pend = None if a is None else ([1, m] + list(rng.uniform(*box, 3)) + [0.5] if a == 1 else
                                        [a, int(rng.integers(0, m))] + list(rng.uniform(*box, 3)) + [rng.normal()])
        if pend is not None and a == 2 and m < 2:
            continue
        check(tt, orc, cells, edits, pend, Q)


def test_ties_duplicates_and_flat_axes(tt, orc):
    # a lattice of cells with duplicated sites (different values) in a flat z plane: the queries at lattice
    # midpoints are equidistant from 2, 4 or 8 cells and the first in Julia order must win
    g = np.arange(6, dtype=np.float64)
    X, Y = np.meshgrid(g, g, indexing="ij")
    x = np.concatenate([X.ravel(), X.ravel()[::-1]])
    y = np.concatenate([Y.ravel(), Y.ravel()[::-1]])
    z = np.zeros_like(x)
    v = np.arange(len(x), dtype=np.float64)
    h = np.arange(-1, 7, 0.5)
    QX, QY = np.meshgrid(h, h, indexing="ij")
    Q = np.stack([QX.ravel(), QY.ravel(), np.zeros(QX.size)], 1)
    Q = np.concatenate([Q, Q + [0, 0, 0.5]])
    cells = [x, y, z, v]
    check(tt, orc, cells, [], None, Q)
    # a death of the first of two coincident cells hands the tie to the other; a move onto a site ties
    check(tt, orc, cells, [], [2, 0, 0, 0, 0, 0], Q)
    check(tt, orc, cells, [[2, 3, 0, 0, 0, 0], [1, 70, 2.5, 2.5, 0.0, -1.0]], [4, 40, 2.0, 3.0, 0.0, 0], Q)
    check(tt, orc, cells, [[3, 7, 0, 0, 0, 9.5]], [1, len(x), 1.0, 1.0, 0.0, 7.0], Q)  # appended: loses ties
    check(tt, orc, cells, [], [3, 1, 0, 0, 0, -4.0], Q)
    # every cell at one site
    same = [np.full(9, 3.0), np.full(9, -1.0), np.full(9, 2.0), np.arange(9.0)]
    check(tt, orc, same, [[2, 0, 0, 0, 0, 0]], [4, 2, 3.0, -1.0, 2.0, 0], Q)


def test_sentinel(tt, orc):
    # v_nearest starts at mdist = 1e9 (:250): a cell at squared distance >= 1e9 never wins, and with none
    # closer the value is 0.0 (position -1)
    r = np.sqrt(1e9)
    x = np.array([0.0, r, np.nextafter(r, 0), 2 * r, 50.0])
    cells = [x, np.zeros(5), np.zeros(5), np.array([1.0, 2.0, 3.0, 4.0, 5.0])]
    Q = np.array([[0.0, 0, 0], [-r, 0, 0], [-np.nextafter(r, 0), 0, 0], [-1e6, 0, 0], [3 * r, 0, 0],
                  [r / 2, r, r], [1e7, 1e7, 1e7], [r + 50.0, 0, 0], [0.0, -r, 0],
                  [np.nan, 0, 0], [np.inf, 0, 0], [-np.inf, 1.0, 1.0], [0.0, np.nan, np.inf]])
    check(tt, orc, cells, [], None, Q)
    check(tt, orc, cells, [[2, 0, 0, 0, 0, 0]], None, Q)
    check(tt, orc, cells, [], [4, 4, -3e4, 0.0, 0.0, 0], Q)
    check(tt, orc, [np.zeros(0)] * 4, [], [1, 0, 1.0, 2.0, 3.0, 8.0], Q)  # an empty model plus a birth
    check(tt, orc, [np.zeros(0)] * 4, [], None, Q[:3])


def test_chain_shaped_sequence(tt, orc):
    # the drop-in host's use: a 5000-cell model walked by a long run of committed edits (deaths shift the
    # Julia positions; slots are reused; cells leave the build box), queried at birth sites after each
    rng = np.random.default_rng(7)
    n = 3000
    cells = [rng.uniform(0, 400, n), rng.uniform(0, 400, n), rng.uniform(0, 660, n), rng.normal(size=n)]
    edits, m = [], n
    for _ in range(600):
        e = random_edit(rng, m, (-40.0, 700.0))
        edits.append(e)
        m += 1 if e[0] == 1 else -1 if e[0] == 2 else 0
    Q = rng.uniform(-50, 700, (60, 3))
    check(tt, orc, cells, edits, None, Q)
    check(tt, orc, cells, edits, [2, m // 3, 0, 0, 0, 0], Q)
