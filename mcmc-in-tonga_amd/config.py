"""Configuration -- mirror of define_TDstructure.jl.

``parameters`` keeps the reference's field names and positional order
(define_TDstructure.jl:1-44); ``define_TDstructrure()`` (sic, the reference's
spelling) returns the reference defaults (define_TDstructure.jl:46-65).
Only ``debug_prior``, ``interp_style`` and ``add_yVec`` reach the forward
model; the chain also reads sig, zeta_scale, max/min_cells, prior, n_iter,
burn_in, keep_each, print_each.
"""
from dataclasses import dataclass, fields, replace
from typing import List


@dataclass
class parameters:  # noqa: N801 -- the reference's type name
    debug_prior: int
    plot_voronoi: int
    add_yVec: int
    sig: int
    zeta_scale: int
    max_cells: int
    min_cells: int
    max_sig: float
    interp_style: int
    enforce_discon: int
    prior: int
    event_statics: int
    demean: int
    n_chains: int
    n_iter: float
    burn_in: float
    keep_each: float
    print_each: float
    max_depth: float
    min_depth: float
    rotation: int
    ZnodeSpacing: int
    buffer: int
    XYnodeSpacing: int
    xyMap: bool
    zSlice: List[int]
    xzMap: bool
    ySlice: List[int]

    def replace(self, **kw):
        return replace(self, **kw)


def define_TDstructrure():  # noqa: N802 -- reference spelling (define_TDstructure.jl:46)
    return parameters(
        # basic parameters
        0, 0, 1,
        # Voronoi diagram parameters
        10, 50, 100, 5, 0.1, 1, 0, 1, 1, 1,
        # Monte Carlo parameters
        2, 1e3, 5e2, 1e1, 1e2,
        # map parameters
        660, 0, 20, 20, 100, 20,
        # cross-section parameters
        True, [50, 300, 500], True, [700, 800],
    )


PARAMETER_NAMES = [f.name for f in fields(parameters)]
