"""tstar-mi355x: MI355X-native forward model for the rj-MCMC Voronoi t* tomography
of Geronimorz/MCMC-in-Tonga.

The directory name contains dashes, so it is imported under the module name
``mcmc_in_tonga_amd`` by ``tonga.py`` at the repository root:

    import tonga; tt = tonga.load()
    ds = tt.load_data_Tonga(); prm = tt.define_TDstructrure()
    model, ds, valid = tt.evaluate(tt.random_model(1000, 2), ds, prm)

Layers: L1 types/config (defstruct, config), L2 data (data),
L3 forward model over the C ABI (forward -> libtdstar.so), L4 chain (chain).
"""
from ._lib import TD_ENGINE_DEVICE, TD_ENGINE_DROPIN, TD_ENGINE_HOST, TdError, lib  # noqa: F401
from .chain import Chain, TD_inversion_function, build_starting, chain_params, main_inversion, run_batch, run_chains  # noqa: F401,E501
from .config import define_TDstructrure, parameters  # noqa: F401
from .data import (CONFIGS, ak135_slowness, box, interp1, load_data_Tonga, lonlat2xy, pad_rays,  # noqa: F401
                   random_model, segments, synthetic_rays)
from .defstruct import DataStruct, Model, Ray  # noqa: F401
from .forward import Interpolation, TdContext, context_for, evaluate, v_nearest  # noqa: F401
from .tempering import Exchange, NativeComm, TemperingLadder, decide_swaps, geometric_ladder  # noqa: F401
from .posterior import plot_model_hist, section  # noqa: F401
from .sharded import RayShardedContext, ray_points, shard_rays, sub_datastruct  # noqa: F401
from . import jld  # noqa: F401  (save/load model.jld, main_inversion.jl:18)
