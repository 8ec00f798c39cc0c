"""ctypes binding of libtdstar.so (include/tdstar.h, include/tdstar_testing.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no fallback: if the shared object is missing or fails to load, every
entry point raises -- the forward model only runs through the HIP kernels.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# (TD_LIB_PATH: a diagnostic A/B of two builds on one box, tools/ only; the product loads the in-tree build)
LIB_PATH = os.environ.get("TD_LIB_PATH") or os.path.join(HERE, "libtdstar.so")

TD_OK, TD_ERR_ARG, TD_ERR_LAYOUT, TD_ERR_HIP, TD_ERR_NOMEM, TD_ERR_BOUNDS = range(6)
TD_ENGINE_DEVICE, TD_ENGINE_HOST, TD_ENGINE_DROPIN = 0, 1, 2

_d = ctypes.c_double
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_pd = ctypes.POINTER(ctypes.c_double)
_pi32 = ctypes.POINTER(ctypes.c_int32)
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pu32 = ctypes.POINTER(ctypes.c_uint32)
_vp = ctypes.c_void_p


class TdInfo(ctypes.Structure):
    _fields_ = [("abi_version", _i32), ("device", _i32), ("m", _i64), ("n", _i64), ("npoints", _i64),
                ("nsegments", _i64), ("likelihood", _d), ("arch", ctypes.c_char * 32), ("num_cus", _i32)]


class TdChainParams(ctypes.Structure):
    _fields_ = [("debug_prior", _i32), ("sig", _i32), ("zeta_scale", _i32), ("max_cells", _i32),
                ("min_cells", _i32), ("prior", _i32), ("n_iter", _d), ("burn_in", _d), ("keep_each", _d),
                ("xmin", _d), ("xmax", _d), ("ymin", _d), ("ymax", _d), ("zmin", _d), ("zmax", _d),
                ("seed", _u64), ("chain", _i32), ("temperature", _d), ("engine", _i32),
                ("start_iter", _i64)]


class TdChainStats(ctypes.Structure):
    _fields_ = [("iterations", _i64), ("evaluations", _i64), ("accepted", _i64 * 5), ("proposed", _i64 * 5),
                ("phi", _d), ("ncells", _i64), ("bytes", _i64), ("last_action", _i32), ("last_accept", _i32)]


# name -> (restype, argtypes); every symbol declared in include/*.h
SIGNATURES = {
    "td_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, _pd, _pd, _pd, _pd, _pd, _i64, _i64, _pd, _pd]),
    "td_destroy": (ctypes.c_int, [_vp]),
    "td_last_error": (ctypes.c_char_p, [_vp]),
    "td_get_info": (ctypes.c_int, [_vp, ctypes.POINTER(TdInfo)]),
    "td_set_sigma": (ctypes.c_int, [_vp, _pd]),
    "td_misfit": (ctypes.c_int, [_vp, _i64, _pd, _pd, _pd, _pd, _pd]),
    "td_set_incremental": (ctypes.c_int, [_vp, ctypes.c_int]),
    "td_rounds_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _i64]),
    "td_rounds_run": (ctypes.c_int, [_vp, _i64, _pd, _pd]),
    "td_rounds_destroy": (ctypes.c_int, [_vp]),
    "td_swap_decide": (ctypes.c_int, [_i64, _pd, _pi64, _pd, _i64, ctypes.c_uint64, _pi64, _pi64, _pi64]),
    "td_rounds_temper": (ctypes.c_int, [_vp, _i64, _i64, _pd, _pi64, _i64, ctypes.c_uint64, _pd, _pi64, _pi64,
                                        _pi64]),
    "td_rounds_exchange": (ctypes.c_int, [_vp, _vp, _i64, _i64, _pd, _pi64, _i64, ctypes.c_uint64, _pd, _pi64,
                                          _pi64, _pi64, _pd]),
    "td_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "td_comm_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    "td_comm_allgather": (ctypes.c_int, [_vp, _pd, _i64, _pd]),
    "td_comm_destroy": (ctypes.c_int, [_vp]),
    "td_timing_enable": (ctypes.c_int, [_vp, ctypes.c_int]),
    "td_timing_reset": (ctypes.c_int, [_vp]),
    "td_timing_get": (ctypes.c_int, [_vp, ctypes.c_char_p, _pi64, _pd]),
    "td_evaluate": (ctypes.c_int, [_vp, _pd, _pd, _pd, _pd, _i64, ctypes.c_int, _pd, _pd, _pd, _pi32]),
    "td_evaluate_batch": (ctypes.c_int, [_vp, _i64, _pi64, _pd, _pd, _pd, _pd, _pd, _pd, _pd]),
    "td_interpolate": (ctypes.c_int, [_vp, _pd, _pd, _pd, _pd, _i64, _pd, _i64, _pd, _i64, _pd, _i64, _pd, _pi32,
                                      _pi64]),
    "td_trilinear": (ctypes.c_int, [ctypes.c_int, _pd, _i64, _pd, _i64, _pd, _i64, _pd, _pd, _pd, _pd, _i64, _pd,
                                     _pi64]),
    "td_rasterize": (ctypes.c_int, [_vp, _i64, _pi64, _pd, _pd, _pd, _pd, _pd, _pd, _pd, _i64, _pd, _pd, _pd]),
    "td_chain_create": (ctypes.c_int, [ctypes.POINTER(_vp), _vp, ctypes.POINTER(TdChainParams), _pd, _pd, _pd, _pd,
                                       _i64]),
    "td_chain_destroy": (ctypes.c_int, [_vp]),
    "td_chain_run": (ctypes.c_int, [_vp, _i64]),
    "td_chain_run_batch": (ctypes.c_int, [ctypes.POINTER(_vp), _i64, _i64]),
    "td_chain_stats_get": (ctypes.c_int, [_vp, ctypes.POINTER(TdChainStats)]),
    "td_chain_get_model": (ctypes.c_int, [_vp, _pd, _pd, _pd, _pd, _i64, _pi64, _pd, _pd]),
    "td_chain_set_temperature": (ctypes.c_int, [_vp, _d]),
    # include/tdstar_testing.h
    "tdt_philox": (None, [_pu32, _pu32, _pu32]),
    "tdt_det_log": (_d, [_d]),
    "tdt_det_exp": (_d, [_d]),
    "tdt_normal_quantile": (_d, [_d]),
    "tdt_draws": (None, [_u64, _u32, _u64, _pd]),
    "tdt_propose": (ctypes.c_int, [ctypes.POINTER(TdChainParams), _u64, _i64, _pd, _pd, _pd, _pd, _d, _pd]),
    "tdt_chain_profile": (ctypes.c_int, [_vp, ctypes.c_int, _pi64]),
    "tdt_chain_lds": (ctypes.c_int, [_vp, _pi64]),
    "tdt_chain_query_lat": (ctypes.c_int, [_vp, _pd, ctypes.c_int, ctypes.c_int, _pi64]),
    "tdt_chain_query_answers": (ctypes.c_int, [_vp, _pd, ctypes.c_int, ctypes.c_int, _pd, _pd, _pi32]),
    "tdt_tile_filter": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), _pd,
                                       ctypes.c_int, _pd, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint8)]),
    "tdt_set_nn_method": (ctypes.c_int, [_vp, ctypes.c_int]),
    "tdt_nn_bench": (ctypes.c_int, [_vp, _pd, _pd, _pd, _pd, _i64, ctypes.c_int, ctypes.c_int, _pd]),
    "tdt_chain_set_lds_mode": (ctypes.c_int, [_vp, ctypes.c_int]),
    "tdt_chain_set_exact_every": (ctypes.c_int, [_vp, ctypes.c_int]),
    "tdt_exact_sum": (ctypes.c_int, [ctypes.c_int, _pd, _i64, _d, _pd, _pd, _pi32]),
    "tdt_wave_delta_sum": (ctypes.c_int, [ctypes.c_int, _pd, _pd, _pi32, _i64, _d, _pd, _pd]),
    "tdt_block_delta_sum": (ctypes.c_int, [ctypes.c_int, _pd, _pd, _pd, _pi32, _i64, _i64, _pd, _pd,
                                            ctypes.POINTER(ctypes.c_int64), _pi32]),
    "tdt_wave_seq_sum": (ctypes.c_int, [ctypes.c_int, _pd, _i64, _d, _pd, _pd, _pi32]),
    "tdt_set_incremental": (ctypes.c_int, [_vp, ctypes.c_int]),
    "tdt_set_server_post_delay": (ctypes.c_int, [ctypes.c_int]),
    "tdt_rounds_force_exit": (ctypes.c_int, [_vp, _pi32, _i64]),
    "tdt_dropin_timing": (ctypes.c_int, [_vp, ctypes.c_int, _pi64]),
    "tdt_host_nn_query": (ctypes.c_int, [_pd, _pd, _pd, _pd, _i64, _pd, _i64, _pd, _pd, _pd, _pd, _i64, _pd, _pi64]),
    "tdt_shadow_diag": (ctypes.c_int, [_vp, _pi64]),
    "tdt_shadow_profile": (ctypes.c_int, [_vp, _pi64]),
    "tdt_chi2": (ctypes.c_int, [_vp, _pd, ctypes.c_int, _pd]),
    "tdt_accept": (ctypes.c_int, [ctypes.POINTER(TdChainParams), ctypes.c_int, _d, _d, _i64, _d, _d, _d, _d, _d]),
    "tdt_decide_sure": (ctypes.c_int, [ctypes.POINTER(TdChainParams), ctypes.c_int, _d, _d, _i64, _d, _d, _d, _d, _d,
                                       _d, _d]),
}

_lib = None


class TdError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("tdstar error %d: %s" % (code, msg))
        self.code = code


def lib():
    """Load libtdstar.so (raises if it was not built -- no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libtdstar.so not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        older = "TD_LIB_PATH" in os.environ  # (an A/B against an older build: newer testing hooks may be absent)
        for name, (res, args) in SIGNATURES.items():
            if older and name.startswith("tdt_") and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            # array arguments are declared as plain addresses: ptr() hands over an array's address as an
            # integer (numpy's __array_interface__), ~1 us cheaper per argument than a typed ctypes pointer
            # (data_as) -- which, like byref(), is still accepted
            f.argtypes = [_vp if a in _ARRAY_PTRS else a for a in args]
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != TD_OK:
        msg = lib().td_last_error(ctx)
        raise TdError(rc, msg.decode() if msg else "")


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


_ARRAY_PTRS = (_pd, _pi32, _pi64, _pu32)


def ptr(a, t=_pd):
    """The address of a C-contiguous numpy array (the declared element type `t` is documentation:
    callers convert with f64() / np.int32 / np.int64 first), or None.  Through the buffer protocol
    (0.3 us) where the array is writable; `__array_interface__` builds a dict per call (1.2 us, five
    of them per td_evaluate)."""
    if a is None:
        return None
    try:
        return ctypes.addressof(ctypes.c_char.from_buffer(a))
    except (TypeError, ValueError, BufferError):  # read-only or empty: the array interface
        return a.__array_interface__["data"][0]
