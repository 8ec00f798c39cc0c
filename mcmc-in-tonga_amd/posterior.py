"""Posterior cross-sections -- the numbers behind plot_model_hist (MCsub.jl:753-825).

For every y-slice (xz maps, MCsub.jl:756-785) and z-slice (xy maps,
MCsub.jl:789-820) the reference evaluates every saved model at every grid
node with v_nearest (`[v_nearest(xs, l0, zs, ...) for xs in xVec, zs in zVec]`,
an nx x nz matrix, xs fastest), then takes the mean and standard deviation
over the models and masks nodes whose std exceeds 5.  Here the model sweep
and both statistics run on the GPU (td_rasterize); plotting is out of scope.
"""
import numpy as np

from .forward import context_for


def _flatten(model_hist):
    """model_hist[i][j] (chain i, saved model j, MCsub.jl:761-763) or a flat list."""
    out = []
    for item in model_hist:
        if isinstance(item, (list, tuple)):
            out.extend(item)
        else:
            out.append(item)
    return out


def section(ctx, models, xs, ys, zs, axis):
    """One cross-section: axis "xz" (ys a scalar) or "xy" (zs a scalar).
    Returns (mean, std) as len(first) x len(second) matrices."""
    if axis == "xz":
        a, b = np.asarray(xs, dtype=np.float64), np.asarray(zs, dtype=np.float64)
        qx, qz = np.tile(a, len(b)), np.repeat(b, len(a))
        qy = np.full(qx.shape, float(ys))
    elif axis == "xy":
        a, b = np.asarray(xs, dtype=np.float64), np.asarray(ys, dtype=np.float64)
        qx, qy = np.tile(a, len(b)), np.repeat(b, len(a))
        qz = np.full(qx.shape, float(zs))
    else:
        raise ValueError(axis)
    mean, std, _ = ctx.rasterize([m.cells() for m in models], qx, qy, qz)
    shape = (len(b), len(a))  # column-major nx x n2 matrix, xs fastest
    return mean.reshape(shape).T.copy(), std.reshape(shape).T.copy()


def plot_model_hist(model_hist, dataStruct, TD_parameters, cmax=None):  # noqa: N802 -- reference name
    """MCsub.jl:753-825 without the plots: {("xz", y) | ("xy", z): {"mean",
    "std", "masked"}} with masked = mean where std <= 5, NaN elsewhere (:776-781)."""
    ctx = context_for(dataStruct)
    models = _flatten(model_hist)
    xv, yv, zv = (np.asarray(v, dtype=np.float64) for v in (dataStruct.xVec, dataStruct.yVec, dataStruct.zVec))
    maps = {}
    todo = []
    if TD_parameters.xzMap:
        todo += [("xz", l0) for l0 in TD_parameters.ySlice]
    if TD_parameters.xyMap:
        todo += [("xy", l0) for l0 in TD_parameters.zSlice]
    for axis, l0 in todo:
        if axis == "xz":
            mean, std = section(ctx, models, xv, l0, zv, "xz")
        else:
            mean, std = section(ctx, models, xv, yv, l0, "xy")
        mask = np.where(std > 5, np.nan, 1.0)
        maps[(axis, l0)] = {"mean": mean, "std": std, "masked": mask * mean}
    return maps
