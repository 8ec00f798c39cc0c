"""Synthetic inputs in the formats pre_process_data.jl / load_3Dvel.jl read
(none of the real files ship with the reference): lau.vel, raypaths.p,
p_tstar.dat, stations.lst.  Test helper, not a test module."""
import os

import numpy as np

LAT0, LON0, BETA = -23.1, 174.6, 0.463647609  # load_data_Tonga.jl:26-28 (also lau.vel's frame here)


def xy2lonlat(lon0, lat0, beta, x1, y1):
    """Inverse of lonlat2xy (MCsub.jl:5-31)."""
    re, r2d = 6371, 180.0 / np.pi
    yy = (y1 - x1 * np.tan(beta)) * np.cos(beta)
    xx = x1 / np.cos(beta) + yy * np.tan(beta)
    return lon0 + xx * r2d / re, lat0 + yy * r2d / re


def write_all(d, seed=0, nx=7, ny=6, nz=8, nrays=12, trailing_separator=False):
    """Writes the four files into d; returns what they encode."""
    rng = np.random.default_rng(seed)
    xs = np.round(np.linspace(-100.0, 1100.0, nx), 2)
    ys = np.round(np.linspace(-200.0, 520.0, ny), 2)
    zs = np.round(np.sort(rng.uniform(0, 700, nz)), 1)
    zs[0], zs[-1] = 0.0, 700.0
    X, Y = np.meshgrid(xs, ys, indexing="ij")
    lon, lat = xy2lonlat(LON0, LAT0, BETA, X, Y)
    vp = 5.5 + 0.01 * zs[None, None, :] + rng.uniform(-0.3, 0.3, (2, nx, ny, nz))
    vp[1] = vp[1] / 1.75
    with open(os.path.join(d, "lau.vel"), "w") as fh:
        fh.write("%d %d %d\n%.4f %.4f %.9f\n" % (nx, ny, nz, LAT0, LON0, BETA))
        for i in range(nx):
            for j in range(ny):
                fh.write("%.12f %.12f\n" % (lat[i, j], lon[i, j]))
        fh.write(" ".join("%.1f" % z for z in zs) + "\n")
        for p in range(2):
            for i in range(nx):
                for j in range(ny):
                    fh.write(" ".join("%.6f" % v for v in vp[p, i, j]) + "\n")
    rays = []
    with open(os.path.join(d, "raypaths.p"), "w") as fh:
        fh.write("1234567 0 0\n")  # a leading separator (skipped)
        for r in range(nrays):
            n = int(rng.integers(3, 40))
            a = np.column_stack([rng.uniform(-99, 1099, n), rng.uniform(-199, 519, n), rng.uniform(0, 699, n)])
            if r == 0:
                a[0] = (xs[2], ys[3], zs[4])  # on knots
                a[1] = (xs[0], ys[0], zs[0])  # on the grid's corner
                a[2] = (xs[-1], ys[-1], zs[-1])  # and the opposite one
            rays.append(a)
            for row in a:
                fh.write("%.6f %.6f %.6f\n" % tuple(row))
            if r < nrays - 1 or trailing_separator:
                fh.write("1234567 %d\n" % r)
    stations = ["ST%02d" % k for k in range(5)]
    slat = rng.uniform(-25, -15, 5)
    slon = rng.uniform(175, 185, 5)
    with open(os.path.join(d, "stations.lst"), "w") as fh:
        for s, a, b in zip(stations, slat, slon):
            fh.write("%s %.4f %.4f 0.0\n" % (s, a, b))
    traces = []
    with open(os.path.join(d, "p_tstar.dat"), "w") as fh:
        for r in range(nrays):
            s = stations[r % 5]
            row = (s, -20 + r * 0.1, 180 + r * 0.05, 100 + r, 0.5 + 0.01 * r, 0.1, 0.02, 0.003 * r)
            traces.append(row)
            fh.write("%s %.4f %.4f %.1f %.4f %.4f %.4f %.5f\n" % row)
    return dict(xs=xs, ys=ys, zs=zs, vp=vp, rays=rays, stations=dict(zip(stations, zip(slat, slon))),
                traces=traces)
