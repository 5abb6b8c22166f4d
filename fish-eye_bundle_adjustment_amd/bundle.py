"""Reference-named host API over libfba.so.

The reference's hot path is a set of MATLAB functions plus an inline loop; these wrappers keep
their names, argument meaning and error behaviour (first output = error flag, 0 ok / 1 fail) so a
caller can switch function by function:

    [error, xhat, xhatnames] = Buildxhat(data, ...)            functions/Buildxhat.m:2
    [error, A, misclosure, G, dist_scaling] = BuildAwG(data, xhat)   functions/BuildAwG.m:14
    RSD = BuildRSD(v, data, xhat)                               functions/BuildRSD.m:1
    main_error = main(folder, plot)                             main.m:10

Every numeric result comes from the HIP path (libfba.so); nothing here computes a Jacobian, a
normal matrix or a solve.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass

import numpy as np

from . import capi
from .io import Dataset, IngestError, load_folder, xhat_names


def _ctx(data: Dataset, device=0, **kw):
    ctx = getattr(data, "_fba_ctx", None)
    if ctx is None or kw:
        ctx = capi.Context(data.pack(), capi.make_settings(data.settings), device=device, **kw)
        if not kw:
            data._fba_ctx = ctx
    return ctx


def Buildxhat(data: Dataset):
    """Buildxhat.m:2 -> (error, xhat, xhatnames)."""
    try:
        ctx = _ctx(data)
        return 0, ctx.buildxhat(), xhat_names(data)
    except capi.FBAError as e:
        print(f"Error Buildxhat(): {e}")
        return 1, None, None


def BuildAwG(data: Dataset, xhat):
    """BuildAwG.m:14 -> (error, A, misclosure, G, dist_scaling); A dense n x u (debug/parity form).

    G is the scalar 0 when inner constraints are off (BuildAwG.m:38); dist_scaling columns 1-2
    carry the reference's 1-based xhat indices of the first radial / decentering unknown."""
    try:
        ctx = _ctx(data)
        A, w, G, ds = ctx.build_awg(np.asarray(xhat, dtype=np.float64))
        return 0, A, w, (G if G is not None else 0), ds
    except capi.FBAError as e:
        print(f"BuildAwG: {e}")
        return 1, None, None, None, None


def BuildRSD(v, data: Dataset, xhat):
    """BuildRSD.m:1-43: rows [targetID, imageID, x, y, r, vx, vy, vr, vt] -- the radial / tangential
    split of a given v, with xp, yp from xhat where estimated (fba_build_rsd on the device)."""
    rsd = _ctx(data).build_rsd(v, xhat)
    return [[data.pho_target[i], data.pho_image[i], data.xy[i, 0], data.xy[i, 1], *rsd[i]] for i in range(len(rsd))]


@dataclass
class Adjustment:
    xhat: np.ndarray
    xhatnames: list
    iterations: int
    deltasum: np.ndarray
    v: np.ndarray
    rsd: np.ndarray          # (n_pts, 5): r vx vy vr vt
    rms: tuple               # RMSx, RMSy, RMS
    sigma02: float
    seconds: float
    cx_diag: np.ndarray = None   # diag of the final Cx (sigma02-scaled, distortions de-scaled)
    corr: np.ndarray = None      # (numImg, u_img+u_cam, u_img+u_cam) EOP/IOP Correlation sub-blocks


def adjust(data: Dataset, device=0, verbose=False, covariance=True) -> Adjustment:
    """main.m:386-602 on one GPU: Buildxhat, the Gauss-Newton loop, residuals, sigma0^2 and (with
    covariance=True) the post-fit Cx diagonal and correlation sub-blocks (main.m:428-482, :602)."""
    t0 = time.perf_counter()
    ctx = capi.Context(data.pack(), capi.make_settings(data.settings), device=device, verbose=verbose)
    try:
        it, hist = ctx.adjust()
        t1 = time.perf_counter()
        xhat = ctx.get_xhat()
        v, rsd, st = ctx.residuals()
        cxd, corr = ctx.covariance(st[3]) if covariance else (None, None)
    finally:
        ctx.close()
    return Adjustment(xhat=xhat, xhatnames=xhat_names(data), iterations=it, deltasum=hist, v=v, rsd=rsd,
                      rms=(st[0], st[1], st[2]), sigma02=st[3], seconds=t1 - t0, cx_diag=cxd, corr=corr)


def write_outputs(data: Dataset, res: Adjustment, folder):
    """main.m:631-958: the .out report, the .rsd residual table and the .par camera file
    (fba_amd/report.py)."""
    from . import report
    name = os.path.splitext(data.settings["Output_Filename"])[0]
    out = os.path.join(folder, data.settings["Output_Filename"])
    par = report.write_out(out, data, res, res.seconds)
    report.write_rsd(os.path.join(folder, name + ".rsd"), data, res.rsd)
    report.write_par(os.path.join(folder, name + ".par"), par)
    return out


def main(folder: str = "", plot: bool = False, device=0) -> int:
    """main.m:10 contract: returns main_error (0 ok, 1 failure).  Plots (main.m:502-584) are not
    produced; `plot` is accepted for signature compatibility."""
    project_dir = os.getcwd()
    folder = folder or project_dir
    try:
        data = load_folder(folder, project_dir=None if folder == project_dir else project_dir)
        res = adjust(data, device=device)
        write_outputs(data, res, folder)
    except (IngestError, capi.FBAError) as e:
        print(f"Error: {e}")
        return 1
    return 0
