"""GPU debug: compare the device-assembled reduced system and one GN step with numpy."""
import os
import sys

import numpy as np
import scipy.linalg as sl

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fba_import  # noqa: E402
import fba_oracle as o  # noqa: E402
from conftest import group_rel_err, variant_folder, CAM0_VARIANTS  # noqa: E402

fba = fba_import.load()
from fba_amd.parallel import hip_memcpy  # noqa: E402

memcpy = hip_memcpy()
variant = sys.argv[1] if len(sys.argv) > 1 else "stage3_pinhole"
import tempfile
folder = variant_folder(tempfile.mkdtemp(), variant, CAM0_VARIANTS[variant])
ds = fba.load_folder(folder)
od = o.load_folder(folder)
ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
x0 = ctx.buildxhat()
nI, cw = ds.numImg, 10
uc = 6 * nI + cw
n_pad = (uc + 63) // 64 * 64

# numpy reduced system at x0 (reference layout == full layout here: all parameters estimated)
A, w, G, dsc = o.build_awg(od, x0)
P = o.weights(od)
u = A.T @ (P * w)
N = A.T @ (P[:, None] * A)
Ncc, Ncp, Npp = N[:uc, :uc], N[:uc, uc:], N[uc:, uc:]
Vi = np.linalg.inv(Npp)
S = Ncc - Ncp @ Vi @ Ncp.T
r = u[:uc] - Ncp @ Vi @ u[uc:]

import ctypes
_hip = ctypes.CDLL("libamdhip64.so")
ctx.accumulate()
assert _hip.hipDeviceSynchronize() == 0
ptr, n = ctx.reduce_buffer()
buf = np.empty(n)
assert memcpy(buf.ctypes.data, ptr, n * 8, 2) == 0
Sg = buf[: n_pad * n_pad].reshape(n_pad, n_pad)[:uc, :uc]
rg = buf[n_pad * n_pad: n_pad * n_pad + uc]
Sl = np.tril(S)
Sgl = np.tril(Sg)
d = np.abs(Sgl - Sl)
scale = np.sqrt(np.outer(np.diag(S), np.diag(S)))
rel = d / np.maximum(scale, 1e-300)
i, j = np.unravel_index(np.argmax(rel), rel.shape)
print(f"S: max |dS|/sqrt(SiiSjj) = {rel.max():.3e} at ({i},{j}) S={S[i, j]:.6e} Sg={Sg[i, j]:.6e}")
for name, (a0, a1, b0, b1) in {"img-img": (0, 6 * nI, 0, 6 * nI), "cam-img": (6 * nI, uc, 0, 6 * nI),
                                "cam-cam": (6 * nI, uc, 6 * nI, uc)}.items():
    print(f"  {name}: {rel[a0:a1, b0:b1].max():.3e}")
print(f"r: max rel {np.max(np.abs(rg - r)) / np.max(np.abs(r)):.3e}")

# one step: GPU vs oracle, and numpy solve of the GPU's own system
dsum = ctx.solve_update()
xg = ctx.get_xhat()
r1 = o.adjust(od, max_iter=1)
print("deltasum gpu %.15e oracle %.15e" % (dsum, r1.deltasum[0]))
print("step-1 xhat:", {k: f"{v:.1e}" for k, v in group_rel_err(xg, r1.xhat, r1.names, r1.dist_scaling).items()})

if G is None:
    sys.exit(0)
Sfull = np.tril(Sg) + np.tril(Sg, -1).T
Gc = G[:uc]
KKT = np.block([[Sfull, Gc], [Gc.T, np.zeros((7, 7))]])
dc = np.linalg.solve(KKT, np.concatenate([-rg, np.zeros(7)]))[:uc]
KKT2 = np.block([[S, Gc], [Gc.T, np.zeros((7, 7))]])
dc2 = np.linalg.solve(KKT2, np.concatenate([-r, np.zeros(7)]))[:uc]
print("numpy solve of GPU S vs numpy S: max rel dc", np.max(np.abs(dc - dc2) / np.maximum(np.abs(dc2), 1e-300)))
a2 = np.trace(Sfull[:6 * nI, :6 * nI]) / np.sum(Gc ** 2)
Gt = np.sqrt(a2) * Gc
M = Sfull + Gt @ Gt.T
L = np.linalg.cholesky(M)
Y = sl.solve_triangular(L, np.column_stack([rg, Gt]), lower=True)
H = Y[:, 1:].T @ Y[:, 1:]
k = -np.linalg.solve(H, Y[:, 1:].T @ Y[:, 0])
dc3 = -sl.solve_triangular(L.T, Y[:, 0] + Y[:, 1:] @ k, lower=False)
print("numpy border-Cholesky of GPU S vs numpy KKT of GPU S: max rel", np.max(np.abs(dc3 - dc) / np.maximum(np.abs(dc), 1e-300)))
print("diag M translation %.3e  S %.3e" % (M[0, 0], Sfull[0, 0]))
dg = xg[:uc] - x0[:uc]
sc = np.ones(uc)
for jj in range(5):
    sc[6 * nI + 3 + jj] = dsc[0, 2 + jj]
sc[6 * nI + 8] = sc[6 * nI + 9] = dsc[0, 2]
print("GPU dc vs numpy(GPU S) dc, per entry rel (scaled):")
e = np.abs(dg - dc / sc) / np.maximum(np.abs(dc / sc), 1e-300)
e3 = np.abs(dg - dc3 / sc) / np.maximum(np.abs(dc3 / sc), 1e-300)
print("  vs numpy border-Cholesky: eop max", e3[:6 * nI].max(), " cam", e3[6 * nI:])
print("  eop max", e[:6 * nI].max(), " cam", e[6 * nI:])
