"""GPU parity: the HIP path (libfba.so through its C-ABI) against the oracle on the same inputs.

Tolerances (fp64 throughout):
* BuildAwG (A, w, G, dist_scaling): A per column <= 1e-12 of the column's max |entry|; w <= 1e-12
  of the image-coordinate scale (w = f - x with |f| ~ 1e3 px); G and dist_scaling <= 1e-14.
* Full adjustment: same iteration count; xhat <= 1e-9 relative per parameter group (north_star
  bar; distortion terms compared in the reference's scaled units K_j*rmax^(2j), P*rmax^2);
  sigma0^2 <= 1e-9 relative; v <= 1e-9 of max|v| (v uses the last linearisation, main.m:569).
The oracle solves with the reference's explicit bordered inverse (main.m:432); the GPU with a
Schur-reduced Cholesky, so agreement is limited by the conditioning of the normal equations, not
by rounding of either side.
"""
import ctypes

import numpy as np
import pytest

from conftest import CAM0_VARIANTS, group_rel_err

pytestmark = pytest.mark.gpu


def _ctx(fba, ds, **kw):
    return fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings), **kw)


def _check_awg(fba, oracle, ds, od, xhat):
    ctx = _ctx(fba, ds)
    try:
        A, w, G, dsc = ctx.build_awg(xhat)
    finally:
        ctx.close()
    Ao, wo, Go, dso = oracle.build_awg(od, xhat)
    colmax = np.maximum(np.abs(Ao).max(axis=0), 1e-300)
    err = np.abs(A - Ao).max(axis=0) / colmax
    assert err.max() <= 1e-12, (err.max(), int(err.argmax()))
    assert ((A != 0) <= (Ao != 0) | (np.abs(A) < 1e-300)).all()
    scale = np.abs(ds.xy).max()
    assert np.abs(w - wo).max() <= 1e-12 * scale
    if Go is not None:
        np.testing.assert_allclose(G, Go, rtol=1e-14, atol=1e-14 * np.abs(Go).max())
    np.testing.assert_allclose(dsc, dso, rtol=1e-14)


@pytest.mark.parametrize("variant", sorted(CAM0_VARIANTS))
def test_buildawg_cam0(fba, oracle, cam0_folders, variant):
    ds = fba.load_folder(cam0_folders[variant])
    od = oracle.load_folder(cam0_folders[variant])
    ctx = _ctx(fba, ds)
    x0 = ctx.buildxhat()
    ctx.close()
    x0o, _ = oracle.buildxhat(od)
    np.testing.assert_array_equal(x0, x0o)  # Buildxhat.m layout, bit-exact
    _check_awg(fba, oracle, ds, od, x0)
    rng = np.random.default_rng(1)
    xp = x0 * (1 + 1e-4 * rng.standard_normal(len(x0)))
    _check_awg(fba, oracle, ds, od, xp)


@pytest.mark.parametrize("variant", sorted(CAM0_VARIANTS))
def test_adjust_cam0(fba, oracle, cam0_folders, variant):
    ds = fba.load_folder(cam0_folders[variant])
    od = oracle.load_folder(cam0_folders[variant])
    ro = oracle.adjust(od)
    res = fba.adjust(ds)
    assert res.iterations == ro.iterations
    err = group_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling)
    assert max(err.values()) <= 1e-9, err
    assert res.sigma02 == pytest.approx(ro.sigma02, rel=1e-9)
    np.testing.assert_allclose(res.rms, ro.rms, rtol=1e-9)
    assert np.abs(res.v - ro.v).max() <= 1e-9 * np.abs(ro.v).max()
    np.testing.assert_allclose(res.rsd[:, 0], ro.rsd[:, 0], rtol=1e-12)
    assert np.abs(res.rsd[:, 1:] - ro.rsd[:, 1:]).max() <= 1e-9 * np.abs(ro.rsd[:, 1:]).max()
    # deltasum history: early iterations to 1e-9, the converged tail is rounding-level noise
    np.testing.assert_allclose(res.deltasum[:2], ro.deltasum[:2], rtol=1e-6)


@pytest.mark.parametrize("typ", ["fisheye", "pinhole", "equisolid", "orthographic", "stereographic"])
def test_adjust_synthetic_types(fba, oracle, tmp_path, typ):
    from fba_amd import synth
    sc = synth.generate(12, 240, seed=17, typ=typ)
    folder = synth.write_folder(sc, str(tmp_path / typ))
    ds = fba.load_folder(folder)
    od = oracle.load_folder(folder)
    ro = oracle.adjust(od)
    res = fba.adjust(ds)
    assert res.iterations == ro.iterations
    err = group_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling)
    assert max(err.values()) <= 1e-9, err
    assert res.sigma02 == pytest.approx(ro.sigma02, rel=1e-9)


def test_step_is_deterministic(fba, cam0_folders):
    ds = fba.load_folder(cam0_folders["stage3_fisheye"])
    out = []
    for _ in range(2):
        ctx = _ctx(fba, ds)
        d = [ctx.step() for _ in range(3)]
        out.append((d, ctx.get_xhat()))
        ctx.close()
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])


class _Hip:
    def __init__(self):
        self.lib = ctypes.CDLL("libamdhip64.so")
        self.lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

    def d2h(self, ptr, n):
        a = np.empty(n)
        assert self.lib.hipMemcpy(a.ctypes.data, ptr, n * 8, 2) == 0
        return a

    def h2d(self, ptr, a):
        assert self.lib.hipMemcpy(ptr, a.ctypes.data, a.size * 8, 1) == 0


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ranks_reassemble_single_gpu_result(fba, cam0_folders, world):
    """world ranks on one GPU, reduce buffers summed on the host: same iterates as one context."""
    ds = fba.load_folder(cam0_folders["stage3_pinhole"])
    hip = _Hip()
    single = _ctx(fba, ds)
    ranks = [_ctx(fba, ds, rank=r, world=world) for r in range(world)]
    for it in range(3):
        d1 = single.step()
        for c in ranks:
            c.accumulate()
        bufs = [c.reduce_buffer() for c in ranks]
        total = sum(hip.d2h(p, n) for p, n in bufs)
        for p, n in bufs:
            hip.h2d(p, total)
        parts = [c.solve_update() for c in ranks]
        assert sum(parts) == pytest.approx(d1, rel=1e-9)
    xs = single.get_xhat()
    xr = sum(c.get_xhat(owned_only=True) for c in ranks)
    names = fba.xhat_names(ds)
    _, _, _, dsc = single.build_awg(xs)
    err = group_rel_err(xr, xs, names, dsc)
    assert max(err.values()) <= 1e-10, err
    single.close()
    for c in ranks:
        c.close()
