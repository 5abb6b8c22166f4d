"""GPU parity on the inputs the reference accepts beyond the single-camera case (fba_general.hip).

The reference loops over every PHO row (BuildAwG.m:46), places each observation's IOP / distortion
columns by its own camera (:448-451), and its tie columns are camera-independent (:501-502), so it
takes tie points seen through several cameras (a multi-camera rig sharing its targets, main.m:323),
tie points seen by any number of images, and a point measured twice in one image.  Such points take
the general path (k_gen_point / k_gen_keys / k_red_gen / k_gen_backsub); the rest stay on the
chunked fast path -- the "blocks" layouts mix both.

Tolerances as tests/test_gpu_parity.py: BuildAwG A per column <= 1e-12; full adjustment: same
iteration count, xhat <= 1e-9 relative per parameter group (distortion terms in scaled units),
sigma0^2 <= 1e-9; covariance diag <= 1e-8 relative and correlation blocks <= 5e-9 absolute.
"""
import numpy as np
import pytest

from conftest import dist_scaling_of, group_rel_err

pytestmark = pytest.mark.gpu

SCENES = {
    "rig2": dict(n_img=18, n_tie=300, n_cam=2),                          # every point through both cameras
    "rig3_blocks": dict(n_img=24, n_tie=400, n_cam=3, cam_layout="blocks"),  # general + regular points
    "dup": dict(n_img=16, n_tie=300, n_dup=30),                         # repeated measurements
    "rig2_dup": dict(n_img=18, n_tie=300, n_cam=2, n_dup=20),
}


def _folder(tmp_path, name, **kw):
    from fba_amd import synth
    kw = dict(kw)
    n_img, n_tie = kw.pop("n_img"), kw.pop("n_tie")
    return synth.write_folder(synth.generate(n_img, n_tie, seed=41, **kw), str(tmp_path / name))


def _general_count(od):
    """tie points the chunked path cannot take: several cameras, > 256 images, a repeated image"""
    cams, imgs = {}, {}
    for t, k, e in zip(od.tie_index, od.cam_num, od.ext_index):
        if t < 0:
            continue
        cams.setdefault(int(t), set()).add(int(k))
        imgs.setdefault(int(t), []).append(int(e))
    return sum(1 for t in cams if len(cams[t]) > 1 or len(imgs[t]) > 256 or len(set(imgs[t])) < len(imgs[t]))


@pytest.mark.parametrize("name", sorted(SCENES))
def test_buildawg_general(fba, oracle, tmp_path, name):
    folder = _folder(tmp_path, name, **SCENES[name])
    ds = fba.load_folder(folder)
    od = oracle.load_folder(folder)
    assert _general_count(od) > 0
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
    try:
        x0 = ctx.buildxhat()
        A, w, G, dsc = ctx.build_awg(x0)
    finally:
        ctx.close()
    Ao, wo, Go, dso = oracle.build_awg(od, x0)
    colmax = np.maximum(np.abs(Ao).max(axis=0), 1e-300)
    assert (np.abs(A - Ao).max(axis=0) / colmax).max() <= 1e-12
    assert np.abs(w - wo).max() <= 1e-12 * np.abs(ds.xy).max()
    np.testing.assert_allclose(dsc, dso, rtol=1e-14)


@pytest.mark.parametrize("name", sorted(SCENES))
def test_adjust_general(fba, oracle, tmp_path, name):
    folder = _folder(tmp_path, name, **SCENES[name])
    ds = fba.load_folder(folder)
    od = oracle.load_folder(folder)
    ro = oracle.adjust(od)
    res = fba.adjust(ds)
    assert res.iterations == ro.iterations
    err = group_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling)
    assert max(err.values()) <= 1e-9, err
    assert res.sigma02 == pytest.approx(ro.sigma02, rel=1e-9)
    np.testing.assert_allclose(res.deltasum, ro.deltasum, rtol=0, atol=1e-9 * ro.deltasum[0])
    print(f"general points: v max error {np.abs(res.v - ro.v).max() / np.abs(ro.v).max():.2e} of its scale")
    # (round 6, profiles/r06_v8_covariance_errors.log: v <= 6.5e-13 of its scale, diag(Cx) <= 5.7e-10
    # relative, correlations <= 4.8e-11 on image 0 -- held to 1e-10, 1e-8 and 5e-9)
    assert np.abs(res.v - ro.v).max() <= 1e-10 * np.abs(ro.v).max()
    # covariance: camera-side diagonal and EOP/IOP correlation blocks, and every tie variance
    cdo, corro = oracle.covariance(od, ro)
    print(f"general points covariance: diag(Cx) max relative error {np.max(np.abs(res.cx_diag - cdo) / np.abs(cdo)):.2e}")
    np.testing.assert_allclose(res.cx_diag, cdo, rtol=1e-8, atol=0)
    u_img, u_cam = oracle.counts(od.settings)
    for e in range(od.numImg):
        idx = list(range(e * u_img, (e + 1) * u_img))
        k = int(od.cam_num[np.nonzero(od.ext_index == e)[0][0]])
        idx += list(range(u_img * od.numImg + k * u_cam, u_img * od.numImg + (k + 1) * u_cam))
        np.testing.assert_allclose(res.corr[e], corro[np.ix_(idx, idx)], rtol=0, atol=5e-9)
        print(f"general points: image {e} correlation block max absolute error "
              f"{np.max(np.abs(res.corr[e] - corro[np.ix_(idx, idx)])):.2e}") if e == 0 else None


def test_point_seen_by_300_images(fba, tmp_path):
    """A tie point observed by >= 300 images (more than one k_lin_reduce chunk holds) next to ordinary
    points: the whole adjustment against the C oracle's direct bordered solve (the scene is too large
    for the dense oracle)."""
    import fba_cpu
    import fba_oracle
    from fba_amd import synth
    fba_cpu.build()
    sc = synth.generate(400, 1500, seed=43, n_wide=2, wide_min_obs=300)
    folder = synth.write_folder(sc, str(tmp_path / "wide"))
    od = fba_oracle.load_folder(folder)
    counts = np.bincount(od.tie_index[od.tie_index >= 0])
    assert counts.max() >= 300
    ref = fba_cpu.CpuAdjustment(od, solver="kkt")
    it = ref.adjust()
    _, s02 = ref.residuals()
    res = fba.adjust(fba.load_folder(folder), covariance=False)
    assert res.iterations == it
    err = group_rel_err(res.xhat, ref.xhat, ref.names, dist_scaling_of(od))
    assert max(err.values()) <= 1e-9, err
    assert abs(res.sigma02 - s02) <= 1e-9 * s02
    np.testing.assert_allclose(res.deltasum, ref.deltasum, rtol=0, atol=1e-9 * ref.deltasum[0])
    ref.close()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_general_points(fba, tmp_path, world):
    """General points are whole points of one rank: world rank contexts on one GPU, reduce buffers
    summed on the host, reproduce the single context's iterates."""
    import ctypes
    folder = _folder(tmp_path, "rig", **SCENES["rig3_blocks"])
    ds = fba.load_folder(folder)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

    def d2h(p, n):
        a = np.empty(n)
        assert hip.hipMemcpy(a.ctypes.data, p, n * 8, 2) == 0
        return a

    mk = lambda **kw: fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings), **kw)  # noqa: E731
    single = mk()
    ranks = [mk(rank=r, world=world) for r in range(world)]
    try:
        d_first = None
        for _ in range(3):
            d1 = single.step()
            d_first = d_first or d1
            for c in ranks:
                c.accumulate()
                c.synchronize()
            bufs = [c.reduce_buffer() for c in ranks]
            total = sum(d2h(p, n) for p, n in bufs)
            for p, n in bufs:
                assert hip.hipMemcpy(p, total.ctypes.data, n * 8, 1) == 0
            parts = [c.solve_update() for c in ranks]
            assert abs(sum(parts) - d1) <= 1e-7 * d_first
        xs = single.get_xhat()
        xr = sum(c.get_xhat(owned_only=True) for c in ranks)
        _, _, _, dsc = single.build_awg(xs)
        err = group_rel_err(xr, xs, fba.xhat_names(ds), dsc)
        assert max(err.values()) <= 1e-10, err
    finally:
        single.close()
        for c in ranks:
            c.close()
