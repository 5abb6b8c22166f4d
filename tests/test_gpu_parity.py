"""GPU parity: the HIP path (libfba.so through its C-ABI) against the oracle on the same inputs.

Tolerances (fp64 throughout):
* BuildAwG (A, w, G, dist_scaling): A per column <= 1e-12 of the column's max |entry|; w <= 1e-12
  of the image-coordinate scale (w = f - x with |f| ~ 1e3 px); G and dist_scaling <= 1e-14.
* Full adjustment: same iteration count; xhat <= 1e-9 relative per element (SURVEY section 8(c);
  conftest.elem_rel_err: entries below 1e-6 of their group's scale -- none on these scenes -- against
  1e-15 of that scale; the small synthetic scenes' floor is conftest.SMALL_SCENE_FLOOR) and per
  parameter group (north_star bar; distortion terms compared in the reference's scaled units
  K_j*rmax^(2j), P*rmax^2);
  sigma0^2 and the first deltasum <= 1e-9 relative -- or, where larger, 20x the spread of the
  reference restatement against itself under rounding-level changes (conftest.solver_spread): on
  cam0 run with a fish-eye model that spread reaches 1e-4 in k3..k5 (tests/test_oracle.py
  test_fisheye_cam0_is_path_sensitive); on the shipped pinhole configuration it is < 2e-12 for
  xhat, so 1e-9 applies there.
The oracle solves with the reference's explicit bordered inverse (main.m:432); the GPU with a
Schur-reduced Cholesky, so agreement is limited by the conditioning of the normal equations, not
by rounding of either side.
"""
import ctypes

import numpy as np
import pytest

from conftest import CAM0_VARIANTS, SMALL_SCENE_FLOOR, elem_rel_err, group_rel_err, solver_spread

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
    err.update({"e_" + g: v for g, v in elem_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling).items()})
    spread = solver_spread(oracle, od, ro)
    err["sigma02"] = abs(res.sigma02 - ro.sigma02) / ro.sigma02
    err["deltasum0"] = abs(res.deltasum[0] - ro.deltasum[0]) / ro.deltasum[0]
    for g, e in err.items():
        # 1e-9 (north_star), or 20x the reference restatement's own rounding/path spread
        assert e <= max(1e-9, 20 * spread[g]), (g, e, spread[g])
    vtol = max(1e-9, 20 * spread["sigma02"])
    np.testing.assert_allclose(res.rms, ro.rms, rtol=vtol)
    assert np.abs(res.v - ro.v).max() <= 10 * vtol * np.abs(ro.v).max()
    # r = |(x, y) - (xp, yp)|: its error is the principal point's, on the scale of the sensor
    xptol = 20 * max(spread.get("xp", 0), spread.get("yp", 0)) * np.abs(ds.xy).max()
    np.testing.assert_allclose(res.rsd[:, 0], ro.rsd[:, 0], rtol=1e-12, atol=max(1e-9, xptol))
    assert np.abs(res.rsd[:, 1:] - ro.rsd[:, 1:]).max() <= 10 * vtol * np.abs(ro.rsd[:, 1:]).max()


@pytest.mark.parametrize("variant", sorted(CAM0_VARIANTS))
def test_adjust_cam0_matches_reference_text(fba, oracle, cam0_folders, variant):
    """The HIP path against the reference's OWN .m text run on the same files (tests/golden/
    ref_cam0_<variant>.npz: main.m:61-628, Buildxhat.m, BuildAwG.m, BuildRSD.m, sumabs.m executed by
    tests/golden/mlang.py; bars as tests/test_reference_text.py holds the oracle): Buildxhat exact,
    BuildAwG <= 1e-12, the same iteration count, xhat after every iteration <= 1e-9 per element on the
    pinhole variants (the converged xhat against 20x the restatement spread on the fish-eye family),
    deltasum history, sigma0^2, RMS, v, RSD, and on the pinhole variants diag(Cx) (1e-9; the distortion
    terms' variances 1e-8) and the EOP/IOP correlation blocks (1e-9 absolute)."""
    from test_reference_text import PINHOLE, assert_within, check_awg, load_ref, loop_errors
    g = load_ref(variant)
    ds = fba.load_folder(cam0_folders[variant])
    ctx = _ctx(fba, ds)
    try:
        x0 = ctx.buildxhat()
        np.testing.assert_array_equal(x0, g["xhat_hist"][0])
        A, w, G, dsc = ctx.build_awg(x0)
        check_awg(A, w, G, dsc, g, np.abs(ds.xy).max())
        hist, dsum = [x0], []
        for _ in range(int(g["iterations"])):
            dsum.append(ctx.step())
            hist.append(ctx.get_xhat())
        v, rsd, st = ctx.residuals()
    finally:
        ctx.close()
    res = fba.adjust(ds)
    assert res.iterations == int(g["iterations"])
    np.testing.assert_array_equal(res.xhat, hist[-1])
    err = loop_errors(g, hist, dsum, st[3], st[:3], v, rsd, g["dist_scaling"], every_iteration=variant in PINHOLE)
    spread = {}
    if variant not in PINHOLE:
        od = oracle.load_folder(cam0_folders[variant])
        spread = solver_spread(oracle, od, oracle.adjust(od))
    assert_within(err, variant, spread)
    if variant in PINHOLE:
        # diag(Cx) 1e-9 relative, except the distortion terms' variances (K_j, P_j: the normal matrix's
        # ill-conditioned directions, the selected inverse of the Cholesky factor against the reference's
        # explicit inverse): 1e-8, measured 2.0e-9 on k1..k5 of the Stage-3 variants
        dist = np.array([nm[0] in "kp" and nm[1:2].isdigit() for nm in g["names"]])
        np.testing.assert_allclose(res.cx_diag[~dist], g["cx_diag"][~dist], rtol=1e-9, atol=0)
        np.testing.assert_allclose(res.cx_diag[dist], g["cx_diag"][dist], rtol=1e-8, atol=0)
        np.testing.assert_allclose(res.corr, g["corr_blocks"], rtol=0, atol=1e-9)


def test_adjust_synthetic_fisheye_matches_reference_text(fba, synth_fe):
    """SURVEY section 8(c) golden 3 on the device: the HIP path on the synthetic equidistant fish-eye free
    network (conftest.SYNTH_FE: 12 images x 300 tie points, inner constraints, no control, all EOP + IOP +
    5 radial + 2 decentering) against the reference's own main.m / BuildAwG.m text run on the same files
    (tests/golden/ref_synth_fisheye_free.npz).  The scene is well conditioned, so the tight bars hold on
    EVERY iteration: Buildxhat exact, BuildAwG <= 1e-12, the same iteration count, xhat after every
    iteration <= 1e-9 per element (entries below 10% of their group's scale at 1e-10 of that scale,
    conftest.SMALL_SCENE_FLOOR), the deltasum history (1e-6 relative or 1e-9 absolute), sigma0^2 and RMS
    <= 1e-9, v and RSD <= 1e-9 of their scale, diag(Cx) <= 1e-9 (the distortion terms' variances 1e-8, as
    on cam0) and the EOP/IOP correlation blocks <= 1e-9 absolute."""
    from test_reference_text import assert_within, check_awg, load_synth_fe, loop_errors
    g = load_synth_fe(synth_fe)
    ds = fba.load_folder(synth_fe[0])
    ctx = _ctx(fba, ds)
    try:
        x0 = ctx.buildxhat()
        np.testing.assert_array_equal(x0, g["xhat_hist"][0])
        A, w, G, dsc = ctx.build_awg(x0)
        check_awg(A, w, G, dsc, g, np.abs(ds.xy).max())
        hist, dsum = [x0], []
        for _ in range(int(g["iterations"])):
            dsum.append(ctx.step())
            hist.append(ctx.get_xhat())
        v, rsd, st = ctx.residuals()
    finally:
        ctx.close()
    res = fba.adjust(ds)
    assert res.iterations == int(g["iterations"])
    np.testing.assert_array_equal(res.xhat, hist[-1])
    err = loop_errors(g, hist, dsum, st[3], st[:3], v, rsd, g["dist_scaling"], floor=SMALL_SCENE_FLOOR)
    print("HIP vs reference text (synthetic fish-eye):", {k: f"{e:.1e}" for k, e in err.items()})
    assert_within(err, "stage3_pinhole", {})
    dist = np.array([nm[0] in "kp" and nm[1:2].isdigit() for nm in g["names"]])
    np.testing.assert_allclose(res.cx_diag[~dist], g["cx_diag"][~dist], rtol=1e-9, atol=0)
    np.testing.assert_allclose(res.cx_diag[dist], g["cx_diag"][dist], rtol=1e-8, atol=0)
    np.testing.assert_allclose(res.corr, g["corr_blocks"], rtol=0, atol=1e-9)


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
    err = elem_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling, floor=SMALL_SCENE_FLOOR)
    assert max(err.values()) <= 1e-9, err
    assert res.sigma02 == pytest.approx(ro.sigma02, rel=1e-9)


@pytest.mark.parametrize("nk", [1, 3, 6, 7, 8])
def test_adjust_synthetic_radial_terms(fba, oracle, tmp_path, nk):
    """Num_Radial_Distortions other than the bundled 5 (BuildAwG.m:18-20, :424-438): nK >= 6 takes the
    smaller k_lin_reduce chunk capacities (chunk_pts / chunk_terms) that keep its LDS within 160 KiB."""
    from fba_amd import synth
    sc = synth.generate(12, 240, seed=23, typ="fisheye")
    folder = synth.write_folder(sc, str(tmp_path / f"nk{nk}"), nk=nk)
    ds = fba.load_folder(folder)
    od = oracle.load_folder(folder)
    ro = oracle.adjust(od)
    res = fba.adjust(ds)
    assert res.iterations == ro.iterations
    err = group_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling)
    err.update({"e_" + g: v for g, v in
                elem_rel_err(res.xhat, ro.xhat, ro.names, ro.dist_scaling, floor=SMALL_SCENE_FLOOR).items()})
    spread = solver_spread(oracle, od, ro, floor=SMALL_SCENE_FLOOR)
    for g, e in err.items():  # 1e-9, or 20x the restatement's own rounding spread (high K_j are weak)
        assert e <= max(1e-9, 20 * spread[g]), (g, e, spread[g])
    assert res.sigma02 == pytest.approx(ro.sigma02, rel=max(1e-9, 20 * spread["sigma02"]))


def test_sync_and_polling_completion_agree(fba, cam0_folders, monkeypatch):
    """The two ways the host learns that a solve is done: the default polls the
    count of finished solves that k_sum_parts writes into host-mapped memory; FBA_SYNC=1 (read when a
    context is created) synchronises the stream instead.  Three iterations of each agree bit for bit."""
    ds = fba.load_folder(cam0_folders["stage3_pinhole"])
    monkeypatch.setenv("FBA_SYNC", "1")
    a = _ctx(fba, ds)
    monkeypatch.delenv("FBA_SYNC")
    b = _ctx(fba, ds)
    try:
        da = [a.step() for _ in range(3)]
        db = [b.step() for _ in range(3)]
        assert da == db and np.array_equal(a.get_xhat(), b.get_xhat())
    finally:
        a.close()
        b.close()


def test_async_solve_then_sync_solve_on_one_context(fba, cam0_folders):
    """fba_solve_update_async left outstanding, the next accumulation enqueued behind it, then a
    synchronous fba_solve_update on the same context: the synchronous call must wait for ITS solve (the
    count of solves enqueued on the context), not return when the outstanding one completes.  Its
    deltasum and xhat match a fresh context's second step; an async solve + fba_solve_finish matches the
    fresh context's first; a second solve of one accumulation is refused (it would factor the factor)."""
    ds = fba.load_folder(cam0_folders["stage3_pinhole"])
    a, b, fresh = _ctx(fba, ds), _ctx(fba, ds), _ctx(fba, ds)
    try:
        f1, f2 = fresh.step(), fresh.step()
        a.accumulate()
        a.solve_update_async()
        a.accumulate()
        d2 = a.solve_update()
        assert d2 == f2 and np.array_equal(a.get_xhat(), fresh.get_xhat())
        b.accumulate()
        b.solve_update_async()
        assert b.solve_finish() == f1
        with pytest.raises(fba.capi.FBAError) as ei:
            b.solve_update()
        assert ei.value.code == 1
    finally:
        a.close()
        b.close()
        fresh.close()


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


def test_graph_replay_matches_eager_launches(fba, cam0_folders):
    """The captured iteration graphs (default) and eager launches (timing events on) give bit-identical
    iterates: same kernels, same order, fixed-order reductions."""
    ds = fba.load_folder(cam0_folders["stage3_fisheye"])
    out = []
    for eager in (False, True):
        ctx = _ctx(fba, ds)
        ctx.set_timing(eager)
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
    d_first = None
    for it in range(3):
        d1 = single.step()
        d_first = d_first or d1
        for c in ranks:
            c.accumulate()
            c.synchronize()
        bufs = [c.reduce_buffer() for c in ranks]
        total = sum(hip.d2h(p, n) for p, n in bufs)
        for p, n in bufs:
            hip.h2d(p, total)
        parts = [c.solve_update() for c in ranks]
        # per-rank partial sums reorder the additions: deltasum sits at its rounding floor (~1e-8,
        # conftest.solver_spread), xhat stays within 1e-10
        assert abs(sum(parts) - d1) <= 1e-7 * d_first
    xs = single.get_xhat()
    xr = sum(c.get_xhat(owned_only=True) for c in ranks)
    names = fba.xhat_names(ds)
    _, _, _, dsc = single.build_awg(xs)
    err = group_rel_err(xr, xs, names, dsc)
    assert max(err.values()) <= 1e-10, err
    single.close()
    for c in ranks:
        c.close()


def test_sharded_step_over_rccl_and_device_views(fba, cam0_folders):
    """The torch plumbing of the multi-GPU path on ROCm: ShardedStep's all-reduce over RCCL
    (world 1, on the context's stream) reproduces fba_step bit for bit, and two rank contexts of a
    world-2 split, their compact reduce buffers summed through torch views of the device memory,
    reproduce it to rounding."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from fba_amd.parallel import ShardedStep, device_view
    ds = fba.load_folder(cam0_folders["stage3_pinhole"])
    dev = torch.device("cuda", 0)
    ref = _ctx(fba, ds)
    d_ref = [ref.step() for _ in range(3)]
    x_ref = ref.get_xhat()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        ctx = _ctx(fba, ds, stream=torch.cuda.current_stream(dev).cuda_stream)
        step = ShardedStep(ctx, device=dev)
        d = [step() for _ in range(3)]
        assert d == d_ref
        assert np.array_equal(ctx.get_xhat(), x_ref)
        ctx.close()
    finally:
        dist.destroy_process_group()
    ranks = [_ctx(fba, ds, rank=r, world=2) for r in range(2)]
    views = []
    n_dense = ref.reduce_buffer()[1]
    for c in ranks:
        p, n = c.reduce_buffer()
        assert n < n_dense  # compact buffer: co-visible blocks, camera rows, RHS row only
        views.append(device_view(p, n, dev))
    for it in range(3):
        for c in ranks:
            c.accumulate()
            c.synchronize()
        total = views[0] + views[1]
        for v in views:
            v.copy_(total)
        torch.cuda.synchronize(dev)
        parts = [c.solve_update() for c in ranks]
        assert abs(sum(parts) - d_ref[it]) <= 1e-7 * d_ref[0]
    xs = sum(c.get_xhat(owned_only=True) for c in ranks)
    _, _, _, dsc = ref.build_awg(x_ref)
    err = group_rel_err(xs, x_ref, fba.xhat_names(ds), dsc)
    assert max(err.values()) <= 1e-10, err
    for c in ranks:
        c.close()
    ref.close()


def _check_cov(res, od, ro, oracle, rtol=1e-8, atol_corr=5e-9):
    """diag(Cx) and the EOP/IOP correlation sub-blocks of fba_covariance against the oracle's dense
    bordered inverse of the last normal matrix (main.m:428-482, :602).  Bars from the round-6 measurements
    (profiles/r06_v8_covariance_errors.log): diag(Cx) <= 1.4e-9 relative, correlations <= 3.9e-10 absolute
    over the cam0 variants and the synthetic scenes -- held to 1e-8 and 5e-9."""
    cdo, corro = oracle.covariance(od, ro)
    print(f"covariance: diag(Cx) max relative error {np.max(np.abs(res.cx_diag - cdo) / np.abs(cdo)):.2e}")
    np.testing.assert_allclose(res.cx_diag, cdo, rtol=rtol, atol=0)
    u_img, u_cam = oracle.counts(od.settings)
    worst = 0.0
    for e in range(od.numImg):
        idx = list(range(e * u_img, (e + 1) * u_img))
        k = int(od.cam_num[np.nonzero(od.ext_index == e)[0][0]])
        idx += list(range(u_img * od.numImg + k * u_cam, u_img * od.numImg + (k + 1) * u_cam))
        worst = max(worst, float(np.max(np.abs(res.corr[e] - corro[np.ix_(idx, idx)]))))
        np.testing.assert_allclose(res.corr[e], corro[np.ix_(idx, idx)], rtol=0, atol=atol_corr)
    print(f"covariance: correlation blocks max absolute error {worst:.2e}")


@pytest.mark.parametrize("variant", ["stage3_pinhole", "stage1_pinhole", "stage3_noic_pinhole", "stage3_sigy_pinhole"])
def test_covariance_cam0(fba, oracle, cam0_folders, variant):
    """Post-fit covariance on cam0: selected inverse of the block Cholesky factor + the border's
    low-rank correction + the tie-point Schur identity, against the reference's explicit inverse."""
    ds = fba.load_folder(cam0_folders[variant])
    od = oracle.load_folder(cam0_folders[variant])
    ro = oracle.adjust(od)
    res = fba.adjust(ds)
    _check_cov(res, od, ro, oracle)


@pytest.mark.parametrize("n_control", [0, 12])
def test_covariance_synthetic(fba, oracle, tmp_path, n_control):
    """Free-network fish-eye scene (inner constraints) and a scene whose datum comes from control
    points (no inner constraints): every estimated unknown's variance, tie points included."""
    from fba_amd import synth
    sc = synth.generate(14, 260, seed=23, typ="fisheye", n_control=n_control)
    folder = synth.write_folder(sc, str(tmp_path / f"c{n_control}"))
    ds = fba.load_folder(folder)
    od = oracle.load_folder(folder)
    ro = oracle.adjust(od)
    res = fba.adjust(ds)
    _check_cov(res, od, ro, oracle)


def test_batch_main_writes_reference_outputs(fba, oracle, tmp_path):
    """BatchRun.m -> main(folder) on the device path: .out / .par / .rsd written next to the data, the
    standard deviations in the .out being sqrt of the device Cx diagonal."""
    import os
    import shutil
    from conftest import CAM0
    from fba_amd import batch
    folder = tmp_path / "proj" / "cam0"
    shutil.copytree(CAM0, folder)
    done = batch.batch_run([str(tmp_path / "proj")])
    assert done == [(str(folder), 0)]
    for ext in (".out", ".par", ".rsd"):
        assert os.path.getsize(folder / ("cam0" + ext)) > 0
    lines = (folder / "cam0.out").read_text().splitlines()
    dof = next(x for x in lines if x.startswith("Total Degrees of Freedom"))
    assert dof.split()[-1] == "1485"
    od = oracle.load_folder(str(folder))
    ro = oracle.adjust(od)
    cdo, _ = oracle.covariance(od, ro)
    xc = next(x for x in lines if x.startswith("Xc "))
    assert float(xc.split()[2]) == pytest.approx(np.sqrt(cdo[0]), abs=2e-5)


def _border_gram(rng, n=200):
    """A 15 x n stand-in for the forward-solved rows [y | A (7) | B (7)] and its Gram matrix."""
    R = rng.standard_normal((15, n))
    return R @ R.T


def test_border_solve_matches_dense(fba):
    """k_border_combine's in-register 14x14 solve (partial pivoting by wave shuffles) against a dense
    solve of [[A'A - I, A'B], [B'A, B'B]] [z; k] = -[A'y; B'y] (the inner-constraint combine)."""
    rng = np.random.default_rng(7)
    for _ in range(3):
        g = _border_gram(rng)
        H = g[1:, 1:].copy()
        H[np.arange(7), np.arange(7)] -= 1.0
        ref = np.linalg.solve(H, -g[1:, 0])
        coef = np.zeros(14)
        fba.capi.check(fba.capi.lib.fba_test_border_solve(0, fba.capi.ptr(np.ascontiguousarray(g)),
                                                          fba.capi.ptr(coef)))
        np.testing.assert_allclose(coef, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())


def test_border_solve_nan_column_stays_local(fba):
    """A NaN pivot column must not pull an already-finished row back into the elimination (the pivot
    search keeps row `col` when no candidate compares): the solve returns without a hang and the NaN
    shows up in the output rather than as silently wrong finite coefficients."""
    rng = np.random.default_rng(8)
    g = _border_gram(rng)
    g[5, 5:] = np.nan
    g[5:, 5] = np.nan
    coef = np.zeros(14)
    fba.capi.check(fba.capi.lib.fba_test_border_solve(0, fba.capi.ptr(np.ascontiguousarray(g)), fba.capi.ptr(coef)))
    assert not np.isfinite(coef).all()


def test_buildrsd_matches_oracle(fba, oracle, cam0_folders):
    """fba.BuildRSD(v, data, xhat) (BuildRSD.m:1, fba_build_rsd on the device) for a given v."""
    for variant in ("stage3_pinhole", "stage1_pinhole"):
        ds = fba.load_folder(cam0_folders[variant])
        od = oracle.load_folder(cam0_folders[variant])
        ro = oracle.adjust(od)
        rows = fba.BuildRSD(ro.v, ds, ro.xhat)
        assert [r[0] for r in rows] == od.target and [r[1] for r in rows] == od.image
        num = np.array([r[4:] for r in rows], dtype=np.float64)
        ref = oracle.build_rsd(od, ro.v, ro.xhat)
        assert np.abs(num - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("t", range(5))
def test_buildawg_matches_reference_text(fba, t):
    """The device BuildAwG (fba_build_awg) against the reference's own BuildAwG.m text evaluated at
    40 digits (tests/golden/jac_golden.json "distortion": generated EOP / tie / c partials and the
    hand-written distortion model, xp / yp partials, scaled K / P columns, dist_scaling and G at
    nonzero distortion), one image and one camera per sample point: <= 1e-12 relative per entry."""
    import json
    import os
    from conftest import GOLDEN
    from test_oracle import EOP_NAMES, TIE_NAMES
    with open(os.path.join(GOLDEN, "jac_golden.json")) as fh:
        g = json.load(fh)["distortion"]
    typ = ["fisheye", "pinhole", "equisolid", "orthographic", "stereographic"][t]
    nk, pts = g["nk"], g["points"]
    n, cw = len(pts), 5 + g["nk"]
    eop = np.array([[p["Xc"], p["Yc"], p["Zc"], p["w"], p["p"], p["k"]] for p in pts])
    iop = np.array([[p["xp"], p["yp"], p["c"], *p["K"], *p["P"]] for p in pts])
    xyz = np.array([[p["X"], p["Y"], p["Z"]] for p in pts])
    cam_info = np.array([[p["y_dir"], p["xmin"], p["ymin"], p["xmax"], p["ymax"]] for p in pts])
    xy = np.array([[p["x"], p["y"]] for p in pts])
    idx = np.arange(n)
    packed = fba.capi.PackedProblem(xy, idx, idx, idx, xyz, eop, iop, cam_info, xyz, n, n, n)
    s = {"type": typ, "Num_Radial_Distortions": nk, "Inner_Constraints": 1, "Iteration_Cap": 1, "threshold": 1e-6,
         "Meas_std": 1.0, "Meas_std_y": 1.0}
    for k in ("Xc", "Yc", "Zc", "w", "p", "k", "c", "xp", "yp", "radial", "decent"):
        s["Estimate_" + k] = 1
    ctx = fba.capi.Context(packed, fba.capi.make_settings(s))
    try:
        xhat = np.concatenate([eop.reshape(-1), iop.reshape(-1), xyz.reshape(-1)])
        A, w, G, ds = ctx.build_awg(xhat)
    finally:
        ctx.close()

    def close(a, b, what):
        assert abs(a - b) <= 1e-12 * max(abs(b), 1e-300), (typ, what, a, b)
    for i, v in enumerate(g["values"][typ]):
        rx, ry, base, tb = 2 * i, 2 * i + 1, 6 * n + cw * i, 6 * n + cw * n + 3 * i
        close(w[rx] + xy[i, 0], v["fx"], (i, "fx"))
        close(w[ry] + xy[i, 1], v["fy"], (i, "fy"))
        for nm, (r, col) in EOP_NAMES.items():
            close(A[2 * i + r, 6 * i + col], v[nm], (i, nm))
        for nm, (r, col) in TIE_NAMES.items():
            close(A[2 * i + r, tb + col], v[nm], (i, nm))
        for q, par in enumerate(("A_xp", "A_yp")):
            close(A[rx, base + q], v[par][0], (i, par))
            close(A[ry, base + q], v[par][1], (i, par))
        close(A[rx, base + 2], v["Ax_c"], (i, "Ax_c"))
        close(A[ry, base + 2], v["Ay_c"], (i, "Ay_c"))
        for j in range(nk):
            close(A[rx, base + 3 + j], v["Ax_K"][j], (i, "Ax_K", j))
            close(A[ry, base + 3 + j], v["Ay_K"][j], (i, "Ay_K", j))
            close(ds[i, 2 + j], v["scale"][j], (i, "dist_scaling", j))
        for j in range(2):
            close(A[rx, base + 3 + nk + j], v["Ax_P"][j], (i, "Ax_P", j))
            close(A[ry, base + 3 + nk + j], v["Ay_P"][j], (i, "Ay_P", j))
        gv = np.array(v["G"])
        assert np.abs(G[6 * i:6 * i + 6] - gv).max() <= 1e-14 * np.abs(gv).max(), (typ, i, "G")
