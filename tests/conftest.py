import os
import shutil
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
CAM0 = os.path.join(GOLDEN, "cam0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def fba():
    import fba_import
    return fba_import.load()


@pytest.fixture(scope="session")
def oracle():
    import fba_oracle
    return fba_oracle


def variant_folder(tmp_root, name, cfg_edits, src=CAM0):
    """Copy cam0 with edited .cfg keys (value strings as in the .cfg; None removes the key's line)."""
    dst = os.path.join(tmp_root, name)
    os.makedirs(dst, exist_ok=True)
    for f in os.listdir(src):
        if not f.endswith(".cfg"):
            shutil.copy(os.path.join(src, f), dst)
    lines = open(os.path.join(src, "config.cfg")).read().splitlines()
    out, seen = [], set()
    for ln in lines:
        toks = ln.split("#", 1)[0].split()
        if toks and toks[0] in cfg_edits:
            if cfg_edits[toks[0]] is not None:
                out.append(f"{toks[0]}\t{cfg_edits[toks[0]]}")
            seen.add(toks[0])
        else:
            out.append(ln)
    for k, v in cfg_edits.items():
        if k not in seen and v is not None:
            out.append(f"{k}\t{v}")
    with open(os.path.join(dst, "config.cfg"), "w") as fh:
        fh.write("\n".join(out) + "\n")
    return dst


STAGE1 = {"Inner_Constraints": "0", "Estimate_xp": "0", "Estimate_yp": "0", "Estimate_c": "0",
          "Estimate_Radial_Distortions": "0", "Estimate_Decentering_Distortions": "0", "Estimate_tie": "0"}

CAM0_VARIANTS = {
    "stage3_pinhole": {},
    "stage3_fisheye": {"Type": "'fisheye'"},
    "stage1_pinhole": STAGE1,
    "stage3_equisolid": {"Type": "'equisolid'"},
    "stage3_orthographic": {"Type": "'orthographic'"},
    "stage3_stereographic": {"Type": "'stereographic'"},
    "stage3_noic_pinhole": {"Inner_Constraints": "0"},
    "stage3_sigy_pinhole": {"Meas_std_y": "0.4"},
}


# SURVEY section 8(c) golden 3: a small synthetic fish-eye free network -- the north-star model
# (equidistant, BuildAwG.m:186-187) with inner constraints and no control (BuildAwG.m:514-527), all EOP +
# IOP + 5 radial + 2 decentering unknowns, at a well-conditioned point (two exact restatements of the
# reference agree to <= 2.3e-12 of every parameter group's scale, solver_spread).  The reference's own
# text run on it: tests/golden/ref_synth_fisheye_free.npz (tests/golden/make_ref_golden.py synth_fe).
SYNTH_FE = {"n_img": 12, "n_tie": 300, "seed": 34, "obs_per_point": 8}


def synth_fe_folder(root):
    """the scene's folder (deterministic: synth.generate with SYNTH_FE, .17g text) and a hash of its files"""
    import hashlib
    import fba_import
    fba_import.load()
    from fba_amd import synth
    p = dict(SYNTH_FE)
    sc = synth.generate(p.pop("n_img"), p.pop("n_tie"), **p)
    folder = synth.write_folder(sc, os.path.join(root, "synth_fe"))
    h = hashlib.sha256()
    for f in sorted(os.listdir(folder)):
        with open(os.path.join(folder, f), "rb") as fh:
            h.update(f.encode() + fh.read())
    return folder, h.hexdigest()


@pytest.fixture(scope="session")
def synth_fe(tmp_path_factory):
    return synth_fe_folder(str(tmp_path_factory.mktemp("synth_fe")))


@pytest.fixture(scope="session")
def cam0_folders(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("cam0v"))
    return {k: variant_folder(root, k, v) for k, v in CAM0_VARIANTS.items()}


def param_groups(names):
    """Group unknown names (Buildxhat.m naming) for normwise-per-group relative errors."""
    groups = {}
    for i, nm in enumerate(names):
        key = nm.split("_", 1)[0]
        if key in ("Xc", "Yc", "Zc"):
            key = "XYZc"
        elif key in ("w", "p", "k"):
            key = "wpk"
        elif key in ("X", "Y", "Z"):
            key = "XYZ"
        groups.setdefault(key, []).append(i)
    return {k: np.array(v) for k, v in groups.items()}


CAMERA_HEADS = ("xp", "yp", "c")


def distortion_scale(names, dist_scaling):
    """Multiply K_j by rmax^(2j) and P by rmax^2 (the reference's own scaling, BuildAwG.m:422-443),
    with each camera's own rmax: row k of dist_scaling is camera k in INT order, the order Buildxhat.m
    lays the cameras out in (Buildxhat.m:65-105; names xp_<cam>, k1_<cam>, ...)."""
    sc = np.ones(len(names))
    cams = {}
    for i, nm in enumerate(names):
        head, _, cid = nm.partition("_")
        dist = head[0] in "kp" and head[1:].isdigit()
        if not (dist or head in CAMERA_HEADS):
            continue
        k = cams.setdefault(cid, len(cams))
        if head[0] == "k" and head[1:].isdigit():
            sc[i] = dist_scaling[k, 1 + int(head[1:])]
        elif head[0] == "p" and head[1:].isdigit():
            sc[i] = dist_scaling[k, 2]
    return sc


def dist_scaling_of(od):
    """The rmax^(2j) columns of dist_scaling (BuildAwG.m:424-426) from the INT bounds, without
    forming the dense A of a large scene (what distortion_scale reads)."""
    nk = max(od.settings["Num_Radial_Distortions"], 1)
    out = np.zeros((od.numCam, 2 + nk))
    for k in range(od.numCam):
        b = od.bounds[np.nonzero(od.cam_num == k)[0][0]]
        rmax = np.sqrt(((b[3] - b[1]) * 0.5) ** 2 + ((b[4] - b[2]) * 0.5) ** 2)
        out[k, 2:] = rmax ** (2 * np.arange(1, nk + 1))
    return out


def group_rel_err(a, b, names, dist_scaling=None):
    """max over parameter groups of max|a-b| / max|b| (distortion terms in the scaled units)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if dist_scaling is not None:
        sc = distortion_scale(names, dist_scaling)
        a, b = a * sc, b * sc
    worst = {}
    for g, idx in param_groups(names).items():
        den = max(np.max(np.abs(b[idx])), 1e-300)
        worst[g] = float(np.max(np.abs(a[idx] - b[idx])) / den)
    return worst


ELEM_FLOOR = 1e-6
# The small synthetic free networks (12-18 images, a few hundred tie points) are ill-conditioned enough
# that two exact restatements of the reference -- the dense explicit inverse (oracle/fba_oracle.py) and
# the block-sparse direct KKT solve (oracle/fba_cpu.c) -- differ by up to 5.3e-11 of a parameter group's
# scale (12 images x 240 points, seed 17; per Type, fisheye / pinhole / equisolid / orthographic /
# stereographic: 1.9e-11 / 7.6e-12 / 2.2e-12 / 4.9e-11 / 5.3e-11).  A coordinate near the datum's origin
# (0.4 mm in a 3.5 m scene) then differs by 3e-8 relative between them although both are exact: a
# coordinate's own magnitude is where the datum puts the origin, not a property of the adjustment.  On
# these scenes entries below 10% of their group's scale are held to 1e-10 of that scale (1e-9 x 0.1),
# the others to 1e-9 of themselves (measured worst: 4.6e-10, orthographic).
SMALL_SCENE_FLOOR = 0.1


def elem_rel_err(a, b, names, dist_scaling=None, floor=ELEM_FLOOR):
    """Per-element relative error, the SURVEY section 8(c) bar: per parameter group, max over its entries
    of |a_i - b_i| / max(|b_i|, floor * max_g |b|) (distortion terms in the reference's scaled units,
    BuildAwG.m:422-443).  The floor only touches entries smaller than `floor` (1e-6) of their group's
    largest value -- a coordinate or angle that happens to sit at the datum's zero; the synthetic and cam0
    scenes have none (config 3's smallest |x| / max is 3e-5), and there two exact restatements
    of the reference (oracle/fba_cpu.c's KKT and Cholesky solvers, or one of them on 3 vs 16 threads)
    agree per element to 1.2e-12 (tests/test_oracle_cpu.py)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if dist_scaling is not None:
        sc = distortion_scale(names, dist_scaling)
        a, b = a * sc, b * sc
    worst = {}
    for g, idx in param_groups(names).items():
        den = np.maximum(np.abs(b[idx]), max(floor * np.max(np.abs(b[idx])), 1e-300))
        worst[g] = float(np.max(np.abs(a[idx] - b[idx]) / den))
    return worst


def solver_spread(oracle, od, ro, perturb=1e-14, floor=ELEM_FLOOR):
    """How far exact restatements of the reference land from each other, per parameter group and for
    sigma0^2 and the first deltasum ("e_<group>": per element, elem_rel_err with `floor`).  Three variants of the oracle run:
      * LU of the bordered system instead of its explicit inverse (main.m:432);
      * the loop started from an xhat perturbed by `perturb` relative (the inner-constraint datum is
        re-derived from every iterate, BuildAwG.m:516-523, so the limit depends on the path);
      * the misclosure w perturbed by one ulp of f (any implementation of the forward model --
        the reference's generated expressions included -- rounds f differently).
    On the path-sensitive cam0 variants (inner constraints + control points + a non-pinhole model)
    the high-order distortion terms move by up to ~1e-4; no implementation can be closer."""
    def solve_lu(data, A, w, G, P):
        u = A.T @ (P * w)
        N = A.T @ (P[:, None] * A)
        if G is None:
            return np.linalg.solve(N, -u)
        NG = np.block([[N, G], [G.T, np.zeros((7, 7))]])
        return np.linalg.solve(NG, np.concatenate([-u, np.zeros(7)]))[: len(u)]
    runs = [oracle.adjust(od, solver=solve_lu)]
    x0, names = oracle.buildxhat(od)
    rng = np.random.default_rng(0)
    orig_x, orig_awg = oracle.buildxhat, oracle.build_awg
    try:
        oracle.buildxhat = lambda d: (x0 * (1 + perturb * rng.standard_normal(len(x0))), names)
        runs.append(oracle.adjust(od))
        oracle.buildxhat = orig_x

        def awg_ulp(d, x):
            A, w, G, ds = orig_awg(d, x)
            f = w + np.column_stack([d.x, d.y]).reshape(-1)
            return A, w + np.spacing(np.abs(f)) * rng.choice([-1.0, 1.0], size=len(w)), G, ds
        oracle.build_awg = awg_ulp
        runs.append(oracle.adjust(od))
    finally:
        oracle.buildxhat, oracle.build_awg = orig_x, orig_awg
    out = {}
    for r in runs:
        e = group_rel_err(r.xhat, ro.xhat, ro.names, ro.dist_scaling)
        e.update({"e_" + g: v for g, v in elem_rel_err(r.xhat, ro.xhat, ro.names, ro.dist_scaling, floor).items()})
        e["sigma02"] = abs(r.sigma02 - ro.sigma02) / ro.sigma02
        e["deltasum0"] = abs(r.deltasum[0] - ro.deltasum[0]) / ro.deltasum[0]
        for k, v in e.items():
            out[k] = max(out.get(k, 0.0), v)
    return out
