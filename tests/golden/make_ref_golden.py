"""Write tests/golden/ref_cam0_<variant>.npz: the reference's OWN .m text run on cam0.

Run in the build container (the only place /root/reference exists):
    python tests/golden/make_ref_golden.py [/root/reference]

tests/golden/mlang.py executes the statements of main.m that start on lines 61-628 -- ReadFiles of the
folder's .pho/.ext/.cnt/.int/.cfg (and .tie), the findSetting calls, the string-to-cell conversions,
the data.points join loop (:280-384), Buildxhat (:388), the weight matrix (:396-405), the whole
Gauss-Newton loop with BuildAwG, A'*P*w, A'*P*A, the bordered explicit inverse, the correlation
matrix, the distortion de-scaling and sumabs (:407-494), v = A*delta + w, BuildRSD, RMS and sigma0^2
(:567-602) -- with the variables main.m:1-60 would have set in a non-batch, no-plot run (batch = 0,
enable_plots = false; the version/date strings only feed the .out header).  The files it calls are
interpreted from their text too: functions/ReadFiles.m, findSetting.m, Buildxhat.m, BuildAwG.m,
BuildRSD.m, sumabs.m.  MATLAB built-ins (readmatrix, inv, mtimes, ...) are restated in mlang.py.

Also (`make_ref_golden.py /root/reference synth_fe`): the same run on conftest.SYNTH_FE, a synthetic
equidistant fish-eye free network (12 images x 300 tie points, inner constraints, no control, all EOP +
IOP + 5 radial + 2 decentering) -> ref_synth_fisheye_free.npz; and (`nostd`) cam0 without its Meas_std
line -> ref_cam0_nostd.json (the reference stops in rmfield at main.m:399).

Only numbers are stored: per-iteration xhat and deltasum, the iteration count, sigma0^2, RMSx / RMSy
/ RMS, v, the numeric RSD columns, dist_scaling, A / w / G of the first BuildAwG call, diag(Cx) after
the de-scaling and the sigma0^2 scaling (main.m:460-482, :602) and the Correlation sub-blocks the
.out writer reads (each image's EOPs with its camera's IOPs, main.m:845-863).
"""
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

import mlang  # noqa: E402
from conftest import CAM0_VARIANTS, synth_fe_folder, variant_folder  # noqa: E402

MAIN_FIRST, MAIN_LAST = 61, 628
FUNCS = ["ReadFiles", "findSetting", "Buildxhat", "BuildAwG", "BuildRSD", "sumabs"]


def run_reference(ref_root, folder, verbose=False):
    it = mlang.Interp(verbose=verbose)
    for f in FUNCS:
        it.load_file(os.path.join(ref_root, "functions", f + ".m"))
    init = {"batch": 0.0, "enable_plots": False, "folder": "", "projectDir": folder, "version": "x",
            "mfiles": "", "date": "", "main_error": 0.0}
    it.load_file(os.path.join(ref_root, "main.m"), main_slice=("main", MAIN_FIRST, MAIN_LAST, list(init)))
    first = {}

    def hook(args, out):
        if not first:
            first["awg"] = out
    it.hooks["BuildAwG"] = hook
    it.cwd = folder
    env = it.run_slice("main", init)
    return env, first["awg"]


def extract(env, awg):
    num = lambda x: np.asarray(x, dtype=np.float64)  # noqa: E731
    data = env["data"]
    st = data.elems[0]["settings"].elems[0]
    u_img = int(sum(st[k] for k in ("Estimate_Xc", "Estimate_Yc", "Estimate_Zc", "Estimate_w", "Estimate_p",
                                    "Estimate_k")))
    nk = int(max(st["Num_Radial_Distortions"], 1))
    u_cam = int(st["Estimate_c"] + st["Estimate_xp"] + st["Estimate_yp"] + st["Estimate_radial"] * nk
                + st["Estimate_decent"] * 2)
    pts = data.elems[0]["points"].elems
    n_img = int(data.elems[0]["numImg"])
    xhat_arr = num(env["xhat_arr"])
    def name_of(x):  # a tie name is a cell inside the cell when TIE is a cell array (Buildxhat.m:111, :132)
        while isinstance(x, mlang.MCell) and x.a.size == 1:
            x = x.a.flat[0]
        return mlang.text_of(x)
    names = [name_of(x) for x in env["xhatnames"].a.reshape(-1, order="F")]
    _, A0, w0, G0, ds0 = awg
    A0 = num(A0)
    rows, cols = np.nonzero(A0)
    Cx = num(env["Cx"])
    corr = num(env["Correlation"])
    blocks = []
    for e in range(n_img):
        idx = list(range(e * u_img, (e + 1) * u_img))
        cam = int(next(p["cam_num"] for p in pts if int(p["ext_index"]) == e + 1)) - 1
        idx += list(range(u_img * n_img + cam * u_cam, u_img * n_img + (cam + 1) * u_cam))
        blocks.append(corr[np.ix_(idx, idx)])
    rsd = env["RSD"].a
    return dict(
        iterations=int(env["count"]), deltasum=num(env["deltasumarr"]).reshape(-1), xhat_hist=xhat_arr,
        xhat=num(env["xhat"]).reshape(-1), names=np.array(names), sigma02=float(env["sigma02"]),
        rms=np.array([env["RMSx"], env["RMSy"], env["RMS"]], dtype=np.float64), v=num(env["v"]).reshape(-1),
        rsd=np.array([[float(rsd[i, j]) for j in range(4, 9)] for i in range(rsd.shape[0])]),
        dist_scaling=num(env["dist_scaling"]).reshape(-1, 2 + nk),
        A0_rows=rows.astype(np.int32), A0_cols=cols.astype(np.int32), A0_vals=A0[rows, cols],
        A0_shape=np.array(A0.shape), w0=num(w0).reshape(-1),
        G0=num(G0) if isinstance(G0, np.ndarray) else np.zeros((0, 7)),
        cx_diag=np.diag(Cx).copy(), corr_blocks=np.array(blocks),
        dof=float(data.elems[0]["n"] - len(names)))


def run_nostd(ref_root, root):
    """cam0 with no Meas_std line in its .cfg: what the reference text does (main.m:123-127 sets
    Meas_std = 1 and no_std_y = 1, then main.m:397-399 calls rmfield on the absent Meas_std_y).  Writes
    ref_cam0_nostd.json: the interpreter's error and the main.m line it was raised at."""
    import json
    folder = variant_folder(root, "nostd", {"Meas_std": None, "Meas_std_y": None})
    try:
        run_reference(ref_root, folder)
        out = {"error": None}
    except mlang.MatlabError as e:
        out = {"error": str(e)}
    out["cfg_edit"] = "cam0 config.cfg without its Meas_std (and Meas_std_y) line"
    with open(os.path.join(HERE, "ref_cam0_nostd.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("nostd:", out["error"], flush=True)


def run_synth(ref_root, root):
    """conftest.SYNTH_FE (12 images x 300 tie points, equidistant fish-eye, inner constraints, no control)
    -> ref_synth_fisheye_free.npz, with the sha256 of the scene's files (the tests regenerate the scene
    and check that hash before comparing)"""
    folder, digest = synth_fe_folder(root)
    t0 = time.time()
    env, awg = run_reference(ref_root, folder)
    out = extract(env, awg)
    out["files_sha256"] = np.array(digest)
    np.savez_compressed(os.path.join(HERE, "ref_synth_fisheye_free.npz"), **out)
    print(f"synth_fe: {out['iterations']} iterations, sigma0^2 {out['sigma02']!r}, "
          f"deltasum {out['deltasum'][-1]:.3e}, {time.time() - t0:.1f} s", flush=True)


def main(ref_root):
    root = tempfile.mkdtemp()
    only = sys.argv[2:] or sorted(CAM0_VARIANTS) + ["nostd", "synth_fe"]
    if "nostd" in only:
        run_nostd(ref_root, root)
        only = [n for n in only if n != "nostd"]
    if "synth_fe" in only:
        run_synth(ref_root, root)
        only = [n for n in only if n != "synth_fe"]
    for name in only:
        folder = variant_folder(root, name, CAM0_VARIANTS[name])
        t0 = time.time()
        env, awg = run_reference(ref_root, folder)
        out = extract(env, awg)
        np.savez_compressed(os.path.join(HERE, f"ref_cam0_{name}.npz"), **out)
        print(f"{name}: {out['iterations']} iterations, sigma0^2 {out['sigma02']!r}, "
              f"deltasum {out['deltasum'][-1]:.3e}, {time.time() - t0:.1f} s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
