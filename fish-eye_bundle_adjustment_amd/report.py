"""Report writers of the reference: the .out summary, the .par camera file and the .rsd residual table.

Restates main.m:631-958 (with functions/printCell.m and main.m's printEOP / printDist / printTIE /
countImagePoints / countTargetImages helpers) so the files a reference user reads come out in the same
layout, from the device results (``bundle.Adjustment``: xhat, the diagonal of the final Cx and the
EOP/IOP correlation sub-blocks from ``fba_covariance``, the residuals of ``fba_residuals``).  Reference
quirks kept on purpose: the "Version:" heading runs into the title line, names
in the EOP/IOP tables are cut to 5 characters (``%-W.5s``), the mean-correlation labels shift by one
after the EOP names (an empty name sits between the EOP and IOP name lists, main.m:847), and
``img_width`` takes the last image ID longer than the longest target ID (main.m:697-703).
Host-side text formatting only; nothing here computes on the device path.
"""
import datetime
import math

import numpy as np

LINE = "*" * 109  # main.m:635
DECIMALS = 5      # main.m:686
PADDING = 4       # main.m:634
VERSION = "fba_amd 1 (MI355X HIP path)"
PRODUCER = "fba_amd, the MI355X-native HIP implementation (not the MATLAB reference)"


def num2str(x, prec=None):
    """MATLAB num2str for a real scalar (or a char array passed through)."""
    if isinstance(x, str):
        return x
    x = float(x)
    if prec is not None:
        return _g(x, prec)
    if math.isfinite(x) and x == int(x) and abs(x) < 1e15:
        return str(int(x))
    if not math.isfinite(x):
        return "NaN" if math.isnan(x) else ("Inf" if x > 0 else "-Inf")
    digits = max(int(math.floor(math.log10(abs(x)))) + 5, 5) if x != 0 else 5
    return _g(x, min(digits, 16))


def _g(x, prec):
    s = f"{x:.{prec}g}"
    return s


def print_cell(fh, rows, prefix="", padding=PADDING):
    """functions/printCell.m: 'name ..... value' rows; '\\line' rows print dashes, '\\n' rows a blank."""
    width = max((len(r[0]) for r in rows), default=0)
    for name, val in rows:
        if name == "\\line":
            fh.write("-" * (width + padding + 6))
        elif name == "\\n":
            pass
        else:
            fh.write(prefix + name + " " + "." * (width + padding - len(name)) + " " + num2str(val))
        fh.write("\n")
    return width + padding + 3


def _settings_rows(s):
    """fieldnames(data.settings) in the order main.m:116-171 assigns them (Meas_std_y removed when it
    was not given, main.m:399)."""
    keys = ["Output_Filename", "Meas_std"]
    if not s.get("no_std_y", 0):
        keys.append("Meas_std_y")
    keys += ["no_std_y", "type", "Check_Points", "Iteration_Cap", "threshold", "Inner_Constraints", "Estimate_Xc",
             "Estimate_Yc", "Estimate_Zc", "Estimate_w", "Estimate_p", "Estimate_k", "Estimate_c", "Estimate_xp",
             "Estimate_yp", "Estimate_radial", "Num_Radial_Distortions", "Estimate_decent", "Estimate_tie",
             "Estimate_AllGCP"]
    return [(k, s.get(k, 0)) for k in keys]


def _line_eop(name, value, std, w):
    """printEOP: '%-W.5s%-W.5f%-W.5f'."""
    return f"{name[:DECIMALS]:<{w}}{value:<{w}.{DECIMALS}f}{std:<{w}.{DECIMALS}f}\n"


def _line_dist(name, value, std, w):
    """printDist: '%-W.5s%-W.5e%-W.5e'."""
    return f"{name[:DECIMALS]:<{w}}{value:<{w}.{DECIMALS}e}{std:<{w}.{DECIMALS}e}\n"


def _corr_rows(fh, names, mat):
    """'%-6.2s' name header, then the lower triangle '%-+6.2f' (main.m:802-815)."""
    for nm in names:
        fh.write(f"{nm[:2]:<6}")
    fh.write("\n")
    for j in range(mat.shape[0]):
        lab = names[j + 1] if j + 1 < len(names) else ""
        fh.write(f"{lab[:2]:<6}")
        for k in range(j + 1):
            fh.write(f"{mat[j, k]:<+6.2f}")
        fh.write("\n")


def write_out(path, data, res, seconds, version=VERSION, date=None):
    """main.m:631-950: the .out report."""
    s = data.settings
    u_img = sum(int(s[k]) for k in ("Estimate_Xc", "Estimate_Yc", "Estimate_Zc", "Estimate_w", "Estimate_p",
                                     "Estimate_k"))
    nK = int(s["Num_Radial_Distortions"])
    u_cam = int(s["Estimate_c"]) + int(s["Estimate_xp"]) + int(s["Estimate_yp"]) + int(s["Estimate_radial"]) * nK + \
        2 * int(s["Estimate_decent"])
    ic = int(s["Inner_Constraints"])
    xhat, cxd = res.xhat, res.cx_diag
    std = np.sqrt(np.maximum(cxd, 0.0)) if cxd is not None else np.full(len(xhat), np.nan)
    date = date or datetime.date.today().strftime("%d-%b-%Y")
    n = data.n
    with open(path, "w") as fh:
        fh.write("Version: " + version)
        # main.m:637's title and author line, with this build named as the producer of the numbers below
        # (the model and the report layout are the reference's; the line count is unchanged)
        fh.write("Fish-eye model Bundle Adjustment\nResults produced by " + PRODUCER + "; model and report format: "
                 "Wynand Tredoux -- University of Calgary -- 2020\n\n")
        fh.write(LINE)
        fh.write(f"\n\nExecution date:\t{date}\nTime Taken:\t\t{num2str(seconds)} seconds\nIterations:\t\t"
                 f"{res.iterations}\nModel Used:\t\t{s['type']}")
        fh.write("\n\nSettings used:\n")
        print_cell(fh, _settings_rows(s), "\t\t")
        fh.write("\n" + LINE + "\n")
        fh.write("\nObservations/Unknowns Summary\n\n")
        rows = [("Number of Photos", num2str(data.numImg)),
                ("Total EOP unknowns", num2str(u_img * data.numImg)),
                ("Number of Cameras", num2str(data.numCam)),
                ("Total IOP unknowns", num2str((int(s["Estimate_c"]) + int(s["Estimate_xp"]) + int(s["Estimate_yp"]))
                                               * data.numCam)),
                ("Total distortion unknowns", num2str((int(s["Estimate_radial"]) * nK + int(s["Estimate_decent"]) * 2)
                                                      * data.numCam)),
                ("Number of tie/control points", num2str(data.numGCP)),
                ("Number of tie/control points to be estimated", num2str(data.numtie)),
                ("Number of control/tie point unknowns", num2str(data.numtie * 3)),
                ("\\line", ""),
                ("Total Unknowns", num2str(len(xhat))),
                ("\\n", ""),
                ("Number of image points", num2str(n // 2)),
                ("Total number of observations", num2str(n)),
                ("Number of Inner Constraints", num2str(7 * ic)),
                ("\\line", ""),
                ("Total Number of Observations", num2str(n + 7 * ic)),
                ("\\n", ""),
                ("Total Degrees of Freedom", num2str(n + 7 * ic - len(xhat))),
                ("\\n", ""),
                ("A-Posteriori", num2str(res.sigma02, 10)),
                ("RMSx", num2str(res.rms[0], 10)),
                ("RMSy", num2str(res.rms[1], 10)),
                ("RMS", num2str(res.rms[2], 10)),
                ("\\n", "")]
        print_cell(fh, rows, "")
        fh.write(LINE + "\n\n")

        # column width (main.m:687-706)
        tw = max((len(t) for t in sorted(set(data.pho_target))), default=0)
        iw = 0
        for t in sorted(set(data.pho_image)):
            if len(t) > tw:
                iw = len(t)
        w = max(tw, iw, 12) + 2

        # Estimated EOPs (main.m:709-770)
        fh.write("Estimated EOPs\nEOP Name\tValue\tStandard Deviation\n")
        img_count = {}
        for im in data.pho_image:
            img_count[im] = img_count.get(im, 0) + 1
        eop_names = [nm for nm, k in zip(("Xc", "Yc", "Zc", "Omega", "Phi", "Kappa"),
                                          ("Estimate_Xc", "Estimate_Yc", "Estimate_Zc", "Estimate_w", "Estimate_p",
                                           "Estimate_k")) if s[k]]
        q = 0
        eop_idx = []
        for i in range(data.numImg):
            r = data.EXT[i]
            fh.write("\n")
            print_cell(fh, [("Image", r[0]), ("Camera", r[1]), ("Number of image points", num2str(img_count.get(r[0], 0))),
                            ("\\line", "")], "")
            idx = []
            for nm in eop_names:
                f = 180.0 / math.pi if nm in ("Omega", "Phi", "Kappa") else 1.0
                fh.write(_line_eop(nm, xhat[q] * f, std[q] * f, w))
                idx.append(q)
                q += 1
            eop_idx.append(idx)

        # IOPs and distortions per camera (main.m:773-840)
        fh.write("\n" + LINE + "\n\nEstimated IOPs and Distortions for each Camera\nIOP Name\tValue\tStandard Deviation\n\n")
        par = [["Created with Fish-eye model Bundle Adjustment version:", version, None], ["Execution date", date, None],
               [None, None, None]]
        iop_names = ([nm for nm, k in (("xp", "Estimate_xp"), ("yp", "Estimate_yp"), ("c", "Estimate_c")) if s[k]]
                     + ([f"k{j + 1}" for j in range(nK)] if s["Estimate_radial"] else [])
                     + (["p1", "p2"] if s["Estimate_decent"] else []))
        cam_iop = {}
        for i in range(data.numCam):
            cid, ydir, xmin, ymin, xmax, ymax = data.INT[i][:6]
            par.append(["Camera", cid, None])
            print_cell(fh, [("Camera", cid), ("y axis dir", num2str(ydir)), ("x min", num2str(xmin)),
                            ("y min", num2str(ymin)), ("x max", num2str(xmax)), ("y max", num2str(ymax)),
                            ("\\line", "")], "")
            start = q
            for nm in iop_names:
                line = _line_eop if nm in ("xp", "yp", "c") else _line_dist
                fh.write(line(nm, xhat[q], std[q], w))
                par.append([nm, xhat[q], std[q]])
                q += 1
            cam_iop[cid] = (start, q)
            fh.write("\nIOP Correlation sub-matrix\n-------------------------------\n")
            sub = _iop_corr(res, data, cid, u_img, u_cam)
            _corr_rows(fh, [""] + iop_names, sub)
            fh.write("\n")

        # ground coordinates (main.m:843-866)
        if s["Estimate_tie"]:
            fh.write("\n" + LINE + "\n\nEstimated Ground Coordinates of targets\n"
                     "TargetID\tnumImages\tX\tY\tZ\tstdX\tstdY\tstdZ\n\n")
            tgt_count = {}
            for t in data.pho_target:
                tgt_count[t] = tgt_count.get(t, 0) + 1
            var = []
            for t in data.TIE:
                X = xhat[q:q + 3]
                sd = std[q:q + 3]
                var.append(sd ** 2)
                fh.write(f"{t:<{w}}{tgt_count.get(t, 0):<{w}d}" + "".join(f"{v:<{w}.{DECIMALS}f}" for v in X)
                         + "".join(f"{v:<{w}.{DECIMALS}f}" for v in sd) + "\n")
                q += 3
            avg = np.sqrt(np.mean(np.array(var), axis=0)) if var else np.full(3, np.nan)
            fh.write("\n\t\tMeanStd X\tMeanStd Y\tMeanStd Z\n")
            fh.write("\t\t" + "".join(f"{v:<{w}.{DECIMALS}f}" for v in avg) + "\n")

        # corrected image measurements (main.m:586-590, :869-873)
        fh.write("\n" + LINE + "\n\nCorrected Image Measurements\nPointID\tImageID\tCorrected x\tCorrected y\n\n")
        for i in range(data.n_pts):
            xc = data.xy[i, 0] + res.rsd[i, 1]
            yc = data.xy[i, 1] + res.rsd[i, 2]
            fh.write(f"{data.pho_target[i]:<{w}}{data.pho_image[i]:<{w}}{xc:<{w}.{DECIMALS}f}{yc:<{w}.{DECIMALS}f}\n")

        # mean absolute EOP/IOP correlations per camera (main.m:879-917)
        fh.write("\n" + LINE + "\n\nAbsolute (positive) mean correlation coefficients between EOPs and IOPs\n\n")
        order = sorted(range(data.numImg), key=lambda e: data.EXT[e][1])  # sortrows(EOP_IOP_Corr, 2): stable
        g = 0
        while g < len(order):
            cid = data.EXT[order[g]][1]
            members = []
            while g < len(order) and data.EXT[order[g]][1] == cid:
                members.append(order[g])
                g += 1
            has_iop = cid in cam_iop and cam_iop[cid][1] > cam_iop[cid][0]
            names = [""] + eop_names + ([""] + iop_names if cid in cam_iop else [])
            fh.write(f"Camera {cid}\n")
            m = u_img + (u_cam if has_iop else 0)
            acc = np.zeros((m, m))
            for e in members:
                acc += np.abs(np.tril(_img_corr(res, e, m)))
            _corr_rows(fh, names, acc / len(members))
            fh.write("\n")

        # check points (main.m:604-628, :920-931)
        if s.get("Check_Points") and data.CZE:
            names_x = {nm: j for j, nm in enumerate(res.xhatnames)}
            diffs = []
            for r in data.CZE:
                j = names_x.get("X_" + r[0])
                if j is None:
                    print(f"Warning: Check point not found in xhat -> {r[0]}")
                    continue
                diffs.append((r[0], *(xhat[j:j + 3] - np.array([float(v) for v in r[1:4]]))))
            fh.write("\n" + LINE + "\n\nCheck point differences\n")
            fh.write(f"{'TargetID':<{w}}{'diff X':<{w}}{'diff Y':<{w}}{'diff Z':<{w}}\n\n")
            for d in diffs:
                fh.write(f"{d[0]:<{w}}" + "".join(f"{v:<{w}.{DECIMALS}f}" for v in d[1:]) + "\n")
            if diffs:
                a = np.array([d[1:] for d in diffs], dtype=float)
                fh.write(f"\n{'Mean':<{w}}" + "".join(f"{v:<{w}.{DECIMALS}f}" for v in a.mean(0)) + "\n")
                fh.write(f"{'RMS':<{w}}" + "".join(f"{v:<{w}.{DECIMALS}f}" for v in np.sqrt((a ** 2).mean(0))) + "\n")
    return par


def _img_corr(res, e, m):
    if res.corr is None:
        return np.full((m, m), np.nan)
    return res.corr[e][:m, :m]


def _iop_corr(res, data, cid, u_img, u_cam):
    """The camera's IOP block of Correlation: the trailing u_cam x u_cam part of any of its images'
    EOP/IOP sub-blocks (they are the same entries of Correlation)."""
    if res.corr is None or u_cam == 0:
        return np.zeros((u_cam, u_cam))
    for e in range(data.numImg):
        if data.EXT[e][1] == cid:
            return res.corr[e][u_img:u_img + u_cam, u_img:u_img + u_cam]
    return np.zeros((u_cam, u_cam))


def _cell(v):
    if v is None:
        return ""
    if isinstance(v, str):
        return v
    return f"{float(v):.15g}"


def write_par(path, par):
    """writecell(PAR, name.par, tab-delimited) (main.m:956)."""
    with open(path, "w") as fh:
        for r in par:
            fh.write("\t".join(_cell(v) for v in r) + "\n")


def write_rsd(path, data, rsd):
    """writecell(RSD, name.rsd, tab-delimited) (main.m:955, BuildRSD.m:29-40): targetID, imageID, x, y,
    r, vx, vy, vr, vt per image point."""
    with open(path, "w") as fh:
        for i in range(data.n_pts):
            r = rsd[i]
            fh.write("\t".join([data.pho_target[i], data.pho_image[i], _cell(data.xy[i, 0]), _cell(data.xy[i, 1])]
                               + [_cell(v) for v in r]) + "\n")
