"""Generate tests/golden/jac_golden.json from the reference's OWN expression text.

Run in the build container (the only place /root/reference exists):
    python tests/golden/make_jac_golden.py /root/reference

`functions/BuildAwG.m` carries its forward model (lines 163-207) and its Jacobian as
machine-generated symbolic text (EOP partials :223-348, d/dc :401-414, tie partials :457-495),
one assignment per line, branched on `typeint` (0 fisheye, 1 pinhole, 2 equisolid,
3 orthographic, 4 stereographic).  This script reads that file at generation time, evaluates each
assignment's right-hand side at 40 significant digits (mpmath) on seeded sample points and on the
cam0 point (image 101, target AL01), and stores only the resulting NUMBERS.  No reference text is
written into the repository.
"""
import json
import math
import os
import re
import sys

import mpmath as mp
import numpy as np

mp.mp.dps = 40

TARGETS = ["A11", "A12", "A13", "A14", "A15", "A16", "A21", "A22", "A23", "A24", "A25", "A26",
           "Ax_c", "Ay_c", "dx_dX", "dx_dY", "dx_dZ", "dy_dX", "dy_dY", "dy_dZ"]
MODEL = ["U", "V", "W", "R"]
ASSIGN = re.compile(r"^\s*([A-Za-z_][A-Za-z0-9_]*)\s*=\s*(.*?);?\s*(%.*)?$")


def to_python(expr):
    expr = expr.strip().rstrip(";")
    expr = expr.replace(".*", "*").replace("./", "/").replace(".^", "^")
    if re.search(r"\^[\w.]+\^", expr):
        raise ValueError("chained power: associativity differs between MATLAB and Python")
    return expr.replace("^", "**")


def extract(path):
    """{typeint: {name: python_expr}} plus the shared model lines."""
    branches = {t: {} for t in range(5)}
    model, fxfy = {}, {t: {} for t in range(5)}
    cur = None
    with open(path) as fh:
        lines = fh.readlines()
    for ln, line in enumerate(lines, 1):
        mt = re.search(r"typeint\s*==\s*(\d)", line)
        if mt and re.match(r"\s*(if|elseif)\b", line):
            cur = int(mt.group(1))
        if re.match(r"\s*if\s+strcmp\(data\.settings\.type", line) or \
                re.match(r"\s*elseif\s+strcmp\(data\.settings\.type", line):
            typ = re.search(r"'(\w+)'", line).group(1)
            cur = ["fisheye", "pinhole", "equisolid", "orthographic", "stereographic"].index(typ)
        m = ASSIGN.match(line)
        if not m:
            continue
        name, rhs = m.group(1), m.group(2)
        if name in MODEL and 160 <= ln <= 170:
            model[name] = to_python(rhs)
        elif name in ("fx", "fy") and cur is not None:
            fxfy[cur][name] = to_python(rhs)
        elif name in TARGETS and cur is not None:
            branches[cur][name] = to_python(rhs)
    return model, fxfy, branches


def ns(vals):
    d = {k: mp.mpf(v) for k, v in vals.items()}
    d.update(sin=mp.sin, cos=mp.cos, tan=mp.tan, atan=mp.atan, sqrt=mp.sqrt, sec=mp.sec)
    return d


def rot(w, p, k):
    cw, sw, cp, sp, ck, sk = map(float, (mp.cos(w), mp.sin(w), mp.cos(p), mp.sin(p), mp.cos(k), mp.sin(k)))
    return np.array([[ck * cp, cw * sk + ck * sp * sw, sk * sw - ck * cw * sp],
                     [-cp * sk, ck * cw - sk * sp * sw, ck * sw + cw * sk * sp],
                     [sp, -cp * sw, cp * cw]])


def samples(rng, n):
    out = []
    for _ in range(n):
        Xc, Yc, Zc = rng.uniform(-5000, 5000, 3)
        w, p, k = rng.uniform(-math.pi / 4, math.pi / 4, 3)
        theta = rng.uniform(0.02, math.radians(80))
        az = rng.uniform(-math.pi, math.pi)
        dist = rng.uniform(500, 8000)
        d_cam = dist * np.array([math.sin(theta) * math.cos(az), math.sin(theta) * math.sin(az),
                                 -math.cos(theta)])  # W < 0: in front (Appendix C-1)
        X, Y, Z = np.array([Xc, Yc, Zc]) + rot(w, p, k).T @ d_cam
        out.append(dict(Xc=Xc, Yc=Yc, Zc=Zc, w=w, p=p, k=k, X=X, Y=Y, Z=Z,
                        c=rng.uniform(300, 1500), y_dir=float(rng.choice([-1.0, 1.0])),
                        xp=rng.uniform(-20, 20), yp=rng.uniform(-20, 20)))
    return out


def main(ref_root):
    path = os.path.join(ref_root, "functions", "BuildAwG.m")
    model, fxfy, branches = extract(path)
    assert set(model) == set(MODEL), model.keys()
    for t in range(5):
        assert set(branches[t]) == set(TARGETS), (t, set(TARGETS) - set(branches[t]))
        assert set(fxfy[t]) == {"fx", "fy"}, t
    rng = np.random.default_rng(20200501)
    pts = samples(rng, 32)
    # cam0 image 101 / target AL01 at the shipped values (cam0.ext row 1, cam0.cnt row 1, cam0.int)
    pts.append(dict(Xc=4264.553, Yc=4557.340, Zc=327.608, w=-90.0413 * math.pi / 180,
                    p=16.0509 * math.pi / 180, k=90.2032 * math.pi / 180, X=2.018, Y=2574.346,
                    Z=3519.110, c=1234.758, y_dir=-1.0, xp=1207.903, yp=1013.724))
    out = {"source": "functions/BuildAwG.m expression text evaluated with mpmath dps=40",
           "types": ["fisheye", "pinhole", "equisolid", "orthographic", "stereographic"],
           "points": pts, "values": {}}
    for t in range(5):
        rows = []
        for pt in pts:
            env = ns(pt)
            env.update(delta_r=mp.mpf(0), x_bar=mp.mpf(0), y_bar=mp.mpf(0), decentering_x=mp.mpf(0),
                       decentering_y=mp.mpf(0))
            for nm in MODEL:
                env[nm] = eval(model[nm], {"__builtins__": {}}, env)
            vals = {nm: float(eval(fxfy[t][nm], {"__builtins__": {}}, env)) for nm in ("fx", "fy")}
            for nm in TARGETS:
                vals[nm] = float(eval(branches[t][nm], {"__builtins__": {}}, env))
            rows.append(vals)
        out["values"][out["types"][t]] = rows
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jac_golden.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
