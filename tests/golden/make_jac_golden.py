"""Generate tests/golden/jac_golden.json from the reference's OWN expression text.

Run in the build container (the only place /root/reference exists):
    python tests/golden/make_jac_golden.py /root/reference

`functions/BuildAwG.m` carries its forward model (lines 163-207) and its Jacobian as
machine-generated symbolic text (EOP partials :223-348, d/dc :401-414, tie partials :457-495),
and hand-written arithmetic (distortion model :167-181, xp / yp partials :373-398, rmax and the
scaled K / P columns :419-445, the inner-constraint block :516-523).  Both are evaluated here: the
generated expressions at zero distortion ("values") and, with the hand-written statements
(translated from the text: 1-based K(j) / P(1) / dist_scaling(cam, 2 + j) indexing, MATLAB row and
matrix literals), everything at nonzero distortion ("distortion"),
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


# ---- the hand-written arithmetic of BuildAwG.m (distortion model :167-181, xp / yp partials
# :373-398, rmax and the scaled K / P columns :419-445, the inner-constraint block :516-523) ----
def statements(path):
    """The file as statements: comments stripped, continuation lines joined until brackets balance."""
    out, cur, depth = [], "", 0
    with open(path) as fh:
        for line in fh:
            code = line.split("%", 1)[0]
            cur += " " + code.strip()
            depth += code.count("[") + code.count("(") - code.count("]") - code.count(")")
            if depth <= 0 and cur.strip():
                out.append(cur.strip())
                cur, depth = "", 0
    return out


def split_elems(body):
    """Elements of a MATLAB row / matrix literal body: rows by ';', elements by whitespace where
    MATLAB splits them (an operand follows, or a unary +/- glued to its operand)."""
    rows, elems, cur, depth = [], [], "", 0
    i = 0
    while i < len(body):
        ch = body[i]
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if depth == 0 and ch == ";":
            if cur.strip():
                elems.append(cur.strip())
            if elems:
                rows.append(elems)
            elems, cur = [], ""
        elif depth == 0 and ch == " " and cur.strip():
            j = i
            while j < len(body) and body[j] == " ":
                j += 1
            nxt = body[j] if j < len(body) else ""
            prev = cur.rstrip()[-1]
            unary = nxt in "+-" and j + 1 < len(body) and body[j + 1] != " "
            operand = nxt and (nxt.isalnum() or nxt in "(._")
            if prev not in "+-*/^,(" and (operand or unary):
                elems.append(cur.strip())
                cur = ""
            else:
                cur += " "
            i = j - 1
        else:
            cur += ch
        i += 1
    if cur.strip():
        elems.append(cur.strip())
    if elems:
        rows.append(elems)
    return rows


class MVec:
    """a MATLAB vector / matrix indexed from 1 (K(j), P(1), dist_scaling(cam, 2 + j))"""

    def __init__(self, f):
        self.f = f

    def __call__(self, *idx):
        return self.f(*[int(i) for i in idx])


def handwritten(path):
    st = statements(path)
    py = lambda e: to_python(e.replace("data.points(i).", "pt_"))  # noqa: E731

    def first(pat, after=0):
        for q in range(after, len(st)):
            if re.match(pat, st[q]):
                return q
        raise KeyError(pat)
    q_model = first(r"R = sqrt\(U\^2")
    h = {}
    for nm in ("x_bar", "y_bar", "r", "decentering_x", "decentering_y"):
        q = first(rf"{nm} = ", q_model)
        h[nm] = py(st[q].split("=", 1)[1])
    q = first(r"for j = 1:length\(K\)", q_model)
    h["delta_r_term"] = py(st[q + 1].split("=", 1)[1].replace("delta_r +", "", 1))
    assert st[q + 1].startswith("delta_r = delta_r +") and st[q + 2] == "end"
    for par in ("xp", "yp"):
        q0 = first(rf"if data\.settings\.Estimate_{par}", q_model)
        qa = first(r"dxp_rad = dxp_rad", q0)
        qb = first(r"dyp_rad = dyp_rad", q0)
        h[f"d{par}_xrad"] = py(st[qa].split("=", 1)[1].replace("dxp_rad", "0", 1))
        h[f"d{par}_yrad"] = py(st[qb].split("=", 1)[1].replace("dyp_rad", "0", 1))
        qc = first(r"Ablock_IOPs\(:,count_A\) = \[", q0)
        body = st[qc].split("=", 1)[1].strip()
        rows = split_elems(body[1:body.rindex("]")])
        assert len(rows) == 2 and all(len(r) == 1 for r in rows), rows
        h[f"A_{par}"] = [py(r[0]) for r in rows]
    h["rmax"] = py(st[first(r"rmax = ")].split("=", 1)[1])
    q = first(r"dist_scaling\(data\.points\(i\)\.cam_num,2\+j\) = ")
    h["scale"] = py(st[q].split("=", 1)[1])
    for nm in ("Ax_K", "Ay_K"):
        h[nm] = py(st[first(rf"{nm}\(1,j\) = ")].split("=", 1)[1])
    for nm in ("Ax_P", "Ay_P"):
        rhs = st[first(rf"{nm} = \[")].split("=", 1)[1].strip()
        close = rhs.index("]")
        rows = split_elems(rhs[1:close])
        assert len(rows) == 1 and len(rows[0]) == 2, rows
        div = rhs[close + 1:].strip()
        assert div.startswith("./")
        h[nm] = [py(e) for e in rows[0]]
        h[nm + "_div"] = py(div[2:])
    rhs = st[first(r"Gblock = \[")].split("=", 1)[1].strip()
    rows = split_elems(rhs[1:rhs.rindex("]")])
    assert len(rows) == 6 and all(len(r) == 7 for r in rows), rows
    h["G"] = [[py(e) for e in r] for r in rows]
    return h


def dist_samples(rng, n, nk):
    """EOP / XYZ / c as samples(); plus observed x, y on a 2048 px sensor, K and P of realistic size
    (each radial term up to ~10 px at the sensor corner), sensor bounds"""
    out = []
    for pt in samples(rng, n):
        xmin, ymin = rng.uniform(-10, 10, 2)
        xmax, ymax = xmin + rng.uniform(1500, 2500), ymin + rng.uniform(1500, 2500)
        rmax = math.hypot((xmax - xmin) / 2, (ymax - ymin) / 2)
        pt.update(x=rng.uniform(xmin, xmax), y=rng.uniform(ymin, ymax), xmin=xmin, ymin=ymin, xmax=xmax,
                  ymax=ymax, K=[float(rng.uniform(-10, 10) / rmax ** (2 * j + 1)) for j in range(1, nk + 1)],
                  P=[float(rng.uniform(-1e-6, 1e-6)) for _ in range(2)])
        pt["xp"] += 0.5 * (xmin + xmax)
        pt["yp"] += 0.5 * (ymin + ymax)
        out.append(pt)
    return out


def eval_handwritten(h, model, fxfy, branches, pt, t, nk):
    env = ns({k: v for k, v in pt.items() if not isinstance(v, list)})
    env["K"] = MVec(lambda j: mp.mpf(pt["K"][j - 1]))
    env["P"] = MVec(lambda j: mp.mpf(pt["P"][j - 1]))
    for k in ("xmin", "ymin", "xmax", "ymax"):
        env["pt_" + k] = mp.mpf(pt[k])
    env["pt_cam_num"] = 1
    ev = lambda e: eval(e, {"__builtins__": {}}, env)  # noqa: E731
    for nm in MODEL:
        env[nm] = ev(model[nm])
    for nm in ("x_bar", "y_bar", "r", "decentering_x", "decentering_y"):
        env[nm] = ev(h[nm])
    env["delta_r"] = mp.mpf(0)
    for j in range(1, nk + 1):
        env["j"] = j
        env["delta_r"] = env["delta_r"] + ev(h["delta_r_term"])
    vals = {nm: float(ev(fxfy[t][nm])) for nm in ("fx", "fy")}
    for nm in TARGETS:
        vals[nm] = float(ev(branches[t][nm]))
    for par in ("xp", "yp"):
        dx = dy = mp.mpf(0)
        for j in range(1, nk + 1):
            env["j"] = j
            dx += ev(h[f"d{par}_xrad"])
            dy += ev(h[f"d{par}_yrad"])
        env["dxp_rad"], env["dyp_rad"] = dx, dy
        vals[f"A_{par}"] = [float(ev(e)) for e in h[f"A_{par}"]]
    rmax = ev(h["rmax"])
    env["rmax"] = rmax
    scale = {}
    for j in range(1, nk + 1):
        env["j"] = j
        scale[j] = ev(h["scale"])
    env["dist_scaling"] = MVec(lambda cam, col: scale[col - 2])
    vals["rmax"] = float(rmax)
    vals["scale"] = [float(scale[j]) for j in range(1, nk + 1)]
    for nm in ("Ax_K", "Ay_K"):
        vals[nm] = []
        for j in range(1, nk + 1):
            env["j"] = j
            vals[nm].append(float(ev(h[nm])))
    for nm in ("Ax_P", "Ay_P"):
        d = ev(h[nm + "_div"])
        vals[nm] = [float(ev(e) / d) for e in h[nm]]
    vals["G"] = [[float(ev(e)) for e in row] for row in h["G"]]
    return vals


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
    # the hand-written terms at nonzero distortion (nK = 5, config.cfg:33)
    h = handwritten(path)
    nk = 5
    dpts = dist_samples(np.random.default_rng(20201017), 24, nk)
    out["distortion"] = {"nk": nk, "points": dpts, "values": {
        out["types"][t]: [eval_handwritten(h, model, fxfy, branches, pt, t, nk) for pt in dpts] for t in range(5)}}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jac_golden.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
