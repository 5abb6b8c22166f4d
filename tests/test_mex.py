"""The MEX drop-ins with the reference's own signatures (mex/BuildAwG.c, mex/Buildxhat.c,
mex/BuildRSD.c), RUN without MATLAB: each is compiled against tests/mexstub (a stand-in for the MEX /
matrix API, test infrastructure) and libfba.so, and its mexFunction is called with the reference's
`data` struct (main.m:280-383) and cell arrays (main.m:196-258) built from the oracle's restatement
of the ingest.

* CPU: every drop-in (and the whole-loop gateway mex/fba_mex.c) compiles and links.
* GPU: on cam0 (shipped Stage-3 and a fish-eye variant, Stage-1) and a 2-camera rig --
    [error, xhat, xhatnames] = Buildxhat(data, EXT, INT, TIE, CNT)   bit-exact vs the oracle
    [error, A, misclosure, G, dist_scaling] = BuildAwG(data, xhat)   A per column <= 1e-12, w, G, ds
    RSD = BuildRSD(v, data, xhat)                                    <= 1e-12 (ids, x, y exact)
  and the reference's error behaviour: error = 1 for an invalid Type (BuildAwG.m:209-213), for a
  TIE target missing from CNT (Buildxhat.m:124-128).
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, CAM0_VARIANTS  # noqa: F401

STUB = os.path.join(ROOT, "tests", "mexstub")
LIBDIR = os.path.join(ROOT, "fish-eye_bundle_adjustment_amd")
DROPINS = ("BuildAwG", "Buildxhat", "BuildRSD")


def _build(out):
    stub = os.path.join(out, "libmxstub.so")
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-Wall", "-Werror", "-I", STUB, "-o", stub,
                    os.path.join(STUB, "mxstub.c")], check=True, capture_output=True, text=True)
    libs = {}
    for name in DROPINS + ("fba_mex",):
        so = os.path.join(out, f"{name}_mex.so")
        r = subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-Wall", "-Werror", "-I", STUB, "-I",
                            os.path.join(ROOT, "include"), "-o", so, os.path.join(ROOT, "mex", f"{name}.c"),
                            "-L", out, "-lmxstub", "-L", LIBDIR, "-lfba", f"-Wl,-rpath,{out}:{LIBDIR}"],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        libs[name] = so
    return stub, libs


def test_mex_dropins_build(tmp_path):
    """Source-level drop-ins (MATLAB is not in this image): each compiles with -Wall -Werror against
    the MEX API declarations and include/fba.h and links against libfba.so."""
    _build(str(tmp_path))


class Mx:
    """Builds / reads mxArrays through the stub's own API (ctypes)."""

    def __init__(self, stub):
        L = self.L = C.CDLL(stub, mode=C.RTLD_GLOBAL)
        P, S = C.c_void_p, C.c_size_t
        for n, a, r in [("mxCreateDoubleScalar", [C.c_double], P), ("mxCreateString", [C.c_char_p], P),
                        ("mxCreateDoubleMatrix", [S, S, C.c_int], P), ("mxCreateCellMatrix", [S, S], P),
                        ("mxCreateStructMatrix", [S, S, C.c_int, C.POINTER(C.c_char_p)], P),
                        ("mxSetCell", [P, S, P], None), ("mxSetField", [P, S, C.c_char_p, P], None),
                        ("mxGetDoubles", [P], C.POINTER(C.c_double)), ("mxGetM", [P], S), ("mxGetN", [P], S),
                        ("mxGetCell", [P, S], P), ("mxArrayToString", [P], C.c_void_p), ("mxFree", [P], None),
                        ("mxIsChar", [P], C.c_int), ("mxIsCell", [P], C.c_int), ("mxDestroyArray", [P], None),
                        ("mxstub_call", [P, C.c_int, P, C.c_int, P], C.c_int), ("mxstub_error", [], C.c_char_p),
                        ("mxstub_exit", [], None)]:
            f = getattr(L, n)
            f.argtypes, f.restype = a, r

    def num(self, v):
        return self.L.mxCreateDoubleScalar(float(v))

    def str(self, s):
        return self.L.mxCreateString(str(s).encode())

    def mat(self, a):
        a = np.atleast_2d(np.asarray(a, dtype=np.float64))
        m = self.L.mxCreateDoubleMatrix(a.shape[0], a.shape[1], 0)
        d = self.L.mxGetDoubles(m)
        for i, v in enumerate(a.reshape(-1, order="F")):
            d[i] = v
        return m

    def cell(self, rows, ncol=None):
        M = len(rows)
        N = ncol or max(len(r) for r in rows)
        c = self.L.mxCreateCellMatrix(M, N)
        for i, r in enumerate(rows):
            for j, v in enumerate(r):
                self.L.mxSetCell(c, j * M + i, self.str(v) if isinstance(v, str) else self.num(v))
        return c

    def struct(self, recs):
        """1 x len(recs) struct array; values already mxArrays"""
        names = list(recs[0])
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        s = self.L.mxCreateStructMatrix(1, len(recs), len(names), arr)
        for i, r in enumerate(recs):
            for k, v in r.items():
                self.L.mxSetField(s, i, k.encode(), v)
        return s

    def get(self, a):
        if self.L.mxIsChar(a):
            p = self.L.mxArrayToString(a)
            out = C.cast(p, C.c_char_p).value.decode()
            self.L.mxFree(p)
            return out
        m, n = self.L.mxGetM(a), self.L.mxGetN(a)
        if self.L.mxIsCell(a):
            return [[self.get(self.L.mxGetCell(a, j * m + i)) for j in range(n)] for i in range(m)]
        d = self.L.mxGetDoubles(a)
        return np.array([d[i] for i in range(m * n)]).reshape((m, n), order="F")

    def call(self, fn, nlhs, args):
        plhs = (C.c_void_p * max(nlhs, 1))()
        prhs = (C.c_void_p * len(args))(*args)
        rc = self.L.mxstub_call(C.cast(fn, C.c_void_p), nlhs, plhs, len(args), prhs)
        if rc:
            raise RuntimeError(self.L.mxstub_error().decode())
        return list(plhs)


def data_struct(mx, od):
    """main.m's `data` (settings, points, counts) and EXT / INT / TIE / CNT cells, from the oracle's
    restatement of main.m:60-384 -- the reference's 1-based indices and field names."""
    s = od.settings
    st = {k: (mx.str(v) if isinstance(v, str) else mx.num(v)) for k, v in s.items() if k != "Check_Points"}
    nk = s["Num_Radial_Distortions"]
    pts = []
    for i in range(len(od.x)):
        e, k, t = int(od.ext_index[i]), int(od.cam_num[i]), int(od.tie_index[i])
        io = od.iop_fixed[i]
        b = od.bounds[i]
        r = {"x": mx.num(od.x[i]), "y": mx.num(od.y[i]), "targetID": mx.str(od.target[i]),
             "imageID": mx.str(od.image[i]), "ext_index": mx.num(e + 1), "cameraID": mx.str(od.EXT[e][1])}
        for j, nm in enumerate(("Xc", "Yc", "Zc", "w", "p", "k")):
            r[nm] = mx.num(od.eop_fixed[i, j])
        r.update({"int_index": mx.num(2 * k + 1), "cam_num": mx.num(k + 1), "xp": mx.num(io[0]), "yp": mx.num(io[1]),
                  "c": mx.num(io[2]), "K": mx.mat(np.asarray(io[3:3 + nk]).reshape(-1, 1)),
                  "P": mx.mat(np.asarray(io[3 + nk:5 + nk]).reshape(-1, 1)), "xmin": mx.num(b[1]), "ymin": mx.num(b[2]),
                  "xmax": mx.num(b[3]), "ymax": mx.num(b[4]), "y_dir": mx.num(b[0]), "X": mx.num(od.xyz_fixed[i, 0]),
                  "Y": mx.num(od.xyz_fixed[i, 1]), "Z": mx.num(od.xyz_fixed[i, 2]),
                  "tieIndex": mx.num(t + 1 if t >= 0 else -1), "isTie": mx.num(1 if t >= 0 else 0)})
        pts.append(r)
    data = mx.struct([{"settings": mx.struct([st]), "points": mx.struct(pts), "numImg": mx.num(od.numImg),
                       "numCam": mx.num(od.numCam), "n": mx.num(od.n), "numGCP": mx.num(od.numGCP),
                       "numtie": mx.num(od.numtie)}])
    EXT = mx.cell(od.EXT)
    int_rows = []
    for r in od.INT:
        int_rows.append([r[0], r[1], r[2], r[3], r[4], r[5]])
        int_rows.append(list(r[6]))
    INT = mx.cell(int_rows, ncol=max(6, 5 + nk))
    TIE = mx.cell([[t] for t in od.TIE], ncol=1) if od.TIE else mx.L.mxCreateCellMatrix(0, 1)
    CNT = mx.cell(od.CNT)
    return data, EXT, INT, TIE, CNT


@pytest.fixture(scope="module")
def mexlibs(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("mex"))
    stub, libs = _build(out)
    mx = Mx(stub)
    fns = {n: getattr(C.CDLL(libs[n]), "mexFunction") for n in DROPINS}
    yield mx, fns
    mx.L.mxstub_exit()  # mexAtExit: the cached libfba context


def _rig_folder(tmp_path):
    from fba_amd import synth
    return synth.write_folder(synth.generate(14, 200, seed=61, n_cam=2), str(tmp_path / "rig"))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["stage3_pinhole", "stage3_fisheye", "stage1_pinhole", "rig2"])
def test_mex_dropins_match_oracle(fba, oracle, mexlibs, cam0_folders, tmp_path, variant):
    mx, fns = mexlibs
    folder = _rig_folder(tmp_path) if variant == "rig2" else cam0_folders[variant]
    od = oracle.load_folder(folder)
    data, EXT, INT, TIE, CNT = data_struct(mx, od)
    # Buildxhat
    err, xhat, names = mx.call(fns["Buildxhat"], 3, [data, EXT, INT, TIE, CNT])
    assert mx.get(err)[0, 0] == 0
    x = mx.get(xhat)[:, 0]
    xo, no = oracle.buildxhat(od)
    np.testing.assert_array_equal(x, xo)
    assert [r[0] for r in mx.get(names)] == no
    # BuildAwG at the start values and at a perturbed xhat
    rng = np.random.default_rng(3)
    for xv in (xo, xo * (1 + 1e-4 * rng.standard_normal(len(xo)))):
        out = mx.call(fns["BuildAwG"], 5, [data, mx.mat(xv.reshape(-1, 1))])
        e, A, w, G, ds = (mx.get(o) for o in out)
        assert e[0, 0] == 0
        Ao, wo, Go, dso = oracle.build_awg(od, xv)
        colmax = np.maximum(np.abs(Ao).max(axis=0), 1e-300)
        assert (np.abs(A - Ao).max(axis=0) / colmax).max() <= 1e-12
        assert np.abs(w[:, 0] - wo).max() <= 1e-12 * np.abs(od.x).max()
        if Go is None:
            assert G.shape == (1, 1) and G[0, 0] == 0  # BuildAwG.m:38: G = 0 without inner constraints
        else:
            np.testing.assert_allclose(G, Go, rtol=1e-14, atol=1e-14 * np.abs(Go).max())
        np.testing.assert_allclose(ds, dso, rtol=1e-14)
    # BuildRSD with the oracle's final v and xhat (main.m:569-571)
    ro = oracle.adjust(od)
    rsd = mx.get(mx.call(fns["BuildRSD"], 1, [mx.mat(ro.v.reshape(-1, 1)), data, mx.mat(ro.xhat.reshape(-1, 1))])[0])
    assert [r[0] for r in rsd] == od.target and [r[1] for r in rsd] == od.image
    assert np.array_equal(np.array([[r[2][0, 0], r[3][0, 0]] for r in rsd]), np.column_stack([od.x, od.y]))
    num = np.array([[v[0, 0] for v in r[4:]] for r in rsd])
    ref = oracle.build_rsd(od, ro.v, ro.xhat)
    assert np.abs(num - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.gpu
def test_mex_dropins_error_behaviour(fba, oracle, mexlibs, cam0_folders):
    """error = 1 and empty outputs where the reference sets error = 1: an invalid Type in BuildAwG
    (BuildAwG.m:209-213), a TIE target missing from CNT in Buildxhat (Buildxhat.m:124-128)."""
    mx, fns = mexlibs
    od = oracle.load_folder(cam0_folders["stage3_pinhole"])
    xo, _ = oracle.buildxhat(od)
    od.settings["type"] = "spherical"
    data, EXT, INT, TIE, CNT = data_struct(mx, od)
    out = [mx.get(o) for o in mx.call(fns["BuildAwG"], 5, [data, mx.mat(xo.reshape(-1, 1))])]
    assert out[0][0, 0] == 1 and out[1].size == 0
    od.settings["type"] = "pinhole"
    od.TIE = list(od.TIE[:-1]) + ["NOT_IN_CNT"]
    data, EXT, INT, TIE, CNT = data_struct(mx, od)
    err, xhat, names = (mx.get(o) for o in mx.call(fns["Buildxhat"], 3, [data, EXT, INT, TIE, CNT]))
    assert err[0, 0] == 1 and xhat.size == 0
