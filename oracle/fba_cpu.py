"""ctypes driver of oracle/libfbo.so (oracle/fba_cpu.c) -- TEST INFRASTRUCTURE ONLY.

The block-sparse CPU restatement of main.m:407-494 for scenes the dense oracle cannot hold:
``fbo_reduce`` (C/OpenMP) linearises and eliminates the tie points, the reduced camera system is
solved here with LAPACK through SciPy, ``fbo_update`` (C) back-substitutes, de-scales and updates.

Two solvers for the bordered system (main.m:432, inner constraints on):
* ``"kkt"``  -- the reference's bordered matrix [S G; G' 0] solved directly (symmetric-indefinite
  LAPACK solve); independent of the GPU's method, used by the parity tests.
* ``"chol"`` -- the regularised border M = S + G W G' (W = equilibrated) with a dense Cholesky
  factorisation and a 7x7 border correction (bench.py's dense ``cpu_baseline_dense``).
* ``"sparse"`` -- the GPU's method on the GPU's block pattern: the reduced system accumulated straight
  into 128 x 128 blocks in the device factorisation's camera-side order (libfba's fba_image_order,
  nested dissection), the local border M = S + A A' with the 14 x 14 combine, and a level-by-level
  block Cholesky in C/OpenMP calling OpenBLAS per block (fbo_sparse_solve); bench.py's ``cpu_baseline``.

Only ``tests/``, ``__graft_entry__`` and ``bench.py``'s ``cpu_baseline`` leg may import this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time

import numpy as np
import scipy.linalg as sla

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfbo.so")
TYPES = ("fisheye", "pinhole", "equisolid", "orthographic", "stereographic")


class Input(C.Structure):
    _fields_ = [("n_pts", C.c_int64), ("n_img", C.c_int32), ("n_cam", C.c_int32), ("n_tie", C.c_int32),
                ("nk", C.c_int32), ("type", C.c_int32), ("est", C.c_int32 * 11), ("ic", C.c_int32),
                ("reserved", C.c_int32), ("sx", C.c_double), ("sy", C.c_double)] + [
        (n, C.c_void_p) for n in ("x", "y", "img", "cam", "tie", "eop", "iop", "bounds", "xyz")]


def build():
    """Compile libfbo.so with the committed Makefile (gcc + OpenMP)."""
    subprocess.run(["make", "-s", "-C", _HERE, "libfbo.so"], check=True)


def _lib():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    lib.fbo_create.argtypes = [P, C.c_int]
    lib.fbo_create.restype = P
    lib.fbo_destroy.argtypes = [P]
    lib.fbo_sizes.argtypes = [P, P]
    lib.fbo_reduce.argtypes = [P, P, P, P, P]
    lib.fbo_reduce.restype = C.c_int
    lib.fbo_update.argtypes = [P, P, P]
    lib.fbo_update.restype = C.c_double
    lib.fbo_set_shard.argtypes = [P, P, C.c_int]
    lib.fbo_residuals.argtypes = [P, P]
    lib.fbo_residuals.restype = C.c_double
    lib.fbo_set_blas.argtypes = [P, P, P, P]
    lib.fbo_sparse_setup.argtypes = [P, P, C.c_int]
    lib.fbo_sparse_setup.restype = C.c_int
    lib.fbo_sparse_info.argtypes = [P, P]
    lib.fbo_set_sparse.argtypes = [P, C.c_int]
    lib.fbo_sparse_solve.argtypes = [P, P, P, P, P]
    lib.fbo_sparse_solve.restype = C.c_int
    lib.fbo_set_blas(*_blas_pointers())
    return lib


def _blas_pointers():
    """dgemm / dsyrk / dtrsm / dpotrf of the OpenBLAS SciPy ships, from its Cython function-pointer
    capsules (called per 128 x 128 block by fbo_sparse_solve's OpenMP threads, OpenBLAS itself on one
    thread)."""
    import scipy.linalg.cython_blas as cb
    import scipy.linalg.cython_lapack as cl
    name = C.pythonapi.PyCapsule_GetName
    name.argtypes, name.restype = [C.py_object], C.c_char_p
    get = C.pythonapi.PyCapsule_GetPointer
    get.argtypes, get.restype = [C.py_object, C.c_char_p], C.c_void_p
    caps = [cb.__pyx_capi__["dgemm"], cb.__pyx_capi__["dsyrk"], cb.__pyx_capi__["dtrsm"], cl.__pyx_capi__["dpotrf"]]
    return [get(c, name(c)) for c in caps]


def image_order(data):
    """The device factorisation's camera-side order (libfba.so fba_image_order, host only): slot -> EXT
    row, -1 for a padding slot."""
    import fba_import
    fba = fba_import.load()
    n = len(data.x)
    eop0 = np.array([r[2:8] for r in data.EXT[: data.numImg]], dtype=np.float64).reshape(-1)
    packed = fba.capi.PackedProblem(np.column_stack([data.x, data.y]), data.ext_index, data.cam_num, data.tie_index,
                                    data.xyz_fixed, eop0, np.zeros(max(data.numCam, 1) * 6),
                                    np.tile([1.0, 0, 0, 0, 0], max(data.numCam, 1)), np.zeros(3 * max(data.numtie, 1)),
                                    data.numImg, data.numCam, data.numtie)
    assert packed.n_pts == n
    return fba.capi.image_order(packed)


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib()
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def default_threads():
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return n if n > 0 else min(os.cpu_count() or 1, 16)


class CpuAdjustment:
    """One scene (an ``oracle.fba_oracle.Data``), iterated on the host."""

    def __init__(self, data, threads=None, solver="kkt"):
        from fba_oracle import buildxhat
        s = data.settings
        if s["type"] not in TYPES:
            raise ValueError("BuildAwG, invalid type in data.settings.type")
        nk = int(s["Num_Radial_Distortions"])
        self.data, self.solver = data, solver
        self.threads = threads or default_threads()
        self._keep = dict(
            x=np.ascontiguousarray(data.x, np.float64), y=np.ascontiguousarray(data.y, np.float64),
            img=np.ascontiguousarray(data.ext_index, np.int64), cam=np.ascontiguousarray(data.cam_num, np.int64),
            tie=np.ascontiguousarray(data.tie_index, np.int64),
            eop=np.ascontiguousarray(data.eop_fixed, np.float64),
            iop=np.ascontiguousarray(data.iop_fixed[:, :5 + nk], np.float64),
            bounds=np.ascontiguousarray(data.bounds, np.float64),
            xyz=np.ascontiguousarray(data.xyz_fixed, np.float64))
        est = (C.c_int32 * 11)(*[int(s[k]) for k in (
            "Estimate_Xc", "Estimate_Yc", "Estimate_Zc", "Estimate_w", "Estimate_p", "Estimate_k",
            "Estimate_xp", "Estimate_yp", "Estimate_c", "Estimate_radial", "Estimate_decent")])
        k = self._keep
        self.inp = Input(len(data.x), data.numImg, data.numCam, data.numtie, nk, TYPES.index(s["type"]), est,
                         int(s["Inner_Constraints"]), 0, float(s["Meas_std"]), float(s["Meas_std_y"]),
                         *[_p(k[n]).value for n in ("x", "y", "img", "cam", "tie", "eop", "iop", "bounds", "xyz")])
        self.h = lib().fbo_create(C.byref(self.inp), int(self.threads))
        if not self.h:
            raise ValueError("fbo_create: unsupported settings")
        sz = np.zeros(4, np.int64)
        lib().fbo_sizes(self.h, _p(sz))
        self.u, self.u_c = int(sz[0]), int(sz[1])
        self.ic = bool(s["Inner_Constraints"])
        self.xhat, self.names = buildxhat(data)
        assert len(self.xhat) == self.u
        self.G = np.zeros((self.u_c, 7)) if self.ic else None
        self.deltasum = []
        self.solve_times = np.zeros(3)  # sparse: border + RHS, factor, triangular solves (s, last solve)
        if solver == "sparse":
            slots = np.ascontiguousarray(image_order(data), dtype=np.int32)
            if lib().fbo_sparse_setup(self.h, _p(slots), len(slots)) != 0:
                raise ValueError("fbo_sparse_setup: the image order does not cover every image")
            lib().fbo_set_sparse(self.h, 1)
            info = np.zeros(6, np.int64)
            lib().fbo_sparse_info(self.h, _p(info))
            self.sparse_info = dict(zip(("n_pad", "blocks", "levels", "panel_blocks", "targets", "updates"),
                                        (int(v) for v in info)))
            self.flat = None
            self.S = None
            self.r = np.zeros(self.u_c)
            return
        # S and r share one flat buffer: the unit a multi-rank caller all-reduces
        self.flat = np.zeros(self.u_c * self.u_c + self.u_c)
        self.S = self.flat[: self.u_c * self.u_c].reshape(self.u_c, self.u_c)
        self.r = self.flat[self.u_c * self.u_c:]

    def close(self):
        if getattr(self, "h", None):
            lib().fbo_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _solve(self):
        S, r, G = self.S, self.r, self.G
        if self.solver == "sparse":
            dc = np.zeros(self.u_c)
            rc = lib().fbo_sparse_solve(self.h, _p(r), _p(G) if self.ic else None, _p(dc), _p(self.solve_times))
            if rc != 0:
                raise FloatingPointError(f"fbo_sparse_solve: {('', 'not positive definite', 'singular border', 'no BLAS')[rc]}")
            return dc
        if not self.ic:
            return sla.cho_solve(sla.cho_factor(S, lower=True, overwrite_a=True, check_finite=False), -r,
                                 check_finite=False)
        if self.solver == "kkt":
            K = np.zeros((self.u_c + 7, self.u_c + 7))
            K[: self.u_c, : self.u_c] = S
            K[: self.u_c, self.u_c:] = G
            K[self.u_c:, : self.u_c] = G.T
            rhs = np.concatenate([-r, np.zeros(7)])
            return sla.solve(K, rhs, assume_a="sym", overwrite_a=True, check_finite=False)[: self.u_c]
        # regularised border: M = S + G W G', M d = -r - G k, G'd = 0
        dg = np.diag(S).copy()
        wm = 1.0 / np.einsum("im,i->m", G * G, 1.0 / dg)
        M = S
        M += (G * wm) @ G.T
        f = sla.cho_factor(M, lower=True, overwrite_a=True, check_finite=False)
        X = sla.cho_solve(f, np.column_stack([-r, G]), check_finite=False)
        x0, Y = X[:, 0], X[:, 1:]
        k = np.linalg.solve(G.T @ Y, G.T @ x0)
        return x0 - Y @ k

    def set_shard(self, owned_obs, count_cam):
        """Restrict to one rank's observations (fba_partition's split); see fbo_set_shard."""
        self._owned = np.ascontiguousarray(owned_obs, dtype=np.uint8)
        lib().fbo_set_shard(self.h, _p(self._owned), int(count_cam))

    def accumulate(self):
        """Linearise + point-reduce into ``self.flat`` (= [S | r])."""
        rc = lib().fbo_reduce(self.h, _p(self.xhat), None if self.S is None else _p(self.S), _p(self.r),
                              _p(self.G) if self.ic else None)
        if rc != 0:
            raise FloatingPointError("singular tie-point block")

    def solve_update(self):
        """Bordered solve of the (summed) reduced system, back-substitution, update; returns this
        context's share of deltasum."""
        dc = np.ascontiguousarray(self._solve())
        return lib().fbo_update(self.h, _p(dc), _p(self.xhat))

    def step(self):
        """One pass of main.m:413-488; returns deltasum."""
        self.accumulate()
        d = self.solve_update()
        self.deltasum.append(d)
        return d

    def adjust(self, max_iter=None):
        """main.m:407-494: while deltasum > threshold, at most Iteration_Cap passes."""
        s = self.data.settings
        cap = s["Iteration_Cap"] if max_iter is None else min(s["Iteration_Cap"], max_iter)
        d, it = 100.0, 0
        while d > s["threshold"]:
            it += 1
            d = self.step()
            if it >= cap:
                break
        return it

    def residuals(self):
        """main.m:569, :601: v and sigma0^2 from the last linearisation and de-scaled delta."""
        v = np.zeros(2 * len(self.data.x))
        vtpv = lib().fbo_residuals(self.h, _p(v))
        return v, vtpv / (len(v) - self.u)


def time_iterations(folder, seconds=20.0, threads=None, data=None, solver="sparse"):
    """cpu_baseline: Gauss-Newton passes per second of the CPU restatement on ``folder``'s scene,
    bounded to ~``seconds``: OpenMP linearise + per-point Schur, then ``solver`` -- "sparse" (the
    default: the block Cholesky of the reduced system on the device factorisation's block pattern,
    OpenMP over blocks, one OpenBLAS thread per block) or "chol" (the dense Cholesky of the bordered
    reduced system, threaded LAPACK) -- then back-substitution and update."""
    from threadpoolctl import threadpool_limits
    import fba_oracle
    if data is None:
        data = fba_oracle.load_folder(folder)
    threads = threads or default_threads()
    ph = {"linearize_reduce": 0.0, "solve": 0.0, "update": 0.0}
    sub = np.zeros(3)
    with threadpool_limits(limits=1 if solver == "sparse" else threads):
        adj = CpuAdjustment(data, threads=threads, solver=solver)
        t0 = time.perf_counter()
        n = 0
        while True:
            # one pass of main.m:413-488 (= adj.step()), timed per phase
            ta = time.perf_counter()
            adj.accumulate()
            tb = time.perf_counter()
            dc = np.ascontiguousarray(adj._solve())
            tc = time.perf_counter()
            adj.deltasum.append(lib().fbo_update(adj.h, _p(dc), _p(adj.xhat)))
            td = time.perf_counter()
            ph["linearize_reduce"] += tb - ta
            ph["solve"] += tc - tb
            ph["update"] += td - tc
            sub += adj.solve_times
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds or n >= 1000:
                break
        adj.close()
    out = {"value": n / el, "iterations": n, "seconds": el, "cores": threads, "solver": solver,
           "n_pts": len(data.x), "u": adj.u, "u_c": adj.u_c, "cpu_model": cpu_model(),
           "phase_ms": {k: 1e3 * v / n for k, v in ph.items()}}
    if solver == "sparse":
        out["solve_ms"] = {k: 1e3 * v / n for k, v in zip(("border_rhs", "factor", "triangular_solves"), sub)}
        out["pattern"] = adj.sparse_info
    return out


def cpu_model():
    """The host CPU's model string (/proc/cpuinfo), for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"
