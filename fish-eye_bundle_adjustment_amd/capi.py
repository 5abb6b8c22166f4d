"""ctypes binding of libfba.so (include/fba.h).

The shared library is built in-tree (``make -C fish-eye_bundle_adjustment_amd/csrc`` or
``__graft_entry__.build()``).  There is no fallback: if the library is missing or fails to load,
importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfba.so")

TYPES = ("fisheye", "pinhole", "equisolid", "orthographic", "stereographic")
NK_MAX = 8

# every symbol include/fba.h declares
EXPORTS = (
    "fba_last_error", "fba_abi_version", "fba_count_unknowns", "fba_partition", "fba_image_order", "fba_create",
    "fba_destroy", "fba_solve_mode", "fba_buildxhat", "fba_set_xhat", "fba_get_xhat", "fba_build_awg",
    "fba_accumulate", "fba_reduce_buffer", "fba_synchronize", "fba_solve_update", "fba_solve_update_async",
    "fba_deltasum_device", "fba_solve_finish", "fba_step", "fba_adjust",
    "fba_residuals", "fba_build_rsd", "fba_finish_stats", "fba_covariance", "fba_last_timings", "fba_set_timing", "fba_set_probe",
    "fba_probe_stats", "fba_set_spin_bound", "fba_test_border_solve",
)


class FBAError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"fba error {code}: {msg}")
        self.code = code


class Settings(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "est_Xc", "est_Yc", "est_Zc", "est_omega", "est_phi", "est_kappa", "est_xp", "est_yp", "est_c",
        "est_radial", "est_decent", "num_radial", "type", "inner_constraints", "iteration_cap", "reserved")] + [
        ("threshold", C.c_double), ("meas_std_x", C.c_double), ("meas_std_y", C.c_double)]


class Problem(C.Structure):
    _fields_ = [("n_pts", C.c_int64), ("n_img", C.c_int32), ("n_cam", C.c_int32), ("n_tie", C.c_int32),
                ("reserved", C.c_int32), ("xy", C.c_void_p), ("img", C.c_void_p), ("cam", C.c_void_p),
                ("tie", C.c_void_p), ("xyz_fixed", C.c_void_p), ("eop0", C.c_void_p), ("iop0", C.c_void_p),
                ("cam_info", C.c_void_p), ("tie0", C.c_void_p)]


class Options(C.Structure):
    _fields_ = [("device", C.c_int32), ("rank", C.c_int32), ("world", C.c_int32), ("verbose", C.c_int32),
                ("stream", C.c_void_p), ("split", C.c_int32)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built: run `make -C {os.path.join(_HERE, 'csrc')}` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    P, I, D = C.c_void_p, C.c_int32, C.c_double
    sig = {
        "fba_last_error": ([], C.c_char_p),
        "fba_abi_version": ([], C.c_int),
        "fba_count_unknowns": ([P, P, P], C.c_int),
        "fba_partition": ([P, I, P, P], C.c_int),
        "fba_image_order": ([P, P, P], C.c_int),
        "fba_create": ([P, P, P, P], C.c_int),
        "fba_destroy": ([P], None),
        "fba_solve_mode": ([P, P], C.c_int),
        "fba_buildxhat": ([P, P, P], C.c_int),
        "fba_set_xhat": ([P, P], C.c_int),
        "fba_get_xhat": ([P, P, I], C.c_int),
        "fba_build_awg": ([P, P, P, P, P, P], C.c_int),
        "fba_accumulate": ([P], C.c_int),
        "fba_reduce_buffer": ([P, P, P], C.c_int),
        "fba_synchronize": ([P], C.c_int),
        "fba_solve_update": ([P, P], C.c_int),
        "fba_solve_update_async": ([P], C.c_int),
        "fba_deltasum_device": ([P, P], C.c_int),
        "fba_solve_finish": ([P, P], C.c_int),
        "fba_step": ([P, P], C.c_int),
        "fba_build_rsd": ([P, P, P, P], C.c_int),
        "fba_adjust": ([P, P, P], C.c_int),
        "fba_residuals": ([P, P, P, P], C.c_int),
        "fba_finish_stats": ([P, P, P, D, P], C.c_int),
        "fba_covariance": ([P, D, P, P], C.c_int),
        "fba_last_timings": ([P, P], C.c_int),
        "fba_set_timing": ([P, I], C.c_int),
        "fba_set_probe": ([P, I], C.c_int),
        "fba_probe_stats": ([P, P], C.c_int),
        "fba_set_spin_bound": ([P, C.c_int64], C.c_int),
        "fba_test_border_solve": ([I, P, P], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


lib = _load()


def last_error() -> str:
    return lib.fba_last_error().decode(errors="replace")


def check(rc: int):
    if rc != 0:
        raise FBAError(rc, last_error())


def ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"] or a.flags["F_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


class PackedProblem:
    """Owns the numpy arrays a ``fba_problem`` points into."""

    def __init__(self, xy, img, cam, tie, xyz_fixed, eop0, iop0, cam_info, tie0, n_img, n_cam, n_tie):
        self.xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1)
        self.img = np.ascontiguousarray(img, dtype=np.int32)
        self.cam = np.ascontiguousarray(cam, dtype=np.int32)
        self.tie = np.ascontiguousarray(tie, dtype=np.int32)
        self.xyz_fixed = np.ascontiguousarray(xyz_fixed, dtype=np.float64).reshape(-1)
        self.eop0 = np.ascontiguousarray(eop0, dtype=np.float64).reshape(-1)
        self.iop0 = np.ascontiguousarray(iop0, dtype=np.float64).reshape(-1)
        self.cam_info = np.ascontiguousarray(cam_info, dtype=np.float64).reshape(-1)
        self.tie0 = np.ascontiguousarray(tie0, dtype=np.float64).reshape(-1)
        self.n_pts = len(self.img)
        self.n_img, self.n_cam, self.n_tie = int(n_img), int(n_cam), int(n_tie)
        self.struct = Problem(self.n_pts, self.n_img, self.n_cam, self.n_tie, 0, ptr(self.xy).value,
                              ptr(self.img).value, ptr(self.cam).value, ptr(self.tie).value,
                              ptr(self.xyz_fixed).value, ptr(self.eop0).value, ptr(self.iop0).value,
                              ptr(self.cam_info).value, ptr(self.tie0).value)


def make_settings(s: dict) -> Settings:
    """From the reference's data.settings field names (main.m:112-171)."""
    nk = int(s["Num_Radial_Distortions"])
    if s["type"] not in TYPES:
        raise FBAError(2, "BuildAwG, invalid type in data.settings.type")
    return Settings(int(s["Estimate_Xc"]), int(s["Estimate_Yc"]), int(s["Estimate_Zc"]), int(s["Estimate_w"]),
                    int(s["Estimate_p"]), int(s["Estimate_k"]), int(s["Estimate_xp"]), int(s["Estimate_yp"]),
                    int(s["Estimate_c"]), int(s["Estimate_radial"]), int(s["Estimate_decent"]), nk,
                    TYPES.index(s["type"]), int(s["Inner_Constraints"]), int(s["Iteration_Cap"]), 0,
                    float(s["threshold"]), float(s["Meas_std"]), float(s["Meas_std_y"]))


class Context:
    """One device-resident adjustment (one GPU / one rank)."""

    def __init__(self, packed: PackedProblem, settings: Settings, device=0, rank=0, world=1, stream=None,
                 verbose=False, split=False):
        self.packed = packed
        self.settings = settings
        self.world = world
        opts = Options(device, rank, world, int(verbose), stream, int(bool(split)))
        h = C.c_void_p()
        check(lib.fba_create(C.byref(packed.struct), C.byref(settings), C.byref(opts), C.byref(h)))
        self.h = h
        # the solve libfba runs: a split request falls back to the replicated solve when the block
        # pattern cannot be cut (fba_solve_mode)
        mode = C.c_int32()
        check(lib.fba_solve_mode(self.h, C.byref(mode)))
        self.split = bool(mode.value)
        u = C.c_int64()
        check(lib.fba_buildxhat(self.h, None, C.byref(u)))
        self.u = u.value

    def close(self):
        if getattr(self, "h", None):
            lib.fba_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def buildxhat(self):
        x = np.zeros(self.u)
        check(lib.fba_buildxhat(self.h, ptr(x), None))
        return x

    def set_xhat(self, xhat):
        x = np.ascontiguousarray(xhat, dtype=np.float64)
        check(lib.fba_set_xhat(self.h, ptr(x)))

    def get_xhat(self, owned_only=False):
        x = np.zeros(self.u)
        check(lib.fba_get_xhat(self.h, ptr(x), int(owned_only)))
        return x

    def build_awg(self, xhat=None, dense=True):
        n = 2 * self.packed.n_pts
        A = np.zeros((n, self.u), order="F") if dense else None
        w = np.zeros(n)
        G = np.zeros((self.u, 7), order="F") if self.settings.inner_constraints else None
        ds = np.zeros((self.packed.n_cam, 2 + self.settings.num_radial), order="F")
        x = None if xhat is None else np.ascontiguousarray(xhat, dtype=np.float64)
        check(lib.fba_build_awg(self.h, ptr(x), ptr(A), ptr(w), ptr(G), ptr(ds)))
        return A, w, G, ds

    def accumulate(self):
        check(lib.fba_accumulate(self.h))

    def reduce_buffer(self):
        p, n = C.c_void_p(), C.c_int64()
        check(lib.fba_reduce_buffer(self.h, C.byref(p), C.byref(n)))
        return p.value, n.value

    def synchronize(self):
        check(lib.fba_synchronize(self.h))

    def solve_update(self):
        d = C.c_double()
        check(lib.fba_solve_update(self.h, C.byref(d)))
        return d.value

    def solve_update_async(self):
        check(lib.fba_solve_update_async(self.h))

    def deltasum_device(self):
        p = C.c_void_p()
        check(lib.fba_deltasum_device(self.h, C.byref(p)))
        return p.value

    def solve_finish(self):
        d = C.c_double()
        check(lib.fba_solve_finish(self.h, C.byref(d)))
        return d.value

    def step(self):
        d = C.c_double()
        check(lib.fba_step(self.h, C.byref(d)))
        return d.value

    def adjust(self):
        cap = max(int(self.settings.iteration_cap), 1)
        hist = np.zeros(cap)
        it = C.c_int32()
        check(lib.fba_adjust(self.h, C.byref(it), ptr(hist)))
        return it.value, hist[: it.value].copy()

    def residuals(self):
        n = self.packed.n_pts
        v = np.zeros(2 * n)
        rsd = np.zeros((n, 5))
        st = np.zeros(6)
        check(lib.fba_residuals(self.h, ptr(v), ptr(rsd), ptr(st)))
        return v, rsd, st

    def build_rsd(self, v, xhat):
        """fba_build_rsd: BuildRSD.m rows [r, vx, vy, vr, vt] for a given v (PHO order) and xhat."""
        n = self.packed.n_pts
        v = np.ascontiguousarray(v, dtype=np.float64)
        x = np.ascontiguousarray(xhat, dtype=np.float64)
        if v.size != 2 * n or x.size != int(self.u):
            raise ValueError("BuildRSD: v must have 2*n_pts entries and xhat u entries")
        rsd = np.zeros((n, 5))
        check(lib.fba_build_rsd(self.h, ptr(v), ptr(x), ptr(rsd)))
        return rsd

    def covariance(self, sigma02, corr=True):
        """fba_covariance: diag of the reference's final Cx (main.m:428-482, :602) in xhat order, and
        per EXT image the Correlation sub-matrix over [its estimated EOPs, its camera's estimated
        IOPs] (main.m:446-456, :831-840), shape (n_img, u_img + u_cam, u_img + u_cam)."""
        st = self.settings
        u_img = sum(int(x) for x in (st.est_Xc, st.est_Yc, st.est_Zc, st.est_omega, st.est_phi, st.est_kappa))
        u_cam = (int(st.est_xp) + int(st.est_yp) + int(st.est_c) + int(st.est_radial) * int(st.num_radial)
                 + 2 * int(st.est_decent))
        mu = u_img + u_cam
        d = np.zeros(max(int(self.u), 1))
        cr = np.zeros((max(self.packed.n_img, 1), mu, mu)) if corr else None
        check(lib.fba_covariance(self.h, float(sigma02), ptr(d), ptr(cr)))
        return d[: int(self.u)], (cr[: self.packed.n_img] if corr else None)

    def set_spin_bound(self, spins=0):
        """(tests) this context's hand-off poll bound in sleeps; 0 restores the default"""
        check(lib.fba_set_spin_bound(self.h, int(spins)))

    def set_timing(self, on=True):
        check(lib.fba_set_timing(self.h, int(on)))

    def set_probe(self, on=True):
        check(lib.fba_set_probe(self.h, int(on)))

    def probe_stats(self):
        out = np.zeros(4)
        check(lib.fba_probe_stats(self.h, ptr(out)))
        return {"launches": int(out[0]), "ms": float(out[1]), "flops": float(out[2])}

    def timings(self):
        ms = np.zeros(8)
        check(lib.fba_last_timings(self.h, ptr(ms)))
        return ms


def count_unknowns(packed: PackedProblem, settings: Settings) -> int:
    u = C.c_int64()
    check(lib.fba_count_unknowns(C.byref(packed.struct), C.byref(settings), C.byref(u)))
    return u.value


def partition(packed: PackedProblem, world: int):
    t = np.zeros(max(packed.n_tie, 1), dtype=np.int32)
    q = np.zeros(max(packed.n_pts, 1), dtype=np.int32)
    check(lib.fba_partition(C.byref(packed.struct), int(world), ptr(t), ptr(q)))
    return t[: packed.n_tie], q[: packed.n_pts]


def image_order(packed: PackedProblem):
    """fba_image_order: slot -> EXT row (-1: padding slot) of the reduced system's image part."""
    n = C.c_int32()
    check(lib.fba_image_order(C.byref(packed.struct), None, C.byref(n)))
    out = np.zeros(max(n.value, 1), dtype=np.int32)
    check(lib.fba_image_order(C.byref(packed.struct), ptr(out), C.byref(n)))
    return out[: n.value]


def finish_stats(packed: PackedProblem, settings: Settings, sx2, sy2, vtpv):
    sums = np.array([sx2, sy2], dtype=np.float64)
    st = np.zeros(6)
    check(lib.fba_finish_stats(C.byref(packed.struct), C.byref(settings), ptr(sums), float(vtpv), ptr(st)))
    return st
