"""GPU diagnostic: per Gauss-Newton pass, how far the 2-rank contexts (host-summed reduce buffers) land
from the single context -- the replicated solve (obs shards) and the subtree split -- per parameter group
and per element (conftest metrics).  Usage: python scripts/split_diag.py <config> [passes]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fba_import  # noqa: E402
from conftest import dist_scaling_of, elem_rel_err, group_rel_err  # noqa: E402

fba = fba_import.load()
config = int(sys.argv[1])
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 2
from fba_amd import synth  # noqa: E402
folder = f"/tmp/split_diag_c{config}"
if not os.path.exists(folder + "/.done"):
    synth.make_config(config, folder)
    open(folder + "/.done", "w").close()
ds = fba.load_folder(folder)
names = fba.xhat_names(ds)
dsc = dist_scaling_of(__import__("fba_oracle").load_folder(folder))
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
mk = lambda **kw: fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings), **kw)  # noqa: E731
single = mk()
import fba_cpu  # noqa: E402
fba_cpu.build()
ref = fba_cpu.CpuAdjustment(__import__("fba_oracle").load_folder(folder), solver="sparse")
runs = {"obs-shard": [mk(rank=r, world=2) for r in range(2)], "split": [mk(rank=r, world=2, split=True) for r in range(2)]}
# the top block columns (printed by the verbose split context) -> the camera-side entries in top blocks
import io as _io, contextlib as _cl  # noqa: E401
top_cols = None
if os.environ.get("SPLIT_DIAG_TOP"):
    top_cols = set(int(v) for v in os.environ["SPLIT_DIAG_TOP"].split(","))
resync = os.environ.get("SPLIT_DIAG_RESYNC") == "1"
selfsync = os.environ.get("SPLIT_DIAG_SELFSYNC", "")
for it in range(passes):
    if selfsync and it > 0:  # each 2-rank run restarts from its OWN assembled iterate (stale entries refreshed)
        t0 = len(names) - 3 * ds.pack().n_tie
        for ranks in runs.values():
            xa = sum(c.get_xhat(owned_only=True) for c in ranks)
            for c in ranks:
                x = c.get_xhat()
                if selfsync in ("1", "cams"):
                    x[:t0] = xa[:t0]
                if selfsync in ("1", "ties"):
                    x[t0:] = xa[t0:]
                c.set_xhat(x)
    if resync and it > 0:  # every context restarts this pass from the single context's iterate
        for ranks in runs.values():
            for c in ranks:
                c.set_xhat(single.get_xhat())
        ref.xhat[:] = single.get_xhat()
    d1 = single.step()
    xs = single.get_xhat()
    ref.step()
    g = group_rel_err(xs, ref.xhat, names, dsc)
    e = elem_rel_err(xs, ref.xhat, names, dsc)
    print(f"pass {it + 1} single vs C oracle (sparse): group max {max(g.values()):.2e} ({max(g, key=g.get)})  "
          f"elem max {max(e.values()):.2e} ({max(e, key=e.get)})", flush=True)
    for name, ranks in runs.items():
        for c in ranks:
            c.accumulate()
            c.synchronize()
        bufs = [c.reduce_buffer() for c in ranks]
        total = np.zeros(bufs[0][1])
        for p, n in bufs:
            a = np.empty(n)
            hip.hipMemcpy(a.ctypes.data, p, n * 8, 2)
            total += a
        for p, n in bufs:
            hip.hipMemcpy(p, total.ctypes.data, n * 8, 1)
        parts = [c.solve_update() for c in ranks]
        xr = sum(c.get_xhat(owned_only=True) for c in ranks)
        if name == "split":  # entries both ranks hold (top images, cameras) must agree bit for bit
            xa, xb = ranks[0].get_xhat(), ranks[1].get_xhat()
            oa, ob = ranks[0].get_xhat(owned_only=True) != 0, ranks[1].get_xhat(owned_only=True) != 0
            both = ~oa & ~ob  # (owned by neither as "owned" means rank 0 for top: use equality where rank 1 is not owner)
            t0 = len(names) - 3 * ds.pack().n_tie
            cam = np.arange(t0)
            nz = cam[(xa[cam] != xb[cam])]
            print(f"   split: camera-side entries differing between the ranks' full xhat: {len(nz)} of {t0}; "
                  f"owned by rank 0 / 1: {int(oa[:t0].sum())} / {int(ob[:t0].sum())}", flush=True)
            if top_cols is not None:  # reference-order index -> internal row: via the image order
                pk = ds.pack()
                order = fba.capi.image_order(pk)  # slot -> EXT row
                slot_of = {int(e): k for k, e in enumerate(order) if e >= 0}
                u_img = 6  # every EOP estimated at configs 3-5
                n_img = pk.n_img
                rows = np.array([6 * slot_of[i // u_img] + i % u_img for i in range(u_img * n_img)])
                in_top = np.array([r // 128 in top_cols for r in rows])
                diff = xa[: u_img * n_img] != xb[: u_img * n_img]
                print(f"   split: image entries in top blocks {int(in_top.sum())}, of which differing between ranks "
                      f"{int((diff & in_top).sum())}; cameras differing {int((xa[u_img * n_img:t0] != xb[u_img * n_img:t0]).sum())}",
                      flush=True)
        e_all = elem_rel_err(xr, ref.xhat, names, dsc)
        print(f"   {name} per-group elem vs oracle: " + " ".join(f"{k}:{v:.1e}" for k, v in e_all.items()), flush=True)
        g = group_rel_err(xr, ref.xhat, names, dsc)
        e = elem_rel_err(xr, ref.xhat, names, dsc)
        print(f"pass {it + 1} {name:9s} vs C oracle: group max {max(g.values()):.2e} ({max(g, key=g.get)})  "
              f"elem max {max(e.values()):.2e} ({max(e, key=e.get)})", flush=True)
        g = group_rel_err(xr, xs, names, dsc)
        e = elem_rel_err(xr, xs, names, dsc)
        if name == "split" and it == passes - 1:  # the worst elements
            sc = __import__("conftest").distortion_scale(names, dsc)
            a, b = xr * sc, xs * sc
            grp = __import__("conftest").param_groups(names)
            rel = np.zeros(len(a))
            for gname, idx in grp.items():
                den = np.maximum(np.abs(b[idx]), 1e-6 * np.max(np.abs(b[idx])))
                rel[idx] = np.abs(a[idx] - b[idx]) / den
            order = np.argsort(-rel)[:12]
            pk = ds.pack()
            tie = np.asarray(pk.tie)
            img = np.asarray(pk.img)
            for i in order:
                nm = names[i]
                extra = ""
                t0 = len(names) - 3 * pk.n_tie
                if i >= t0:
                    t = (i - t0) // 3
                    slots = np.argsort(fba.capi.image_order(pk))  # (EXT row -> position among slots, approx.)
                    ims = sorted(set(img[tie == t].tolist()))
                    extra = f" tie {t}: {int((tie == t).sum())} obs, images {ims[:8]}"
                print(f"   {nm:12s} single {b[i]: .12e} split {a[i]: .12e} |d| {abs(a[i]-b[i]):.3e} rel {rel[i]:.2e}{extra}", flush=True)
        print(f"pass {it + 1} {name:9s} buffer {bufs[0][1] * 8 / 1e6:7.1f} MB  d {sum(parts):.9e} vs {d1:.9e}  "
              f"group max {max(g.values()):.2e} ({max(g, key=g.get)})  elem max {max(e.values()):.2e} ({max(e, key=e.get)})",
              flush=True)
