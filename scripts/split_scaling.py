"""Per-rank cost of the two multi-GPU solves, measured on ONE GPU (each rank context runs alone on the
device, as it would on its own GPU; the collective is not measured -- its bytes are reported).

For world W in {2, 4, 8}: W rank contexts (replicated: obs shards + the summed reduced system factored
on every rank; subtree: fba_options.split), host-summed reduce buffers as the all-reduce would.  Per
iteration and rank: t_acc (fba_accumulate: linearise + reduce [+ the rank's subtree factorisation]) and
t_solve (fba_solve_update: [the top columns,] backward solve, back-substitution, update).  The iteration
time on W GPUs is then max_r t_acc + t_allreduce(bytes) + max_r t_solve.

    python scripts/split_scaling.py <config> [worlds, e.g. 2,4,8] [iterations]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fba_import  # noqa: E402

fba = fba_import.load()
config = int(sys.argv[1])
worlds = [int(w) for w in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
from fba_amd import synth  # noqa: E402
folder = f"/tmp/split_scaling_c{config}"
if not os.path.exists(folder + "/.done"):
    synth.make_config(config, folder)
    open(folder + "/.done", "w").close()
ds = fba.load_folder(folder)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
mk = lambda **kw: fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings), **kw)  # noqa: E731

single = mk()
single.step()
t = []
for _ in range(iters):
    t0 = time.perf_counter()
    single.step()
    t.append(time.perf_counter() - t0)
t_single = float(np.median(t))
single.close()
out = {"config": config, "single_ms": 1e3 * t_single, "worlds": {}}
print(f"config {config}: single context {1e3 * t_single:.3f} ms/iter", flush=True)
for W in worlds:
    for solve in ("replicated", "subtree"):
        ranks = [mk(rank=r, world=W, split=solve == "subtree") for r in range(W)]
        ta = np.zeros((iters, W))
        ts = np.zeros((iters, W))
        nbytes = 0
        for it in range(iters + 1):
            for r, c in enumerate(ranks):
                c.synchronize()
                t0 = time.perf_counter()
                c.accumulate()
                c.synchronize()
                if it > 0:
                    ta[it - 1, r] = time.perf_counter() - t0
            bufs = [c.reduce_buffer() for c in ranks]
            nbytes = bufs[0][1] * 8
            total = np.zeros(bufs[0][1])
            for p, n in bufs:
                a = np.empty(n)
                hip.hipMemcpy(a.ctypes.data, p, n * 8, 2)
                total += a
            for p, n in bufs:
                hip.hipMemcpy(p, total.ctypes.data, n * 8, 1)
            for r, c in enumerate(ranks):
                t0 = time.perf_counter()
                c.solve_update()
                if it > 0:
                    ts[it - 1, r] = time.perf_counter() - t0
        for c in ranks:
            c.close()
        acc = float(np.median(ta.max(axis=1)))
        sol = float(np.median(ts.max(axis=1)))
        rec = {"t_acc_max_ms": 1e3 * acc, "t_solve_max_ms": 1e3 * sol, "compute_ms": 1e3 * (acc + sol),
               "reduce_bytes": nbytes, "t_acc_per_rank_ms": [1e3 * v for v in np.median(ta, axis=0)],
               "t_solve_per_rank_ms": [1e3 * v for v in np.median(ts, axis=0)]}
        out["worlds"].setdefault(str(W), {})[solve] = rec
        print(f"  W={W} {solve:10s}: max acc {1e3 * acc:7.3f} ms + max solve {1e3 * sol:7.3f} ms = {1e3 * (acc + sol):7.3f} ms "
              f"compute per iteration (single {1e3 * t_single:.3f}); all-reduce {nbytes / 1e6:.1f} MB", flush=True)
print(json.dumps(out))
