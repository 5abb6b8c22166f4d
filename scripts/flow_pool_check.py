"""k_chol_flow's two-pool persistent dispatch (FBA_FLOW_MAIN = K, read at context creation) against the
per-record grid: the same records, so the iterates must agree bit for bit.
    python scripts/flow_pool_check.py <config> <K> [<K> ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import fba_import  # noqa: E402
from bench import scene_folder  # noqa: E402

fba = fba_import.load()
cfg = int(sys.argv[1])
ds = fba.load_folder(scene_folder(cfg, 0, 1))


def run(k):
    os.environ["FBA_FLOW_MAIN"] = str(k)
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
    os.environ.pop("FBA_FLOW_MAIN")
    try:
        d = [ctx.step() for _ in range(3)]
        return d, ctx.get_xhat()
    finally:
        ctx.close()


d0, x0 = run(0)
for k in sys.argv[2:]:
    d, x = run(int(k))
    print(f"config {cfg} K={k}: deltasums equal {d == d0}, xhat equal {np.array_equal(x, x0)}", flush=True)
    assert d == d0 and np.array_equal(x, x0)
