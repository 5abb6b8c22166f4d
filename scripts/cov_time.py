"""Time fba_covariance (post-fit Cx diagonal + EOP/IOP correlation blocks) after two Gauss-Newton
iterations of a benchmark scene:  python scripts/cov_time.py [config]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import fba_import
    fba = fba_import.load()
    from fba_amd import synth
    folder = os.path.join(os.environ.get("FBA_BENCH_DIR", "/tmp/fba_bench"), f"c{config}")
    if not os.path.exists(os.path.join(folder, ".done")):
        synth.make_config(config, folder)
        open(os.path.join(folder, ".done"), "w").close()
    ds = fba.load_folder(folder)
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
    for _ in range(2):
        ctx.step()
    _, _, st = ctx.residuals()
    t0 = time.perf_counter()
    cx, corr = ctx.covariance(st[3])
    dt = time.perf_counter() - t0
    # a second call after one more iteration (the covariance consumes the factor): the context's
    # workspace is allocated by the first call and reused
    ctx.step()
    _, _, st = ctx.residuals()
    t1 = time.perf_counter()
    ctx.covariance(st[3])
    dt2 = time.perf_counter() - t1
    ctx.close()
    print(f"config {config}: fba_covariance {dt * 1e3:.1f} ms (first call, workspace allocated), {dt2 * 1e3:.1f} ms "
          f"(second call) for u = {len(cx)}; finite {np.isfinite(cx).all()}, positive {(cx > 0).all()}; "
          f"median std of tie XYZ {np.median(np.sqrt(cx[-3 * ds.numtie:])):.4g}")


if __name__ == "__main__":
    main()
