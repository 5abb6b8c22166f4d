"""Sensitivity of one Gauss-Newton pass to the summation order of the reduced system: the C oracle
(fba_cpu.c, bordered system solved directly, "kkt") run with different OpenMP thread counts -- its
camera block is summed as per-thread partials, so the thread count changes only the association of
the same floating-point sums.  The spread between such runs is the rounding-level sensitivity of
the pass that any exact restatement (the GPU path included) carries.  Measurement for DESIGN.md 6.

    python scripts/order_spread.py CONFIG [THREADS ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import fba_cpu  # noqa: E402
import fba_oracle  # noqa: E402
from conftest import dist_scaling_of, group_rel_err  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402


def main():
    config = int(sys.argv[1])
    threads = [int(t) for t in sys.argv[2:]] or [1, 8]
    folder = f"/tmp/fba_spread/c{config}"
    if not os.path.exists(folder + "/.done"):
        sys.path.insert(0, ROOT)
        import fba_import
        fba_import.load()
        from fba_amd import synth
        synth.make_config(config, folder)
        open(folder + "/.done", "w").close()
    od = fba_oracle.load_folder(folder)
    dsc = dist_scaling_of(od)
    xs = {}
    with threadpool_limits(limits=8):
        for t in threads:
            r = fba_cpu.CpuAdjustment(od, threads=t, solver="kkt")
            d = r.step()
            xs[t] = r.xhat.copy()
            names = r.names
            r.close()
            print(f"threads {t}: deltasum {d:.15e}", flush=True)
    t0 = threads[0]
    for t in threads[1:]:
        e = group_rel_err(xs[t], xs[t0], names, dsc)
        print(f"  {t} vs {t0} threads: max {max(e.values()):.3e}", {k: f"{v:.1e}" for k, v in e.items()}, flush=True)


if __name__ == "__main__":
    main()
