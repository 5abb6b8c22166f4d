"""Config-5 first-pass spread: the GPU path vs the C oracle's two exact solvers of the bordered
system (the reference's [S G; G' 0] by LDL' "kkt", and the regularised-border Cholesky "chol"),
per parameter group after each of the first two passes.  Measurement script for DESIGN.md section 6."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import fba_cpu  # noqa: E402
import fba_import  # noqa: E402
import fba_oracle  # noqa: E402
from conftest import dist_scaling_of, group_rel_err  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    fba = fba_import.load()
    from fba_amd import synth
    folder = f"/tmp/fba_spread/c{config}"
    if not os.path.exists(folder + "/.done"):
        synth.make_config(config, folder)
        open(folder + "/.done", "w").close()
    ds = fba.load_folder(folder)
    od = fba_oracle.load_folder(folder)
    dsc = dist_scaling_of(od)
    refs = {s: fba_cpu.CpuAdjustment(od, solver=s) for s in ("kkt", "chol")}
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
    for it in range(2):
        t0 = time.time()
        d = {s: r.step() for s, r in refs.items()}
        d["gpu"] = ctx.step()
        x = {s: r.xhat.copy() for s, r in refs.items()}
        x["gpu"] = ctx.get_xhat()
        names = refs["kkt"].names
        print(f"pass {it + 1} ({time.time() - t0:.0f} s): deltasum", {k: f"{v:.15e}" for k, v in d.items()}, flush=True)
        for a, b in (("gpu", "kkt"), ("chol", "kkt"), ("gpu", "chol")):
            e = group_rel_err(x[a], x[b], names, dsc)
            print(f"  {a} vs {b}: max {max(e.values()):.3e}", {k: f"{v:.1e}" for k, v in e.items()}, flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
