"""Timing harness for ablated library builds (measurement only): N Gauss-Newton steps of a bench scene,
failures ignored (an ablated kernel computes garbage; the launches and their hand-offs are unchanged), so
a rocprofv3 kernel trace shows how much each kernel's time depends on the ablated part.

    rocprofv3 --kernel-trace --stats ... -- python scripts/ablate_time.py [config] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    import fba_import
    fba = fba_import.load()
    import bench
    ds = fba.load_folder(bench.scene_folder(config, 0, 1))
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
    x0 = ctx.get_xhat()
    fails = 0
    try:
        for _ in range(steps):
            ctx.set_xhat(x0)  # the same linearisation point every step (an ablated step leaves garbage)
            try:
                ctx.step()
            except fba.capi.FBAError:
                fails += 1
    finally:
        ctx.close()
    print(f"ablate_time: {steps} steps, {fails} reported a failure", flush=True)


if __name__ == "__main__":
    main()
