"""How much does a concurrent linearisation slow the block factorisation down?  (Measurement only.)

Two contexts of the same scene on one GPU, each on its own stream.  Phase 1 (alone): context A steps
normally.  Phase 2 (together): context A accumulates, then context B's accumulation (k_params,
k_lin_reduce, the reductions) is enqueued right before A's solve, so B's k_lin_reduce runs beside A's
k_chol_flow.  Run under `rocprofv3 --kernel-trace` and read the trace with --analyse: per phase the
k_chol_flow and k_lin_reduce durations and how long they overlapped.  Progress is safe: B's kernels wait
for nothing, and A's flow records wait only for records of A's own launch that started before them.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl -o run -- python scripts/overlap_probe.py 4
    python scripts/overlap_probe.py --analyse gpurun_out/ovl
"""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(config):
    import fba_import
    fba = fba_import.load()
    import bench
    folder = bench.scene_folder(config, 0, 1)
    ds = fba.load_folder(folder)
    mk = lambda: fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))  # noqa: E731
    a, b = mk(), mk()
    try:
        for _ in range(3):
            a.step()
            b.step()
        n = 10
        for _ in range(n):  # phase 1: A alone
            a.step()
        b.synchronize()
        for _ in range(n):  # phase 2: B's accumulation beside A's solve
            a.accumulate()
            a.synchronize()
            b.accumulate()
            a.solve_update_async()
            a.solve_finish()
            b.synchronize()
            b.solve_update()  # (keeps B's context consistent: one solve per accumulation)
        print("overlap probe done", flush=True)
    finally:
        a.close()
        b.close()


def analyse(d):
    import csv
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(f)):
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fba::", "").split("<")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm, int(r["Queue_Id"]) if "Queue_Id" in r else 0))
    rows.sort()
    chol = [x for x in rows if x[2] == "k_chol_flow"]
    lin = [x for x in rows if x[2] == "k_lin_reduce"]
    print(f"{len(chol)} k_chol_flow, {len(lin)} k_lin_reduce launches")
    for c in chol:
        ov = [l for l in lin if l[0] < c[1] and l[1] > c[0]]
        s = f"chol {(c[1] - c[0]) / 1e3:8.1f} us"
        for l in ov:
            s += (f" | lin {(l[1] - l[0]) / 1e3:7.1f} us, starts {(l[0] - c[0]) / 1e3:+7.1f}, ends "
                  f"{(l[1] - c[0]) / 1e3:+7.1f} from chol start; union {(max(c[1], l[1]) - min(c[0], l[0])) / 1e3:7.1f}")
        print(s)


if __name__ == "__main__":
    if sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run(int(sys.argv[1]))
