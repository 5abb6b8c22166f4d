"""Per-kernel HBM traffic and MFMA activity from rocprofv3 passes, tagged with the build they measured.

    python scripts/pmc_summary.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        [--mfma gpurun_out/pmc_mfma] [--trace gpurun_out/prof] --config 4 [--network grid] \
        --out profiles/<name>.json

Passes (each its own rocprofv3 run of `bench.py --steps 2 --warmup 1 --no-cpu`, scripts/gpu_pmc.sh):
  * FETCH_SIZE, WRITE_SIZE (KB): per MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports half the
    bytes of wide (16 B/lane) coalesced reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.
    They do not fit one TCC pass.
  * SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE: MFMA-busy fraction of the SIMD cycles =
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs) (GRBM_GUI_ACTIVE sums the 8 XCDs'
    clocks; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over the SIMDs).
  * --trace: a `rocprofv3 --kernel-trace --stats` run of the same command; its average durations (not
    the PMC passes', which serialise and slow the dispatches) turn bytes per launch into GB/s.
Averages are per launch over all launches of the run.  `build_id` (bench.build_id(): a hash of the
library's sources) names the build the passes measured; bench.py takes `roofline.traffic` and
`roofline.mfma_busy` only from a summary whose build_id is the running tree's.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N_SIMD = 1024  # 256 CUs x 4 SIMDs
N_XCD = 8


def kname(raw):
    return raw.split("(")[0].replace("void ", "").replace("fba::", "").split("<")[0]


def load_counters(d):
    """{kernel: {counter: [launches, summed value]}} from a counter-collection CSV"""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for r in csv.DictReader(open(f)):
        a = agg[kname(r["Kernel_Name"])][r["Counter_Name"]]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
    return agg


def load_trace(d):
    """{kernel: average duration in ns} from a --kernel-trace --stats run"""
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        return {}
    out = {}
    for r in csv.DictReader(open(f[0])):
        out[kname(r["Name"])] = float(r["AverageNs"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--mfma")
    ap.add_argument("--trace")
    ap.add_argument("--config", type=int, required=True)
    ap.add_argument("--network", default="grid")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import bench
    fe, wr = load_counters(a.fetch), load_counters(a.write)
    mf = load_counters(a.mfma) if a.mfma else {}
    tr = load_trace(a.trace) if a.trace else {}
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        nf, bf = fe.get(k, {}).get("FETCH_SIZE", [0, 0.0])
        nw, bw = wr.get(k, {}).get("WRITE_SIZE", [0, 0.0])
        fetch = 2.0 * 1024.0 * bf / max(nf, 1)
        write = 1024.0 * bw / max(nw, 1)
        e = {"launches": max(nf, nw, 1), "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
             "hbm_bytes_per_launch": fetch + write}
        if k in tr:
            e["avg_launch_us"] = tr[k] * 1e-3
            e["hbm_GBs"] = (fetch + write) / (tr[k] * 1e-9) / 1e9
        m = mf.get(k)
        if m and "GRBM_GUI_ACTIVE" in m:
            n = max(m["GRBM_GUI_ACTIVE"][0], 1)
            grbm = m["GRBM_GUI_ACTIVE"][1] / n
            busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", [0, 0.0])[1] / n
            e["GRBM_GUI_ACTIVE"] = grbm
            e["SQ_VALU_MFMA_BUSY_CYCLES"] = busy
            e["SQ_BUSY_CYCLES"] = m.get("SQ_BUSY_CYCLES", [0, 0.0])[1] / n
            e["mfma_busy_frac"] = busy / (grbm / N_XCD * N_SIMD) if grbm > 0 else None
        kernels[k] = e
    doc = {"config": a.config, "network": a.network, "build_id": bench.build_id(),
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
                     "GRBM_GUI_ACTIVE, separate passes, and --kernel-trace --stats, each of bench.py --config "
                     f"{a.config}{'' if a.network == 'grid' else ' --network ' + a.network} --steps 2 --warmup 1 "
                     "--no-cpu; FETCH_SIZE x2 (gfx950 correction); mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / "
                     "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); hbm_GBs = bytes per launch / the trace's average "
                     "duration",
           "kernels": kernels}
    with open(a.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(f"build {doc['build_id']}, config {a.config} {a.network}")
    print("| kernel | launches | avg us | HBM MB/launch (read + write) | GB/s | MFMA busy |")
    print("|---|---:|---:|---|---:|---:|")
    for k, v in sorted(kernels.items(), key=lambda x: -x[1].get("avg_launch_us", 0.0) * x[1]["launches"])[:14]:
        us = v.get("avg_launch_us")
        gbs = v.get("hbm_GBs")
        mb = v.get("mfma_busy_frac")
        print(f"| {k} | {v['launches']} | {us:.1f} | {v['hbm_bytes_per_launch'] / 1e6:.1f} "
              f"({v['fetch_bytes_per_launch'] / 1e6:.1f} + {v['write_bytes_per_launch'] / 1e6:.1f}) | "
              f"{gbs:.0f} | {'-' if mb is None else f'{mb:.3f}'} |" if us else
              f"| {k} | {v['launches']} | - | {v['hbm_bytes_per_launch'] / 1e6:.1f} | - | "
              f"{'-' if mb is None else f'{mb:.3f}'} |")


if __name__ == "__main__":
    main()
