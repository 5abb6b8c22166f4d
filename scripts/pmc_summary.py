"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; counters in KB).

    python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write <config> profiles/<name>.json

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced
reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.  Both come from separate passes (they do
not fit one TCC pass).  Averages are per launch over all launches in the run.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fba::", "").split("<")[0]
        agg[k][0] += 1
        agg[k][1] += float(r["Counter_Value"]) * 1024.0
    return agg


def main(fetch_dir, write_dir, config, out):
    fe, wr = load(fetch_dir), load(write_dir)
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        nf, bf = fe.get(k, [0, 0.0])
        nw, bw = wr.get(k, [0, 0.0])
        n = max(nf, nw, 1)
        fetch = 2.0 * bf / max(nf, 1)
        write = bw / max(nw, 1)
        kernels[k] = {"launches": n, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                      "hbm_bytes_per_launch": fetch + write}
    doc = {"config": int(config), "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
           "bench.py --steps 2 --warmup 1 --no-cpu; FETCH_SIZE x2 (gfx950 correction)", "kernels": kernels}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, v in sorted(kernels.items(), key=lambda x: -x[1]["hbm_bytes_per_launch"] * x[1]["launches"])[:12]:
        print(f"{k:28s} launches {v['launches']:5d}  fetch {v['fetch_bytes_per_launch']/1e6:9.2f} MB  "
              f"write {v['write_bytes_per_launch']/1e6:9.2f} MB per launch")


if __name__ == "__main__":
    main(*sys.argv[1:5])
