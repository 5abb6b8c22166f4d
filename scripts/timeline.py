"""Per-step timeline of the Cholesky phase from a rocprofv3 kernel_trace.csv (last iteration)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fba::", ""), int(r["Start_Timestamp"]),
       int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows]
ks.sort(key=lambda k: k[1])
# last iteration: from the last k_potrf128 preceded by k_border_weights/k_border
starts = [i for i, k in enumerate(ks) if k[0].startswith("k_border_weights")]
seg = ks[starts[-1]:]
t0 = seg[0][1]
prev_end = t0
for name, s, e, q in seg[: int(sys.argv[2]) if len(sys.argv) > 2 else 60]:
    print(f"{name[:22]:22s} q{q} start {(s - t0) / 1e3:9.2f} dur {(e - s) / 1e3:7.2f}  gap {(s - prev_end) / 1e3:7.2f}")
    prev_end = max(prev_end, e)
