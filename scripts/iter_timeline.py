"""One Gauss-Newton iteration from a rocprofv3 kernel_trace.csv: per-kernel start, duration and gap
(the second-to-last iteration, delimited by k_params launches), plus per-name totals."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted([(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fba::", ""), int(r["Start_Timestamp"]),
              int(r["End_Timestamp"])) for r in rows], key=lambda k: k[1])
st = [i for i, k in enumerate(ks) if k[0].startswith("k_params")]
seg = ks[st[-2]:st[-1]] if len(st) > 1 else ks
t0 = seg[0][1]
prev = t0
tot = defaultdict(float)
for n, s, e in seg:
    if len(sys.argv) < 3:
        print(f"{n[:26]:26s} start {(s - t0) / 1e3:8.2f} dur {(e - s) / 1e3:7.2f} gap {(s - prev) / 1e3:6.2f}")
    prev = max(prev, e)
    tot[n] += (e - s) / 1e3
print(f"iteration span {(seg[-1][2] - t0) / 1e3:.1f} us")
for n, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {n[:30]:30s} {v:8.1f}")
