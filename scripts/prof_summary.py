"""Summarise a rocprofv3 kernel trace (results .db or kernel_stats/kernel_trace .csv) per kernel."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4])) for r in rows]


def from_csv(path):
    out = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(src, dst, title):
    dbs = glob.glob(os.path.join(src, "**", "*results.db"), recursive=True)
    csvs = glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True)
    rows = from_csv(csvs[0]) if csvs else from_db(dbs[0])
    with open(dst, "w") as fh:
        fh.write(f"# {title}\n\n| kernel | calls | total us | avg us | % |\n|---|---:|---:|---:|---:|\n")
        for n, c, t, a, p in rows:
            short = n.split("(")[0].replace("void ", "")
            fh.write(f"| `{short}` | {c} | {t:.1f} | {a:.2f} | {p:.2f} |\n")
    print(open(dst).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 kernel summary")
