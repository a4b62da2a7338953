"""Summarise a rocprofv3 output (results .db or *_kernel_stats.csv) into a small markdown/CSV
table for profiles/.  Usage: python tools/prof_summary.py <rocprof dir> <out prefix>"""
import csv
import glob
import os
import sqlite3
import sys


def rows_from_db(path):
    db = sqlite3.connect(path)
    cur = db.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    return [dict(name=r[0], calls=r[1], total_us=r[2], avg_us=r[3], pct=r[4]) for r in cur]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append(dict(name=r["Name"], calls=int(r["Calls"]), total_us=float(r["TotalDurationNs"]) / 1e3,
                            avg_us=float(r["AverageNs"]) / 1e3, pct=float(r["Percentage"])))
    return out


def main(d, prefix):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    rows = rows_from_csv(csvs[0]) if csvs else rows_from_db(dbs[0])
    with open(prefix + ".csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["name", "calls", "total_us", "avg_us", "pct"])
        w.writeheader()
        w.writerows(rows)
    with open(prefix + ".md", "w") as f:
        f.write("| kernel | calls | total us | avg us | % |\n|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['name']}` | {r['calls']} | {r['total_us']:.1f} | {r['avg_us']:.3f} | {r['pct']:.2f} |\n")
    print(open(prefix + ".md").read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
