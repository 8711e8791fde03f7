"""Write the per-kernel summary (name, calls, total/avg duration) of a rocprofv3 run to CSV.
usage: python scripts/prof_summary.py <run_results.db | run_kernel_stats.csv> <out.csv>"""
import csv
import sqlite3
import sys


def main(src, dst):
    rows = []
    if src.endswith(".db"):
        db = sqlite3.connect(src)
        for name, calls, total, avg, pct in db.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            rows.append((name[:160], calls, round(total * 1e3), round(avg * 1e3), round(pct, 3)))
    else:
        with open(src) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"][:160], int(r["Calls"]), int(r["TotalDurationNs"]), round(float(r["AverageNs"])),
                             round(float(r["Percentage"]), 3)))
    rows.sort(key=lambda r: -r[2])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        w.writerows(rows)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
