"""Kernel statistics (the rocprofv3 --stats kernel_stats.csv columns) from a rocprofv3 rocpd SQLite database
(ROCm 7.2's default output format when --output-format is not given).
usage: python scripts/rocpd_stats.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys


def main(db, out):
    con = sqlite3.connect(db)
    rows = con.execute("SELECT name, COUNT(*), SUM(end - start), AVG(end - start), MIN(end - start), MAX(end - start) "
                       "FROM kernels GROUP BY name ORDER BY SUM(end - start) DESC").fetchall()
    total = sum(r[2] for r in rows)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 4), mn, mx])
    return rows, total


if __name__ == "__main__":
    rows, total = main(sys.argv[1], sys.argv[2])
    for name, n, tot, avg, *_ in rows[:12]:
        print(f"{n:6d} {avg / 1e3:10.1f} us {100.0 * tot / total:6.2f} %  {name[:90]}")
