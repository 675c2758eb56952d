"""Per-kernel summary (calls, total, average, min, max in ms) from a rocprofv3
rocpd SQLite database (rocprofv3's default output), as CSV.
    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_x_kernel_stats.csv"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    rows = con.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                       "max(end - start) from kernels group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationMs", "AverageMs", "MinMs", "MaxMs", "Percentage"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, "%.4f" % (tot / 1e6), "%.4f" % (avg / 1e6), "%.4f" % (mn / 1e6), "%.4f" % (mx / 1e6),
                    "%.2f" % (100.0 * tot / total)])


if __name__ == "__main__":
    main()
