"""Per-kernel time table from a rocprofv3 SQLite output (``run_results.db``): the same columns
as ``--stats`` CSVs (Name, Calls, TotalDurationNs, AverageNs, Percentage).

    python scripts/rocpd_stats.py gpurun_out/x/prof/run_results.db [--csv out.csv] [--top 30]
"""
import argparse
import csv
import sqlite3
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args(argv)
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                      "max(duration) from kernels group by name order by sum(duration) desc"
                      ).fetchall()
    tot = sum(r[2] for r in rows) or 1
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                        "MaxNs"])
            for r in rows:
                w.writerow([r[0], r[1], r[2], round(r[3], 1), round(100 * r[2] / tot, 3), r[4],
                            r[5]])
    for r in rows[:a.top]:
        print(f"{100 * r[2] / tot:5.1f}% {r[1]:6d} {r[3] / 1e3:9.1f} us  {r[0][:110]}")
    print(f"total {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} dispatches")
    return 0


if __name__ == "__main__":
    sys.exit(main())
