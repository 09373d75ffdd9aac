"""Export a rocprofv3 SQLite result (run_results.db, this image's default output) to the CSV forms the
other tools read: <out>_kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs,
MaxNs — the --stats summary) and, when counters were collected, <out>_counter_collection.csv
(Dispatch_Id, Kernel_Name, Counter_Name, Counter_Value: one row per dispatch and counter, summed over
the counter's dimensions).

    python tools/rocpd_export.py gpurun_out/<dir>/<tag>/run_results.db profiles/r05/<name>
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, tot, round(avg, 3), round(100.0 * tot / total, 4), mn, mx])
    cc = c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                   "group by dispatch_id, counter_name order by dispatch_id").fetchall()
    if cc:
        with open(out + "_counter_collection.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            for d, k, n, v in cc:
                w.writerow([d, k, n, v])
    print(out, len(rows), "kernels,", len(cc), "counter rows")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
