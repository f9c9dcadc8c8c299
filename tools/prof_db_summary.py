"""Kernel statistics from a rocprofv3 output (rocpd SQLite .db or kernel_stats.csv) as CSV:
Name, Calls, TotalDurationNs, AverageNs, Percentage (short kernel names)."""
import csv
import glob
import re
import sqlite3
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name) if not name.startswith("void rocprim") else "rocprim::" + \
        (re.search(r"detail::(\w+)", name).group(1) if re.search(r"detail::(\w+)", name) else "kernel")
    return name.replace("void ", "")


def main(path, out=sys.stdout):
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for db in dbs:
        c = sqlite3.connect(db)
        for name, calls, tot, avg, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            # the rocpd top_kernels view reports microseconds
            w.writerow([short(name), calls, round(tot * 1e3), round(avg * 1e3), round(pct, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
