"""Per-kernel duration statistics from a rocprofv3 SQLite output (rocpd
schema), in the columns of rocprofv3's --stats kernel_stats.csv.
usage: python tools/rocpd_stats.py <results.db> > kernel_stats.csv"""
import csv
import sqlite3
import statistics
import sys

con = sqlite3.connect(sys.argv[1])
rows = con.execute(
    "select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
    "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
by = {}
for name, dur in rows:
    by.setdefault(name, []).append(dur)
total = sum(sum(v) for v in by.values()) or 1
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                statistics.pstdev(v) if len(v) > 1 else 0.0])
