"""Print a rocprofv3 kernel_stats.csv as a compact table."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("%-60s %6s %10s %10s %6s" % ("kernel", "calls", "avg_us", "total_ms", "pct"))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print("%-60s %6s %10.2f %10.2f %6.1f" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3,
                                           float(r['TotalDurationNs']) / 1e6, 100 * float(r['TotalDurationNs']) / tot))
