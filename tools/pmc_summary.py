"""Average PMC counters per kernel over the passes written by tools/pmc.sh."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(root, "p1", "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in acc.items():
    print("==", k, " avg_us=%.2f" % (sum(dur[k]) / len(dur[k]) if dur[k] else -1))
    for c, v in sorted(cs.items()):
        print("   %-28s %16.1f" % (c, sum(v) / len(v)))
