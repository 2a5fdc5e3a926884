"""Per-training-step kernel time from a rocprofv3 kernel trace of bench.py:
a step is every launch up to and including its k_adam (round 6: the
multi-stage net opens each stage with a k_theta_to_w_pack, and the round-5
segmentation from the last of them to k_adam missed the step's first part);
the standalone block-roofline launches after the last step are excluded.
usage: step_breakdown.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# a step: every launch after the previous step's k_adam up to and including its own (the single-stage
# net opens a step with k_theta_to_w_pack; the multi-stage net launches one per stage, so the
# first-to-adam segmentation counts every launch of the step); the launches after the last step
# (block-roofline legs) are excluded
steps, cur = [], []
for r in rows:
    cur.append(r)
    if "k_adam" in r["Kernel_Name"]:
        steps.append(cur)
        cur = []
steps = steps[-10:]  # timed-region steps
per = defaultdict(float)
wall = busy = 0.0
for st in steps:
    t0 = int(st[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in st)
    wall += (t1 - t0) / 1e3
    for r in st:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        name = r["Kernel_Name"]
        for key in ("k_bwd2<64, 32, 4, 2, true", "k_bwd2", "k_fwd_pipe", "k_bwd<", "k_fwd<", "k_head", "k_stem", "reduce", "project", "adam",
                    "theta", "sum_groups", "relu_grad", "k_fwd_tf", "k_bwd_tf"):
            if key in name:
                name = key
                break
        per[name[:60]] += d
n = len(steps)
print(f"{n} steps: wall {wall / n:.1f} us/step (first launch to last end), kernels busy {busy / n:.1f} us/step, "
      f"{sum(len(st) for st in steps) / n:.0f} launches/step")
for k, v in sorted(per.items(), key=lambda x: -x[1]):
    print(f"  {k:<40s} {v / n:9.1f} us/step")
