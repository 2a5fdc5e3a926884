"""Per-training-step kernel time from a rocprofv3 kernel trace of bench.py:
steps are delimited by k_theta_to_w_pack (first launch of every step); the
standalone block-roofline launches after the last step are excluded.
usage: step_breakdown.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = []
i = 0
while i < len(rows):  # a step: k_theta_to_w_pack ... k_adam (the network's first and last launch)
    if "theta_to_w_pack" in rows[i]["Kernel_Name"]:
        j = next((j for j in range(i + 1, len(rows)) if "k_adam" in rows[j]["Kernel_Name"]
                  or "theta_to_w_pack" in rows[j]["Kernel_Name"]), None)
        if j is not None and "k_adam" in rows[j]["Kernel_Name"]:
            steps.append(rows[i:j + 1])
            i = j
    i += 1
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
print(f"{n} steps: wall {wall / n:.1f} us/step (first launch to last end), kernels busy {busy / n:.1f} us/step")
for k, v in sorted(per.items(), key=lambda x: -x[1]):
    print(f"  {k:<40s} {v / n:9.1f} us/step")
