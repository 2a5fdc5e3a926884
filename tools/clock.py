"""Held clock and MFMA busy of the block kernels from one rocprofv3 PMC pass
over the bench command (tools/clock_pass.sh): clock = GRBM_GUI_ACTIVE / 8 XCDs
/ kernel time (MI355X_MICROARCH.md, DVFS give-back: within a few % of the
in-kernel clock on dispatches of a millisecond and more), MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), VALU
instructions per MFMA = SQ_INSTS_VALU / SQ_INSTS_MFMA (SQ_INSTS_VALU counts the
MFMAs too).  usage: clock.py PMC_DIR CONFIG OUT_JSON ROUND_TAG"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, config, out, tag = sys.argv[1:5]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        vals[r["Kernel_Name"]][r["Counter_Name"]].append((key, float(r["Counter_Value"])))
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)


def short(name):
    """k_fwd3_stack<C, W, BR, RK2> / k_bwd3_stack<C, W, BR, RK2, PAIR>: RK2 is the first bool
    template argument (mangled ...Li4ELb<RK2>E..., demangled '<64, 32, 4, true' ...)."""
    import re
    for k in ("k_fwd3_stack", "k_bwd3_stack", "k_fwd16_fused", "k_bwd16_fused"):
        if k in name:
            m = re.search(r"Li4ELb([01])E", name) or re.search(r"<64, 32, 4, (true|false)", name)
            rk2 = m is not None and m.group(1) in ("1", "true")
            return k + ("<RK2>" if rk2 and "stack" in k else "")
    return None


per = {}
for name, cs in vals.items():
    k = short(name)
    if k is None or not dur.get(name):
        continue
    n = len(cs["GRBM_GUI_ACTIVE"])
    avg = lambda c: sum(v for _, v in cs[c]) / max(len(cs[c]), 1)  # noqa: E731
    t = sum(dur[name]) / len(dur[name])
    cyc = avg("GRBM_GUI_ACTIVE") / 8.0
    d = {"launches": n, "avg_us": round(t * 1e6, 2), "clock_ghz": round(cyc / t / 1e9, 4)}
    if cs.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        d["mfma_busy"] = round(avg("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024), 4)
    if cs.get("SQ_INSTS_MFMA") and cs.get("SQ_INSTS_VALU"):
        d["valu_per_mfma"] = round(avg("SQ_INSTS_VALU") / avg("SQ_INSTS_MFMA"), 3)
    per[k] = d


def weighted(keys):
    ks = [k for k in keys if k in per]
    if not ks:
        return None
    tt = sum(per[k]["avg_us"] for k in ks)
    return round(sum(per[k]["avg_us"] * per[k]["clock_ghz"] for k in ks) / tt, 4)


fwd = [k for k in per if "fwd" in k]
res = {"config": config, "round": tag, "per_kernel": per, "clock_ghz_fwd": weighted(fwd),
       "clock_ghz_train": weighted(list(per)),
       "method": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-trace "
                 "over bench.py --no-random-leg (the network's own block kernels); clock = GRBM_GUI_ACTIVE / 8 / "
                 "kernel time; profiled passes hold a clock a few % below an unprofiled run (DVFS item 2)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
