"""Summarise hipcc -Rpass-analysis=kernel-resource-usage for a HIP source."""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-c", src, "-o", "/dev/null",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    name = name.split("(")[0]
    print("%-44s vgpr=%s agpr=%s spill=%s scratch=%s occ=%s sgpr=%s" % (
        name, r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("ScratchSize [bytes/lane]"),
        r.get("Occupancy [waves/SIMD]"), r.get("TotalSGPRs")))
