"""Per-kernel register / spill / occupancy table of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/resource_usage.py [source.hip] [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "raytracing_test_amd/csrc/svo_cast.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-c", src,
       "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in err.splitlines():
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    name = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    name = re.sub(r"\(anonymous namespace\)::", "", name)[:70]
    print("%-70s VGPR %3s AGPR %3s SGPR %3s spillV %2s spillS %2s scratch %3s occ %s" % (
        name, r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"), r.get("ScratchSize [bytes/lane]"),
        r.get("Occupancy [waves/SIMD]")))
