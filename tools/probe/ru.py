"""Register / LDS / occupancy summary of every kernel in a HIP source
(hipcc -Rpass-analysis=kernel-resource-usage).  usage: python tools/probe/ru.py <file.hip> [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src,
                    "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: (?:\s*)([A-Za-z ]+?)(?: \[bytes/(?:block|lane)\])?: (\S+) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for f, d in rows.items():
    if flt in f:
        print("%-60s vgpr %4s agpr %3s spill %3s lds %6s occ %s" % (
            f[:60], d.get("VGPRs"), d.get("AGPRs"), d.get("VGPRs Spill"), d.get("LDS Size"),
            d.get("Occupancy [waves/SIMD]", d.get("Occupancy"))))
