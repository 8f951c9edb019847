"""Per-kernel register/scratch/occupancy table from `make resource` (clang kernel-resource-usage remarks)."""
import re
import subprocess
import sys
import os

root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hyper-ray-tracer_amd")
out = subprocess.run(["make", "-s", "resource"], cwd=root, capture_output=True, text=True)
txt = out.stdout + out.stderr
rows, cur = [], None
for line in txt.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    n = r["name"].replace("(anonymous namespace)::", "").split("(")[0]
    if pat in n:
        print(f"{n:60s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} scratch {r.get('ScratchSize','?'):>4} occ {r.get('Occupancy','?')}")
