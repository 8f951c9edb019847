"""Static instruction mix of the walk loop (the loop holding the LDS node loads) of a kernel.
  python scripts/walk_isa.py [kernel-mangled-substring] [extra hipcc flags...]"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pat = sys.argv[1] if len(sys.argv) > 1 else "render_basic_kernelILi2ELb0ELb1E"
extra = sys.argv[2:]
out = "/tmp/walk_isa.s"
sphere = "basic" in pat  # render_basic_kernel lives in render_sphere.hip, built without SLP (Makefile)
src = os.path.join(ROOT, "hyper-ray-tracer_amd", "csrc", "render_sphere.hip" if sphere else ("render_general.hip" if "gwalk" in pat else "render.hip"))
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "hyper-ray-tracer_amd", "csrc"),
                "--offload-arch=gfx950", "--cuda-device-only", "-S", src, "-o", out]
               + (["-fno-slp-vectorize"] if sphere else []) + extra,
               check=True, capture_output=True)
s = open(out).read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(s) if re.match(r"^_Z\S+:", l)]
body = None
for k, (i, name) in enumerate(starts):
    if pat in name:
        body = s[i:starts[k + 1][0] if k + 1 < len(starts) else len(s)]
        break
loops, cur = {}, "top"
for l in body:
    m = re.match(r"^(\.LBB\S+|; %bb\.\d+):.*?(Loop: Header=\S+ Depth=\d|$)", l)
    if m:
        cur = m.group(2) or "top"
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    d = loops.setdefault(cur, {"n": 0, "valu": 0, "salu": 0, "ds": 0, "pk": 0, "scr": 0})
    d["n"] += 1
    op = t.split()[0]
    if op.startswith("v_"):
        d["valu"] += 1
        if op.startswith("v_pk_"):
            d["pk"] += 1
    elif op.startswith("s_"):
        d["salu"] += 1
    if op.startswith("ds_read"):
        d["ds"] += 1
    if "scratch_" in op:
        d["scr"] += 1
for k, v in loops.items():
    if v["ds"]:
        print(k, v)
