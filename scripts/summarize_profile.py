"""Summarise rocprofv3 outputs (kernel stats + FETCH/WRITE/SQ PMC passes) of one bench run.

  python scripts/summarize_profile.py <tag> <preset> <W> <H> <spp>
Reads gpurun_out/prof_<tag>_{kt,fetch,write,sq}/, writes profiles/<tag>_summary.md (+ the raw
kernel_stats csv) and updates profiles/pmc_traffic.json (HBM bytes per launch of the render kernel,
FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note; bench.py reports it as roofline.traffic).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, preset, W, H, spp = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5]
src = os.path.join(ROOT, "gpurun_out")
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)


def rows(name):
    p = os.path.join(src, f"prof_{tag}_{name}", "run_counter_collection.csv")
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


def per_dispatch(rs):
    out = {}
    for r in rs:
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        out.setdefault(k, {})
        out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def is_render(name):
    return "render_kernel" in name or "render_basic_kernel" in name


lines = [f"# rocprofv3 summary `{tag}`: bench.py, {preset} {W}x{H} {spp} spp\n"]
kt = os.path.join(src, f"prof_{tag}_kt", "run_kernel_stats.csv")
if os.path.exists(kt):
    shutil.copy(kt, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    lines.append("## kernel stats (`--kernel-trace --stats`)\n\n| kernel | calls | avg ms | total ms |\n|---|---|---|---|")
    for r in csv.DictReader(open(kt)):
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | {float(r['TotalDurationNs'])/1e6:.3f} |")
fetch, write, sq = per_dispatch(rows("fetch")), per_dispatch(rows("write")), per_dispatch(rows("sq"))
main_f = [v for (d, n), v in sorted(fetch.items()) if is_render(n)]
main_w = [v for (d, n), v in sorted(write.items()) if is_render(n)]
main_sq = [(n, v) for (d, n), v in sorted(sq.items()) if is_render(n)]
traffic = None
if main_f and main_w:
    # the first render dispatch of the run is the timed kernel's twin (stats warm-up)
    f_kb, w_kb = main_f[0].get("FETCH_SIZE", 0.0), main_w[0].get("WRITE_SIZE", 0.0)
    traffic = int(2 * f_kb * 1024 + w_kb * 1024)
    lines.append(f"\n## HBM traffic per launch (PMC, separate passes)\n\nFETCH_SIZE {f_kb:.0f} KB (x2 gfx950 correction), "
                 f"WRITE_SIZE {w_kb:.0f} KB -> **{traffic/1e9:.3f} GB per launch**\n")
if main_sq:
    n, v = main_sq[0]
    waves = v.get("SQ_WAVES", 0)
    lines.append("## SQ counters (first render dispatch)\n")
    for k in sorted(v):
        lines.append(f"- {k}: {v[k]:.4g}")
    if v.get("GRBM_GUI_ACTIVE") and v.get("SQ_INSTS_VALU"):
        lines.append(f"- VALU instructions per wave: {v['SQ_INSTS_VALU']/max(1,waves):.4g}")
with open(os.path.join(dst, f"{tag}_summary.md"), "w") as fh:
    fh.write("\n".join(lines) + "\n")
pj = os.path.join(dst, "pmc_traffic.json")
d = json.load(open(pj)) if os.path.exists(pj) else {}
if traffic is not None:
    d[f"{preset}_{W}x{H}_{spp}"] = {"hbm_bytes_per_launch": traffic, "source": f"profiles/{tag}_summary.md"}
    json.dump(d, open(pj, "w"), indent=1)
print("\n".join(lines))
