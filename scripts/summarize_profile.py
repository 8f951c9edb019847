"""Summarise rocprofv3 outputs (kernel stats + FETCH/WRITE/SQ PMC passes) of one bench run.

  python scripts/summarize_profile.py <tag> <preset> <W> <H> <spp> [share]
Reads gpurun_out/prof_<tag>_{kt,fetch,write,sq,sq2}/ (scripts/profile.sh), writes
profiles/<tag>_summary.md (+ the raw kernel_stats csv) and updates profiles/roofline_pmc.json, which
bench.py reads for its `roofline` object:
  - valu_insts  : SQ_INSTS_VALU of one render launch (wave-instructions, all SIMDs);
  - clock_hz    : GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH.md, DVFS give-back);
  - hbm_bytes   : 2 x FETCH_SIZE + WRITE_SIZE (FETCH_SIZE doubled per the gfx950 note of the guide);
  - lds_*       : SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE;
  - lib_sha16   : which libhrt.so build the counters belong to (bench reports whether it matches);
  - launch      : bench.py's record of the launch (hrt_last_launch: kernel, grid, occupancy, VGPRs, scratch).
The launch profiled is the first timed-kernel dispatch of the run (the warm-up frame with stats) whose SQ_WAVES
equal the launch record's waves; the same dispatch (by its order among the timed kernel's dispatches) is read in
every pass.  (r05c, C4's 8-s whole frame: the first dispatch reported SQ_WAVES 12288 against 6144 launched, with
every other counter of every pass equal to the next two dispatches'.)  A record whose SQ_WAVES differs from the waves the launch record says were launched (grid x block / 64) is
REJECTED: its counters describe another launch shape (a box whose occupancy answer differed, another
build), so bench.py does not price a launch with them.
"""
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 256 * 4


def lib_sha16():
    p = os.path.join(ROOT, "hyper-ray-tracer_amd", "lib", "libhrt.so")
    return hashlib.sha256(open(p, "rb").read()).hexdigest()[:16] if os.path.exists(p) else None


def main():
    tag, preset, W, H, spp = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    share = int(sys.argv[6]) if len(sys.argv) > 6 and sys.argv[6].isdigit() else 1
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)

    def per_dispatch(name):
        p = os.path.join(src, f"prof_{tag}_{name}", "run_counter_collection.csv")
        out = {}
        if not os.path.exists(p):
            return out
        for r in csv.DictReader(open(p)):
            k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            out.setdefault(k, {})
            out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        return out

    def first_render(d):
        """fallback without a kernel trace: the run's first render dispatch (bench's warm-up frame)"""
        for (disp, name), v in sorted(d.items()):
            if "render" in name and "reduce" not in name:
                return name, v
        return None, {}

    lines = [f"# rocprofv3 summary `{tag}`: bench.py, {preset} {W}x{H} {spp} spp"
             + (f", rank 0's share of a {share}-way tile split" if share > 1 else "") + "\n"]
    kt = os.path.join(src, f"prof_{tag}_kt", "run_kernel_stats.csv")
    kern_ms = None
    kname = None
    if os.path.exists(kt):
        shutil.copy(kt, os.path.join(dst, f"{tag}_kernel_stats.csv"))
        lines.append("## kernel stats (`--kernel-trace --stats`)\n\n| kernel | calls | avg ms | total ms |\n|---|---|---|---|")
        rows = list(csv.DictReader(open(kt)))
        for r in rows:
            lines.append(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | {float(r['TotalDurationNs'])/1e6:.3f} |")
        # the timed kernel: the most-called render instantiation (the COUNT twin runs once)
        rk = [r for r in rows if "render" in r["Name"] and "reduce" not in r["Name"]]
        if rk:
            best = max(rk, key=lambda r: (int(r["Calls"]), -float(r["AverageNs"])))
            kern_ms, kname = float(best["AverageNs"]) / 1e6, best["Name"]
    sq, sq2 = per_dispatch("sq"), per_dispatch("sq2")
    fetch, write = per_dispatch("fetch"), per_dispatch("write")

    launch = None
    for name in ("sq2", "sq", "kt"):
        lp = os.path.join(src, f"prof_{tag}_{name}", "launch.json")
        if os.path.exists(lp):
            launch = json.load(open(lp))
            break
    want = launch["grid"] * launch["block"] // 64 if launch else None

    def dispatches(d):
        """the timed kernel's dispatches of one pass, in order"""
        if kname is None:
            name, v = first_render(d)
            return [v] if name else []
        short = kname.split("(")[0]
        return [v for (disp, name), v in sorted(d.items()) if name.split("(")[0] == short]

    ordinal = 0
    for i, v in enumerate(dispatches(sq2)):
        if want is not None and int(round(v.get("SQ_WAVES", -1))) == want:
            ordinal = i
            break

    def timed(d):
        ds = dispatches(d)
        return ds[ordinal] if ordinal < len(ds) else (ds[0] if ds else {})

    s1, s2, f, w = timed(sq), timed(sq2), timed(fetch), timed(write)
    c = {**s1, **s2}
    res = {"source": f"profiles/{tag}_summary.md", "kernel": kname, "kernel_avg_ms": kern_ms,
           "lib_sha16": None if "--no-sha" in sys.argv else lib_sha16()}
    if f and w:
        res["hbm_bytes"] = int(2 * f.get("FETCH_SIZE", 0) * 1024 + w.get("WRITE_SIZE", 0) * 1024)
        res["fetch_bytes_x2"] = int(2 * f.get("FETCH_SIZE", 0) * 1024)
        res["write_bytes"] = int(w.get("WRITE_SIZE", 0) * 1024)
        lines.append(f"\n## HBM traffic per launch (PMC, separate passes)\n\nFETCH_SIZE {f.get('FETCH_SIZE', 0):.0f} KB (x2 gfx950 "
                     f"correction), WRITE_SIZE {w.get('WRITE_SIZE', 0):.0f} KB -> **{res['hbm_bytes']/1e9:.3f} GB per launch**"
                     + (f" = {res['hbm_bytes']/1e9/(kern_ms*1e-3):.1f} GB/s over the kernel" if kern_ms else "") + "\n")
    if c:
        lines.append("## SQ / GRBM counters (one timed-kernel launch)\n")
        for k in sorted(c):
            lines.append(f"- {k}: {c[k]:.4g}")
        g = c.get("GRBM_GUI_ACTIVE")
        iv = c.get("SQ_INSTS_VALU")
        if g and kern_ms:
            cyc = g / 8.0  # per XCD
            res["clock_hz"] = cyc / (kern_ms * 1e-3)
            res["cycles_per_xcd"] = cyc
        if iv:
            res["valu_insts"] = iv
        for k in ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAVE_CYCLES",
                  "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VMEM"):
            if k in c:
                res[k.lower()] = c[k]
        if g and iv:
            frac = iv * 2.0 / (SIMDS * g / 8.0)
            res["valu_issue_frac_measured_clock"] = frac
            lines.append(f"\n**VALU issue**: {iv:.4g} wave-instructions x 2 cycles (wave64 on SIMD32) / (1024 SIMDs x {g/8:.4g} "
                         f"cycles per XCD) = **{frac:.3f}** of issue capacity at the measured clock "
                         f"({res.get('clock_hz', 0)/1e9:.2f} GHz)")
            if "SQ_LDS_IDX_ACTIVE" in c:
                lines.append(f"\n**LDS**: {c['SQ_INSTS_LDS']:.4g} LDS instructions, bank-conflict cycles "
                             f"{c['SQ_LDS_BANK_CONFLICT']/c['SQ_LDS_IDX_ACTIVE']*100:.1f}% of {c['SQ_LDS_IDX_ACTIVE']:.4g} "
                             f"LDS-array cycles = {c['SQ_LDS_IDX_ACTIVE']/256/(g/8)*100:.1f}% of each CU's cycles")
            if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_INST_ANY" in c:
                wc = c["SQ_WAVE_CYCLES"]
                lines.append(f"\n**Wave time**: issuing {c['SQ_ACTIVE_INST_ANY']/wc*100:.1f}%, waiting to issue (pipe busy / "
                             f"dependency) {c['SQ_WAIT_INST_ANY']/wc*100:.1f}%, waiting on s_waitcnt {c['SQ_WAIT_ANY']/wc*100:.1f}%")
    if launch:
        res["launch"] = launch
        res["dispatch_ordinal"] = ordinal
        lines.append(f"\n**Launch** (hrt_last_launch): `{launch['kernel']}`, grid {launch['grid']} x {launch['block']} "
                     f"({launch['blocks_per_cu']} workgroups per CU x {launch['cus']} CUs, {launch['waves_per_simd']} waves/SIMD), "
                     f"{launch['vgprs']} VGPRs, {launch['scratch_bytes']} B scratch per lane, {launch['lds_bytes']} B LDS")
        if "SQ_WAVES" in c and int(round(c["SQ_WAVES"])) != want:
            res["rejected"] = (f"SQ_WAVES {c['SQ_WAVES']:.0f} != the launch's {want} waves: the counters describe another "
                               "launch shape")
            lines.append(f"\n**REJECTED**: {res['rejected']}")
    elif "--allow-no-launch" not in sys.argv:
        res["rejected"] = "no launch record (bench.py --launch-record): the launch shape cannot be checked"
        lines.append(f"\n**REJECTED**: {res['rejected']}")
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    pj = os.path.join(dst, "roofline_pmc.json")
    d = json.load(open(pj)) if os.path.exists(pj) else {}
    d[f"{preset}_{W}x{H}_{spp}" + (f"_share{share}" if share > 1 else "")] = res
    with open(pj, "w") as fh:
        json.dump(d, fh, indent=1)
    print("\n".join(lines))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
