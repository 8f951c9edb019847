"""Derived SQ metrics of the longest dispatch per kernel from scripts/pmc.sh passes.
  python scripts/pmc_summary.py <tag> [kernel-substring]"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "render"
vals = {}   # (kernel, dispatch) -> counter -> value
for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_*", "run_counter_collection.csv"))):
    per = {}
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"], int(r["Dispatch_Id"]))
        per.setdefault(k, {})
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # per kernel name keep the dispatch with the most SQ_WAVE_CYCLES / largest first counter
    best = {}
    for (name, d), c in per.items():
        score = max(c.values())
        if name not in best or score > best[name][0]:
            best[name] = (score, c)
    for name, (_, c) in best.items():
        vals.setdefault(name, {}).update(c)
for name, c in vals.items():
    short = name.replace("(anonymous namespace)::", "").split("(")[0]
    print(f"## {short}")
    g = lambda k: c.get(k, float("nan"))
    waves = g("SQ_WAVES")
    print(f"  waves {waves:.0f}  wave-cycles(q) {g('SQ_WAVE_CYCLES'):.3e}  GRBM {g('GRBM_GUI_ACTIVE'):.3e}")
    wc = g("SQ_WAVE_CYCLES")
    for k in ["SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_FLAT"]:
        print(f"  {k:24s} {g(k):.3e}  = {g(k)/wc*100:6.1f}% of wave-cycles")
    iv = g("SQ_INSTS_VALU")
    print(f"  VALU insts {iv:.3e}  SALU {g('SQ_INSTS_SALU'):.3e}  LDS {g('SQ_INSTS_LDS'):.3e}  BRANCH {g('SQ_INSTS_BRANCH'):.3e}  VMEM {g('SQ_INSTS_VMEM'):.3e}  SMEM {g('SQ_INSTS_SMEM'):.3e}")
    print(f"  VALU lane utilisation (THREAD_CYCLES_VALU / (ACTIVE_INST_VALU*4*64)) {g('SQ_THREAD_CYCLES_VALU')/(g('SQ_ACTIVE_INST_VALU')*4*64):.3f}"
          f"   per-inst: {g('SQ_THREAD_CYCLES_VALU')/max(1,iv):.1f} thread-cycles")
    print(f"  LDS bank conflict / idx active {g('SQ_LDS_BANK_CONFLICT'):.3e} / {g('SQ_LDS_IDX_ACTIVE'):.3e}")
    print(f"  icache hits {g('SQC_ICACHE_HITS'):.3e} misses {g('SQC_ICACHE_MISSES'):.3e} ifetch {g('SQ_IFETCH'):.3e}")
    clk = g("GRBM_GUI_ACTIVE") / 8
    simds = 256 * 4
    print(f"  per-SIMD: VALU issue busy ~ {iv/simds*2/clk*100 if clk else float('nan'):.1f}% (2 cyc/inst), waves/SIMD avg {wc*4/clk/simds if clk else float('nan'):.2f}")
