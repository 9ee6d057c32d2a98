"""Summarise scripts/r5_pmc_first.sh output: per tick-kernel launch, SQ counters per wave and the
issue / wait split (diagnostic). Usage: pmc_first_summary.py DIR"""
import glob
import sqlite3
import sys

for wl in ("c2_init", "c3", "c4_n9"):
    vals = {}
    for p in ("p1", "p2"):
        for f in glob.glob(f"{sys.argv[1]}/{wl}_{p}/*.db"):
            db = sqlite3.connect(f)
            cols = [r[1] for r in db.execute("pragma table_info(counters_collection)")]
            for r in db.execute("select * from counters_collection"):
                d = dict(zip(cols, r))
                if "tick_kernel" in str(d["kernel_name"]):
                    vals[d["counter_name"]] = vals.get(d["counter_name"], 0) + d["value"]
    if not vals:
        continue
    wc = vals["SQ_WAVE_CYCLES"]
    print(f"{wl}: waves {vals['SQ_WAVES']:.0f}  VALU {vals['SQ_INSTS_VALU']:.3g} SALU "
          f"{vals['SQ_INSTS_SALU']:.3g} LDS {vals.get('SQ_INSTS_LDS', 0):.3g} VMEM_RD "
          f"{vals['SQ_INSTS_VMEM_RD']:.3g} WR {vals.get('SQ_INSTS_VMEM_WR', 0):.3g} BR "
          f"{vals.get('SQ_INSTS_BRANCH', 0):.3g}")
    print(f"   active {vals['SQ_ACTIVE_INST_ANY'] / wc:.2f} wait {vals['SQ_WAIT_ANY'] / wc:.2f} "
          f"wait_inst {vals['SQ_WAIT_INST_ANY'] / wc:.2f}  lds_conflict/lds "
          f"{vals.get('SQ_LDS_BANK_CONFLICT', 0) / max(vals.get('SQ_INSTS_LDS', 1), 1):.2f}  "
          f"gui_active {vals.get('GRBM_GUI_ACTIVE', 0):.3g}")
