"""VALUBusy / VALUUtilization per dlsm kernel from a rocprofv3 --pmc CSV holding
SQ_ACTIVE_INST_VALU, SQ_THREAD_CYCLES_VALU, SQ_INSTS_VALU and GRBM_GUI_ACTIVE
(rocprofv3 -L's derived formulas: VALUBusy = 100*sum(SQ_ACTIVE_INST_VALU)/CU_NUM/
max(GRBM_GUI_ACTIVE); VALUUtilization = 100*sum(SQ_THREAD_CYCLES_VALU)/
(sum(SQ_ACTIVE_INST_VALU)*64)).  On gfx950 the CSV's GRBM_GUI_ACTIVE is summed
over the 8 XCDs (it reads 8 x 2.34 cycles per ns of kernel time), so VALUBusy
divides it by XCC = 8.  issue% = SQ_INSTS_VALU x 2 cycles / 1,024 SIMDs / kernel
cycles (one VALU instruction per SIMD every 2 cycles at 64 lanes).
   python scripts/valu_summary.py run_counter_collection.csv"""
import collections
import csv
import re
import statistics as st
import sys

CU = 256
XCC = 8
per = collections.defaultdict(lambda: collections.defaultdict(dict))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"dlsm::\(anonymous namespace\)::(\w+)(<[^(]*>)?", r["Kernel_Name"])
    if not m:
        continue
    name = m.group(1) + (m.group(2) or "")
    c, v = r["Counter_Name"], float(r["Counter_Value"])
    d = per[name][r["Dispatch_Id"]]
    d[c] = max(d.get(c, 0.0), v) if c.startswith("GRBM") else d.get(c, 0.0) + v
for name, disp in per.items():
    xs = [x for x in disp.values() if x.get("SQ_ACTIVE_INST_VALU") and x.get("GRBM_GUI_ACTIVE")]
    if not xs:
        continue
    busy = st.median(100 * x["SQ_ACTIVE_INST_VALU"] / CU / (x["GRBM_GUI_ACTIVE"] / XCC) for x in xs)
    issue = st.median(100 * x["SQ_INSTS_VALU"] * 2 / (CU * 4) / (x["GRBM_GUI_ACTIVE"] / XCC) for x in xs)
    util = st.median(100 * x["SQ_THREAD_CYCLES_VALU"] / (x["SQ_ACTIVE_INST_VALU"] * 64) for x in xs)
    insts = st.median(x["SQ_INSTS_VALU"] for x in xs)
    print(f"{name:34s} n={len(xs):3d}  VALUBusy={busy:5.1f}%  VALUUtilization={util:5.1f}%  "
          f"issue={issue:5.1f}%  SQ_INSTS_VALU={insts:.3g}  GRBM_GUI_ACTIVE={st.median(x['GRBM_GUI_ACTIVE'] for x in xs):.3g}")
