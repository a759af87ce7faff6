#!/usr/bin/env python3
"""Clock and MFMA-pipe busy per kernel from one rocprofv3 --pmc pass of
GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA (tools/pmc_clock.sh's
method, for any command).  Usage: pmc_clock_summary.py <rocprof out dir> <json out>

clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; busy = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs
x cycles).  One record per kernel name (averaged over its dispatches).
"""
import collections
import csv
import glob
import json
import sys

d, out = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/*/run_counter_collection.csv") + glob.glob(d + "/run_counter_collection.csv")
per = collections.defaultdict(lambda: collections.defaultdict(dict))   # kernel -> dispatch -> ctr
dur = collections.defaultdict(dict)
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"].split("(")[0]
    disp = r.get("Dispatch_Id") or r.get("Correlation_Id") or r["Start_Timestamp"]
    per[k][disp][r["Counter_Name"]] = per[k][disp].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur[k][disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
res = {}
for k, ds in per.items():
    n = len(ds)
    t = sum(dur[k].values()) / n
    g = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in ds.values()) / n
    m = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for v in ds.values()) / n
    mi = sum(v.get("SQ_INSTS_MFMA", 0) for v in ds.values()) / n
    clk = g / 8 / t if t > 0 else 0.0
    busy = m / (256 * 4 * clk * t) if clk > 0 else 0.0
    res[k] = {"dispatches": n, "clock_ghz": clk / 1e9, "mfma_busy": busy,
              "dur_ms_under_pmc": t * 1e3, "mfma_insts": mi,
              "note": "clock = GRBM_GUI_ACTIVE / 8 XCDs / duration; busy = "
                      "SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x cycles)"}
    print(f"{k[:60]:60s} n={n:3d} dur {t*1e3:.3f} ms clock {clk/1e9:.2f} GHz MFMA busy {busy:.1%}")
json.dump(res, open(out, "w"), indent=1)
