"""Per-dispatch durations of the last render in a rocprofv3 kernel trace: python tools/ktrace_summary.py gpurun_out/kq"""
import csv
import glob
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last k_generate starts the last render
last = max(i for i, r in enumerate(rows) if "k_generate" in r["Kernel_Name"])
tot = {}
for r in rows[last:]:
    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    tot[name] = tot.get(name, 0) + ms
    print("%-28s %8.3f ms  grid %s  vgpr %s" % (name[:28], ms, r["Grid_Size_X"], r["VGPR_Count"]))
print({k: round(v, 3) for k, v in tot.items()})
