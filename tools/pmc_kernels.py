"""Aggregate rocprofv3 --pmc counter CSVs per kernel (sum over dispatches) and print derived ratios.
usage: python tools/pmc_kernels.py gpurun_out/sq1 gpurun_out/tcc ..."""
import csv
import glob
import os
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((d, r["Dispatch_Id"]))
for k, c in agg.items():
    if "k_trace" not in k and "k_shade" not in k:
        continue
    print("==", k, "dispatch-sets", len(disp[k]))
    for n in sorted(c):
        print("   %-24s %.4g" % (n, c[n]))
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if n in c:
                print("   %-24s %.3f of wave cycles" % (n, c[n] / w))
    if c.get("TCC_HIT_sum"):
        print("   L2 hit rate %.3f" % (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))
