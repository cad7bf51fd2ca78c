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
    if c.get("TCP_TCC_READ_REQ_sum"):
        print("   L1->L2 read latency %.0f cycles" % (c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"]))
    if c.get("TCP_TCC_WRITE_REQ_sum"):
        print("   L1->L2 write latency %.0f cycles" % (c["TCP_TCC_WRITE_REQ_LATENCY_sum"] / c["TCP_TCC_WRITE_REQ_sum"]))
    if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
        print("   VALU instructions per wave %.0f, VMEM rd %.1f wr %.1f per wave" % (
            c["SQ_INSTS_VALU"] / c["SQ_WAVES"], c.get("SQ_INSTS_VMEM_RD", 0) / c["SQ_WAVES"],
            c.get("SQ_INSTS_VMEM_WR", 0) / c["SQ_WAVES"]))
    if c.get("TCC_HIT_sum"):
        print("   L2 hit rate %.3f" % (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))
