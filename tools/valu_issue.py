#!/usr/bin/env python3
"""VALU issue rate of k_trace and k_shade from a rocprofv3 --pmc counter-collection CSV that holds
SQ_INSTS_VALU and SQ_WAVES (tools/r04_pmc_shade.sh, pass 1): wave-instructions per second over the
kernels' own dispatch time, against the chip's wave64 VALU issue peak (a SIMD-32 issues one wave64
instruction per 2 cycles: 256 CUs x 4 SIMDs x 2.4 GHz / 2 = 1228.8 G/s,
/opt/skills/guides/MI355X_MICROARCH.md). python tools/valu_issue.py counters.csv out.json"""
import collections
import csv
import json
import sys

PEAK = 256 * 4 * 2.4e9 / 2 / 1e9  # G wave64 VALU instructions per second


def main(src, out):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(src)):
        n = r["Kernel_Name"]
        k = "k_shade<false, ...>" if n.startswith("void k_shade<false") else \
            "k_trace<false, false>" if n.startswith("void k_trace<false, false>") else None
        if k is None:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    res = {"peak_g_per_s": PEAK, "source": src, "kernels": {}}
    for k, c in agg.items():
        t = sum(dur[k].values()) / 1e9
        rate = c["SQ_INSTS_VALU"] / t / 1e9
        res["kernels"][k] = {"dispatches": len(dur[k]), "ms": round(t * 1e3, 3), "valu_wave_instr": c["SQ_INSTS_VALU"],
                             "valu_per_wave": round(c["SQ_INSTS_VALU"] / max(c["SQ_WAVES"], 1), 1),
                             "achieved_g_per_s": round(rate, 1), "frac": round(rate / PEAK, 4)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["kernels"], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
