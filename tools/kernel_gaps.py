"""Launch gaps of the wavefront loop in a rocprofv3 kernel trace: for every k_shade dispatch, the time
from the end of the k_trace dispatch before it on the same queue to its own start (the host has to
know the shading grid by then), plus the count of runtime blit kernels (__amd_rocclr_copyBuffer) in
the trace. usage: python tools/kernel_gaps.py <rocprofv3 output dir> [label]"""
import csv
import glob
import json
import os
import sys


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Queue_Id" if rows and "Queue_Id" in rows[0] else "Stream_Id"
    blits = [r for r in rows if "copyBuffer" in r["Kernel_Name"]]
    last_trace = {}
    gaps = []
    for r in rows:
        name = r["Kernel_Name"]
        q = r.get(qkey)
        if "k_trace" in name:
            last_trace[q] = r
        elif "k_shade" in name and q in last_trace:
            t = last_trace.pop(q)
            gaps.append((int(r["Start_Timestamp"]) - int(t["End_Timestamp"])) / 1e3)  # us
    gaps.sort()
    out = {"label": sys.argv[2] if len(sys.argv) > 2 else os.path.basename(sys.argv[1].rstrip("/")),
           "trace_to_shade_gaps": len(gaps),
           "gap_us": ({"p50": round(gaps[len(gaps) // 2], 2), "p90": round(gaps[int(0.9 * (len(gaps) - 1))], 2),
                       "max": round(gaps[-1], 2), "mean": round(sum(gaps) / len(gaps), 2)} if gaps else None),
           "copyBuffer_dispatches": len(blits),
           "copyBuffer_ms_total": round(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in blits) / 1e6, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
