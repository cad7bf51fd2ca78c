#!/usr/bin/env python3
"""Kernel overlap in a rocprofv3 kernel trace: per hardware queue, the busy time,
and how much of the GPU-busy time has kernels of two or more queues running at once.

  python tools/overlap.py <..._kernel_trace.csv> [--last-ms 300]
"""
import argparse
import csv
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--last-ms", type=float, default=0.0, help="only the last this many ms of the trace")
    a = p.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"].split("(")[0][:40])
          for r in rows]
    iv.sort()
    if a.last_ms:
        t_end = max(e for _, e, _, _ in iv)
        iv = [x for x in iv if x[0] >= t_end - a.last_ms * 1e6]
    ev = []
    for s, e, q, _ in iv:
        ev.append((s, 1, q))
        ev.append((e, -1, q))
    ev.sort()
    active = defaultdict(int)
    busy = multi = 0
    last = ev[0][0]
    for t, d, q in ev:
        nq = sum(1 for v in active.values() if v > 0)
        if nq >= 1:
            busy += t - last
        if nq >= 2:
            multi += t - last
        active[q] += d
        last = t
    per_q = defaultdict(float)
    per_k = defaultdict(lambda: [0, 0.0])
    for s, e, q, k in iv:
        per_q[q] += (e - s) / 1e6
        per_k[k][0] += 1
        per_k[k][1] += (e - s) / 1e6
    span = (iv[-1][1] - iv[0][0]) / 1e6
    print("span %.2f ms, GPU busy %.2f ms, two or more queues busy %.2f ms (%.1f %% of busy)"
          % (span, busy / 1e6, multi / 1e6, 100.0 * multi / max(busy, 1)))
    for q, t in sorted(per_q.items()):
        print("  queue %s: kernel time %.2f ms" % (q, t))
    for k, (n, t) in sorted(per_k.items(), key=lambda x: -x[1][1])[:8]:
        print("  %-40s x%-5d %.3f ms total, %.4f ms avg" % (k, n, t, t / n))


if __name__ == "__main__":
    main()
