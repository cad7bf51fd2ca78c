"""Summarise a rocprofv3 kernel-trace CSV: per-kernel busy time, the gaps between kernels, and how
much kernels on different queues overlap (tools/overlap_trace.sh).

Usage: python tools/timeline.py kt_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")[:28]


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"])))
    rows.sort()
    # only the render kernels (drop torch / copy kernels before the first k_generate)
    first = next((i for i, r in enumerate(rows) if r[3].startswith("k_generate")), 0)
    rows = rows[first:]
    if not rows:
        print("no kernels")
        return
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    span = (t1 - t0) / 1e6
    # union of busy intervals and pairwise overlap between queues
    busy = 0
    cur_s, cur_e = rows[0][0], rows[0][1]
    for s, e, _, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    overlap = 0
    for i, (s, e, q, _) in enumerate(rows):
        for s2, e2, q2, _ in rows[i + 1:]:
            if s2 >= e:
                break
            if q2 != q:
                overlap += min(e, e2) - s2
    per = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, _, n in rows:
        per[n] += (e - s) / 1e6
        cnt[n] += 1
    queues = sorted(set(r[2] for r in rows))
    print(f"span {span:.2f} ms, kernels busy (union) {busy / 1e6:.2f} ms, idle {span - busy / 1e6:.2f} ms, "
          f"cross-queue overlap {overlap / 1e6:.2f} ms, queues {queues}")
    for n in sorted(per, key=lambda k: -per[k]):
        print(f"  {n:28s} {cnt[n]:4d} launches {per[n]:9.2f} ms")
    # first step's sequence (up to the second k_generate on the first queue)
    print("  sequence (start offset, duration, queue):")
    shown = 0
    for s, e, q, n in rows:
        print(f"    {(s - t0) / 1e3:9.1f} us {(e - s) / 1e3:8.1f} us  q{q} {n}")
        shown += 1
        if shown >= 40:
            break


if __name__ == "__main__":
    main(sys.argv[1])
