"""Summarise rocprofv3 runs into profiles/: kernel-trace stats + FETCH_SIZE / WRITE_SIZE per launch.

gfx950 corrections: FETCH_SIZE (KiB) counts 64 B per L2->fabric read request. For a wide coalesced
stream that is half the bytes (MI355X_MICROARCH.md §HBM: x2). For k_trace's 64-B per-lane record
gathers it is exactly the requested bytes of the L2-missing records (profiles/r02_fetch_calibration.json,
tools/micro/roof.hip on a 1 GiB table): x1. So k_trace's reads are taken x1 (its per-ray queue/ray
stream reads, ~10 % of its fetches, are then under-counted by half) and every other kernel's x2.
WRITE_SIZE (KiB) is taken as-is.
"""
import csv, json, sys, collections

def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc

def main(fetch_csv, write_csv, stats_csv, out_json, dram_csv=None, config=None, spp=None):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    rq = per_kernel(dram_csv, "TCC_EA0_RDREQ_sum") if dram_csv else {}
    rd = per_kernel(dram_csv, "TCC_EA0_RDREQ_DRAM_sum") if dram_csv else {}
    stats = {r["Name"]: r for r in csv.DictReader(open(stats_csv))}
    out = {"note": "per-launch averages; FETCH_SIZE/WRITE_SIZE in KiB from rocprofv3 --pmc (separate passes); "
                   "read bytes: k_trace x1 (64-B gathers, profiles/r02_fetch_calibration.json), other kernels x2 "
                   "(gfx950 wide-stream under-count)", "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fk = sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wk = sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        st = stats.get(k, {})
        out["kernels"][k] = {"launches_pmc": len(f.get(k, [])), "fetch_kib_raw": round(fk, 1),
                             "read_bytes_corrected": round(fk * 1024 * (1 if "k_trace" in k else 2)), "write_bytes": round(wk * 1024),
                             "avg_ns_trace": float(st["AverageNs"]) if st else None,
                             "calls_trace": int(st["Calls"]) if st else None}
        if k in rq and sum(rq[k]) > 0:
            # share of L2 read requests that went to DRAM (the rest hit the Infinity Cache)
            out["kernels"][k]["dram_share_of_l2_read_requests"] = round(sum(rd.get(k, [0])) / sum(rq[k]), 4)
    if config:
        out["config"] = config
    if spp:
        out["spp"] = int(spp)
    # the traversal kernel of the bench (not the counting variant): k_trace<false, SMALL>, the one
    # with the most kernel-trace time (the small-scene variant on C2)
    ext = [k for k in out["kernels"] if k.startswith("void k_trace<false")]
    ext.sort(key=lambda k: -(out["kernels"][k]["avg_ns_trace"] or 0) * (out["kernels"][k]["calls_trace"] or 0))
    if ext:
        out["extend_kernel"] = ext[0]
        e = out["kernels"][ext[0]]
        out["extend_l2_fabric_bytes_per_launch"] = e["read_bytes_corrected"] + e["write_bytes"]
        share = e.get("dram_share_of_l2_read_requests")
        out["extend_hbm_bytes_per_launch"] = (round(e["read_bytes_corrected"] * share) + e["write_bytes"]
                                              if share is not None else e["read_bytes_corrected"] + e["write_bytes"])
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))

if __name__ == "__main__":
    main(*sys.argv[1:8])
