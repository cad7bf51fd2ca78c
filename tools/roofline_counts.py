"""Per-config walk counts behind the roofline (SURVEY.md §8d asks for them committed per config):
box / triangle tests per ray of the reference BVH2 walk (algorithmic) and of the 4-wide walk, the
random record fetches per ray, and the ceiling row each config is priced against.

Usage: python tools/roofline_counts.py bench_line.json configs.jsonl ... > profiles/r02_roofline_counts.json
"""
import json
import sys


def main(paths):
    out = {}
    for p in paths:
        for line in open(p):
            line = line.strip()
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            r, a = d["roofline"], d["roofline"]["algorithmic"]
            key = d["config"]["workload"].split(":")[0]
            out[key] = {
                "workload": d["config"]["workload"],
                "triangles": d["config"]["triangles"],
                "reference_bvh2": {"box_tests_per_ray": a["box_tests_per_ray"], "tri_tests_per_ray": a["tri_tests_per_ray"],
                                   "shadow_box_tests_per_ray": a["shadow_box_tests_per_ray"],
                                   "shadow_tri_tests_per_ray": a["shadow_tri_tests_per_ray"],
                                   "bytes_per_ray": a["bytes_per_ray"], "bytes_per_shadow_ray": a["bytes_per_shadow_ray"]},
                "wide_walk": {"slot_tests_per_ray": r["walk_box_tests_per_ray"], "tri_tests_per_ray": r["walk_tri_tests_per_ray"],
                              "node_steps_per_ray": r["node_steps_per_ray"], "fetches_per_ray": r.get("fetches_per_ray"),
                              "tri_tail_loads_per_ray": r.get("tri_tail_loads_per_ray"),
                              "leafbox_tests_per_ray": r.get("leafbox_tests_per_ray")},
                "roofline": {"achieved": r["achieved"], "peak": r["peak"], "frac": r["frac"], "unit": r["unit"],
                             "ceiling": r["ceiling"]},
                "mrays_per_s": d["value"],
            }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1:])
