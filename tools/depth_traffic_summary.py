#!/usr/bin/env python3
"""Table of tools/depth_traffic.sh's output: per depth the HBM bytes of one
launch (FETCH_SIZE x 2 x 1 KiB, the gfx950 correction, + WRITE_SIZE x 1 KiB),
the rays by kind and the stack spills, and the bytes each depth step adds
per secondary ray it adds.

  python tools/depth_traffic_summary.py gpurun_out/s14/depth"""
import json
import os
import sys


def main():
    base = sys.argv[1]
    rows = []
    for name in sorted(os.listdir(base)):
        if not (name.startswith("d") and name.endswith("_pmc.json")):
            continue
        d = int(name[1:-len("_pmc.json")])
        p = json.load(open(os.path.join(base, name)))
        b = json.load(open(os.path.join(base, f"d{d}_bench.json")))
        per = p["per_render"]
        rd, wr = 2 * per["FETCH_SIZE"] * 1024, per["WRITE_SIZE"] * 1024
        rc = b["ray_counts"]
        rows.append(dict(depth=d, read_GB=round(rd / 1e9, 2), write_GB=round(wr / 1e9, 2),
                         kernel_ms=round(p["kernel_ns_mean"] / 1e6, 2), primary=rc["primary"], shadow=rc["shadow"],
                         refraction=rc["refraction"], reflection=rc["reflection"],
                         spills=b["work"]["stack_spills"]))
    rows.sort(key=lambda r: r["depth"])
    for a, b in zip(rows, rows[1:]):
        sec = (b["refraction"] + b["reflection"]) - (a["refraction"] + a["reflection"])
        rays = sum(b[k] for k in ("primary", "shadow", "refraction", "reflection")) - \
            sum(a[k] for k in ("primary", "shadow", "refraction", "reflection"))
        b["added_read_B_per_added_secondary"] = round((b["read_GB"] - a["read_GB"]) * 1e9 / max(sec, 1), 1)
        b["added_write_B_per_added_secondary"] = round((b["write_GB"] - a["write_GB"]) * 1e9 / max(sec, 1), 1)
        b["added_read_B_per_added_ray"] = round((b["read_GB"] - a["read_GB"]) * 1e9 / max(rays, 1), 1)
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
