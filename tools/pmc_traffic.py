#!/usr/bin/env python3
"""profiles/pmc_traffic.json from committed PMC summaries (tools/pmc_summary.py):

  python tools/pmc_traffic.py C3=profiles/r04/final_C3_pmc.json C4=... C5=...

One entry per config: HBM bytes per launch (gfx950-corrected FETCH_SIZE reads
+ WRITE_SIZE writes), the L2 hit rate and the sha of the librt_hip.so the
passes ran -- bench.py reports the traffic only for that library."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METHOD = ("rocprofv3 --kernel-trace --pmc, one counter group per pass (tools/gpu_session.sh pmc step, bench.py "
          "--inflight 1 --steps 1 --warmup 0 --count-render off: 2 renders of the kernel without counters per pass, RENDERS=2); read = 2 x FETCH_SIZE x 1024 "
          "(gfx950 correction, MI355X_MICROARCH.md HBM), write = WRITE_SIZE x 1024")


def main():
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        out = json.load(open(path))
    except (OSError, ValueError):
        out = {}
    for a in sys.argv[1:]:
        cfg, src = a.split("=", 1)
        j = json.load(open(os.path.join(ROOT, src)))
        d = j["derived"]
        rd, wr = d["hbm_read_bytes_corrected"], d["hbm_write_bytes"]
        out[cfg] = {"hbm_bytes_per_launch": rd + wr, "read_bytes": rd, "write_bytes": wr,
                    "l2_hit_rate": round(d.get("l2_hit_rate", float("nan")), 4), "method": METHOD,
                    "source": src, "lib_sha16": j.get("lib_sha16")}
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
