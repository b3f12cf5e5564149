#!/usr/bin/env python3
"""Turn scripts/pmc_traffic.sh output (gpurun_out/traffic) into the
profiles/pmc_<workload>.json files bench.py reads for roofline.traffic.

Calibration (tools/ubench/traffic_calib.hip, known byte counts, same run):
  FETCH_SIZE / true bytes for per-lane 16-B loads    -> fetch_factor
  WRITE_SIZE is taken as the true EA write traffic (it reads 1.0x for merged
  64-B segments and 2x for isolated 16-B pieces, which is real amplification)
HBM bytes per launch = median FETCH_SIZE / fetch_factor + median WRITE_SIZE,
over the crypt_kernel dispatches of the timed bench steps (the first dispatch,
the state pre-advance, is excluded).
"""
import csv
import collections
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SHAPES = {"cfg2": (4096, 1024), "cfg3": (65536, 256), "cfg4": (1024, 65536), "cfg5": (524288, 1024)}


def per_dispatch(path, name_filter):
    agg, names = collections.defaultdict(float), {}
    for r in csv.DictReader(open(path)):
        if name_filter in r["Kernel_Name"]:
            agg[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return [(names[d], agg[d]) for d in sorted(agg)]


def main(src="gpurun_out/traffic", tag=None):
    args = [a for a in sys.argv[1:] if not a.startswith("--round=")]
    tag = tag or next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--round=")), "r03")
    src = ROOT / src
    calib = per_dispatch(src / "calib_FETCH_SIZE" / "run_counter_collection.csv", "calib_load_lane")
    calib_bytes = 1 << 30
    fetch_factor = statistics.median(v * 1024 / calib_bytes for _, v in calib)
    for wl in args or ["cfg2", "cfg5"]:
        fr = per_dispatch(src / f"{wl}_FETCH_SIZE" / "run_counter_collection.csv", "zrc4::crypt_")[1:]
        wr = per_dispatch(src / f"{wl}_WRITE_SIZE" / "run_counter_collection.csv", "zrc4::crypt_")[1:]
        f, w = [v for _, v in fr], [v for _, v in wr]
        kname = collections.Counter(n.split("(")[0].replace("void ", "") for n, _ in fr).most_common(1)[0][0]
        S, L = SHAPES[wl.split("-")[0]]
        fb, wb = statistics.median(f) * 1024, statistics.median(w) * 1024
        out = {
            "kernel": kname, "workload": wl, "dispatches": len(f),
            "fetch_size_bytes_raw": fb, "write_size_bytes_raw": wb,
            "fetch_factor_per_lane_16B_loads": round(fetch_factor, 4),
            "read_bytes": round(fb / fetch_factor), "write_bytes": round(wb),
            "hbm_bytes_per_launch": round(fb / fetch_factor + wb),
            "algorithmic_bytes_per_launch": 2 * S * L + 516 * S,
            "source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) over "
                      f"bench.py --workload {wl.split('-')[0]} --ids {(wl.split('-') + ['range'])[1]} --steps 20; "
                      f"calibrated with tools/ubench/traffic_calib.hip",
            "round": tag,
        }
        out["traffic_over_algorithmic"] = round(out["hbm_bytes_per_launch"] / out["algorithmic_bytes_per_launch"], 3)
        (ROOT / "profiles" / f"pmc_{wl}.json").write_text(json.dumps(out, indent=1) + "\n")
        print(wl, out["hbm_bytes_per_launch"], out["traffic_over_algorithmic"])


if __name__ == "__main__":
    main()
