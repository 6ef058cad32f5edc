#!/usr/bin/env python3
"""Summarise the PMC passes of tools/pmc_bench.sh into profiles/pmc_<workload>.json.

Per kernel: mean FETCH_SIZE / WRITE_SIZE (rocprofv3 reports KiB per dispatch) and the L2 hit rate.
hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (bytes): MI355X_MICROARCH.md "HBM [CDNA4]" —
on gfx950 FETCH_SIZE counts 64 B per 128-B memory request, i.e. half the bytes read.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def load(prefix, counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{prefix}.p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    prefix, wl = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    fetch, write = load(prefix, "FETCH_SIZE"), load(prefix, "WRITE_SIZE")
    hit, miss = load(prefix, "TCC_HIT_sum"), load(prefix, "TCC_MISS_sum")
    kernels = {}
    for k in fetch:
        short = k.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [0])))
        h, m = sum(hit.get(k, [0])), sum(miss.get(k, [0]))
        kernels[short] = {"dispatches": len(fetch[k]), "fetch_size_kib": round(f, 2), "write_size_kib": round(w, 2),
                          "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                          "l2_hit_rate": round(h / (h + m), 4) if h + m else None}
    forest = [k for k in kernels if "forest_kernel" in k and "double" not in k]
    dom = max(forest, key=lambda k: kernels[k]["dispatches"]) if forest else None
    out = {"workload": wl, "batch": batch, "dominant_kernel": dom,
           "hbm_bytes_per_launch": kernels[dom]["hbm_bytes_per_launch"] if dom else None,
           "correction": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B); gfx950 FETCH_SIZE halves wide reads",
           "kernels": kernels}
    p = REPO / "profiles" / f"pmc_{wl}.json"
    p.write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
