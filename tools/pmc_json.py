#!/usr/bin/env python3
"""rocprofv3 --pmc runs (FETCH_SIZE and WRITE_SIZE passes of tools/pmc.sh) -> profiles/pmc_<workload>.json, the
file bench.py reads for `roofline.traffic`: HBM-side bytes per launch of every kernel with the gfx950
correction of /opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide reads):
hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> B).

    python tools/pmc_json.py WORKLOAD BATCH DOMINANT_SUBSTRING OUT.json DIR [DIR ...]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)", "anon")
    return re.sub(r"\(.*", "", name)


def main(workload, batch, dominant, out, dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    per[(short(r["Kernel_Name"]), r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), cs in per.items():
                for c, v in cs.items():
                    acc[k][c].append(v)
    kernels = {}
    for k, cs in acc.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fs = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        ws = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        kernels[k] = {"dispatches": len(cs["FETCH_SIZE"]), "fetch_size_kib": round(fs, 2),
                      "write_size_kib": round(ws, 2), "hbm_bytes_per_launch": int(round((2 * fs + ws) * 1024))}
    dom = [k for k in kernels if dominant in k]
    doc = {"workload": workload, "batch": int(batch), "dominant_kernel": dom[0] if dom else None,
           "hbm_bytes_per_launch": kernels[dom[0]]["hbm_bytes_per_launch"] if dom else None,
           "correction": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B); gfx950 FETCH_SIZE halves wide reads",
           "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: v for k, v in doc.items() if k != "kernels"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])
