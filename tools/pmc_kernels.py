#!/usr/bin/env python3
"""rocprofv3 --pmc passes (tools/gpu/pmc_r03.sh) -> one JSON of the hot kernels' counters per dispatch and the
derived figures north_star names: HBM bytes (2*FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md), L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS), LDS bank-conflict share,
wave-state split, effective clock (GRBM_GUI_ACTIVE / 8 / duration is not available here: cycles only), MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs), per CU-cycle).

    python tools/pmc_kernels.py WORKLOAD BATCH DOMINANT OUT.json DIR [DIR ...]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KEEP = ("ensemble_kernel", "feat_slot_kernel", "feat_bucket_lean_kernel", "feat_bucket_kernel", "feat_bucket_gather_kernel",
        "lstm_kernel4",
        "lstm_kernel", "split_walk_kernel", "split_sum_kernel", "split_bin_pair_kernel", "pipe_out_copy_kernel",
        "split_walk_pair_kernel", "split_sum_pair_blend_kernel",
        "ingest_json_kernel", "forest_kernel6", "blend_kernel", "route_")


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
                    g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
                    per[(short(r["Kernel_Name"]), g, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, g, _), cs in per.items():
                for c, v in cs.items():
                    acc[(k, g)][c].append(v)
    # a kernel launched with several grid sizes (the warm-history setup's large batches beside the timed steps'
    # 64 k ones) is reported per grid size: "name [grid G]"
    grids = defaultdict(set)
    for k, g in acc:
        grids[k].add(g)
    acc = {(k if len(grids[k]) == 1 else f"{k} [grid {g}]"): cs for (k, g), cs in acc.items()}
    kernels = {}
    for k, cs in acc.items():
        if not any(x in k for x in KEEP):
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "counters": {c: round(v, 1) for c, v in sorted(m.items())}}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            d["hbm_bytes_per_launch"] = int(round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024))
        if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0) > 0:
            d["l2_hit_rate"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_share"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
        if m.get("SQ_WAVE_CYCLES"):
            w = m["SQ_WAVE_CYCLES"]
            d["wave_state"] = {c[3:].lower(): round(m[c] / w, 4) for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
                                                                          "SQ_WAIT_ANY") if c in m}
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") and m.get("SQ_BUSY_CU_CYCLES"):
            d["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * m["SQ_BUSY_CU_CYCLES"]), 4)
        if m.get("SQ_INSTS_LDS") and m.get("SQ_INSTS_VALU"):
            d["lds_per_valu"] = round(m["SQ_INSTS_LDS"] / m["SQ_INSTS_VALU"], 4)
        kernels[k] = d
    dom = [k for k in kernels if dominant in k]
    doc = {"workload": workload, "batch": int(batch), "dominant_kernel": dom[0] if dom else None,
           "hbm_bytes_per_launch": kernels[dom[0]].get("hbm_bytes_per_launch") if dom else None,
           "correction": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B); gfx950 FETCH_SIZE halves wide reads",
           "collection": "rocprofv3 --pmc, one pass per counter group (tools/gpu/pmc_r03.sh); kernels serialised "
                         "by the counter collection (no pipeline overlap)",
           "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, d in kernels.items():
        print(k, {x: d[x] for x in d if x not in ("counters",)})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])
