"""Per-kernel mean of every PMC counter over the dispatches of rocprofv3 --pmc runs (tools/pmc.sh).

    python tools/pmc_summary.py DIR [DIR ...]    (each DIR holds a run_counter_collection.csv, at any depth)

Prints, per kernel (short name), dispatch count and the mean per dispatch of each counter, then the derived
ratios the forest / feature kernels are tuned on: LDS-array busy fraction, bank-conflict share, wave-state
split (active / issue-stalled / parked), and HBM bytes with the gfx950 FETCH_SIZE correction noted in
/opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide coalesced reads; the
raw value is printed, the correction is applied only in the 'fetch_x2' column)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name.replace("void ", "").replace("(anonymous namespace)", "anon"))
    return name.split("::")[-1]


def main(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    key = (short(r["Kernel_Name"]), r["Dispatch_Id"])
                    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), cs in per.items():
                for c, v in cs.items():
                    acc[k][c].append(v)
    for k in sorted(acc):
        cs = acc[k]
        n = max(len(v) for v in cs.values())
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}  (dispatches {n})")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.1f}")
        if "SQ_LDS_IDX_ACTIVE" in m and "SQ_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
            pass
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            w = m["SQ_WAVE_CYCLES"]
            parts = [f"{c[3:]} {m[c] / w:.3f}" for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                                        "SQ_WAIT_INST_LDS") if c in m]
            print("   wave-state fractions:", ", ".join(parts))
        if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            print(f"   bank-conflict share of LDS cycles: {m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "FETCH_SIZE" in m:
            print(f"   fetch_x2 (KB, gfx950 correction for wide reads): {2 * m['FETCH_SIZE']:.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
