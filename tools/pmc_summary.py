"""Aggregate a rocprofv3 ``*_counter_collection.csv`` into per-kernel means.

Usage: python tools/pmc_summary.py <csv> [<csv> ...] > summary.json
Groups by (kernel name, grid size); for every counter reports the mean over
dispatches, plus derived ratios when the inputs are present.
"""

import csv
import json
import sys
from collections import defaultdict


def summarize(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p, newline="") as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "?")
                key = f"{name[:90]}|grid={row.get('Grid_Size', '?')}"
                acc[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for key, ctrs in acc.items():
        m = {c: sum(v) / len(v) for c, v in ctrs.items()}
        m["dispatches"] = max(len(v) for v in ctrs.values())
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            wc = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    m[c + "/WAVE_CYCLES"] = m[c] / wc
        if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
            m["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over 8 XCDs; MFMA busy is summed over all SIMDs (1024)
            m["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        out[key] = m
    return out


if __name__ == "__main__":
    json.dump(summarize(sys.argv[1:]), sys.stdout, indent=1, sort_keys=True)
    print()
