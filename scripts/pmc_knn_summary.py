"""Sums the SQ / GRBM counters of scripts/pmc_knn.sh over the K4 launches (knn_sims_mfma_kernel) and
derives the issue picture of the kernel: MFMA pipe busy (SQ_VALU_MFMA_BUSY_CYCLES over the SIMD
cycles of the active span, GRBM_GUI_ACTIVE being summed over the 8 XCDs), the parked / stalled /
issuing split of the wave cycles, and VALU instructions per MFMA."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    tot = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "knn_sims_mfma_kernel" in row.get("Kernel_Name", ""):
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
    c = dict(tot)
    der = {}
    if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        der["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
    if c.get("SQ_WAVE_CYCLES"):
        for k, n in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_frac"),
                     ("SQ_ACTIVE_INST_ANY", "active_inst_frac")):
            if k in c:
                der[n] = c[k] / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_INSTS_MFMA"):
        der["valu_per_mfma"] = c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"]
    if c.get("SQ_LDS_IDX_ACTIVE"):
        der["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
    print(json.dumps({"kernel": "knn_sims_mfma_kernel<Cosine, PIPE 2, eight waves> (14 group launches)",
                      "workload": "configs[3] ML-20M-shaped item Cosine (scripts/bench_configs.py --only 3)",
                      "counters": c, "derived": der,
                      "note": "GRBM_GUI_ACTIVE summed over 8 XCD entries; counters summed over the launches"},
                     indent=1))


if __name__ == "__main__":
    main()
