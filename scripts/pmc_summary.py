"""Summarises rocprofv3 --pmc CSVs (FETCH_SIZE, WRITE_SIZE passes) for one kernel name, or for every
kernel (--all, the calibration run).
gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads 1/2 of the bytes of wide coalesced
streaming reads; it is reported raw and x2-corrected, WRITE_SIZE raw (exact for 16-B stores and
float atomics).  Units of both counters are KB.  scripts/experiments/pmc_calib.hip calibrates the
4-byte-per-lane loads and integer atomics of the SGD kernels."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def values(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                vals[row.get("Kernel_Name", "")].append(float(row["Counter_Value"]))
    return vals


def summary(name, f, w):
    out = {"kernel": name, "dispatches": [len(f), len(w)]}
    if f and w:
        fk, wk = sum(f) / len(f), sum(w) / len(w)
        out.update({"fetch_kb_raw": fk, "write_kb_raw": wk,
                    "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
                    "hbm_bytes_per_launch_uncorrected": (fk + wk) * 1024})
    return out


def main():
    if sys.argv[1] == "--all":
        d = sys.argv[2]
        f, w = values(d, "FETCH_SIZE"), values(d, "WRITE_SIZE")
        for name in sorted(set(f) | set(w)):
            print(json.dumps(summary(name.split("(")[0], f.get(name, []), w.get(name, []))))
        return
    d, kernel = sys.argv[1], sys.argv[2]
    f, w = values(d, "FETCH_SIZE"), values(d, "WRITE_SIZE")
    fv = [x for k, v in f.items() if kernel in k for x in v]
    wv = [x for k, v in w.items() if kernel in k for x in v]
    out = summary(kernel, fv, wv)
    out["note"] = ("FETCH_SIZE x2 per the gfx950 correction for wide reads; the 4-byte-per-lane sc1 "
                   "loads and integer atomics are calibrated by pmc_calib (profiles/*pmc_calib*)")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
