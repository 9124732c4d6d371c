"""Generates the committed fixtures under tests/golden/ (run once in the build container).

- ml100k.npz: core/data/ml-100k/u.data of the reference (a data file its own tests load via
  core/base_test.go -> LoadDataFromBuiltIn("ml-100k") -> data.go:404-407), stored as
  (users int32, items int32, ratings int8) in file order.  Ratings parsed as integers exactly as
  the reference's loader does (data.go:302-304 strconv.Atoi; ML-100K ratings are integers 1-5).
- sim_kat.json: the known-answer vectors of core/sim_test.go:10-59 with their analytically exact
  values (Cosine = 14/sqrt(205), MSD = 1/10, Pearson = 0) next to the test's own expectation and
  tolerance (sim_test.go:8 epsilon 0.01).
"""
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/core/data/ml-100k/u.data"


def main():
    if os.path.exists(REF):
        raw = np.loadtxt(REF, dtype=np.int64, usecols=(0, 1, 2))
        np.savez_compressed(os.path.join(HERE, "ml100k.npz"), users=raw[:, 0].astype(np.int32),
                            items=raw[:, 1].astype(np.int32), ratings=raw[:, 2].astype(np.int8))
    else:
        print("reference data absent; keeping committed ml100k.npz", file=sys.stderr)
    a = {"ids": [1, 2, 3], "ratings": [4.0, 5.0, 6.0]}   # sim_test.go:11-15
    b = {"ids": [0, 1, 2], "ratings": [0.0, 1.0, 2.0]}   # sim_test.go:16-20
    kat = {
        "source": "core/sim_test.go:10-59",
        "epsilon": 0.01,
        "a": a,
        "b": b,
        "cases": [
            {"sim": "Cosine", "expect": 0.978, "exact": 14.0 / (math.sqrt(41.0) * math.sqrt(5.0)),
             "line": "sim_test.go:21-24"},
            {"sim": "MSD", "expect": 0.1, "exact": 1.0 / (18.0 / 2.0 + 1.0),
             "line": "sim_test.go:38-41"},
            {"sim": "Pearson", "expect": 0.0, "exact": 0.0, "line": "sim_test.go:55-58"},
        ],
    }
    with open(os.path.join(HERE, "sim_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)


if __name__ == "__main__":
    main()
