#!/usr/bin/env python3
"""Command line of tests/config4_fit.py: BASELINE configs[4] as a sharded fit at full size on ONE MI355X next to
the whole-set fit (see there for the options).  Reference: core/svd.go:92-130."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import config4_fit  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(config4_fit.run(config4_fit.parse())), flush=True)
