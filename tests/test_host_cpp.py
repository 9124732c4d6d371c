"""The C++ mirror of the Go core API (recommend-sys_amd/host) run through its own test binary, which
restates the reference's sim_test.go / base_test.go / eval_test.go over the C-ABI.  The ML-100K
fixture is written back to u.data's tab-separated layout for core::LoadDataFromFile."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

BIN = os.path.join(REPO, "recommend-sys_amd", "host", "tests", "core_test")


@pytest.fixture(scope="module")
def udata(tmp_path_factory, ml100k):
    from rsgpu import _build
    _build.build_host()
    u, i, r = ml100k
    p = tmp_path_factory.mktemp("ml100k") / "u.data"
    lines = [f"{a}\t{b}\t{int(c)}\t0" for a, b, c in zip(u, i, r)]
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def _run(args, timeout):
    res = subprocess.run([BIN] + args, capture_output=True, text=True, timeout=timeout)
    assert res.returncode == 0, res.stdout + res.stderr
    return res.stdout


def test_host_mirror_cpu(udata):
    out = _run(["--cpu-only", udata], 120)
    assert "7/7 passed" in out, out


@pytest.mark.gpu
def test_host_mirror_reference_tests(udata):
    out = _run([udata], 900)
    print(out)
    assert "FAIL" not in out
