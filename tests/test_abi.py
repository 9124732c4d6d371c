"""CPU tests of the C-ABI boundary: the library builds, loads and exports every symbol that
include/*.h declares.  No compute calls (no GPU here)."""
import ctypes
import glob
import os
import re

import pytest

import rsgpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(rs[a-z]*_\w+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(rsgpu.LIB_PATH)
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(rsgpu.HEADER_SYMBOLS) <= set(declared_symbols())


def test_version():
    assert rsgpu.lib().rs_version() >= 1


def test_library_is_gfx950_code_object():
    data = open(rsgpu.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_device_fails_loudly():
    if rsgpu.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(rsgpu.RsError):
        rsgpu.Context(0)


def test_null_arguments_rejected_without_device():
    L = rsgpu.lib()
    assert L.rs_svd_fit(None, None, None, None, None, None, None, None) == rsgpu.RS_ERR_INVALID
    assert b"NULL" in L.rs_last_error(None)
