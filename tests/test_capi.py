"""The C-ABI library loads and exports every symbol include/cobrix_hip.h declares (no GPU calls)."""
from __future__ import annotations

import ctypes
import os
import re

from cobrix_amd import native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "cobrix_hip.h")).read()
    declared = set(re.findall(r"\b(cbx_[a-z_0-9]+)\s*\(", hdr))
    assert set(N.EXPORTED_SYMBOLS) == declared
    lib = N.load()
    for s in declared:
        assert getattr(lib, s) is not None
    assert lib.cbx_abi_version() == 1


def test_struct_layout_matches_header():
    # sizes of the ABI structs as compiled into the library's consumers
    assert ctypes.sizeof(N.CbxField) == 4 * (12 + 3 * N.CBX_MAX_DIMS + 2)
    assert ctypes.sizeof(N.CbxArray) == 32
    assert ctypes.sizeof(N.CbxColumn) == 48
