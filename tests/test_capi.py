"""The C-ABI library loads and exports every symbol include/cobrix_hip.h declares, and the
ctypes mirror of every ABI struct matches the C layout (no GPU calls)."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

from cobrix_amd import native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "cobrix_hip.h")


def test_header_symbols_exported():
    hdr = open(HDR).read()
    declared = set(re.findall(r"\b(cbx_[a-z_0-9]+)\s*\(", hdr))
    assert set(N.EXPORTED_SYMBOLS) == declared
    lib = N.load()
    for s in declared:
        assert getattr(lib, s) is not None
    assert lib.cbx_abi_version() == N.ABI_VERSION
    assert int(re.search(r"#define CBX_ABI_VERSION (\d+)", hdr).group(1)) == N.ABI_VERSION


STRUCTS = {"cbx_field": N.CbxField, "cbx_array": N.CbxArray, "cbx_segment_map": N.CbxSegmentMap,
           "cbx_plan_options": N.CbxPlanOptions, "cbx_column": N.CbxColumn, "cbx_rdw_params": N.CbxRdwParams,
           "cbx_index_entry": N.CbxIndexEntry, "cbx_index_params": N.CbxIndexParams, "cbx_selection": N.CbxSelection,
           "cbx_hier_params": N.CbxHierParams, "cbx_walk_node": N.CbxWalkNode, "cbx_walk_array": N.CbxWalkArray,
           "cbx_walk_handler": N.CbxWalkHandler, "cbx_hier_dependee": N.CbxHierDependee,
           "cbx_hier_odo_array": N.CbxHierOdoArray, "cbx_hier_walk": N.CbxHierWalk}


def test_struct_layout_matches_header(tmp_path):
    """sizeof / offsetof of every ABI struct as a C compiler sees include/cobrix_hip.h."""
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "cobrix_hip.h"', "int main(void) {"]
    for cname, py in STRUCTS.items():
        src.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            src.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    try:
        r = subprocess.run(["gcc", "-I", os.path.dirname(HDR), "-o", str(exe), str(c)], capture_output=True, text=True)
    except OSError as e:  # pragma: no cover
        pytest.skip(f"no C compiler: {e}")
    # a ctypes field the C struct lacks is a compile error here: a mismatch, not a missing compiler
    assert r.returncode == 0, r.stderr[-2000:]
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, out):
        cname, what, val = line.split()
        py = STRUCTS[cname]
        got = ctypes.sizeof(py) if what == "sizeof" else getattr(py, what).offset
        assert got == int(val), f"{cname}.{what}: ctypes {got} != C {val}"
