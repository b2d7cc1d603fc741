"""Helpers to compare decoded rows with the reference's Spark `toJSON` goldens.

Spark's JSON writer omits null struct fields; numbers are compared by value (decimal goldens
are printed at the schema scale; float/double goldens are Java's shortest round-trip text).
"""
from __future__ import annotations

import base64
import json
import os
from decimal import Decimal
from typing import Any, List

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def java_trim(s: str) -> str:
    """java.lang.String.trim: strip code points <= U+0020."""
    b, e = 0, len(s)
    while b < e and s[b] <= " ":
        b += 1
    while e > b and s[e - 1] <= " ":
        e -= 1
    return s[b:e]


def path(*p: str) -> str:
    return os.path.join(GOLDEN, *p)


def read(*p: str) -> bytes:
    with open(path(*p), "rb") as f:
        return f.read()


def load_lines(*p: str) -> List[Any]:
    with open(path(*p), encoding="utf-8") as f:
        return [json.loads(l, parse_float=Decimal) for l in f if l.strip()]


def _eq(a, g, where: str, na_fill: bool) -> List[str]:
    """a = our value, g = golden (json) value."""
    if isinstance(g, dict):
        if a is None:
            a = {}
        if not isinstance(a, dict):
            return [f"{where}: expected struct, got {a!r}"]
        errs = []
        keys_a = [k for k, v in a.items() if v is not None]
        if na_fill:
            keys_a = [k for k, v in a.items() if v is not None or _is_numeric_null_fill(k)]
        for k in g:
            errs += _eq(a.get(k), g[k], f"{where}.{k}", na_fill)
        extra = [k for k in a if k not in g and a[k] is not None and not isinstance(a[k], dict)]
        extra += [k for k in a if k not in g and isinstance(a[k], dict) and any(v is not None for v in a[k].values())]
        if extra:
            errs.append(f"{where}: unexpected non-null fields {extra[:5]}")
        return errs
    if isinstance(g, list):
        if not isinstance(a, list) or len(a) != len(g):
            return [f"{where}: array mismatch {a!r} vs {g!r}"[:300]]
        errs = []
        for i, (x, y) in enumerate(zip(a, g)):
            errs += _eq(x, y, f"{where}[{i}]", na_fill)
        return errs
    if g is None:
        return [] if a is None else [f"{where}: expected null, got {a!r}"]
    if a is None:
        if na_fill and isinstance(g, (int, Decimal)) and g == 0:
            return []
        return [f"{where}: expected {g!r}, got null"]
    if isinstance(g, str) and isinstance(a, (bytes, bytearray)):
        # Spark's JSON writer prints BinaryType values base64-encoded (debug=raw fields, test24b)
        got = base64.b64encode(bytes(a)).decode("ascii")
        return [] if got == g else [f"{where}: {a!r} ({got}) != {g!r}"]
    if isinstance(g, str):
        return [] if a == g else [f"{where}: {a!r} != {g!r}"]
    if isinstance(a, np.float32):
        return [] if np.float32(float(g)) == a else [f"{where}: float {a!r} != {g!r}"]
    if isinstance(a, (float, np.float64)):
        return [] if float(g) == float(a) else [f"{where}: double {a!r} != {g!r}"]
    if isinstance(a, (int, Decimal)):
        return [] if Decimal(a) == Decimal(g) else [f"{where}: {a!r} != {g!r}"]
    return [f"{where}: unsupported {a!r} vs {g!r}"]


def _is_numeric_null_fill(k):
    return False


def compare_rows(rows: List[dict], golden: List[Any], na_fill: bool = False) -> List[str]:
    errs = []
    if len(rows) < len(golden):
        errs.append(f"only {len(rows)} rows, golden has {len(golden)}")
    for i, (r, g) in enumerate(zip(rows, golden)):
        errs += _eq(r, g, f"row{i}", na_fill)
    return errs
