"""CPU fuzz: the device field decoders (cbx_decode.h, executed on the host through the test
shim tests/native/libcbx_decode_host.so) against the oracle restatement, value by value.

This pins the GPU arithmetic (COMP-3 nibbles, binary widths, zoned overpunch/sign/dot rules,
IBM/IEEE floats, Spark HALF_UP/overflow conversion, string trimming + UTF-8) without a GPU.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from cobrix_amd import copybook as cbk
from cobrix_amd import native as N
from cobrix_amd.codepages import lut_for, utf8_lut
from cobrix_amd.plan import build_plan
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
SHIM = os.path.join(HERE, "native", "libcbx_decode_host.so")

FUZZ_COPYBOOK = """
       01  R.
           05  S1    PIC X(12).
           05  S2    PIC X(3).
           05  A1    PIC A(5).
           05  Z01   PIC 9(1).
           05  Z02   PIC 9(4).
           05  Z03   PIC S9(4).
           05  Z04   PIC 9(9).
           05  Z05   PIC S9(9).
           05  Z06   PIC 9(10).
           05  Z07   PIC S9(18).
           05  Z08   PIC 9(20).
           05  Z09   PIC S9(37).
           05  Z10   PIC 99V9.
           05  Z11   PIC S9(5)V99.
           05  Z12   PIC S9(13)V9(5).
           05  Z13   PIC 9(16)V9(10).
           05  Z14   PIC S9(3).99.
           05  Z15   PIC 9(4),9(2).
           05  Z16   PIC SPPP9(5).
           05  Z17   PIC S9(5)PPP.
           05  Z18   PIC +9(6)V99.
           05  Z19   PIC Z(6)VZZ-.
           05  Z20   PIC 9(6).99-.
           05  Z21   PIC S9(7) SIGN LEADING SEPARATE.
           05  Z22   PIC S9(5)V99 SIGN TRAILING SEPARATE.
           05  Z23   PIC SV9(7) SIGN LEADING.
           05  Z24   PIC Z(8)-.
           05  Z25   PIC 9(3)PP.
           05  Z26   PIC SVPP9(3).
           05  B01   PIC 9(1) COMP.
           05  B02   PIC S9(4) COMP.
           05  B03   PIC 9(4) COMP.
           05  B04   PIC 9(9) COMP.
           05  B05   PIC S9(9) COMP.
           05  B06   PIC 9(18) COMP.
           05  B07   PIC S9(18) COMP.
           05  B08   PIC 9(20) COMP.
           05  B09   PIC S9(38) COMP.
           05  B10   PIC S9(3)V99 COMP.
           05  B11   PIC 9(7)V99 COMP.
           05  B12   PIC S9(15)V9(3) COMP.
           05  B13   PIC 9(16)V99 COMP.
           05  B14   PIC SPPP9(5) COMP.
           05  B15   PIC S9(5)PPP COMP.
           05  B16   PIC S9(2) COMP-5.
           05  B17   PIC S9(20)V9(5) COMP.
           05  B18   PIC SPPP9 COMP.
           05  P01   PIC 9(1) COMP-3.
           05  P02   PIC S9(4) COMP-3.
           05  P03   PIC 9(9) COMP-3.
           05  P04   PIC S9(10) COMP-3.
           05  P05   PIC S9(18) COMP-3.
           05  P06   PIC 9(19) COMP-3.
           05  P07   PIC S9(20) COMP-3.
           05  P08   PIC S9(37) COMP-3.
           05  P09   PIC S9(13)V99 COMP-3.
           05  P10   PIC S9(3)V9(6) COMP-3.
           05  P11   PIC 9(2)V9(2) COMP-3.
           05  P12   PIC S9(18)V9(10) COMP-3.
           05  P13   PIC SV9(5) COMP-3.
           05  P14   PIC PPP9(5) COMP-3.
           05  P15   PIC SPP9(4) COMP-3.
           05  P16   PIC 9(5)PPP COMP-3.
           05  P17   PIC S9(38) COMP-3.
           05  F01   COMP-1.
           05  F02   COMP-2.
"""

ZONED_ALPHABET = np.array(list(range(0xF0, 0xFA)) * 6 + list(range(0xC0, 0xCA)) + list(range(0xD0, 0xDA))
                          + [0x40] * 8 + [0x00] * 2 + [0x4B, 0x6B, 0x60, 0x4E] * 2 + [0xC1, 0x81, 0x5B, 0xFA, 0xAB],
                          dtype=np.uint8)
STRING_ALPHABET = np.array([0x40] * 10 + [0x00, 0x05, 0x15, 0x41, 0x25, 0x0D] + list(range(0xC1, 0xCA)) +
                           list(range(0x81, 0x8A)) + list(range(0xF0, 0xFA)) + [0x4B, 0x6B, 0x5B, 0x9F, 0xFF, 0x74, 0xA1],
                           dtype=np.uint8)


def _shim():
    if not os.path.exists(SHIM):
        subprocess.run(["make", "-s", "-C", os.path.dirname(SHIM)], check=True)
    L = ctypes.CDLL(SHIM)
    P = ctypes.c_void_p
    L.cbxh_decode.argtypes = [P, P, ctypes.c_int, P, P, P, P, P]
    return L


def _random_bytes(rng, p: cbk.Primitive, n: int) -> bytes:
    d = p.dtype
    if isinstance(d, cbk.AlphaNumeric):
        return bytes(rng.choice(STRING_ALPHABET, n))
    if d.compact is None:
        if rng.random() < 0.5:
            # mostly well-formed: digits with optional sign/overpunch/dot/spaces
            b = bytearray(rng.choice(np.arange(0xF0, 0xFA, dtype=np.uint8), n))
            for _ in range(rng.integers(0, 3)):
                b[rng.integers(0, n)] = int(rng.choice(ZONED_ALPHABET))
            return bytes(b)
        return bytes(rng.choice(ZONED_ALPHABET, n))
    if d.compact == cbk.COMP3:
        digits = rng.integers(0, 10, 2 * n)
        if rng.random() < 0.1:
            digits[rng.integers(0, 2 * n)] = rng.integers(10, 16)
        sign = int(rng.choice([0xC, 0xD, 0xF, 0xC, 0xD, 0xA, 0xB, 0xE, 0x0, 0x5]))
        b = bytearray(n)
        for i in range(n):
            hi_n = int(digits[2 * i])
            lo_n = int(digits[2 * i + 1]) if i < n - 1 else sign
            b[i] = (hi_n << 4) | lo_n
        if rng.random() < 0.05:
            b = bytearray(rng.integers(0, 256, n, dtype=np.uint8))
        return bytes(b)
    if rng.random() < 0.2:
        return bytes([0] * (n - 1) + [int(rng.integers(0, 256))])
    return bytes(rng.integers(0, 256, n, dtype=np.uint8))


@pytest.mark.parametrize("fmt", ["IBM", "IEEE754", "IBM_LE"])
@pytest.mark.parametrize("code_page,trim", [("common", "both"), ("cp037", "both"), ("cp037_extended", "left"),
                                            ("cp875", "right"), ("common", "none")])
def test_field_decoders_match_oracle(fmt, code_page, trim):
    if fmt != "IBM" and (code_page, trim) != ("common", "both"):
        pytest.skip("float formats only vary float fields")
    cb = cbk.parse_copybook(FUZZ_COPYBOOK, floating_point_format=fmt, code_page=code_page, string_trimming=trim)
    plan = build_plan(cb)
    ast = O.OracleAst(cb)
    lut = np.array(utf8_lut(lut_for(code_page)), dtype=np.uint32)
    L = _shim()
    OL = O.lib()
    rng = np.random.default_rng(20261015)
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    sbuf = (ctypes.c_uint8 * 4096)()
    slen = ctypes.c_int32()
    heap = np.zeros(1 << 16, dtype=np.uint8)
    ev = np.zeros(1, dtype=O.EVENT_DTYPE)
    hl = ctypes.c_int64()
    mismatches = []
    n_checked = 0
    for p in O._iter_leaves(cb.ast):
        fi = plan.field_of_node[id(p)]
        cf = plan.fields[fi]
        node = ast.nodes[ast.node_of(p)]
        for _ in range(400):
            b = _random_bytes(rng, p, p.data_size)
            buf = np.frombuffer(b, dtype=np.uint8)
            n_avail = len(b)
            if cf.out_type in (N.O_STRING, N.O_BINARY) and rng.random() < 0.3:
                n_avail = int(rng.integers(0, len(b) + 1))   # record ends inside the string: truncated
            valid = L.cbxh_decode(ctypes.byref(cf), buf.ctypes.data, n_avail, lut.ctypes.data,
                                  ctypes.byref(lo), ctypes.byref(hi), sbuf, ctypes.byref(slen))
            assert valid != -1, f"{p.name}: width-specialised decoder disagrees with the byte loop on {b.hex()}"
            hl.value = 0
            rc = OL.ora_decode_field(ctypes.byref(node), ctypes.byref(ast.opts), buf.ctypes.data, n_avail,
                                     ev.ctypes.data, heap.ctypes.data, len(heap), ctypes.byref(hl))
            assert rc == 0
            e = ev[0]
            exp_valid = not e["isnull"]
            ok = exp_valid == bool(valid)
            if ok and exp_valid:
                if cf.out_type in (N.O_STRING, N.O_BINARY):
                    got = bytes(sbuf[: slen.value])
                    want = heap[int(e["lo"]): int(e["lo"]) + int(e["hi"])].tobytes()
                    ok = got == want
                elif cf.out_type == N.O_I32:
                    ok = np.int32(np.uint64(lo.value).astype(np.uint32).view(np.int32)) == np.int32(int(e["lo"]) & 0xFFFFFFFF if int(e["lo"]) >= 0 else int(e["lo"]))
                elif cf.out_type in (N.O_I64, N.O_DEC64):
                    ok = np.uint64(lo.value) == np.uint64(int(e["lo"]) & 0xFFFFFFFFFFFFFFFF)
                elif cf.out_type == N.O_DEC128:
                    ok = (lo.value == (int(e["lo"]) & 0xFFFFFFFFFFFFFFFF)) and (hi.value == (int(e["hi"]) & 0xFFFFFFFFFFFFFFFF))
                elif cf.out_type == N.O_F32:
                    ok = (lo.value & 0xFFFFFFFF) == (int(e["lo"]) & 0xFFFFFFFF)
                elif cf.out_type == N.O_F64:
                    ok = lo.value == (int(e["lo"]) & 0xFFFFFFFFFFFFFFFF)
            n_checked += 1
            if not ok:
                mismatches.append((p.name, b.hex(), bool(valid), lo.value, hi.value, exp_valid, int(e["lo"]), int(e["hi"])))
    assert n_checked > 20000
    assert not mismatches, f"{len(mismatches)} mismatches, first: {mismatches[:8]}"


# ASCII data (data_encoding=ascii): DISPLAY numbers go through decodeAsciiNumber + the Int / Long /
# BigNumber / BigDecimal wrappers (StringDecoders.scala:221-361), strings through decodeAsciiString,
# PIC N through decodeUtf16String (StringDecoders.scala:98-114) in either byte order.
ASCII_COPYBOOK = """
       01  R.
           05  S1    PIC X(10).
           05  N1    PIC N(1).
           05  N2    PIC N(5).
           05  N3    PIC N(12).
           05  A01   PIC 9(1).
           05  A02   PIC S9(4).
           05  A03   PIC 9(9).
           05  A04   PIC S9(9).
           05  A05   PIC S9(10).
           05  A06   PIC S9(18).
           05  A07   PIC 9(20).
           05  A08   PIC S9(30).
           05  A09   PIC 99V9.
           05  A10   PIC S9(5)V99.
           05  A11   PIC S9(13)V9(5).
           05  A12   PIC S9(20)V9(10).
           05  A13   PIC S9(3).99.
           05  A14   PIC 9(4),9(2).
           05  A15   PIC SPPP9(5).
           05  A16   PIC S9(5)PPP.
           05  A17   PIC S9(7) SIGN LEADING SEPARATE.
           05  A18   PIC S9(5)V99 SIGN TRAILING SEPARATE.
           05  A19   PIC 9(6).99-.
           05  A20   PIC S9(30)V9(8).
"""

ASCII_NUM_ALPHABET = np.frombuffer(b"0123456789" * 4 + b"   ++--..,,eE\x00\x09A#" + bytes([0x80, 0xFF, 0x1F]),
                                   dtype=np.uint8)
UTF16_UNITS = [0x20, 0x20, 0x09, 0x00, 0x41, 0x62, 0x7A, 0x30, 0xE9, 0xA0, 0x3A9, 0x20AC, 0x4E2D, 0xFEFF,
               0xFFFE, 0xFFFD, 0xD83D, 0xDE00, 0xD800, 0xDFFF, 0xDBFF, 0xDC00]


def _random_ascii_bytes(rng, p: cbk.Primitive, n: int, big_endian: bool) -> bytes:
    d = p.dtype
    if isinstance(d, cbk.AlphaNumeric):
        if d.enc == cbk.UTF16:
            units = rng.choice(UTF16_UNITS, (n + 1) // 2)
            b = b"".join(int(u).to_bytes(2, "big" if big_endian else "little") for u in units)[:n]
            return b
        return bytes(rng.integers(0, 256, n, dtype=np.uint8)) if rng.random() < 0.3 else \
            bytes(rng.choice(np.frombuffer(b"  \x00\x09abcXYZ019.-\x7f", dtype=np.uint8), n))
    if rng.random() < 0.5:
        # mostly well-formed: spaces, an optional sign anywhere, digits, an optional separator
        k = int(rng.integers(0, n + 1))
        body = bytearray(rng.choice(np.frombuffer(b"0123456789", dtype=np.uint8), k))
        if k and rng.random() < 0.3:
            body[int(rng.integers(0, k))] = int(rng.choice(np.frombuffer(b".,eE", dtype=np.uint8)))
        pad = n - k
        lead = int(rng.integers(0, pad + 1))
        b = bytearray(b" " * lead + bytes(body) + b" " * (pad - lead))
        if rng.random() < 0.5:
            b[int(rng.integers(0, n))] = int(rng.choice(np.frombuffer(b"+-", dtype=np.uint8)))
        return bytes(b)
    return bytes(rng.choice(ASCII_NUM_ALPHABET, n))


@pytest.mark.parametrize("big_endian,trim,charset", [(True, "both", ""), (False, "both", "US-ASCII"),
                                                     (True, "left", "ISO-8859-1"), (False, "right", "windows-1252"),
                                                     (True, "none", "cp1250")])
def test_ascii_and_utf16_decoders_match_oracle(big_endian, trim, charset):
    cb = cbk.parse_copybook(ASCII_COPYBOOK, data_encoding=cbk.ASCII, string_trimming=trim,
                            is_utf16_big_endian=big_endian, ascii_charset=charset)
    plan = build_plan(cb)
    ast = O.OracleAst(cb)
    lut = np.array([plan.options.lut[i] for i in range(256)], dtype=np.uint32)   # the plan's byte table
    L = _shim()
    OL = O.lib()
    rng = np.random.default_rng(7 + int(big_endian) + 2 * len(trim) + len(charset))
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    sbuf = (ctypes.c_uint8 * 4096)()
    slen = ctypes.c_int32()
    heap = np.zeros(1 << 16, dtype=np.uint8)
    ev = np.zeros(1, dtype=O.EVENT_DTYPE)
    hl = ctypes.c_int64()
    mismatches = []
    n_checked = n_valid = 0
    kinds = set()
    for p in O._iter_leaves(cb.ast):
        cf = plan.fields[plan.field_of_node[id(p)]]
        kinds.add(cf.kind)
        node = ast.nodes[ast.node_of(p)]
        for _ in range(600):
            b = _random_ascii_bytes(rng, p, p.data_size, big_endian)
            buf = np.frombuffer(b, dtype=np.uint8)
            n_avail = len(b)
            if cf.out_type == N.O_STRING and rng.random() < 0.3:
                n_avail = int(rng.integers(0, len(b) + 1))
            valid = L.cbxh_decode(ctypes.byref(cf), buf.ctypes.data, n_avail, lut.ctypes.data,
                                  ctypes.byref(lo), ctypes.byref(hi), sbuf, ctypes.byref(slen))
            assert valid != -1, f"{p.name}: fast path disagrees with the byte loop on {b.hex()}"
            hl.value = 0
            assert OL.ora_decode_field(ctypes.byref(node), ctypes.byref(ast.opts), buf.ctypes.data, n_avail,
                                       ev.ctypes.data, heap.ctypes.data, len(heap), ctypes.byref(hl)) == 0
            e = ev[0]
            exp_valid = not e["isnull"]
            ok = exp_valid == bool(valid)
            if ok and exp_valid:
                n_valid += 1
                if cf.out_type == N.O_STRING:
                    ok = bytes(sbuf[: slen.value]) == heap[int(e["lo"]): int(e["lo"]) + int(e["hi"])].tobytes()
                else:
                    mask = 0xFFFFFFFF if cf.out_type == N.O_I32 else 0xFFFFFFFFFFFFFFFF
                    ok = (lo.value & mask) == (int(e["lo"]) & mask)
                    if cf.out_type == N.O_DEC128:
                        ok &= hi.value == (int(e["hi"]) & 0xFFFFFFFFFFFFFFFF)
            n_checked += 1
            if not ok:
                mismatches.append((p.name, b.hex(), n_avail, bool(valid), lo.value, hi.value, exp_valid,
                                   int(e["lo"]), int(e["hi"])))
    assert {N.K_ASCII_NUM, N.K_STRING_ASCII if charset in ("", "US-ASCII") else N.K_STRING,
            N.K_UTF16_BE if big_endian else N.K_UTF16_LE} <= kinds
    assert n_valid > n_checked // 4
    assert not mismatches, f"{len(mismatches)} mismatches, first: {mismatches[:8]}"


def _decode_one(pic: str, raw: bytes, big_endian: bool = True):
    """One ASCII-file field `05 F PIC <pic>` of exactly len(raw) bytes through the device decoders."""
    cb = cbk.parse_copybook(f"       01  R.\n           05  F   PIC {pic}.\n", data_encoding=cbk.ASCII,
                            is_utf16_big_endian=big_endian)
    plan = build_plan(cb)
    f = plan.fields[0]
    assert f.size == len(raw), (pic, f.size, raw)
    L = _shim()
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    sbuf = (ctypes.c_uint8 * 256)()
    slen = ctypes.c_int32()
    buf = np.frombuffer(raw, dtype=np.uint8)
    v = L.cbxh_decode(ctypes.byref(f), buf.ctypes.data, len(buf), None, ctypes.byref(lo), ctypes.byref(hi), sbuf,
                      ctypes.byref(slen))
    assert v != -1
    if not v:
        return None
    if f.out_type == N.O_STRING:
        return bytes(sbuf[: slen.value]).decode("utf-8")
    x = (hi.value << 64) | lo.value
    return x - (1 << 128) if x >> 127 else x


def test_ascii_number_and_utf16_known_answers():
    """Literals of StringDecodersSpec.scala:104-160, 237-275, 297-421 and Test23NationalTypeSpec.scala:36-60
    (decimals as unscaled values at the Spark schema scale)."""
    d = _decode_one
    # decodeAsciiInt (StringDecodersSpec.scala:297-322)
    for raw, want in [(b"+100", 100), (b"100+", 100), (b"-100", -100), (b"100-", -100)]:
        assert d("S9(4)", raw) == want
    for raw, want in [(b"+100", 100), (b"100+", 100), (b"-100", None), (b"100-", None)]:
        assert d("9(4)", raw) == want
    assert d("9(6)", b"+100,0") is None and d("S9(7)", b"100.00+") is None
    assert d("S9(8)", b"-100,000") is None and d("S9(8)", b"100.000-") is None
    assert d("9(9)", b"+10000000") == 10 ** 7
    assert d("S9(3)", b"AAA") is None
    # decodeAsciiLong (StringDecodersSpec.scala:353-377)
    for raw, want in [(b"+1000000000000000", 10 ** 15), (b"1000000000000000+", 10 ** 15),
                      (b"-1000000000000000", -10 ** 15), (b"1000000000000000-", -10 ** 15)]:
        assert d("S9(17)", raw) == want
    assert d("9(17)", b"-1000000000000000") is None
    assert d("S9(18)", b"+100000000000000,0") is None
    # decodeAsciiBigNumber with scale / scale factor (StringDecodersSpec.scala:400-421)
    assert d("S9(5)", b"+1000") == 1000
    assert d("S9(4)V9", b"+1000") == 1000            # 100.0 at scale 1
    assert d("S9(2)V9(3)", b"+1000") == 1000         # 1.000
    assert d("S9V9(4)", b"+1000") == 1000            # "+.1000" = 0.1000
    assert d("SV9(5)", b"+1000") is None             # "0.+1000"
    assert d("SP9(5)", b"+1000") == 10000            # 0.01000 -> unscaled at Spark scale 6
    # UTF-16 national strings (Test23NationalTypeSpec.scala:36-60, StringDecodersSpec.scala:104-160)
    assert d("N(3)", bytes([0x00, 0x31, 0x00, 0x32, 0x00, 0x33])) == "123"
    assert d("N(3)", bytes([0x61, 0x00, 0x62, 0x00, 0x63, 0x00]), big_endian=False) == "abc"
    assert d("N(6)", "  \t Ωx".encode("utf-16-be")) == "Ωx"
    assert d("N(2)", "\U0001F600".encode("utf-16-be")) == "\U0001F600"    # surrogate pair -> 4-byte UTF-8
    assert d("N(2)", bytes([0xD8, 0x3D, 0x00, 0x41])) == "\ufffd"          # malformed(4): ONE U+FFFD
    assert d("N(2)", bytes([0xFF, 0xFE, 0xDC, 0x00])) == "\ufffd\ufffd"    # U+FFFE, lone low surrogate
