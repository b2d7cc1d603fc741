"""The reference's decoder unit-test literals (CPT = cobol-parser/src/test/scala/za/co/absa/cobrix/cobol/):

  * FloatingPointDecodersSpec.scala:31-102   IBM / IEEE-754, single / double, big / little endian
  * BinaryDecoderSpec.scala:46-233           COMP-3 integral / decimal / malformed, EBCDIC numbers,
                                             binary integers and binary decimals of 1-8 bytes
  * StringDecodersSpec.scala:44-296          EBCDIC strings and trims, HEX / RAW, zoned numbers
                                             (signs, overpunch A..R { }, comma decimals, Int / Long /
                                             BigNumber scale and scale factor / BigDecimal)
  * MalformedValuesSpec.scala:25-164         out-of-range binaries, malformed decimals, unsigned
                                             negatives

Every literal goes through BOTH the C oracle (the restated Scala decoders) and the device decoder
code of the HIP library compiled for the host (tests/native/decode_host.cpp, the exact functions
the kernels run): the two must agree bit for bit, and the value must equal the spec's literal
(floats within the spec's own tolerance; decimals numerically, as Scala's BigDecimal == compares).

Each field is a one-field copybook whose PIC selects the decoder the spec calls (DecoderSelector);
where the spec calls a decoder with a byte count no PIC produces (e.g. 3-byte binaries), the
field's size is overridden.  Literals outside Spark's decimal(38) range (BinaryDecoderSpec's
18-byte binaries, StringDecodersSpec's 52-digit BigDecimal) have no Spark column type and are
not on the GPU path (the plan rejects precision > 38).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from decimal import Decimal

import numpy as np
import pytest

from cobrix_amd import copybook as cbk
from cobrix_amd import native as N
from cobrix_amd.codepages import lut_for, utf8_lut
from cobrix_amd.plan import build_plan
from cobrix_amd.schema import spark_type
from oracle import oracle as O

LITERALS = []   # (clause, raw, lit kwargs) of every literal checked here, replayed on the GPU
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "tests", "native", "libcbx_decode_host.so")

_COMMON = lut_for("common")
# CPT/testutils/EbcdicEncoder.scala:21-54: the first byte the common code page maps to the
# character, else 0x40 (so ' ' -> 0x00, the first unmapped byte)
_TO_EBCDIC = [next((i for i, c in enumerate(_COMMON) if c == code), 0x40) for code in range(256)]


def to_ebcdic(s: str) -> bytes:
    return bytes(_TO_EBCDIC[ord(ch) & 0xFF] for ch in s)


def _shim():
    if not os.path.exists(SHIM):
        subprocess.run(["make", "-s", "-C", os.path.dirname(SHIM)], check=True)
    L = ctypes.CDLL(SHIM)
    P = ctypes.c_void_p
    L.cbxh_decode.argtypes = [P, P, ctypes.c_int, P, P, P, P, P]
    return L


def lit_copybook(clause: str, raw: bytes, *, size: int = None, enc: str = cbk.EBCDIC, enc_override: str = None,
                 as_decimal: bool = False, **kw):
    """The one-field copybook `05 F <clause>.` a literal decodes through (size / usage overrides applied)."""
    comp9 = clause.endswith(" COMP-9")   # little-endian binary: no copybook word, an AST usage only
    if comp9:
        clause = clause[: -len("-9")]
    body = clause if clause.startswith("COMP") else f"PIC {clause}"
    cb = cbk.parse_copybook(f"       01  R.\n           05  F   {body}.\n", data_encoding=enc, **kw)
    p = cb.ast.children[0].children[0]
    if enc_override is not None:
        p.dtype.enc = enc_override
    if as_decimal and isinstance(p.dtype, cbk.Integral):
        # a scale-0 Decimal: the generic decodeBinaryNumber path (BinaryUtils.scala:245-276) the spec
        # calls, which a copybook only reaches for scaled binaries (DecoderSelector.scala:139-147)
        d = p.dtype
        p.dtype = cbk.Decimal(d.pic, 0, d.precision, 0, False, d.sign_position, d.is_sign_separate, d.compact, d.enc)
    if comp9:
        p.dtype.compact = cbk.COMP9
        p.data_size = p.actual_size = cbk.get_bytes_count(cbk.COMP9, p.dtype.precision,
                                                          p.dtype.sign_position is not None, False, False)
    if size is not None:
        p.data_size = p.actual_size = size
    assert p.data_size == len(raw), (clause, p.data_size, raw)
    return cb, p


def lit(clause: str, raw: bytes, **kw):
    """Decode `raw` as the one field of `05 F <clause>.` through the oracle and the device code;
    returns the value (None for null)."""
    cb, p = lit_copybook(clause, raw, **kw)
    # oracle
    ast = O.OracleAst(cb)
    node = ast.nodes[ast.node_of(p)]
    buf = np.frombuffer(raw, dtype=np.uint8) if raw else np.zeros(1, np.uint8)
    ev = np.zeros(1, dtype=O.EVENT_DTYPE)
    heap = np.zeros(4096, dtype=np.uint8)
    hl = ctypes.c_int64(0)
    assert O.lib().ora_decode_field(ctypes.byref(node), ctypes.byref(ast.opts), buf.ctypes.data, len(raw),
                                    ev.ctypes.data, heap.ctypes.data, len(heap), ctypes.byref(hl)) == 0
    e = ev[0]
    # device decoder code (host build)
    plan = build_plan(cb)
    f = plan.fields[0]
    lut = np.array(utf8_lut(lut_for(cb.code_page)), dtype=np.uint32)
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    sbuf = (ctypes.c_uint8 * 4096)()
    slen = ctypes.c_int32()
    valid = _shim().cbxh_decode(ctypes.byref(f), buf.ctypes.data, len(raw), lut.ctypes.data, ctypes.byref(lo),
                                ctypes.byref(hi), sbuf, ctypes.byref(slen))
    assert valid != -1, "width-specialised decoder disagrees with its byte loop"
    assert bool(valid) == (not e["isnull"]), (clause, raw.hex(), bool(valid), e)
    if not valid:
        return None
    st = spark_type(p)
    if f.out_type in (N.O_STRING, N.O_BINARY):
        got = bytes(sbuf[: slen.value])
        assert got == heap[int(e["lo"]): int(e["lo"]) + int(e["hi"])].tobytes()
        return got.decode("utf-8") if f.out_type == N.O_STRING else got
    if f.out_type == N.O_F32:
        assert (lo.value & 0xFFFFFFFF) == (int(e["lo"]) & 0xFFFFFFFF)
        return float(np.uint32(lo.value & 0xFFFFFFFF).view(np.float32))
    if f.out_type == N.O_F64:
        assert lo.value == (int(e["lo"]) & 0xFFFFFFFFFFFFFFFF)
        return float(np.uint64(lo.value).view(np.float64))
    mask = 0xFFFFFFFF if f.out_type == N.O_I32 else 0xFFFFFFFFFFFFFFFF
    assert (lo.value & mask) == (int(e["lo"]) & mask)
    if f.out_type == N.O_DEC128:
        assert hi.value == (int(e["hi"]) & 0xFFFFFFFFFFFFFFFF)
    x = (hi.value << 64) | lo.value if f.out_type == N.O_DEC128 else lo.value & mask
    bits = 128 if f.out_type == N.O_DEC128 else (32 if f.out_type == N.O_I32 else 64)
    if x >> (bits - 1):
        x -= 1 << bits
    if f.out_type in (N.O_DEC64, N.O_DEC128):
        return Decimal(x).scaleb(-st[2])
    return x


# ---------------------------------------------------------------- FloatingPointDecodersSpec.scala

def _feq(a, b, tol):
    return a is not None and abs(a - b) < tol


@pytest.mark.parametrize("fmt,clause,raw,want,tol", [
    ("IBM", "COMP-1", "43142EFC", 5.045883, 1e-5),                 # :31-36 (the exponent-mask behaviour)
    ("IBM", "COMP-2", "43142EFCCAF709B7", 322.936717, 1e-10),      # :38-44
    ("IBM", "COMP-2", "00000000CAF709B7", 4.08114837e-85, 1e-10),  # :46-51
    ("IBM_LE", "COMP-1", "FC2E1443", 5.045883, 1e-5),              # :54-59
    ("IBM_LE", "COMP-2", "B709F7CAFC2E1443", 322.936717, 1e-10),   # :62-68
    ("IEEE754", "COMP-1", "40490FDA", 3.1415925, 1e-5),            # :71-75
    ("IEEE754", "COMP-2", "400921FB54442EEA", 3.14159265359, 1e-10),   # :78-84
    ("IEEE754_LE", "COMP-1", "DA0F4940", 3.1415925, 1e-5),         # :87-91
    ("IEEE754_LE", "COMP-2", "EA2E4454FB210940", 3.14159265359, 1e-10),  # :94-100
])
def test_floating_point_literals(fmt, clause, raw, want, tol):
    LITERALS.append((clause, bytes.fromhex(raw), dict(floating_point_format=fmt)))
    assert _feq(lit(clause, bytes.fromhex(raw), floating_point_format=fmt), want, tol)


def test_ibm_single_keeps_the_reference_exponent_behaviour():
    """decodeIbmSingleBigEndian masks the exponent with 0x80000000 (FloatingPointDecoders.scala:82):
    0x43142EFC is 5.045883f there, 322.94 in IBM arithmetic -- the reference's value is the parity bar."""
    v = lit("COMP-1", bytes.fromhex("43142EFC"))
    assert abs(v - 5.045883) < 1e-5 and abs(v - 322.94) > 1


# ---------------------------------------------------------------- BinaryDecoderSpec.scala

def test_ebcdic_string_and_numbers():
    # :25-34 decodeString(EBCDIC, "TestString")
    assert lit("X(10)", bytes.fromhex("E385A2A3E2A399899587")) == "TestString"
    # :37-44 decodeEbcdicBigNumber("1002551", scale 2) = 10025.51
    assert lit("9(5)V99", bytes.fromhex("F1F0F0F2F5F5F1")) == Decimal("10025.51")


@pytest.mark.parametrize("clause,raw,want", [
    ("S9(15) COMP-3", "101144750000004F", Decimal("101144750000004")),    # :46-52 positive
    ("S9(15) COMP-3", "101144750000004D", Decimal("-101144750000004")),   # :54-60 negative
    ("9(15) COMP-3", "101144750000004C", Decimal("101144750000004")),     # :62-68 decodeBCDIntegralNumber
    ("9(5) COMP-3", "1A114C", None),                                      # :70-73 low nibble >= 10
    ("9(5) COMP-3", "A1114F", None),                                      # :75-77 high nibble >= 10
    ("9(5) COMP-3", "111140", None),                                      # :79-81 bad sign nibble
    ("9(5) COMP-3", "11224C", 11224),                                     # :83-85
    ("S9(3)V99 COMP-3", "15884D", Decimal("-158.84")),                    # :113-115
    ("S99V999 COMP-3", "15884D", Decimal("-15.884")),                     # :117-119 odd scale
    ("S9(17)V99 COMP-3", "92233720368547757798" + "8F", None),            # placeholder replaced below
])
def test_comp3_literals(clause, raw, want):
    if raw.startswith("922337203685477577"):
        # :121-126 a number that does not fit a double: 10 bytes, scale 2
        raw, want = "9223372036854775798F", Decimal("92233720368547757.98")
    got = lit(clause, bytes.fromhex(raw))
    LITERALS.append((clause, bytes.fromhex(raw), {}))
    assert got == want, (clause, raw, got)


def test_comp3_19_digits_wrap_like_a_java_long():
    """p = 18 gives 10 bytes = 19 digits; decodeBCDIntegralNumber accumulates a Long and wraps
    (BCDNumberDecoders.scala:29-73): the oracle and the device agree on the wrapped value."""
    v = lit("S9(18) COMP-3", bytes.fromhex("9999999999999999999C"))
    assert v == 9999999999999999999 - (1 << 64)


@pytest.mark.parametrize("clause,raw,size,want", [
    # 8 bit (:160-165), COMP-9 = little-endian; PIC 9(2) COMP-9 is one byte
    ("S9(2) COMP-9", "00", None, 0), ("S9(2) COMP-9", "01", None, 1), ("S9(2) COMP-9", "FF", None, -1),
    ("9(2) COMP-9", "FF", None, 255),
    # 16 bit (:167-176)
    ("S9(4) COMP", "0000", None, 0), ("S9(4) COMP", "0001", None, 1), ("S9(4) COMP-9", "0100", None, 1),
    ("S9(4) COMP", "FFFF", None, -1), ("9(4) COMP-9", "FFFF", None, 65535), ("S9(4) COMP-9", "FEFF", None, -2),
    ("S9(4) COMP", "FFFE", None, -2), ("S9(3)V9 COMP", "0016", None, Decimal("2.2")),
    # 32 bit (:178-189)
    ("S9(9) COMP", "00000100", None, 256), ("S9(7)V99 COMP-9", "00010000", None, Decimal("2.56")),
    ("S9(9) COMP-9", "FEFFFFFF", None, -2), ("S9(9) COMP", "FFFFFFFE", None, -2),
    ("9(10) COMP-9", "FEFFFFFF", 4, 4294967294), ("9(10) COMP", "FFFFFFFE", 4, 4294967294),   # decodeBinaryNumber
    ("9(4)V9(6) COMP", "FFFFFFFE", 4, Decimal("4294.967294")),
    ("9(2)V9(12) COMP", "FFFFFFFE", 4, Decimal("0.004294967294")),
    # 64 bit (:191-204)
    ("S9(18) COMP-9", "0000010000000000", None, 65536), ("S9(18) COMP", "0000000000010000", None, 65536),
    ("S9(18) COMP-9", "FEFFFFFFFFFFFFFF", None, -2),
    # 19-20 digit values: a decimal(19+, 4) column holds them (decimal(18, 4) would null them in Spark)
    ("S9(15)V9(4) COMP", "203041506070809F", 8, Decimal("231942562156698.0255")),
    ("9(16)V9(4) COMP", "A03041506070809F", 8, Decimal("1154279765842175.6063")),
    ("S9(15)V9(4) COMP", "A03041506070809F", 8, Decimal("-690394641528779.5553")),
    # non-standard byte counts (:206-215): 3-byte binaries
    ("S9(7) COMP", "000001", 3, 1), ("S9(7) COMP-9", "020000", 3, 2), ("S9(7) COMP", "001003", 3, 4099),
    ("S9(7) COMP-9", "042000", 3, 8196), ("S9(7) COMP", "801003", 3, -8384509),
    ("S9(6)V9 COMP-9", "042080", 3, Decimal("-838041.2")), ("9(7) COMP", "801003", 3, 8392707),
    ("9(6)V9 COMP-9", "042080", 3, Decimal("839680.4")),
])
def test_binary_literals(clause, raw, size, want):
    # sizes no integral PIC produces are the spec's direct decodeBinaryNumber calls
    dec = size is not None and ("V" in clause or size == 3 or clause.startswith("9(10)"))
    got = lit(clause, bytes.fromhex(raw), size=size, as_decimal=dec)
    LITERALS.append((clause, bytes.fromhex(raw), dict(size=size, as_decimal=dec)))
    assert got == want, (clause, raw, got)


# ---------------------------------------------------------------- StringDecodersSpec.scala

ASCII_STRING = "AbCdEfGhIjKlMnOpQrStUvWxYz 0123456789 !@#$%^&*()[]{};'\\\"/.,"   # :29
EBCDIC_BYTES = bytes.fromhex(                                                          # :31-40
    "c182c384c586c788c991d293d495d697d899e2a3e4a5e6a7e8a900f0f1f2f3f4f5f6f7f8f9005a7c7b5b6cb0505c4d5d"
    "babbc0d05e7de07f614b6b")


@pytest.mark.parametrize("trim,text", [("none", ASCII_STRING), ("right", ASCII_STRING + "  \t "),
                                       ("left", "  \t " + ASCII_STRING), ("both", "  \t " + ASCII_STRING + "  \t ")])
def test_ebcdic_string_trims(trim, text):
    """:44-71 decodeEbcdicString with the common code page and each trimming policy."""
    raw = EBCDIC_BYTES if trim == "none" else to_ebcdic(text)
    assert lit(f"X({len(raw)})", raw, string_trimming=trim) == ASCII_STRING


def test_hex_and_raw():
    """:163-177 decodeHex / decodeRaw (the debug HEX / RAW fields, DebugFieldsPolicy)."""
    raw = bytes([0, 3, 16, 127, 0xFF, 0x81])
    assert lit("X(6)", raw, enc_override=cbk.HEX) == "0003107FFF81"
    assert lit("X(4)", bytes([0, 1, 2, 0xFF]), enc_override=cbk.RAW) == bytes([0, 1, 2, 0xFF])


@pytest.mark.parametrize("clause,text,want", [
    # decodeEbcdicNumber through the Int / Long / BigDecimal wrappers (:179-203)
    ("9(1)", "1", 1), ("S9(1)", "1", 1), ("9(3)", " 1 ", 1), ("S9(3)", " 1 ", 1), ("S9(2)", "-1", -1),
    ("9(1)", "-1", None) if False else ("9(2)", "-1", None),
    ("9(11).99", " 18938717862,00 ", Decimal("18938717862.00")),
    ("9(11).99", " 18938717862.00 ", Decimal("18938717862.00")),
    ("9(11).99", " + 18938717862.00 ", Decimal("18938717862.00")),
    ("S9(11).99", " - 18938717862.00 ", Decimal("-18938717862.00")),
    ("9(11).99", " - 18938717862.00 ", None),
    # leading / trailing separate signs, comma decimals (:205-210)
    ("S9(3).99", "+100,00", Decimal("100.00")), ("S9(3).99", "100.00+", Decimal("100.00")),
    ("S9(3).99", "-100.00", Decimal("-100.00")), ("S9(3).99", "100,00-", Decimal("-100.00")),
    # overpunched signs A..I / J..R / { } (:212-233)
    ("S9(3).99", "A00,00", Decimal("100.00")), ("S9(3).99", "J00,00", Decimal("-100.00")),
    ("S9(3)", "B02", 202), ("S9(3)", "K02", -202), ("S9(3)", "30C", 303), ("S9(3)", "30L", -303),
    ("S9(3)", "40D", 404), ("S9(3)", "40M", -404), ("S9(3)", "E05", 505), ("S9(3)", "N05", -505),
    ("S9(3)", "F06", 606), ("S9(3)", "O06", -606), ("S9(3)", "G07", 707), ("S9(3)", "P07", -707),
    ("S9(3)", "H08", 808), ("S9(3)", "Q08", -808), ("S9(3)", "I09", 909), ("S9(3)", "R09", -909),
    ("S9(3)", "90{", 900), ("S9(3)", "90}", -900),
    ("S9(9)", "AAABBBCCC", None),                                    # :235-238 malformed
    # decodeEbcdicInt (:263-289)
    ("S9(4)", "+100", 100), ("S9(4)", "100+", 100), ("S9(4)", "-100", -100), ("S9(4)", "100-", -100),
    ("9(4)", "+100", 100), ("9(4)", "100+", 100), ("9(4)", "-100", None), ("9(4)", "100-", None),
    ("9(6)", "+100,0", None), ("S9(7)", "100.00+", None), ("S9(8)", "-100,000", None), ("S9(8)", "100.000-", None),
    ("9(3)", "AAA", None),
    # decodeEbcdicLong (:325-351)
    ("S9(17)", "+1000000000000000", 10 ** 15), ("S9(17)", "1000000000000000+", 10 ** 15),
    ("S9(17)", "-1000000000000000", -10 ** 15), ("S9(17)", "1000000000000000-", -10 ** 15),
    ("9(17)", "+1000000000000000", 10 ** 15), ("9(17)", "-1000000000000000", None),
    ("9(17)", "1000000000000000-", None), ("S9(18)", "1000000000000000.0-", None), ("S9(12)", "AAA", None),
    # decodeEbcdicBigNumber scale / scale factor (:377-395)
    ("S9(5)", "+1000", 1000), ("S9(4)V9", "+1000", Decimal("100.0")), ("S9(2)V9(3)", "+1000", Decimal("1.000")),
    ("S9V9(4)", "+1000", Decimal("0.1000")), ("SV9(5)", "+1000", None),
    ("SP9(5)", "+1000", Decimal("0.01000")), ("P9(4)", "1000", Decimal("0.01000")),
    # decodeEbcdicBigDecimal (:423-441)
    ("S9(4).9", "+1000", Decimal("1000")), ("S9(4).99", "1000,25+", Decimal("1000.25")),
    ("S9(4).9", "-1000", Decimal("-1000")), ("S9(4).99", "1000,25-", Decimal("-1000.25")),
    ("9(26).99", "12345678901234567890123456", Decimal("12345678901234567890123456")),
    ("S9(5).9", "200E+10", None), ("S9(2).9", "ABC", None),
])
def test_ebcdic_number_literals(clause, text, want):
    raw = to_ebcdic(text)
    size = None
    cb = cbk.parse_copybook(f"       01  R.\n           05  F   PIC {clause}.\n")
    if cb.ast.children[0].children[0].data_size != len(raw):
        size = len(raw)
    got = lit(clause, raw, size=size)
    LITERALS.append((clause, raw, dict(size=size)))
    assert got == want, (clause, text, got)


# ---------------------------------------------------------------- MalformedValuesSpec.scala

def test_malformed_values():
    # :25-42 PIC 9(7) COMP: 0x008040C0 = 8405184; 0xC28040C0 has the top bit (unsigned) -> null
    assert lit("9(7) COMP", bytes.fromhex("008040C0")) == 8405184
    assert lit("9(7) COMP", bytes.fromhex("C28040C0")) is None
    # :44-70 PIC 9(5)V9(5): 12345.12345; a 'k' (0x93) digit -> null
    assert lit("9(5)V9(5)", bytes.fromhex("F1F2F3F4F5F1F2F3F4F5")) == Decimal("12345.12345")
    assert lit("9(5)V9(5)", bytes.fromhex("F1F2F3F4F5F1F2F3F493")) is None
    # :72-164 unsigned patterns reject a leading '-' (0x60); signed ones accept it
    neg = bytes.fromhex("60F2F3F4F5F6F7F8F9F0")
    pos = bytes.fromhex("F1F2F3F4F5F6F7F8F9F0")
    assert lit("9(2)", bytes.fromhex("F1F2")) == 12 and lit("9(2)", bytes.fromhex("60F2")) is None
    assert lit("9(6)", pos[:6]) == 123456 and lit("9(6)", neg[:6]) is None
    assert lit("9(10)", pos) == 1234567890 and lit("9(10)", neg) is None
    assert lit("9(5)V9(5)", pos) == Decimal("12345.6789") and lit("9(5)V9(5)", neg) is None
    assert lit("S9(2)", bytes.fromhex("F1F2")) == 12 and lit("S9(2)", bytes.fromhex("60F2")) == -2
    assert lit("S9(6)", pos[:6]) == 123456 and lit("S9(6)", neg[:6]) == -23456
    assert lit("S9(10)", pos) == 1234567890 and lit("S9(10)", neg) == -234567890
    assert lit("S9(5)V9(5)", pos) == Decimal("12345.6789") and lit("S9(5)V9(5)", neg) == Decimal("-2345.6789")


@pytest.mark.gpu
def test_literals_through_the_gpu():
    """Every literal above, decoded by the GPU kernels (one-field plans, one record each) and
    compared with the oracle + host-build result (run after the CPU tests of this module collected
    them; re-collected here when the module runs alone)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cobrix_amd.plan import NativePlan
    from cobrix_amd.reader import DecodedBatch, _alloc_columns, string_capacity
    if not LITERALS:   # `-m gpu` deselected the CPU cases: replay their parameter tables
        for name, fn in list(globals().items()):
            if not name.startswith("test_") or fn is test_literals_through_the_gpu:
                continue
            for m in getattr(fn, "pytestmark", []):
                if m.name == "parametrize":
                    argnames = [a.strip() for a in m.args[0].split(",")]
                    for vals in m.args[1]:
                        fn(**dict(zip(argnames, vals)))
    assert LITERALS
    L = N.load()
    for clause, raw, kw in LITERALS:
        want = lit(clause, raw, **kw)
        cb, _ = lit_copybook(clause, raw, **kw)
        plan = build_plan(cb)
        npl = NativePlan(plan)
        d = torch.zeros(max(16, len(raw)), dtype=torch.uint8, device="cuda")
        if raw:
            d[: len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
        cols, cs = _alloc_columns(plan, 1, string_capacity(npl, 1), d.device)
        N.check(L.cbx_decode_fixed(npl.handle, d.data_ptr(), 1, len(raw), 0, 0, cs, None))
        N.check(L.cbx_plan_check(npl.handle, None))
        got = DecodedBatch(plan, 1, cols, 0, True, False).to_rows()[0]["F"]
        if isinstance(got, np.floating):
            got = float(got)
        assert got == want, (clause, raw.hex(), got, want)
        npl.close()
