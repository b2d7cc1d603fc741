"""Synthetic EBCDIC record generators for the BASELINE configs.

SYN200 (config C2): 200-byte fixed-length records, numeric mix -- COMP, COMP-3, zoned DISPLAY
with overpunch, IBM COMP-2, a cp037 name -- with 0.5 % deliberately malformed numeric fields.
Generated with torch so the same code fills host memory (tests) or HBM (bench.py).
"""
from __future__ import annotations

import random

import torch

SYN200_COPYBOOK = """
       01  SYN200-REC.
           05  REC-ID        PIC 9(9)  COMP.
           05  BR-ID         PIC S9(4) COMP.
           05  ACCT-NO       PIC S9(18) COMP.
           05  CUST-KEY      PIC S9(9) COMP.
           05  AMT-01        PIC S9(13)V99 COMP-3.
           05  AMT-02        PIC S9(13)V99 COMP-3.
           05  AMT-03        PIC S9(13)V99 COMP-3.
           05  AMT-04        PIC S9(13)V99 COMP-3.
           05  AMT-05        PIC S9(13)V99 COMP-3.
           05  AMT-06        PIC S9(13)V99 COMP-3.
           05  AMT-07        PIC S9(13)V99 COMP-3.
           05  AMT-08        PIC S9(13)V99 COMP-3.
           05  RATE-01       PIC S9(3)V9(6) COMP-3.
           05  RATE-02       PIC S9(3)V9(6) COMP-3.
           05  RATE-03       PIC S9(3)V9(6) COMP-3.
           05  RATE-04       PIC S9(3)V9(6) COMP-3.
           05  QTY-01        PIC S9(7) COMP-3.
           05  QTY-02        PIC S9(7) COMP-3.
           05  QTY-03        PIC S9(7) COMP-3.
           05  QTY-04        PIC S9(7) COMP-3.
           05  ZN-01         PIC S9(9).
           05  ZN-02         PIC S9(9).
           05  ZN-03         PIC S9(9).
           05  ZN-04         PIC S9(9).
           05  ZD-01         PIC S9(7)V99.
           05  ZD-02         PIC S9(7)V99.
           05  FX-RATE       COMP-2.
           05  NAME          PIC X(18).
           05  FILLER        PIC X(2).
"""
SYN200_RECORD_SIZE = 200

_CP037_ALNUM = [*range(0xC1, 0xCA), *range(0xD1, 0xDA), *range(0xE2, 0xEA), *range(0x81, 0x8A),
                *range(0x91, 0x9A), *range(0xA2, 0xAA), *range(0xF0, 0xFA)]


def _digits(g, n, k, device):
    return torch.randint(0, 10, (n, k), generator=g, device=device, dtype=torch.int32)


def _bcd(g, n, nbytes, device, malformed_rate):
    d = _digits(g, n, 2 * nbytes - 1, device)
    sign = torch.where(torch.rand((n, 1), generator=g, device=device) < 0.5, 0xC, 0xD).to(torch.int32)
    nib = torch.cat([d, sign], dim=1)
    bad = torch.rand((n,), generator=g, device=device) < malformed_rate
    if bool(bad.any()):
        pos = torch.randint(0, 2 * nbytes - 1, (n,), generator=g, device=device)
        nib[bad, pos[bad]] = 0xA
    b = (nib[:, 0::2] << 4) | nib[:, 1::2]
    return b.to(torch.uint8)


def _zoned_overpunch(g, n, nbytes, device, malformed_rate):
    d = _digits(g, n, nbytes, device)
    b = (0xF0 + d)
    neg = torch.rand((n,), generator=g, device=device) < 0.5
    b[:, -1] = torch.where(neg, 0xD0 + d[:, -1], 0xC0 + d[:, -1])
    bad = torch.rand((n,), generator=g, device=device) < malformed_rate
    if bool(bad.any()):
        pos = torch.randint(0, nbytes - 1, (n,), generator=g, device=device)
        b[bad, pos[bad]] = 0x5B
    return b.to(torch.uint8)


def _be_bytes(v: torch.Tensor, nbytes: int) -> torch.Tensor:
    v = v.to(torch.int64)
    cols = [((v >> (8 * (nbytes - 1 - i))) & 0xFF) for i in range(nbytes)]
    return torch.stack(cols, dim=1).to(torch.uint8)


def syn200(n: int, seed: int = 20261015, device="cpu", malformed_rate: float = 0.005) -> torch.Tensor:
    """[n, 200] uint8 records of the SYN200 layout."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    parts = []
    parts.append(_be_bytes(torch.randint(0, 1_000_000_000, (n,), generator=g, device=device), 4))      # REC-ID
    parts.append(_be_bytes(torch.randint(-9999, 10000, (n,), generator=g, device=device), 2))           # BR-ID
    hi = torch.randint(-(2**31), 2**31, (n,), generator=g, device=device, dtype=torch.int64)
    lo = torch.randint(0, 2**32, (n,), generator=g, device=device, dtype=torch.int64)
    parts.append(_be_bytes((hi << 32) | lo, 8))                                                          # ACCT-NO
    parts.append(_be_bytes(torch.randint(-999_999_999, 1_000_000_000, (n,), generator=g, device=device), 4))  # CUST-KEY
    for _ in range(8):
        parts.append(_bcd(g, n, 8, device, malformed_rate))                                              # AMT
    for _ in range(4):
        parts.append(_bcd(g, n, 5, device, malformed_rate))                                              # RATE
    for _ in range(4):
        parts.append(_bcd(g, n, 4, device, malformed_rate))                                              # QTY
    for _ in range(4):
        parts.append(_zoned_overpunch(g, n, 9, device, malformed_rate))                                  # ZN
    for _ in range(2):
        parts.append(_zoned_overpunch(g, n, 9, device, malformed_rate))                                  # ZD
    # FX-RATE: IBM hex double, exponent 64 +- 8, normalised fraction
    sgn = (torch.rand((n,), generator=g, device=device) < 0.5).to(torch.int64)
    ex = torch.randint(56, 73, (n,), generator=g, device=device)
    top = torch.randint(1, 16, (n,), generator=g, device=device)
    fr = torch.randint(0, 2**52, (n,), generator=g, device=device, dtype=torch.int64)
    bits = (sgn << 63) | (ex << 56) | (top << 52) | fr
    parts.append(_be_bytes(bits, 8))
    # NAME: cp037 letters/digits, length 0..18, 0x40 padded
    alnum = torch.tensor(_CP037_ALNUM, dtype=torch.uint8, device=device)
    ch = alnum[torch.randint(0, len(_CP037_ALNUM), (n, 18), generator=g, device=device)]
    ln = torch.randint(0, 19, (n, 1), generator=g, device=device)
    pos = torch.arange(18, device=device).unsqueeze(0)
    parts.append(torch.where(pos < ln, ch, torch.full_like(ch, 0x40)))
    parts.append(torch.full((n, 2), 0x40, dtype=torch.uint8, device=device))
    rec = torch.cat(parts, dim=1)
    assert rec.shape[1] == SYN200_RECORD_SIZE, rec.shape
    return rec.contiguous()


# --------------------------------------------------------------------------------------------
# RDW narrow multisegment file (config C4, exp2_multiseg_narrow / test5 layout): segment 'C'
# (STATIC-DETAILS, 64-byte payload) or 'P' (CONTACTS, 60-byte payload) behind a 4-byte RDW, so
# records are 68 / 64 bytes on disk (~65 B per record).
# --------------------------------------------------------------------------------------------
RDW_NARROW_COPYBOOK = """
        01  COMPANY-DETAILS.
            05  SEGMENT-ID        PIC X(5).
            05  COMPANY-ID        PIC X(10).
            05  STATIC-DETAILS.
               10  COMPANY-NAME      PIC X(15).
               10  ADDRESS           PIC X(25).
               10  TAXPAYER.
                  15  TAXPAYER-TYPE  PIC X(1).
                  15  TAXPAYER-STR   PIC X(8).
                  15  TAXPAYER-NUM  REDEFINES TAXPAYER-STR
                                     PIC 9(8) COMP.
            05  CONTACTS REDEFINES STATIC-DETAILS.
               10  PHONE-NUMBER      PIC X(17).
               10  CONTACT-PERSON    PIC X(28).
"""
RDW_NARROW_SEGMENTS = {"C": "STATIC-DETAILS", "P": "CONTACTS"}


def rdw_narrow(n: int, seed: int = 20261016, device="cpu", big_endian: bool = False):
    """n records of the C4 layout with RDW headers -> (bytes [total] uint8, header offsets [n] int64)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    is_c = torch.rand((n,), generator=g, device=device) < 0.35
    plen = torch.where(is_c, 64, 60).to(torch.int64)
    hdr = torch.cumsum(plen + 4, 0) - (plen + 4)                     # header offsets
    total = int((plen + 4).sum().item()) if n else 0
    alnum = torch.tensor(_CP037_ALNUM, dtype=torch.uint8, device=device)
    out = alnum[torch.randint(0, len(_CP037_ALNUM), (max(total, 1),), generator=g, device=device)][:total].clone()
    if n == 0:
        return out, hdr
    # RDW: length in bytes 2-3 little-endian (bytes 0-1 zero), or bytes 0-1 big-endian
    lo, hi = (plen & 0xFF).to(torch.uint8), (plen >> 8).to(torch.uint8)
    z = torch.zeros_like(lo)
    for j, col in enumerate((hi, lo, z, z) if big_endian else (z, z, lo, hi)):
        out[hdr + j] = col
    # SEGMENT-ID 'C    ' / 'P    ' (cp037 C = 0xC3, P = 0xD7, space 0x40)
    out[hdr + 4] = torch.where(is_c, 0xC3, 0xD7).to(torch.uint8)
    for j in range(1, 5):
        out[hdr + 4 + j] = 0x40
    # COMPANY-ID: digits
    for j in range(10):
        out[hdr + 9 + j] = (0xF0 + torch.randint(0, 10, (n,), generator=g, device=device)).to(torch.uint8)
    return out, hdr


def _cat_chunks(make, n: int, chunk: int):
    """Concatenate generator chunks (bounded temporaries for multi-GB inputs)."""
    parts = [make(i, min(chunk, n - s)) for i, s in enumerate(range(0, n, chunk))]
    return torch.cat(parts) if len(parts) > 1 else parts[0]


# --------------------------------------------------------------------------------------------
# SYNSTR200 (config C3): 10 x PIC X(20), cp037, trim both.  Per value: length uniform 0-20,
# 10 % shifted right behind leading spaces, each byte 25 % a Latin-1 accented letter (2-byte
# UTF-8), 1 % a control byte (HT / LF / NEL / NUL); padding 0x40.
# --------------------------------------------------------------------------------------------
SYNSTR200_COPYBOOK = """
       01  SYNSTR200-REC.
""" + "".join(f"           05  STR-{i:02d}        PIC X(20).\n" for i in range(1, 11))
SYNSTR200_RECORD_SIZE = 200
# cp037 bytes of a-with-grave .. y-with-acute etc. (CodePage037: U+00C0..U+00FF)
_CP037_ACCENTED = [0x42, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x51, 0x52, 0x53, 0x54, 0x55, 0x56, 0x57,
                   0x58, 0x62, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x71, 0x72, 0x73, 0x74, 0x75, 0x76,
                   0x77, 0x78, 0xCB, 0xCC, 0xCD, 0xCE, 0xCF, 0xDB, 0xDC, 0xDD, 0xDE, 0xEB, 0xEC, 0xED, 0xEE]
_CP037_CONTROL = [0x05, 0x25, 0x15, 0x00]


def synstr200(n: int, seed: int = 20261017, device="cpu", chunk: int = 4_000_000) -> torch.Tensor:
    """n SYNSTR200 records -> uint8 [n, 200]."""
    alnum = torch.tensor(_CP037_ALNUM, dtype=torch.uint8, device=device)
    acc = torch.tensor(_CP037_ACCENTED, dtype=torch.uint8, device=device)
    ctl = torch.tensor(_CP037_CONTROL, dtype=torch.uint8, device=device)

    def make(ci: int, m: int) -> torch.Tensor:
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1000 + ci)
        shape = (m, 10, 20)
        b = alnum[torch.randint(0, len(_CP037_ALNUM), shape, generator=g, device=device)]
        u = torch.rand(shape, generator=g, device=device)
        b = torch.where(u < 0.25, acc[torch.randint(0, len(_CP037_ACCENTED), shape, generator=g, device=device)], b)
        b = torch.where(u > 0.99, ctl[torch.randint(0, len(_CP037_CONTROL), shape, generator=g, device=device)], b)
        ln = torch.randint(0, 21, (m, 10, 1), generator=g, device=device)
        shift = (torch.rand((m, 10, 1), generator=g, device=device) * (21 - ln).float()).long()
        shift = torch.where(torch.rand((m, 10, 1), generator=g, device=device) < 0.1, shift, 0)
        j = torch.arange(20, device=device).view(1, 1, 20)
        keep = (j >= shift) & (j < shift + ln)
        return torch.where(keep, b, torch.tensor(0x40, dtype=torch.uint8, device=device)).view(m, 200)

    if n == 0:
        return torch.zeros((0, 200), dtype=torch.uint8, device=device)
    return _cat_chunks(make, n, chunk).contiguous()


def rdw_narrow_large(n: int, seed: int = 20261016, device="cpu", chunk: int = 16_000_000, out=None):
    """rdw_narrow in chunks (bounded temporaries): -> (bytes, header offsets).  out: a uint8 tensor of
    rdw_narrow_large_size(...) bytes to generate into (no concatenated copy)."""
    outs, hdrs, base = [], [], 0
    for ci, s in enumerate(range(0, n, chunk)):
        m = min(chunk, n - s)
        o, h = rdw_narrow(m, seed=seed * 1000 + ci, device=device)
        if out is not None:
            out[base:base + o.numel()].copy_(o)
        else:
            outs.append(o)
        hdrs.append(h + base)
        base += int(o.numel())
        del o
    if out is not None:
        return out[:base], torch.cat(hdrs)
    return torch.cat(outs), torch.cat(hdrs)


def rdw_narrow_large_size(n: int, seed: int = 20261016, device="cpu", chunk: int = 16_000_000) -> int:
    """Bytes rdw_narrow_large(n, seed, device, chunk) writes (its first draw fixes every record's size)."""
    total = 0
    for ci, s in enumerate(range(0, n, chunk)):
        m = min(chunk, n - s)
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1000 + ci)
        is_c = torch.rand((m,), generator=g, device=device) < 0.35
        total += int(torch.where(is_c, 68, 64).sum().item())
    return total


# --------------------------------------------------------------------------------------------
# WIDE_ODO (config C5): the exp3_multiseg_wide layout (GEN/TestDataGen4CompaniesWide.scala:35-55)
# with NUM-STRAT PIC 9(4) COMP in front of STRATEGY-DETAIL OCCURS 0 TO 2000 DEPENDING ON
# NUM-STRAT; each element 9(7) COMP + 9(7) COMP-3.  C root: 4 + 16,066 bytes (records stay at the
# maximum size, variable_size_occurs = false), P child: 4 + 60 bytes, 0-4 children per root.
# --------------------------------------------------------------------------------------------
WIDE_ODO_COPYBOOK = """
        01  COMPANY-DETAILS.
            05  SEGMENT-ID        PIC X(5).
            05  COMPANY-ID        PIC X(10).
            05  STATIC-DETAILS.
               10  COMPANY-NAME      PIC X(15).
               10  ADDRESS           PIC X(25).
               10  TAXPAYER.
                  15  TAXPAYER-TYPE  PIC X(1).
                  15  TAXPAYER-STR   PIC X(8).
                  15  TAXPAYER-NUM  REDEFINES TAXPAYER-STR
                                     PIC 9(8) COMP.
               10  NUM-STRAT         PIC 9(4) COMP.
               10  STRATEGY.
                 15  STRATEGY-DETAIL OCCURS 0 TO 2000
                         DEPENDING ON NUM-STRAT.
                   25  NUM1 PIC 9(7) COMP.
                   25  NUM2 PIC 9(7) COMP-3.
            05  CONTACTS REDEFINES STATIC-DETAILS.
               10  PHONE-NUMBER      PIC X(17).
               10  CONTACT-PERSON    PIC X(28).
"""
WIDE_ODO_SEGMENTS = RDW_NARROW_SEGMENTS
WIDE_C_PAYLOAD, WIDE_P_PAYLOAD = 16066, 60


def wide_odo_size(n_roots: int, seed: int = 20261018, device="cpu") -> int:
    """Bytes wide_odo(n_roots, seed, device) writes (its first draw fixes the children per root)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    kids = torch.randint(0, 5, (n_roots,), generator=g, device=device)
    return n_roots * (WIDE_C_PAYLOAD + 4) + int(kids.sum().item()) * (WIDE_P_PAYLOAD + 4)


def wide_odo(n_roots: int, seed: int = 20261018, device="cpu", out=None):
    """n_roots C records, each followed by 0-4 P records, with LE RDW headers ->
    (bytes uint8 [total], header offsets int64 [n_records]).  out: a uint8 tensor of
    wide_odo_size(...) bytes to generate into."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    kids = torch.randint(0, 5, (n_roots,), generator=g, device=device)
    is_c = torch.zeros(int(n_roots + kids.sum().item()), dtype=torch.bool, device=device)
    root_pos = torch.cumsum(kids + 1, 0) - (kids + 1)
    is_c[root_pos] = True
    n = is_c.numel()
    plen = torch.where(is_c, WIDE_C_PAYLOAD, WIDE_P_PAYLOAD).to(torch.int64)
    hdr = torch.cumsum(plen + 4, 0) - (plen + 4)
    total = int((plen + 4).sum().item())
    if out is None:
        out = torch.randint(0, 256, (total,), generator=g, device=device, dtype=torch.uint8)
    else:
        out = out[:total]
        out.random_(0, 256, generator=g)
    lo, hi = (plen & 0xFF).to(torch.uint8), (plen >> 8).to(torch.uint8)
    z = torch.zeros_like(lo)
    for j, col in enumerate((z, z, lo, hi)):
        out[hdr + j] = col
    out[hdr + 4] = torch.where(is_c, 0xC3, 0xD7).to(torch.uint8)
    for j in range(1, 5):
        out[hdr + 4 + j] = 0x40
    # C roots: NUM-STRAT (big-endian, 0..2000) at payload offset 64; elements: NUM1 binary,
    # NUM2 packed 7 digits + F sign
    c = hdr[is_c] + 4
    cnt = torch.randint(0, 2001, (c.numel(),), generator=g, device=device)
    out[c + 64] = (cnt >> 8).to(torch.uint8)
    out[c + 65] = (cnt & 0xFF).to(torch.uint8)
    nc = c.numel()
    for k0 in range(0, 2000, 250):
        k = torch.arange(k0, k0 + 250, device=device)
        base = (c.view(-1, 1) + 66 + 8 * k.view(1, -1)).reshape(-1)
        v = torch.randint(0, 9999999, (nc * 250,), generator=g, device=device)
        for j in range(4):
            out[base + j] = ((v >> (8 * (3 - j))) & 0xFF).to(torch.uint8)
        d = v.clone()
        digs = []
        for _ in range(7):
            digs.append(d % 10)
            d = d // 10
        digs = digs[::-1] + [torch.full_like(v, 0xF)]      # 7 digits + sign nibble
        for j in range(4):
            out[base + 4 + j] = ((digs[2 * j] << 4) | digs[2 * j + 1]).to(torch.uint8)
    return out, hdr


# --------------------------------------------------------------------------------------------
# WALK_NESTED: a layout for the record walk (cbx_walk.h, variable_size_occurs): an OCCURS 0 TO 3
# DEPENDING ON holding an OCCURS 1 TO 4 DEPENDING ON, COMP-3 / zoned / strings around them
# (tests/test_gpu_walk.py parity, tools/bench_walk.py timing).
# --------------------------------------------------------------------------------------------
WALK_NESTED_COPYBOOK = """
       01  REC.
           05  SEG         PIC X(1).
           05  N-OUT       PIC 9(1).
           05  OUTER       OCCURS 0 TO 3 TIMES DEPENDING ON N-OUT.
               10  N-IN    PIC 9(1).
               10  KIND    PIC X(2).
               10  INNER   OCCURS 1 TO 4 TIMES DEPENDING ON N-IN.
                   15  AMT   PIC S9(5) COMP-3.
                   15  NAME  PIC X(3).
           05  TAIL-NUM    PIC 9(4) COMP.
           05  TAIL-TXT    PIC X(6).
"""


def _ebcdic(s: str) -> bytes:
    return s.encode("cp037")


def walk_nested_record(rnd: random.Random, var_size: bool) -> bytes:
    """One NESTED record: counts sometimes out of range or non-numeric (the reference then takes the
    maximum), the arrays' bytes as the layout variant lays them out."""
    n_out = rnd.choice([0, 1, 2, 3, 3, 7])
    b = bytearray(_ebcdic(rnd.choice("ABC")))
    b += bytes([0xF0 + n_out]) if rnd.random() < 0.95 else b"\x40"
    eff_out = n_out if 0 <= n_out <= 3 else 3
    for i in range(3):
        if var_size and i >= eff_out:
            break
        n_in = rnd.choice([1, 2, 3, 4, 0, 9])
        b += bytes([0xF0 + n_in])
        b += _ebcdic(rnd.choice(["AA", "BB", "  ", "ZZ"]))
        eff_in = n_in if 1 <= n_in <= 4 else 4
        for j in range(4):
            if var_size and j >= eff_in:
                break
            dg = [int(c) for c in f"{rnd.randrange(100000):05d}"]
            sign = rnd.choice([0x0C, 0x0D, 0x0F, 0x0A])   # 0x0A: a bad sign nibble -> null
            b += bytes([dg[0] << 4 | dg[1], dg[2] << 4 | dg[3], dg[4] << 4 | sign])
            b += _ebcdic(rnd.choice(["ABC", "X  ", "   ", "Q1 "]))
    b += rnd.randrange(65536).to_bytes(2, "big")
    b += _ebcdic(rnd.choice(["TAIL  ", "T", "      "]).ljust(6))
    cut = len(b) if rnd.random() < 0.85 else rnd.randint(1, len(b))
    return bytes(b[:cut])


def rdw_file(recs) -> bytes:
    return b"".join(bytes([0, 0, len(r) & 0xFF, len(r) >> 8]) + r for r in recs)
