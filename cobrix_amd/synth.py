"""Synthetic EBCDIC record generators for the BASELINE configs.

SYN200 (config C2): 200-byte fixed-length records, numeric mix -- COMP, COMP-3, zoned DISPLAY
with overpunch, IBM COMP-2, a cp037 name -- with 0.5 % deliberately malformed numeric fields.
Generated with torch so the same code fills host memory (tests) or HBM (bench.py).
"""
from __future__ import annotations

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
