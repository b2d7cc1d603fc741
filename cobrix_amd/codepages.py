"""EBCDIC code pages (CP/parser/encoding/codepage/CodePage.scala:59-68) and their UTF-8 LUT form.

The GPU kernels take each code page as a 256 x 4-byte table: byte b -> (UTF-8 length, up to 3
UTF-8 bytes) of the code point the reference maps b to, plus a "trimmable" flag (code point
<= U+0020, the Java `String.trim` predicate).
"""
from __future__ import annotations

from typing import List

import numpy as np

from .codepages_data import CODE_PAGES


def lut_for(name) -> List[int]:
    """Code-page table by name (CodePage.getCodePageByName), or a custom CodePage's own
    256-entry table (ebcdic_code_page_class, CodePage.getCodePageByClass)."""
    if isinstance(name, (list, tuple)):
        if len(name) != 256:
            raise ValueError("a code page table has 256 entries")
        return [int(c) for c in name]
    if name not in CODE_PAGES:
        raise ValueError(f"The code page '{name}' is not one of the builtin EBCDIC code pages.")
    return CODE_PAGES[name]


def utf8_lut(table: List[int]) -> np.ndarray:
    """uint32[256]: bits 0-23 UTF-8 bytes (first byte lowest), bits 24-25 length, bit 31 trimmable."""
    out = np.zeros(256, dtype=np.uint32)
    for b, cp in enumerate(table):
        enc = chr(cp).encode("utf-8")
        assert 1 <= len(enc) <= 3, (b, cp)
        v = 0
        for i, x in enumerate(enc):
            v |= x << (8 * i)
        v |= len(enc) << 24
        if cp <= 0x20:
            v |= 1 << 31
        out[b] = v
    return out


def ascii_charset_table(name: str) -> List[int]:
    """AsciiStringDecoderWrapper (CP/parser/decoders/AsciiStringDecoderWrapper.scala:43-67) as a
    code-page table: bytes 0x00-0x1F become ' ', every other byte is decoded by the single-byte
    charset `name` (Charset.forName aliases as Python's codec registry knows them; an unmappable
    byte decodes to U+FFFD, as Java's decoder replaces it).  Multi-byte charsets cannot be a
    per-byte table and raise ValueError."""
    import codecs
    info = codecs.lookup(name)
    if info.name.startswith(("utf", "ascii")) or "jis" in info.name or info.name in (
            "cp932", "cp936", "cp949", "cp950", "gb2312", "gbk", "gb18030", "big5", "big5hkscs", "euc_jp",
            "euc_kr", "johab", "hz", "iso2022_jp", "iso2022_kr"):
        raise ValueError(f"ascii_charset {name!r} is not a single-byte charset")
    whole = bytes(range(256)).decode(info.name, errors="replace")
    if len(whole) != 256:
        raise ValueError(f"ascii_charset {name!r} is not a single-byte charset")
    return [0x20 if b < 32 else ord(whole[b]) for b in range(256)]


def is_us_ascii(name: str) -> bool:
    """DecoderSelector.scala:79 -- an empty name or US-ASCII keeps decodeAsciiString."""
    if not name:
        return True
    import codecs
    return codecs.lookup(name).name == "ascii"
