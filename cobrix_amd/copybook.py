"""Copybook front-end: COBOL copybook text -> Cobrix-equivalent AST with binary layout.

This is the host-side stand-in for the JVM parser that the production path keeps
(`CopybookParser.parseTree`, CP/parser/CopybookParser.scala:148-262).  It exists so the
GPU path can be driven and tested without a JVM: the GPU library itself only ever sees the
flattened field-descriptor table built from this AST (cobrix_amd/plan.py).

Behaviour restated from the reference (file:line into /root/reference,
CP = cobol-parser/src/main/scala/za/co/absa/cobrix/cobol/):
  * comment truncation, cols 7..72            CP/parser/antlr/ANTLRParser.scala:55-112
  * PIC -> type rules (Integral/Decimal/Alpha) CP/parser/antlr/ParserVisitor.scala:63-440, 574-821
  * level nesting rules                        CP/parser/antlr/ParserVisitor.scala:184-203
  * sizes (getBytesCount)                      CP/parser/decoders/BinaryUtils.scala:129-155
  * calculateSchemaSizes / getSchemaWithOffsets CP/parser/CopybookParser.scala:336-414
  * markDependeeFields                         CP/parser/CopybookParser.scala:423-506
  * markSegmentRedefines / setSegmentParents   CP/parser/CopybookParser.scala:523-667
  * renameGroupFillers / calculateNonFillerSizes CP/parser/CopybookParser.scala:780-958
  * generateRecordLayoutPositions              CP/parser/Copybook.scala:193-265
Pinned by the reference's `data/*_layout.txt` goldens (tests/test_copybook.py).
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Union

# --------------------------------------------------------------------------------------
# Data types (CP/parser/ast/datatype/*.scala)
# --------------------------------------------------------------------------------------

# usages (CP/parser/ast/datatype/Usage.scala); None means DISPLAY
COMP1, COMP2, COMP3, COMP4, COMP5, COMP9 = "COMP-1", "COMP-2", "COMP-3", "COMP-4", "COMP-5", "COMP-9"

# encodings (CP/parser/encoding/Encoding.scala)
EBCDIC, ASCII, UTF16, HEX, RAW = "EBCDIC", "ASCII", "UTF16", "HEX", "RAW"

# sign positions
LEFT, RIGHT = "L", "R"

MAX_INTEGER_PRECISION = 9      # CP/parser/common/Constants.scala:37
MAX_LONG_PRECISION = 18        # CP/parser/common/Constants.scala:42
MAX_BIN_INT_PRECISION = 38
MAX_DECIMAL_PRECISION = 38
MAX_DECIMAL_SCALE = 18
MAX_FIELD_LENGTH = 100000


class CopybookSyntaxError(Exception):
    """Mirrors SyntaxErrorException (CP/parser/exceptions/SyntaxErrorException.scala)."""

    def __init__(self, line: int, field: str, msg: str):
        super().__init__(f"Syntax error in the copybook at line {line}, field {field}: {msg}")
        self.line, self.field, self.msg = line, field, msg


@dataclass
class AlphaNumeric:
    pic: str
    length: int
    enc: str = EBCDIC


@dataclass
class Integral:
    pic: str
    precision: int
    sign_position: Optional[str] = None
    is_sign_separate: bool = False
    compact: Optional[str] = None
    enc: str = EBCDIC


@dataclass
class Decimal:
    pic: str
    scale: int
    precision: int
    scale_factor: int
    explicit_decimal: bool = False
    sign_position: Optional[str] = None
    is_sign_separate: bool = False
    compact: Optional[str] = None
    enc: str = EBCDIC

    # CP/parser/ast/datatype/Decimal.scala:48-61
    def effective_precision(self) -> int:
        return self.precision + abs(self.scale_factor)

    def effective_scale(self) -> int:
        if self.scale_factor > 0:
            return 0
        if self.scale_factor < 0:
            return self.effective_precision()
        return self.scale


CobolType = Union[AlphaNumeric, Integral, Decimal]


# --------------------------------------------------------------------------------------
# AST (CP/parser/ast/{Statement,Group,Primitive}.scala)
# --------------------------------------------------------------------------------------

@dataclass(eq=False)
class Statement:
    level: int
    name: str
    line: int
    redefines: Optional[str] = None
    is_redefined: bool = False
    occurs: Optional[int] = None
    to: Optional[int] = None
    depending_on: Optional[str] = None
    depending_on_handlers: Dict[str, int] = field(default_factory=dict)
    is_filler: bool = False
    offset: int = 0
    data_size: int = 0
    actual_size: int = 0
    parent: Optional["Group"] = None

    @property
    def is_array(self) -> bool:
        return self.occurs is not None

    # Statement.scala:51-69
    @property
    def array_min_size(self) -> int:
        if self.occurs is None:
            return 1
        if self.to is None:
            return 1
        return self.occurs

    @property
    def array_max_size(self) -> int:
        if self.occurs is None:
            return 1
        if self.to is None:
            return self.occurs
        return self.to

    @property
    def is_child_segment(self) -> bool:
        return False


@dataclass(eq=False)
class Primitive(Statement):
    dtype: CobolType = None  # type: ignore[assignment]
    is_dependee: bool = False
    # encoding-independent decoder flavour: set for debug fields ("hex"/"raw")
    debug_kind: Optional[str] = None

    @property
    def is_string(self) -> bool:
        return isinstance(self.dtype, AlphaNumeric)

    # Primitive.scala:84-93
    def binary_size_bytes(self) -> int:
        d = self.dtype
        if isinstance(d, AlphaNumeric):
            return d.length
        if isinstance(d, Decimal):
            return get_bytes_count(d.compact, d.precision, d.sign_position is not None,
                                   d.explicit_decimal, d.is_sign_separate)
        return get_bytes_count(d.compact, d.precision, d.sign_position is not None,
                               False, d.is_sign_separate)


@dataclass(eq=False)
class Group(Statement):
    children: List[Statement] = field(default_factory=list)
    is_segment_redefine: bool = False
    parent_segment: Optional["Group"] = None
    group_usage: Optional[str] = None
    non_filler_size: int = 0

    @property
    def is_child_segment(self) -> bool:
        return self.parent_segment is not None


def get_bytes_count(compression: Optional[str], precision: int, is_signed: bool,
                    is_explicit_decimal_pt: bool, is_sign_separate: bool) -> int:
    """BinaryUtils.getBytesCount (CP/parser/decoders/BinaryUtils.scala:129-155)."""
    if compression in (COMP4, COMP5, COMP9):
        p = precision
        if 1 <= p <= 2 and compression == COMP9:
            return 1
        if 1 <= p <= 4:
            return 2
        if 5 <= p <= 9:
            return 4
        if 10 <= p <= 18:
            return 8
        return int(math.ceil(((math.log(10) / math.log(2)) * p + 1) / 8))
    if compression == COMP1:
        return 4
    if compression == COMP2:
        return 8
    if compression == COMP3:
        return precision // 2 + 1
    if compression is not None:
        raise ValueError(f"Illegal clause {compression}.")
    size = precision
    if is_sign_separate:
        size += 1
    if is_explicit_decimal_pt:
        size += 1
    return size


# --------------------------------------------------------------------------------------
# Lexing
# --------------------------------------------------------------------------------------

_USAGE_WORDS = {
    "COMP": COMP4, "COMPUTATIONAL": COMP4, "COMP-0": COMP4, "COMPUTATIONAL-0": COMP4,
    "COMP-1": COMP1, "COMPUTATIONAL-1": COMP1,
    "COMP-2": COMP2, "COMPUTATIONAL-2": COMP2,
    "COMP-3": COMP3, "COMPUTATIONAL-3": COMP3, "PACKED-DECIMAL": COMP3,
    "COMP-4": COMP4, "COMPUTATIONAL-4": COMP4,
    "COMP-5": COMP5, "COMPUTATIONAL-5": COMP5,
    "BINARY": COMP4,
    "DISPLAY": None,
}
_KEYWORDS = {"PIC", "PICTURE", "USAGE", "REDEFINES", "OCCURS", "SIGN", "JUST", "JUSTIFIED",
             "BLANK", "VALUE", "VALUES", "SYNC", "SYNCHRONIZED"} | set(_USAGE_WORDS)


@dataclass
class _Tok:
    text: str
    line: int
    quoted: bool = False


def _preprocess(contents: str, comments_up_to: int = 6, comments_after: int = 72,
                truncate: bool = True) -> List[str]:
    # ANTLRParser.filterSpecialCharacters + truncateComments (ANTLRParser.scala:85-111)
    contents = contents.replace(" ", " ").replace("\t", " ")
    lines = re.split(r"\r?\n", contents)
    out = []
    for ln in lines:
        if truncate:
            if comments_up_to >= 0 and comments_after >= 0:
                ln = ln[comments_up_to:comments_after]
            elif comments_up_to >= 0:
                ln = ln[comments_up_to:]
            else:
                ln = ln[:len(ln) - comments_after] if comments_after > 0 else ln
        out.append(ln)
    return out


def _tokenize(lines: List[str]) -> List[List[_Tok]]:
    """Split into statements terminated by '.' followed by whitespace/EOF (lexer TERMINAL)."""
    statements: List[List[_Tok]] = []
    cur: List[_Tok] = []
    text = "\n".join(lines) + "\n"
    i, n, line = 0, len(text), 1
    while i < n:
        c = text[i]
        if c == "\n":
            line += 1
            i += 1
            continue
        if c in " \r\f":
            i += 1
            continue
        if c == "*":  # COMMENT: '*' ~[\r\n]* -> skip
            while i < n and text[i] != "\n":
                i += 1
            continue
        if c in "'\"":
            q = c
            j = i + 1
            while j < n:
                if text[j] == q:
                    if j + 1 < n and text[j + 1] == q:
                        j += 2
                        continue
                    break
                if text[j] == "\n":
                    break
                j += 1
            cur.append(_Tok(text[i:j + 1], line, quoted=True))
            i = j + 1
            continue
        if c == "." and (i + 1 >= n or text[i + 1] in " \r\n\f"):
            if cur:
                statements.append(cur)
            cur = []
            i += 1
            continue
        j = i
        while j < n and text[j] not in " \r\n\f'\"":
            if text[j] == "." and (j + 1 >= n or text[j + 1] in " \r\n\f"):
                break
            j += 1
        cur.append(_Tok(text[i:j], line))
        i = j
    if cur:
        statements.append(cur)
    return statements


# --------------------------------------------------------------------------------------
# PIC rules (ParserVisitor.scala:63-440)
# --------------------------------------------------------------------------------------

_REPEAT = re.compile(r"([9XNPZASVxnpzasv])\((\d+)\)")


def _expand_pic(pic: str) -> str:
    return _REPEAT.sub(lambda m: m.group(1) * int(m.group(2)), pic).upper()


def _transform_identifier(s: str) -> str:
    # CopybookParser.transformIdentifier (CopybookParser.scala:942-946)
    return s.replace("'", "").replace('"', "").replace(":", "").replace("-", "_")


def _parse_pic(pic_text: str, line: int, name: str, enc: str) -> CobolType:
    raw = pic_text
    lead_sign = trail_sign = None
    body = raw
    if body[:1] in "+-" and len(body) > 1:
        lead_sign, body = body[0], body[1:]
    elif body[-1:] in "+-" and len(body) > 1:
        trail_sign, body = body[-1], body[:-1]
    e = _expand_pic(body)
    if not e:
        raise CopybookSyntaxError(line, name, f"Error reading PIC {raw}")
    # alphanumeric (visitAlphaX / A / N)
    if re.fullmatch(r"X+", e):
        return AlphaNumeric(f"X({len(e)})", len(e), enc)
    if re.fullmatch(r"A+", e):
        return AlphaNumeric(f"A({len(e)})", len(e), enc)
    if re.fullmatch(r"N+", e):
        return AlphaNumeric(f"N({len(e)})", len(e) * 2, UTF16)

    t: Optional[CobolType] = None
    m = re.fullmatch(r"(S?)(9*)V(P*)(9*)", e)
    if m:  # fromNumericSPicRegexDecimalScaled
        s, n1, p, n2 = m.group(1), len(m.group(2)), len(m.group(3)), len(m.group(4))
        t = Decimal(e, n2, n1 + n2, p, False, LEFT if s else None, False, None, enc)
    if t is None:
        m = re.fullmatch(r"(S?)(9+)(P*)", e)
        if m:  # fromNumericSPicRegexScaled
            s, n, p = m.group(1), len(m.group(2)), len(m.group(3))
            t = Decimal(e, 0, n, p, False, LEFT if s else None, False, None, enc)
    if t is None:
        m = re.fullmatch(r"(S?)(P+)(9+)", e)
        if m:  # fromNumericSPicRegexDecimalScaledLead
            s, p, n = m.group(1), len(m.group(2)), len(m.group(3))
            t = Decimal(e, 0, n, -p, False, LEFT if s else None, False, None, enc)
    if t is None:
        m = re.fullmatch(r"(S?)(9*)[.,](9+)", e)
        if m:  # fromNumericSPicRegexExplicitDot
            s, n1, n2 = m.group(1), len(m.group(2)), len(m.group(3))
            t = Decimal(e, n2, n1 + n2, 0, True, LEFT if s else None, False, None, enc)
    if t is None:
        m = re.fullmatch(r"(Z+)(9*)[.,](9*)(Z*)", e)
        if m and (m.group(3) or m.group(4)):  # fromNumericZPicRegexExplicitDot
            z1, n1, n2, z2 = (len(g) for g in m.groups())
            t = Decimal(e, n2 + z2, z1 + n1 + n2 + z2, 0, True, None, False, None, enc)
    if t is None:
        m = re.fullmatch(r"(Z+)(9*)V(P*)(9*)(Z*)", e)
        if m:  # fromNumericZPicRegexDecimalScaled
            z1, n1, p, n2, z2 = (len(g) for g in m.groups())
            t = Decimal(e, n2 + z2, z1 + n1 + n2 + z2, -p, False, None, False, None, enc)
    if t is None:
        m = re.fullmatch(r"(Z+)(9*)(P*)", e)
        if m:  # fromNumericZPicRegexScaled
            z, n, p = (len(g) for g in m.groups())
            t = Decimal(e, 0, z + n, p, False, None, False, None, enc)
    if t is None:
        raise CopybookSyntaxError(line, name, f"Error reading PIC {raw}")

    # replaceSign for leading/trailing +/- in the PIC (visitLeadingSign / visitTrailingSign)
    if lead_sign or trail_sign:
        t.sign_position = LEFT if lead_sign else RIGHT
        t.is_sign_separate = True
    return t


def _replace_decimal0(t: CobolType) -> CobolType:
    # ParserVisitor.replaceDecimal0 (ParserVisitor.scala:166-181)
    if isinstance(t, Decimal) and t.scale == 0 and t.scale_factor == 0:
        return Integral(t.pic, t.precision, t.sign_position, t.is_sign_separate, t.compact, t.enc)
    return t


def _replace_usage(t: CobolType, usage: Optional[str], line: int, name: str) -> CobolType:
    # ParserVisitor.replaceUsage (ParserVisitor.scala:127-149)
    if usage is None:
        return t
    if isinstance(t, AlphaNumeric):
        raise CopybookSyntaxError(line, name, f"USAGE {usage} is not applicable to alphanumeric fields.")
    if t.compact is not None and t.compact != usage:
        raise CopybookSyntaxError(line, name,
                                  f"Field USAGE ({t.compact}) doesn't match group's USAGE ({usage}).")
    t.compact = usage
    return t


def _check_bounds(t: CobolType, line: int, name: str) -> None:
    # ParserVisitor.checkBounds (ParserVisitor.scala:541-572)
    if isinstance(t, Decimal):
        if t.is_sign_separate and t.compact is not None:
            raise CopybookSyntaxError(line, name, f"SIGN SEPARATE clause is not supported for {t.compact}.")
        if t.scale > MAX_DECIMAL_SCALE:
            raise CopybookSyntaxError(line, name, f"Decimal numbers with scale bigger than {MAX_DECIMAL_SCALE} are not supported.")
        if t.precision > MAX_DECIMAL_PRECISION:
            raise CopybookSyntaxError(line, name, f"Decimal numbers with precision bigger than {MAX_DECIMAL_PRECISION} are not supported.")
        if t.compact is not None and t.explicit_decimal:
            raise CopybookSyntaxError(line, name, f"Explicit decimal point is not supported for {t.compact}.")
    elif isinstance(t, Integral):
        if t.is_sign_separate and t.compact is not None:
            raise CopybookSyntaxError(line, name, f"SIGN SEPARATE clause is not supported for {t.compact}.")
        if t.precision > MAX_BIN_INT_PRECISION and t.compact == COMP4:
            raise CopybookSyntaxError(line, name, f"BINARY-encoded integers with precision bigger than {MAX_BIN_INT_PRECISION} are not supported.")
        if t.precision < 1 or t.precision >= MAX_FIELD_LENGTH:
            raise CopybookSyntaxError(line, name, f"Incorrect field size of {t.precision}.")
    elif isinstance(t, AlphaNumeric):
        if t.length < 1 or t.length >= MAX_FIELD_LENGTH:
            raise CopybookSyntaxError(line, name, f"Incorrect field size of {t.length}.")


# --------------------------------------------------------------------------------------
# Statement parsing (ParserVisitor.visitGroup / visitPrimitive)
# --------------------------------------------------------------------------------------

_LEVEL_RE = re.compile(r"0[1-9]|[1-4][0-9]")


def _parse_statements(contents: str, enc: str, comment_policy) -> Group:
    truncate, up_to, after = comment_policy
    stmts = _tokenize(_preprocess(contents, up_to, after, truncate))
    root = Group(level=0, name="_ROOT_", line=-1)
    levels: List[list] = [[0, root, None]]  # (level, group, children-level)

    def get_parent(section: int, line: int) -> Group:
        # ParserVisitor.getParentFromLevel (ParserVisitor.scala:184-203)
        while section <= levels[-1][0]:
            levels.pop()
        top = levels[-1]
        if top[2] is None or top[2] > section:
            top[2] = section
        elif top[2] != section:
            last = top[1].children[-1]
            raise CopybookSyntaxError(last.line, last.name,
                                      "The field is a leaf element and cannot contain nested fields.")
        return top[1]

    for toks in stmts:
        lvl_text = toks[0].text
        if lvl_text in ("88",):
            continue
        if lvl_text == "66":
            raise CopybookSyntaxError(toks[0].line, "", "Renames not supported yet")
        if not _LEVEL_RE.fullmatch(lvl_text):
            raise CopybookSyntaxError(toks[0].line, lvl_text, f"Unexpected token '{lvl_text}'.")
        line = toks[0].line
        if len(toks) < 2:
            raise CopybookSyntaxError(line, "", "A field name is expected after the level number.")
        name = _transform_identifier(toks[1].text)
        section = int(lvl_text)
        pic: Optional[str] = None
        float_usage: Optional[str] = None
        usage_set = False
        usage: Optional[str] = None
        redefines = None
        occurs = to = None
        depending = None
        sign_clause = None  # (side, separate)
        i = 2
        words = toks

        def up(k):
            return words[k].text.upper() if k < len(words) else ""

        while i < len(words):
            w = up(i)
            if words[i].quoted:
                i += 1
                continue
            if w in ("PIC", "PICTURE"):
                i += 1
                if up(i) == "IS":
                    i += 1
                if i >= len(words):
                    raise CopybookSyntaxError(line, name, "PIC clause without a picture string.")
                pic = words[i].text
                i += 1
            elif w == "USAGE":
                i += 1
                if up(i) == "IS":
                    i += 1
                u = up(i)
                if u not in _USAGE_WORDS:
                    raise CopybookSyntaxError(line, name, f"Unknown Usage literal {u}")
                if _USAGE_WORDS[u] in (COMP1, COMP2):
                    float_usage = _USAGE_WORDS[u]
                else:
                    usage, usage_set = _USAGE_WORDS[u], True
                i += 1
            elif w in _USAGE_WORDS:
                if _USAGE_WORDS[w] in (COMP1, COMP2):
                    float_usage = _USAGE_WORDS[w]
                else:
                    usage, usage_set = _USAGE_WORDS[w], True
                i += 1
            elif w == "REDEFINES":
                redefines = _transform_identifier(words[i + 1].text)
                i += 2
            elif w == "OCCURS":
                occurs = int(words[i + 1].text)
                i += 2
                if up(i) == "TO":
                    to = int(words[i + 1].text)
                    i += 2
                if up(i) == "TIMES":
                    i += 1
                if up(i) == "DEPENDING":
                    i += 1
                    if up(i) == "ON":
                        i += 1
                    depending = _transform_identifier(words[i].text)
                    i += 1
                while up(i) in ("ASCENDING", "DESCENDING"):
                    i += 1
                    if up(i) == "KEY":
                        i += 1
                    if up(i) == "IS":
                        i += 1
                    i += 1
                if up(i) == "INDEXED":
                    i += 1
                    if up(i) == "BY":
                        i += 1
                    i += 1
            elif w == "SIGN":
                i += 1
                if up(i) == "IS":
                    i += 1
                side = up(i)
                if side not in ("LEADING", "TRAILING"):
                    raise CopybookSyntaxError(line, name, "SIGN must be LEADING or TRAILING.")
                i += 1
                sep = False
                if up(i) == "SEPARATE":
                    sep = True
                    i += 1
                if up(i) == "CHARACTER":
                    i += 1
                sign_clause = (LEFT if side == "LEADING" else RIGHT, sep)
            elif w in ("JUST", "JUSTIFIED"):
                i += 1
                if up(i) == "RIGHT":
                    i += 1
            elif w == "BLANK":
                i += 1
                if up(i) == "WHEN":
                    i += 1
                if up(i) in ("ZERO", "ZEROS", "ZEROES"):
                    i += 1
            elif w in ("VALUE", "VALUES"):
                i += 1
                while i < len(words) and (words[i].quoted or up(i) not in _KEYWORDS):
                    i += 1
            elif w in ("SYNC", "SYNCHRONIZED"):
                i += 1
                if up(i) in ("LEFT", "RIGHT"):
                    i += 1
            else:
                raise CopybookSyntaxError(line, name, f"Unexpected token '{words[i].text}'.")

        parent = get_parent(section, line)
        is_filler = name.upper() == "FILLER"
        if pic is None and float_usage is None:
            if usage_set and usage is None:
                usage = None  # DISPLAY group usage
            grp = Group(level=section, name=name, line=line, redefines=redefines,
                        occurs=occurs, to=to, depending_on=depending, is_filler=is_filler,
                        group_usage=usage if usage_set else None, parent=parent)
            parent.children.append(grp)
            levels.append([section, grp, None])
            continue

        if float_usage is not None and pic is None:
            # ParserVisitor.visitPic COMP_1 / COMP_2 branch
            t: CobolType = Decimal("9(16)V9(16)", 16, 32, 0, False, None, False, float_usage, enc)
        else:
            t = _replace_decimal0(_parse_pic(pic, line, name, enc))
            if float_usage is not None:
                t = _replace_usage(t, float_usage, line, name)
        if usage_set:
            t = _replace_usage(t, usage, line, name)
        elif parent.group_usage is not None:
            t = _replace_usage(t, parent.group_usage, line, name)
        if sign_clause is not None:
            if isinstance(t, AlphaNumeric):
                raise CopybookSyntaxError(line, name, "SIGN clause is not applicable to alphanumeric fields.")
            if t.is_sign_separate:
                raise CopybookSyntaxError(line, name, "Cannot mix explicit signs and SEPARATE clauses")
            t.sign_position, t.is_sign_separate = sign_clause
        _check_bounds(t, line, name)
        prim = Primitive(level=section, name=name, line=line, redefines=redefines,
                         occurs=occurs, to=to, depending_on=depending, is_filler=is_filler,
                         dtype=t, parent=parent)
        parent.children.append(prim)
    return root


# --------------------------------------------------------------------------------------
# AST passes (CopybookParser.scala)
# --------------------------------------------------------------------------------------

def _calculate_schema_sizes(grp: Group) -> None:
    # CopybookParser.calculateSchemaSizes (CopybookParser.scala:336-384)
    redefined_sizes: List[int] = []
    redefined_names: set = set()
    kids = grp.children
    for i, child in enumerate(kids):
        if child.redefines is None:
            redefined_sizes.clear()
            redefined_names.clear()
        else:
            if i == 0:
                raise CopybookSyntaxError(child.line, child.name,
                                          "The first field of a group cannot use REDEFINES keyword.")
            if child.redefines.upper() not in redefined_names:
                raise CopybookSyntaxError(child.line, child.name,
                                          f"The field {child.name} redefines {child.redefines}, "
                                          "which is not part if the redefined fields block.")
            kids[i - 1].is_redefined = True
        if isinstance(child, Group):
            _calculate_schema_sizes(child)
        else:
            size = child.binary_size_bytes()
            child.data_size = size
            child.actual_size = size * child.array_max_size
        redefined_sizes.append(child.actual_size)
        redefined_names.add(child.name.upper())
        if child.redefines is not None:
            mx = max(redefined_sizes)
            for j in range(len(redefined_sizes)):
                kids[i - j].actual_size = mx
    gsize = sum(c.actual_size for c in kids if c.redefines is None)
    grp.data_size = gsize
    grp.actual_size = gsize * grp.array_max_size


def _schema_with_offsets(offset: int, grp: Group) -> None:
    # CopybookParser.getSchemaWithOffsets (CopybookParser.scala:391-414)
    cur = offset
    redefined_offset = offset
    for f in grp.children:
        if f.redefines is None:
            redefined_offset = cur
            use = cur
        else:
            use = redefined_offset
        if isinstance(f, Group):
            _schema_with_offsets(use, f)
        else:
            f.offset = use
        if f.redefines is None:
            cur += f.actual_size
    grp.offset = offset


def _iter_primitives(grp: Group):
    for c in grp.children:
        if isinstance(c, Group):
            yield from _iter_primitives(c)
        else:
            yield c


def _mark_dependee_fields(root: Group, occurs_handlers: Dict[str, Dict[str, int]]) -> None:
    # CopybookParser.markDependeeFields (CopybookParser.scala:423-506)
    flat: List[Primitive] = []
    dependees: Dict[int, List[Statement]] = {}

    def traverse(g: Group):
        for f in g.children:
            if f.depending_on is not None:
                nu = f.depending_on.upper()
                found = [p for p in flat if p.name.upper() == nu]
                if not found:
                    raise ValueError(f"Unable to find dependee field {nu} from DEPENDING ON clause.")
                if f.name in occurs_handlers:
                    f.depending_on_handlers = dict(occurs_handlers[f.name])
                dependees.setdefault(id(found[0]), []).append(f)
            if isinstance(f, Group):
                traverse(f)
            else:
                flat.append(f)

    traverse(root)
    for p in _iter_primitives(root):
        if id(p) in dependees:
            if not isinstance(p.dtype, Integral):
                for st in dependees[id(p)]:
                    if not st.depending_on_handlers:
                        raise ValueError(f"Field {p.name} is a DEPENDING ON field of an OCCURS, "
                                         f"should be integral, found {type(p.dtype).__name__}.")
            p.is_dependee = True


def _mark_segment_redefines(root: Group, segment_redefines: Sequence[str]) -> None:
    # CopybookParser.markSegmentRedefines (CopybookParser.scala:523-598)
    if not segment_redefines:
        return
    found: set = set()
    wanted = [_transform_identifier(s) for s in segment_redefines]
    allow_non_redefines = len(segment_redefines) == 1
    state = [0]

    def ensure(cur: str, is_seg: bool):
        if state[0] == 0 and is_seg:
            state[0] = 1
        elif state[0] == 1 and not is_seg:
            state[0] = 2
        elif state[0] == 2 and is_seg:
            raise ValueError(f"The '{cur}' field is specified to be a segment redefine. "
                             "However, it is not in the same group of REDEFINE fields")

    def is_seg(g: Group) -> bool:
        return (allow_non_redefines or g.is_redefined or g.redefines is not None) and g.name in wanted

    def process(g: Group):
        for c in g.children:
            if isinstance(c, Primitive):
                ensure(c.name, False)
            elif is_seg(c):
                if c.name in found:
                    raise ValueError(f"Duplicate segment redefine field '{c.name}' found.")
                ensure(c.name, True)
                found.add(c.name)
                c.is_segment_redefine = True
            else:
                ensure(c.name, False)
                if state[0] == 0:
                    process(c)

    for c in root.children:
        if isinstance(c, Group):
            process(c)
    missing = [w for w in wanted if w not in found]
    if missing:
        raise ValueError(f"The following segment redefines not found: [ {','.join(missing)} ]. "
                         "Please check the fields exist and are redefines/redefined by.")


def _all_segment_redefines(g: Group) -> List[Group]:
    out = []
    for c in g.children:
        if isinstance(c, Group):
            if c.is_segment_redefine:
                out.append(c)
            out.extend(_all_segment_redefines(c))
    return out


def _set_segment_parents(root: Group, field_parent_map: Dict[str, str]) -> None:
    # CopybookParser.setSegmentParents (CopybookParser.scala:611-667)
    if not field_parent_map:
        return
    fpm = {_transform_identifier(k): _transform_identifier(v) for k, v in field_parent_map.items()}
    redefs = _all_segment_redefines(root)
    roots: List[str] = []

    def process(g: Group):
        for c in g.children:
            if isinstance(c, Group):
                if c.is_segment_redefine:
                    pname = fpm.get(c.name)
                    if pname is not None:
                        par = [r for r in redefs if r.name == pname]
                        if not par:
                            raise ValueError(f"Field {pname} is specified to be the parent of {c.name}, "
                                             f"but {pname} is not a segment redefine.")
                        c.parent_segment = par[0]
                    else:
                        roots.append(c.name)
                else:
                    if c.name in fpm:
                        raise ValueError("Parent field is defined for a field that is not a segment redefine.")
                    process(c)

    process(root)
    if len(roots) > 1:
        raise ValueError(f"Only one root segment is allowed. Found root segments: [ {', '.join(roots)} ]. ")
    if not roots:
        raise ValueError("No root segment found in the segment parent-child map.")


def _rename_group_fillers(root: Group, drop_group_fillers: bool, drop_value_fillers: bool) -> None:
    # CopybookParser.renameGroupFillers (CopybookParser.scala:780-833)
    counters = {"grp": 0, "prim": 0}

    def process_prim(p: Primitive):
        if drop_value_fillers or not p.is_filler:
            return p
        counters["prim"] += 1
        p.name = f"FILLER_P{counters['prim']}"
        p.is_filler = False
        return p

    def rename_fillers(g: Group) -> bool:
        new_kids = []
        has_non_fillers = False
        for c in g.children:
            if isinstance(c, Group):
                was_filler = c.is_filler
                rename_sub(c)
                if c.children:
                    new_kids.append(c)
                if not was_filler:
                    has_non_fillers = True
            else:
                process_prim(c)
                new_kids.append(c)
                if not c.is_filler:
                    has_non_fillers = True
        g.children = new_kids
        return has_non_fillers

    def rename_sub(g: Group):
        has_non = rename_fillers(g)
        if has_non:
            if g.is_filler and not drop_group_fillers:
                counters["grp"] += 1
                g.name = f"FILLER_{counters['grp']}"
                g.is_filler = False
        else:
            g.is_filler = True

    if not rename_fillers(root):
        raise ValueError("The copybook is empty of consists only of FILLER fields.")


def _process_group_fillers(root: Group, drop_value_fillers: bool) -> None:
    # CopybookParser.processGroupFillers (CopybookParser.scala:846-878)
    def process(g: Group) -> bool:
        new_kids = []
        has_non = False
        for c in g.children:
            if isinstance(c, Group):
                was_filler = c.is_filler
                if not process(c):
                    c.is_filler = True
                if c.children:
                    new_kids.append(c)
                if not was_filler:
                    has_non = True
            else:
                new_kids.append(c)
                if not c.is_filler or not drop_value_fillers:
                    has_non = True
        g.children = new_kids
        return has_non

    if not process(root):
        raise ValueError("The copybook is empty of consists only of FILLER fields.")


def _add_debug_fields(root: Group, policy: str) -> None:
    # CopybookParser.addDebugFields (CopybookParser.scala:887-934)
    if policy == "none":
        return

    def process(g: Group):
        new_kids = []
        for c in g.children:
            if isinstance(c, Group):
                process(c)
                new_kids.append(c)
            else:
                # the debug field is field.copy(...) of the original: it keeps the original's
                # isRedefined (a redefined field's debug twin does not advance the offset either),
                # while the original itself becomes isRedefined = true (:913-922)
                was_redefined = c.is_redefined
                c.is_redefined = True
                new_kids.append(c)
                size = c.data_size
                dbg = Primitive(level=c.level, name=c.name + "_debug", line=c.line,
                                redefines=c.name, is_redefined=was_redefined, occurs=c.occurs, to=c.to,
                                depending_on=c.depending_on,
                                depending_on_handlers=c.depending_on_handlers,
                                is_filler=c.is_filler, offset=c.offset, data_size=c.data_size,
                                actual_size=c.actual_size, parent=c.parent,
                                dtype=AlphaNumeric(f"X({size})", size,
                                                   HEX if policy == "hex" else RAW),
                                debug_kind=policy)
                new_kids.append(dbg)
        g.children = new_kids

    process(root)


def _calculate_non_filler_sizes(g: Group) -> None:
    # CopybookParser.calculateNonFillerSizes (CopybookParser.scala:942-968)
    new_kids = []
    for c in g.children:
        if isinstance(c, Group):
            _calculate_non_filler_sizes(c)
            c.non_filler_size = sum(1 for k in c.children if not k.is_filler and not k.is_child_segment)
            if c.children:
                new_kids.append(c)
        else:
            new_kids.append(c)
    g.children = new_kids


def _add_non_terminals(g: Group, non_terminals: set, enc: str) -> None:
    # CopybookParser.addNonTerminals (CopybookParser.scala:264-317)
    new_kids: List[Statement] = []
    for c in g.children:
        if isinstance(c, Primitive):
            new_kids.append(c)
            continue
        _add_non_terminals(c, non_terminals, enc)
        new_kids.append(c)
        if c.name in non_terminals:
            c.is_redefined = True
            existing = {k.name for k in g.children}
            mod, want = 0, c.name + "_NT"
            while want in existing:
                mod += 1
                want = c.name + "_NT" + str(mod)
            sz = c.actual_size
            new_kids.append(Primitive(level=c.level, name=want, line=c.line, redefines=c.name,
                                      dtype=AlphaNumeric(f"X({sz})", sz, enc), offset=c.offset,
                                      data_size=c.data_size, actual_size=c.actual_size,
                                      parent=g))
    g.children = new_kids


# --------------------------------------------------------------------------------------
# Copybook
# --------------------------------------------------------------------------------------

class Copybook:
    """Parsed copybook (CP/parser/Copybook.scala) plus the decode options bound at parse time."""

    def __init__(self, ast: Group, *, code_page: str = "common", string_trimming: str = "both",
                 floating_point_format: str = "IBM", is_utf16_big_endian: bool = True,
                 ascii_charset: str = "", data_encoding: str = EBCDIC):
        self.ast = ast
        self.code_page = code_page
        self.string_trimming = string_trimming
        self.floating_point_format = floating_point_format
        self.is_utf16_big_endian = is_utf16_big_endian
        self.ascii_charset = ascii_charset
        self.data_encoding = data_encoding

    # Copybook.getRecordSize (Copybook.scala:33-35)
    @property
    def record_size(self) -> int:
        return self.ast.offset + self.ast.actual_size

    @property
    def is_hierarchical(self) -> bool:
        return any(g.parent_segment is not None for g in _all_segment_redefines(self.ast))

    def all_segment_redefines(self) -> List[Group]:
        return _all_segment_redefines(self.ast)

    def get_field_by_name(self, field_name: str) -> Statement:
        # Copybook.getFieldByName (Copybook.scala:58-152)
        def in_group(g: Group, nm: str):
            out = [g] if g.name.lower() == nm.lower() else []
            for c in g.children:
                if isinstance(c, Group):
                    out += in_group(c, nm)
                elif c.name.lower() == nm.lower():
                    out.append(c)
            return out

        def by_path(g: Group, path: List[str]):
            if not path:
                raise ValueError(f"'{field_name}' is a GROUP and not a primitive field.")
            out = []
            for c in g.children:
                if c.name.lower() == path[0].lower():
                    if isinstance(c, Group):
                        out += by_path(c, path[1:])
                    else:
                        out.append(c)
            return out

        if "." in field_name:
            path = [_transform_identifier(p) for p in field_name.split(".")]
            roots = self.ast.children
            if not any(r.name.lower() == path[0].lower() for r in roots[-1:]):
                path = [roots[0].name] + path
            found = []
            for r in roots:
                if r.name.lower() == path[0].lower():
                    found += by_path(r, path[1:])
        else:
            nm = _transform_identifier(field_name)
            found = []
            for r in self.ast.children:
                found += in_group(r, nm)
        if not found:
            raise ValueError(f"Field '{field_name}' is not found in the copybook.")
        if len(found) > 1:
            raise ValueError(f"Multiple fields with name '{field_name}' found in the copybook. "
                             "Please specify the exact field using '.' notation.")
        return found[0]

    def generate_record_layout_positions(self) -> str:
        # Copybook.generateRecordLayoutPositions (Copybook.scala:193-265)
        counter = [0]

        def al(s, w):
            return s if len(s) >= w else s + " " * (w - len(s))

        def ar(s, w):
            return s if len(s) >= w else " " * (w - len(s)) + s

        def gen(g: Group, path: str = "  ") -> str:
            parts = []
            for f in g.children:
                counter[0] += 1
                r = "R" if f.redefines is not None else ""
                rr = "r" if f.is_redefined else ""
                arr = "[]" if f.occurs is not None else ""
                start = f.offset + 1
                length = f.actual_size
                end = start + length - 1
                if isinstance(f, Group):
                    mods = f"{rr}{r}{arr}"
                    sub = gen(f, path + "  ")
                    parts.append(al(f"{path}{f.level} {f.name}", 39) + al(mods, 11) +
                                 ar(str(counter[0]), 5) + ar(str(start), 7) + ar(str(end), 7) +
                                 ar(str(length), 7) + "\n" + sub)
                else:
                    d = "D" if f.is_dependee else ""
                    mods = f"{d}{rr}{r}{arr}"
                    parts.append(al(f"{path}{f.level} {f.name}", 39) + al(mods, 11) +
                                 ar(str(counter[0]), 5) + ar(str(start), 7) + ar(str(end), 7) +
                                 ar(str(length), 7))
            return "\n".join(parts)

        strings = []
        for grp in self.ast.children:
            start = grp.offset + 1
            length = grp.actual_size
            end = start + length - 1
            body = gen(grp)
            strings.append(al(grp.name, 55) + ar(str(start), 7) + ar(str(end), 7) +
                           ar(str(length), 7) + "\n" + body)
        header = "-------- FIELD LEVEL/NAME --------- --ATTRIBS--    FLD  START     END  LENGTH\n\n"
        return header + "\n".join(strings)


def parse_copybook(contents: str, *, data_encoding: str = EBCDIC, drop_group_fillers: bool = False,
                   drop_value_fillers: bool = True, segment_redefines: Sequence[str] = (),
                   field_parent_map: Optional[Dict[str, str]] = None, string_trimming: str = "both",
                   comment_policy=(True, 6, 72), code_page: str = "common",
                   floating_point_format: str = "IBM", is_utf16_big_endian: bool = True,
                   non_terminals: Sequence[str] = (), occurs_handlers: Optional[Dict[str, Dict[str, int]]] = None,
                   debug_fields_policy: str = "none", ascii_charset: str = "") -> Copybook:
    """CopybookParser.parseTree (CP/parser/CopybookParser.scala:200-262)."""
    root = _parse_statements(contents, data_encoding, comment_policy)
    _calculate_schema_sizes(root)
    _schema_with_offsets(0, root)
    if non_terminals:
        _add_non_terminals(root, {_transform_identifier(n) for n in non_terminals}, data_encoding)
    _mark_dependee_fields(root, occurs_handlers or {})
    if drop_group_fillers:
        _process_group_fillers(root, drop_value_fillers)
    _rename_group_fillers(root, drop_group_fillers, drop_value_fillers)
    _mark_segment_redefines(root, segment_redefines)
    _set_segment_parents(root, field_parent_map or {})
    _add_debug_fields(root, debug_fields_policy)
    _calculate_non_filler_sizes(root)
    return Copybook(root, code_page=code_page, string_trimming=string_trimming,
                    floating_point_format=floating_point_format,
                    is_utf16_big_endian=is_utf16_big_endian, ascii_charset=ascii_charset,
                    data_encoding=data_encoding)
