"""Spark-facing schema of a parsed copybook (SC/schema/CobolSchema.scala).

`spark_type` restates `CobolSchema.parsePrimitive` (SC/schema/CobolSchema.scala:144-173):
the output column type every decoded value is converted to.  `SparkSchema` restates
`createSparkSchema` (:77-113): generated File_Id/Record_Id/Seg_IdN columns, root collapse.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

from .copybook import (COMP1, COMP2, RAW, AlphaNumeric, Copybook, Decimal, Group, Integral,
                       Primitive, Statement)

# Spark result type tags
ST_INT, ST_LONG, ST_DECIMAL, ST_FLOAT, ST_DOUBLE, ST_STRING, ST_BINARY = 1, 2, 3, 4, 5, 6, 7
ST_NAMES = {ST_INT: "integer", ST_LONG: "long", ST_DECIMAL: "decimal", ST_FLOAT: "float",
            ST_DOUBLE: "double", ST_STRING: "string", ST_BINARY: "binary"}


def spark_type(p: Primitive) -> Tuple[int, int, int]:
    """(type tag, decimal precision, decimal scale) for a primitive."""
    d = p.dtype
    if isinstance(d, AlphaNumeric):
        return (ST_BINARY if d.enc == RAW else ST_STRING, 0, 0)
    if isinstance(d, Decimal):
        if d.compact == COMP1:
            return (ST_FLOAT, 0, 0)
        if d.compact == COMP2:
            return (ST_DOUBLE, 0, 0)
        return (ST_DECIMAL, d.effective_precision(), d.effective_scale())
    assert isinstance(d, Integral)
    if d.precision > 18:
        return (ST_DECIMAL, d.precision, 0)
    if d.precision > 9:
        return (ST_LONG, 0, 0)
    return (ST_INT, 0, 0)


@dataclass
class SparkField:
    name: str
    kind: str                 # "struct" | "primitive" | "generated"
    node: Optional[Statement]
    is_array: bool = False
    children: Optional[List["SparkField"]] = None
    stype: Tuple[int, int, int] = (0, 0, 0)


def _parse_group(g: Group, redefines: List[Group]) -> SparkField:
    """parseGroup (:116-139): child segments are skipped where they sit and appended, as arrays of
    structs, to the group named as their parent (getChildSegments, :175-192)."""
    kids: List[SparkField] = []
    for c in g.children:
        if c.is_filler:
            continue
        if isinstance(c, Group):
            if c.parent_segment is None:
                kids.append(_parse_group(c, redefines))
        else:
            kids.append(SparkField(c.name, "primitive", c, c.is_array, None, spark_type(c)))
    for seg in redefines:
        if seg.parent_segment is not None and seg.parent_segment.name.upper() == g.name.upper():
            child = _parse_group(seg, redefines)
            kids.append(SparkField(seg.name, "struct", seg, True, child.children))
    return SparkField(g.name, "struct", g, g.is_array, kids)


def spark_schema(cb: Copybook, collapse_root: bool, generate_record_id: bool = False,
                 seg_id_levels: int = 0, input_file_name_field: str = "") -> List[SparkField]:
    """CobolSchema.createSparkSchema (SC/schema/CobolSchema.scala:77-113)."""
    redefines = cb.all_segment_redefines()
    records = [_parse_group(r, redefines) for r in cb.ast.children if isinstance(r, Group)]
    fields: List[SparkField] = []
    if collapse_root:
        for r in records:
            fields.extend(r.children or [])
    else:
        fields = records
    gen: List[SparkField] = []
    if generate_record_id:
        gen += [SparkField("File_Id", "generated", None, stype=(ST_INT, 0, 0)),
                SparkField("Record_Id", "generated", None, stype=(ST_LONG, 0, 0))]
    if input_file_name_field:
        gen.append(SparkField(input_file_name_field, "generated", None, stype=(ST_STRING, 0, 0)))
    gen += [SparkField(f"Seg_Id{i}", "generated", None, stype=(ST_STRING, 0, 0))
            for i in range(seg_id_levels)]
    return gen + fields


def _type_json(f: SparkField):
    if f.kind == "struct":
        t = {"type": "struct", "fields": [field_json(c) for c in (f.children or [])]}
    else:
        tag, p, s = f.stype
        t = f"decimal({p},{s})" if tag == ST_DECIMAL else ST_NAMES[tag]
    if f.is_array:
        return {"type": "array", "elementType": t, "containsNull": True}
    return t


def field_json(f: SparkField) -> dict:
    """StructField.jsonValue: generated File_Id / Record_Id are non-nullable
    (SC/schema/CobolSchema.scala:104-107), every other field nullable."""
    nullable = not (f.kind == "generated" and f.name in ("File_Id", "Record_Id"))
    return {"name": f.name, "type": _type_json(f), "nullable": nullable, "metadata": {}}


def schema_json(fields: List[SparkField]) -> dict:
    """`df.schema.json` of the reference's DataFrame, as a parsed JSON value."""
    return {"type": "struct", "fields": [field_json(f) for f in fields]}
