"""Spark `.option(...)` maps -> ReaderParameters (the reference's CobolParametersParser).

The host of the GPU path keeps the reference's DataSource option names, defaults and checks so
a job switching to it keeps its `spark.read.format("cobol").option(...)` calls:

  * option names / defaults         SC/parameters/CobolParametersParser.scala:40-104, 191-240
  * variable-length reader trigger  :242-290 (parseVariableLengthParameters)
  * multisegment options            :298-404 (segment_id_level*, redefine-segment-id-map*)
  * pedantic unknown-key rejection  :473-  (validateSparkCobolOptions)
  * ReaderParameters mapping        SC/source/DefaultSource.scala:141-209

(SC = spark-cobol/src/main/scala/za/co/absa/cobrix/spark/cobol/.)  Options of subsystems outside
the accelerated path (custom record header parsers / extractors, multiple copybooks) raise
UnsupportedOption instead of being dropped; the reference's option-combination checks
(validateSparkCobolOptions) raise ValueError as its IllegalArgumentException does.
"""
from __future__ import annotations

import json
from typing import Dict, List, Mapping, Optional, Tuple

from .copybook import _transform_identifier
from .reader import ReaderParameters

# option names (CobolParametersParser.scala:40-104)
KNOWN = {
    "copybook", "copybooks", "copybook_contents", "path", "encoding", "pedantic",
    "record_length_field", "record_start_offset", "record_end_offset", "file_start_offset",
    "file_end_offset", "generate_record_id", "schema_retention_policy", "drop_group_fillers",
    "drop_value_fillers", "non_terminals", "occurs_mappings", "debug", "truncate_comments",
    "comments_lbound", "comments_ubound", "string_trimming_policy", "ebcdic_code_page",
    "ebcdic_code_page_class", "ascii_charset", "is_utf16_big_endian", "floating_point_format",
    "variable_size_occurs", "record_length", "is_xcom", "is_record_sequence", "is_text",
    "is_rdw_big_endian", "is_rdw_part_of_record_length", "rdw_adjustment", "segment_field",
    "segment_id_root", "segment_filter", "record_header_parser", "record_extractor",
    "rhp_additional_info", "re_additional_info", "with_input_file_name_col", "enable_indexes",
    "input_split_records", "input_split_size_mb", "segment_id_prefix", "optimize_allocation",
    "improve_locality", "debug_ignore_file_size",
}

# options whose subsystem the GPU path does not cover (never silently ignored)
UNSUPPORTED = {
    "record_header_parser": "custom record header parsers",
    "record_extractor": "custom raw record extractors",
    "copybooks": "multiple copybooks (Copybook.merge)",
}

# custom code pages (`ebcdic_code_page_class`): the JVM loads a CodePage class by name
# (CodePage.getCodePageByClass, CP/parser/encoding/codepage/CodePage.scala:70-77); the host of the
# GPU path registers the class's 256-entry EBCDIC -> Unicode table under that name instead
_CODE_PAGE_CLASSES: Dict[str, List[int]] = {}


class UnsupportedOption(ValueError):
    pass


def register_code_page_class(class_name: str, table: List[int]) -> None:
    if len(table) != 256 or any(not 0 <= int(c) <= 0xFFFF for c in table):
        raise ValueError("a code page table has 256 UTF-16 code units")
    _CODE_PAGE_CLASSES[class_name] = [int(c) for c in table]


def _bool(v: str, key: str) -> bool:
    s = str(v).strip().lower()
    if s in ("true", "false"):
        return s == "true"
    raise ValueError(f"For input string: \"{v}\" ({key})")   # String.toBoolean


def segment_levels(opts: Mapping[str, str]) -> List[str]:
    """parseSegmentLevels (CobolParametersParser.scala:339-356)."""
    levels: List[str] = []
    i = 0
    while True:
        name = f"segment_id_level{i}"
        if name in opts:
            levels.append(opts[name])
        elif i == 0 and "segment_id_root" in opts:
            levels.append(opts["segment_id_root"])
        else:
            return levels
        i += 1


def redefine_map(opts: Mapping[str, str]) -> Dict[str, str]:
    """getSegmentIdRedefineMapping (:389-404): segment id -> redefine group name."""
    out: Dict[str, str] = {}
    for k, v in opts.items():
        kl = k.lower()
        if kl.startswith("redefine-segment-id-map") or kl.startswith("redefine_segment_id_map"):
            parts = v.split("=>")
            if len(parts) != 2:
                raise ValueError(f"Illegal argument for the 'redefine-segment-id-map' option: '{v}'.")
            grp = parts[0].strip()
            for sid in parts[1].split(","):
                out[sid.strip()] = _transform_identifier(grp)
    return out


def segment_redefine_parents(opts: Mapping[str, str]) -> Dict[str, str]:
    """getSegmentRedefineParents (:433-465): `segment-children:N` = "PARENT => CHILD1,CHILD2" ->
    child redefine -> parent redefine (transformed identifiers)."""
    out: Dict[str, str] = {}
    for k, v in opts.items():
        if not k.lower().startswith(("segment-children", "segment_children")):
            continue
        parts = v.split("=>")
        if len(parts) != 2:
            raise ValueError(f"Illegal argument for the 'segment-children' option: '{v}'.")
        parent = _transform_identifier(parts[0].strip())
        for child in (_transform_identifier(c.strip()) for c in parts[1].split(",")):
            if child in out and out[child] != parent:
                raise ValueError(f"Duplicate child '{child}' for parents {out[child]} and {parent} "
                                 "specified for 'segment-children' option.")
            out[child] = parent
    return out


def _flag(opts: Mapping[str, str], key: str) -> bool:
    return _bool(opts.get(key, "false"), key)


# options that cannot accompany `record_extractor` / `record_length` / `is_text`
# (CobolParametersParser.validateSparkCobolOptions, :495-610), in the reference's order
_NOT_WITH_EXTRACTOR = ("is_text", "record_length", "is_record_sequence", "is_xcom", "is_rdw_big_endian",
                       "is_rdw_part_of_record_length", "rdw_adjustment", "record_length_field",
                       "record_header_parser", "rhp_additional_info")
_NOT_WITH_RECORD_LENGTH = ("is_text", "is_record_sequence", "is_xcom", "is_rdw_big_endian",
                           "is_rdw_part_of_record_length", "rdw_adjustment", "record_length_field",
                           "record_header_parser", "rhp_additional_info")
_NOT_WITH_TEXT = ("is_rdw_big_endian", "is_rdw_part_of_record_length", "rdw_adjustment", "is_xcom",
                  "record_length", "record_header_parser", "rhp_additional_info")


def validate_options(opts: Mapping[str, str]) -> None:
    """validateSparkCobolOptions (CobolParametersParser.scala:473-620): option combinations the
    reference rejects with IllegalArgumentException (ValueError here), checked before any reader
    is built.  `is_text` counts as set when it is "true" (the reference reads it as a boolean);
    the other options count when present, whatever their value (`params.contains`)."""
    is_text = _flag(opts, "is_text")
    # a "record sequence" for the input-file-name column (:474-479)
    is_seq = (_flag(opts, "is_xcom") or _flag(opts, "is_record_sequence") or _flag(opts, "variable_size_occurs")
              or "file_start_offset" in opts or "file_end_offset" in opts or "record_length_field" in opts)

    def clash(lead: str, keys) -> None:
        bad = [k for k in keys if (is_text if k == "is_text" else k in opts)]
        if bad:
            raise ValueError(f"Option '{lead}' and {', '.join(bad)} cannot be used together.")

    if "record_extractor" in opts:
        clash("record_extractor", _NOT_WITH_EXTRACTOR)
    if "record_length" in opts:
        clash("record_length", _NOT_WITH_RECORD_LENGTH)
    if segment_redefine_parents(opts) and segment_levels(opts):
        raise ValueError("Options 'segment-children:*' cannot be used with 'segment_id_level*' or 'segment_id_root' "
                         "since ID fields generation is not supported for hierarchical records reader.")
    # (the message names a custom record extractor, the condition does not test for one: as in :581)
    if not is_seq and "with_input_file_name_col" in opts:
        raise ValueError("Option 'with_input_file_name_col' is supported only when one of this holds: "
                         "'is_record_sequence' = true or 'variable_size_occurs' = true or one of these options is set: "
                         "'record_length_field', 'file_start_offset', 'file_end_offset' or a custom record extractor "
                         "is specified")
    if is_text:
        clash("is_text", _NOT_WITH_TEXT)


def is_variable_length(opts: Mapping[str, str]) -> bool:
    """parseVariableLengthParameters (:242-290): which options select VarLenNestedReader."""
    if "record_length_field" in opts and ("is_record_sequence" in opts or "is_xcom" in opts):
        raise ValueError("Option 'record_length_field' cannot be used together with 'is_record_sequence' or 'is_xcom'.")
    seq = _bool(opts.get("is_xcom", opts.get("is_record_sequence", "false")), "is_record_sequence")
    return ("record_length_field" in opts or seq or _bool(opts.get("generate_record_id", "false"), "generate_record_id")
            or int(opts.get("file_start_offset", "0")) > 0 or int(opts.get("file_end_offset", "0")) > 0
            or "record_extractor" in opts or _bool(opts.get("variable_size_occurs", "false"), "variable_size_occurs"))


def parse_options(options: Mapping[str, object]) -> Tuple[ReaderParameters, bool]:
    """CobolParametersParser.parse + DefaultSource.getReaderProperties.

    Returns (ReaderParameters, variable_length) where variable_length says whether the reference
    would build a VarLenNestedReader (DefaultSource.buildEitherReader, :72-81)."""
    opts = {str(k): str(v) for k, v in options.items()}
    var_len = is_variable_length(opts)   # parseVariableLengthParameters runs before the validation
    validate_options(opts)
    pedantic = _bool(opts.get("pedantic", "false"), "pedantic")
    if pedantic:
        unknown = [k for k in opts if k not in KNOWN and not k.lower().startswith(("segment_id_level", "redefine-segment-id-map", "redefine_segment_id_map", "segment-children"))]
        if unknown:
            raise ValueError(f"Redundant or unrecognized option(s) to 'spark-cobol': {', '.join(unknown)}.")
    for k, what in UNSUPPORTED.items():
        if k in opts:
            raise UnsupportedOption(f"option '{k}': {what} are not on the GPU path")

    enc = opts.get("encoding", "")
    if enc == "" or enc.lower() == "ebcdic":
        is_ebcdic = True
    elif enc.lower() == "ascii":
        is_ebcdic = False
    else:
        raise ValueError(f"Invalid value '{enc}' for 'encoding' option. Should be either 'EBCDIC' or 'ASCII'.")
    policy = opts.get("schema_retention_policy", "keep_original")
    if policy.lower() not in ("keep_original", "collapse_root"):
        raise ValueError(f"Invalid value '{policy}' for 'schema_retention_policy' option.")
    trim = opts.get("string_trimming_policy", "both")
    if trim.lower() not in ("none", "left", "right", "both"):
        raise ValueError(f"Invalid value '{trim}' for 'string_trimming_policy' option.")
    fp = opts.get("floating_point_format", "IBM")
    if fp.upper() not in ("IBM", "IBM_LE", "IEEE754", "IEEE754_LE"):
        raise ValueError(f"Invalid value '{fp}' for 'floating_point_format' option.")
    debug = opts.get("debug", "false").lower()
    debug_policy = {"false": "none", "none": "none", "true": "hex", "hex": "hex", "raw": "raw"}.get(debug)
    if debug_policy is None:
        raise ValueError(f"Invalid value '{debug}' for 'debug' option. Allowed one of: 'true' = 'hex', 'raw', 'false' = 'none'. ")

    code_page_table = None
    if "ebcdic_code_page_class" in opts:
        cls = opts["ebcdic_code_page_class"]
        if cls not in _CODE_PAGE_CLASSES:
            raise ValueError(f"Code page class '{cls}' is not registered (register_code_page_class)")
        code_page_table = _CODE_PAGE_CLASSES[cls]

    seg_field = opts.get("segment_field")
    levels = segment_levels(opts) if seg_field is not None else []
    filt = opts["segment_filter"].split(",") if (seg_field is not None and "segment_filter" in opts) else None
    parents = segment_redefine_parents(opts)
    occurs = json.loads(opts.get("occurs_mappings", "{}"))
    non_terminals = [s for s in opts.get("non_terminals", "").split(",") if s]
    p = ReaderParameters(
        is_ebcdic=is_ebcdic,
        ebcdic_code_page=opts.get("ebcdic_code_page", "common"),
        ebcdic_code_page_table=code_page_table,
        floating_point_format=fp.upper(),
        is_utf16_big_endian=_bool(opts.get("is_utf16_big_endian", "true"), "is_utf16_big_endian"),
        ascii_charset=opts.get("ascii_charset", ""),
        variable_size_occurs=_bool(opts.get("variable_size_occurs", "false"), "variable_size_occurs") if var_len else False,
        record_length=int(opts["record_length"]) if "record_length" in opts else None,
        record_length_field=opts.get("record_length_field") if var_len else None,
        is_record_sequence=_bool(opts.get("is_xcom", opts.get("is_record_sequence", "false")), "is_record_sequence") if var_len else False,
        is_text=_bool(opts.get("is_text", "false"), "is_text"),
        is_rdw_big_endian=_bool(opts.get("is_rdw_big_endian", "false"), "is_rdw_big_endian") if var_len else False,
        is_rdw_part_rec_length=_bool(opts.get("is_rdw_part_of_record_length", "false"), "is_rdw_part_of_record_length") if var_len else False,
        rdw_adjustment=int(opts.get("rdw_adjustment", "0")) if var_len else 0,
        enable_indexes=_bool(opts.get("enable_indexes", "true"), "enable_indexes") if var_len else False,
        input_split_records=int(opts["input_split_records"]) if (var_len and "input_split_records" in opts) else None,
        input_split_size_mb=int(opts["input_split_size_mb"]) if (var_len and "input_split_size_mb" in opts) else None,
        start_offset=int(opts.get("record_start_offset", "0")),
        end_offset=int(opts.get("record_end_offset", "0")),
        file_start_offset=int(opts.get("file_start_offset", "0")) if var_len else 0,
        file_end_offset=int(opts.get("file_end_offset", "0")) if var_len else 0,
        generate_record_id=_bool(opts.get("generate_record_id", "false"), "generate_record_id") if var_len else False,
        schema_policy=policy.lower(),
        string_trimming_policy=trim.lower(),
        segment_field=seg_field,
        segment_id_redefine_map=redefine_map(opts) if seg_field is not None else {},
        segment_redefine_parents=parents,
        segment_id_filter=filt,
        segment_id_levels=levels,
        segment_id_prefix=opts.get("segment_id_prefix", "") if seg_field is not None else "",
        drop_group_fillers=_bool(opts.get("drop_group_fillers", "false"), "drop_group_fillers"),
        drop_value_fillers=_bool(opts.get("drop_value_fillers", "true"), "drop_value_fillers"),
        non_terminals=non_terminals,
        occurs_mappings=occurs,
        debug_fields_policy=debug_policy,
        # VariableLengthParameters.inputFileNameColumn: only the variable-length readers generate the
        # column (the fixed-length defaults carry "", DefaultSource.scala:141-162)
        input_file_name_column=opts.get("with_input_file_name_col", "") if var_len else "",
        debug_ignore_file_size=_bool(opts.get("debug_ignore_file_size", "false"), "debug_ignore_file_size"),
    )
    return p, var_len
