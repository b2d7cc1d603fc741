"""Spark option handling on the host (cobrix_amd/options.py): the reference's option-combination
checks (CobolParametersParser.validateSparkCobolOptions, SC/parameters/CobolParametersParser.scala:473-620)
and the reader parameters the options select.  CPU only: nothing here decodes."""
from __future__ import annotations

import pytest

from cobrix_amd.options import UnsupportedOption, parse_options
from cobrix_amd.reader import parse_copybook_for, reader_schema

import goldens as G


@pytest.mark.parametrize("extra", ["record_length_field", "is_record_sequence", "is_xcom", "is_rdw_big_endian",
                                   "is_rdw_part_of_record_length", "rdw_adjustment"])
def test_record_length_clashes(extra):
    """`record_length` with any framing option is an IllegalArgumentException
    (CobolParametersParser.scala:533-565; Test27RecordLengthSpec.scala:112 for record_length_field)."""
    opts = {"record_length": "10", extra: "false" if extra.startswith("is_") else "2"}
    with pytest.raises(ValueError) as e:
        parse_options(opts)
    assert e.type is ValueError
    assert f"Option 'record_length' and {extra} cannot be used together." in str(e.value)


def test_record_length_with_text_flag():
    """is_text counts only when true (the reference reads it as a boolean)."""
    parse_options({"record_length": "10", "is_text": "false"})
    with pytest.raises(ValueError, match="Option 'record_length' and is_text cannot be used together."):
        parse_options({"record_length": "10", "is_text": "true"})


def test_text_clashes():
    with pytest.raises(ValueError, match="Option 'is_text' and is_rdw_big_endian, rdw_adjustment cannot be used together."):
        parse_options({"is_text": "true", "is_rdw_big_endian": "true", "rdw_adjustment": "4"})


def test_record_extractor_clashes_before_unsupported():
    """The combination check comes first (IllegalArgumentException), as in the reference."""
    with pytest.raises(ValueError, match="Option 'record_extractor' and is_record_sequence cannot be used together."):
        parse_options({"record_extractor": "com.example.X", "is_record_sequence": "true"})
    with pytest.raises(UnsupportedOption):
        parse_options({"record_extractor": "com.example.X"})


def test_record_length_field_with_record_sequence():
    with pytest.raises(ValueError, match="cannot be used together with 'is_record_sequence' or 'is_xcom'"):
        parse_options({"record_length_field": "LEN", "is_record_sequence": "true"})


def test_input_file_name_needs_record_sequence():
    """Test20InputFileNameSpec.scala:79-90 and Test08InputFileName.scala:62-72: the column needs a
    variable-length read."""
    with pytest.raises(ValueError, match="'with_input_file_name_col' is supported only when one of this holds"):
        parse_options({"with_input_file_name_col": "file_name"})
    with pytest.raises(ValueError, match="'with_input_file_name_col' is supported only when one of this holds"):
        parse_options({"with_input_file_name_col": "file", "schema_retention_policy": "collapse_root"})
    p, var_len = parse_options({"with_input_file_name_col": "F", "is_record_sequence": "true"})
    assert var_len and p.input_file_name_column == "F"
    # file offsets make it legal (Test08InputFileName.scala:48-57)
    p, var_len = parse_options({"with_input_file_name_col": "file", "file_start_offset": "4", "file_end_offset": "5"})
    assert var_len and p.input_file_name_column == "file"


def test_input_file_name_schema_position():
    """CobolSchema.createSparkSchema (SC/schema/CobolSchema.scala:99-110): the file column comes first,
    after File_Id / Record_Id when those are generated (Test20InputFileNameSpec.scala:112, 142)."""
    cb_text = G.read("test4_copybook.cob").decode("latin-1")
    for gen, pos in ((False, 0), (True, 2)):
        opts = {"is_record_sequence": "true", "encoding": "ascii", "with_input_file_name_col": "F"}
        if gen:
            opts["generate_record_id"] = "true"
        p, var_len = parse_options(opts)
        names = [f.name for f in reader_schema(parse_copybook_for(cb_text, p), p, var_len)]
        assert names.index("F") == pos


def test_segment_children_with_levels():
    with pytest.raises(ValueError, match="cannot be used with 'segment_id_level\\*' or 'segment_id_root'"):
        parse_options({"is_record_sequence": "true", "segment_field": "S", "segment_id_level0": "1",
                       "segment-children:1": "A => B"})


def _fixed_reader(opts):
    """A FixedLenNestedReader's host half (parameters + copybook) without the device plan: the
    size checks are host logic."""
    from cobrix_amd.reader import FixedLenNestedReader
    p, var_len = parse_options(opts)
    assert not var_len
    rd = object.__new__(FixedLenNestedReader)
    rd.params = p
    rd.copybook = parse_copybook_for("       01  R.\n          05  A  PIC X(5).\n          05  B  PIC X(11).\n", p)
    return rd


def test_file_size_rule():
    """A file whose size is not a multiple of getRecordSize is rejected -- `record_length`
    included -- unless debug_ignore_file_size is set (CobolScanners.scala:86-90;
    Test1FixedLengthRecordsSpec.scala:62-105)."""
    rd = _fixed_reader({})
    rd.check_binary_data_validity(32)
    with pytest.raises(ValueError, match="Binary record size 16 does not divide data size 33."):
        rd.check_binary_data_validity(33)
    with pytest.raises(ValueError, match="Binary record too small"):
        rd.check_binary_data_validity(10)
    rd = _fixed_reader({"record_length": "10"})
    assert rd.get_record_size() == 10
    rd.check_binary_data_validity(30)
    with pytest.raises(ValueError, match=r"NOT DIVISIBLE by the RECORD SIZE calculated from the copybook \(10 bytes"):
        rd.check_binary_data_validity(33)
    rd = _fixed_reader({"record_length": "10", "record_start_offset": "2"})
    with pytest.raises(ValueError, match=r"\(12 bytes per record\)"):
        rd.check_binary_data_validity(30)
    for opts in ({"debug_ignore_file_size": "true"}, {"debug_ignore_file_size": "true", "record_length": "10"}):
        rd = _fixed_reader(opts)
        assert rd.params.debug_ignore_file_size
        rd.check_binary_data_validity(33)
        rd.check_binary_data_validity(7)
    with pytest.raises(ValueError):
        parse_options({"debug_ignore_file_size": "yes"})
