"""ctypes binding of libcobrix_hip.so (include/cobrix_hip.h).

This is the Python counterpart of the JNI / Panama FFM stub a JVM host would use
(INTEGRATION.md).  There is no fallback: if the HIP library is missing, every product call
raises `NativeLibraryError`.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CBX_LIB_VARIANT=stamps selects the diagnostic build (tools/stamps.py); the product library otherwise
LIB_PATH = os.path.join(_HERE, "libcobrix_hip_%s.so" % os.environ["CBX_LIB_VARIANT"]
                        if os.environ.get("CBX_LIB_VARIANT") else "libcobrix_hip.so")

CBX_MAX_DIMS = 4
CBX_MAX_SEG_KEYS = 32
CBX_MAX_SEG_KEY_LEN = 32
CBX_MAX_SEG_LEVELS = 8
CBX_MAX_SEG_PREFIX = 64

# kinds / out types / flags (keep in sync with include/cobrix_hip.h)
K_STRING, K_STRING_ASCII, K_HEX, K_RAW, K_BCD, K_BINARY, K_ZONED = 1, 2, 3, 4, 5, 6, 7
K_ASCII_NUM, K_UTF16_BE, K_UTF16_LE = 8, 13, 14
K_FLOAT, K_DOUBLE, K_RECORD_ID, K_FILE_ID = 9, 10, 11, 12
O_I32, O_I64, O_DEC64, O_DEC128, O_F32, O_F64, O_STRING, O_BINARY = 1, 2, 3, 4, 5, 6, 7, 8
F_SIGNED, F_BIG_ENDIAN, F_EXPLICIT_DOT, F_INTEGRAL, F_IBM, F_LITTLE_ENDIAN_FP, F_DEPENDEE = (
    0x1, 0x2, 0x4, 0x8, 0x10, 0x20, 0x40)
F_LIST = 0x80
TRIM = {"none": 1, "left": 2, "right": 3, "both": 4}

CBX_OK, CBX_E_ARGUMENT, CBX_E_STATE, CBX_E_CAPACITY, CBX_E_HIP, CBX_E_UNSUPPORTED = 0, -1, -2, -3, -4, -5

OUT_WIDTH = {O_I32: 4, O_I64: 8, O_DEC64: 8, O_DEC128: 16, O_F32: 4, O_F64: 8}

# every symbol include/cobrix_hip.h declares
EXPORTED_SYMBOLS = ("cbx_abi_version", "cbx_last_error", "cbx_plan_create", "cbx_plan_destroy",
                    "cbx_string_bound", "cbx_string_view_geometry", "cbx_string_sizes_fixed", "cbx_decode_fixed", "cbx_decode_var",
                    "cbx_string_sizes_var", "cbx_plan_check", "cbx_frame_rdw", "cbx_frame_rdw_async", "cbx_frame_rdw_state",
                    "cbx_plan_set_profiling",
                    "cbx_plan_kernel_times", "cbx_plan_kernel_kind", "cbx_plan_frame_kind", "cbx_plan_specialize", "cbx_frame_text",
                    "cbx_sparse_index", "cbx_select_records", "cbx_decode_selected", "cbx_hier_select",
                    "cbx_hier_list_offsets", "cbx_plan_set_walk", "cbx_frame_var_occurs",
                    "cbx_plan_set_record_base", "cbx_frame_length_field", "cbx_plan_set_odo_counts",
                    "cbx_hier_dependee_counts", "cbx_hier_dependee_values", "cbx_plan_set_dep_seed", "cbx_views_to_utf8", "cbx_plan_pipeline")
ABI_VERSION = 20


class NativeLibraryError(RuntimeError):
    pass


class CbxError(RuntimeError):
    """Structural error reported by the library (IllegalArgument/IllegalState in the reference)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"cbx error {code}: {msg}")
        self.code = code


class CbxField(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("out_type", ctypes.c_int32), ("offset", ctypes.c_int32),
                ("size", ctypes.c_int32), ("precision", ctypes.c_int32), ("scale", ctypes.c_int32),
                ("scale_factor", ctypes.c_int32), ("out_precision", ctypes.c_int32),
                ("out_scale", ctypes.c_int32), ("flags", ctypes.c_int32), ("trim", ctypes.c_int32),
                ("n_dims", ctypes.c_int32), ("dim_count", ctypes.c_int32 * CBX_MAX_DIMS),
                ("dim_stride", ctypes.c_int32 * CBX_MAX_DIMS), ("dim_array", ctypes.c_int32 * CBX_MAX_DIMS),
                ("segment", ctypes.c_int32), ("column", ctypes.c_int32)]


class CbxArray(ctypes.Structure):
    _fields_ = [("max_count", ctypes.c_int32), ("min_count", ctypes.c_int32), ("dependee", ctypes.c_int32),
                ("segment", ctypes.c_int32), ("count_column", ctypes.c_int32), ("n_dims", ctypes.c_int32),
                ("parent", ctypes.c_int32), ("offsets_column", ctypes.c_int32)]


class CbxSegmentMap(ctypes.Structure):
    _fields_ = [("field_offset", ctypes.c_int32), ("field_size", ctypes.c_int32), ("n_keys", ctypes.c_int32),
                ("key_len", ctypes.c_int32 * CBX_MAX_SEG_KEYS),
                ("key", (ctypes.c_uint16 * CBX_MAX_SEG_KEY_LEN) * CBX_MAX_SEG_KEYS),
                ("key_segment", ctypes.c_int32 * CBX_MAX_SEG_KEYS),
                ("key_level", ctypes.c_int32 * CBX_MAX_SEG_KEYS),
                ("key_in_filter", ctypes.c_int32 * CBX_MAX_SEG_KEYS),
                ("key_is_int", ctypes.c_int32 * CBX_MAX_SEG_KEYS),
                ("key_int", ctypes.c_int64 * CBX_MAX_SEG_KEYS),
                ("field", ctypes.c_int32), ("field_is_int", ctypes.c_int32), ("n_levels", ctypes.c_int32),
                ("has_filter", ctypes.c_int32), ("level_column", ctypes.c_int32 * CBX_MAX_SEG_LEVELS),
                ("prefix_len", ctypes.c_int32), ("prefix", ctypes.c_uint8 * CBX_MAX_SEG_PREFIX)]


class CbxPlanOptions(ctypes.Structure):
    _fields_ = [("n_columns", ctypes.c_int32), ("file_id", ctypes.c_int32), ("has_segments", ctypes.c_int32),
                ("window_bytes", ctypes.c_int32), ("segment_column", ctypes.c_int32),
                ("jit_min_records", ctypes.c_int32), ("string_views", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("lut", ctypes.c_uint32 * 256),
                ("segments", CbxSegmentMap)]


class CbxColumn(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("data", ctypes.c_void_p), ("data_capacity", ctypes.c_int64), ("data_sizes", ctypes.c_void_p)]


class CbxRdwParams(ctypes.Structure):
    _fields_ = [("big_endian", ctypes.c_int32), ("adjustment", ctypes.c_int32),
                ("file_header_bytes", ctypes.c_int32), ("file_footer_bytes", ctypes.c_int32)]


class CbxIndexEntry(ctypes.Structure):
    _fields_ = [("offset_from", ctypes.c_int64), ("offset_to", ctypes.c_int64), ("record_index", ctypes.c_int64),
                ("file_id", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class CbxIndexParams(ctypes.Structure):
    _fields_ = [("records_per_entry", ctypes.c_int64), ("bytes_per_entry", ctypes.c_int64),
                ("subtract_size", ctypes.c_int32), ("header_bytes", ctypes.c_int32),
                ("has_file_header", ctypes.c_int32), ("hierarchical", ctypes.c_int32),
                ("file_id", ctypes.c_int32), ("reserved", ctypes.c_int32), ("start_bytes", ctypes.c_int64)]


class CbxSelection(ctypes.Structure):
    _fields_ = [("rec_off", ctypes.c_void_p), ("rec_len", ctypes.c_void_p), ("record_id", ctypes.c_void_p),
                ("segment", ctypes.c_void_p), ("seg_state", ctypes.c_void_p), ("file_id", ctypes.c_int32),
                ("footer_bytes", ctypes.c_int32)]


W_GROUP, W_PRIM = 0, 1
W_REDEFINED, W_REDEFINES = 0x1, 0x2


class CbxWalkNode(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("kind", "next", "child", "field", "array", "flags", "data_size",
                                                "actual_size", "segment", "dep_slot")]


class CbxWalkArray(ctypes.Structure):
    _fields_ = [("dep_slot", ctypes.c_int32), ("h_begin", ctypes.c_int32), ("h_end", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class CbxWalkHandler(ctypes.Structure):
    _fields_ = [("key_id", ctypes.c_int32), ("key_len", ctypes.c_int32), ("value", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("key", ctypes.c_uint8 * 64)]


class CbxHierParams(ctypes.Structure):
    _fields_ = [("n_segments", ctypes.c_int32), ("root_segment", ctypes.c_int32),
                ("parent", ctypes.c_int32 * CBX_MAX_SEG_KEYS), ("first_record_id", ctypes.c_int64),
                ("start_offset", ctypes.c_int32), ("flags", ctypes.c_int32), ("row_capacity", ctypes.c_int64)]


CBX_HIER_MAX_SEG, CBX_HIER_MAX_EVENTS, CBX_HIER_MAX_DEPS = 16, 32, 16
HIER_EVENT_END = -32768


class CbxHierDependee(ctypes.Structure):
    _fields_ = [("values", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("out_type", ctypes.c_int32),
                ("walk_slot", ctypes.c_int32)]


class CbxHierOdoArray(ctypes.Structure):
    _fields_ = [("dependee", ctypes.c_int32), ("out_row", ctypes.c_int32), ("min_count", ctypes.c_int32),
                ("max_count", ctypes.c_int32), ("first_counts", ctypes.c_void_p)]


class CbxHierWalk(ctypes.Structure):
    _fields_ = [("n_segments", ctypes.c_int32), ("root_segment", ctypes.c_int32),
                ("table_base", ctypes.c_int64 * (CBX_HIER_MAX_SEG + 1)),
                ("table_rows", ctypes.c_int64 * (CBX_HIER_MAX_SEG + 1)),
                ("child_offsets", ctypes.c_void_p * CBX_HIER_MAX_SEG),
                ("children", (ctypes.c_int8 * CBX_HIER_MAX_SEG) * CBX_HIER_MAX_SEG),
                ("events", (ctypes.c_int16 * CBX_HIER_MAX_EVENTS) * (CBX_HIER_MAX_SEG + 1)),
                ("seeds", ctypes.c_void_p)]


_lib = None


def lib_path() -> str:
    return LIB_PATH


def load():
    """Load the HIP library; raises NativeLibraryError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    P, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.cbx_abi_version.restype = i32
    L.cbx_last_error.restype = ctypes.c_char_p
    L.cbx_plan_create.argtypes = [P, i32, P, i32, P, ctypes.POINTER(P)]
    L.cbx_plan_destroy.argtypes = [P]
    L.cbx_plan_destroy.restype = None
    L.cbx_string_bound.argtypes = [P, i64, P]
    L.cbx_string_view_geometry.argtypes = [P, P, P]
    L.cbx_string_sizes_fixed.argtypes = [P, P, i64, i32, i32, P, P]
    L.cbx_plan_check.argtypes = [P, P]
    L.cbx_decode_fixed.argtypes = [P, P, i64, i32, i32, i64, P, P]
    L.cbx_decode_var.argtypes = [P, P, i64, P, P, i64, i32, i64, P, P]
    L.cbx_string_sizes_var.argtypes = [P, P, i64, P, P, i64, i32, P, P]
    L.cbx_frame_rdw.argtypes = [P, i64, P, i32, P, P, P, i64, P, P]
    L.cbx_frame_rdw_async.argtypes = [P, i64, P, i32, P, P, P, i64, P, i32, P]
    L.cbx_frame_rdw_state.argtypes = [P, P, P]
    L.cbx_frame_text.argtypes = [P, i64, i32, P, P, i64, P, P, P]
    L.cbx_plan_set_profiling.argtypes = [P, i32]
    L.cbx_plan_kernel_times.argtypes = [P, P, P, i32, P]
    L.cbx_plan_kernel_kind.argtypes = [P, P]
    L.cbx_plan_frame_kind.argtypes = [P, P]
    L.cbx_plan_specialize.argtypes = [P, P, i64, P, i32]
    L.cbx_sparse_index.argtypes = [P, P, i64, P, P, i64, P, P, i64, P, P]
    L.cbx_select_records.argtypes = [P, P, i64, P, P, i64, i32, P, i32, P, P, P]
    L.cbx_decode_selected.argtypes = [P, P, i64, P, i64, i32, P, P]
    for name, at in (("cbx_hier_select", [P, P, i64, P, P, i64, P, P, P, P, P, P]),
                     ("cbx_hier_list_offsets", [P, i64, i64, i64, i64, P, P]),
                     ("cbx_plan_set_walk", [P, P, i32, i32, P, P, i32, i32]),
                     ("cbx_frame_var_occurs", [P, P, i64, i64, P, P, i64, P, P, P]),
                     ("cbx_plan_set_record_base", [P, P]),
                     ("cbx_frame_length_field", [P, P, i64, i32, i32, i32, i32, P, P, i64, P, P]),
                     ("cbx_plan_set_odo_counts", [P, P, i64]),
                     ("cbx_hier_dependee_counts", [P, P, i32, P, i32, P, i64, P, P]),
                     ("cbx_hier_dependee_values", [P, P, i64, P, P, i64, i32, i32, P, P, P]),
                     ("cbx_plan_set_dep_seed", [P, P, i64, i32]),
                     ("cbx_views_to_utf8", [P, i64, P, i64, P, P, i64, P, P]),
                     ("cbx_plan_pipeline", [P, P, i32, i32])):
        if hasattr(L, name):   # (diagnostic builds of older revisions lack the newest entry points)
            getattr(L, name).argtypes = at
    if L.cbx_abi_version() != ABI_VERSION and not os.environ.get("CBX_LIB_VARIANT"):
        # (a diagnostic variant built from an older revision -- tools/build_variant.py -- is timed on the
        # entry points both revisions share)
        raise NativeLibraryError(f"{LIB_PATH}: ABI {L.cbx_abi_version()} != {ABI_VERSION}; rebuild it")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != CBX_OK:
        raise CbxError(rc, load().cbx_last_error().decode(errors="replace"))
