"""Diagnostic: decode the test5 layout as fixed-length records with the specialised kernel forced
and print why it was not used (cbx_plan_kernel_kind + cbx_last_error) and its source."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    assert torch.cuda.is_available()   # torch first: the library's own HIP calls come after its runtime is up
    import goldens as G
    from cobrix_amd import native as N
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters
    cb_text = G.read("test5_copybook.cob").decode()
    p = ReaderParameters(segment_field="SEGMENT-ID", segment_id_redefine_map={"C": "STATIC-DETAILS", "P": "CONTACTS"},
                         start_offset=3, end_offset=1, jit_min_records=1)
    rd = FixedLenNestedReader(cb_text, p)
    data = bytes(rd.get_record_size() * 100)
    rd.decode(data)
    k = ctypes.c_int32(-1)
    L = N.load()
    N.check(L.cbx_plan_kernel_kind(rd.native.handle, ctypes.byref(k)))
    print("kind", k.value, L.cbx_last_error().decode(errors="replace")[:4000])
    buf = ctypes.create_string_buffer(1 << 20)
    n = ctypes.c_int64()
    L.cbx_plan_specialize(rd.native.handle, buf, len(buf), ctypes.byref(n), 0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    open(os.path.join(ROOT, "gpurun_out", "jit_why.hip"), "w").write(buf.value.decode())


if __name__ == "__main__":
    main()
