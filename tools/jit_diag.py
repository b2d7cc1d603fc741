"""Diagnostic: source, hipRTC compile time and one decode of a golden case's specialised kernel.
Usage: python tools/jit_diag.py CASE [large|views|utf8] -> gpurun_out/jitdiag_<case>_<layout>.hip"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    assert torch.cuda.is_available()
    import golden_cases as GC
    from cobrix_amd import native as N
    from cobrix_amd.reader import FixedLenNestedReader
    name = sys.argv[1]
    layout = sys.argv[2] if len(sys.argv) > 2 else "large"
    case = GC.CASES[name]
    p, _ = GC.params(case)
    p.string_views = layout == "views"
    p.string_utf8 = layout == "utf8"
    p.jit_min_records = 1
    L = N.load()
    rd = FixedLenNestedReader(GC.copybook_text(case), p)
    buf = ctypes.create_string_buffer(16 << 20)
    n = ctypes.c_int64()
    rc = L.cbx_plan_specialize(rd.native.handle, buf, len(buf), ctypes.byref(n), 0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"jitdiag_{name}_{layout}.hip"), "w") as f:
        f.write(buf.value.decode())
    print("source rc", rc, "bytes", n.value, flush=True)
    t0 = time.time()
    rc = L.cbx_plan_specialize(rd.native.handle, buf, len(buf), ctypes.byref(n), 1)
    print("compile rc", rc, "s", round(time.time() - t0, 2), L.cbx_last_error().decode()[:500] if rc else "", flush=True)
    t0 = time.time()
    b = rd.decode(GC.data_bytes(case))
    torch.cuda.synchronize()
    k = ctypes.c_int32()
    L.cbx_plan_kernel_kind(rd.native.handle, ctypes.byref(k))
    print("decode s", round(time.time() - t0, 2), "kind", k.value, "rows", b.n_rec, flush=True)


if __name__ == "__main__":
    main()
