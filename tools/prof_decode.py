"""Profiling driver: decode N SYN200 records `--iters` times (for rocprofv3 runs)."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=5_000_000)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--offsets", action="store_true", help="large-string layout instead of string views (bench default)")
    a = ap.parse_args()
    import torch
    from cobrix_amd import native as N
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, _alloc_columns, string_capacity
    from cobrix_amd.synth import SYN200_COPYBOOK, syn200
    rec = syn200(a.records, device="cuda").view(-1)
    rd = FixedLenNestedReader(SYN200_COPYBOOK, ReaderParameters(window_bytes=a.window, string_views=not a.offsets, occurs_lists=True))
    L = N.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cols, cs = _alloc_columns(rd.plan, a.records, string_capacity(rd.native, a.records), rec.device)
    for _ in range(a.iters):
        N.check(L.cbx_decode_fixed(rd.native.handle, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
    N.check(L.cbx_plan_check(rd.native.handle, st))
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
