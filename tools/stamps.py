"""Diagnostic: where the contiguous decode loop spends its wave-cycles (s_memtime stamps).

Builds nothing: run `tools/build_stamps.sh` first (hipcc -DCBX_STAMPS -> libcobrix_hip_stamps.so).
Prints each segment's share of the summed wave time.  Shares only: the stamps' waits forbid
overlaps the product kernel has, so the diagnostic build's run time is not quoted anywhere.
"""
import argparse
import ctypes
import os
import sys

os.environ["CBX_LIB_VARIANT"] = "stamps"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

SEG = ["stage (prefetched loads -> LDS)", "prefetch issue", "prologue", "strings", "numerics", "tile end sync"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--variant", default="full")
    ap.add_argument("--views", action="store_true")
    a = ap.parse_args()
    import torch
    from cobrix_amd import native as N
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, _alloc_columns, string_capacity
    from cobrix_amd.synth import SYN200_COPYBOOK, syn200
    from prof_variants import variant, VARIANTS
    rec = syn200(a.records, device="cuda").view(-1)
    L = N.load()
    L.cbx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rd = FixedLenNestedReader(variant(SYN200_COPYBOOK, VARIANTS[a.variant]), ReaderParameters(string_views=a.views))
    cols, cs = _alloc_columns(rd.plan, a.records, string_capacity(rd.native, a.records), rec.device)
    h = rd.native.handle
    out = (ctypes.c_uint64 * 8)()
    N.check(L.cbx_decode_fixed(h, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
    N.check(L.cbx_debug_stamps(h, out))
    N.check(L.cbx_decode_fixed(h, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
    N.check(L.cbx_debug_stamps(h, out))
    tot = sum(out[:6])
    print(f"variant={a.variant} waves={out[7]} total_wave_clk={tot}")
    for k, name in enumerate(SEG):
        print(f"  {name:34s} {100.0 * out[k] / max(tot, 1):6.2f} %  ({out[k] / max(out[7], 1) / 1e3:9.1f} k clk/wave)")


if __name__ == "__main__":
    main()
