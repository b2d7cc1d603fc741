"""Diagnostic: where a decode kernel's waves spend their cycles (s_memtime stamps).

Builds nothing: run `tools/build_stamps.sh` first (hipcc -DCBX_STAMPS -> libcobrix_hip_stamps.so; the
specialised kernels then compile with -DCBX_STAMPS too).  Prints each segment's share of the summed
wave time.  Shares only: the stamps' waits forbid overlaps the product kernel has, so the diagnostic
build's run time is not quoted anywhere.

usage: python tools/stamps.py [--workload syn200|synstr200] [--records N] [--views]
  syn200 / synstr200 (views or Utf8 count + decode): the contiguous decode loop's segments."""
import argparse
import ctypes
import os
import sys

os.environ["CBX_LIB_VARIANT"] = "stamps"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SEG = ["stage (prefetched loads -> LDS)", "prefetch issue", "prologue", "strings", "numerics", "tile end sync"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="syn200", choices=["syn200", "synstr200"])
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--views", action="store_true")
    a = ap.parse_args()
    import torch
    from cobrix_amd import native as N
    from cobrix_amd import synth
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, _alloc_columns, string_capacity
    if a.workload == "syn200":
        rec = synth.syn200(a.records, device="cuda").view(-1)
        rd = FixedLenNestedReader(synth.SYN200_COPYBOOK, ReaderParameters(string_views=a.views))
    else:
        rec = synth.synstr200(a.records, seed=20261017, device="cuda").view(-1)
        rd = FixedLenNestedReader(synth.SYNSTR200_COPYBOOK, ReaderParameters(
            ebcdic_code_page="cp037", string_views=a.views, string_utf8=not a.views))
    L = N.load()
    L.cbx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cols, cs = _alloc_columns(rd.plan, a.records, string_capacity(rd.native, a.records), rec.device)
    h = rd.native.handle
    out = (ctypes.c_uint64 * 8)()
    N.check(L.cbx_decode_fixed(h, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
    torch.cuda.synchronize()
    N.check(L.cbx_debug_stamps(h, out))   # (reads and resets: the second call alone below)
    N.check(L.cbx_decode_fixed(h, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
    torch.cuda.synchronize()
    N.check(L.cbx_debug_stamps(h, out))
    d = list(out)
    kind = ctypes.c_int32()
    N.check(L.cbx_plan_kernel_kind(h, ctypes.byref(kind)))
    names = SEG
    tot = sum(d[:6])
    print(f"workload={a.workload} kind={kind.value} waves={d[7]} total_wave_clk={tot}")
    for k, name in enumerate(names):
        print(f"  {name:34s} {100.0 * d[k] / max(tot, 1):6.2f} %  ({d[k] / max(d[7], 1) / 1e3:9.1f} k clk/wave)")


if __name__ == "__main__":
    main()
