"""A/B timing of decode variants on one 50 M-record SYNSTR200 batch in the Arrow Utf8 layout (GPU), or
on a SYN200 batch with --syn200.

Each variant is a set of environment knobs read by the library at compile / launch time
(CBX_JIT_DEFINES, CBX_UTF8_ONEPASS, CBX_LB_SPIN, CBX_MAX_BLOCKS_PER_CU, ...); every variant gets
a fresh reader (plan), so its kernels are compiled with its knobs.  Prints one JSON line per variant:
decode-chain ms per call (HIP events), kernel kind, look-back recounts.

usage: python tools/u8_ab.py [--syn200] [records] [VAR=VAL;VAR=VAL ...]...   (a bare "-" = no knobs)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cobrix_amd import native as N
    from cobrix_amd import synth
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, _alloc_columns, string_capacity
    args = sys.argv[1:]
    syn = "--syn200" in args
    args = [a for a in args if a != "--syn200"]
    n = int(args[0]) if args and args[0].isdigit() else 50_000_000
    variants = [a for a in args if not a.isdigit()] or ["-"]
    rec = (synth.syn200(n, seed=20261015, device="cuda") if syn else synth.synstr200(n, seed=20261017, device="cuda")).view(-1)
    torch.cuda.synchronize()
    L = N.load()
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    base_env = dict(os.environ)
    for v in variants:
        os.environ.clear()
        os.environ.update(base_env)
        knobs = {} if v == "-" else dict(kv.split("=", 1) for kv in v.split(";") if kv)
        os.environ.update(knobs)
        rd = (FixedLenNestedReader(synth.SYN200_COPYBOOK, ReaderParameters(string_views=True)) if syn else
              FixedLenNestedReader(synth.SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_utf8=True)))
        h = rd.native.handle
        cols, cs = _alloc_columns(rd.plan, n, string_capacity(rd.native, n), rec.device)
        N.check(L.cbx_plan_set_profiling(h, 1))
        times = []
        for it in range(6):
            N.check(L.cbx_decode_fixed(h, rec.data_ptr(), n, 200, 0, 0, cs, sp))
        torch.cuda.synchronize()
        dec = (ctypes.c_float * 16)()
        fix = (ctypes.c_float * 16)()
        nc = ctypes.c_int32()
        N.check(L.cbx_plan_kernel_times(h, dec, fix, 16, ctypes.byref(nc)))
        times = [round(dec[i], 3) for i in range(nc.value)]
        kind = ctypes.c_int32()
        N.check(L.cbx_plan_kernel_kind(h, ctypes.byref(kind)))
        rc = ctypes.c_int64()
        N.check(L.cbx_plan_lookback_stats(h, ctypes.byref(rc), sp))
        status = L.cbx_plan_check(h, sp)
        print(json.dumps({"variant": knobs, "records": n, "decode_ms": times, "best_ms": min(times[1:] or times),
                          "kind": kind.value, "recounts": rc.value, "check": status}), flush=True)
        del cols, cs
        rd.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
