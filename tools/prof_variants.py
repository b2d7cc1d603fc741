"""Cost breakdown: decode-kernel time for variants of the SYN200 layout over the same bytes.

Variants blank out field groups with FILLER (not decoded) so the difference in kernel time
attributes cost to staging, numeric fields and the string field.  Prints one line per variant.
"""
import argparse
import ctypes
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def variant(cb: str, keep) -> str:
    out = []
    for line in cb.split("\n"):
        m = re.match(r"(\s+05\s+)([A-Z0-9-]+)(\s+.*)", line)
        if m and m.group(2) != "FILLER" and not keep(m.group(2)):
            line = m.group(1) + "FILLER" + m.group(3)
        out.append(line)
    return "\n".join(out)


VARIANTS = {
    "full": lambda n: True,
    "no_string": lambda n: n != "NAME",
    "string_only": lambda n: n == "NAME",
    "bcd8_only": lambda n: n.startswith("AMT"),
    "zoned_only": lambda n: n.startswith("ZN") or n.startswith("ZD"),
    "binary_only": lambda n: n in ("REC-ID", "BR-ID", "ACCT-NO", "CUST-KEY"),
    "one_field": lambda n: n == "REC-ID",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default=None, help="run one variant (for rocprofv3 passes)")
    ap.add_argument("--views", action="store_true", help="string columns in the string-view layout")
    a = ap.parse_args()
    import torch
    from cobrix_amd import native as N
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, _alloc_columns, string_capacity
    from cobrix_amd.synth import SYN200_COPYBOOK, syn200
    rec = syn200(a.records, device="cuda").view(-1)
    L = N.load()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, keep in VARIANTS.items():
        if a.only and name != a.only:
            continue
        rd = FixedLenNestedReader(variant(SYN200_COPYBOOK, keep), ReaderParameters(string_views=a.views))
        cols, cs = _alloc_columns(rd.plan, a.records, string_capacity(rd.native, a.records), rec.device)
        h = rd.native.handle
        N.check(L.cbx_decode_fixed(h, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
        N.check(L.cbx_plan_set_profiling(h, 1))
        for _ in range(a.iters):
            N.check(L.cbx_decode_fixed(h, rec.data_ptr(), a.records, 200, 0, 0, cs, st))
        dec = (ctypes.c_float * a.iters)()
        fix = (ctypes.c_float * a.iters)()
        nc = ctypes.c_int32()
        N.check(L.cbx_plan_kernel_times(h, dec, fix, a.iters, ctypes.byref(nc)))
        N.check(L.cbx_plan_check(h, st))
        d = sorted(dec[: nc.value])[nc.value // 2]
        print(f"{name:12s} cols={rd.plan.n_columns:3d} decode_ms={d:.4f} per_rec_ns={d * 1e6 / a.records:.3f}", flush=True)
        rd.close()
        del cols


if __name__ == "__main__":
    main()
