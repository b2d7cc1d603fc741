"""Experiment: do two SYNSTR200 Utf8 decode chains (count + scan + decode) on two streams overlap?

Two readers (plans) decode two 25 M-record halves of one 50 M batch, each on its own stream, with
the resident workgroups per CU of each kernel capped (CBX_MAX_BLOCKS_PER_CU) so both fit on the
chip at once; prints the wall time of the pair (HIP events on the launching stream, both streams
joined) against one 50 M chain on one stream.  A pair well under the single chain says the count
pass (HBM-read bound) and the decode (issue bound) gain from running side by side.

usage: python tools/overlap_ab.py [cap ...]   (default caps: 8 4 3 2)"""
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
    caps = [int(x) for x in sys.argv[1:]] or [8, 4, 3, 2]
    n = 50_000_000
    h = n // 2
    rec = synth.synstr200(n, seed=20261017, device="cuda").view(-1)
    L = N.load()
    torch.cuda.synchronize()

    def reader(m):
        rd = FixedLenNestedReader(synth.SYNSTR200_COPYBOOK, ReaderParameters(ebcdic_code_page="cp037", string_utf8=True))
        cols, cs = _alloc_columns(rd.plan, m, string_capacity(rd.native, m), rec.device)
        return rd, cols, cs

    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    # one chain over the whole batch, default occupancy
    os.environ.pop("CBX_MAX_BLOCKS_PER_CU", None)
    rd, cols, cs = reader(n)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = 1e9
    for it in range(5):
        ev[0].record(s0)
        N.check(L.cbx_decode_fixed(rd.native.handle, rec.data_ptr(), n, 200, 0, 0, cs, ctypes.c_void_p(s0.cuda_stream)))
        ev[1].record(s0)
        torch.cuda.synchronize()
        if it:
            best = min(best, ev[0].elapsed_time(ev[1]))
    print(json.dumps({"mode": "single", "records": n, "ms": round(best, 3)}), flush=True)
    del cols, cs
    rd.close()
    for cap in caps:
        os.environ["CBX_MAX_BLOCKS_PER_CU"] = str(cap)
        ra, ca, csa = reader(h)
        rb, cb, csb = reader(n - h)
        best = 1e9
        for it in range(5):
            ev[0].record(s0)
            s1.wait_stream(s0)
            N.check(L.cbx_decode_fixed(ra.native.handle, rec.data_ptr(), h, 200, 0, 0, csa, ctypes.c_void_p(s0.cuda_stream)))
            N.check(L.cbx_decode_fixed(rb.native.handle, rec.data_ptr() + 200 * h, n - h, 200, 0, 0, csb,
                                       ctypes.c_void_p(s1.cuda_stream)))
            s0.wait_stream(s1)
            ev[1].record(s0)
            torch.cuda.synchronize()
            if it:
                best = min(best, ev[0].elapsed_time(ev[1]))
        print(json.dumps({"mode": "two streams", "cap_blocks_per_cu": cap, "records": n, "ms": round(best, 3)}), flush=True)
        del ca, csa, cb, csb
        ra.close()
        rb.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
