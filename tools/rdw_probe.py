"""RDW framing probe (diagnostic): C5 (wide_odo) data framed by cbx_frame_rdw with CBX_RDW_DEBUG=1 (the
library prints how many speculated chunk entries the fix rounds changed), timed, and checked against the
generator's header offsets.  usage: CBX_RDW_DEBUG=1 [CBX_LIB_VARIANT=x] python tools/rdw_probe.py [N_ROOTS]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cobrix_amd import synth
    from cobrix_amd.options import parse_options
    from cobrix_amd.reader import VarLenNestedReader
    n_roots = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    raw, hdr = synth.wide_odo(n_roots, device="cuda")
    p, _ = parse_options({"is_record_sequence": "true", "is_rdw_big_endian": "false"})
    rd = VarLenNestedReader(synth.WIDE_ODO_COPYBOOK, p)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        off, ln = rd.frame(raw, raw.numel())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = off.numel() == hdr.numel() and bool(torch.equal(off.cpu(), hdr.cpu() + 4))
        print(f"rep {rep}: {raw.numel() / 1e6:.0f} MB, {off.numel()} records, {dt * 1e3:.2f} ms, matches generator: {ok}", flush=True)


if __name__ == "__main__":
    main()
