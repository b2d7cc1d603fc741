"""Dump the specialised kernels' sources of a bench workload (CBX_JIT_DUMP) for offline ISA study
(tools/jit_isa.py): a small batch of the workload's layout decoded once per string layout given.

usage: python tools/jit_dump.py OUTDIR syn200|synstr200|rdw_narrow|wide_odo [views|utf8|large ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    out, work = sys.argv[1], sys.argv[2]
    layouts = sys.argv[3:] or ["views"]
    import torch
    from cobrix_amd import synth
    from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters, VarLenNestedReader
    for lay in layouts:
        os.environ["CBX_JIT_DUMP"] = os.path.join(out, f"{work}_{lay}")
        os.makedirs(os.environ["CBX_JIT_DUMP"], exist_ok=True)
        kw = dict(string_views=lay == "views", string_utf8=lay == "utf8", jit_min_records=1)
        if work in ("syn200", "synstr200"):
            n = 200_000
            cb = synth.SYN200_COPYBOOK if work == "syn200" else synth.SYNSTR200_COPYBOOK
            rec = (synth.syn200 if work == "syn200" else synth.synstr200)(n, device="cuda").view(-1)
            rd = FixedLenNestedReader(cb, ReaderParameters(ebcdic_code_page="cp037", **kw))
            rd.decode_device(rec, n * 200)
        else:
            if work == "rdw_narrow":
                raw, _ = synth.rdw_narrow(300_000, device="cuda")
                cb, segs = synth.RDW_NARROW_COPYBOOK, synth.RDW_NARROW_SEGMENTS
            else:
                raw, _ = synth.wide_odo(2_000, device="cuda")
                cb, segs = synth.WIDE_ODO_COPYBOOK, synth.WIDE_ODO_SEGMENTS
            rd = VarLenNestedReader(cb, ReaderParameters(is_record_sequence=True, segment_field="SEGMENT-ID",
                                                         segment_id_redefine_map=segs, generate_record_id=True,
                                                         occurs_lists=True, **kw))
            off, ln = rd.frame(raw, raw.numel())
            rd.decode_device(raw, raw.numel(), off, ln)
        torch.cuda.synchronize()
        print(work, lay, sorted(os.listdir(os.environ["CBX_JIT_DUMP"])), flush=True)


if __name__ == "__main__":
    main()
