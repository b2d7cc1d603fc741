"""Summary of one workload's GPU evidence (tools/evidence.sh): the bench JSON line, the
rocprofv3 kernel trace of the SAME process and the PMC passes of a 1-step run.

* per kernel: calls, rocprof average over all calls, and the average over the timed steps only
  (dispatches warmup .. warmup + steps - 1: warm-up first, the end-to-end pass's chunks after);
* roofline recomputed from the trace: algorithmic bytes (from the bench line) / the traced average
  of the decode kernel over the timed steps, next to the bench's HIP-event figure;
* HBM traffic per step: FETCH_SIZE (KiB) x 2 for the kernels that read with 16-byte-per-lane
  streaming loads (MI355X_MICROARCH.md, HBM: gfx950 counts half of those), WRITE_SIZE as is, from
  the last dispatch of the kernel in the pass (the last KPS dispatches, summed, when the step decodes
  its shard in KPS batches);
* SQ counters per launch of each cbx kernel (the last dispatch).
Usage: prof_summary.py <workload dir> -> JSON on stdout."""
import collections
import csv
import glob
import gzip
import json
import os
import sys

D = sys.argv[1]
# kernels whose reads are 16-byte-per-lane streaming loads (register staging or LDS-DMA `buffer_load_dwordx4
# ... lds`): FETCH_SIZE counts half of those bytes on gfx950 (MI355X_MICROARCH.md, HBM)
STAGED16 = ("cbx_jit_decode", "cbx_jit_count", "cbx_jit_list", "cbx::decode_kernel", "cbx::list_kernel",
            "cbx::rdw_wave_kernel")


def base(name: str) -> str:
    """Kernel name without its parameter list (template arguments kept: list_kernel<false> and
    list_kernel<true> are two launches of a step)."""
    return name.split("(")[0].replace("void ", "", 1).strip()


def rows(pattern):
    """CSV rows of the files matching pattern (or their gzip-compressed copies, pattern + ".gz")."""
    out = []
    for f in glob.glob(os.path.join(D, pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    for f in glob.glob(os.path.join(D, pattern + ".gz"), recursive=True):
        with gzip.open(f, "rt") as g:
            out += list(csv.DictReader(g))
    return out


bench = json.loads([ln for ln in open(os.path.join(D, "bench.json")) if ln.startswith("{")][-1])
steps = bench["steps"]
trace = rows("trace/**/run_kernel_trace.csv")
per = collections.defaultdict(list)
spans = collections.defaultdict(list)   # kernel -> [(start, end)] in ns, launch order
for r in sorted(trace, key=lambda r: int(r["Start_Timestamp"])):
    per[base(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    spans[base(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
# launches of the record kernel per step: a fixed-length shard decoded in batches (C3's 64 GB job)
# runs one call per batch
KPS = int(bench["config"].get("batches_per_gpu", 1) or 1)
kernels = {}
for k, d in per.items():
    if not (k.startswith("cbx") or "cbx" in k):
        continue
    w0 = bench.get("warmup", 0) * KPS     # warm-up launches, the timed steps', then end-to-end chunks
    timed = d[w0:w0 + steps * KPS] if len(d) >= w0 + steps * KPS else d
    kernels[k] = {"calls": len(d), "avg_ms_all": round(sum(d) / len(d), 4), "avg_ms_timed_steps": round(sum(timed) / len(timed), 4),
                  "max_ms": round(max(d), 4)}

dec = [k for k in kernels if k.startswith("cbx_jit_decode") or k == "cbx::decode_kernel" or k == "cbx::walk_kernel"]
alg = bench["roofline"]["algorithmic_bytes_per_launch"]
check = {}
if dec:
    k = dec[0]
    # the bench's decode time (HIP events) covers the record kernel, the list kernels after it and,
    # in the Utf8 layout, the count pass and its scan before it.  Each part kernel is attributed to
    # the timed steps by its side of the record kernel: a list kernel from the START of the first
    # timed record launch up to the first record-kernel launch of ANY kind after the last timed one
    # (the end-to-end pieces may run the table-driven kernel), a count/scan kernel from the END of
    # the last warm-up record launch up to the START of the last timed one -- so the warm-up step's
    # list kernels and the end-to-end pieces' parts (smaller batches) do not count
    w0 = bench.get("warmup", 0) * KPS
    sp = spans[k]
    n_t = min(steps, (len(sp) - w0) // KPS)     # timed steps in the trace
    first, last = sp[w0][0], sp[w0 + n_t * KPS - 1][0]
    lo = sp[w0 - 1][1] if w0 > 0 else 0
    after = [s0 for x in dec for s0, _ in spans[x] if s0 > last]
    hi = min(after) if after else float("inf")
    window = {k: (first - 1, last + 1)}
    for x in kernels:
        if x.startswith(("cbx::list_kernel", "cbx_jit_list", "cbx::fixup_kernel")):   # (the bench's time includes the fixup pass)
            window[x] = (first, hi)
    if "cbx_jit_count" in kernels or bench["config"].get("string_layout", "").startswith("Arrow Utf8"):
        for x in kernels:
            if x.startswith(("cbx_jit_count", "cbx::scan_")):
                window[x] = (lo, last)
    parts, t = [], 0.0
    piped = bench["roofline"].get("timing", "").startswith("wall time")
    if piped:
        # batches of two plans overlapped on two streams (cbx_plan_pipeline): the bench times the step's
        # wall clock, so the trace's figure is the span of the timed steps' cbx kernels per step
        lo_s, hi_e = float("inf"), 0
        for x, (a_, b_) in window.items():
            for s0, e in spans[x]:
                if a_ < s0 < b_:
                    lo_s, hi_e = min(lo_s, s0), max(hi_e, e)
                    if x not in parts:
                        parts.append(x)
        t = (hi_e - lo_s) / 1e6 / n_t if parts else 0.0
    for x, (a_, b_) in window.items():
        if piped:
            break
        d_in = [(e - s0) / 1e6 for s0, e in spans[x] if a_ < s0 < b_]
        if d_in:
            parts.append(x)
            t += sum(d_in) / n_t
    frac = alg / (t * 1e-3) / 1e9 / bench["roofline"]["peak"]
    check = {"kernel": " + ".join(parts), "rocprof_ms": round(t, 4),
             "hip_event_ms": round(bench["kernel_ms"]["decode_kernel"] + bench["kernel_ms"].get("post_kernels", 0.0), 4),
             "frac_rocprof": round(frac, 4),
             "frac_bench": bench["roofline"]["frac"],
             "agree_within": round(abs(frac - bench["roofline"]["frac"]) / bench["roofline"]["frac"], 4)}

pmc = collections.defaultdict(lambda: collections.defaultdict(dict))   # kernel -> counter -> dispatch -> value
for i in range(1, 9):
    for r in rows(f"pmc{i}/**/run_counter_collection.csv"):
        k = base(r["Kernel_Name"])
        if "cbx" not in k:
            continue
        d = pmc[k][r["Counter_Name"]]
        d[int(r["Dispatch_Id"])] = d.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
counters, traffic = {}, {}
for k, cs in pmc.items():
    # the last step of the 1-step pass: its KPS dispatches (one per batch) summed; one dispatch otherwise
    last = {c: sum(v[d] for d in sorted(v)[-KPS:]) if len(v) >= KPS else v[max(v)] for c, v in cs.items()}
    counters[k] = {c: int(v) for c, v in sorted(last.items())}
    if "FETCH_SIZE" in last or "WRITE_SIZE" in last:
        f = last.get("FETCH_SIZE", 0.0) * 1024.0
        w = last.get("WRITE_SIZE", 0.0) * 1024.0
        scale = 2.0 if k.startswith(STAGED16) else 1.0
        traffic[k] = {"fetch_bytes_raw": int(f), "fetch_bytes": int(f * scale), "write_bytes": int(w),
                      "traffic_bytes": int(f * scale + w), "fetch_scale": scale}
    if "SQ_LDS_BANK_CONFLICT" in last and last.get("SQ_ACTIVE_INST_LDS"):
        counters[k]["lds_conflict_per_active_lds"] = round(last["SQ_LDS_BANK_CONFLICT"] / last["SQ_ACTIVE_INST_LDS"], 3)
    if last.get("SQ_LDS_IDX_ACTIVE") and last.get("GRBM_GUI_ACTIVE"):
        # LDS-array cycles per CU over the kernel's cycles (GRBM_GUI_ACTIVE sums the 8 XCDs); raw
        # counter units as rocprofv3 reports them
        counters[k]["lds_idx_active_per_cu_cycle"] = round(last["SQ_LDS_IDX_ACTIVE"] / (last["GRBM_GUI_ACTIVE"] / 8.0 * 256.0), 3)
    if last.get("SQ_WAVE_CYCLES"):
        counters[k]["wait_any_frac"] = round(last.get("SQ_WAIT_ANY", 0) / last["SQ_WAVE_CYCLES"], 3)
# the decode chain's traffic (the kernels the HIP-event window covers; framing kernels apart)
chain = check.get("kernel", "").split(" + ") if check else []
dec_traffic = sum(v["traffic_bytes"] for k, v in traffic.items() if k in chain)
print(json.dumps({"workload": bench["config"]["workload"][:60], "records": bench["config"]["records_per_gpu"],
                  "bench": {k: bench[k] for k in ("value", "ms_per_step", "kernel_ms", "roofline", "hbm_frac_step")},
                  "kernels": kernels, "check": check, "traffic": traffic,
                  "decode_traffic_bytes": dec_traffic or None,
                  "decode_traffic_over_algorithmic": round(dec_traffic / alg, 3) if dec_traffic else None,
                  "counters": counters}, indent=1))
