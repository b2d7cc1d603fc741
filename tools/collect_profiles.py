"""Copy one gpu_r0N.sh run's evidence from gpurun_out/r0N_<TAG>/ into profiles/r0N_<TAG>/ (tracked):
per workload the bench JSON line, the rocprofv3 kernel stats (cbx kernels + the totals of the rest),
the PMC summary (tools/prof_summary.py) and traffic_<tag>.json, the per-launch HBM bytes of the
decode kernels that bench.py's measured_traffic() reads.  Usage: collect_profiles.py TAG [ROUND, default r04]"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
rnd = sys.argv[2] if len(sys.argv) > 2 else "r04"
src = os.path.join(ROOT, "gpurun_out", f"{rnd}_{tag}")
dst = os.path.join(ROOT, "profiles", f"{rnd}_{tag}")
os.makedirs(dst, exist_ok=True)
for w in sorted(os.listdir(src)):
    d = os.path.join(src, w)
    if not os.path.isfile(os.path.join(d, "summary.json")):
        if os.path.isfile(os.path.join(d, "gpu_tests.log")) or w.endswith(".log"):
            continue
        continue
    out = os.path.join(dst, w)
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(d, "summary.json"), os.path.join(out, "summary.json"))
    bench = [ln for ln in open(os.path.join(d, "bench.json")) if ln.startswith("{")][-1]
    with open(os.path.join(out, "bench.json"), "w") as f:
        f.write(bench)
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        rows = list(csv.DictReader(open(stats)))
        keep = [r for r in rows if "cbx" in r["Name"]]
        other = [r for r in rows if "cbx" not in r["Name"]]
        with open(os.path.join(out, "kernel_stats.csv"), "w", newline="") as f:
            wr = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            wr.writeheader()
            for r in keep:
                wr.writerow(r)
            if other:   # torch's generator / setup kernels, summed
                tot = sum(int(r["TotalDurationNs"]) for r in other)
                calls = sum(int(r["Calls"]) for r in other)
                wr.writerow({**{k: "" for k in rows[0]}, "Name": f"(other: {len(other)} non-cbx kernels, setup)",
                             "Calls": calls, "TotalDurationNs": tot})
    s = json.load(open(os.path.join(d, "summary.json")))
    b = json.loads(bench)
    if s.get("decode_traffic_bytes"):
        strings = "views" if "views" in b["config"]["string_layout"] else (
            "offsets" if "Utf8" in b["config"]["string_layout"] else "large")
        slots = "" if b["config"]["occurs_layout"].startswith("Arrow lists") else "_slots"
        wl = {"C2": "syn200", "C3": "synstr200", "C4": "rdw_narrow", "C5": "wide_odo"}[b["config"]["baseline_config"]]
        t = f"{wl}_{strings}{slots}_{b['config']['records_per_gpu']}"
        with open(os.path.join(dst, f"traffic_{t}.json"), "w") as f:
            json.dump({"traffic_bytes": s["decode_traffic_bytes"], "kernels": s["traffic"],
                       "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, 1-step run, last dispatch); "
                                 "FETCH_SIZE x 2 for kernels reading with 16-byte/lane loads (MI355X_MICROARCH.md)"}, f, indent=1)
print("collected", dst)
