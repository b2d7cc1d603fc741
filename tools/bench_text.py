"""Time cbx_frame_text (is_text framing) on synthetic text resident in HBM.

Lines of 20-200 printable bytes ending in LF (every 7th CR LF); prints framing GB/s and
records/s.  Usage: python tools/bench_text.py [--gb 4] [--iters 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cobrix_amd import native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--record-size", type=int, default=200)
    a = ap.parse_args()
    n = int(a.gb * 1e9)
    g = torch.Generator(device="cuda").manual_seed(3)
    data = torch.randint(65, 91, (n + a.record_size + 64,), dtype=torch.uint8, device="cuda", generator=g)
    # line ends: gaps of 20-200 bytes
    gaps = torch.randint(21, 201, (n // 20 + 1,), device="cuda", generator=g)
    pos = torch.cumsum(gaps, 0)
    pos = pos[pos < n]
    data[pos] = 10
    crlf = pos[::7]
    data[crlf - 1] = 13
    data[n:] = 0
    torch.cuda.synchronize()
    cap = n // 20 + 16
    off = torch.empty(cap, dtype=torch.int64, device="cuda")
    ln = torch.empty(cap, dtype=torch.int32, device="cuda")
    L = N.load()
    st = torch.cuda.current_stream()
    cnt, vb = ctypes.c_int64(0), ctypes.c_int64(0)

    def run():
        N.check(L.cbx_frame_text(data.data_ptr(), n, a.record_size, off.data_ptr(), ln.data_ptr(), cap,
                                 ctypes.byref(cnt), ctypes.byref(vb), ctypes.c_void_p(st.cuda_stream)))

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(json.dumps({"bytes": n, "records": cnt.value, "ms": round(dt * 1e3, 3), "GB_per_s": round(n / dt / 1e9, 1),
                      "records_per_s": round(cnt.value / dt, 1)}))


if __name__ == "__main__":
    main()
