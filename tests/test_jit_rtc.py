"""The copybook-specialised kernels are compiled at run time by hipRTC (cobrix_amd/csrc/cbx_jit.h),
whose headers differ from hipcc's (no <cstdint> extras such as uintptr_t, no hip_runtime.h): a device
header that only hipcc accepts makes every specialised kernel fall back to the table-driven one on
the GPU.  These CPU tests compile, through hipRTC (no device needed), sources of the shapes
jit_source / jit_list_source generate -- the record kernel in the three string layouts and in the
Utf8 count mode, and the list kernel -- against the headers the library bundles.

Two compilers: the image's (/opt/rocm) and the one bundled with torch.  Both have the soname
libhiprtc.so.7, so in a process that imported torch first (every product process) the library's
hipRTC calls resolve to torch's -- an older LLVM, which crashed (SIGSEGV) on the cooperative kernel's
constant image address before coop_lds made it opaque.  Each compile runs in a child process, so a
compiler crash fails its test instead of the test run."""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cobrix_amd", "csrc")
HEADERS = [("cobrix_hip.h", os.path.join(ROOT, "include", "cobrix_hip.h"))] + [
    (n, os.path.join(CSRC, n)) for n in ("cbx_decode.h", "cbx_internal.h", "cbx_device.h", "cbx_list.h", "cbx_walk.h",
                                          "cbx_chain.h")]


def _torch_hiprtc() -> str | None:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    hits = glob.glob(os.path.join(list(spec.submodule_search_locations)[0], "lib", "libhiprtc.so*"))
    return hits[0] if hits else None


COMPILERS = [p for p in ("/opt/rocm/lib/libhiprtc.so", _torch_hiprtc()) if p and os.path.exists(p)]


def _compile_here(lib_path: str, src: str) -> str:
    lib = ctypes.CDLL(lib_path)
    texts = [open(p).read().encode() for _, p in HEADERS]
    names = [n.encode() for n, _ in HEADERS]
    prog = ctypes.c_void_p()
    H = (ctypes.c_char_p * len(texts))(*texts)
    N = (ctypes.c_char_p * len(names))(*names)
    assert lib.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"cbx_jit.hip", len(texts), H, N) == 0
    opts = [b"--offload-arch=gfx950", b"-O3", b"-std=c++17"]
    rc = lib.hiprtcCompileProgram(prog, len(opts), (ctypes.c_char_p * len(opts))(*opts))
    n = ctypes.c_size_t()
    lib.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
    log = ctypes.create_string_buffer(n.value + 1)
    lib.hiprtcGetProgramLog(prog, log)
    lib.hiprtcDestroyProgram(ctypes.byref(prog))
    return "" if rc == 0 else (log.value.decode(errors="replace") or f"hiprtc error {rc}")


def _compile(src: str, lib_path: str | None = None) -> str:
    """Compile src with the hipRTC at lib_path (default: the image's) in a child process; returns the
    error log, "" on success."""
    if not COMPILERS:
        pytest.skip("libhiprtc not available")
    lib_path = lib_path or COMPILERS[0]
    code = ("import sys; sys.path.insert(0, %r); import test_jit_rtc as t; "
            "err = t._compile_here(sys.argv[1], sys.stdin.read()); sys.stdout.write(err); sys.exit(3 if err else 0)"
            % os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code, lib_path], input=src, capture_output=True, text=True, timeout=600)
    if r.returncode == 0:
        return ""
    return r.stdout or f"hipRTC ({lib_path}) died: exit {r.returncode}\n{r.stderr[-2000:]}"


def _record_kernel(layout: int, count: bool, loop: bool, pair: bool = False, coop: bool = False, seg_pair: bool = False) -> str:
    """The specialised record kernel's source as cbx_jit.h emits it (jit_source), for a 3-element
    string layout; coop: the cooperative form (jit_coop: coop_lds / coop_loop<KP, kW>, ops split on the wave, part<kW>);
    seg_pair: two segment-redefine elements in one pass (str_utf8_pair / str_count_pair)."""
    view = "true" if layout == 1 else "false"
    ops = [f"{{{20 * i},20,1,4,0,2,{i},0,{i},-1,{{0,0,0,0}},{{0,0,0,0}},0}}" for i in range(3)]
    if seg_pair:
        sa = "{0,20,1,4,0,2,0,0,0,0,{0,0,0,0},{0,0,0,0},0}"
        sb = "{0,17,1,4,0,2,1,0,1,1,{0,0,0,0},{0,0,0,0},0}"
        if count:
            body = (f"    {{ constexpr StrOp opa = {sa}; constexpr StrOp opb = {sb}; if (!str_count_pair(a, opa, opb, t, img, rec_addr, l.lut, lane)) {{\n"
                    "      str_element<false>(a, opa, a.sops + 0, ldc(a.scall + 0), t, l.cnt, img, rec_addr, false, l.lut, l.str, lane);\n"
                    "      str_element<false>(a, opb, a.sops + 1, ldc(a.scall + 1), t, l.cnt, img, rec_addr, false, l.lut, l.str, lane); } }\n")
        else:
            body = (f"    {{ constexpr StrOp opa = {sa}; constexpr StrOp opb = {sb}; str_utf8_pair(a, opa, ldc(a.scall + 0), opb, "
                    "ldc(a.scall + 1), t, img, rec_addr, l.lut, l.str, lane); }\n")
    elif pair:
        body = (f"    {{ constexpr StrOp opa = {ops[0]}; constexpr StrOp opb = {ops[1]}; str_utf8_two(a, opa, a.sops + 0, "
                f"ldc(a.scall + 0), opb, a.sops + 1, ldc(a.scall + 1), t, l.cnt, img, rec_addr, l.lut, l.str, lane); }}\n")
    elif loop:
        body = f"    for (int i = 0; i < 3; i++) str_element<{view}>(a, ldc(a.sops + i), a.sops + i, ldc(a.scall + i), t, l.cnt, img, rec_addr, false, l.lut, l.str, lane);\n"
    else:
        body = "".join(f"    {{ constexpr StrOp op = {o}; str_element<{view}>(a, op, a.sops + {i}, ldc(a.scall + {i}), t, l.cnt, img, rec_addr, false, l.lut, l.str, lane); }}\n"
                       + ("    } else {\n" if coop and i == 0 else "") for i, o in enumerate(ops))
        if coop:
            body = "    if constexpr (kW == 0) {\n" + body + "    }\n"
    lds = "coop_lds" if coop else "wave_lds"
    lut = (f"  WaveLds l = {lds}(a, smem + 1024, wid);\n  l.lut = (uint32_t*)smem;\n"
           "  for (int i = threadIdx.x; i < 256; i += blockDim.x) { const uint32_t e = a.lut[i]; l.lut[i] = e; ((uint8_t*)(l.lut + 256))[i] = count_lut_byte(e); }\n"
           if count else
           f"  const WaveLds l = {lds}(a, smem, wid);\n  lut_lds_fill(a, l.lut);\n")
    loop_call = ("  if (wid == 0) coop_loop<13, 0>(a, l, (int64_t)blockIdx.x, (int64_t)gridDim.x, lane, JitBody{});\n"
                 "  else coop_loop<13, 1>(a, l, (int64_t)blockIdx.x, (int64_t)gridDim.x, lane, JitBody{});\n}\n" if coop else
                 "  int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;\n"
                 "  const int64_t tstep = (int64_t)gridDim.x * kWavesPerBlock;\n"
                 "  contig_loop<13, 0, false>(a, l, tile, tstep, lane, JitBody{});\n}\n")
    sig = ("(const KernelArgs& a, const TileCtx& t, const uint8_t* img,\n"
           "      uint32_t rec_addr, const WaveLds& l, int lane, Stamps& st) {\n")
    return (f"#define CBX_STR_LAYOUT {layout}\n#define CBX_MODE {1 if count else 0}\n" + ("#define CBX_COUNT_LUT 1\n" if count else "") +
            "#include \"cbx_device.h\"\nnamespace cbx {\nstruct JitBody {\n  static constexpr int kWords = 0;\n  int wid = 0;\n  DirectSink vw;\n"
            "  __device__ __forceinline__ void begin(int64_t) {}\n"
            "  __device__ __forceinline__ void flush(const KernelArgs&, int64_t, int) {}\n"
            + ("  template <int kW>\n  __device__ __forceinline__ void part" + sig + body + "  }\n"
               "  __device__ __forceinline__ void pre" + sig + "  }\n" if coop else
               "  __device__ __forceinline__ void pre" + sig + body + "  }\n") +
            "  __device__ __forceinline__ void post" + sig + "  }\n};\n}  // namespace cbx\n"
            "extern \"C\" __global__ __launch_bounds__(cbx::kWave * cbx::kWavesPerBlock) void k(cbx::KernelArgs a) {\n"
            "  using namespace cbx;\n  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
            "  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);\n  const int lane = threadIdx.x % kWave;\n"
            "  if (!lds_base_ok(smem)) { if (threadIdx.x == 0) atomicOr(a.status, 4); return; }\n"
            + lut + "  __syncthreads();\n" + loop_call)


LIST_KERNEL = """#define CBX_STR_LAYOUT 0
#define CBX_MODE 0
#include "cbx_list.h"
namespace cbx {
struct JitListBody {
  __device__ __forceinline__ bool group(const KernelArgs& a, int ai, const uint8_t* e0, const ListRec& r, int g0,
                                        int gn, int lane, bool& deferred) {
    const int kmax = ((g0 + gn) * kWave < r.rlen ? (g0 + gn) * kWave : r.rlen) - 1;
    const int lim = r.ravail < r.rsafe ? r.ravail : r.rsafe;
    switch (ai) {
    case 0: {
      constexpr NumOp op0 = {66,3,4,1,6,1,32,0,0,5,0,-1,0,0,0xffffffffull,0x0ull,0x1ull,0x1ull,0x0ull,0x1ull,{0,0,0,0},{0,0,0,0}};
      if (a.start_off + op0.eo + op0.size + kmax * 8 > lim) return false;
      const DevColumn c0 = ldc(a.cols + op0.column);
      for (int st = 0; st < gn; st++) {
        const int cb = (g0 + st) * kWave;
        const uint8_t* el = e0 + (st * kWave + lane) * 8;
        list_jit_field<3, 4>(op0, c0, el + 4, r.rstart + cb, cb + lane < r.rlen, lane, deferred);
      }
      return true;
    }
    }
    return false;
  }
};
}  // namespace cbx
extern "C" __global__ __launch_bounds__(cbx::kWave * cbx::kListWaves) void cbx_jit_list(cbx::KernelArgs a,
    const CBX_CONST cbx::ListOp* lops, int32_t n_lops) {
  cbx::JitListBody body;
  cbx::list_run<false>(a, lops, n_lops, body);
}
"""


@pytest.mark.parametrize("layout,count,loop,pair,coop", [(0, False, False, False, False), (1, False, False, False, False),
                                                         (2, False, False, False, False), (2, True, False, False, False),
                                                         (0, False, True, False, False), (2, False, False, True, False),
                                                         (1, False, False, False, True), (2, False, False, False, True),
                                                         (2, True, False, False, True), (2, False, False, "seg", False),
                                                         (2, True, False, "seg", False)])
@pytest.mark.parametrize("compiler", range(2), ids=["rocm", "torch"])
def test_record_kernel_compiles_with_hiprtc(layout, count, loop, pair, coop, compiler):
    if compiler >= len(COMPILERS):
        pytest.skip("no second hipRTC")
    src = _record_kernel(layout, count, loop, pair is True, coop, seg_pair=pair == "seg")
    err = _compile(src, COMPILERS[compiler])
    assert not err, err[:3000]


# the element's fields from aligned 8-byte words (list_words / list_jit_field_w: C5's element of a
# 4-byte binary + a 4-byte COMP-3 field, 8-byte stride)
LIST_KERNEL_WORDS = LIST_KERNEL.replace(
    "        list_jit_field<3, 4>(op0, c0, el + 4, r.rstart + cb, cb + lane < r.rlen, lane, deferred);\n",
    "        uint32_t ph, d[6];\n        list_words<0, 2>(el, ph, d);\n"
    "        list_jit_field_w<3, 4, true, 4, 0, 2>(op0, c0, d, ph, r.rstart + cb, cb + lane < r.rlen, lane, deferred);\n"
    "        list_jit_field_w<1, 8, true, 8, 0, 2>(op0, c0, d, ph, r.rstart + cb, cb + lane < r.rlen, lane, deferred);\n")


@pytest.mark.parametrize("words", [False, True])
@pytest.mark.parametrize("compiler", range(2), ids=["rocm", "torch"])
def test_list_kernel_compiles_with_hiprtc(compiler, words):
    if compiler >= len(COMPILERS):
        pytest.skip("no second hipRTC")
    src = LIST_KERNEL_WORDS if words else LIST_KERNEL
    assert words == ("list_words" in src)
    err = _compile(src, COMPILERS[compiler])
    assert not err, err[:3000]


WALK_KERNEL = """#define CBX_STR_LAYOUT 1
#define CBX_MODE 0
#define CBX_JIT_WALK 1
#include "cbx_device.h"
#include "cbx_walk.h"
namespace cbx {
struct JitWalk {
  static constexpr bool kTyped = true;
  template <typename RP>
  __device__ __forceinline__ void operator()(const WalkArgs& a, const WalkLds& wl, uint8_t* area, RP rec,
      int avail, int seg, int64_t r, int64_t tile, int lane, bool act) const {
    WalkDeps dep;
    dep.clear();
    int off0 = 0;
    { constexpr Field f = {7,1,1,1,1,0,0,0,0,72,4,0,{0,0,0,0},{0,0,0,0},{0,0,0,0},-1,1,1,4,-1,1,0,0,0,0,0,1ull,0ull};
      walk_prim_f(a, wl, f, 1, 0, off0, 0, rec, avail, r, tile, lane, act, dep, false); }
    if (act) off0 += 1;
    {
      const int cnt3 = act ? walk_count(a, 0, dep) : 0;
      const int cmax3 = (int)wave_max64(cnt3);
      int eo3 = off0;
      for (int e3 = 0; e3 < cmax3; e3++) {
        const bool le3 = act && e3 < cnt3;
        const int s3 = (0) * 3 + e3;
        { constexpr Field f = {5,1,5,3,5,0,0,0,0,9,4,1,{3,0,0,0},{3,0,0,0},{0,0,0,0},-1,2,3,1,-1,1,-1,0,0,0,0,1ull,0ull};
          walk_prim_f(a, wl, f, 3, -1, eo3, s3, rec, avail, r, tile, lane, le3, dep, true); }
        if (le3) eo3 += 3;
      }
      if (act) off0 += eo3 - off0;
    }
    { constexpr Field f = {1,7,8,3,0,0,0,0,0,0,4,0,{0,0,0,0},{0,0,0,0},{0,0,0,0},-1,3,1,6,0,1,-1,0,0,0,0,1ull,0ull};
      walk_prim_f(a, wl, f, 3, -1, off0, 0, rec, avail, r, tile, lane, act, dep, false); }
  }
};
}  // namespace cbx
extern "C" __global__ __launch_bounds__(256) void cbx_jit_walk(cbx::WalkArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t wsm[];
  cbx::walk_tiles(a, wsm, cbx::JitWalk{});
}
"""


@pytest.mark.parametrize("compiler", range(2), ids=["rocm", "torch"])
def test_walk_kernel_compiles_with_hiprtc(compiler):
    """The copybook-specialised record walk (jit_walk_source: a prim, an OCCURS of a COMP-3 element,
    a string) compiles against the bundled headers with both compilers."""
    if compiler >= len(COMPILERS):
        pytest.skip("no second hipRTC")
    err = _compile(WALK_KERNEL, COMPILERS[compiler])
    assert not err, err[:3000]


CHAIN_KERNELS = """#define CBX_STR_LAYOUT 1
#define CBX_MODE 0
#define CBX_JIT_WALK 1
#include "cbx_device.h"
#include "cbx_walk.h"
#include "cbx_chain.h"
namespace cbx {
__device__ __forceinline__ int jit_walk_length(const WalkArgs& a, const CBX_GLOBAL uint8_t* rec, int avail) {
  WalkDeps dep;
  dep.clear();
  int off0 = 0;
  {   // dependee (node 2)
    constexpr Field f = {7,1,1,1,1,0,0,0,0,72,4,0,{0,0,0,0},{0,0,0,0},{0,0,0,0},-1,1,1,4,-1,1,0,0,0,0,0,1ull,0ull};
    uint8_t zb[64];
    if (off0 + 1 <= avail) {
      for (int i = 0; i < 1; i++) zb[i] = rec[off0 + i];
    } else {
      for (int i = 0; i < 1; i++) zb[i] = off0 + i < avail ? rec[off0 + i] : 0;
    }
    { const Val dv = decode_count_int(f, zb); dep.set(0, dv.valid, WalkDep{1, (int32_t)dv.lo}); }
  }
  off0 += 1;
  {   // OCCURS (node 3)
    const int cnt1 = walk_count(a, 0, dep);
    int eo1 = off0;
    for (int e1 = 0; e1 < cnt1; e1++) {
      {   // dependee (node 4)
        constexpr Field f = {1,7,8,3,0,0,0,0,0,0,4,0,{0,0,0,0},{0,0,0,0},{0,0,0,0},-1,3,1,6,0,1,-1,0,0,0,0,1ull,0ull};
        uint8_t zb[64];
        if (eo1 + 3 <= avail) {
          for (int i = 0; i < 3; i++) zb[i] = rec[eo1 + i];
        } else {
          for (int i = 0; i < 3; i++) zb[i] = eo1 + i < avail ? rec[eo1 + i] : 0;
        }
        walk_len_str_dep(a, f, zb, 3, 1, dep);
      }
      eo1 += 3;
      {   // OCCURS (node 5)
        const int cnt2 = walk_count(a, 1, dep);
        const int w2 = cnt2 * 5;
        eo1 += w2;
      }
    }
    const int w1 = eo1 - off0;
    off0 += w1;
  }
  off0 += 3;
  return off0;
}
struct JitVarOccursStep {   // VarOccursStep's layout and semantics
  WalkArgs a;
  int64_t n_bytes;
  __device__ __forceinline__ ChainStep at(int64_t pos) const {
    ChainStep s{kChainStop, 0, 0};
    if (pos >= n_bytes) return s;
    const int64_t left = n_bytes - pos;
    const int len = jit_walk_length(a, gp(a.data) + pos, left < 0x7fffffff ? (int)left : 0x7fffffff);
    if (len <= 0) return s;
    s.len = len;
    s.next = pos + len;
    return s;
  }
};
}  // namespace cbx
using cbx::JitVarOccursStep;
using cbx::ChainArgs;
extern "C" __global__ void cbx_jit_chain_sample(JitVarOccursStep s, ChainArgs c, int n_max) { cbx::chain_sample_run(s, c, n_max); }
extern "C" __global__ __launch_bounds__(256) void cbx_jit_chain_spec(JitVarOccursStep s, ChainArgs c) { cbx::chain_spec_run(s, c); }
extern "C" __global__ __launch_bounds__(256) void cbx_jit_chain_fix(JitVarOccursStep s, ChainArgs c, const int64_t* ex_in, int64_t* ex_out) {
  cbx::chain_fix_run(s, c, ex_in, ex_out);
}
extern "C" __global__ void cbx_jit_chain_settle(JitVarOccursStep s, ChainArgs c, int64_t* ex) { cbx::chain_settle_run(s, c, ex); }
extern "C" __global__ __launch_bounds__(256) void cbx_jit_chain_write(JitVarOccursStep s, ChainArgs c, const int64_t* base, int64_t capacity,
                                                  int64_t* rec_off, int32_t* rec_len) {
  cbx::chain_write_run(s, c, base, capacity, rec_off, rec_len);
}
"""


@pytest.mark.parametrize("compiler", range(2), ids=["rocm", "torch"])
def test_var_occurs_framing_compiles_with_hiprtc(compiler):
    """The copybook-specialised var-occurs framing (jit_chain_source: a numeric dependee, an OCCURS of
    groups each with a string dependee and a nested OCCURS, the five chain passes) compiles against the
    bundled headers with both compilers."""
    if compiler >= len(COMPILERS):
        pytest.skip("no second hipRTC")
    err = _compile(CHAIN_KERNELS, COMPILERS[compiler])
    assert not err, err[:3000]
