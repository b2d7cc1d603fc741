"""Disassembly of a specialised-kernel source as the product compiles it (offline ISA study).

The library's hipRTC calls resolve to the libhiprtc.so.7 already loaded in the process -- torch's
bundled one when torch was imported first (every product process) -- so the code that runs on the
GPU comes from that compiler, not from the image's hipcc.  This compiles a source dumped with
CBX_JIT_DUMP through that hipRTC (or the image's: --rocm) and disassembles the code object.

usage: python tools/jit_isa.py SRC.hip [--rocm] -> SRC.co, SRC.dis (+ VGPR / SGPR / scratch / LDS)"""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import test_jit_rtc as t  # noqa: E402  (the header list and the compiler paths)


def compile_co(src: str, lib_path: str) -> bytes:
    lib = ctypes.CDLL(lib_path)
    texts = [open(p).read().encode() for _, p in t.HEADERS]
    names = [n.encode() for n, _ in t.HEADERS]
    prog = ctypes.c_void_p()
    H = (ctypes.c_char_p * len(texts))(*texts)
    N = (ctypes.c_char_p * len(names))(*names)
    assert lib.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"cbx_jit.hip", len(texts), H, N) == 0
    opts = [b"--offload-arch=gfx950", b"-O3", b"-std=c++17"]
    rc = lib.hiprtcCompileProgram(prog, len(opts), (ctypes.c_char_p * len(opts))(*opts))
    if rc != 0:
        n = ctypes.c_size_t()
        lib.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
        log = ctypes.create_string_buffer(n.value + 1)
        lib.hiprtcGetProgramLog(prog, log)
        raise SystemExit(log.value.decode(errors="replace")[:4000])
    n = ctypes.c_size_t()
    lib.hiprtcGetCodeSize(prog, ctypes.byref(n))
    buf = ctypes.create_string_buffer(n.value)
    lib.hiprtcGetCode(prog, buf)
    lib.hiprtcDestroyProgram(ctypes.byref(prog))
    return buf.raw


def main():
    src_path = sys.argv[1]
    lib_path = t.COMPILERS[0] if "--rocm" in sys.argv else t.COMPILERS[-1]
    co = compile_co(open(src_path).read(), lib_path)
    base = os.path.splitext(src_path)[0]
    open(base + ".co", "wb").write(co)
    bin_dir = "/opt/rocm/lib/llvm/bin"
    dis = subprocess.run([f"{bin_dir}/llvm-objdump", "-d", "--mcpu=gfx950", base + ".co"], capture_output=True, text=True).stdout
    open(base + ".dis", "w").write(dis)
    notes = subprocess.run([f"{bin_dir}/llvm-readobj", "--notes", base + ".co"], capture_output=True, text=True).stdout
    keep = [ln.strip() for ln in notes.splitlines()
            if any(k in ln for k in (".vgpr_count", ".sgpr_count", ".private_segment_fixed_size", ".group_segment_fixed_size",
                                     ".vgpr_spill_count", ".sgpr_spill_count", ".name:"))]
    print(lib_path)
    print("\n".join(keep))
    ops = [ln.split()[0] for ln in dis.splitlines() if ln.startswith("\t") and ln.split()]
    print("instructions:", len(ops))


if __name__ == "__main__":
    main()
