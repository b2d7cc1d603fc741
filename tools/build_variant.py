"""Build the library from another git revision as cobrix_amd/libcobrix_hip_<name>.so (A/B timing
within one GPU call: CBX_LIB_VARIANT=<name> python bench.py ...).  Diagnostic; never shipped.

Usage: python tools/build_variant.py <git rev | .> <name> [-DMACRO=value ...]
("." builds the working tree; -D defines go to hipcc, e.g. -DCBX_DIAG=1 for cbx_device.h's store
diagnostics, which the specialised kernels inherit through cbx_jit.h.)
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rev, name = sys.argv[1], sys.argv[2]
    defines = [x for x in sys.argv[3:] if x.startswith("-D")]
    import __graft_entry__ as G
    with tempfile.TemporaryDirectory() as d:
        if rev == ".":
            subprocess.run(["cp", "-r", os.path.join(ROOT, "cobrix_amd"), os.path.join(ROOT, "include"), d], check=True)
        else:
            arch = subprocess.run(["git", "archive", rev, "cobrix_amd/csrc", "include"], cwd=ROOT, check=True,
                                  capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", d], input=arch, check=True)
        csrc = os.path.join(d, "cobrix_amd", "csrc")
        inc = os.path.join(d, "include")
        # the bundle's header set as __graft_entry__ lists it, taken from the revision's tree
        G.JIT_HEADERS = tuple((n, os.path.join(inc if n == "cobrix_hip.h" else csrc, n)) for n, _ in G.JIT_HEADERS
                              if os.path.exists(os.path.join(inc if n == "cobrix_hip.h" else csrc, n)))
        G.CSRC = csrc
        G._write_jit_bundle()
        out = os.path.join(ROOT, "cobrix_amd", f"libcobrix_hip_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + inc, "-I" + csrc, *defines, "-o", out, os.path.join(csrc, "cbx_capi.hip"), "-lhiprtc"], check=True)
        print(out)


if __name__ == "__main__":
    main()
