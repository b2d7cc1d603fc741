"""Dump (and hipRTC-compile) the copybook-specialised kernel of a layout: SYN200 by default.

Usage: python tools/jit_check.py [copybook file | syn200 | synstr200] [views | utf8] -> gpurun_out/jit_<name>[_views].hip;
prints the status.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cobrix_amd import native as N  # noqa: E402
from cobrix_amd.reader import FixedLenNestedReader, ReaderParameters  # noqa: E402
from cobrix_amd.synth import SYN200_COPYBOOK, SYNSTR200_COPYBOOK  # noqa: E402


def main():
    name, text, cp = "syn200", SYN200_COPYBOOK, "common"
    if len(sys.argv) > 1 and sys.argv[1] == "synstr200":
        name, text, cp = "synstr200", SYNSTR200_COPYBOOK, "cp037"
    elif len(sys.argv) > 1 and sys.argv[1] != "syn200":
        name, text = os.path.splitext(os.path.basename(sys.argv[1]))[0], open(sys.argv[1]).read()
    views = len(sys.argv) > 2 and sys.argv[2] == "views"
    utf8 = len(sys.argv) > 2 and sys.argv[2] == "utf8"
    if views or utf8:
        name += "_" + sys.argv[2]
    L = N.load()
    rd = FixedLenNestedReader(text, ReaderParameters(ebcdic_code_page=cp, string_views=views, string_utf8=utf8))
    buf = ctypes.create_string_buffer(4 << 20)
    n = ctypes.c_int64()
    rc = L.cbx_plan_specialize(rd.native.handle, buf, len(buf), ctypes.byref(n), 1)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"jit_{name}.hip"), "w") as f:
        f.write(buf.value.decode())
    print("rc", rc, "source bytes", n.value, L.cbx_last_error().decode()[:3000] if rc else "")


if __name__ == "__main__":
    main()
