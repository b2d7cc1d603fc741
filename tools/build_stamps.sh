#!/bin/bash
# Diagnostic build of the library with s_memtime stamps (tools/stamps.py); never shipped.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DCBX_STAMPS -Iinclude -Icobrix_amd/csrc \
    -o cobrix_amd/libcobrix_hip_stamps.so cobrix_amd/csrc/cbx_capi.hip -lhiprtc
