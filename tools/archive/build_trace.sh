#!/bin/bash
# Diagnostic build with per-wave phase stamps (tools/wave_trace.py).
set -eu
mkdir -p shippingenv_amd/_lib/trace
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -DSHIPENV_TRACE=1 -o shippingenv_amd/_lib/trace/libshipenv_hip.so shippingenv_amd/csrc/shipenv.hip \
  shippingenv_amd/csrc/mapload.cpp
