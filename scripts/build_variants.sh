#!/bin/bash
# Diagnostic timing builds of libfjsp (not used by the product): each argument is
# name=flags, e.g. libv_x.so="-DFJSP_AG_PSPEC"; run them with VARIANT_LIBS in gpu_variants.sh.
cd "$(dirname "$0")/../multi-agent-rl-for-fjsp_amd"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function"
for v in "$@"; do
  name="${v%%=*}"; flags="${v#*=}"
  hipcc $F $flags -o "$name" csrc/fjsp_hip.hip csrc/fjsp_policy.hip &
done
wait
