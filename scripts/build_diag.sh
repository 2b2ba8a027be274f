#!/bin/bash
# Diagnostic builds of libfjsp (per-phase s_memtime stamps); not used by the product.
cd "$(dirname "$0")/../multi-agent-rl-for-fjsp_amd"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function"
hipcc $F -DFJSP_STAMPS -o libfjsp_stamps.so csrc/fjsp_hip.hip csrc/fjsp_policy.hip csrc/fjsp_group.hip &
hipcc $F -DFJSP_STAMPS -DFJSP_STAMPS_FINE -o libfjsp_stamps_fine.so csrc/fjsp_hip.hip csrc/fjsp_policy.hip &
wait
