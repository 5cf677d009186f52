#!/bin/bash
# builds scripts/probes/solve_bench (stage stamps) and solve_bench_plain (the library's k_solve as is)
set -e
cd "$(dirname "$0")"
F="-O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -I ../../generalized-icp_amd/csrc -I ../../include -L/opt/rocm/lib -lrccl"
/opt/rocm/bin/hipcc $F solve_bench.hip -o solve_bench &
/opt/rocm/bin/hipcc $F -DNO_STAMPS solve_bench.hip -o solve_bench_plain &
wait
