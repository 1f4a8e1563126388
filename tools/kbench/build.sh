#!/bin/bash
# Builds the kernel harnesses in tools/kbench (on the CPU container; the binaries travel to the GPU box):
#   blk_trace  per-wave timelines of one launch (SPEF_TRACE probes compiled in)
#   blk_bench  the same harness with the probes compiled out (timing only)
set -e
cd "$(dirname "$0")/../.."
F="-O3 -std=c++17 --offload-arch=gfx950 -fno-honor-nans -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -I include -I spacecraft-pose-estimation-framework_amd/csrc"
/opt/rocm/bin/hipcc $F tools/kbench/blk_trace.hip -o tools/kbench/blk_trace &
/opt/rocm/bin/hipcc $F -DSPEF_KBENCH_TIMING_ONLY tools/kbench/blk_trace.hip -o tools/kbench/blk_bench &
wait
/opt/rocm/bin/hipcc ${F/-fno-honor-nans /} tools/kbench/head_bench.hip -o tools/kbench/head_bench &
/opt/rocm/bin/hipcc ${F/-fno-honor-nans /} -DSPEF_KTRACE tools/kbench/head_bench.hip -o tools/kbench/head_trace &
wait
