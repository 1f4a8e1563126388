#!/bin/bash
# Timing-ablation builds of the blk_trace harness (probes compiled out): one binary per SPEF_KBENCH_* switch
# (csrc/k_irw.hip). Results are wrong by construction; only the launch times matter. Binaries: tools/kbench/abl/.
set -e
cd "$(dirname "$0")/../.."
F="-O3 -std=c++17 --offload-arch=gfx950 -fno-honor-nans -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -I include -I spacecraft-pose-estimation-framework_amd/csrc -DSPEF_KBENCH_TIMING_ONLY"
for v in "$@"; do
  case $v in
    base) D="" ;;
    no_xload|no_ystore) D="-DSPEF_KBENCH_${v^^}" ;;
    no_mem) D="-DSPEF_KBENCH_NO_XLOAD -DSPEF_KBENCH_NO_YSTORE" ;;
    irp_late) D="-DSPEF_IRP_EARLY=0" ;;
    *) D="-DSPEF_KBENCH_IRW_${v^^}" ;;
  esac
  /opt/rocm/bin/hipcc $F $D tools/kbench/blk_trace.hip -o tools/kbench/abl/blk_$v &
done
wait
