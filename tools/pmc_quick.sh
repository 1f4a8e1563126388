#!/bin/bash
# One SQ counter pass (instruction mix + LDS conflicts) over tools/fwd_only.py, then the per-kernel table.
# Run on the GPU box from the repo root: bash tools/pmc_quick.sh [tag]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-q}
set -e
rm -rf $R/gpurun_out/pmcq_$T
(cd /tmp && timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU \
   SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES -d $R/gpurun_out/pmcq_$T/pmc_1 -o run --output-format csv \
   -- python3 $R/tools/fwd_only.py 2) > $R/gpurun_out/pmcq_$T.log 2>&1
python3 $R/tools/pmc_table.py $R/gpurun_out/pmcq_$T > $R/gpurun_out/pmcq_$T.txt
