#!/bin/bash
# Round-6 measurement artefacts on the GPU box (run from the repo root): bash tools/r6_profile.sh <tag> [full]
#   gpurun_out/bench_<tag>.json        the bench line (with "full": every sub-record, CPU baseline included)
#   gpurun_out/prof_<tag>/             rocprofv3 --kernel-trace --stats of the headline (fp16mx) workload alone
#   gpurun_out/pmc_fetch_<tag>/, pmc_write_<tag>/   FETCH_SIZE / WRITE_SIZE passes of the fp16mx forward (separate)
#   gpurun_out/pmc_<tag>_sq{1,2}/      SQ instruction / cycle counters of the fp16mx forward
#   gpurun_out/pmc_<tag>_i8/           SQ counters of the int8 forward (the C5 statement)
# then: python tools/rocprof_summary.py --tag <tag> --stats gpurun_out/prof_<tag> --fetch gpurun_out/pmc_fetch_<tag> \
#         --write gpurun_out/pmc_write_<tag> --leg 10 --per-step front_mx_kernel
set -e
TAG=${1:-r06}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
if [ "$2" = full ]; then
  timeout -k 10 400 python3 $R/bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
  echo "bench ok"
fi
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv \
  -- python3 $R/bench.py --steps 10 --no-cpu-baseline --no-int8 --no-keypoint --no-x2 --no-fp16 --sharp-frames 0 --no-peaks) \
  > $O/prof_$TAG.log 2>&1
echo "stats ok"
(cd /tmp && DT=fp16mx timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_fetch_$TAG.log 2>&1
echo "fetch ok"
(cd /tmp && DT=fp16mx timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o run --output-format csv \
  -- python3 $R/tools/fwd_only.py 2) > $O/pmc_write_$TAG.log 2>&1
echo "write ok"
(cd /tmp && DT=fp16mx timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -d $O/pmc_${TAG}_sq1 -o run --output-format csv -- python3 $R/tools/fwd_only.py 2) > $O/pmc_${TAG}_sq1.log 2>&1
echo "sq1 ok"
(cd /tmp && DT=fp16mx timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES \
  -d $O/pmc_${TAG}_sq2 -o run --output-format csv -- python3 $R/tools/fwd_only.py 2) > $O/pmc_${TAG}_sq2.log 2>&1
echo "sq2 ok"
(cd /tmp && DT=int8 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d $O/pmc_${TAG}_i8 -o run --output-format csv -- python3 $R/tools/fwd_only.py 2) > $O/pmc_${TAG}_i8.log 2>&1
echo "int8 sq ok"
(cd /tmp && DT=fp16 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  -d $O/pmc_${TAG}_f16 -o run --output-format csv -- python3 $R/tools/fwd_only.py 2) > $O/pmc_${TAG}_f16.log 2>&1
echo "fp16 sq ok"
