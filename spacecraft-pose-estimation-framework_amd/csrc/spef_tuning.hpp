// Internal kernel-tuning options of spef_set_option (not part of the public ABI in include/spef.h).
// Used by the sweep tools (tools/explore.py, tools/ab.py) to time alternative schedules on the GPU box.
//   SPEF_OPT_FUSE_MIN_HW: fuse only blocks whose input has at least this many pixels per image (the rest run as
//                         GEMM + depthwise + GEMM).
//   SPEF_OPT_PW_GEMM    : LDS-tiled MFMA GEMM (1, default) or register-direct kernel (0) for unfused 1x1 convs.
//   SPEF_OPT_IRB_VARIANT: fused-block tile variant (0 = tuned default).
//   SPEF_OPT_TEST_FAIL_BCAST: failure injection for spef_bcast_weights tests: 1 = this rank fails its local check
//                         before the data broadcast, 2 = fails staging after it, 3 = the header wait never completes
//                         (exercises the timeout -> ncclCommAbort path without a hung peer). 0 = off.
//   SPEF_OPT_MX_KERNELS : fp16mx blocks 2-7 on the dedicated kernels of k_mx.hip (1, default) or on the fp16x2 slab
//                         kernels with fp16 block I/O (0).
#pragma once

enum spef_tuning_option {
  SPEF_OPT_FUSE_MIN_HW = 2,
  SPEF_OPT_PW_GEMM = 3,
  SPEF_OPT_IRB_VARIANT = 4,
  SPEF_OPT_TEST_FAIL_BCAST = 5,
  SPEF_OPT_MX_KERNELS = 8
};
