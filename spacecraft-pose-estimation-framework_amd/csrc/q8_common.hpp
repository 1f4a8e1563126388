// Shared integer helpers of the fused INT8 inverted-residual kernels (k_q8irb.hip slab form, k_q8irw.hip
// role-split form): requant records, the v_med3 clamp, the biased-fp16 hidden encoding, the int8 MFMA.
#pragma once
#include "spef_common.hpp"

namespace spef {
namespace q8 {

typedef int i32x4_t __attribute__((ext_vector_type(4)));

struct RQ16 {
  int32_t M, S;
  int64_t B;
};

// The packer guarantees S >= 32 for fused blocks (blob_q8.py), so (acc * M + B) >> S is the high word of the
// 64-bit v_mad_i64_i32 result shifted by S - 32: three VALU ops with the clamp (v_med3_i32).
// clamp to [lo, hi] (lo <= hi) as one v_med3_i32: the compiler only forms med3 from min(max()) with constant bounds,
// and the quantizer tops here are kernel arguments (two VALU ops per requantised value otherwise)
__device__ __forceinline__ int med3i(int x, int lo, int hi) {
  int r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
  return r;
}

__device__ __forceinline__ int rq_apply(int acc, const RQ16& r, int lo, int hi) {
  const int64_t t = (int64_t)acc * r.M + r.B;
  const int v = (int)(t >> 32) >> (r.S - 32);
  return med3i(v, lo, hi);
}

// A requant record held in registers for a whole chunk, with the shift already reduced to S - 32. SH32 (blob flag 4:
// every shift of the block is exactly 32): no shift at all, and a constant added to the offset moves the clamped
// result straight into the encoding the consumer wants (B + (c << 32) adds c to the high word exactly).
template <bool SH32>
struct RQR {
  int M, sh;
  int64_t B;
  __device__ __forceinline__ void set(const RQ16& r, int64_t add) {
    M = r.M;
    sh = r.S - 32;
    B = SH32 ? r.B + add * 4294967296LL : r.B;
  }
  __device__ __forceinline__ int hi(int acc) const {   // v_mad_i64_i32 (+ v_ashrrev_i32 unless SH32)
    const int v = (int)(((int64_t)acc * M + B) >> 32);
    return SH32 ? v : v >> sh;
  }
};

// Hidden u8 values live in the LDS slab as the fp16 number 1024 + n, i.e. the bit pattern 0x6400 | n (exact: fp16
// has an 11-bit significand): two values pack into one dword with a shift-or, no int -> float conversion. The
// depthwise sum then carries + 1024 * sum_taps w, which the packer folded into the depthwise requant offset.
constexpr uint32_t kF16Bias2 = 0x64006400u;   // two fp16 1024.0
// expand output: u8 n (unsigned quantizer of eh + 1 levels, eh = 2^b - 1) of two channels -> one dword of fp16 (1024 + n)
template <bool SH32>
__device__ __forceinline__ uint32_t expand_pair(const RQR<SH32>& r0, int a0, const RQR<SH32>& r1, int a1, int eh) {
  if constexpr (SH32) {   // the offset carries + 0x6400: clamp to [0x6400, 0x6400 + eh], two low halves -> one v_perm_b32
    const int v0 = med3i(r0.hi(a0), 0x6400, 0x6400 + eh), v1 = med3i(r1.hi(a1), 0x6400, 0x6400 + eh);
    return __builtin_amdgcn_perm((uint32_t)v1, (uint32_t)v0, 0x05040100u);
  } else {
    const int v0 = med3i(r0.hi(a0), 0, eh), v1 = med3i(r1.hi(a1), 0, eh);
    return ((uint32_t)v1 << 16) | (uint32_t)v0 | kF16Bias2;
  }
}

__device__ __forceinline__ i32x4_t mfma_i8(long a, long b, i32x4_t c) {
  return __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c, 0, 0, 0);
}

}  // namespace q8
}  // namespace spef
