// Shared device helpers for the SPEF MI355X (gfx950 / CDNA4) kernels.
//
// Storage types: activations are NHWC, fp16 (parity default) or bf16, 16-B aligned per pixel row
// (every channel count on the path is a multiple of 8). Accumulation is always fp32 (MFMA f32 C/D).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spef {

// "Done once per device" flag (bit d: device d) for host-side launch set-up such as hipFuncSetAttribute: one process
// may drive several GPUs, and the attribute applies to the current device's instance of the kernel. (A race only
// repeats the idempotent set-up.)
struct DevOnce {
  uint32_t mask = 0;
  static int dev() {
    int d = 0;
    return hipGetDevice(&d) == hipSuccess ? (d & 31) : 0;
  }
  bool done() const { return (mask >> dev()) & 1u; }
  void set() { mask |= 1u << dev(); }
};

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Element-type traits: the MFMA used for a 16x16 output tile with K = 32 per instruction.
// gfx950 lane map (cdna_hip_programming.md §3): A[i = l&15][k = 8(l>>4)+e], B[k = 8(l>>4)+e][j = l&15],
// D[i = 4(l>>4)+r][j = l&15].
// mfma16: K = 16 form, lane holds A[i = l&15][k = 4(l>>4)+e], B[k = 4(l>>4)+e][j = l&15] (4 elements).
struct F16 {
  using T = _Float16;
  using DW = _Float16;   // depthwise weights: fp16 (one v_fma_mix per tap with fp16 x and w, fp32 accumulate)
  using x8 = f16x8;
  using x4 = f16x4;
  static __device__ __forceinline__ f32x4 mfma(x8 a, x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mfma16(x4 a, x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
  }
};
struct BF16 {
  using T = __bf16;
  using DW = float;      // depthwise weights stay fp32 (v_fma_mix has no bf16 form)
  using x8 = bf16x8;
  using x4 = bf16x4;
  static __device__ __forceinline__ f32x4 mfma(x8 a, x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mfma16(x4 a, x4 b, f32x4 c) {
    typedef short s4 __attribute__((ext_vector_type(4)));
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s4, a), __builtin_bit_cast(s4, b), c, 0, 0, 0);
  }
};

// fp32 storage (blob dtype 4, k_f32.hip): stem and depthwise kernels only (the 1x1 convs use gemm_f32_kernel)
typedef float f32x8 __attribute__((ext_vector_type(8)));
struct F32 {
  using T = float;
  using DW = float;
  using x8 = f32x8;
  using x4 = f32x4;
};

template <typename DT>
__device__ __forceinline__ typename DT::x8 load8(const typename DT::T* p) {
  return *reinterpret_cast<const typename DT::x8*>(p);
}
// ReLU + round 4 fp32 values to the activation type: fp16 converts pairs (v_cvt_pk_f16_f32, RNE) and clamps
// with one v_pk_max_f16 per pair -- the same values as fmaxf-then-convert (conversion is monotonic, 0 -> 0).
template <typename DT>
__device__ __forceinline__ typename DT::x4 relu_cvt4(f32x4 v) {
  typename DT::x4 o;
  if constexpr (sizeof(typename DT::T) == 2 && __is_same(typename DT::T, _Float16)) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 z = {(_Float16)0.0f, (_Float16)0.0f};
    h2 a = {(_Float16)v[0], (_Float16)v[1]}, b = {(_Float16)v[2], (_Float16)v[3]};
    a = __builtin_elementwise_max(a, z);
    b = __builtin_elementwise_max(b, z);
    o[0] = a[0]; o[1] = a[1]; o[2] = b[0]; o[3] = b[1];
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (typename DT::T)fmaxf(v[r], 0.f);
  }
  return o;
}

// ReLU + round of 8 fp32 values (a depthwise output B fragment): 4 v_cvt_pk + 4 v_pk_max instead of 8 v_max_f32 +
// 4 v_cvt_pk on fp16 (VALU issue is the limit of the depthwise-heavy kernels)
// (pairs are built from the scalars: an f32x4 temporary lets the SLP vectorizer turn the producing v_fma_mix chain
// into v_cvt + v_pk_fma_f32, which issues more instructions)
template <typename DT>
__device__ __forceinline__ typename DT::x8 relu_cvt8(const float a[8]) {
  typename DT::x8 o;
  if constexpr (__is_same(typename DT::T, _Float16)) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 z = {(_Float16)0.0f, (_Float16)0.0f};
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      // the empty asm keeps the fp32 values: otherwise the producing FMA and the convert fuse into one
      // v_fma_mixlo/hi_f16 (a single rounding to fp16), which differs from the unfused kernels' fp32 -> fp16
      // double rounding in rare ties (1 ulp; test_fused_blocks_bit_identical_to_unfused)
      float x0 = a[e], x1 = a[e + 1];
      asm("" : "+v"(x0), "+v"(x1));
      h2 p = {(_Float16)x0, (_Float16)x1};
      p = __builtin_elementwise_max(p, z);
      o[e] = p[0];
      o[e + 1] = p[1];
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (typename DT::T)fmaxf(a[e], 0.f);
  }
  return o;
}

// 8 consecutive depthwise weights kept in their storage type (fp16: 4 VGPRs, read by v_fma_mix directly)
template <typename DT, bool H = (sizeof(typename DT::DW) == 2)>
struct DW8 {
  f16x8 v;
  __device__ __forceinline__ void load(const typename DT::DW* p) { v = *reinterpret_cast<const f16x8*>(p); }
  __device__ __forceinline__ float operator[](int e) const { return (float)v[e]; }
};
template <typename DT>
struct DW8<DT, false> {
  float v[8];
  __device__ __forceinline__ void load(const typename DT::DW* p) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ float operator[](int e) const { return v[e]; }
};

// 8 consecutive depthwise weights -> fp32 (exact conversion from fp16)
template <typename DT>
__device__ __forceinline__ void load_dw8(const typename DT::DW* p, float w[8]) {
  if constexpr (sizeof(typename DT::DW) == 2) {
    const f16x8 v = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) w[e] = (float)v[e];
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  }
}

// Vertical-pair depthwise (fp16): a dword holds one channel of two vertically adjacent rows (lo = upper row).
// Two taps of a kernel column are one v_dot2_f32_f16, the third a v_fma_mix on one half (op_sel), so a 3x3 tap
// costs 6 VALU instead of 9. Fused and unfused kernels evaluate exactly these operations in the same order.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float h_lo(uint32_t v) { return (float)__builtin_bit_cast(f16x2, v)[0]; }
__device__ __forceinline__ float h_hi(uint32_t v) { return (float)__builtin_bit_cast(f16x2, v)[1]; }
__device__ __forceinline__ float dot2h(uint32_t x, uint32_t w, float acc) {
  return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, x), __builtin_bit_cast(f16x2, w), acc, false);
}
__device__ __forceinline__ uint32_t pack_h2(_Float16 lo, _Float16 hi) {
  return __builtin_bit_cast(uint32_t, f16x2{lo, hi});
}
// ReLU + fp16 rounding of two fp32 values into one dword (v_cvt_pk_f16_f32 + v_pk_max_f16, as relu_cvt4)
__device__ __forceinline__ uint32_t relu_pk2(float lo, float hi) {
  const f16x2 z = {(_Float16)0.0f, (_Float16)0.0f};
  f16x2 p = {(_Float16)lo, (_Float16)hi};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(p, z));
}

// Packed-fp16 depthwise step (fp16 stride-2 blocks): a[i] += x[i] * w[i] for 8 channels as 4 v_pk_fma_f16 (fused,
// one fp16 rounding per tap), and the ReLU of the 8 sums as 4 v_pk_max_f16
__device__ __forceinline__ void pk_fma4(f16x2 a[4], uint4 x, uint4 w) {
  const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    a[i] = __builtin_elementwise_fma(__builtin_bit_cast(f16x2, xs[i]), __builtin_bit_cast(f16x2, ws[i]), a[i]);
}
__device__ __forceinline__ uint4 relu_pk4(const f16x2 a[4]) {
  const f16x2 z = {(_Float16)0.0f, (_Float16)0.0f};
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(a[i], z));
  return make_uint4(o[0], o[1], o[2], o[3]);
}

template <typename DT>
__device__ __forceinline__ typename DT::x8 zero8() {
  typename DT::x8 z;
#pragma unroll
  for (int e = 0; e < 8; ++e) z[e] = (typename DT::T)0.0f;
  return z;
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5, "XCD swizzle must be
// bijective"): consecutive logical ids land on one XCD (blocks b and b+8 share an XCD under the
// observed round-robin placement). Speed only -- correctness never depends on placement.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  const uint32_t q = nwg >> 3, r = nwg & 7, xcd = bid & 7, off = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + off;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Per-wave timeline probes for the kernel tracing harness (tools/kbench): compiled to nothing in the library.
// With SPEF_KTRACE defined, SPEF_TRACE(slot) stores s_memtime of the calling wave into
// spef_ktrace[(workgroup * 16 + wave) * SPEF_TRACE_SLOTS + slot] (lane 0 only, vector store). The counter is per
// XCD: only deltas within one workgroup are meaningful.
#define SPEF_TRACE_SLOTS 72
#ifdef SPEF_KTRACE
__device__ unsigned long long* spef_ktrace;
#define SPEF_TRACE(slot)                                                                                        \
  do {                                                                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                                 \
    if ((threadIdx.x & 63) == 0)                                                                                \
      spef_ktrace[((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * SPEF_TRACE_SLOTS + (slot)] = t_;              \
  } while (0)
#else
#define SPEF_TRACE(slot) ((void)0)
#endif

// Timing ablations of the kernel harness (tools/kbench/ablate.sh; wrong results, never in the library):
// SPEF_KBENCH_NO_XLOAD points every input-tile load of the fused blocks at the image's first pixels (the same
// instructions, served from L2: no HBM input traffic); SPEF_KBENCH_NO_YSTORE drops the output stores of the fused
// blocks and the front kernel (values kept live).
#ifdef SPEF_KBENCH_NO_XLOAD
#define SPEF_KB_XOFF(off) ((size_t)0 * (off))
#else
#define SPEF_KB_XOFF(off) (off)
#endif
#ifdef SPEF_KBENCH_NO_YSTORE
#define SPEF_KB_YSTORE(store, v) asm volatile("" ::"v"(v))
#else
#define SPEF_KB_YSTORE(store, v) store
#endif

}  // namespace spef
