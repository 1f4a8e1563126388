// On-box measurement kernels for bench.py (peaks "re-measured by the build's own microbenchmark";
// BASELINE.md §3 item 3): dense fp16 and int8 MFMA issue rate, HBM stream copy / read bandwidth, and the shader
// clock the chip holds (in-kernel s_memtime ticks -- shader cycles -- over s_memrealtime's fixed 100 MHz,
// MI355X_MICROARCH.md "DVFS give-back" item 6). Measurement only: nothing here is on the inference path.
#include "../../include/spef.h"

#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "spef_common.hpp"
#include "spef_kernels.hpp"

namespace spef {

// Location of the executing wave: XCD (hwreg XCC_ID, id 20 on gfx940+, bits [3:0]) in bits [11:8], and HW_ID
// (id 4) bits [15:8] = CU, SH and SE id in bits [7:0]. s_memtime counters are only comparable within one CU.
__device__ __forceinline__ uint32_t cu_key() {
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  return (xcc << 8) | ((hw >> 8) & 0xffu);
}

// 8 independent accumulator chains per wave on random operands (zero operands run at a higher clock than real
// data, MI355X_MICROARCH.md "DVFS give-back" item 1); lane 0 of each workgroup stamps the clock around the loop.
template <bool I8>
__global__ __launch_bounds__(256) void mfma_peak_kernel(const uint32_t* __restrict__ seed, int iters,
                                                        float* __restrict__ sink, unsigned long long* __restrict__ clk) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  typedef long i64x2 __attribute__((ext_vector_type(2)));
  const int t = threadIdx.x;
  const uint32_t* s = seed + ((blockIdx.x * 256 + t) & 4095) * 4;
  f16x8 a, b;
  i64x2 ia, ib;
  {
    const uint4 v = *reinterpret_cast<const uint4*>(s);
    const uint4 w = *reinterpret_cast<const uint4*>(seed + (((blockIdx.x * 256 + t) * 7 + 1) & 4095) * 4);
    a = __builtin_bit_cast(f16x8, v);
    b = __builtin_bit_cast(f16x8, w);
    ia = __builtin_bit_cast(i64x2, v);
    ib = __builtin_bit_cast(i64x2, w);
  }
  f32x4 acc[8];
  i32x4 iacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    iacc[j] = i32x4{0, 0, 0, 0};
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (I8)
        iacc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, ia), __builtin_bit_cast(i32x4, ib),
                                                        iacc[j], 0, 0, 0);
      else
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float r = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) r += I8 ? (float)(iacc[j][0] + iacc[j][3]) : acc[j][0] + acc[j][3];
  if (r == 1.2345f) sink[blockIdx.x * 256 + t] = r;   // keeps the loop alive; practically never stores
  if (t == 0) {
    clk[blockIdx.x * 2 + 0] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

// Streaming kernels: a workgroup moves one contiguous block of 256 x U x 16 B per iteration (thread t: pieces
// t, t + 256, ...: U loads in flight, every wave-instruction one 1 KiB contiguous run), blocks grid-strided over the
// buffer (n % (256 U) == 0 for the 1 GiB buffers). NT: nontemporal loads / stores (the streams have no reuse).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // native vector: the nontemporal builtins need one
template <int U, bool NT>
__global__ __launch_bounds__(256) void hbm_copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t blk = 256 * U, nblk = n / blk;
  for (size_t bi = blockIdx.x; bi < nblk; bi += gridDim.x) {
    const size_t o = bi * blk + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + o + 256 * u) : src[o + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        __builtin_nontemporal_store(v[u], dst + o + 256 * u);
      else
        dst[o + 256 * u] = v[u];
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void hbm_read_kernel(const u32x4* __restrict__ src, size_t n, uint32_t* __restrict__ sink) {
  const size_t blk = 256 * U, nblk = n / blk;
  uint32_t x = 0;
  for (size_t bi = blockIdx.x; bi < nblk; bi += gridDim.x) {
    const size_t o = bi * blk + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + o + 256 * u) : src[o + 256 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

// One record per workgroup: (cu_key, s_memtime, s_memrealtime).
__global__ void clock_stamp_kernel(unsigned long long* __restrict__ out) {
  if (threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 3 + 0] = cu_key();
    out[blockIdx.x * 3 + 1] = t;
    out[blockIdx.x * 3 + 2] = r;
  }
}

}  // namespace spef

using namespace spef;

namespace {
int ub_fail(const std::string& m) { return report_error(SPEF_ERR_HIP, m); }
#define UB_TRY(expr)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return ub_fail(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct Scratch {
  void* p[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  hipEvent_t e0 = nullptr, e1 = nullptr;
  ~Scratch() {
    for (void* q : p)
      if (q) (void)hipFree(q);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};

double median(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}
}  // namespace

// out[0] fp16 MFMA TFLOP/s, out[1] int8 MFMA TOP/s, out[2] HBM copy GB/s (read + write bytes), out[3] HBM read
// GB/s, out[4] shader clock MHz held in the fp16 loop, out[5] in the int8 loop, out[6] / out[7] the stream
// configuration that gave out[2] / out[3] (workgroups per CU * 100 + loads in flight per thread * 10 + nontemporal).
// Best of `reps` launches each (streams: best configuration of a small sweep).
static int measure_peaks_on(int device, int reps, double* out);
extern "C" int spef_measure_peaks(int device, int reps, double* out) {
  if (!out || reps < 1) return ub_fail("bad arguments");
  int prev = -1;   // restore the calling thread's current device on every exit path (torch shares the runtime)
  UB_TRY(hipGetDevice(&prev));
  UB_TRY(hipSetDevice(device));
  const int rc = measure_peaks_on(device, reps, out);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  return rc;
}

static int measure_peaks_on(int device, int reps, double* out) {
  hipDeviceProp_t prop;
  UB_TRY(hipGetDeviceProperties(&prop, device));
  const int cus = prop.multiProcessorCount;
  Scratch sc;
  const size_t hbm_bytes = (size_t)4 << 30;   // 4 GiB per buffer: 16x the 256 MB Infinity Cache, launch costs < 1 %
  UB_TRY(hipMalloc(&sc.p[0], 4096 * 16));
  UB_TRY(hipMalloc(&sc.p[1], (size_t)cus * 4 * 256 * sizeof(float)));
  UB_TRY(hipMalloc(&sc.p[2], (size_t)cus * 4 * 2 * sizeof(unsigned long long)));
  UB_TRY(hipMalloc(&sc.p[3], hbm_bytes));
  UB_TRY(hipMalloc(&sc.p[4], hbm_bytes));
  UB_TRY(hipEventCreate(&sc.e0));
  UB_TRY(hipEventCreate(&sc.e1));
  {
    std::vector<uint32_t> seed(4096 * 4);
    uint32_t x = 0x12345678u;
    for (auto& v : seed) {   // xorshift; fp16 bit patterns with the exponent kept moderate (finite, non-zero)
      x ^= x << 13;
      x ^= x >> 17;
      x ^= x << 5;
      v = (x & 0x83ff83ffu) | 0x38003800u;
    }
    UB_TRY(hipMemcpy(sc.p[0], seed.data(), seed.size() * 4, hipMemcpyHostToDevice));
  }
  UB_TRY(hipMemset(sc.p[3], 1, hbm_bytes));
  UB_TRY(hipMemset(sc.p[4], 0, hbm_bytes));
  const int wgs = cus * 4;   // 16 waves per CU = 4 per SIMD, 8 independent chains each
  auto time_launch = [&](auto&& launch, float* ms) -> int {
    UB_TRY(hipEventRecord(sc.e0, nullptr));
    launch();
    UB_TRY(hipGetLastError());
    UB_TRY(hipEventRecord(sc.e1, nullptr));
    UB_TRY(hipEventSynchronize(sc.e1));
    UB_TRY(hipEventElapsedTime(ms, sc.e0, sc.e1));
    return SPEF_OK;
  };
  for (int kind = 0; kind < 2; ++kind) {
    const int iters = 4096;
    double best = 0.0, clk = 0.0;
    for (int r = 0; r < reps + 1; ++r) {   // first launch = warm-up (clock ramp)
      float ms = 0.f;
      int rc = time_launch([&] {
        if (kind == 0)
          mfma_peak_kernel<false><<<wgs, 256>>>((const uint32_t*)sc.p[0], iters, (float*)sc.p[1], (unsigned long long*)sc.p[2]);
        else
          mfma_peak_kernel<true><<<wgs, 256>>>((const uint32_t*)sc.p[0], iters, (float*)sc.p[1], (unsigned long long*)sc.p[2]);
      }, &ms);
      if (rc) return rc;
      const double ops = (double)wgs * 4 * iters * 8 * (kind == 0 ? 16.0 * 16 * 32 * 2 : 16.0 * 16 * 64 * 2);
      const double rate = ops / (ms * 1e-3) / 1e12;
      if (r > 0 && rate > best) {
        best = rate;
        std::vector<unsigned long long> ck((size_t)wgs * 2);
        UB_TRY(hipMemcpy(ck.data(), sc.p[2], ck.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> mhz;
        for (int w = 0; w < wgs; ++w)
          if (ck[2 * w + 1]) mhz.push_back((double)ck[2 * w] / (double)ck[2 * w + 1] * 100.0);
        clk = median(mhz);
      }
    }
    out[kind] = best;
    out[4 + kind] = clk;
  }
  const size_t n16 = hbm_bytes / 16;
  double best_copy = 0.0, best_read = 0.0, cfg_copy = 0.0, cfg_read = 0.0;
  for (int wpc : {4, 8, 16, 0}) {       // workgroups (of 4 waves) per CU; 0: one workgroup per block (no grid stride)
    for (int ui = 0; ui < 4; ++ui) {    // (loads in flight, nontemporal)
      const int U = ui < 2 ? 4 : 8;
      const bool nt = ui & 1;
      const double cfg = wpc * 100 + U * 10 + (nt ? 1 : 0);
      const size_t grid = wpc ? (size_t)cus * wpc : n16 / (256 * (size_t)U);
      auto copy = [&] {
        const u32x4* a = (const u32x4*)sc.p[3];
        u32x4* d = (u32x4*)sc.p[4];
        if (ui == 0) hbm_copy_kernel<4, false><<<grid, 256>>>(a, d, n16);
        else if (ui == 1) hbm_copy_kernel<4, true><<<grid, 256>>>(a, d, n16);
        else if (ui == 2) hbm_copy_kernel<8, false><<<grid, 256>>>(a, d, n16);
        else hbm_copy_kernel<8, true><<<grid, 256>>>(a, d, n16);
      };
      auto read = [&] {
        const u32x4* a = (const u32x4*)sc.p[4];
        uint32_t* k = (uint32_t*)sc.p[1];
        if (ui == 0) hbm_read_kernel<4, false><<<grid, 256>>>(a, n16, k);
        else if (ui == 1) hbm_read_kernel<4, true><<<grid, 256>>>(a, n16, k);
        else if (ui == 2) hbm_read_kernel<8, false><<<grid, 256>>>(a, n16, k);
        else hbm_read_kernel<8, true><<<grid, 256>>>(a, n16, k);
      };
      for (int r = 0; r < reps + 3; ++r) {   // streams: best of reps + 2 (the copy's spread is a few %)
        float ms = 0.f;
        int rc = time_launch(copy, &ms);
        if (rc) return rc;
        const double gc = 2.0 * hbm_bytes / (ms * 1e-3) / 1e9;
        if (r > 0 && gc > best_copy) best_copy = gc, cfg_copy = cfg;
        rc = time_launch(read, &ms);
        if (rc) return rc;
        const double gr = (double)hbm_bytes / (ms * 1e-3) / 1e9;
        if (r > 0 && gr > best_read) best_read = gr, cfg_read = cfg;
      }
    }
  }
  out[2] = best_copy;
  out[3] = best_read;
  out[6] = cfg_copy;
  out[7] = cfg_read;
  return SPEF_OK;
}

// n_wg single-wave workgroups each write (xcc id, s_memtime, s_memrealtime) to out (device, n_wg x 3 uint64).
extern "C" int spef_clock_stamp(void* out, int n_wg, void* stream) {
  if (!out || n_wg < 1) return ub_fail("bad arguments");
  clock_stamp_kernel<<<n_wg, 64, 0, (hipStream_t)stream>>>((unsigned long long*)out);
  UB_TRY(hipGetLastError());
  return SPEF_OK;
}
