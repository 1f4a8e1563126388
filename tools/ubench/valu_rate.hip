// VALU issue-rate microbenchmark (GPU box): 8 and 2 waves/SIMD, 8 independent accumulators per lane, N iterations.
// Prints cycles per wave64 instruction per SIMD for fp32/fp16 ops and the int8 requant ops (v_mad_i64_i32, v_med3_i32, ...):
// Build: hipcc -O3 --offload-arch=gfx950 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, int n, float s) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
  unsigned h = 0x3c003c00u ^ (threadIdx.x & 1);   // two fp16 values
  float b = s;
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(b));
        if constexpr (OP == 1) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(a[i]) : "v"(h), "v"(h));
        if constexpr (OP == 2) asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(a[i]) : "v"(h));
        if constexpr (OP == 3) {
          asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&a[i & 6])) : "v"(*reinterpret_cast<double*>(&a[(i + 2) & 6])), "v"(*reinterpret_cast<double*>(&a[(i + 4) & 6])));
        }
        if constexpr (OP == 4) asm volatile("v_dot2_f32_f16 %0, %1, %2, %0" : "+v"(a[i]) : "v"(h), "v"(h));
        if constexpr (OP == 5) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
        if constexpr (OP == 6) asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(b));
        if constexpr (OP == 7) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[i]) : "v"(h));
        // integer / fp64 ops of the int8 requant epilogue
        if constexpr (OP == 8)
          asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(*reinterpret_cast<long*>(&a[i & 6])) : "v"(h), "v"(b) : "vcc");
        if constexpr (OP == 9)
          asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(*reinterpret_cast<double*>(&a[i & 6])) : "v"(*reinterpret_cast<double*>(&a[(i + 2) & 6])), "v"(*reinterpret_cast<double*>(&a[(i + 4) & 6])));
        if constexpr (OP == 10) asm volatile("v_mul_hi_i32 %0, %1, %0" : "+v"(a[i]) : "v"(h));
        if constexpr (OP == 11) asm volatile("v_med3_i32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(h), "v"(b));
        if constexpr (OP == 12) asm volatile("v_cvt_f32_i32 %0, %1" : "=v"(a[i]) : "v"(h));
        if constexpr (OP == 13) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(*reinterpret_cast<double*>(&a[i & 6])) : "v"(h));
        if constexpr (OP == 14) asm volatile("v_mul_i32_i24 %0, %1, %0" : "+v"(a[i]) : "v"(h));
        if constexpr (OP == 15) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a[i]) : "v"(h));
      }
    }
  }
  float t = 0;
  for (int i = 0; i < 8; ++i) t += a[i];
  if (t == 12345.f) out[threadIdx.x] = t;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  int ncu = 256, wgs_per_cu = 8;   // 256-thread WGs: 8 per CU = 32 waves/CU = 8 waves/SIMD
  const int n = 2000;
  const char* names[] = {"v_fma_f32", "v_fma_mix_f32", "v_cvt_f32_f16", "v_pk_fma_f32", "v_dot2_f32_f16", "v_max_f32",
                         "v_cvt_pk_f16_f32", "v_add_u32", "v_mad_i64_i32", "v_fma_f64", "v_mul_hi_i32",
                         "v_med3_i32", "v_cvt_f32_i32", "v_cvt_f64_i32", "v_mul_i32_i24", "v_mul_lo_u32"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int waves_per_simd : {8, 2}) {
    int wgs = ncu * waves_per_simd;   // 4 waves per WG -> waves_per_simd WGs per CU
    for (int op = 0; op < 16; ++op) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        switch (op) {
          case 0: k<0><<<wgs, 256>>>(out, n, 1.f); break;
          case 1: k<1><<<wgs, 256>>>(out, n, 1.f); break;
          case 2: k<2><<<wgs, 256>>>(out, n, 1.f); break;
          case 3: k<3><<<wgs, 256>>>(out, n, 1.f); break;
          case 4: k<4><<<wgs, 256>>>(out, n, 1.f); break;
          case 5: k<5><<<wgs, 256>>>(out, n, 1.f); break;
          case 6: k<6><<<wgs, 256>>>(out, n, 1.f); break;
          case 7: k<7><<<wgs, 256>>>(out, n, 1.f); break;
          case 8: k<8><<<wgs, 256>>>(out, n, 1.f); break;
          case 9: k<9><<<wgs, 256>>>(out, n, 1.f); break;
          case 10: k<10><<<wgs, 256>>>(out, n, 1.f); break;
          case 11: k<11><<<wgs, 256>>>(out, n, 1.f); break;
          case 12: k<12><<<wgs, 256>>>(out, n, 1.f); break;
          case 13: k<13><<<wgs, 256>>>(out, n, 1.f); break;
          case 14: k<14><<<wgs, 256>>>(out, n, 1.f); break;
          case 15: k<15><<<wgs, 256>>>(out, n, 1.f); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1) {
          const double instr_per_simd = (double)waves_per_simd * n * 64;   // per SIMD, wave instructions
          const double cyc = ms * 1e-3 * 2.4e9;
          printf("waves/SIMD %d  %-18s %.2f cycles per wave-instruction per SIMD\n", waves_per_simd, names[op],
                 cyc / instr_per_simd);
        }
      }
    }
  }
  (void)wgs_per_cu;
  return 0;
}
