// Timeline harness for the fused block kernels (csrc/k_irb.hip, k_irw.hip, k_irp.hip): times one geometry with HIP events and
// records every wave's s_memtime at the SPEF_TRACE probes of one launch, then prints where a workgroup's time goes
// (prologue, per-chunk work and barrier wait per role, epilogue, launch ramp). Not part of the library.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-honor-nans -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form \
//     -I include -I spacecraft-pose-estimation-framework_amd/csrc tools/kbench/blk_trace.hip -o tools/kbench/blk_trace
//   ./tools/kbench/blk_trace irb|irw|irp CIN HID COUT STRIDE RES H W [B=64] [variant=0] [iters=50] [xscale=2]
//   ./tools/kbench/blk_trace front 3 32 16 2 0 H W [B=64] ...   (fp16 stem + block 1 on uint8 frames; timing only)
#ifndef SPEF_KBENCH_TIMING_ONLY   // -DSPEF_KBENCH_TIMING_ONLY: same harness, probes compiled out (timing only)
#define SPEF_KTRACE
#endif
#include "k_irb.hip"
#include "k_irp.hip"
#include "k_irw.hip"
#include "k_front.hip"


#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace spef;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static void* dev_random_f16(size_t n, float scale, unsigned seed) {
  std::vector<_Float16> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) h[i] = (_Float16)(scale * ((rand() & 0xffff) / 65535.0f - 0.5f));
  void* d;
  CK(hipMalloc(&d, n * 2));
  CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  return d;
}
static float* dev_random_f32(size_t n, float scale, unsigned seed) {
  std::vector<float> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((rand() & 0xffff) / 65535.0f - 0.5f);
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  if (argc < 9) {
    fprintf(stderr, "usage: %s irb|irw|irp CIN HID COUT STRIDE RES H W [B] [variant] [iters] [xscale]\n", argv[0]);
    return 2;
  }
  const bool irp = argv[1][2] == 'p', irb = argv[1][2] == 'b', front = argv[1][0] == 'f';
  const char* kname = front ? "front" : irb ? "irb" : irp ? "irp" : "irw";
  ++argv;
  --argc;
  const int cin = atoi(argv[1]), hid = atoi(argv[2]), cout = atoi(argv[3]), st = atoi(argv[4]);
  const bool res = atoi(argv[5]) != 0;
  const int H = atoi(argv[6]), W = atoi(argv[7]);
  const int B = argc > 8 ? atoi(argv[8]) : 64, variant = argc > 9 ? atoi(argv[9]) : 0;
  const int iters = argc > 10 ? atoi(argv[10]) : 50;
  const float xs = argc > 11 ? (float)atof(argv[11]) : 2.0f;   // input value range (data-dependent clocks)
  const int OH = (H + st - 1) / st, OW = (W + st - 1) / st;
  const int hidp = (hid + 31) / 32 * 32 + 32, wkp = (cin + 31) / 32 * 32, coutp = (cout + 15) / 16 * 16;
  void* x = dev_random_f16((size_t)B * H * W * cin, xs, 1);
  void* we = dev_random_f16((size_t)hidp * wkp, 0.2f, 2);
  float* be = dev_random_f32(hidp, 0.1f, 3);
  void* wd = dev_random_f16((size_t)9 * hidp, 0.5f, 4);
  float* bd = dev_random_f32(hidp, 0.1f, 5);
  void* wp = dev_random_f16((size_t)coutp * hidp, 0.2f, 6);
  float* bp = dev_random_f32(coutp, 0.1f, 7);
  void* y;
  CK(hipMalloc(&y, (size_t)B * OH * OW * cout * 2));

  // trace buffer: generous upper bound on workgroups (1 per 16 output pixels)
  const size_t max_wg = (size_t)B * ((OH * OW + 15) / 16);
  const size_t tn = max_wg * 16 * SPEF_TRACE_SLOTS;
  unsigned long long* tr;
  CK(hipMalloc(&tr, tn * 8));
  CK(hipMemset(tr, 0, tn * 8));
#ifdef SPEF_KTRACE
  CK(hipMemcpyToSymbol(HIP_SYMBOL(spef::spef_ktrace), &tr, sizeof(tr)));
#endif

  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto go = [&]() {
    if (front)
      CK(launch_front(DT_F16, x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s));
    else if (irb)
      CK(launch_irb(variant, DT_F16, cin, hid, cout, st, true, res, x, we, be, wd, bd, wp, bp, y, B, H, W, OH, OW, s));
    else
      CK((irp ? launch_irp : launch_irw)(variant, DT_F16, cin, hid, cout, st, res, x, we, be, wd, bd, wp, bp, y, B, H,
                                          W, OH, OW, s));
  };
  for (int i = 0; i < 5; ++i) go();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) go();
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1e3 * ms / iters;

  if (front) {   // no probes in the front kernel
    printf("%s avg launch %.2f us (%d iters)\n", kname, us, iters);
    return 0;
  }
#ifndef SPEF_KTRACE
  printf("%s avg launch %.2f us (%d iters, no probes)\n", kname, us, iters);
  return 0;
#endif
  CK(hipMemset(tr, 0, tn * 8));
  CK(hipEventRecord(e0, s));
  go();
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(tn);
  CK(hipMemcpy(h.data(), tr, tn * 8, hipMemcpyDeviceToHost));

  // geometry of the launched variant: workgroups / waves that wrote the end slot
  auto D = [](unsigned long long a, unsigned long long b) { return (double)(b - a); };
  int nwg = 0, nwaves = 0;
  std::vector<unsigned long long> hk(tn);
  CK(hipMemset(tr, 0xff, tn * 8));
  go();
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(hk.data(), tr, tn * 8, hipMemcpyDeviceToHost));
  for (size_t g = 0; g < max_wg; ++g) {
    int w = 0;
    for (int v = 0; v < 16; ++v)
      if (hk[(g * 16 + v) * SPEF_TRACE_SLOTS + SPEF_TRACE_SLOTS - 1] != ~0ull) ++w;
    if (w) {
      ++nwg;
      nwaves = std::max(nwaves, w);
    }
  }
  const int nch = (hid + 31) / 32;
  printf("%s geometry %d->%d->%d s%d res%d %dx%d B=%d variant %d: %d workgroups x %d waves, %d chunks\n", kname, cin, hid, cout,
         st, (int)res, H, W, B, variant, nwg, nwaves, nch);
  printf("avg launch %.2f us (%d iters, probes compiled in); traced launch %.2f us\n", us, iters, 1e3 * ms);
  double wall = 0;
  for (int g = 0; g < nwg; ++g) {
    double m = 0;
    for (int v = 0; v < nwaves; ++v) {
      const unsigned long long* r = &h[((size_t)g * 16 + v) * SPEF_TRACE_SLOTS];
      m = std::max(m, D(r[0], r[SPEF_TRACE_SLOTS - 1]));
    }
    wall += m;
  }
  printf("workgroup lifetime (max over its waves): %.0f cycles avg\n", wall / nwg);
  if (irb) {   // slots: 0 start, 1 prologue done, 2 after first barrier, per chunk c: 3+3c start, 4+3c expand done,
               // 5+3c after the chunk barrier (depthwise + project run to the next chunk's start), last = end
    printf("wave  prologue  firstbar  per chunk: expand  barrier  dw+project   epilogue\n");
    for (int v = 0; v < nwaves; ++v) {
      double pro = 0, b0 = 0, ex = 0, ba = 0, dw = 0, epi = 0;
      for (int g = 0; g < nwg; ++g) {
        const unsigned long long* r = &h[((size_t)g * 16 + v) * SPEF_TRACE_SLOTS];
        pro += D(r[0], r[1]);
        b0 += D(r[1], r[2]);
        for (int c = 0; c < nch; ++c) {
          ex += D(r[3 + 3 * c], r[4 + 3 * c]);
          ba += D(r[4 + 3 * c], r[5 + 3 * c]);
          dw += D(r[5 + 3 * c], c + 1 < nch ? r[6 + 3 * c] : r[SPEF_TRACE_SLOTS - 1]);
        }
        epi += 0;
      }
      const double n = (double)nwg * nch;
      printf("%4d  %8.0f  %8.0f  %17.0f  %7.0f  %10.0f\n", v, pro / nwg, b0 / nwg, ex / n, ba / n, dw / n);
    }
    return 0;
  }
  printf("wave  prologue  firstbar  expand0  chunk-work  chunk-barrier  (per chunk: work  barrier)  epilogue\n");
  for (int v = 0; v < nwaves; ++v) {
    double pro = 0, sync0 = 0, w0 = 0, work = 0, wait = 0, epi = 0;
    for (int g = 0; g < nwg; ++g) {
      const unsigned long long* r = &h[((size_t)g * 16 + v) * SPEF_TRACE_SLOTS];
      pro += D(r[0], r[1]);
      sync0 += D(r[2], r[3]) + D(r[4], r[5]);
      w0 += D(r[3], r[4]);
      for (int c = 0; c < nch; ++c) {
        work += D(r[5 + 2 * c], r[6 + 2 * c]);
        wait += D(r[6 + 2 * c], r[7 + 2 * c]);
      }
      epi += D(r[7 + 2 * (nch - 1)], r[SPEF_TRACE_SLOTS - 1]);
    }
    const double n = nwg;
    printf("%4d  %8.0f  %8.0f  %7.0f  %10.0f  %13.0f  %12.0f  %8.0f  %8.0f\n", v, pro / n, sync0 / n, w0 / n, work / n,
           wait / n, work / n / nch, wait / n / nch, epi / n);
  }
  return 0;
}
