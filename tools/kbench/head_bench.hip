// Timing harness for the head and decode kernels (csrc/k_head.hip) at the bench workload: FC 1280 -> 1728 + 3 and
// the orientation decode (softmax + Markley average) over B images. Not part of the library.
//
//   tools/kbench/build.sh; ./tools/kbench/head_bench [B=64] [iters=200]
//   ./tools/kbench/head_trace [B=64]: the same, plus the decode_ori SPEF_TRACE timeline of one launch
#include "k_head.hip"

#include <cmath>
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

template <typename F>
static double time_us(hipStream_t s, int iters, F&& f) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return 1e3 * ms / iters;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 64, iters = argc > 2 ? atoi(argv[2]) : 200;
  const int K = 1280, n0 = 1728, n1 = 3, Np = (n0 + n1 + 15) / 16 * 16;
  srand(3);
  auto rnd = [](float s) { return s * ((rand() & 0xffff) / 65535.0f - 0.5f); };
  std::vector<float> hx((size_t)B * K), hw((size_t)Np * K), hb(Np), hq(4 * (size_t)n0 * 2);
  for (auto& v : hx) v = fabsf(rnd(2.f));
  for (auto& v : hw) v = rnd(0.05f);
  for (auto& v : hb) v = rnd(0.1f);
  std::vector<double> hbins((size_t)n0 * 4);
  for (int i = 0; i < n0; ++i) {   // random unit quaternions as bins
    double q[4], n = 0;
    for (int k = 0; k < 4; ++k) n += (q[k] = rnd(2.f)) * q[k];
    for (int k = 0; k < 4; ++k) hbins[4 * i + k] = q[k] / sqrt(n);
  }
  float *x, *w, *bias, *o0, *o1, *soft, *quat;
  double* bins;
  int* status;
  CK(hipMalloc(&x, hx.size() * 4));
  CK(hipMalloc(&w, hw.size() * 4));
  CK(hipMalloc(&bias, hb.size() * 4));
  CK(hipMalloc(&o0, (size_t)B * n0 * 4));
  CK(hipMalloc(&o1, (size_t)B * n1 * 4));
  CK(hipMalloc(&soft, (size_t)B * n0 * 4));
  CK(hipMalloc(&quat, (size_t)B * 4 * 4));
  CK(hipMalloc(&bins, hbins.size() * 8));
  CK(hipMalloc(&status, B * 4));
  CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bins, hbins.data(), hbins.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemset(status, 0, B * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t kFlush = (size_t)512 << 20;   // > the 256 MB MALL: evicts every cache level
  void* flush;
  CK(hipMalloc(&flush, kFlush));
#ifdef SPEF_KTRACE
  // the probe buffer is set before the first launch of the traced kernel (a null spef_ktrace faults)
  unsigned long long* tr;
  const size_t nt = (size_t)B * 16 * SPEF_TRACE_SLOTS;
  CK(hipMalloc(&tr, nt * 8));
  CK(hipMemset(tr, 0, nt * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(spef::spef_ktrace), &tr, sizeof(tr)));
#endif
  const double t_fc = time_us(s, iters, [&] { CK(launch_fc(x, w, bias, o0, n0, o1, n1, B, K, s)); });
  const double t_dec =
      time_us(s, iters, [&] { CK(launch_decode_ori(o0, B, n0, bins, soft, quat, status, nullptr, nullptr, s)); });
#ifdef SPEF_KTRACE
  {   // one traced launch after an L2 flush (as in the network, where the forward evicts the bins): per workgroup
      // (wave 0), the s_memtime deltas between consecutive probes
    constexpr int NS = 9;
    CK(hipMemsetAsync(flush, 1, kFlush, s));
    CK(launch_decode_ori(o0, B, n0, bins, soft, quat, status, nullptr, nullptr, s));
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(nt);
    CK(hipMemcpy(h.data(), tr, nt * 8, hipMemcpyDeviceToHost));
    double acc[NS] = {0}, mx[NS] = {0};
    for (int b = 0; b < B; ++b) {
      const unsigned long long* w0 = &h[(size_t)b * 16 * SPEF_TRACE_SLOTS];
      for (int k = 1; k < NS; ++k) {
        const double d = (double)(w0[k] - w0[k - 1]);
        acc[k] += d / B;
        mx[k] = d > mx[k] ? d : mx[k];
      }
    }
    const char* nm[NS] = {"", "load+local max", "max reduce", "exp+sum reduce", "moments", "LDS write+barrier",
                          "16x16 reduce+barrier", "10-lane reduce", "eigvec"};
    printf("decode_ori timeline (s_memtime ticks, wave 0; mean / max over %d workgroups):\n", B);
    for (int k = 1; k < NS; ++k) printf("  %-22s %8.0f %8.0f\n", nm[k], acc[k], mx[k]);
  }
#endif
  {   // cold: every decode after an L2/MALL flush, events around the decode only
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double tot = 0;
    const int n = 20;
    for (int i = 0; i < n; ++i) {
      CK(hipMemsetAsync(flush, i & 0xff, kFlush, s));
      CK(hipEventRecord(e0, s));
      CK(launch_decode_ori(o0, B, n0, bins, soft, quat, status, nullptr, nullptr, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
    }
    printf("decode_ori_kernel after a cache flush: %.2f us (events around one launch, mean of %d)\n", tot / n * 1e3, n);
  }
  std::vector<float> hq4((size_t)B * 4);
  CK(hipMemcpy(hq4.data(), quat, hq4.size() * 4, hipMemcpyDeviceToHost));
  printf("B=%d: fc_kernel %.2f us (%.1f GB/s of weights+inputs), decode_ori_kernel %.2f us; quat[0] = %.5f %.5f %.5f %.5f\n",
         B, t_fc, ((double)Np * K + (double)B * K) * 4 / t_fc / 1e3, t_dec, hq4[0], hq4[1], hq4[2], hq4[3]);
  return 0;
}
