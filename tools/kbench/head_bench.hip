// Timing harness for the head and decode kernels (csrc/k_head.hip) at the bench workload: FC 1280 -> 1728 + 3 and
// the orientation decode (softmax + Markley average) over B images. Not part of the library.
//
//   tools/kbench/build.sh; ./tools/kbench/head_bench [B=64] [iters=200]
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
  const double t_fc = time_us(s, iters, [&] { CK(launch_fc(x, w, bias, o0, n0, o1, n1, B, K, s)); });
  const double t_dec =
      time_us(s, iters, [&] { CK(launch_decode_ori(o0, B, n0, bins, soft, quat, status, s)); });
  std::vector<float> hq4((size_t)B * 4);
  CK(hipMemcpy(hq4.data(), quat, hq4.size() * 4, hipMemcpyDeviceToHost));
  printf("B=%d: fc_kernel %.2f us (%.1f GB/s of weights+inputs), decode_ori_kernel %.2f us; quat[0] = %.5f %.5f %.5f %.5f\n",
         B, t_fc, ((double)Np * K + (double)B * K) * 4 / t_fc / 1e3, t_dec, hq4[0], hq4[1], hq4[2], hq4[3]);
  return 0;
}
