// C ABI (include/spef.h) and the layer executor of the SPEF MI355X target.
//
// The executor walks the blob's op list (stem -> 17 inverted residuals -> last 1x1 -> head) over four NHWC
// activation buffers sized at spef_reserve time. Default schedule: the uint8 front kernel (stem + block 1), one
// fused kernel per inverted residual (LDS-slab or wave-specialised), the last 1x1 conv fused with the global mean,
// the FC head; SPEF_OPT_FUSE_BLOCKS=0 runs one kernel per conv instead (bit-identical). Also here: blob
// validation and loading, the RCCL weight broadcast, decode dispatch and the per-launch profiler.
#include "../../include/spef.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <map>
#include <mutex>
#include <thread>

#include <string>
#include <vector>

#include "spef_blob.hpp"
#include "spef_kernels.hpp"
#include "spef_tuning.hpp"

using namespace spef;

static thread_local std::string g_err;
static const int kKpSplits = 60;   // split-K slices of the keypoint head (K = 122880 -> 2048 per slice)

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
namespace spef {
int report_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace spef

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t e_ = (expr);                                                                            \
    if (e_ != hipSuccess) return fail(SPEF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct spef_ctx {
  int device = 0;
  BlobHeader hdr{};
  std::vector<OpDesc> ops;
  uint8_t* d_data = nullptr;  // device copy of the blob's data section
  size_t data_bytes = 0;
  bool loaded = false;
  // workspace
  int ws_B = 0, ws_H = 0, ws_W = 0;
  size_t buf_bytes = 0;
  void* buf[4] = {nullptr, nullptr, nullptr, nullptr};
  float* pooled = nullptr;  // [B][1280] fp32
  float* kpfeat = nullptr;  // keypoint head: fp32 NHWC feature map [B][fh*fw*1280]
  float* kppart = nullptr;  // keypoint head: split-K partials
  // keypoint decode configuration (KeyPoints, keypoints_utils.py:19-45; Camera, speed.py:18-32)
  float* kp3d = nullptr;
  double* kp_model = nullptr;  // control points [4][3] + alphas [n][4] (fp64, computed once on the host)
  int kp_n = 0;
  double camK[9] = {0};
  float cam_nu = 0.f, cam_nv = 0.f;
  EpnpDist kp_dist = {0, 0, 0, 0, 0, 0};   // spef_set_keypoint_distortion
  // decode tables
  double* d_ori_bins = nullptr;
  int n_ori_bins = 0;
  double* d_pos_grid = nullptr;
  int n_pos_bins = 0;
  int fuse = 1;              // SPEF_OPT_FUSE_BLOCKS: 0 never, 1 when input H*W >= fuse_min_hw
  int64_t fuse_min_hw = 0;   // SPEF_OPT_FUSE_MIN_HW
  int gemm = 1;              // SPEF_OPT_PW_GEMM: 1 LDS-tiled GEMM, 0 register-direct pw kernel
  int irb_variant = -1;      // SPEF_OPT_IRB_VARIANT: fused-block tile variant (tuning sweeps; -1 = library default)
  int wavespec = 2;          // SPEF_OPT_WAVESPEC: 2 = pipelined (k_irp.hip), 1 = wave-specialised (k_irw.hip)
  int q8_rolesplit = 0;      // SPEF_OPT_Q8_ROLESPLIT: int8 blocks 8-17 role-split (k_q8irw.hip)
  int test_fail_bcast = 0;   // SPEF_OPT_TEST_FAIL_BCAST (spef_tuning.hpp): failure injection in spef_bcast_weights
  bool probe_f16 = false;    // run_backbone: the activation it stopped at is fp16 (fp16mx: blocks 1-3)
  int mx_kernels = 1;        // SPEF_OPT_MX_KERNELS (spef_tuning.hpp): fp16mx blocks 2-7 on k_mx.hip
  // int8 blob: host copies of the FC quantisation constants, and their per-map-size device forms
  std::vector<double> q8_sw, q8_bias;
  std::vector<int32_t> q8_wsum;
  double q8_sl = 0.0;
  int32_t* q8_fc_init = nullptr;   // [Np] 128 * sum_k q_w + q_b (q_b depends on the pooled map size)
  float* q8_fc_sc = nullptr;       // [Np] f32(s_pool * s_w)
  int q8_fc_hw = 0, q8_fc_tb = 0;
  float q8_s_img = 0.f;                        // input scale (f32 NCHW path)
  int q8_last_bits = 8, q8_pool_bits = 8, q8_fc_bias_bits = 8;   // bit_width.json: last_conv act, pooling, FC bias
  // preprocessing (Pillow BILINEAR resize): coefficient tables for the last (Hin, Win, H, W), temp image
  int pre_key[4] = {0, 0, 0, 0};
  int* pre_bh = nullptr;   // [W][2] (xmin, count), then [W][ksize_h] coefficients
  int* pre_bv = nullptr;   // [H][2] (ymin - y0, count), then [H][ksize_v]
  int pre_ksh = 0, pre_ksv = 0, pre_y0 = 0, pre_ht = 0;
  uint8_t* pre_tmp = nullptr;
  size_t pre_tmp_bytes = 0;
  std::vector<std::array<int64_t, 3>> q8_res;  // per op: residual-join rescale (R, RB, RS)
  // per-launch HIP-event profiling (bench.py roofline leg)
  bool profiling = false;
  struct Rec {
    std::string key;
    hipEvent_t a, b;
    double bytes, flops;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t pool_next = 0;
};

namespace {

struct Dev {  // RAII device guard
  int prev = -1;
  explicit Dev(int d) {
    hipGetDevice(&prev);
    if (prev != d) hipSetDevice(d);
  }
  ~Dev() {
    if (prev >= 0) hipSetDevice(prev);
  }
};

inline int conv_out(int h, int s) { return (h + 2 - 3) / s + 1; }

hipEvent_t next_event(spef_ctx* c) {
  if (c->pool_next >= c->pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->pool.push_back(e);
  }
  return c->pool[c->pool_next++];
}

// Launch `fn` (returns hipError_t); when profiling, bracket it with events tagged by kernel key and its
// algorithmic bytes / flops (what roofline.achieved is priced in).
template <typename F>
hipError_t prof_launch(spef_ctx* c, hipStream_t s, const char* key, double bytes, double flops, F&& fn) {
  if (!c->profiling) return fn();
  hipEvent_t a = next_event(c), b = next_event(c);
  if (!a || !b) return hipErrorOutOfMemory;
  hipEventRecord(a, s);
  hipError_t e = fn();
  hipEventRecord(b, s);
  c->recs.push_back({key, a, b, bytes, flops});
  return e;
}

hipError_t pw_any(spef_ctx* c, int dt, int epi, const void* x, const void* wt, const float* bias, const void* r,
                  void* y, int64_t M, int K, int N, hipStream_t s) {
  if (dt == DT_F32) return launch_gemm_f32(epi, x, wt, bias, r, y, M, K, N, s);
  return c->gemm ? launch_gemm_pw(dt, epi, x, wt, bias, r, y, M, K, N, s)
                 : launch_pw(dt, epi, x, wt, bias, r, y, M, K, N, s);
}

const char* pw_key(int dt, int epi, int N);
const char* pw_any_key(spef_ctx* c, int dt, int epi, int N) {
  if (dt == DT_F32) return gemm_f32_key(N);
  return c->gemm ? gemm_key(dt, epi, N) : pw_key(dt, epi, N);
}

const char* pw_key(int dt, int epi, int N) {
  // mirrors pw_dispatch's tile choice so keys name the kernel instantiation rocprof reports
  static thread_local std::string k;
  const int n16 = ((N + 15) & ~15) / 16;
  int nt = 1, mt = 4;
  if (n16 == 1) { nt = 1; mt = 4; }
  else if (n16 == 2) { nt = 2; mt = 4; }
  else if (n16 == 4) { nt = 4; mt = 4; }
  else if (n16 % 6 == 0) { nt = 6; mt = 2; }
  else if (n16 % 5 == 0) { nt = 5; mt = 2; }
  else if (n16 % 4 == 0) { nt = 4; mt = 4; }
  else if (n16 % 3 == 0) { nt = 3; mt = 4; }
  else if (n16 % 2 == 0) { nt = 2; mt = 4; }
  k = std::string("pw_kernel<") + (dt == DT_F16 ? "F16" : "BF16") + "," + std::to_string(nt) + "," +
      std::to_string(mt) + "," + std::to_string(epi) + ">";
  return k.c_str();
}

template <typename T>
inline const T* ptr(const spef_ctx* c, uint64_t off) {
  return off == kAbsent ? nullptr : reinterpret_cast<const T*>(c->d_data + off);
}

// quantizer bit width of an int8 op (spef_blob.hpp qbits; 0 = 8)
static inline int qbits(const OpDesc& op, int i) { return op.qbits[i] ? op.qbits[i] : 8; }
// compute units of the current device (cached per device; launch_x2_irb sizes its tiles by the same query)
static int num_cus() {
  static int cus[32] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  dev &= 31;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 256;
  return cus[dev];
}

// QuantAvgPool2d + TruncTo8bit (ursonet.py:61-62, 88): the HW-pixel sum of last_conv's b_last-bit codes has
// b_last + ceil(log2 HW) bits; truncation to the pooling width drops the rest (oracle/int8_ref.py pool_shift).
static inline int q8_pool_shift(const spef_ctx* c, int hw) {
  int tb = 0;
  while ((1 << tb) < hw) ++tb;
  const int sh = c->q8_last_bits + tb - c->q8_pool_bits;
  return sh > 0 ? sh : 0;
}

size_t elem_size(const spef_ctx* c) {   // int8 | fp16 / bf16 | fp32 activations (fp32 and fp16x2 schedules)
  return c->hdr.dtype == DT_I8 ? 1 : (c->hdr.dtype == DT_F32 || c->hdr.dtype == DT_X2 || c->hdr.dtype == DT_MX) ? 4 : 2;
}

// algorithmic HBM bytes of one pointwise launch: read X, write Y (+ read residual), weights + bias once
double pw_bytes(int64_t M, uint32_t K, uint32_t N, bool res) {
  const double kp = (K + 31) & ~31u, np_ = (N + 15) & ~15u;
  return (double)M * K * 2 + (double)M * N * 2 * (res ? 2 : 1) + np_ * kp * 2 + np_ * 4;
}

// Max activation elements per image over the backbone schedule for an H x W input.
int64_t max_act_elems(const spef_ctx* c, int H, int W, int* fh, int* fw) {
  int64_t mx = 0;
  int h = H, w = W;
  for (const OpDesc& op : c->ops) {
    if (op.kind == OP_STEM || op.kind == OP_QSTEM) {
      h = conv_out(h, 2);
      w = conv_out(w, 2);
      mx = std::max<int64_t>(mx, (int64_t)h * w * op.cout);
    } else if (op.kind == OP_IRB || op.kind == OP_QIRB) {
      mx = std::max<int64_t>(mx, (int64_t)h * w * op.hidden);  // expand output
      const int oh = conv_out(h, op.stride), ow = conv_out(w, op.stride);
      mx = std::max<int64_t>(mx, (int64_t)oh * ow * op.hidden);
      mx = std::max<int64_t>(mx, (int64_t)oh * ow * op.cout);
      h = oh;
      w = ow;
    } else if (op.kind == OP_LAST || op.kind == OP_QLAST) {
      mx = std::max<int64_t>(mx, (int64_t)h * w * op.cout);  // unfused last conv (spef_backbone)
    }
  }
  if (fh) *fh = h;
  if (fw) *fw = w;
  return mx;
}

int check_ready(spef_ctx* c, int B, int H, int W) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  if (!c->loaded) return fail(SPEF_ERR_STATE, "weights not loaded (spef_load_weights)");
  if (B <= 0 || H < 32 || W < 32) return fail(SPEF_ERR_ARG, "bad input shape");
  if (B > c->ws_B || (int64_t)H * W > (int64_t)c->ws_H * c->ws_W || H != c->ws_H || W != c->ws_W)
    return fail(SPEF_ERR_STATE, "workspace not reserved for this shape (spef_reserve)");
  return SPEF_OK;
}

// Runs the backbone. mode: 0 = full (pool into c->pooled), 1 = stop after op `stop` and leave the
// activation in *out_buf, 2 = unfused last conv (feature map in *out_buf).
int run_backbone(spef_ctx* c, const void* input, int layout, int B, int H, int W, hipStream_t s, int mode,
                 int stop, void** out_buf, int* oc, int* oh, int* ow, float* feat_f32 = nullptr) {
  const int dt = (int)c->hdr.dtype;
  const bool f32 = dt == DT_F32;   // fp32 schedule: one kernel per conv (k_f32.hip), no fused kernels
  const bool x2 = dt == DT_X2 || dt == DT_MX;   // fp16x2 kernels: fused split-fp16 blocks (k_x2.hip)
  // fp16mx: the same weights; the block outputs with <= 24 channels (blocks 1-3: the 256^2 / 128^2 maps, DESIGN.md
  // section 5) are stored fp16, every other block output fp32
  const bool mx = dt == DT_MX;
  auto out16 = [&](const OpDesc& o) { return mx && o.cout <= 24; };
  bool cur16 = false;                  // the current activation is fp16 (fp16mx early blocks)
  const double es = (f32 || x2) ? 4.0 : 2.0;   // activation bytes per element (profiler byte counts)
  void* cur = nullptr;
  int h = H, w = W, ch = 3;
  int op_index = 0;
  bool skip_next = false;
  auto pick = [&](std::initializer_list<void*> busy) -> void* {
    for (void* b : c->buf) {
      bool used = false;
      for (void* u : busy) used |= (u == b);
      if (!used) return b;
    }
    return nullptr;
  };
  for (const OpDesc& op : c->ops) {
    if (skip_next) {  // block 1 already produced by the fused front kernel
      skip_next = false;
      if (mode == 1 && op_index == stop) break;
      ++op_index;
      continue;
    }
    if (op.kind == OP_STEM) {
      const int OH = conv_out(h, 2), OW = conv_out(w, 2);
      const OpDesc* nx = (&op + 1 < c->ops.data() + c->ops.size()) ? &op + 1 : nullptr;
      const bool front = !f32 && !x2 && c->fuse && layout == IN_U8_NHWC && !(mode == 1 && stop == 0) && nx && nx->kind == OP_IRB &&
                         nx->cin == 32 && nx->hidden == 32 && nx->cout == 16 && nx->expand == 1 && nx->stride == 1 &&
                         op.cout == 32 && op.x0 != kAbsent;
      const bool front_x2 = x2 && c->fuse && layout == IN_U8_NHWC && !(mode == 1 && stop == 0) && nx &&
                            nx->kind == OP_IRB && nx->cin == 32 && nx->hidden == 32 && nx->cout == 16 &&
                            nx->expand == 1 && nx->stride == 1 && op.cout == 32 && op.x0 != kAbsent;
      if (front_x2) {   // fp16x2: stem (MFMA, exact u8 operand) + block 1 in one kernel, fp32 (fp16mx: fp16) output
        void* y = c->buf[0];
        const double px = (double)B * OH * OW;
        const bool o16 = out16(*nx);
        const bool mxf = mx && o16 && c->mx_kernels && op.x1 != kAbsent;
        HIP_TRY(prof_launch(c, s, mxf ? "mx_front_kernel<stem+block1>" : "x2_front_kernel<stem+block1>",
                            (double)B * h * w * 3 + px * 16 * (o16 ? 2 : 4), px * (2 * 27 * 32 + 18 * 32 + 2 * 32 * 16),
                            [&] {
          if (mxf)
            return launch_mx_front(input, ptr<void>(c, op.x1), ptr<float>(c, op.b0), ptr<float>(c, nx->w1),
                                   ptr<float>(c, nx->b1), ptr<void>(c, nx->w2), ptr<float>(c, nx->b2), y, B, h, w, OH,
                                   OW, s);
          return launch_x2_front(input, ptr<void>(c, op.x0), ptr<float>(c, op.b0), ptr<float>(c, nx->w1),
                                 ptr<float>(c, nx->b1), ptr<void>(c, nx->w2), ptr<float>(c, nx->b2), y, B, h, w, OH,
                                 OW, s, o16);
        }));
        cur = y;
        cur16 = o16;
        h = OH;
        w = OW;
        ch = (int)nx->cout;
        skip_next = true;
        ++op_index;
        continue;
      }
      if (front) {
        void* y = c->buf[0];
        const double px = (double)B * OH * OW;
        HIP_TRY(prof_launch(c, s, "front_kernel<stem+block1>", (double)B * h * w * 3 + px * 16 * 2,
                            px * (2 * 27 * 32 + 18 * 32 + 2 * 32 * 16), [&] {
          return launch_front(dt, input, ptr<void>(c, op.x0), ptr<float>(c, op.b0), ptr<void>(c, nx->w1),
                              ptr<float>(c, nx->b1), ptr<void>(c, nx->w2), ptr<float>(c, nx->b2), y, B, h, w, OH, OW, s);
        }));
        cur = y;
        h = OH;
        w = OW;
        ch = (int)nx->cout;
        skip_next = true;
        ++op_index;
        continue;
      }
      void* y = c->buf[0];
      const double px = (double)B * OH * OW;
      const double in_b = (double)B * h * w * 3 * (layout == IN_U8_NHWC ? 1 : 4);
      HIP_TRY(prof_launch(c, s, layout == IN_U8_NHWC ? "stem_kernel<u8>" : "stem_kernel<f32>",
                          in_b + px * 32 * es, px * 2 * 27 * 32, [&] {
        return launch_stem(x2 ? (int)DT_F32 : dt, layout, input, ptr<float>(c, op.w0), ptr<float>(c, op.b0), y, B, h,
                           w, OH, OW, s);
      }));
      cur = y;
      h = OH;
      w = OW;
      ch = (int)op.cout;
    } else if (op.kind == OP_IRB) {
      const int64_t M = (int64_t)B * h * w;
      const int OH = conv_out(h, (int)op.stride), OW = conv_out(w, (int)op.stride);
      const bool res = op.flags & 1u;
      const bool expand = op.expand != 1;
      void* x = cur;
      if (x2) {   // fp16x2: one fused kernel per block, no unfused form
        if (!x2_irb_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res))
          return fail(SPEF_ERR_ARG, "fp16x2 schedule: unsupported inverted-residual geometry");
        void* y = pick({x});
        const int64_t M2 = (int64_t)B * OH * OW;
        const double flops = 2.0 * M * op.cin * op.hidden * (expand ? 1 : 0) + 18.0 * M2 * op.hidden +
                             2.0 * M2 * op.hidden * op.cout;
        const double hp = (op.hidden + 31) & ~31u;
        const bool o16 = out16(op);
        const int io = (cur16 ? 1 : 0) | (o16 ? 2 : 0);
        const double ib = cur16 ? 2 : 4, ob = o16 ? 2 : 4;
        // compulsory bytes: the block input once (a stride-1 residual IS that input: not counted twice), the output,
        // the weights once (the fp16 formula below counts the same way)
        const double bytes = (double)M * op.cin * ib + (double)M2 * op.cout * ob +
                             (expand ? hp * ((op.cin + 31) & ~31u) * 4 : 0) + hp * 48 +
                             ((op.cout + 15) & ~15u) * (hp * 4 + 4);
        char key[96];
        const bool mxk = mx && c->mx_kernels &&
                         mx_irb_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res, cur16,
                                          o16);
        const char* kn = mxk ? "mx_irb_kernel"
                             : x2_irb_kernel_name((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand,
                                                  res, B, OH, OW, true, io, num_cus());
        snprintf(key, sizeof(key), "%s<%u,%u,%u,s%u>", kn ? kn : "x2_irb_kernel", op.cin, op.hidden, op.cout,
                 op.stride);
        HIP_TRY(prof_launch(c, s, key, bytes, flops, [&] {
          if (mxk)
            return launch_mx_irb((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res, cur16, o16, x,
                                 ptr<void>(c, op.w0), ptr<float>(c, op.b0), ptr<float>(c, op.w1), ptr<float>(c, op.b1),
                                 ptr<void>(c, op.w2), ptr<float>(c, op.b2), y, B, h, w, OH, OW, s);
          // a third activation buffer (each holds the largest map) is the hidden-split form's partial-sum scratch
          return launch_x2_irb((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res, x,
                               ptr<void>(c, op.w0), ptr<float>(c, op.b0), ptr<float>(c, op.w1), ptr<float>(c, op.b1),
                               ptr<void>(c, op.w2), ptr<float>(c, op.b2), y, B, h, w, OH, OW, s,
                               (float*)pick({x, y}), io);
        }));
        cur = y;
        cur16 = o16;
        h = OH;
        w = OW;
        ch = (int)op.cout;
      } else if (!f32 && c->fuse && (int64_t)h * w >= c->fuse_min_hw && irb_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res)) {
        void* y = pick({x});
        const int64_t M2 = (int64_t)B * OH * OW;
        const double flops = 2.0 * M * op.cin * op.hidden * (expand ? 1 : 0) + 18.0 * M2 * op.hidden +
                             2.0 * M2 * op.hidden * op.cout;
        const double bytes = (double)M * op.cin * 2 + (double)M2 * op.cout * 2 +
                             (expand ? pw_bytes(0, op.cin, op.hidden, false) : 0) + 40.0 * op.hidden +
                             pw_bytes(0, op.hidden, op.cout, false);
        const bool pipe3 = c->wavespec >= 2 &&
                           irp_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res);
        const bool wspec = !pipe3 && c->wavespec &&
                           irw_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res);
        char key[96];
        snprintf(key, sizeof(key), "%s<%u,%u,%u,s%u>", pipe3 ? "irp_kernel" : wspec ? "irw_kernel" : "irb_kernel",
                 op.cin, op.hidden, op.cout, op.stride);
        HIP_TRY(prof_launch(c, s, key, bytes, flops, [&] {
          if (pipe3)
            return launch_irp(c->irb_variant, dt, (int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res, x,
                              ptr<void>(c, op.w0), ptr<float>(c, op.b0), ptr<void>(c, op.w1), ptr<float>(c, op.b1),
                              ptr<void>(c, op.w2), ptr<float>(c, op.b2), y, B, h, w, OH, OW, s);
          if (wspec)
            return launch_irw(c->irb_variant, dt, (int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res, x, ptr<void>(c, op.w0),
                              ptr<float>(c, op.b0), ptr<void>(c, op.w1), ptr<float>(c, op.b1), ptr<void>(c, op.w2),
                              ptr<float>(c, op.b2), y, B, h, w, OH, OW, s);
          return launch_irb(c->irb_variant, dt, (int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, expand, res, x,
                            ptr<void>(c, op.w0), ptr<float>(c, op.b0), ptr<void>(c, op.w1), ptr<float>(c, op.b1),
                            ptr<void>(c, op.w2), ptr<float>(c, op.b2), y, B, h, w, OH, OW, s);
        }));
        cur = y;
        h = OH;
        w = OW;
        ch = (int)op.cout;
      } else {
        void* h1 = x;
        if (expand) {
          h1 = pick({x});
          HIP_TRY(prof_launch(c, s, pw_any_key(c, dt, EPI_RELU, op.hidden), pw_bytes(M, op.cin, op.hidden, false) * es / 2,
                              2.0 * M * op.cin * op.hidden, [&] {
            return pw_any(c, dt, EPI_RELU, x, ptr<void>(c, op.w0), ptr<float>(c, op.b0), nullptr, h1, M,
                             (int)op.cin, (int)op.hidden, s);
          }));
        }
        void* h2 = pick({x, h1});
        const double opx = (double)B * OH * OW;
        const int dw_mode = irb_dw_mode(dt, (int)op.hidden, expand, (int)op.stride);
        static const char* const dw_names[2][3] = {{"dw_kernel<1>", "dw_kernel<1,pairs>", "dw_kernel<1,pk16>"},
                                                   {"dw_kernel<2>", "dw_kernel<2,pairs>", "dw_kernel<2,pk16>"}};
        HIP_TRY(prof_launch(c, s, dw_names[op.stride == 1 ? 0 : 1][dw_mode],
                            ((double)B * h * w + opx) * op.hidden * es + 40.0 * op.hidden, opx * op.hidden * 18.0, [&] {
          return launch_dw(dt, h1, ptr<void>(c, op.w1), ptr<float>(c, op.b1), h2, B, h, w, (int)op.hidden,
                           (int)op.stride, OH, OW, dw_mode, s);
        }));
        void* y = res ? pick({x, h2}) : pick({h2});
        const int64_t M2 = (int64_t)B * OH * OW;
        HIP_TRY(prof_launch(c, s, pw_any_key(c, dt, res ? EPI_RES : EPI_NONE, op.cout),
                            pw_bytes(M2, op.hidden, op.cout, res) * es / 2, 2.0 * M2 * op.hidden * op.cout, [&] {
          return pw_any(c, dt, res ? EPI_RES : EPI_NONE, h2, ptr<void>(c, op.w2), ptr<float>(c, op.b2),
                           res ? x : nullptr, y, M2, (int)op.hidden, (int)op.cout, s);
        }));
        cur = y;
        h = OH;
        w = OW;
        ch = (int)op.cout;
      }
    } else if (op.kind == OP_LAST) {
      if (x2 && mode == 0 && x2_pw_pool_supported(h * w, (int)op.cout)) {   // last conv + mean, map never stored
        float* part = (float*)pick({cur});
        const double M3 = (double)B * h * w;
        HIP_TRY(prof_launch(c, s, "x2_pw_kernel<pool>", M3 * op.cin * 4 + (double)op.cout * (op.cin * 4 + 4) +
                            (double)B * op.cout * 4, 2.0 * M3 * op.cin * op.cout, [&] {
          return launch_x2_pw_pool(cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), part, c->pooled, B, h * w,
                                   (int)op.cin, (int)op.cout, s);
        }));
      } else if (x2) {   // fp32 map (keypoint head input, feature export, or the URSONet mean's input)
        float* y = (mode == 2 && feat_f32) ? feat_f32 : (float*)pick({cur});
        const double M3 = (double)B * h * w;
        HIP_TRY(prof_launch(c, s, "x2_pw_kernel<4,4>", M3 * (op.cin + op.cout) * 4 + (double)op.cout * (op.cin * 4 + 4),
                            2.0 * M3 * op.cin * op.cout, [&] {
          return launch_x2_pw_relu(cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), y, (int64_t)B * h * w, (int)op.cin,
                                   (int)op.cout, s);
        }));
        cur = y;
        ch = (int)op.cout;
        if (mode == 0)
          HIP_TRY(prof_launch(c, s, "mean_hw_kernel", M3 * op.cout * 4 + (double)B * op.cout * 4, M3 * op.cout, [&] {
            return launch_mean_hw((const float*)cur, c->pooled, B, h * w, (int)op.cout, s);
          }));
      } else if (f32 && (mode == 0 || (mode == 2 && !feat_f32))) {   // fp32 map into a workspace buffer, then the mean
        void* y = pick({cur});
        const double M3 = (double)B * h * w;
        HIP_TRY(prof_launch(c, s, gemm_f32_key(op.cout), M3 * (op.cin + op.cout) * 4 + (double)op.cout * (op.cin + 1) * 4,
                            2.0 * M3 * op.cin * op.cout, [&] {
          return launch_gemm_f32(EPI_RELU, cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), nullptr, y,
                                 (int64_t)B * h * w, (int)op.cin, (int)op.cout, s);
        }));
        cur = y;
        ch = (int)op.cout;
        if (mode == 0)
          HIP_TRY(prof_launch(c, s, "mean_hw_kernel", M3 * op.cout * 4 + (double)B * op.cout * 4, M3 * op.cout, [&] {
            return launch_mean_hw((const float*)cur, c->pooled, B, h * w, (int)op.cout, s);
          }));
      } else if (f32 && mode == 2) {
        HIP_TRY(prof_launch(c, s, gemm_f32_key(op.cout), (double)B * h * w * (op.cin + op.cout) * 4,
                            2.0 * B * h * w * op.cin * op.cout, [&] {
          return launch_gemm_f32(EPI_RELU, cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), nullptr, feat_f32,
                                 (int64_t)B * h * w, (int)op.cin, (int)op.cout, s);
        }));
        cur = feat_f32;
        ch = (int)op.cout;
      } else if (mode == 0) {
        const double M3 = (double)B * h * w;
        const bool tiled = c->gemm && ((op.cout + 15) & ~15u) % 128 == 0;
        HIP_TRY(prof_launch(c, s, tiled ? "pool_gemm_kernel" : "pw_pool_kernel<4>",
                            M3 * op.cin * 2 + (double)op.cout * (op.cin * 2 + 4) + (double)B * op.cout * 4,
                            2.0 * M3 * op.cin * op.cout, [&] {
          return tiled ? launch_pool_gemm(dt, cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), c->pooled, B, h * w,
                                          (int)op.cin, (int)op.cout, s)
                       : launch_pw_pool(dt, cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), c->pooled, B, h * w,
                                        (int)op.cin, (int)op.cout, s);
        }));
      } else if (mode == 2 && feat_f32) {   // fp32 feature map straight from the GEMM epilogue
        HIP_TRY(prof_launch(c, s, gemm_key(dt, EPI_RELU_F32, op.cout), pw_bytes(B * h * w, op.cin, op.cout, false) +
                            (double)B * h * w * op.cout * 2, 2.0 * B * h * w * op.cin * op.cout, [&] {
          return launch_gemm_pw(dt, EPI_RELU_F32, cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), nullptr, feat_f32,
                                (int64_t)B * h * w, (int)op.cin, (int)op.cout, s);
        }));
        cur = feat_f32;
        ch = (int)op.cout;
      } else if (mode == 2) {
        void* y = pick({cur});
        HIP_TRY(pw_any(c, dt, EPI_RELU, cur, ptr<void>(c, op.w0), ptr<float>(c, op.b0), nullptr, y,
                          (int64_t)B * h * w, (int)op.cin, (int)op.cout, s));
        cur = y;
        ch = (int)op.cout;
      }
      break;
    }
    if (mode == 1 && op_index == stop) break;
    ++op_index;
  }
  c->probe_f16 = cur16;
  if (out_buf) *out_buf = cur;
  if (oc) *oc = ch;
  if (oh) *oh = h;
  if (ow) *ow = w;
  return SPEF_OK;
}

// ---- INT8 schedule (k_q8.hip): one kernel per conv. Activations: stem / expand outputs u8, depthwise outputs
// offset int8 (u - 128), block outputs int8 at the next consumer's scale, last conv u8.
// mode: 0 = full (pooled offset-int8 codes into c->pooled), 1 = stop after op `stop`, 2 = last conv map.
// *is_unsigned tells the caller how to read the returned codes.
int run_backbone_q8(spef_ctx* c, const void* input, int layout, int B, int H, int W, hipStream_t s, int mode,
                    int stop, void** out_buf, int* oc, int* oh, int* ow, int* is_unsigned) {
  void* cur = nullptr;
  int h = H, w = W, ch = 3, uns = 0;
  int op_index = 0;
  auto pick = [&](std::initializer_list<void*> busy) -> void* {
    for (void* b : c->buf) {
      bool used = false;
      for (void* u : busy) used |= (u == b);
      if (!used) return b;
    }
    return nullptr;
  };
  auto rqM = [&](uint64_t off) { return ptr<int64_t>(c, off); };
  auto rqB = [&](uint64_t off, uint32_t n) { return ptr<int64_t>(c, off) + ((n + 15) & ~15u); };
  auto rqS = [&](uint64_t off, uint32_t n) {
    return reinterpret_cast<const int32_t*>(ptr<int64_t>(c, off) + 2 * ((n + 15) & ~15u));
  };
  for (const OpDesc& op : c->ops) {
    if (op.kind == OP_QSTEM) {
      const int OH = conv_out(h, 2), OW = conv_out(w, 2);
      uint8_t* y = (uint8_t*)c->buf[0];
      const float s_img = c->q8_s_img;
      const double px = (double)B * OH * OW;
      HIP_TRY(prof_launch(c, s, layout == IN_U8_NHWC ? "q_stem_kernel<u8>" : "q_stem_kernel<f32>",
                          (double)B * h * w * 3 * (layout == IN_U8_NHWC ? 1 : 4) + px * 32, px * 2 * 27 * 32, [&] {
        return launch_q_stem(input, layout == IN_F32_NCHW, ptr<int8_t>(c, op.w1), s_img, qbits(op, 1),
                             ptr<int8_t>(c, op.w0), rqM(op.b0), rqB(op.b0, 32), rqS(op.b0, 32), qbits(op, 0), y, B, h,
                             w, OH, OW, s);
      }));
      cur = y;
      h = OH;
      w = OW;
      ch = 32;
      uns = 1;
    } else if (op.kind == OP_QIRB) {
      const int64_t M = (int64_t)B * h * w;
      const int OH = conv_out(h, (int)op.stride), OW = conv_out(w, (int)op.stride);
      const int64_t M2 = (int64_t)B * OH * OW;
      const bool res = op.flags & 1u;
      void* x = cur;
      if (c->fuse && op.x2 != kAbsent &&
          q_irb_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res, op.expand != 1)) {
        void* y = pick({x});
        const std::array<int64_t, 3>& r3 = c->q8_res[&op - c->ops.data()];
        // role-split form for blocks 8-17 with SPEF_OPT_Q8_ROLESPLIT (bit-identical either way)
        const bool qw = c->q8_rolesplit && op.expand != 1 &&
                        q_irw_supported((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res);
        char key[96];
        snprintf(key, sizeof(key), "%s<%u,%u,%u,s%u>", qw ? "q_irw_kernel" : "q_irb_kernel", op.cin, op.hidden,
                 op.cout, op.stride);
        HIP_TRY(prof_launch(c, s, key, (double)M * op.cin + (double)M2 * op.cout + (double)op.hidden * (op.cin + op.cout + 9),
                            2.0 * M * op.cin * op.hidden + 18.0 * M2 * op.hidden + 2.0 * M2 * op.hidden * op.cout, [&] {
          const QBits qb{qbits(op, 0), qbits(op, 1), qbits(op, 2)};
          if (qw)
            return launch_q_irw((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res, (op.flags & 4u) != 0,
                                (const int8_t*)x, ptr<int8_t>(c, op.w0), ptr<int8_t>(c, op.w2), ptr<int32_t>(c, op.x0),
                                ptr<uint8_t>(c, op.x2), r3[0], r3[1], (int)r3[2], qb, (int8_t*)y, B, h, w, OH, OW, s);
          return launch_q_irb((int)op.cin, (int)op.hidden, (int)op.cout, (int)op.stride, res, op.expand != 1,
                              (op.flags & 4u) != 0, (const int8_t*)x,
                              ptr<int8_t>(c, op.w0), ptr<int8_t>(c, op.w2), ptr<int32_t>(c, op.x0),
                              ptr<uint8_t>(c, op.x2), r3[0], r3[1], (int)r3[2], qb, (int8_t*)y, B, h, w, OH, OW, s);
        }));
        cur = y;
        h = OH;
        w = OW;
        ch = (int)op.cout;
        uns = 0;
        if (mode == 1 && op_index == stop) break;
        ++op_index;
        continue;
      }
      void* h1 = x;
      if (op.expand != 1) {
        h1 = pick({x});
        QGemmArgs a{};
        a.epi = QEPI_RELU;
        a.x = (const int8_t*)x;
        a.w = ptr<int8_t>(c, op.w0);
        a.rqM = rqM(op.b0);
        a.rqB = rqB(op.b0, op.hidden);
        a.rqS = rqS(op.b0, op.hidden);
        a.out_bits = qbits(op, 0);
        a.y = h1;
        a.M = M;
        a.K = (int)op.cin;
        a.N = (int)op.hidden;
        HIP_TRY(prof_launch(c, s, "q_gemm<relu>", (double)M * (op.cin + op.hidden) + (double)op.hidden * op.cin,
                            2.0 * M * op.cin * op.hidden, [&] { return launch_q_gemm(a, s); }));
      }
      void* h2 = pick({x, h1});
      HIP_TRY(prof_launch(c, s, "q_dw_kernel", (double)(M + M2) * op.hidden + 9.0 * op.hidden,
                          18.0 * M2 * op.hidden, [&] {
        return launch_q_dw((const uint8_t*)h1, ptr<int8_t>(c, op.w1), rqM(op.b1), rqB(op.b1, op.hidden),
                           rqS(op.b1, op.hidden), qbits(op, 1), (int8_t*)h2, B, h, w, (int)op.hidden, (int)op.stride,
                           OH, OW, s);
      }));
      void* y = res ? pick({x, h2}) : pick({h2});
      QGemmArgs a{};
      a.epi = res ? QEPI_PROJ_RES : QEPI_PROJ;
      a.x = (const int8_t*)h2;
      a.w = ptr<int8_t>(c, op.w2);
      a.init = ptr<int32_t>(c, op.x0);
      a.rqM = rqM(op.b2);
      a.rqB = rqB(op.b2, op.cout);
      a.rqS = rqS(op.b2, op.cout);
      a.out_bits = qbits(op, 2);
      if (res) {
        const std::array<int64_t, 3>& r3 = c->q8_res[&op - c->ops.data()];
        a.r = (const int8_t*)x;
        a.rm = r3[0];
        a.rb = r3[1];
        a.rs = (int)r3[2];
      }
      a.y = y;
      a.M = M2;
      a.K = (int)op.hidden;
      a.N = (int)op.cout;
      HIP_TRY(prof_launch(c, s, res ? "q_gemm<proj_res>" : "q_gemm<proj>",
                          (double)M2 * (op.hidden + op.cout * (res ? 2 : 1)) + (double)op.cout * op.hidden,
                          2.0 * M2 * op.hidden * op.cout, [&] { return launch_q_gemm(a, s); }));
      cur = y;
      h = OH;
      w = OW;
      ch = (int)op.cout;
      uns = 0;
    } else if (op.kind == OP_QLAST) {
      const int64_t M = (int64_t)B * h * w;
      void* y = pick({cur});
      QGemmArgs a{};
      a.epi = QEPI_RELU;
      a.x = (const int8_t*)cur;
      a.w = ptr<int8_t>(c, op.w0);
      a.rqM = rqM(op.b0);
      a.rqB = rqB(op.b0, op.cout);
      a.rqS = rqS(op.b0, op.cout);
      a.out_bits = qbits(op, 0);
      a.y = y;
      a.M = M;
      a.K = (int)op.cin;
      a.N = (int)op.cout;
      HIP_TRY(prof_launch(c, s, "q_gemm<last>", (double)M * (op.cin + op.cout) + (double)op.cout * op.cin,
                          2.0 * M * op.cin * op.cout, [&] { return launch_q_gemm(a, s); }));
      cur = y;
      ch = (int)op.cout;
      uns = 1;
      if (mode == 0) {
        const int tb = q8_pool_shift(c, h * w);
        HIP_TRY(prof_launch(c, s, "q_pool_kernel", (double)M * op.cout + (double)B * op.cout, (double)M * op.cout, [&] {
          return launch_q_pool((const uint8_t*)cur, (int8_t*)c->pooled, B, h * w, (int)op.cout, tb, s);
        }));
      }
      break;
    }
    if (mode == 1 && op_index == stop) break;
    ++op_index;
  }
  if (out_buf) *out_buf = cur;
  if (oc) *oc = ch;
  if (oh) *oh = h;
  if (ow) *ow = w;
  if (is_unsigned) *is_unsigned = uns;
  return SPEF_OK;
}

// FC constants for a pooled map of `hw` pixels (oracle/int8_ref.py head_params, same float64 expression order).
int q8_prepare_fc(spef_ctx* c, int hw) {
  if (c->q8_fc_hw == hw && c->q8_fc_init) return SPEF_OK;
  const int tb = q8_pool_shift(c, hw);
  const double s_pool = c->q8_sl * ldexp(1.0, tb) / hw;
  const double blo = -ldexp(1.0, c->q8_fc_bias_bits - 1), bhi = ldexp(1.0, c->q8_fc_bias_bits - 1) - 1;
  const size_t np_ = c->q8_sw.size();
  std::vector<int32_t> init(np_, 0);
  std::vector<float> sc(np_, 0.f);
  for (size_t i = 0; i < np_; ++i) {
    if (c->q8_sw[i] == 0.0) continue;   // padding rows
    double qb = nearbyint(c->q8_bias[i] / (s_pool * c->q8_sw[i]));
    qb = qb < blo ? blo : (qb > bhi ? bhi : qb);
    init[i] = c->q8_wsum[i] + (int32_t)qb;
    sc[i] = (float)(s_pool * c->q8_sw[i]);
  }
  if (!c->q8_fc_init) HIP_TRY(hipMalloc(&c->q8_fc_init, np_ * sizeof(int32_t)));
  if (!c->q8_fc_sc) HIP_TRY(hipMalloc(&c->q8_fc_sc, np_ * sizeof(float)));
  HIP_TRY(hipMemcpy(c->q8_fc_init, init.data(), np_ * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->q8_fc_sc, sc.data(), np_ * sizeof(float), hipMemcpyHostToDevice));
  c->q8_fc_hw = hw;
  c->q8_fc_tb = tb;
  return SPEF_OK;
}

void free_workspace(spef_ctx* c) {
  for (void*& b : c->buf) {
    if (b) hipFree(b);
    b = nullptr;
  }
  if (c->pooled) hipFree(c->pooled);
  c->pooled = nullptr;
  if (c->kpfeat) hipFree(c->kpfeat);
  c->kpfeat = nullptr;
  if (c->kppart) hipFree(c->kppart);
  c->kppart = nullptr;
  c->ws_B = c->ws_H = c->ws_W = 0;
  c->buf_bytes = 0;
}

}  // namespace

extern "C" {

int spef_abi_version(void) { return SPEF_ABI_VERSION; }

const char* spef_last_error(void) { return g_err.c_str(); }

int spef_init(int device, spef_ctx** out) {
  if (!out) return fail(SPEF_ERR_ARG, "out is null");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(SPEF_ERR_ARG, "device index out of range");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(SPEF_ERR_ARG, std::string("SPEF kernels are built for gfx950 only, device is ") + prop.gcnArchName);
  spef_ctx* c = new spef_ctx();
  c->device = device;
  *out = c;
  return SPEF_OK;
}

int spef_destroy(spef_ctx* c) {
  if (!c) return SPEF_OK;
  Dev d(c->device);
  free_workspace(c);
  if (c->d_data) hipFree(c->d_data);
  if (c->d_ori_bins) hipFree(c->d_ori_bins);
  if (c->d_pos_grid) hipFree(c->d_pos_grid);
  if (c->kp3d) hipFree(c->kp3d);
  if (c->kp_model) hipFree(c->kp_model);
  if (c->q8_fc_init) hipFree(c->q8_fc_init);
  if (c->pre_bh) hipFree(c->pre_bh);
  if (c->pre_bv) hipFree(c->pre_bv);
  if (c->pre_tmp) hipFree(c->pre_tmp);
  if (c->q8_fc_sc) hipFree(c->q8_fc_sc);
  for (hipEvent_t e : c->pool) hipEventDestroy(e);
  delete c;
  return SPEF_OK;
}

// Minimum byte extent of each tensor an op references (w0, b0, w1, b1, w2, b2, x0, x1, x2), from the op
// geometry and the blob layout in spef_blob.hpp; 0 where the op has no such tensor.
static void op_extents(const OpDesc& op, uint32_t dtype, uint64_t ext[9]) {
  auto r16 = [](uint64_t n) { return (n + 15) & ~15ull; };
  auto r32 = [](uint64_t n) { return (n + 31) & ~31ull; };
  auto r64 = [](uint64_t n) { return (n + 63) & ~63ull; };
  const uint64_t a = dtype == DT_F32 ? 4 : 2;             // fp16 / bf16 | fp32 weight storage
  const uint64_t rq = 20;                                 // int64 M + int64 B + int32 S per channel
  for (int i = 0; i < 9; ++i) ext[i] = 0;
  const uint64_t ci = op.cin, co = op.cout, h = op.hidden;
  if (dtype == DT_X2 || dtype == DT_MX) {   // fp16x2 / fp16mx: 1x1 weights as [2][rows][Kp] fp16 planes (hi, lo);
                                            // depthwise / biases padded to 32
    switch (op.kind) {
      case OP_STEM:
        ext[0] = 27 * co * 4; ext[1] = co * 4; ext[6] = 2 * 3 * co * 32 * 2;
        if (dtype == DT_MX) ext[7] = 2 * co * 32 * 2;   // front_mx_kernel's operand (row-triple k order)
        break;
      case OP_IRB:
        if (op.expand != 1) { ext[0] = 2 * r32(h) * r32(ci) * 2; ext[1] = r32(h) * 4; }
        ext[2] = 9 * r32(h) * 4; ext[3] = r32(h) * 4;
        ext[4] = 2 * r16(co) * r32(h) * 2; ext[5] = r16(co) * 4;
        break;
      case OP_LAST: ext[0] = 2 * r16(co) * r32(ci) * 2; ext[1] = r16(co) * 4; break;
      case OP_FC: case OP_FCKP: ext[0] = r16(co) * ci * 4; ext[1] = r16(co) * 4; break;
      default: break;
    }
    return;
  }
  switch (op.kind) {
    case OP_STEM: ext[0] = 27 * co * 4; ext[1] = co * 4; ext[6] = 2 * co * 32 * a; break;
    case OP_IRB:
      if (op.expand != 1) { ext[0] = r16(h) * r32(ci) * a; ext[1] = r16(h) * 4; }
      ext[2] = 9 * h * (dtype == DT_F16 ? 2 : 4); ext[3] = h * 4;
      ext[4] = r16(co) * r32(h) * a; ext[5] = r16(co) * 4;
      break;
    case OP_LAST: ext[0] = r16(co) * r32(ci) * a; ext[1] = r16(co) * 4; break;
    case OP_FC: case OP_FCKP: ext[0] = r16(co) * ci * 4; ext[1] = r16(co) * 4; break;
    case OP_QSTEM: ext[0] = 32 * 28; ext[1] = 32 * rq; ext[2] = 256; ext[6] = 4; break;
    case OP_QIRB: {
      if (op.expand != 1) { ext[0] = r16(h) * r64(ci); ext[1] = r16(h) * rq; }
      ext[2] = 9 * h; ext[3] = r16(h) * rq;
      ext[4] = r16(co) * r64(h); ext[5] = r16(co) * rq;
      ext[6] = r16(co) * 4;
      if (op.flags & 1u) ext[7] = 24;
      if (op.x2 != kAbsent) ext[8] = 16 * r32(h) * 2 + 16 * r16(co) + 2 * 9 * r32(h);
      break;
    }
    case OP_QLAST: ext[0] = r16(co) * r64(ci); ext[1] = r16(co) * rq; break;
    case OP_QFC: ext[0] = r16(co) * ci; ext[1] = r16(co) * 8; ext[2] = r16(co) * 8; ext[6] = r16(co) * 4; ext[7] = 8; break;
    default: break;
  }
}

// Parse and validate a blob's header + op table (host bytes: at least the first `meta_bytes` of the blob; `bytes`
// is the whole blob's size). Pure host code -- writes nothing but *h / *ops, and only on success.
static int parse_blob(const uint8_t* head_bytes, size_t meta_bytes, size_t bytes, BlobHeader* h_out,
                      std::vector<OpDesc>* ops_out) {
  if (meta_bytes < sizeof(BlobHeader) || bytes < sizeof(BlobHeader)) return fail(SPEF_ERR_BLOB, "blob too small");
  BlobHeader h;
  memcpy(&h, head_bytes, sizeof(h));
  if (memcmp(h.magic, kBlobMagic, 8) != 0) return fail(SPEF_ERR_BLOB, "bad blob magic");
  if (h.version != kBlobVersion) return fail(SPEF_ERR_BLOB, "unsupported blob version");
  if (h.dtype != DT_F16 && h.dtype != DT_BF16 && h.dtype != DT_I8 && h.dtype != DT_F32 && h.dtype != DT_X2 &&
      h.dtype != DT_MX)
    return fail(SPEF_ERR_BLOB, "unsupported blob dtype");
  if (h.n_ops == 0 || h.n_ops > 4096) return fail(SPEF_ERR_BLOB, "bad op count");
  // every term bounded on its own before any sum (a crafted ops_off near 2^64 must not wrap ops_end)
  if (h.ops_off < sizeof(BlobHeader) || h.ops_off > bytes || (uint64_t)h.n_ops * sizeof(OpDesc) > bytes - h.ops_off)
    return fail(SPEF_ERR_BLOB, "blob truncated");
  const uint64_t ops_end = h.ops_off + (uint64_t)h.n_ops * sizeof(OpDesc);
  if (ops_end > h.data_off || h.data_off > bytes ||
      h.data_bytes > bytes - h.data_off || ops_end > meta_bytes)
    return fail(SPEF_ERR_BLOB, "blob truncated");
  if (h.feat_c != 1280) return fail(SPEF_ERR_BLOB, "feature width must be 1280 (mobilenet_v2.py:232)");
  std::vector<OpDesc> ops(h.n_ops);
  memcpy(ops.data(), head_bytes + h.ops_off, h.n_ops * sizeof(OpDesc));
  int n_head = 0;
  for (const OpDesc& op : ops) {
    uint64_t ext[9];
    op_extents(op, h.dtype, ext);
    const uint64_t offs[9] = {op.w0, op.b0, op.w1, op.b1, op.w2, op.b2, op.x0, op.x1, op.x2};
    for (int i = 0; i < 9; ++i) {
      if (offs[i] == kAbsent) {
        if (ext[i] && !(op.kind == OP_QIRB && i == 8)) return fail(SPEF_ERR_BLOB, "op lacks a required tensor");
        continue;
      }
      if ((offs[i] & 15) || offs[i] >= h.data_bytes || ext[i] > h.data_bytes - offs[i])
        return fail(SPEF_ERR_BLOB, "tensor extent out of range / misaligned (op kind " + std::to_string(op.kind) + ")");
    }
    if ((op.kind == OP_IRB || op.kind == OP_QIRB) &&
        (op.cin % 8 || op.cout % 8 || op.hidden % 8 || (op.stride != 1 && op.stride != 2)))
      return fail(SPEF_ERR_BLOB, "unsupported inverted-residual geometry");
    const bool qop = op.kind >= OP_QSTEM && op.kind <= OP_QFC;
    if (qop != (h.dtype == DT_I8)) return fail(SPEF_ERR_BLOB, "op kind does not match the blob dtype");
    if (op.kind == OP_QSTEM && op.cout != 32) return fail(SPEF_ERR_BLOB, "int8 stem needs 32 outputs");
    for (int k = 0; k < 4; ++k)
      if (op.qbits[k] == 1 || op.qbits[k] == 2 || op.qbits[k] > 8 || (op.qbits[k] && !qop))
        return fail(SPEF_ERR_BLOB, "quantizer bit widths must be 3..8 (int8 ops only; quant.check_bit_width)");
    if (op.kind == OP_FC || op.kind == OP_QFC) {
      ++n_head;
      if (h.head != HEAD_URSONET || op.cin != h.feat_c || op.cout != h.n_out0 + h.n_out1)
        return fail(SPEF_ERR_BLOB, "URSONet head widths do not match the header");
    }
    if (op.kind == OP_FCKP) {
      ++n_head;
      if (h.head != HEAD_KEYPOINTS || op.cout != h.n_out0 || op.cin != (uint64_t)h.kp_fh * h.kp_fw * h.feat_c)
        return fail(SPEF_ERR_BLOB, "keypoint head widths do not match the header");
    }
  }
  if (n_head != 1) return fail(SPEF_ERR_BLOB, "blob must hold exactly one head op");
  *h_out = h;
  *ops_out = std::move(ops);
  return SPEF_OK;
}

// A blob parsed and copied into fresh device storage, not yet owned by any context (the first half of a
// transactional load: a failure anywhere leaves the context's current model untouched).
struct Staged {
  BlobHeader h{};
  std::vector<OpDesc> ops;
  uint8_t* dd = nullptr;
  std::vector<std::array<int64_t, 3>> q8_res;
  std::vector<double> q8_sw, q8_bias;
  std::vector<int32_t> q8_wsum;
  double q8_sl = 0.0;
  float q8_s_img = 0.f;
  int q8_last_bits = 8, q8_pool_bits = 8, q8_fc_bias_bits = 8;
  Staged() = default;
  Staged(const Staged&) = delete;
  Staged& operator=(const Staged&) = delete;
  ~Staged() {
    if (dd) hipFree(dd);
  }
};

// Stage the blob at `blob` (host or device memory) into `st`.
static int stage_blob(spef_ctx* c, const void* blob, size_t bytes, bool on_device, Staged* st) {
  if (!c || !blob) return fail(SPEF_ERR_ARG, "null argument");
  Dev d(c->device);
  std::vector<uint8_t> head;
  const uint8_t* hb;
  size_t meta;
  if (on_device) {   // header + op table live in the first bytes; fetch them to the host
    if (bytes < sizeof(BlobHeader)) return fail(SPEF_ERR_BLOB, "blob too small");
    BlobHeader h0;
    HIP_TRY(hipMemcpy(&h0, blob, sizeof(h0), hipMemcpyDeviceToHost));
    meta = std::max<size_t>(sizeof(h0), std::min<size_t>(bytes, (size_t)h0.data_off));
    head.resize(meta);
    HIP_TRY(hipMemcpy(head.data(), blob, meta, hipMemcpyDeviceToHost));
    hb = head.data();
  } else {
    hb = (const uint8_t*)blob;
    meta = bytes;
  }
  int rc = parse_blob(hb, meta, bytes, &st->h, &st->ops);
  if (rc) return rc;
  const BlobHeader& h = st->h;
  const std::vector<OpDesc>& ops = st->ops;
  HIP_TRY(hipMalloc(&st->dd, std::max<uint64_t>(h.data_bytes, 256)));
  uint8_t* dd = st->dd;
  const uint8_t* src = (const uint8_t*)blob + h.data_off;
  HIP_TRY(hipMemcpy(dd, src, h.data_bytes, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
  if (h.dtype == DT_I8) {   // small host-side constants of the int8 schedule, fetched once
    st->q8_res.assign(ops.size(), {0, 0, 0});
    for (size_t i = 0; i < ops.size(); ++i) {
      const OpDesc& op = ops[i];
      if (op.kind == OP_QSTEM) HIP_TRY(hipMemcpy(&st->q8_s_img, dd + op.x0, sizeof(float), hipMemcpyDeviceToHost));
      if (op.kind == OP_QLAST) {
        st->q8_last_bits = qbits(op, 0);
        st->q8_pool_bits = qbits(op, 1);
      }
      if (op.kind == OP_QFC) st->q8_fc_bias_bits = qbits(op, 0);
      if (op.kind == OP_QIRB && (op.flags & 1u))
        HIP_TRY(hipMemcpy(st->q8_res[i].data(), dd + op.x1, 3 * sizeof(int64_t), hipMemcpyDeviceToHost));
      if (op.kind == OP_QFC) {
        const size_t np_ = (op.cout + 15) & ~15u;
        st->q8_sw.resize(np_);
        st->q8_bias.resize(np_);
        st->q8_wsum.resize(np_);
        HIP_TRY(hipMemcpy(st->q8_sw.data(), dd + op.b0, np_ * sizeof(double), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(st->q8_bias.data(), dd + op.w1, np_ * sizeof(double), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(st->q8_wsum.data(), dd + op.x0, np_ * sizeof(int32_t), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&st->q8_sl, dd + op.x1, sizeof(double), hipMemcpyDeviceToHost));
      }
    }
  }
  return SPEF_OK;
}

// Second half: the context takes the staged model (cannot fail).
static void commit_staged(spef_ctx* c, Staged* st) {
  Dev d(c->device);
  free_workspace(c);
  if (c->d_data) hipFree(c->d_data);
  c->d_data = st->dd;
  st->dd = nullptr;
  c->data_bytes = st->h.data_bytes;
  c->hdr = st->h;
  c->ops = std::move(st->ops);
  c->q8_res = std::move(st->q8_res);
  c->q8_sw = std::move(st->q8_sw);
  c->q8_bias = std::move(st->q8_bias);
  c->q8_wsum = std::move(st->q8_wsum);
  c->q8_sl = st->q8_sl;
  c->q8_s_img = st->q8_s_img;
  c->q8_last_bits = st->q8_last_bits;
  c->q8_pool_bits = st->q8_pool_bits;
  c->q8_fc_bias_bits = st->q8_fc_bias_bits;
  c->q8_fc_hw = 0;
  c->loaded = true;
}

static int load_common(spef_ctx* c, const void* blob, size_t bytes, bool on_device) {
  Staged st;
  const int rc = stage_blob(c, blob, bytes, on_device, &st);
  if (rc) return rc;
  commit_staged(c, &st);
  return SPEF_OK;
}

int spef_load_weights(spef_ctx* c, const void* blob, size_t bytes) { return load_common(c, blob, bytes, false); }

int spef_load_weights_device(spef_ctx* c, const void* blob, size_t bytes) { return load_common(c, blob, bytes, true); }

int spef_validate_blob(const void* blob, size_t bytes, int* dtype, int* head, int* n_out0, int* n_out1) {
  if (!blob) return fail(SPEF_ERR_ARG, "null blob");
  BlobHeader h;
  std::vector<OpDesc> ops;
  const int rc = parse_blob((const uint8_t*)blob, bytes, bytes, &h, &ops);
  if (rc) return rc;
  if (dtype) *dtype = (int)h.dtype;
  if (head) *head = (int)h.head;
  if (n_out0) *n_out0 = (int)h.n_out0;
  if (n_out1) *n_out1 = (int)h.n_out1;
  return SPEF_OK;
}

#define NCCL_TRY(expr)                                                                                      \
  do {                                                                                                      \
    ncclResult_t r_ = (expr);                                                                               \
    if (r_ != ncclSuccess) return fail(SPEF_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_));  \
  } while (0)

// Communicators made by spef_comm_init: nonblocking (ncclConfig_t.blocking = 0) with a per-communicator timeout, so
// every wait below is bounded and a dead peer ends in ncclCommAbort instead of a hang. A communicator
// the host made itself is unknown here and gets kDefaultCommTimeoutMs.
namespace {
const int kDefaultCommTimeoutMs = 120000;
struct CommInfo {
  int timeout_ms;
  bool aborted;
};
std::mutex g_comm_mu;
std::map<void*, CommInfo> g_comms;

int comm_timeout(void* comm) {
  std::lock_guard<std::mutex> g(g_comm_mu);
  auto it = g_comms.find(comm);
  return it == g_comms.end() ? kDefaultCommTimeoutMs : it->second.timeout_ms;
}

using Clock = std::chrono::steady_clock;

// Abort the communicator (unblocks every kernel of it on this rank; the handle is dead afterwards) and fail.
int comm_abort_fail(ncclComm_t comm, const std::string& msg) {
  ncclCommAbort(comm);
  {
    std::lock_guard<std::mutex> g(g_comm_mu);
    auto it = g_comms.find((void*)comm);
    if (it != g_comms.end()) it->second.aborted = true;
    else g_comms[(void*)comm] = {kDefaultCommTimeoutMs, true};
  }
  return fail(SPEF_ERR_COMM, msg + " -- communicator aborted (ncclCommAbort)");
}

// Wait until a nonblocking RCCL call has left ncclInProgress; abort on error or at the deadline.
int comm_settle(ncclComm_t comm, ncclResult_t r, Clock::time_point deadline, const char* what) {
  while (r == ncclInProgress) {
    if (Clock::now() > deadline) return comm_abort_fail(comm, std::string(what) + ": timed out");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
    if (ncclCommGetAsyncError(comm, &r) != ncclSuccess) r = ncclSystemError;
  }
  if (r != ncclSuccess) return comm_abort_fail(comm, std::string(what) + ": " + ncclGetErrorString(r));
  return SPEF_OK;
}

// Wait for the stream's collectives to finish, polling the communicator's async error; abort at the deadline.
int comm_wait_stream(ncclComm_t comm, hipStream_t s, Clock::time_point deadline, const char* what, int inject) {
  for (;;) {
    const hipError_t e = inject ? hipErrorNotReady : hipStreamQuery(s);
    if (e == hipSuccess) return SPEF_OK;
    if (e != hipErrorNotReady) return comm_abort_fail(comm, std::string(what) + ": " + hipGetErrorString(e));
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(comm, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
      return comm_abort_fail(comm, std::string(what) + ": " + ncclGetErrorString(ae));
    if (Clock::now() > deadline) return comm_abort_fail(comm, std::string(what) + ": timed out");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}
}  // namespace

int spef_comm_unique_id(void* id_out, size_t cap) {
  if (!id_out || cap < sizeof(ncclUniqueId)) return fail(SPEF_ERR_ARG, "id buffer smaller than SPEF_COMM_ID_BYTES");
  static_assert(sizeof(ncclUniqueId) == SPEF_COMM_ID_BYTES, "SPEF_COMM_ID_BYTES != sizeof(ncclUniqueId)");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(id_out, &id, sizeof(id));
  return SPEF_OK;
}

int spef_comm_init(int device, int nranks, int rank, const void* id, int timeout_ms, void** comm_out) {
  if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks) return fail(SPEF_ERR_ARG, "bad communicator arguments");
  if (timeout_ms <= 0) timeout_ms = kDefaultCommTimeoutMs;
  Dev d(device);
  HIP_TRY(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, uid, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) return fail(SPEF_ERR_COMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  {
    std::lock_guard<std::mutex> g(g_comm_mu);
    g_comms[(void*)comm] = {timeout_ms, false};
  }
  const int rc = comm_settle(comm, r, Clock::now() + std::chrono::milliseconds(timeout_ms), "communicator init");
  if (rc) {   // aborted: the handle is gone
    std::lock_guard<std::mutex> g(g_comm_mu);
    g_comms.erase((void*)comm);
    return rc;
  }
  *comm_out = comm;
  return SPEF_OK;
}

int spef_comm_abort(void* comm) {
  if (!comm) return SPEF_OK;
  {
    std::lock_guard<std::mutex> g(g_comm_mu);
    auto it = g_comms.find(comm);
    if (it != g_comms.end() && it->second.aborted) return SPEF_OK;
  }
  comm_abort_fail((ncclComm_t)comm, "spef_comm_abort");
  return SPEF_OK;
}

int spef_comm_destroy(void* comm) {
  if (!comm) return SPEF_OK;
  bool aborted = false;
  {
    std::lock_guard<std::mutex> g(g_comm_mu);
    auto it = g_comms.find(comm);
    if (it != g_comms.end()) {
      aborted = it->second.aborted;
      g_comms.erase(it);
    }
  }
  if (aborted) return SPEF_OK;   // ncclCommAbort already released it
  ncclComm_t cm = (ncclComm_t)comm;
  const Clock::time_point dl = Clock::now() + std::chrono::milliseconds(kDefaultCommTimeoutMs);
  ncclResult_t r = ncclCommFinalize(cm);   // nonblocking communicators finalize asynchronously
  if (r == ncclInProgress) {
    while (r == ncclInProgress && Clock::now() < dl) {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
      if (ncclCommGetAsyncError(cm, &r) != ncclSuccess) r = ncclSystemError;
    }
  }
  if (r != ncclSuccess) {
    ncclCommAbort(cm);
    return fail(SPEF_ERR_COMM, std::string("ncclCommFinalize: ") + ncclGetErrorString(r) + " -- aborted");
  }
  NCCL_TRY(ncclCommDestroy(cm));
  return SPEF_OK;
}

// Collective weight broadcast with agreement: no rank enters a data collective unless every rank reported a good
// local state, and every rank returns the same verdict. Steps: header broadcast -> local checks + allocation ->
// all-reduce(MAX) of the status words -> op table + data broadcasts -> receivers stage (parse, copy, validate) ->
// second all-reduce(MAX) -> receivers commit. Any RCCL error or a wait past the communicator's timeout aborts the
// communicator (ncclCommAbort) and returns SPEF_ERR_COMM; a failing rank is named in spef_last_error on every rank.
// Status word: 0 = ok, else (error code << 16) | (failing rank + 1); MAX picks one failing rank deterministically.
int spef_bcast_weights(spef_ctx* c, void* comm_, int root) {
  if (!c || !comm_) return fail(SPEF_ERR_ARG, "null argument");
  ncclComm_t comm = (ncclComm_t)comm_;
  {
    std::lock_guard<std::mutex> g(g_comm_mu);
    auto it = g_comms.find(comm_);
    if (it != g_comms.end() && it->second.aborted) return fail(SPEF_ERR_COMM, "communicator was aborted");
  }
  int rank = 0, n = 0;
  NCCL_TRY(ncclCommUserRank(comm, &rank));
  NCCL_TRY(ncclCommCount(comm, &n));
  if (root < 0 || root >= n) return fail(SPEF_ERR_ARG, "root out of range");
  Dev d(c->device);
  const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(comm_timeout(comm_));
  const int inject = c->test_fail_bcast;   // spef_tuning.hpp SPEF_OPT_TEST_FAIL_BCAST
  struct Tmp {   // scratch freed on every exit path
    hipStream_t s = nullptr;
    uint8_t* hdr = nullptr;
    uint8_t* img = nullptr;
    int32_t* st = nullptr;
    ~Tmp() {   // (after an abort the communicator's kernels have been told to exit)
      if (s) hipStreamDestroy(s);
      if (hdr) hipFree(hdr);
      if (img) hipFree(img);
      if (st) hipFree(st);
    }
  } t;
  HIP_TRY(hipStreamCreateWithFlags(&t.s, hipStreamNonBlocking));
  HIP_TRY(hipMalloc(&t.hdr, sizeof(BlobHeader)));
  HIP_TRY(hipMalloc(&t.st, sizeof(int32_t)));
  int rc;
#define COMM_CALL(expr, what)                                                        \
  do {                                                                               \
    if ((rc = comm_settle(comm, (expr), deadline, what)) != SPEF_OK) return rc;      \
  } while (0)
#define COMM_WAIT(what, inj)                                                         \
  do {                                                                               \
    if ((rc = comm_wait_stream(comm, t.s, deadline, what, inj)) != SPEF_OK) return rc; \
  } while (0)
  // agree on a local status word; returns the MAX over ranks (or an error: communicator aborted)
  std::string local_msg;
  auto agree = [&](int local_code, int32_t* agreed, int inj) -> int {
    const int32_t w = local_code ? (int32_t)((local_code << 16) | (rank + 1)) : 0;
    HIP_TRY(hipMemcpyAsync(t.st, &w, sizeof(w), hipMemcpyHostToDevice, t.s));
    COMM_CALL(ncclAllReduce(t.st, t.st, 1, ncclInt32, ncclMax, comm, t.s), "status all-reduce");
    COMM_WAIT("status all-reduce", inj);
    HIP_TRY(hipMemcpy(agreed, t.st, sizeof(int32_t), hipMemcpyDeviceToHost));
    return SPEF_OK;
  };
  auto verdict = [&](int32_t agreed) -> int {
    const int code = agreed >> 16, bad = (agreed & 0xffff) - 1;
    if (bad == rank) return fail(code, local_msg + " (rank " + std::to_string(rank) + ", weight broadcast)");
    return fail(code, "weight broadcast failed on rank " + std::to_string(bad) + " (error " + std::to_string(code) +
                          "); every rank returns it and keeps its previous model");
  };

  // 1. header (a root without weights sends an all-zero header; the receivers' checks then fail together)
  BlobHeader h{};
  if (rank == root && c->loaded) h = c->hdr;
  HIP_TRY(hipMemcpy(t.hdr, &h, sizeof(h), hipMemcpyHostToDevice));
  COMM_CALL(ncclBroadcast(t.hdr, t.hdr, sizeof(h), ncclUint8, root, comm, t.s), "header broadcast");
  COMM_WAIT("header broadcast", inject == 3);
  HIP_TRY(hipMemcpy(&h, t.hdr, sizeof(h), hipMemcpyDeviceToHost));

  // 2. local checks and allocation, then agreement before any bulk collective
  int local = SPEF_OK;
  const size_t ops_bytes = (size_t)h.n_ops * sizeof(OpDesc);
  if (memcmp(h.magic, kBlobMagic, 8) != 0) {
    local = fail(SPEF_ERR_STATE, "broadcast root has no weights loaded");
  } else if (h.data_off > (1ull << 30) || h.data_bytes > (1ull << 36) || h.ops_off > h.data_off ||
             ops_bytes > h.data_off - h.ops_off) {
    local = fail(SPEF_ERR_BLOB, "broadcast header out of range");
  } else if (inject == 1) {
    local = fail(SPEF_ERR_HIP, "injected failure before the data broadcast (SPEF_OPT_TEST_FAIL_BCAST=1)");
  } else if (rank != root) {
    const size_t total = (size_t)h.data_off + (size_t)h.data_bytes;
    const hipError_t e = hipMalloc(&t.img, std::max<size_t>(total, 256));
    if (e != hipSuccess) {
      t.img = nullptr;
      local = fail(SPEF_ERR_HIP, std::string("hipMalloc of the broadcast image: ") + hipGetErrorString(e));
    }
  }
  if (local) local_msg = g_err;
  int32_t agreed = 0;
  if ((rc = agree(local, &agreed, 0)) != SPEF_OK) return rc;
  if (agreed) return verdict(agreed);

  // 3. op table + data section (receivers: into a full blob image they then stage like spef_load_weights_device)
  if (rank == root) {
    HIP_TRY(hipMalloc(&t.img, std::max<size_t>(ops_bytes, 256)));
    HIP_TRY(hipMemcpy(t.img, c->ops.data(), ops_bytes, hipMemcpyHostToDevice));
    COMM_CALL(ncclGroupStart(), "group start");
    COMM_CALL(ncclBroadcast(t.img, t.img, ops_bytes, ncclUint8, root, comm, t.s), "op-table broadcast");
    COMM_CALL(ncclBroadcast(c->d_data, c->d_data, h.data_bytes, ncclUint8, root, comm, t.s), "data broadcast");
    COMM_CALL(ncclGroupEnd(), "group end");
  } else {
    HIP_TRY(hipMemcpy(t.img, &h, sizeof(h), hipMemcpyHostToDevice));
    COMM_CALL(ncclGroupStart(), "group start");
    COMM_CALL(ncclBroadcast(t.img + h.ops_off, t.img + h.ops_off, ops_bytes, ncclUint8, root, comm, t.s),
              "op-table broadcast");
    COMM_CALL(ncclBroadcast(t.img + h.data_off, t.img + h.data_off, h.data_bytes, ncclUint8, root, comm, t.s),
              "data broadcast");
    COMM_CALL(ncclGroupEnd(), "group end");
  }
  COMM_WAIT("data broadcast", 0);

  // 4. receivers stage (full validation + device copy); all ranks agree before anyone commits
  Staged st;
  local = SPEF_OK;
  if (inject == 2) local = fail(SPEF_ERR_BLOB, "injected failure after the data broadcast (SPEF_OPT_TEST_FAIL_BCAST=2)");
  else if (rank != root) local = stage_blob(c, t.img, (size_t)h.data_off + (size_t)h.data_bytes, true, &st);
  local_msg = local ? g_err : std::string();
  if ((rc = agree(local, &agreed, 0)) != SPEF_OK) return rc;
  if (agreed) return verdict(agreed);
  if (rank != root) commit_staged(c, &st);   // the root keeps its loaded model
  return SPEF_OK;
#undef COMM_CALL
#undef COMM_WAIT
}

int spef_model_info(const spef_ctx* c, int* head, int* n_out0, int* n_out1, int* dtype, int* n_ops) {
  if (!c || !c->loaded) return fail(SPEF_ERR_STATE, "weights not loaded");
  if (head) *head = (int)c->hdr.head;
  if (n_out0) *n_out0 = (int)c->hdr.n_out0;
  if (n_out1) *n_out1 = (int)c->hdr.n_out1;
  if (dtype) *dtype = (int)c->hdr.dtype;
  if (n_ops) *n_ops = (int)c->ops.size();
  return SPEF_OK;
}

int spef_reserve(spef_ctx* c, int B, int H, int W) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  if (!c->loaded) return fail(SPEF_ERR_STATE, "weights not loaded");
  if (B <= 0 || H < 32 || W < 32) return fail(SPEF_ERR_ARG, "bad shape");
  if (B <= c->ws_B && H == c->ws_H && W == c->ws_W) return SPEF_OK;
  Dev d(c->device);
  int fh = 0, fw = 0;
  const int64_t per_img = max_act_elems(c, H, W, &fh, &fw);
  if (c->hdr.head == HEAD_KEYPOINTS && (fh != (int)c->hdr.kp_fh || fw != (int)c->hdr.kp_fw))
    return fail(SPEF_ERR_ARG, "keypoint head expects a fixed feature map size (keypoints.py:20)");
  free_workspace(c);
  const size_t bytes = (size_t)per_img * B * elem_size(c) + 256;
  for (void*& b : c->buf) HIP_TRY(hipMalloc(&b, bytes));
  HIP_TRY(hipMalloc(&c->pooled, (size_t)B * c->hdr.feat_c * sizeof(float)));
  if (c->hdr.head == HEAD_KEYPOINTS) {
    HIP_TRY(hipMalloc(&c->kpfeat, (size_t)B * fh * fw * c->hdr.feat_c * sizeof(float)));
    HIP_TRY(hipMalloc(&c->kppart, (size_t)kKpSplits * B * ((c->hdr.n_out0 + 15) & ~15u) * sizeof(float)));
  }
  if (c->hdr.dtype == DT_I8) {
    const int rc = q8_prepare_fc(c, fh * fw);
    if (rc) return rc;
  }
  c->buf_bytes = bytes;
  c->ws_B = B;
  c->ws_H = H;
  c->ws_W = W;
  return SPEF_OK;
}

int spef_forward(spef_ctx* c, const void* input, int layout, int B, int H, int W, float* out0, float* out1,
                 void* stream) {
  int rc = check_ready(c, B, H, W);
  if (rc) return rc;
  if (!input || !out0) return fail(SPEF_ERR_ARG, "null input/output");
  if (layout != SPEF_IN_U8_NHWC && layout != SPEF_IN_F32_NCHW) return fail(SPEF_ERR_ARG, "bad layout");
  Dev d(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (c->hdr.dtype == DT_I8) {   // INT8 path: backbone + TruncTo8bit pool + int8 FC (ursonet.py:36-93)
    if (!out1 && c->hdr.n_out1) return fail(SPEF_ERR_ARG, "null position output");
    int fh = 0, fw = 0;
    rc = run_backbone_q8(c, input, layout, B, H, W, s, 0, -1, nullptr, nullptr, &fh, &fw, nullptr);
    if (rc) return rc;
    if (fh * fw != c->q8_fc_hw) return fail(SPEF_ERR_STATE, "int8 head constants not prepared (spef_reserve)");
    for (const OpDesc& op : c->ops)
      if (op.kind == OP_QFC) {
        QGemmArgs a{};
        a.epi = QEPI_FC;
        a.x = (const int8_t*)c->pooled;
        a.w = ptr<int8_t>(c, op.w0);
        a.init = c->q8_fc_init;
        a.y = out0;
        a.y1 = out1;
        a.sc = c->q8_fc_sc;
        a.n_split = (int)c->hdr.n_out0;
        a.M = B;
        a.K = (int)op.cin;
        a.N = (int)op.cout;
        HIP_TRY(prof_launch(c, s, "q_gemm<fc>", (double)B * op.cin + (double)op.cout * op.cin + (double)B * op.cout * 4,
                            2.0 * B * op.cin * op.cout, [&] { return launch_q_gemm(a, s); }));
      }
    return SPEF_OK;
  }
  if (c->hdr.head == HEAD_URSONET) {
    if (!out1 && c->hdr.n_out1) return fail(SPEF_ERR_ARG, "null position output");
    rc = run_backbone(c, input, layout, B, H, W, s, 0, -1, nullptr, nullptr, nullptr, nullptr);
    if (rc) return rc;
    for (const OpDesc& op : c->ops)
      if (op.kind == OP_FC)
        HIP_TRY(prof_launch(c, s, "fc_kernel", ((double)B + op.cout) * op.cin * 4 + (double)B * op.cout * 4,
                            2.0 * B * op.cin * op.cout, [&] {
          return launch_fc(c->pooled, ptr<float>(c, op.w0), ptr<float>(c, op.b0), out0, (int)c->hdr.n_out0, out1,
                           (int)c->hdr.n_out1, B, (int)c->hdr.feat_c, s);
        }));
    return SPEF_OK;
  }
  // keypoint head (keypoints.py:24-27): flatten of the unpooled 1280 x fh x fw map -> Linear(122880, 24).
  // The blob stores the weight columns in NHWC flatten order, so the NHWC map is used as is.
  void* feat = nullptr;
  int fc_ = 0, fh = 0, fw = 0;
  rc = run_backbone(c, input, layout, B, H, W, s, 2, -1, &feat, &fc_, &fh, &fw, c->kpfeat);
  if (rc) return rc;
  const int64_t F = (int64_t)fh * fw * fc_;
  for (const OpDesc& op : c->ops)
    if (op.kind == OP_FCKP) {
      if ((int64_t)op.cin != F) return fail(SPEF_ERR_ARG, "keypoint head size does not match the feature map");
      HIP_TRY(prof_launch(c, s, "fc_splitk_kernel", ((double)B + op.cout) * F * 4, 2.0 * B * F * op.cout, [&] {
        return launch_fc_splitk(c->kpfeat, ptr<float>(c, op.w0), ptr<float>(c, op.b0), out0, (int)op.cout, B, (int)F,
                                kKpSplits, c->kppart, s);
      }));
    }
  return SPEF_OK;
}

int spef_backbone(spef_ctx* c, const void* input, int layout, int B, int H, int W, float* features, void* stream) {
  int rc = check_ready(c, B, H, W);
  if (rc) return rc;
  if (!input || !features) return fail(SPEF_ERR_ARG, "null input/output");
  Dev d(c->device);
  hipStream_t s = (hipStream_t)stream;
  void* feat = nullptr;
  int fc_ = 0, fh = 0, fw = 0;
  if (c->hdr.dtype == DT_I8) {   // dequantized last-conv map: code * s_l
    rc = run_backbone_q8(c, input, layout, B, H, W, s, 2, -1, &feat, &fc_, &fh, &fw, nullptr);
    if (rc) return rc;
    HIP_TRY(launch_q_to_f32(feat, features, (int64_t)B * fh * fw * fc_, 1, (float)c->q8_sl, s));
    return SPEF_OK;
  }
  rc = run_backbone(c, input, layout, B, H, W, s, 2, -1, &feat, &fc_, &fh, &fw, features);
  if (rc) return rc;
  return SPEF_OK;
}

int spef_probe(spef_ctx* c, const void* input, int layout, int B, int H, int W, int stop_op, float* out, int* oc,
               int* oh, int* ow, void* stream) {
  int rc = check_ready(c, B, H, W);
  if (rc) return rc;
  if (!input || !out) return fail(SPEF_ERR_ARG, "null input/output");
  Dev d(c->device);
  hipStream_t s = (hipStream_t)stream;
  void* act = nullptr;
  int ch = 0, h = 0, w = 0;
  if (c->hdr.dtype == DT_I8) {   // raw integer codes (stem: u8, block outputs: int8)
    int uns = 0;
    rc = run_backbone_q8(c, input, layout, B, H, W, s, 1, stop_op, &act, &ch, &h, &w, &uns);
    if (rc) return rc;
    HIP_TRY(launch_q_to_f32(act, out, (int64_t)B * h * w * ch, uns, 1.0f, s));
  } else {
    rc = run_backbone(c, input, layout, B, H, W, s, 1, stop_op, &act, &ch, &h, &w);
    if (rc) return rc;
    const int adt = c->hdr.dtype == DT_MX ? (c->probe_f16 ? (int)DT_F16 : (int)DT_F32) : (int)c->hdr.dtype;
    HIP_TRY(launch_to_f32(adt, act, out, (int64_t)B * h * w * ch, s));
  }
  if (oc) *oc = ch;
  if (oh) *oh = h;
  if (ow) *ow = w;
  return SPEF_OK;
}

int spef_set_decode_tables(spef_ctx* c, const double* ori_bins, int n_ori_bins, const double* pos_grid,
                           int n_pos_bins) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  if (n_ori_bins > 8192) return fail(SPEF_ERR_ARG, "at most 8192 orientation bins");
  Dev d(c->device);
  if (c->d_ori_bins) hipFree(c->d_ori_bins);
  if (c->d_pos_grid) hipFree(c->d_pos_grid);
  c->d_ori_bins = nullptr;
  c->d_pos_grid = nullptr;
  c->n_ori_bins = c->n_pos_bins = 0;
  if (ori_bins && n_ori_bins > 0) {
    HIP_TRY(hipMalloc(&c->d_ori_bins, sizeof(double) * 4 * n_ori_bins));
    HIP_TRY(hipMemcpy(c->d_ori_bins, ori_bins, sizeof(double) * 4 * n_ori_bins, hipMemcpyHostToDevice));
    c->n_ori_bins = n_ori_bins;
  }
  if (pos_grid && n_pos_bins > 0) {
    HIP_TRY(hipMalloc(&c->d_pos_grid, sizeof(double) * 3 * n_pos_bins));
    HIP_TRY(hipMemcpy(c->d_pos_grid, pos_grid, sizeof(double) * 3 * n_pos_bins, hipMemcpyHostToDevice));
    c->n_pos_bins = n_pos_bins;
  }
  return SPEF_OK;
}

int spef_decode(spef_ctx* c, int ori_mode, int pos_mode, const float* ori_raw, int n_ori, const float* pos_raw,
                int n_pos, int B, float* ori_soft, float* quat, float* pos_soft, float* pos, int* status, void* stream) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  if (B <= 0 || !ori_raw || !quat || !pos_raw || !pos || !status) return fail(SPEF_ERR_ARG, "null argument");
  // row widths must be the ones the decode describes (the kernels stride rows by the table sizes)
  if (ori_mode == SPEF_CLASSIFICATION && c->d_ori_bins && n_ori != c->n_ori_bins)
    return fail(SPEF_ERR_ARG, "orientation logits are " + std::to_string(n_ori) + " wide, the histogram has " +
                                  std::to_string(c->n_ori_bins) + " bins");
  if (ori_mode == SPEF_REGRESSION && n_ori != 4) return fail(SPEF_ERR_ARG, "orientation regression needs 4 outputs");
  if (pos_mode == SPEF_CLASSIFICATION && c->d_pos_grid && n_pos != c->n_pos_bins)
    return fail(SPEF_ERR_ARG, "position logits are " + std::to_string(n_pos) + " wide, the grid has " +
                                  std::to_string(c->n_pos_bins) + " bins");
  if (pos_mode == SPEF_REGRESSION && n_pos != 3) return fail(SPEF_ERR_ARG, "position regression needs 3 outputs");
  if (ori_mode != SPEF_CLASSIFICATION && ori_mode != SPEF_REGRESSION)
    return fail(SPEF_ERR_ARG, "ori_mode must be regression or classification");
  if (pos_mode != SPEF_CLASSIFICATION && pos_mode != SPEF_REGRESSION)
    return fail(SPEF_ERR_ARG, "pos_mode must be regression or classification");
  if (ori_mode == SPEF_CLASSIFICATION && !c->d_ori_bins)
    return fail(SPEF_ERR_STATE, "orientation bins not set (spef_set_decode_tables)");
  if (pos_mode == SPEF_CLASSIFICATION && !c->d_pos_grid)
    return fail(SPEF_ERR_STATE, "position grid not set (spef_set_decode_tables)");
  Dev d(c->device);
  hipStream_t s = (hipStream_t)stream;
  // the orientation kernel runs first: it writes every status word and, in position regression mode, copies the
  // raw position (no memset / copy launches); the position decode then ORs its bits in, in stream order
  const float* pos_src = (pos_mode == SPEF_REGRESSION && pos != pos_raw) ? pos_raw : nullptr;
  if (ori_mode == SPEF_CLASSIFICATION) {
    HIP_TRY(prof_launch(c, s, "decode_ori_kernel", (double)B * c->n_ori_bins * (ori_soft ? 8 : 4) + 32.0 * c->n_ori_bins,
                        (double)B * c->n_ori_bins * 30, [&] {
      return launch_decode_ori(ori_raw, B, c->n_ori_bins, c->d_ori_bins, ori_soft, quat, status, pos_src, pos, s);
    }));
  } else {
    HIP_TRY(launch_normalize_ori(ori_raw, B, quat, status, pos_src, pos, s));
  }
  if (pos_mode == SPEF_CLASSIFICATION)
    HIP_TRY(launch_decode_pos(pos_raw, B, c->n_pos_bins, c->d_pos_grid, pos_soft, pos, status, s));
  return SPEF_OK;
}

int spef_set_keypoints(spef_ctx* c, const float* kp3d, int n, const double* K, float nu, float nv) {
  if (!c || !kp3d || !K || n < 4 || n > 16) return fail(SPEF_ERR_ARG, "bad keypoint configuration");
  Dev d(c->device);
  if (c->kp3d) hipFree(c->kp3d);
  if (c->kp_model) hipFree(c->kp_model);
  c->kp3d = nullptr;
  c->kp_model = nullptr;
  HIP_TRY(hipMalloc(&c->kp3d, sizeof(float) * 3 * n));
  HIP_TRY(hipMemcpy(c->kp3d, kp3d, sizeof(float) * 3 * n, hipMemcpyHostToDevice));
  // epnp.cpp choose_control_points + compute_barycentric_coordinates depend only on the 3-D model: do them
  // once here (fp64). PCA axis signs are canonical (largest-|component| positive; oracle/epnp_ref.py too).
  std::vector<double> model(12 + 4 * (size_t)n);
  {
    double pw[16][3], c0[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j) {
        pw[i][j] = (double)kp3d[3 * i + j];
        c0[j] += pw[i][j] / n;
      }
    double a[3][3] = {}, v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j)
        for (int k = 0; k < 3; ++k) a[j][k] += (pw[i][j] - c0[j]) * (pw[i][k] - c0[k]);
    for (int sweep = 0; sweep < 50; ++sweep) {
      double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
      if (off < 1e-40) break;
      for (int p = 0; p < 2; ++p)
        for (int q = p + 1; q < 3; ++q) {
          if (fabs(a[p][q]) < 1e-300) continue;
          const double th = (a[q][q] - a[p][p]) / (2 * a[p][q]);
          const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1));
          const double cs = 1 / sqrt(t * t + 1), sn = t * cs;
          for (int k = 0; k < 3; ++k) {
            const double x = a[k][p], y = a[k][q];
            a[k][p] = cs * x - sn * y;
            a[k][q] = sn * x + cs * y;
          }
          for (int k = 0; k < 3; ++k) {
            const double x = a[p][k], y = a[q][k];
            a[p][k] = cs * x - sn * y;
            a[q][k] = sn * x + cs * y;
          }
          for (int k = 0; k < 3; ++k) {
            const double x = v[k][p], y = v[k][q];
            v[k][p] = cs * x - sn * y;
            v[k][q] = sn * x + cs * y;
          }
        }
    }
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
      for (int j = i + 1; j < 3; ++j)
        if (a[ord[j]][ord[j]] > a[ord[i]][ord[i]]) std::swap(ord[i], ord[j]);
    double cws[4][3];
    for (int j = 0; j < 3; ++j) cws[0][j] = c0[j];
    for (int i = 1; i < 4; ++i) {
      const int e = ord[i - 1];
      int big = 0;
      for (int j = 1; j < 3; ++j)
        if (fabs(v[j][e]) > fabs(v[big][e])) big = j;
      const double sgn = v[big][e] >= 0 ? 1.0 : -1.0;
      const double k = sqrt(std::max(a[e][e], 0.0) / n);
      for (int j = 0; j < 3; ++j) cws[i][j] = c0[j] + k * sgn * v[j][e];
    }
    double cc[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 1; j < 4; ++j) cc[i][j - 1] = cws[j][i] - cws[0][i];
    const double det = cc[0][0] * (cc[1][1] * cc[2][2] - cc[1][2] * cc[2][1]) -
                       cc[0][1] * (cc[1][0] * cc[2][2] - cc[1][2] * cc[2][0]) +
                       cc[0][2] * (cc[1][0] * cc[2][1] - cc[1][1] * cc[2][0]);
    if (fabs(det) < 1e-300) return fail(SPEF_ERR_ARG, "degenerate 3-D keypoint model");
    double ci[3][3];
    ci[0][0] = (cc[1][1] * cc[2][2] - cc[1][2] * cc[2][1]) / det;
    ci[0][1] = (cc[0][2] * cc[2][1] - cc[0][1] * cc[2][2]) / det;
    ci[0][2] = (cc[0][1] * cc[1][2] - cc[0][2] * cc[1][1]) / det;
    ci[1][0] = (cc[1][2] * cc[2][0] - cc[1][0] * cc[2][2]) / det;
    ci[1][1] = (cc[0][0] * cc[2][2] - cc[0][2] * cc[2][0]) / det;
    ci[1][2] = (cc[0][2] * cc[1][0] - cc[0][0] * cc[1][2]) / det;
    ci[2][0] = (cc[1][0] * cc[2][1] - cc[1][1] * cc[2][0]) / det;
    ci[2][1] = (cc[0][1] * cc[2][0] - cc[0][0] * cc[2][1]) / det;
    ci[2][2] = (cc[0][0] * cc[1][1] - cc[0][1] * cc[1][0]) / det;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 3; ++j) model[3 * i + j] = cws[i][j];
    for (int i = 0; i < n; ++i) {
      double al[3];
      for (int j = 0; j < 3; ++j)
        al[j] = ci[j][0] * (pw[i][0] - cws[0][0]) + ci[j][1] * (pw[i][1] - cws[0][1]) + ci[j][2] * (pw[i][2] - cws[0][2]);
      model[12 + 4 * i + 0] = 1.0 - al[0] - al[1] - al[2];
      model[12 + 4 * i + 1] = al[0];
      model[12 + 4 * i + 2] = al[1];
      model[12 + 4 * i + 3] = al[2];
    }
  }
  HIP_TRY(hipMalloc(&c->kp_model, sizeof(double) * model.size()));
  HIP_TRY(hipMemcpy(c->kp_model, model.data(), sizeof(double) * model.size(), hipMemcpyHostToDevice));
  c->kp_n = n;
  memcpy(c->camK, K, sizeof(c->camK));
  c->cam_nu = nu;
  c->cam_nv = nv;
  return SPEF_OK;
}

int spef_set_keypoint_distortion(spef_ctx* c, const double* dist, int n) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  if (n != 0 && n != 4 && n != 5) return fail(SPEF_ERR_ARG, "distortion: 0, 4 (k1 k2 p1 p2) or 5 (+ k3) coefficients");
  if (n && !dist) return fail(SPEF_ERR_ARG, "null distortion coefficients");
  EpnpDist d = {0, 0, 0, 0, 0, 0};
  if (n) {
    d.k1 = dist[0];
    d.k2 = dist[1];
    d.p1 = dist[2];
    d.p2 = dist[3];
    d.k3 = n == 5 ? dist[4] : 0.0;
    d.on = (d.k1 != 0 || d.k2 != 0 || d.p1 != 0 || d.p2 != 0 || d.k3 != 0) ? 1 : 0;
  }
  c->kp_dist = d;
  return SPEF_OK;
}

int spef_decode_keypoints(spef_ctx* c, const float* raw, int B, int apply_sigmoid, float* kp_out, float* quat,
                          float* pos, int* status, void* stream) {
  if (!c || !raw || !quat || !pos || !status || B <= 0) return fail(SPEF_ERR_ARG, "null argument");
  if (!c->kp3d) return fail(SPEF_ERR_STATE, "keypoints not configured (spef_set_keypoints)");
  Dev d(c->device);
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemsetAsync(status, 0, sizeof(int) * B, s));
  HIP_TRY(prof_launch(c, s, "epnp_kernel", (double)B * (2 * (c->kp_n + 1) * 8 + 28), (double)B * 1.0e5, [&] {
    return launch_epnp(raw, B, c->kp_n, c->kp3d, c->kp_model, c->camK, c->cam_nu, c->cam_nv, c->kp_dist, apply_sigmoid, kp_out,
                       quat, pos, status, s);
  }));
  return SPEF_OK;
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc (libImaging/Resample.c), BILINEAR filter (support 1):
// bounds [out][2] = (xmin, count), coefficients [out][ksize] in fixed point with 22 fractional bits.
static int pil_coeffs(int in_size, int out_size, std::vector<int>& bounds, std::vector<int>& kk) {
  const double scale = (double)(float)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  bounds.assign(2 * out_size, 0);
  kk.assign((size_t)out_size * ksize, 0);
  std::vector<double> k(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double w = t < 1.0 ? 1.0 - t : 0.0;
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (int x = 0; x < xmax; ++x)
      kk[(size_t)xx * ksize + x] = k[x] < 0 ? (int)(-0.5 + k[x] * (1 << 22)) : (int)(0.5 + k[x] * (1 << 22));
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}

int spef_preprocess(spef_ctx* c, const uint8_t* frames, int B, int Hin, int Win, uint8_t* out, int H, int W,
                    void* stream) {
  if (!c || !frames || !out) return fail(SPEF_ERR_ARG, "null argument");
  if (B <= 0 || Hin <= 0 || Win <= 0 || H <= 0 || W <= 0) return fail(SPEF_ERR_ARG, "bad preprocess shape");
  Dev d(c->device);
  hipStream_t s = (hipStream_t)stream;
  const int key[4] = {Hin, Win, H, W};
  if (memcmp(key, c->pre_key, sizeof(key)) != 0) {
    std::vector<int> bh, kh, bv, kv;
    c->pre_ksh = pil_coeffs(Win, W, bh, kh);
    c->pre_ksv = pil_coeffs(Hin, H, bv, kv);
    c->pre_y0 = bv[0];
    c->pre_ht = bv[2 * H - 2] + bv[2 * H - 1] - c->pre_y0;
    for (int i = 0; i < H; ++i) bv[2 * i] -= c->pre_y0;   // vertical bounds relative to the temp image
    std::vector<int> th(bh), tv(bv);
    th.insert(th.end(), kh.begin(), kh.end());
    tv.insert(tv.end(), kv.begin(), kv.end());
    if (c->pre_bh) hipFree(c->pre_bh);
    if (c->pre_bv) hipFree(c->pre_bv);
    c->pre_bh = c->pre_bv = nullptr;
    memset(c->pre_key, 0, sizeof(c->pre_key));
    HIP_TRY(hipMalloc(&c->pre_bh, th.size() * sizeof(int)));
    HIP_TRY(hipMalloc(&c->pre_bv, tv.size() * sizeof(int)));
    HIP_TRY(hipMemcpy(c->pre_bh, th.data(), th.size() * sizeof(int), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->pre_bv, tv.data(), tv.size() * sizeof(int), hipMemcpyHostToDevice));
    memcpy(c->pre_key, key, sizeof(key));
  }
  const size_t tmp = (size_t)B * c->pre_ht * W * 3;
  if (tmp > c->pre_tmp_bytes) {
    if (c->pre_tmp) hipFree(c->pre_tmp);
    c->pre_tmp = nullptr;
    c->pre_tmp_bytes = 0;
    HIP_TRY(hipMalloc(&c->pre_tmp, tmp));
    c->pre_tmp_bytes = tmp;
  }
  HIP_TRY(prof_launch(c, s, "resize_h_kernel", (double)B * c->pre_ht * Win * 3 + (double)tmp, 0.0, [&] {
    return launch_resize_h(frames, c->pre_tmp, c->pre_bh, c->pre_bh + 2 * W, c->pre_ksh, B, Hin, Win, c->pre_y0,
                           c->pre_ht, W, s);
  }));
  HIP_TRY(prof_launch(c, s, "resize_v_kernel", (double)tmp + (double)B * H * W * 3, 0.0, [&] {
    return launch_resize_v(c->pre_tmp, out, c->pre_bv, c->pre_bv + 2 * H, c->pre_ksv, B, c->pre_ht, H, W, s);
  }));
  return SPEF_OK;
}

int spef_set_option(spef_ctx* c, int option, int value) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  if (option == SPEF_OPT_FUSE_BLOCKS) {
    c->fuse = value != 0;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_FUSE_MIN_HW) {   // spef_tuning.hpp
    c->fuse_min_hw = value;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_IRB_VARIANT) {
    c->irb_variant = value;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_TEST_FAIL_BCAST) {
    if (value < 0 || value > 3) return fail(SPEF_ERR_ARG, "SPEF_OPT_TEST_FAIL_BCAST: 0..3");
    c->test_fail_bcast = value;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_PW_GEMM) {
    c->gemm = value != 0;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_Q8_ROLESPLIT) {
    if (value < 0 || value > 1) return fail(SPEF_ERR_ARG, "SPEF_OPT_Q8_ROLESPLIT: 0 or 1");
    c->q8_rolesplit = value;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_MX_KERNELS) {   // spef_tuning.hpp
    c->mx_kernels = value ? 1 : 0;
    return SPEF_OK;
  }
  if (option == SPEF_OPT_WAVESPEC) {
    if (value < 0 || value > 2) return fail(SPEF_ERR_ARG, "SPEF_OPT_WAVESPEC: 0, 1 or 2");
    c->wavespec = value;
    return SPEF_OK;
  }
  return fail(SPEF_ERR_ARG, "unknown option");
}

int spef_profile_begin(spef_ctx* c) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  c->recs.clear();
  c->pool_next = 0;
  c->profiling = true;
  return SPEF_OK;
}

int spef_profile_end(spef_ctx* c, char* buf, size_t cap, size_t* needed) {
  if (!c) return fail(SPEF_ERR_ARG, "null context");
  Dev d(c->device);
  c->profiling = false;
  // aggregate per kernel key: launches, total ms, algorithmic bytes, flops
  struct Agg {
    long n = 0;
    double ms = 0, bytes = 0, flops = 0;
  };
  std::vector<std::pair<std::string, Agg>> agg;
  for (auto& r : c->recs) {
    HIP_TRY(hipEventSynchronize(r.b));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
    Agg* a = nullptr;
    for (auto& kv : agg)
      if (kv.first == r.key) a = &kv.second;
    if (!a) {
      agg.push_back({r.key, Agg{}});
      a = &agg.back().second;
    }
    a->n += 1;
    a->ms += ms;
    a->bytes += r.bytes;
    a->flops += r.flops;
  }
  std::string js = "{";
  char tmp[512];
  for (size_t i = 0; i < agg.size(); ++i) {
    snprintf(tmp, sizeof(tmp), "%s\"%s\": [%ld, %.6f, %.1f, %.1f]", i ? ", " : "", agg[i].first.c_str(),
             agg[i].second.n, agg[i].second.ms, agg[i].second.bytes, agg[i].second.flops);
    js += tmp;
  }
  js += "}";
  c->recs.clear();
  c->pool_next = 0;
  if (needed) *needed = js.size() + 1;
  if (buf && cap > 0) {
    const size_t n = std::min(cap - 1, js.size());
    memcpy(buf, js.data(), n);
    buf[n] = 0;
    if (n < js.size()) return fail(SPEF_ERR_ARG, "profile buffer too small");
  }
  return SPEF_OK;
}

}  // extern "C"
