// Host-side launchers of the SPEF HIP kernels (internal; the public C ABI is include/spef.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace spef {

// Sets the calling thread's spef_last_error() message and returns `code` (spef_api.cpp).
int report_error(int code, const std::string& msg);

enum Dtype : int {
  DT_F16 = 1, DT_BF16 = 2, DT_I8 = 3, DT_F32 = 4,
  DT_X2 = 5,   // fp32 I/O, split-fp16 MFMA (k_x2.hip)
  DT_MX = 6    // fp16mx: the fp16x2 weights; stem map, block outputs of blocks 1-3, hidden of blocks 2-4 stored fp16
};
enum Epi : int { EPI_NONE = 0, EPI_RELU = 1, EPI_RES = 2, EPI_RELU_F32 = 3 /* ReLU, fp32 output */ };
enum InLayout : int { IN_U8_NHWC = 0, IN_F32_NCHW = 1 };

// Stem ConvBnAct 3->32, 3x3, stride 2, pad 1, BN folded, ReLU. W: fp32 [27][32] (k = ky*9+kx*3+ci).
hipError_t launch_stem(int dtype, int in_layout, const void* in, const float* w, const float* bias, void* y,
                       int B, int H, int W, int OH, int OW, hipStream_t s);

// Pointwise 1x1 conv as C^T = W * X^T on MFMA: X [M][K] NHWC, Wt [Np][Kp] (zero padded), bias fp32 [Np],
// optional residual R [M][N]; Y [M][N].
hipError_t launch_pw(int dtype, int epi, const void* x, const void* wt, const float* bias, const void* r,
                     void* y, int64_t M, int K, int N, hipStream_t s);

// Same contract, LDS-tiled double-buffered MFMA GEMM (k_gemm.hip); gemm_key names the instantiation used.
hipError_t launch_gemm_pw(int dtype, int epi, const void* x, const void* wt, const float* bias, const void* r,
                          void* y, int64_t M, int K, int N, hipStream_t s);
const char* gemm_key(int dtype, int epi, int N);

// Depthwise 3x3 conv, pad 1, stride 1|2, BN folded, ReLU. W9: [9][C] (fp16 for fp16 blobs, fp32 for bf16),
// bias fp32 [C]. mode (irb_dw_mode; fp16 only for mode > 0): DW_PAIRS = the vertical-pair tap order of the fused fp16
// stride-1 blocks, DW_PK16 = the packed-fp16 accumulation of the fused fp16 stride-2 blocks.
hipError_t launch_dw(int dtype, const void* x, const void* w9, const float* bias, void* y, int B, int H, int W,
                     int C, int stride, int OH, int OW, int mode, hipStream_t s);

// Last 1x1 conv (+BN, ReLU) fused with the global mean over HW: pooled fp32 [B][N].
hipError_t launch_pw_pool(int dtype, const void* x, const void* wt, const float* bias, float* pooled, int B,
                          int HW, int K, int N, hipStream_t s);

// Same contract, LDS-tiled GEMM with a pixel-reducing epilogue (k_pool.hip); needs round_up(N,16) % 128 == 0.
hipError_t launch_pool_gemm(int dtype, const void* x, const void* wt, const float* bias, float* pooled, int B, int HW,
                            int K, int N, hipStream_t s);

// fp32 head GEMM (f32-input MFMA): out[b][i] = sum_k X[b][k] W[i][k] + bias[i], columns [0,n0) -> out0,
// [n0, n0+n1) -> out1. W fp32 [Np][K], K % 16 == 0.
hipError_t launch_fc(const float* x, const float* w, const float* bias, float* out0, int n0, float* out1, int n1,
                     int B, int K, hipStream_t s);

// Fused InvertedResidual block (expand -> depthwise -> project [+x]) for the geometries in k_irb.hip's table.
bool irb_supported(int cin, int hid, int cout, int stride, bool expand, bool res);
// How the fused kernel of this block evaluates its depthwise: DW_FP32 (v_fma_mix, fp32 accumulation), DW_PAIRS
// (vertical pairs: v_dot2_f32_f16 + v_fma_mix) or DW_PK16 (v_pk_fma_f16: two channels per op, fp16 accumulation).
// The unfused schedule runs dw_kernel in the same mode to stay bit-identical.
enum { DW_FP32 = 0, DW_PAIRS = 1, DW_PK16 = 2 };
int irb_dw_mode(int dtype, int hid, bool expand, int stride);
hipError_t launch_irb(int variant, int dtype, int cin, int hid, int cout, int stride, bool expand, bool res, const void* x,
                      const void* we, const float* be, const void* wd, const float* bd, const void* wp,
                      const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s);

// Wave-specialised fused block (expand waves feed depthwise/project waves through a double-buffered LDS slab) for
// the low-resolution geometries in k_irw.hip's table (same contract, bit-identical to the unfused kernels).
// Three-stage pipelined fused block (k_irp.hip): MFMA waves expand + project, VALU waves depthwise; same contract.
bool irp_supported(int cin, int hid, int cout, int stride, bool expand, bool res);
hipError_t launch_irp(int variant, int dtype, int cin, int hid, int cout, int stride, bool res, const void* x, const void* we,
                      const float* be, const void* wd, const float* bd, const void* wp, const float* bp, void* y, int B,
                      int H, int W, int OH, int OW, hipStream_t s);
bool irw_supported(int cin, int hid, int cout, int stride, bool expand, bool res);
hipError_t launch_irw(int variant, int dtype, int cin, int hid, int cout, int stride, bool res, const void* x, const void* we,
                      const float* be, const void* wd, const float* bd, const void* wp, const float* bp, void* y,
                      int B, int H, int W, int OH, int OW, hipStream_t s);

// Stem (u8 NHWC input) fused with inverted-residual block 1 (32 -> dw -> 16), k_front.hip. wsp: /255-folded stem
// weights split hi + lo in the activation dtype, [2][32][32] (blob OP_STEM x0).
hipError_t launch_front(int dtype, const void* x, const void* wsp, const float* bs, const void* wd, const float* bd,
                        const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s);

// fp32 schedule (k_f32.hip, blob dtype 4): 1x1 conv on the exact fp32 MFMA, same contract as launch_pw with fp32
// activations and weights ([Np][Kp] fp32); EPI_RELU_F32 = EPI_RELU. K % 4 == 0, N % 4 == 0.
hipError_t launch_gemm_f32(int epi, const void* x, const void* wt, const float* bias, const void* r, void* y,
                           int64_t M, int K, int N, hipStream_t s);
const char* gemm_f32_key(int N);
// fp16x2 schedule (k_x2.hip, blob dtype 5): fused inverted residual on fp32 NHWC activations with hi + lo fp16
// operands (3 MFMAs per product). we: [2][r32(hid)][r32(cin)] fp16 (hi plane, lo plane), be fp32 [r32(hid)],
// wd fp32 [9][r32(hid)], bd fp32 [r32(hid)], wp [2][r16(cout)][r32(hid)] fp16, bp fp32 [r16(cout)]; zero padded.
bool x2_irb_supported(int cin, int hid, int cout, int stride, bool expand, bool res);
// the kernel launch_x2_irb runs for these arguments ("x2_irb_kernel" / "x2_irw_kernel" / "x2_irp_kernel"; profiling
// labels), nullptr when none
const char* x2_irb_kernel_name(int cin, int hid, int cout, int stride, bool expand, bool res, int B, int OH, int OW,
                               bool scratch, int io, int num_cu);
// scratch (nullable): B * OH * OW * cout * 2 floats for the hidden-split form of the late blocks on small maps.
// io: bit 0 = fp16 input x, bit 1 = fp16 output y (the fp16mx schedule; slab-kernel geometries, blocks 1-7, only).
hipError_t launch_x2_irb(int cin, int hid, int cout, int stride, bool expand, bool res, const void* x, const void* we,
                         const float* be, const float* wd, const float* bd, const void* wp, const float* bp, void* y,
                         int B, int H, int W, int OH, int OW, hipStream_t s, float* scratch = nullptr, int io = 0);
// fp16mx blocks 2-4 (k_mx.hip): fp16 input, hi + lo fp16 weights (blob dtype 5 / 6 layout), fp16 hidden slab, fp32
// depthwise, hi + lo project operand; fp16 (out16: blocks 2-3) or fp32 (block 4) output.
bool mx_irb_supported(int cin, int hid, int cout, int stride, bool expand, bool res, bool in16, bool out16);
hipError_t launch_mx_irb(int cin, int hid, int cout, int stride, bool res, bool in16, bool out16, const void* x,
                         const void* we,
                         const float* be, const float* wd, const float* bd, const void* wp, const float* bp, void* y,
                         int B, int H, int W, int OH, int OW, hipStream_t s);
// fp16mx front (k_mx.hip front_mx_kernel): uint8 NHWC -> stem + block 1 -> fp16 [B][OH][OW][16]; wsp = OP_STEM x1.
hipError_t launch_mx_front(const void* x, const void* wsp, const float* bs, const float* wd, const float* bd,
                           const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW,
                           hipStream_t s);
// uint8 NHWC frames -> stem + block 1 -> [B][OH][OW][16] (x2_front_kernel), fp32 or (out16) fp16; wsx: blob OP_STEM
// x0 of dtype 5 / 6.
hipError_t launch_x2_front(const void* x, const void* wsx, const float* bs, const float* wd, const float* bd,
                           const void* wp, const float* bp, void* y, int B, int H, int W, int OH, int OW, hipStream_t s,
                           bool out16 = false);
// 1x1 conv + BN + ReLU on fp32 activations X [M][K] with wt [2][Np][Kp] fp16 (hi, lo) -> fp32 Y [M][N]; Np % 64 == 0.
hipError_t launch_x2_pw_relu(const void* x, const void* wt, const float* bias, float* y, int64_t M, int K, int N,
                             hipStream_t s);
// Same conv fused with URSONetHead's mean over HW (HW % 64 == 0, N % 64 == 0): part = workspace [B * HW / 64][N].
bool x2_pw_pool_supported(int HW, int N);
hipError_t launch_x2_pw_pool(const void* x, const void* wt, const float* bias, float* part, float* pooled, int B,
                             int HW, int K, int N, hipStream_t s);
// URSONetHead mean([2,3]) over an fp32 NHWC map: pooled [B][C].
hipError_t launch_mean_hw(const float* x, float* pooled, int B, int HW, int C, hipStream_t s);

// Split-K fp32 head GEMM for very long K: part = workspace [splits][B][round_up(n,16)] floats.
hipError_t launch_fc_splitk(const float* x, const float* w, const float* bias, float* out, int n, int B, int K,
                            int splits, float* part, hipStream_t s);

// Keypoint decode: sigmoid (optional) + EPnP + dcm2quat per problem (k_epnp.hip). raw: B x 2(n+1) (origin +
// n keypoints, normalised x,y); kp3d: n x 3 fp32 (device); K: host 3x3 row-major. status |= 8 on failure.
// Brown-Conrady lens distortion of the keypoint camera (OpenCV's 5-coefficient order); on = 0: none.
struct EpnpDist {
  double k1, k2, p1, p2, k3;
  int on;
};
// model = control points [4][3] + alphas [n][4] (fp64, device), computed once by spef_set_keypoints.
hipError_t launch_epnp(const float* raw, int B, int n, const float* kp3d, const double* model, const double* K,
                       float nu, float nv, const EpnpDist& dist, int apply_sigmoid, float* kp_out, float* quat,
                       float* pos, int* status, hipStream_t s);

// Activation dtype -> fp32 NHWC copy (debug probes / backbone feature export).
hipError_t launch_to_f32(int dtype, const void* x, float* y, int64_t n, hipStream_t s);

// Decode (src/spe/spe_utils.py:56-101): ori softmax + Markley average; pos softmax + soft-argmax.
// status[b] |= 1 (NaN orientation moments), 2 (pos zero sum), 4 (NaN position).
// The orientation kernels write status[b] (=, not |=) and copy pos_src -> pos when pos_src is not null.
hipError_t launch_decode_ori(const float* logits, int B, int n_bins, const double* q_bins, float* soft,
                             float* quat, int* status, const float* pos_src, float* pos, hipStream_t s);
hipError_t launch_normalize_ori(const float* raw, int B, float* quat, int* status, const float* pos_src, float* pos,
                                hipStream_t s);
hipError_t launch_decode_pos(const float* logits, int B, int n_bins, const double* grid, float* soft,
                             float* pos, int* status, hipStream_t s);

// ---- INT8 path (k_q8.hip; integer semantics of oracle/int8_ref.py) ----
enum QEpi : int { QEPI_RELU = 0, QEPI_PROJ = 1, QEPI_PROJ_RES = 2, QEPI_FC = 3 };

// Input quant + stem (u8 NHWC via `lut`, or f32 NCHW via round(x / s_img)) -> u8 NHWC [B][OH][OW][32].
// w28: int8 [32][28] (k = ky*9+kx*3+ci, k 27 zero); M/B/S: requant [32].
hipError_t launch_q_stem(const void* in, int f32in, const int8_t* lut, float s_img, int in_bits, const int8_t* w28,
                         const int64_t* M, const int64_t* Bq, const int32_t* S, int out_bits, uint8_t* y, int B, int H,
                         int W, int OH, int OW, hipStream_t s);
// Depthwise 3x3: u8 in, int8 [9][C] weights -> ReLU-quant, stored offset (u - 128) int8.
hipError_t launch_q_dw(const uint8_t* x, const int8_t* w9, const int64_t* M, const int64_t* Bq, const int32_t* S,
                       int out_bits, int8_t* y, int B, int H, int W, int C, int stride, int OH, int OW, hipStream_t s);
struct QGemmArgs {
  int epi;
  const int8_t* x;          // [M][K] int8 rows
  const int8_t* w;          // [Np][Kp64] int8
  const int32_t* init;      // [Np] accumulator init (offset correction, FC bias) or null
  const int64_t* rqM;       // requant [Np] (RELU / PROJ / PROJ_RES)
  const int64_t* rqB;
  const int32_t* rqS;
  const int8_t* r;          // PROJ_RES: residual [M][N] int8
  int64_t rm, rb;           // PROJ_RES: residual-join rescale
  int rs;
  void* y;                  // int8/u8 [M][N]; FC: float [M][n_split]
  float* y1;                // FC: float [M][N - n_split]
  const float* sc;          // FC: per-column output scale [Np]
  int n_split;
  int64_t M;
  int K, N;
  int out_bits = 8;         // output quantizer bit width (RELU unsigned, PROJ / PROJ_RES signed; bit_width.json)
};
hipError_t launch_q_gemm(const QGemmArgs& a, hipStream_t s);
// TruncTo8bit average pool over the whole map: u8 [B][HW][C] -> offset int8 [B][C] = ((sum) >> tb) - 128.
hipError_t launch_q_pool(const uint8_t* x, int8_t* p, int B, int HW, int C, int tb, hipStream_t s);
// Fused int8 inverted-residual block (expand blocks 2-17; k_q8irb.hip). tabs = blob OP_QIRB x2.
bool q_irb_supported(int cin, int hid, int cout, int stride, bool res, bool expand);
// Quantizer bit widths (bit_width.json, 2..8): eb / db expand / depthwise ReLU quantizers (unsigned), sb the
// shared signed quantizer the block's output is requantised to.
struct QBits {
  int eb, db, sb;
};
hipError_t launch_q_irb(int cin, int hid, int cout, int stride, bool res, bool expand, bool sh32, const int8_t* x, const int8_t* we,
                        const int8_t* wp, const int32_t* pinit, const uint8_t* tabs, int64_t rm, int64_t rb, int rs,
                        QBits qb, int8_t* y, int B, int H, int W, int OH, int OW, hipStream_t s);
// Role-split form of the same block for MobileNet-V2 blocks 8-17 (k_q8irw.hip; bit-identical, same arguments).
bool q_irw_supported(int cin, int hid, int cout, int stride, bool res);
hipError_t launch_q_irw(int cin, int hid, int cout, int stride, bool res, bool sh32, const int8_t* x, const int8_t* we,
                        const int8_t* wp, const int32_t* pinit, const uint8_t* tabs, int64_t rm, int64_t rb, int rs,
                        QBits qb, int8_t* y, int B, int H, int W, int OH, int OW, hipStream_t s);
// int8 (is_unsigned 0) or u8 codes -> fp32 code * scale.
hipError_t launch_q_to_f32(const void* x, float* y, int64_t n, int is_unsigned, float scale, hipStream_t s);

// ---- input preprocessing (k_pre.hip): Pillow BILINEAR resize with its integer coefficient tables ----
hipError_t launch_resize_h(const uint8_t* in, uint8_t* tmp, const int* bounds, const int* kk, int ksize, int B,
                           int Hin, int Win, int y0, int Ht, int Wo, hipStream_t s);
hipError_t launch_resize_v(const uint8_t* tmp, uint8_t* out, const int* bounds, const int* kk, int ksize, int B,
                           int Ht, int Ho, int Wo, hipStream_t s);

}  // namespace spef
