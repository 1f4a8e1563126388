/* spef.h -- C ABI of the SPEF MI355X (gfx950) inference target.
 *
 * This is the drop-in boundary for the reference's duck-typed "SPE model" interface
 *     predict(images NCHW float32 in [0,1]) -> (pose dict, latency_ms)
 * implemented by SPETorch.predict   (src/spe/spe_torch.py:41-76),
 *                SPETVMARM.predict  (src/tvm/spe_tvm.py:45),
 *                SPEJetson.predict  (src/nvidia/spe_nvidia.py:105).
 * The Python class spef_amd.spe_mi355x.SPEMi355x implements that interface on top of these entry points
 * (ctypes); INTEGRATION.md shows the binding a reference maintainer adds.
 *
 * Conventions: every function returns 0 (SPEF_OK) or a positive error code; spef_last_error() returns the
 * calling thread's last message. Tensor pointers are DEVICE pointers unless a parameter says "host".
 * `stream` is a hipStream_t (NULL = default stream). One context per GPU; a context is not thread-safe.
 */
#ifndef SPEF_H_
#define SPEF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPEF_ABI_VERSION 1

enum spef_status {
  SPEF_OK = 0,
  SPEF_ERR_ARG = 1,      /* invalid argument (AssertionError in the reference, spe_torch.py:55)       */
  SPEF_ERR_HIP = 2,      /* HIP runtime error                                                        */
  SPEF_ERR_BLOB = 3,     /* malformed / incompatible weight blob                                      */
  SPEF_ERR_STATE = 4,    /* weights or decode tables not loaded, workspace too small                  */
  SPEF_ERR_NUMERIC = 5   /* NaN / zero-sum in decode (ValueError, classification_utils.py:134,253,262) */
};

/* input layouts of spef_forward */
enum spef_layout {
  SPEF_IN_U8_NHWC = 0,   /* uint8 frames B x H x W x 3 (ToTensor's /255 fused into the stem)          */
  SPEF_IN_F32_NCHW = 1   /* float32 B x 3 x H x W in [0,1]: the reference `images` tensor             */
};

/* decode modes (MODEL.HEAD.ORI / MODEL.HEAD.POS, src/config/train/config.py:19-20) */
enum spef_mode { SPEF_REGRESSION = 0, SPEF_CLASSIFICATION = 1, SPEF_KEYPOINTS = 2 };

typedef struct spef_ctx spef_ctx;

int spef_abi_version(void);
const char* spef_last_error(void);

/* Create a context on HIP device `device` (SPETorch.__init__, spe_torch.py:24-39). */
int spef_init(int device, spef_ctx** out);
/* Release everything (SPETorch.delete_model, spe_torch.py:97-106). */
int spef_destroy(spef_ctx* ctx);

/* Load a packed weight blob (built by build_mi355x.py from parameters.pt, model.py:261-266 layout).
 * _host: blob in host memory; _device: blob already in this device's memory (e.g. after an RCCL
 * broadcast from rank 0) -- copied device-to-device. */
int spef_load_weights(spef_ctx* ctx, const void* host_blob, size_t bytes);
int spef_load_weights_device(spef_ctx* ctx, const void* dev_blob, size_t bytes);
/* Query the loaded model: head (0 URSONet, 1 keypoints), output widths, storage dtype (1 fp16, 2 bf16). */
int spef_model_info(const spef_ctx* ctx, int* head, int* n_out0, int* n_out1, int* dtype, int* n_ops);

/* Allocate activation workspace for batches up to B of H x W frames. Must precede spef_forward for that
 * size (keeps hipMalloc out of the forward so the forward can be stream-captured). */
int spef_reserve(spef_ctx* ctx, int B, int H, int W);

/* ModelWrapper.forward (pytorch_layers.py:29-32): frames -> raw head outputs (fp32).
 * URSONet head: out0 = orientation logits/raw [B x n_out0], out1 = position [B x n_out1].
 * Keypoint head: out0 = keypoint regression [B x 24] (pre-sigmoid), out1 unused (may be NULL). */
int spef_forward(spef_ctx* ctx, const void* input, int layout, int B, int H, int W, float* out0, float* out1,
                 void* stream);

/* Backbone only (MobileNetV2.forward, mobilenet_v2.py:269-271): 1280-channel feature map as fp32 NHWC
 * [B x H/32 x W/32 x 1280] (the C2 feature-MSE check). */
int spef_backbone(spef_ctx* ctx, const void* input, int layout, int B, int H, int W, float* features,
                  void* stream);

/* Debug probe: run the backbone through op `stop_op` (0 = stem, i = inverted-residual block i) and write that
 * activation as fp32 NHWC; *c, *h, *w receive its shape. */
int spef_probe(spef_ctx* ctx, const void* input, int layout, int B, int H, int W, int stop_op, float* out,
               int* c, int* h, int* w, void* stream);

/* Decode constants (host, float64, as built by OrientationSoftClassification.build_histogram,
 * classification_utils.py:39-83, and PositionSoftClassification.build_histogram, :201-215). */
int spef_set_decode_tables(spef_ctx* ctx, const double* ori_bins, int n_ori_bins, const double* pos_grid,
                           int n_pos_bins);

/* SPEUtils.last_activ + SPEUtils.decode (spe_utils.py:56-101) for the URSONet head.
 * ori_mode: SPEF_CLASSIFICATION (softmax -> ori_soft [B x n_ori_bins], Markley average -> quat [B x 4]) or
 *           SPEF_REGRESSION (L2 normalise ori_raw [B x 4] -> quat).
 * pos_mode: SPEF_CLASSIFICATION (softmax -> pos_soft [B x n_pos_bins], soft-argmax -> pos [B x 3]) or
 *           SPEF_REGRESSION (pos = pos_raw copied).
 * status: device int[B], zeroed by this call; bit 1 NaN orientation, 2 position zero sum, 4 NaN position.
 * ori_soft / pos_soft may be NULL. */
int spef_decode(spef_ctx* ctx, int ori_mode, int pos_mode, const float* ori_raw, const float* pos_raw, int B,
                float* ori_soft, float* quat, float* pos_soft, float* pos, int* status, void* stream);

/* Keypoint mode (ORI == POS == 'keypoints', config.py:53-58): the 3-D model points (host float32 n x 3,
 * e.g. tangoPoints.mat's 11 Tango keypoints, keypoints_utils.py:31-45), the camera matrix (host float64
 * 3x3 row-major) and the image size the keypoints are normalised by (Camera nu, nv; speed.py:18-32). */
int spef_set_keypoints(spef_ctx* ctx, const float* kp3d, int n, const double* K, float nu, float nv);

/* SPEUtils.last_activ (sigmoid, spe_utils.py:68) + KeyPoints.decode_batch (keypoints_utils.py:152-174):
 * raw [B x 2(n+1)] (origin + n keypoints) -> optional kp_out (sigmoid values, same shape), quat [B x 4],
 * pos [B x 3] by batched EPnP (cv2.SOLVEPNP_EPNP semantics) + dcm2quat. status bit 8 = EPnP failure. */
int spef_decode_keypoints(spef_ctx* ctx, const float* raw, int B, int apply_sigmoid, float* kp_out, float* quat,
                          float* pos, int* status, void* stream);

/* Input preprocessing on the device (SPEDataset.__getitem__ + transforms.Resize(img_size), utils.py:212-249,
 * speed.py:66-69): decoded frames uint8 [B x Hin x Win x 3] (RGB, HWC) -> uint8 [B x H x W x 3], bit-identical to
 * Pillow's Image.resize((W, H), BILINEAR). The result feeds spef_forward with SPEF_IN_U8_NHWC (ToTensor's /255
 * is fused into the stem). Temporary storage is owned by the context. */
int spef_preprocess(spef_ctx* ctx, const uint8_t* frames, int B, int Hin, int Win, uint8_t* out, int H, int W,
                    void* stream);

/* Options. SPEF_OPT_FUSE_BLOCKS (default 1): run each inverted-residual block as one fused kernel
 * (expand + depthwise + project on-chip) where its geometry is in the fused table; 0 = one kernel per conv. */
/* SPEF_OPT_FUSE_MIN_HW: fuse only blocks whose input has at least this many pixels per image (late,
 * low-resolution blocks then run as GEMM + depthwise + GEMM with the hidden tensor L2/MALL-resident).
 * SPEF_OPT_PW_GEMM (default 1): LDS-tiled MFMA GEMM for unfused 1x1 convs; 0 = register-direct kernel. */
/* SPEF_OPT_IRB_VARIANT: fused-block tile variant (0 = tuned default; others for tuning sweeps).
 * SPEF_OPT_STRIP (default 0, experimental): register-streaming fused blocks for the high-resolution geometries; 0 = LDS-slab
 * fused blocks everywhere.
 * SPEF_OPT_WAVESPEC (default 1): wave-specialised fused blocks for the low-resolution geometries (expand waves
 * and depthwise/project waves pipelined over hidden chunks); 0 = LDS-slab fused blocks. */
enum spef_option {
  SPEF_OPT_FUSE_BLOCKS = 1,
  SPEF_OPT_FUSE_MIN_HW = 2,
  SPEF_OPT_PW_GEMM = 3,
  SPEF_OPT_IRB_VARIANT = 4,
  SPEF_OPT_STRIP = 5,
  SPEF_OPT_WAVESPEC = 6
};
int spef_set_option(spef_ctx* ctx, int option, int value);

/* Per-launch HIP-event profiling of every kernel the context enqueues between begin and end (bench.py's
 * roofline leg). spef_profile_end synchronises, then writes a JSON object
 *   {"<kernel key>": [launches, total_ms, algorithmic_bytes, algorithmic_flops], ...}
 * into buf (host, cap bytes); *needed receives the size required including the terminating NUL. */
int spef_profile_begin(spef_ctx* ctx);
int spef_profile_end(spef_ctx* ctx, char* buf, size_t cap, size_t* needed);

#ifdef __cplusplus
}
#endif
#endif /* SPEF_H_ */
