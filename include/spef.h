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

#define SPEF_ABI_VERSION 3
#define SPEF_COMM_ID_BYTES 128   /* size of the RCCL unique id (ncclUniqueId) */

enum spef_status {
  SPEF_OK = 0,
  SPEF_ERR_ARG = 1,      /* invalid argument (AssertionError in the reference, spe_torch.py:55)       */
  SPEF_ERR_HIP = 2,      /* HIP runtime error                                                        */
  SPEF_ERR_BLOB = 3,     /* malformed / incompatible weight blob                                      */
  SPEF_ERR_STATE = 4,    /* weights or decode tables not loaded, workspace too small                  */
  SPEF_ERR_NUMERIC = 5,  /* NaN / zero-sum in decode (ValueError, classification_utils.py:134,253,262) */
  SPEF_ERR_COMM = 6      /* RCCL error or timeout: the communicator was aborted (ncclCommAbort)       */
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
 * _host: blob in host memory; _device: blob already in this device's memory -- copied device-to-device.
 * The blob is validated in full first (spef_validate_blob); on any failure the context keeps the model it had
 * (or stays empty), so a failed reload never leaves a half-loaded context. */
int spef_load_weights(spef_ctx* ctx, const void* host_blob, size_t bytes);
int spef_load_weights_device(spef_ctx* ctx, const void* dev_blob, size_t bytes);
/* Query the loaded model: head (0 URSONet, 1 keypoints), output widths, storage dtype (1 fp16, 2 bf16, 3 int8,
 * 4 fp32 = the reference's own arithmetic: exact-fp32 MFMA, one kernel per conv; 5 fp16x2 = fp32 activations with
 * hi + lo fp16 MFMA operands, the fp32-accurate fused schedule; 6 fp16mx = the fp16x2 weights and kernels with the
 * stem map, the block outputs of blocks 1-3 and the hidden tensors of blocks 2-4 stored fp16: the headline schedule,
 * within 1e-3 of float32 at trained head scales). */
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
 * classification_utils.py:39-83, and PositionSoftClassification.build_histogram, :201-215). At most 8192
 * orientation bins (SPEF_ERR_ARG above; the default 12^3 grid has 1728, 1232 with unused bins deleted). */
int spef_set_decode_tables(spef_ctx* ctx, const double* ori_bins, int n_ori_bins, const double* pos_grid,
                           int n_pos_bins);

/* SPEUtils.last_activ + SPEUtils.decode (spe_utils.py:56-101) for the URSONet head.
 * ori_mode: SPEF_CLASSIFICATION (softmax -> ori_soft [B x n_ori], Markley average -> quat [B x 4]) or
 *           SPEF_REGRESSION (L2 normalise ori_raw [B x 4] -> quat, spe_utils.py:72).
 * pos_mode: SPEF_CLASSIFICATION (softmax -> pos_soft [B x n_pos], soft-argmax -> pos [B x 3]) or
 *           SPEF_REGRESSION (pos = pos_raw copied).
 * n_ori / n_pos: the row widths of ori_raw / pos_raw (the shapes NumPy carries in the reference). They must equal
 *           the decode tables' bin counts in classification mode (spef_set_decode_tables) and 4 / 3 in regression
 *           mode, else SPEF_ERR_ARG -- the kernels never read rows of a width the tables do not describe.
 * status: device int[B], zeroed by this call; bit 1 NaN orientation, 2 position zero sum, 4 NaN position.
 * ori_soft / pos_soft may be NULL. */
int spef_decode(spef_ctx* ctx, int ori_mode, int pos_mode, const float* ori_raw, int n_ori, const float* pos_raw,
                int n_pos, int B, float* ori_soft, float* quat, float* pos_soft, float* pos, int* status, void* stream);

/* Keypoint mode (ORI == POS == 'keypoints', config.py:53-58): the 3-D model points (host float32 n x 3,
 * e.g. tangoPoints.mat's 11 Tango keypoints, keypoints_utils.py:31-45), the camera matrix (host float64
 * 3x3 row-major) and the image size the keypoints are normalised by (Camera nu, nv; speed.py:18-32). */
int spef_set_keypoints(spef_ctx* ctx, const float* kp3d, int n, const double* K, float nu, float nv);

/* Lens distortion of the keypoint camera, OpenCV order (k1, k2, p1, p2[, k3]); n = 0 removes it. The keypoint
 * decode then undistorts the 2-D points as cv2.solvePnP does before EPnP (undistortPoints, 5 iterations) -- the
 * reference passes camera.distCoeffs (keypoints_utils.py:136-142; SPEED+ camera, speed_plus.py:18-40). */
int spef_set_keypoint_distortion(spef_ctx* ctx, const double* dist, int n);

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

/* Schedule options (both choices of each are bit-identical; the parity tests switch them):
 * SPEF_OPT_FUSE_BLOCKS (default 1): each inverted-residual block as one fused kernel (expand + depthwise + project
 *   on-chip); 0 = one kernel per conv (the reference's module-by-module schedule).
 * SPEF_OPT_WAVESPEC (default 2): role-split fused kernels for the low-resolution blocks. 2 = three-stage pipeline
 *   (MFMA waves expand + project, VALU waves depthwise); 1 = two-stage (expand waves, depthwise + project waves);
 *   0 = LDS-slab fused kernels everywhere.
 * SPEF_OPT_Q8_ROLESPLIT (default 0): int8 blobs run blocks 8-17 as role-split kernels (expand waves vs depthwise +
 *   project waves) instead of the LDS-slab kernels: faster with one batch in flight, slower when several batches
 *   share the GPU (the role-split workgroups hold a CU's LDS; DESIGN.md section 3, INT8 path).
 * (Kernel-tuning knobs used by the sweep tools are internal: csrc/spef_tuning.hpp.) */
enum spef_option {
  SPEF_OPT_FUSE_BLOCKS = 1,
  SPEF_OPT_WAVESPEC = 6,
  SPEF_OPT_Q8_ROLESPLIT = 7
};
int spef_set_option(spef_ctx* ctx, int option, int value);

/* Host-only validation of a weight blob (no device needed: build tools and CPU tests use it). Checks the header,
 * the op table, every tensor's extent against the data section (from the op geometry) and the head widths;
 * returns SPEF_ERR_BLOB with a message on the first problem. Outputs may be NULL. */
int spef_validate_blob(const void* host_blob, size_t bytes, int* dtype, int* head, int* n_out0, int* n_out1);

/* Weight broadcast over RCCL (xGMI) -- SURVEY.md §8b/§8e: rank `root` sends the blob its context holds, every
 * other rank's context receives and loads it (header, op table and data section, device to device; no host
 * round trip). Collective: every rank of `comm` calls it with the same root. Replaces each rank reading
 * parameters.pt itself (modeling/model.py:261-266).
 * Failure handling (the reference's analogue is the socket timeouts of spe_nvidia.py:82-103):
 *  - the ranks agree (all-reduce MAX of a status word) after the header broadcast and again after the receivers
 *    have staged the blob; no rank enters a data collective unless all are ready, no receiver commits the new
 *    model unless all staged it, and every rank returns the same status, naming the failing rank;
 *  - every wait is bounded by the communicator's timeout; an RCCL error or a timeout aborts the communicator
 *    (ncclCommAbort) and returns SPEF_ERR_COMM -- the handle is then dead (spef_comm_destroy only forgets it).
 * On any failure a receiving context keeps the model it had.
 * `comm` is an RCCL communicator (ncclComm_t): one made with spef_comm_init (nonblocking, ncclConfig_t.blocking
 * = 0, bounded by `timeout_ms`; <= 0 = 120 s) from an id that rank 0 drew with spef_comm_unique_id and the host
 * shipped to the other ranks (any side channel: torch.distributed, MPI, a file), or the host's own (120 s).
 * spef_comm_abort aborts a communicator from the host (e.g. when the launcher learns a peer died). */
int spef_comm_unique_id(void* id_out, size_t cap);
int spef_comm_init(int device, int nranks, int rank, const void* id, int timeout_ms, void** comm_out);
int spef_comm_abort(void* comm);
int spef_comm_destroy(void* comm);
int spef_bcast_weights(spef_ctx* ctx, void* comm, int root);

/* Per-launch HIP-event profiling of every kernel the context enqueues between begin and end (bench.py's
 * roofline leg). spef_profile_end synchronises, then writes a JSON object
 *   {"<kernel key>": [launches, total_ms, algorithmic_bytes, algorithmic_flops], ...}
 * into buf (host, cap bytes); *needed receives the size required including the terminating NUL. */
int spef_profile_begin(spef_ctx* ctx);
int spef_profile_end(spef_ctx* ctx, char* buf, size_t cap, size_t* needed);

/* On-box measurement (bench.py; SURVEY.md §8d "peaks re-measured by the build's own microbenchmark"), no model
 * involved. spef_measure_peaks runs, on `device`, `reps` timed launches (after one warm-up) of each of: a dense
 * v_mfma_f32_16x16x32_f16 loop, a v_mfma_i32_16x16x64_i8 loop (random operands, 8 independent chains per wave,
 * 4 waves per SIMD), a 4 GiB HBM copy and a 4 GiB HBM read, and writes the best rates: out[0] fp16 TFLOP/s,
 * out[1] int8 TOP/s, out[2] copy GB/s (read + write bytes), out[3] read GB/s, out[4] / out[5] the shader clock in
 * MHz held inside the fp16 / int8 loop (median over workgroups of delta s_memtime / delta s_memrealtime x 100),
 * out[6] / out[7] the stream configuration behind out[2] / out[3] (workgroups per CU x 100 + 16-B loads in flight
 * per thread x 10 + 1 if nontemporal): `out` holds 8 doubles. The calling thread's current device is restored.
 * spef_clock_stamp enqueues n_wg one-wave workgroups on `stream`, each writing (location, s_memtime,
 * s_memrealtime) as three uint64 into the device buffer `out` -- location = XCD id << 8 | HW_ID[15:8] (CU, SH,
 * SE): two stamps around a timed region give the clock held during it (deltas within one CU). */
int spef_measure_peaks(int device, int reps, double* out);
int spef_clock_stamp(void* out, int n_wg, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SPEF_H_ */
