"""Device-side engine: one SPEF context (one GPU) driven through the C ABI.

PyTorch-ROCm is plumbing here: it owns device memory (output tensors) and the current HIP stream;
every computation is a HIP kernel in libspef_mi355x.so.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib as L


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Engine:
    """Loaded weights + workspace on one GPU.

    ``forward`` maps NHWC uint8 frames (or the reference's NCHW float32 [0,1] tensor) to the raw head
    outputs; ``decode`` applies SPEUtils.last_activ + decode on the device.
    """

    def __init__(self, blob: bytes | torch.Tensor | None, device: int | str | torch.device = 0):
        """``blob``: packed weights in host memory (bytes) or on this device (uint8 tensor), or None for an empty
        context that receives its weights with ``bcast_weights``."""
        self.lib = L.load()
        self.device = torch.device(device if not isinstance(device, int) else f'cuda:{device}')
        if self.device.type != 'cuda':
            raise AssertionError('SPEMi355x runs on a HIP device only (no CPU fallback)')
        idx = self.device.index or 0
        h = C.c_void_p()
        L.check(self.lib.spef_init(idx, C.byref(h)))
        self.ctx = h
        self._reserved = (0, 0, 0)
        self._decode_tables = None
        # bumped by every call that moves device buffers or changes what a recorded forward / decode would do
        # (workspace reallocation, weights, decode tables, options, camera): StreamPipeline's recorded HIP graphs key on it
        self.epoch = 0
        self.head = self.n_out0 = self.n_out1 = self.n_ops = None
        self.dtype = None
        if blob is not None:
            self.load(blob)

    # ------------------------------------------------------------------ weights
    def load(self, blob: bytes | torch.Tensor) -> None:
        if isinstance(blob, torch.Tensor):
            assert blob.is_cuda and blob.dtype == torch.uint8 and blob.is_contiguous()
            L.check(self.lib.spef_load_weights_device(self.ctx, C.c_void_p(blob.data_ptr()), blob.numel()))
        else:
            buf = C.create_string_buffer(bytes(blob), len(blob))
            L.check(self.lib.spef_load_weights(self.ctx, buf, len(blob)))
        self._model_info()

    def bcast_weights(self, comm, root: int = 0) -> None:
        """Collective over the RCCL communicator ``comm`` (spef_amd.shard.RcclComm): rank ``root``'s weights are
        broadcast into every rank's context (spef_bcast_weights)."""
        L.check(self.lib.spef_bcast_weights(self.ctx, C.c_void_p(int(comm)), root))
        self._model_info()

    def _model_info(self) -> None:
        head, n0, n1, dt, nops = (C.c_int(), C.c_int(), C.c_int(), C.c_int(), C.c_int())
        L.check(self.lib.spef_model_info(self.ctx, C.byref(head), C.byref(n0), C.byref(n1), C.byref(dt),
                                         C.byref(nops)))
        self.head, self.n_out0, self.n_out1 = head.value, n0.value, n1.value
        self.dtype = {1: 'fp16', 2: 'bf16', 3: 'int8', 4: 'fp32', 5: 'fp16x2', 6: 'fp16mx'}[dt.value]
        self.n_ops = nops.value
        self._reserved = (0, 0, 0)
        self.epoch += 1

    def reserve(self, B: int, H: int, W: int) -> None:
        rb, rh, rw = self._reserved
        if B <= rb and (H, W) == (rh, rw):
            return
        L.check(self.lib.spef_reserve(self.ctx, B, H, W))
        self._reserved = (B, H, W)
        self.epoch += 1

    def set_decode_tables(self, ori_bins: Optional[np.ndarray], pos_grid: Optional[np.ndarray]) -> None:
        ob = None if ori_bins is None else np.ascontiguousarray(ori_bins, np.float64)
        pg = None if pos_grid is None else np.ascontiguousarray(pos_grid, np.float64)
        L.check(self.lib.spef_set_decode_tables(
            self.ctx, None if ob is None else ob.ctypes.data_as(C.c_void_p), 0 if ob is None else ob.shape[0],
            None if pg is None else pg.ctypes.data_as(C.c_void_p), 0 if pg is None else pg.shape[0]))
        self._decode_tables = (ob, pg)
        self.epoch += 1

    # ------------------------------------------------------------------ compute
    @staticmethod
    def _layout(x: torch.Tensor) -> Tuple[int, int, int, int]:
        if x.dtype == torch.uint8:
            assert x.dim() == 4 and x.shape[3] == 3, 'uint8 frames must be B x H x W x 3 (NHWC)'
            return L.IN_U8_NHWC, x.shape[0], x.shape[1], x.shape[2]
        assert x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == 3, 'expected B x 3 x H x W float32'
        return L.IN_F32_NCHW, x.shape[0], x.shape[2], x.shape[3]

    def forward(self, x: torch.Tensor, out0: Optional[torch.Tensor] = None, out1: Optional[torch.Tensor] = None):
        assert x.device == self.device and x.is_contiguous()
        layout, B, H, W = self._layout(x)
        self.reserve(B, H, W)
        if out0 is None:
            out0 = torch.empty((B, self.n_out0), dtype=torch.float32, device=self.device)
        if out1 is None and self.n_out1:
            out1 = torch.empty((B, self.n_out1), dtype=torch.float32, device=self.device)
        L.check(self.lib.spef_forward(self.ctx, _ptr(x), layout, B, H, W, _ptr(out0), _ptr(out1),
                                      _stream(self.device)))
        return out0, out1

    def preprocess(self, frames: torch.Tensor, size, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Decoded frames uint8 [B, Hin, Win, 3] (device) -> uint8 [B, H, W, 3] = Pillow BILINEAR resize
        (transforms.Resize(img_size), speed.py:66-69), ready for ``forward``."""
        assert frames.device == self.device and frames.dtype == torch.uint8 and frames.is_contiguous()
        assert frames.dim() == 4 and frames.shape[3] == 3, 'frames must be B x H x W x 3 uint8'
        B, Hin, Win, _ = frames.shape
        H, W = int(size[0]), int(size[1])
        if out is None:
            out = torch.empty((B, H, W, 3), dtype=torch.uint8, device=self.device)
        L.check(self.lib.spef_preprocess(self.ctx, _ptr(frames), B, Hin, Win, _ptr(out), H, W, _stream(self.device)))
        return out

    def backbone(self, x: torch.Tensor) -> torch.Tensor:
        layout, B, H, W = self._layout(x)
        self.reserve(B, H, W)
        fh, fw = H, W
        for _ in range(5):
            fh, fw = (fh - 1) // 2 + 1, (fw - 1) // 2 + 1
        f = torch.empty((B, fh, fw, 1280), dtype=torch.float32, device=self.device)
        L.check(self.lib.spef_backbone(self.ctx, _ptr(x), layout, B, H, W, _ptr(f), _stream(self.device)))
        return f

    def probe(self, x: torch.Tensor, stop_op: int) -> torch.Tensor:
        layout, B, H, W = self._layout(x)
        self.reserve(B, H, W)
        out = torch.empty(B * H * W * 96 // 4 + 64, dtype=torch.float32, device=self.device)  # >= any act
        c, h, w = C.c_int(), C.c_int(), C.c_int()
        L.check(self.lib.spef_probe(self.ctx, _ptr(x), layout, B, H, W, stop_op, _ptr(out), C.byref(c), C.byref(h),
                                    C.byref(w), _stream(self.device)))
        return out[:B * h.value * w.value * c.value].view(B, h.value, w.value, c.value)

    def decode(self, ori_mode: int, pos_mode: int, ori_raw: torch.Tensor, pos_raw: torch.Tensor,
               want_soft: bool = True):
        B = ori_raw.shape[0]
        dev = self.device
        quat = torch.empty((B, 4), dtype=torch.float32, device=dev)
        pos = torch.empty((B, 3), dtype=torch.float32, device=dev)
        status = torch.empty((B,), dtype=torch.int32, device=dev)
        ori_soft = torch.empty_like(ori_raw) if (want_soft and ori_mode == L.CLASSIFICATION) else None
        pos_soft = torch.empty_like(pos_raw) if (want_soft and pos_mode == L.CLASSIFICATION) else None
        assert ori_raw.dim() == 2 and pos_raw.dim() == 2 and pos_raw.shape[0] == B
        assert ori_raw.is_contiguous() and pos_raw.is_contiguous()
        assert ori_raw.dtype == torch.float32 and pos_raw.dtype == torch.float32
        L.check(self.lib.spef_decode(self.ctx, ori_mode, pos_mode, _ptr(ori_raw), ori_raw.shape[1], _ptr(pos_raw),
                                     pos_raw.shape[1], B, _ptr(ori_soft), _ptr(quat), _ptr(pos_soft), _ptr(pos),
                                     _ptr(status), _stream(dev)))
        return {'ori': quat, 'pos': pos, 'ori_soft': ori_soft, 'pos_soft': pos_soft, 'status': status}

    def set_fused(self, on: bool) -> None:
        """Fused inverted-residual blocks (default) or one kernel per conv (reference schedule)."""
        L.check(self.lib.spef_set_option(self.ctx, L.OPT_FUSE_BLOCKS, 1 if on else 0))

    def set_option(self, option: int, value: int) -> None:
        L.check(self.lib.spef_set_option(self.ctx, option, int(value)))
        self.epoch += 1

    def set_keypoints(self, kp3d: np.ndarray, K: np.ndarray, nu: float, nv: float, dist=None) -> None:
        """Keypoint-mode camera: 3-D model points, K, image size; ``dist`` = the camera's distCoeffs (k1, k2, p1,
        p2[, k3]; SPEED+) or None (SPEED: cv2.solvePnP gets zeros, keypoints_utils.py:136)."""
        kp = np.ascontiguousarray(kp3d, np.float32)
        kk = np.ascontiguousarray(K, np.float64).reshape(9)
        L.check(self.lib.spef_set_keypoints(self.ctx, kp.ctypes.data_as(C.c_void_p), kp.shape[0],
                                            kk.ctypes.data_as(C.c_void_p), float(nu), float(nv)))
        dd = np.zeros(0) if dist is None else np.ascontiguousarray(np.asarray(dist, np.float64).reshape(-1))
        L.check(self.lib.spef_set_keypoint_distortion(self.ctx, dd.ctypes.data_as(C.c_void_p) if dd.size else None,
                                                      int(dd.size)))
        self.epoch += 1
        self._kp = (kp, kk, dd)

    def decode_keypoints(self, raw: torch.Tensor, apply_sigmoid: bool = True):
        B = raw.shape[0]
        dev = self.device
        kp = torch.empty_like(raw)
        quat = torch.empty((B, 4), dtype=torch.float32, device=dev)
        pos = torch.empty((B, 3), dtype=torch.float32, device=dev)
        status = torch.empty((B,), dtype=torch.int32, device=dev)
        L.check(self.lib.spef_decode_keypoints(self.ctx, _ptr(raw), B, 1 if apply_sigmoid else 0, _ptr(kp), _ptr(quat),
                                               _ptr(pos), _ptr(status), _stream(dev)))
        return {'keypoints': kp, 'ori': quat, 'pos': pos, 'status': status}

    # ------------------------------------------------------------------ profiling
    def profile_begin(self) -> None:
        L.check(self.lib.spef_profile_begin(self.ctx))

    def profile_end(self) -> dict:
        """-> {kernel key: (launches, total_ms, algorithmic_bytes, algorithmic_flops)}."""
        import json
        need = C.c_size_t(0)
        buf = C.create_string_buffer(1 << 16)
        L.check(self.lib.spef_profile_end(self.ctx, buf, len(buf), C.byref(need)))
        return {k: tuple(v) for k, v in json.loads(buf.value.decode()).items()}

    def close(self) -> None:
        if getattr(self, 'ctx', None):
            self.lib.spef_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
