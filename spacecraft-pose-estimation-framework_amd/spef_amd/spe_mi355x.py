"""``SPEMi355x`` -- the MI355X inference target behind the reference's "SPE model" interface.

Drop-in for ``SPETorch`` (src/spe/spe_torch.py:12-124), ``SPETVMARM`` (src/tvm/spe_tvm.py:12) and
``SPEJetson`` (src/nvidia/spe_nvidia.py:53): same ``predict(images) -> (pose, latency_ms)`` contract, same
pose-dict keys, same exception types, so ``tools/evaluation.py:71`` and the ``deploy_*`` throughput loops
(``num_predict``, deploy_nvidia.py:93) call it unchanged.

Differences from SPETorch, all deliberate:
  * forward AND decode run on the GPU (HIP kernels); the reference decodes on the host in NumPy
    (spe_torch.py:73-74, classification_utils.py:163-164);
  * latency is measured with HIP events after a device sync (the reference's ``time.time()`` around an
    un-synchronised forward times only the launch, spe_torch.py:57-61);
  * ``num_predict`` > 1 repeats the device work and reports the mean, like SPEJetson's server loop
    (jetson_inference_server.py:129-141).
"""
from __future__ import annotations

import gc
from typing import Dict, Tuple, Union

import numpy as np
import torch

from . import _lib as L
from .engine import Engine

_MODES = {'regression': L.REGRESSION, 'classification': L.CLASSIFICATION, 'keypoints': L.KEYPOINTS}


class SPEMi355x:
    """Args:
        model: a weight blob (bytes, from build_mi355x.py / ``spef_amd.blob.pack``), a path to one, or an
            already-loaded ``Engine``.
        device: HIP device (``cuda:N``).
        spe_utils: the reference ``SPEUtils`` (or ``spef_amd.spe.spe_utils.SPEUtils``): provides ori/pos mode
            and the decode histograms.
    """

    def __init__(self, model: Union[bytes, str, Engine], device: Union[str, torch.device], spe_utils) -> None:
        self.spe_utils = spe_utils
        self.device = torch.device(device)
        self.engine = None
        self.update_model(model, self.device)

    # ------------------------------------------------------------------ lifecycle (spe_torch.py:78-124)
    def update_model(self, model, device) -> None:
        if self.engine is not None:
            self.delete_model()
        self.device = torch.device(device)
        if isinstance(model, Engine):
            self.engine = model
        else:
            if isinstance(model, str):
                with open(model, 'rb') as f:
                    model = f.read()
            self.engine = Engine(model, self.device)
        su = self.spe_utils
        self.ori_mode, self.pos_mode = _MODES[su.ori_mode], _MODES[su.pos_mode]
        self.keypoint_mode = self.ori_mode == L.KEYPOINTS and self.pos_mode == L.KEYPOINTS
        if (self.ori_mode == L.KEYPOINTS) != (self.pos_mode == L.KEYPOINTS):
            raise ValueError('keypoints mode must be used for both orientation and position')  # spe_utils.py:66
        if self.keypoint_mode:
            kp = su.keypoints
            if kp is None:
                raise ValueError('keypoints mode needs SPEUtils.keypoints (a KeyPoints with keypoints3d)')
            cam = kp.camera
            self.engine.set_keypoints(np.asarray(kp.keypoints3d, np.float32), np.asarray(cam.K, np.float64),
                                      float(cam.nu), float(cam.nv), getattr(cam, 'distCoeffs', None))
            if self.engine.n_out0 != 2 * (kp.keypoints3d.shape[0] + 1):   # model.py:236
                raise AssertionError(f'keypoint head width {self.engine.n_out0} != 2 * (n_keypoints + 1)')
            return
        ori_bins = su.orientation.histogram if self.ori_mode == L.CLASSIFICATION else None
        pos_grid = su.position.histogram if self.pos_mode == L.CLASSIFICATION else None
        self.engine.set_decode_tables(ori_bins, pos_grid)
        # the head widths in the blob must agree with the decode configuration (model.py:225-234)
        want0 = su.orientation.n_bins if self.ori_mode == L.CLASSIFICATION else 4
        want1 = su.position.n_bins if self.pos_mode == L.CLASSIFICATION else 3
        # (raised, not asserted: python -O must not drop it; spef_decode re-checks the widths in C as well)
        if (self.engine.n_out0, self.engine.n_out1) != (want0, want1):
            raise AssertionError(f'model head {(self.engine.n_out0, self.engine.n_out1)} != decode config '
                                 f'{(want0, want1)}')

    def delete_model(self) -> None:
        if self.engine is not None:
            self.engine.close()
        self.engine = None
        gc.collect()

    def close(self) -> None:
        self.delete_model()

    # ------------------------------------------------------------------ inference
    def _run(self, x: torch.Tensor):
        raw0, raw1 = self.engine.forward(x)
        if self.keypoint_mode:   # sigmoid + batched EPnP on the GPU (spe_utils.py:66-68, keypoints_utils.py:152)
            return raw0, None, self.engine.decode_keypoints(raw0, apply_sigmoid=True)
        return raw0, raw1, self.engine.decode(self.ori_mode, self.pos_mode, raw0, raw1)

    def predict_frames(self, frames: torch.Tensor, img_size, num_predict: int = 1) -> Tuple[Dict, float]:
        """Raw decoded camera frames (uint8 [B, Hin, Win, 3], e.g. 1200 x 1920 SPEED images converted to RGB)
        -> the pose dict: the DataLoader's ``Resize(img_size)`` + ``ToTensor`` (speed.py:66-69, utils.py:212-249)
        run on the GPU (bit-identical to Pillow's BILINEAR resize), then ``predict``. Latency covers both."""
        x = frames.to(self.device, non_blocking=True).contiguous()
        torch.cuda.synchronize(self.device)
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(max(1, num_predict)):
            small = self.engine.preprocess(x, img_size)
            raw0, raw1, dec = self._run(small)
        end.record()
        end.synchronize()
        return self._pose(dec), start.elapsed_time(end) / max(1, num_predict)

    def predict(self, images: torch.Tensor, num_predict: int = 1) -> Tuple[Dict, float]:
        """images: NCHW float32 in [0,1] (the reference ``images['torch']``) or NHWC uint8 frames."""
        if self.engine is None:
            raise AssertionError('no model loaded')            # spe_torch.py:55 (assert hasattr(self, 'model'))
        x = images.to(self.device, non_blocking=True).contiguous()
        torch.cuda.synchronize(self.device)
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        start.record()
        for _ in range(max(1, num_predict)):
            raw0, raw1, dec = self._run(x)
        end.record()
        end.synchronize()
        latency_ms = start.elapsed_time(end) / max(1, num_predict)
        return self._pose(dec), latency_ms

    def _pose(self, dec) -> Dict:
        status = dec['status'].cpu().numpy()
        if np.any(status & 1):
            raise ValueError('Error during orientation decoding')                       # classification_utils.py:135
        if np.any(status & 2):
            raise ValueError('Encoded position vector sum is zero, cannot decode.')     # :254
        if np.any(status & 4):
            raise ValueError('Error during position decoding, NaN found in decoded position.')  # :263
        if np.any(status & 8):
            raise ValueError('EPnP failed on a batch row (degenerate keypoints)')   # cv2.solvePnP error analogue

        if self.keypoint_mode:
            return {'keypoints': dec['keypoints'].cpu().numpy(), 'ori': dec['ori'].cpu().numpy(),
                    'pos': dec['pos'].cpu().numpy()}

        pose = {'ori': dec['ori'].cpu().numpy(), 'pos': dec['pos'].cpu().numpy()}
        if self.ori_mode == L.CLASSIFICATION:
            pose['ori_soft'] = dec['ori_soft'].cpu().numpy()
        if self.pos_mode == L.CLASSIFICATION:
            pose['pos_soft'] = dec['pos_soft'].cpu().numpy()
        return pose
