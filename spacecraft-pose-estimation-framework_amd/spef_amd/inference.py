"""The reference's ``Inference`` engine (src/temporal/inference.py:19-191) with an MI355X slot: ``'gpu_mi355x'``.

``select_inference_engine`` (inference.py:46-80) asserts one of the reference's four device names and builds a
``SPETorch`` / Jetson engine; here the same class accepts ``'gpu_mi355x'`` and builds ``SPEMi355x`` (the drop-in
for ``SPETorch.predict``), so the GUI and the temporal tools (``TemporalPDF.update_pdf``, pdf_compare.py:94) run
on the new target. The reference's own devices can be served through ``engine_factories`` (device name ->
``factory(model, spe_utils)`` returning an object with ``predict``), e.g. the reference ``SPETorch`` for
'gpu_host' / 'cpu_host'; without a factory they raise, since those targets are the reference's, not this one's.

``predict`` keeps the reference's post-processing exactly: batch squeeze, quaternion pole continuity against the
previous still frame (:136-144), keypoints / bounding box for visualisation (:146-155), and the optional
'Adaptative' video filter (:158-190) -- whose filtered PDFs are decoded on the GPU (``Engine.decode`` on
``log(pdf)``: its softmax returns the PDF).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib as L
from .engine import Engine
from .spe_mi355x import SPEMi355x
from .temporal import TemporalPDF

REFERENCE_DEVICES = ('gpu_host', 'cpu_host', 'gpu_jetson', 'cpu_ultra96')   # inference.py:47
DEVICES = REFERENCE_DEVICES + ('gpu_mi355x',)


def model_to_blob(model, dtype: str = 'fp16'):
    """What ``SPEMi355x`` accepts: a packed blob (bytes / path / Engine) passes through; a torch ``nn.Module``
    (the reference's ``ModelWrapper``) or a reference-layout state_dict is BN-folded and packed (spef_amd.blob)."""
    if isinstance(model, (bytes, bytearray, str, Engine)):
        return model
    from . import blob
    sd = model.state_dict() if hasattr(model, 'state_dict') else model
    sd = {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in sd.items()}
    return blob.pack(sd, dtype=dtype)


class Inference:
    def __init__(self, model, inference_device: str, spe_utils, device: str = 'cuda:0', dtype: str = 'fp16',
                 engine_factories: Optional[Dict[str, Callable]] = None):
        """Same arguments as the reference (inference.py:20-44); ``device`` / ``dtype`` select the MI355X GPU
        and the blob precision when ``model`` still has to be packed."""
        self.model = model
        self.inference_device = inference_device
        self.spe_utils = spe_utils
        self.inference_engine = None
        self.prev_still_ori = None
        self.prev_video_ori = None
        self.pdf_adapt_ori = TemporalPDF(n=0.8, alpha=16.49, distance_metric='l2')    # inference.py:38-39
        self.pdf_adapt_pos = TemporalPDF(n=0.5, alpha=48.64, distance_metric='l2')
        self.img_size = None
        self.device = device
        self.dtype = dtype
        self.engine_factories = dict(engine_factories or {})
        self.select_inference_engine(self.inference_device)

    def select_inference_engine(self, device: str, model_name: str = None) -> None:
        assert device in DEVICES
        self.close()
        self.inference_device = device
        if device == 'gpu_mi355x':
            self.inference_engine = SPEMi355x(model_to_blob(self.model, self.dtype), self.device, self.spe_utils)
        elif device in self.engine_factories:
            self.inference_engine = self.engine_factories[device](self.model, self.spe_utils)
        else:
            raise ValueError(f"inference device '{device}' is one of the reference's own targets: pass its engine "
                             f"through engine_factories, or use 'gpu_mi355x'")

    def close(self) -> None:
        if self.inference_engine is not None and hasattr(self.inference_engine, 'close'):
            self.inference_engine.close()
        self.inference_engine = None

    def reset(self) -> None:
        """inference.py:93-101."""
        self.prev_still_ori = None
        self.prev_video_ori = None
        self.pdf_adapt_ori.reset()
        self.pdf_adapt_pos.reset()

    def update(self, model, spe_utils) -> None:
        """inference.py:103-115."""
        self.model = model
        self.spe_utils = spe_utils
        self.select_inference_engine(self.inference_device)
        self.reset()

    # ------------------------------------------------------------------ per frame
    def _visual(self, pose: dict) -> None:
        """Keypoints / bounding box for visualisation (inference.py:146-155)."""
        su = self.spe_utils
        if su.keypoints is None:
            return
        if su.ori_mode == 'keypoints' and su.pos_mode == 'keypoints':
            pose['bbox'] = su.keypoints.create_bbox_from_keypoints(pose['keypoints'])
        elif su.pos_mode in ('classification', 'regression') and su.ori_mode in ('classification', 'regression'):
            pose['keypoints'] = su.keypoints.create_keypoints2d(pose['ori'], pose['pos'])
            pose['bbox'] = su.keypoints.create_bbox_from_keypoints(pose['keypoints'])

    def _decode_pdfs(self, ori_pdf: np.ndarray, pos_pdf: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """orientation.decode / position.decode of one filtered PDF pair (inference.py:167-168), on the GPU: the
        decode kernels' softmax of log(pdf) is the PDF itself."""
        eng = self.inference_engine.engine
        dev = eng.device
        with np.errstate(divide='ignore'):
            lo = torch.from_numpy(np.log(ori_pdf.astype(np.float32))[None].copy()).to(dev)
            lp = torch.from_numpy(np.log(pos_pdf.astype(np.float32))[None].copy()).to(dev)
        dec = eng.decode(L.CLASSIFICATION, L.CLASSIFICATION, lo, lp)
        st = dec['status'].cpu().numpy()
        if st.any():
            raise ValueError('Weighted PDF contains NaN or sums to zero')   # classification_utils.py:134-135, 253
        return dec['ori'][0].cpu().numpy(), dec['pos'][0].cpu().numpy()

    def predict(self, image: torch.Tensor, video_type: str = None) -> Tuple[dict, float, Optional[dict]]:
        """inference.py:117-191: -> (pose of the still frame, latency ms, filtered video pose or None)."""
        if not self.img_size or self.img_size != tuple(image.size()):
            self.img_size = tuple(image.size())
        pose_still, latency_ms = self.inference_engine.predict(image)
        pose_still = {k: v.squeeze(0) for k, v in pose_still.items()}
        if self.prev_still_ori is not None:   # no quaternion sign flips between frames
            dot = np.dot(self.prev_still_ori, pose_still['ori'])
            if dot < 0:
                pose_still['ori'] = -pose_still['ori']
            if np.abs(dot) > 0.5:            # an outlier does not move the pole
                self.prev_still_ori = pose_still['ori']
        else:
            self.prev_still_ori = pose_still['ori']
        self._visual(pose_still)

        pose_video = None
        if video_type is not None:
            if video_type != 'Adaptative':
                raise ValueError(f'type of video filtering not implemented: {video_type}')
            assert self.spe_utils.ori_mode == 'classification'
            assert self.spe_utils.pos_mode == 'classification'
            pose_video = {}
            pose_video['ori_soft'], pose_video['ori_distance'] = self.pdf_adapt_ori.update_pdf(pose_still['ori_soft'])
            pose_video['pos_soft'], pose_video['pos_distance'] = self.pdf_adapt_pos.update_pdf(pose_still['pos_soft'])
            pose_video['ori'], pose_video['pos'] = self._decode_pdfs(pose_video['ori_soft'], pose_video['pos_soft'])
            if self.prev_video_ori is not None:
                dot = np.dot(self.prev_video_ori, pose_video['ori'])
                if dot < 0:
                    pose_video['ori'] = -pose_video['ori']
                if np.abs(dot) > 0.5:
                    self.prev_video_ori = pose_video['ori']
            else:
                self.prev_video_ori = pose_video['ori']
            self._visual(pose_video)
        return pose_still, latency_ms, pose_video
