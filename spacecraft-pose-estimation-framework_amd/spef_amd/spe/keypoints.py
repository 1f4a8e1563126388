"""Host mirror of the reference ``KeyPoints`` (src/spe/keypoints_utils.py:13-174).

Holds the 3-D keypoints and the camera (with its lens distortion, if any) that the MI355X keypoint decode (sigmoid +
undistortPoints + batched EPnP, csrc/k_epnp.hip) is configured with through ``Engine.set_keypoints``. The solve itself is not here: ``pnp`` /
``decode_batch`` run on the GPU via ``SPEMi355x``; this class only loads the model points and builds the
normalised 2-D keypoint vectors (``create_keypoints2d``) used to make targets and synthetic test inputs.
"""
from __future__ import annotations

import numpy as np

from .. import quaternion as Q


class KeyPoints:
    def __init__(self, camera, keypoints_dir=None):
        """``keypoints_dir``: path to a MAT file holding ``tango3Dpoints`` [3 x N] (keypoints_utils.py:30-45), or
        the [N x 3] array itself."""
        assert keypoints_dir is not None
        self.camera = camera
        if isinstance(keypoints_dir, np.ndarray):
            self.keypoints3d = np.asarray(keypoints_dir, np.float32).reshape(-1, 3)
        else:
            self.keypoints3d = self.load_3d_keypoints(keypoints_dir)

    @staticmethod
    def load_3d_keypoints(mat_path: str, name: str = 'tango3Dpoints') -> np.ndarray:
        from scipy.io import loadmat   # MAT v5 reader: parses arrays, executes nothing from the file
        return np.transpose(np.array(loadmat(mat_path)[name], dtype=np.float32))

    def project(self, ori: np.ndarray, pos: np.ndarray) -> np.ndarray:
        """Projection (keypoints_utils.py:47-86): -> [2 x (N+1)] pixels, origin first; the camera's distCoeffs
        (k1, k2, p1, p2, k3), when it has them, add the radial + tangential distortion of :74-80 (SPEED+)."""
        pts = np.concatenate([np.zeros((1, 3)), self.keypoints3d.astype(np.float64)], axis=0)
        xc = pts @ Q.quat2dcm(ori).T + np.asarray(pos, np.float64)
        K = np.asarray(self.camera.K, np.float64)
        x, y = xc[:, 0] / xc[:, 2], xc[:, 1] / xc[:, 2]
        d = getattr(self.camera, 'distCoeffs', None)
        if d is not None:
            d = np.asarray(d, np.float64).reshape(-1)
            r2 = x * x + y * y
            cdist = 1 + d[0] * r2 + d[1] * r2 * r2 + d[4] * r2 * r2 * r2
            x, y = (x * cdist + d[2] * 2 * x * y + d[3] * (r2 + 2 * x * x),
                    y * cdist + d[2] * (r2 + 2 * y * y) + d[3] * 2 * x * y)
        return np.stack([K[0, 0] * x + K[0, 2], K[1, 1] * y + K[1, 2]])

    def create_bbox_from_keypoints(self, keypoints2d: np.ndarray) -> np.ndarray:
        """keypoints_utils.py:176-198: [x_min, y_min, x_max, y_max] of normalised (x0, y0, x1, y1, ...)."""
        x = keypoints2d[::2] * self.camera.nu
        y = keypoints2d[1::2] * self.camera.nv
        return np.array([np.min(x) / self.camera.nu, np.min(y) / self.camera.nv, np.max(x) / self.camera.nu,
                         np.max(y) / self.camera.nv])

    def create_keypoints2d(self, ori: np.ndarray, pos: np.ndarray) -> np.ndarray:
        """keypoints_utils.py:88-110: normalised (x0, y0, x1, y1, ...) float32 vector incl. the frame origin."""
        kp = self.project(ori, pos)
        kp[0] /= self.camera.nu
        kp[1] /= self.camera.nv
        return np.reshape(kp.T, (-1,)).astype(np.float32)
