"""Camera intrinsics of the datasets the reference ships (src/data/datasets/speed.py:18-32,
speed_plus.py:18-40). Same class attributes (``K``, ``nu``, ``nv``, ``distCoeffs``) so code written against the
reference's ``Camera`` classes reads them unchanged."""
from __future__ import annotations

import numpy as np


class SpeedCamera:
    fx = 0.0176
    fy = 0.0176
    nu = 1920
    nv = 1200
    ppx = 5.86e-6
    ppy = ppx
    fpx = fx / ppx
    fpy = fy / ppy
    K = np.array([[fpx, 0, nu / 2], [0, fpy, nv / 2], [0, 0, 1]])


class SpeedPlusCamera:
    fx = 0.017513075965995915
    fy = 0.017511673079277208
    nu = 1920
    nv = 1200
    ppx = 5.86e-6
    ppy = ppx
    fpx = fx / ppx
    fpy = fy / ppy
    K = np.array([[fpx, 0, nu / 2], [0, fpy, nv / 2], [0, 0, 1]])
    distCoeffs = [-0.22383016606510672, 0.51409797089106379, -0.00066499611998340662, -0.00021404771667484594,
                  -0.13124227429077406]


CAMERAS = {'speed': SpeedCamera, 'speed_plus': SpeedPlusCamera}
