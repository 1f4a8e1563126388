"""ctypes binding of the C ABI in include/spef.h (libspef_mi355x.so, built in-tree by _build.py).

There is no CPU fallback: if the library is missing or fails to load, importing the product path raises.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _build

OK, ERR_ARG, ERR_HIP, ERR_BLOB, ERR_STATE, ERR_NUMERIC, ERR_COMM = range(7)
IN_U8_NHWC, IN_F32_NCHW = 0, 1
REGRESSION, CLASSIFICATION, KEYPOINTS = 0, 1, 2
ABI_VERSION = 3
COMM_ID_BYTES = 128
OPT_FUSE_BLOCKS, OPT_WAVESPEC, OPT_Q8_ROLESPLIT = 1, 6, 7     # public schedule options (include/spef.h)
OPT_FUSE_MIN_HW, OPT_PW_GEMM, OPT_IRB_VARIANT, OPT_TEST_FAIL_BCAST = 2, 3, 4, 5   # internal (csrc/spef_tuning.hpp)
OPT_MX_KERNELS = 8   # internal: fp16mx blocks 2-7 on k_mx.hip (1) or the fp16x2 slab kernels (0)

# name -> (restype, argtypes); keep in sync with include/spef.h (tests/test_abi.py checks the header)
_vp, _i, _sz = C.c_void_p, C.c_int, C.c_size_t
_ip = C.POINTER(C.c_int)
SIGNATURES = {
    'spef_abi_version': (_i, []),
    'spef_last_error': (C.c_char_p, []),
    'spef_init': (_i, [_i, C.POINTER(_vp)]),
    'spef_destroy': (_i, [_vp]),
    'spef_load_weights': (_i, [_vp, _vp, _sz]),
    'spef_load_weights_device': (_i, [_vp, _vp, _sz]),
    'spef_model_info': (_i, [_vp, _ip, _ip, _ip, _ip, _ip]),
    'spef_reserve': (_i, [_vp, _i, _i, _i]),
    'spef_preprocess': (_i, [_vp, _vp, _i, _i, _i, _vp, _i, _i, _vp]),
    'spef_forward': (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp]),
    'spef_backbone': (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    'spef_probe': (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _ip, _ip, _ip, _vp]),
    'spef_set_decode_tables': (_i, [_vp, _vp, _i, _vp, _i]),
    'spef_decode': (_i, [_vp, _i, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    'spef_validate_blob': (_i, [_vp, _sz, _ip, _ip, _ip, _ip]),
    'spef_comm_unique_id': (_i, [_vp, _sz]),
    'spef_comm_init': (_i, [_i, _i, _i, _vp, _i, C.POINTER(_vp)]),
    'spef_comm_abort': (_i, [_vp]),
    'spef_comm_destroy': (_i, [_vp]),
    'spef_bcast_weights': (_i, [_vp, _vp, _i]),
    'spef_set_option': (_i, [_vp, _i, _i]),
    'spef_set_keypoints': (_i, [_vp, _vp, _i, _vp, C.c_float, C.c_float]),
    'spef_set_keypoint_distortion': (_i, [_vp, _vp, _i]),
    'spef_decode_keypoints': (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    'spef_profile_begin': (_i, [_vp]),
    'spef_profile_end': (_i, [_vp, C.c_char_p, _sz, C.POINTER(_sz)]),
    'spef_measure_peaks': (_i, [_i, _i, C.POINTER(C.c_double)]),
    'spef_clock_stamp': (_i, [_vp, _i, _vp]),
}


class SpefError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f'[spef error {code}] {msg}')
        self.code = code


_LIB = None


def load(path: str | None = None) -> C.CDLL:
    """Load (once) and return the HIP library; raises if it is absent -- never falls back."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # torch first: its bundled libamdhip64 (SONAME libamdhip64.so.7) then satisfies this library's dependency, so
    # the process holds ONE HIP runtime. Loaded the other way round, torch's libraries pull in their own copy next
    # to /opt/rocm's (they name the unversioned file) and the two runtimes' teardown double-frees at exit.
    import torch  # noqa: F401
    override = path or os.environ.get('SPEF_LIB')    # SPEF_LIB: A/B timing of two builds (tools/ab.py)
    path = override or _build.lib_path()
    if not os.path.exists(path):
        raise ImportError(f'SPEF HIP library not built: {path} (run __graft_entry__.build() or '
                          f'python -m spef_amd._build)')
    if not override:   # the in-tree library must have been linked from exactly the sources beside it
        info = _build.read_info()
        if info.get('source_digest') != _build.source_digest():
            raise ImportError(f'SPEF HIP library {path} is stale or has no BUILD_INFO.json: it was not built from '
                              f'the current csrc/ + include/ (run __graft_entry__.build())')
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.spef_abi_version() != ABI_VERSION:
        raise ImportError('SPEF ABI version mismatch')
    _LIB = lib
    return lib


def check(rc: int) -> None:
    if rc != OK:
        msg = _LIB.spef_last_error().decode(errors='replace') if _LIB else ''
        if rc == ERR_NUMERIC:
            raise ValueError(msg)
        if rc == ERR_ARG:
            raise AssertionError(msg)
        raise SpefError(rc, msg)
