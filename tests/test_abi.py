"""The C-ABI library builds for gfx950, loads without a GPU, and exports exactly what include/spef.h declares."""
import os
import re

from spef_amd import _build, _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include', 'spef.h')


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:int|const char\*)\s+(spef_\w+)\s*\(', src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert 'spef_forward' in names and 'spef_decode' in names and len(names) >= 10


def test_library_exports_every_declared_symbol():
    lib = _lib.load(_build.build())
    for name in _declared():
        assert hasattr(lib, name), name


def test_ctypes_signatures_cover_header():
    assert sorted(_lib.SIGNATURES) == _declared()


def test_no_gpu_calls_fail_loudly():
    """Without a GPU, spef_init must return an error code (never a silent CPU path)."""
    import ctypes as C
    import torch
    if torch.cuda.is_available():
        return
    lib = _lib.load()
    h = C.c_void_p()
    rc = lib.spef_init(0, C.byref(h))
    assert rc != 0
