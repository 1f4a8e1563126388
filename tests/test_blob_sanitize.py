"""The host-side blob validation under AddressSanitizer + UndefinedBehaviorSanitizer: the C ABI's
parse_blob / op_extents compiled with the sanitizers (tools/sanitize_blob.py, a host executable; no GPU), fed the
corrupted blobs of test_blob_validation.py and seeded random mutations of the header and op table of fp16, fp16mx,
fp16x2 and int8 blobs. Every blob must come back OK or ERR_BLOB with no sanitizer report, and with the same return
code as the shipped library gives through ctypes."""
import os
import shutil
import struct
import subprocess
import sys

import numpy as np
import pytest

from spef_amd import _lib as L
from spef_amd import blob as Bl
from spef_amd.arch import mobilenet_v2
from spef_amd.weights import synthetic_state_dict

from test_blob_validation import _validate

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(shutil.which('hipcc') is None and not os.path.exists('/opt/rocm/bin/hipcc'),
                                reason='hipcc needed for the sanitizer build')


@pytest.fixture(scope='module')
def exe():
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    import sanitize_blob
    return sanitize_blob.build()


def _blobs():
    sd = synthetic_state_dict(mobilenet_v2('ursonet', 1728, 3), seed=7)
    out = {d: Bl.pack(sd, dtype=d) for d in ('fp16', 'fp16mx', 'fp16x2')}
    from spef_amd.blob_q8 import pack_int8
    from spef_amd.data.synthetic import synth_frames
    from spef_amd.quant import calibrate
    out['int8'] = pack_int8(sd, calibrate(sd, synth_frames(2, 64, 64, 900)))
    kp = mobilenet_v2('keypoints')
    out['kp_fp16x2'] = Bl.pack(synthetic_state_dict(kp, seed=3), kp, dtype='fp16x2')
    return out


def _corruptions(name, b, rng):
    """The targeted cases of test_blob_validation.py, then random overwrites of header / op-table bytes (values
    biased to the edges: 0, all-ones, 2^31, 2^32 - 16, small) and random truncations."""
    info = Bl.describe(b)
    ops_off, n_ops, data_bytes = info['ops_off'], info['n_ops'], info['data_bytes']
    meta_end = ops_off + n_ops * 128
    cases = [(f'{name}_good', b), (f'{name}_magic', b'X' + b[1:]), (f'{name}_empty', b''), (f'{name}_hdr', b[:60])]
    for cut in (1, 4096, len(b) - 200, len(b) - meta_end + 5):
        cases.append((f'{name}_cut{cut}', b[:-cut]))
    for field, off, fmt, val in (('ops_off', 48, '<Q', 0xFFFFFFFFFFFFFFC0), ('version', 8, '<I', 1),
                                 ('n_out0', 24, '<I', 1232), ('n_ops', 12, '<I', 0xFFFFFFFF)):
        m = bytearray(b)
        struct.pack_into(fmt, m, off, val)
        cases.append((f'{name}_{field}', bytes(m)))
    m = bytearray(b)                                   # the last op's w0 in range but too short (extent check)
    struct.pack_into('<Q', m, ops_off + (n_ops - 1) * 128 + 32, (data_bytes - 1024) // 256 * 256)
    cases.append((f'{name}_extent', bytes(m)))
    edges = [0, 0xFFFFFFFFFFFFFFFF, 1 << 31, (1 << 32) - 16, 1 << 63, 16, 7, 4096]
    for k in range(60):
        m = bytearray(b)
        for _ in range(int(rng.integers(1, 4))):
            pos = int(rng.integers(0, meta_end - 8)) & ~3
            width = int(rng.choice([1, 2, 4, 8]))
            v = int(rng.choice(edges)) if rng.random() < 0.6 else int(rng.integers(0, 1 << 62))
            m[pos:pos + width] = (v & ((1 << (8 * width)) - 1)).to_bytes(width, 'little')
        cut = int(rng.integers(0, len(b))) if rng.random() < 0.2 else len(b)
        cases.append((f'{name}_mut{k}', bytes(m[:cut])))
    return cases


def test_corrupted_blobs_under_asan_ubsan(exe, tmp_path):
    rng = np.random.Generator(np.random.PCG64(2024))
    cases = [c for name, b in _blobs().items() for c in _corruptions(name, b, rng)]
    paths = []
    for name, data in cases:
        p = tmp_path / f'{name}.spef'
        p.write_bytes(data)
        paths.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:abort_on_error=0:halt_on_error=1',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1')
    r = subprocess.run([exe] + paths, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and 'Sanitizer' not in r.stderr and 'runtime error' not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == len(cases)
    n_ok = 0
    for (name, data), line in zip(cases, lines):
        rc = int(line.split()[0])
        assert rc in (L.OK, L.ERR_BLOB), (name, line)
        assert rc == _validate(data)[0] if data else rc == L.ERR_BLOB, (name, line)   # same verdict as the library
        n_ok += rc == L.OK
        if name.endswith('_good'):
            assert rc == L.OK, line
    assert n_ok < len(cases) // 2, 'mutations should mostly be rejected'
    print(f'{len(cases)} blobs under ASan + UBSan: {n_ok} accepted, {len(cases) - n_ok} rejected, no reports')


def test_sanitizer_is_live(exe, tmp_path):
    """The driver's self-test reads one byte past its buffer: an ASan report proves the instrumentation is on."""
    p = tmp_path / 'x.spef'
    p.write_bytes(b'\0' * 64)
    r = subprocess.run([exe, str(p)], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, BLOB_CHECK_SELFTEST='1', ASAN_OPTIONS='detect_leaks=0'))
    assert r.returncode != 0 and 'heap-buffer-overflow' in r.stderr
