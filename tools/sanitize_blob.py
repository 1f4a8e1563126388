"""AddressSanitizer + UndefinedBehaviorSanitizer build of the host-side blob validation:
    python tools/sanitize_blob.py            ->  spacecraft-pose-estimation-framework_amd/build/asan/blob_check

spef_api.cpp (the C ABI: parse_blob, op_extents, spef_validate_blob) is compiled with the sanitizers on the host side
only (``-Xarch_host -fsanitize=...``; device code is untouched and never runs: there is no GPU in the build container),
linked with the library's other objects as built by spef_amd._build and the driver tools/sanitize/blob_check.cpp into
an executable, so the sanitizer runtime is linked in rather than preloaded. tests/test_blob_sanitize.py feeds it the
corrupted blobs of tests/test_blob_validation.py plus seeded random mutations of the header and op table.
Development / test tool: not part of the shipped library."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'))
from spef_amd import _build as B  # noqa: E402

SAN = ['-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fsanitize=undefined',
       '-Xarch_host', '-fno-sanitize-recover=all', '-Xarch_host', '-fno-omit-frame-pointer', '-g']
OUT_DIR = os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd', 'build', 'asan')
EXE = os.path.join(OUT_DIR, 'blob_check')


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(' '.join(cmd) + '\n' + r.stderr[-4000:])


def build() -> str:
    B.build()                                    # the library's objects (content-keyed, usually up to date)
    os.makedirs(OUT_DIR, exist_ok=True)
    api = os.path.join(B.CSRC, 'spef_api.cpp')
    drv = os.path.join(ROOT, 'tools', 'sanitize', 'blob_check.cpp')
    hdr = ''.join(B._file_sha(h) for h in B._headers())
    key = hashlib.sha256((B._file_sha(api) + B._file_sha(drv) + hdr + ' '.join(SAN)).encode()).hexdigest()[:16]
    stamp = EXE + '.key'
    if os.path.exists(EXE) and os.path.exists(stamp) and open(stamp).read() == key:
        return EXE
    api_o = os.path.join(OUT_DIR, 'spef_api.asan.o')
    drv_o = os.path.join(OUT_DIR, 'blob_check.o')
    _run([B.HIPCC] + B._flags(api) + SAN + ['-x', 'hip', '-c', api, '-o', api_o])
    _run([B.HIPCC] + SAN + ['-O1', '-std=c++17', f'-I{B.INCLUDE}', '-c', drv, '-o', drv_o])
    others = [os.path.join(B.OBJDIR, o) for o in B.read_info()['objects'] if not o.startswith('spef_api.cpp.')]
    _run([B.HIPCC, f'--offload-arch={B.ARCH}', '-Xarch_host', '-fsanitize=address', '-Xarch_host',
          '-fsanitize=undefined', drv_o, api_o] + others + B.LDFLAGS + ['-o', EXE])
    with open(stamp, 'w') as f:
        f.write(key)
    return EXE


if __name__ == '__main__':
    print(build())
