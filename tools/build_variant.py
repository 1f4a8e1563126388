"""Build an A/B variant of the HIP library with extra compile flags (development tool, not product code):
    python tools/build_variant.py <name> [-DFOO=1 ...]   ->   abx2/<name>.so
Objects go to build/var_<name>/ (content-keyed like spef_amd._build); the GPU-box scripts load a variant with
SPEF_LIB=abx2/<name>.so (spef_amd._lib.load skips the in-tree digest check for an explicit override)."""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd'))
from spef_amd import _build as B  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    odir = os.path.join(ROOT, 'spacecraft-pose-estimation-framework_amd', 'build', f'var_{name}')
    os.makedirs(odir, exist_ok=True)
    os.makedirs(os.path.join(ROOT, 'abx2'), exist_ok=True)
    hdr = hashlib.sha256(''.join(B._file_sha(h) for h in B._headers()).encode()).hexdigest()

    def comp(src):
        flags = B._flags(src) + extra
        key = hashlib.sha256((B._file_sha(src) + hdr + ' '.join(flags)).encode()).hexdigest()[:24]
        obj = os.path.join(odir, f'{os.path.basename(src)}.{key}.o')
        if not os.path.exists(obj):
            r = subprocess.run([B.HIPCC] + flags + ['-x', 'hip', '-c', src, '-o', obj], capture_output=True, text=True)
            if r.returncode:
                raise RuntimeError(r.stderr[-4000:])
        return obj
    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, B._sources()))
    out = os.path.join(ROOT, 'abx2', f'{name}.so')
    r = subprocess.run([B.HIPCC, f'--offload-arch={B.ARCH}', '-shared', '-fPIC'] + objs + B.LDFLAGS + ['-o', out],
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    print(out)


if __name__ == '__main__':
    main()
