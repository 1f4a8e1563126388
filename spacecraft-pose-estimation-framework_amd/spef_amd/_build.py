"""Build driver for the in-tree HIP library ``spef_amd/lib/libspef_mi355x.so`` (gfx950 only).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container; the built .so
travels to the GPU box with the repository snapshot. Rebuilds are content-addressed, not mtime-based: every
object is keyed by the SHA-256 of its source, all headers and its compile flags, and ``lib/BUILD_INFO.json``
records the digest of the whole source set the library was linked from. ``_lib.load()`` refuses a library
whose recorded digest differs from the sources beside it (a stale .so fails loudly instead of running old
kernels).
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                       # spacecraft-pose-estimation-framework_amd/
CSRC = os.path.join(ROOT, 'csrc')
INCLUDE = os.path.join(os.path.dirname(ROOT), 'include')
LIBDIR = os.path.join(PKG, 'lib')
OBJDIR = os.path.join(ROOT, 'build', 'obj')
LIBNAME = 'libspef_mi355x.so'
ARCH = 'gfx950'
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
# -amdgpu-mfma-vgpr-form: MFMA results go straight to VGPRs (gfx950's register file is unified) instead of AGPRs
# that every epilogue then copies back with v_accvgpr_read -- fewer VALU ops and fewer registers per wave.
CXXFLAGS = ['-O3', '-fPIC', '-std=c++17', f'--offload-arch={ARCH}', '-Wall', '-Wno-unused-function',
            '-munsafe-fp-atomics', '-mllvm', '-amdgpu-mfma-vgpr-form', f'-I{INCLUDE}', f'-I{CSRC}']


# Convolution kernels never see NaN (finite frames, finite folded weights): dropping NaN semantics lets the
# compiler emit a single v_max_f32 per ReLU instead of canonicalize + max (~18 % fewer VALU ops in the fused
# block loop). Decode / EPnP keep IEEE NaN semantics (they detect NaNs, classification_utils.py:134).
NO_NAN_SOURCES = {'k_irb.hip', 'k_irw.hip', 'k_irp.hip', 'k_front.hip', 'k_conv.hip', 'k_gemm.hip', 'k_pool.hip',
                  'k_x2.hip', 'k_mx.hip'}
# The SLP vectorizer packs the depthwise FMAs into v_pk_fma_f32 with explicit fp16->fp32 converts (in the fused
# block kernels as soon as their outputs are converted pairwise); scalar v_fma_mix_f32 (fp16 operands read in place)
# is fewer instructions, and every fp32 VALU op costs the same 4 cycles (profiles/r01_valu_rate.txt).
NO_SLP_SOURCES = {'k_irb.hip', 'k_irw.hip', 'k_irp.hip', 'k_front.hip', 'k_mx.hip'}


def lib_path() -> str:
    return os.path.join(LIBDIR, LIBNAME)


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')) + glob.glob(os.path.join(CSRC, '*.cpp')))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, '*.hpp')) + glob.glob(os.path.join(INCLUDE, '*.h')))


LDFLAGS = ['-L/opt/rocm/lib', '-lrccl', '-Wl,-rpath,/opt/rocm/lib']   # RCCL: spef_bcast_weights


def _file_sha(path: str) -> str:
    with open(path, 'rb') as f:
        return hashlib.sha256(f.read()).hexdigest()


def _flags(src: str):
    base = os.path.basename(src)
    return CXXFLAGS + (['-fno-honor-nans'] if base in NO_NAN_SOURCES else []) + \
        (['-fno-slp-vectorize'] if base in NO_SLP_SOURCES else [])


def source_digest() -> str:
    """SHA-256 over every source and header (path + content) and the compile / link flags."""
    top = os.path.dirname(ROOT)
    h = hashlib.sha256()
    for p in _sources() + _headers():
        h.update(os.path.relpath(p, top).encode())
        h.update(_file_sha(p).encode())
        h.update(' '.join(_flags(p)).replace(top, '<repo>').encode())   # -I paths: location-independent
    h.update(' '.join(LDFLAGS).encode())
    return h.hexdigest()


def info_path() -> str:
    return os.path.join(LIBDIR, 'BUILD_INFO.json')


def read_info() -> dict:
    try:
        with open(info_path()) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _compile(src: str, verbose: bool, hdr_sha: str) -> tuple:
    """-> (object path, whether it was (re)compiled)."""
    base = os.path.basename(src)
    flags = _flags(src)
    key = hashlib.sha256((_file_sha(src) + hdr_sha + ' '.join(flags)).encode()).hexdigest()[:24]
    obj = os.path.join(OBJDIR, f'{base}.{key}.o')
    if os.path.exists(obj):
        return obj, False
    cmd = [HIPCC] + flags + ['-x', 'hip', '-c', src, '-o', obj + '.tmp']
    if verbose:
        print(' '.join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed on {src}:\n{r.stdout}\n{r.stderr}')
    os.replace(obj + '.tmp', obj)
    for old in glob.glob(os.path.join(OBJDIR, base + '.*.o')):   # drop objects of older versions of this source
        if old != obj:
            os.remove(old)
    return obj, True


def build(verbose: bool = False, jobs: int = 8, force: bool = False) -> str:
    """Compile every HIP source for gfx950 and link the shared library; returns its path. ``force`` recompiles
    every object and relinks."""
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    if force:
        for o in glob.glob(os.path.join(OBJDIR, '*.o')):
            os.remove(o)
    hdr_sha = hashlib.sha256(''.join(_file_sha(h) for h in _headers()).encode()).hexdigest()
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        res = list(ex.map(lambda s: _compile(s, verbose, hdr_sha), _sources()))
    objs = [o for o, _ in res]
    out = lib_path()
    digest = source_digest()
    if force or any(c for _, c in res) or not os.path.exists(out) or read_info().get('source_digest') != digest:
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC'] + objs + LDFLAGS + ['-o', out + '.tmp']
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
        os.replace(out + '.tmp', out)
        ver = subprocess.run([HIPCC, '--version'], capture_output=True, text=True).stdout.strip().splitlines()
        with open(info_path(), 'w') as f:
            json.dump({'source_digest': digest, 'lib_sha256': _file_sha(out), 'arch': ARCH,
                       'hipcc': ver[0] if ver else '', 'objects': [os.path.basename(o) for o in objs]}, f, indent=1)
    return out


if __name__ == '__main__':
    print(build(verbose='-v' in sys.argv, force='--force' in sys.argv))
