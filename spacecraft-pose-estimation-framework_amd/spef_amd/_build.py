"""Build driver for the in-tree HIP library ``spef_amd/lib/libspef_mi355x.so`` (gfx950 only).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build container; the built .so
travels to the GPU box with the repository snapshot. Objects are rebuilt only when a source or header
is newer than the object.
"""
from __future__ import annotations

import glob
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
NO_NAN_SOURCES = {'k_irb.hip', 'k_irs.hip', 'k_irw.hip', 'k_front.hip', 'k_conv.hip', 'k_gemm.hip', 'k_pool.hip'}
# The SLP vectorizer packs the depthwise FMAs into v_pk_fma_f32 with explicit fp16->fp32 converts (in the fused
# block kernels as soon as their outputs are converted pairwise); scalar v_fma_mix_f32 (fp16 operands read in place)
# is fewer instructions, and every fp32 VALU op costs the same 4 cycles (profiles/r01_valu_rate.txt).
NO_SLP_SOURCES = {'k_irs.hip', 'k_irb.hip', 'k_irw.hip', 'k_front.hip'}


def lib_path() -> str:
    return os.path.join(LIBDIR, LIBNAME)


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')) + glob.glob(os.path.join(CSRC, '*.cpp')))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, '*.hpp')) + glob.glob(os.path.join(INCLUDE, '*.h')))


def _compile(src: str, verbose: bool) -> str:
    base = os.path.basename(src)
    extra = (['-fno-honor-nans'] if base in NO_NAN_SOURCES else []) + (['-fno-slp-vectorize'] if base in NO_SLP_SOURCES else [])
    obj = os.path.join(OBJDIR, base + ('.nn' if extra else '') + '.o')
    newest_dep = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest_dep:
        return obj
    cmd = [HIPCC] + CXXFLAGS + extra + ['-x', 'hip', '-c', src, '-o', obj]
    if verbose:
        print(' '.join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed on {src}:\n{r.stdout}\n{r.stderr}')
    return obj


def build(verbose: bool = False, jobs: int = 8) -> str:
    """Compile every HIP source for gfx950 and link the shared library; returns its path."""
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), _sources()))
    out = lib_path()
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC'] + objs + ['-o', out]
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f'link failed:\n{r.stdout}\n{r.stderr}')
    return out


if __name__ == '__main__':
    print(build(verbose='-v' in sys.argv))
