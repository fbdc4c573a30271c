"""Build libsirilgpu.so in-tree (hipcc, gfx950).

Compiles every .hip/.cpp under siril_amd/csrc in parallel into build/obj and
links siril_amd/libsirilgpu.so.  Objects are rebuilt when their source or any
header in csrc/ or include/ is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import time

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(PKG, "libsirilgpu.so")
ARCH = os.environ.get("SGPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: the reference is built for x86-64 without FMA; fused
# multiply-adds would change f32/f64 rounding.
#
# -pragma-unroll-threshold: the register-resident column kernels rely on
# every `#pragma unroll` loop being fully unrolled (all slot indices compile-
# time constants).  At the default threshold the bitonic networks of the
# larger columns (NP >= 512) stay partly rolled and the column arrays fall
# back to scratch memory (measured at N=400: 2 KB/lane, 50x slower).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
         "-mllvm", "-pragma-unroll-threshold=1000000",
         "-Wall", "-Wno-unused-function", "-I" + CSRC, "-I" + os.path.join(ROOT, "include")]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers_mtime():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src: str, hdr_mtime: float, extra=(), obj_dir: str = OBJ) -> str:
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    if os.path.exists(obj):
        om = os.path.getmtime(obj)
        if om >= os.path.getmtime(src) and om >= hdr_mtime:
            return obj
    cmd = [HIPCC] + FLAGS + list(extra) + ["-c", src, "-o", obj]
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
    # hipcc compiles the device and the host side of a file in separate
    # passes: a header edited between them leaves kernel stubs whose device
    # code is missing ("Cannot find Symbol" at launch).  An object whose
    # inputs changed while it compiled is dropped, so the next build redoes it.
    if max(os.path.getmtime(src), _headers_mtime()) >= t0:
        os.remove(obj)
        raise RuntimeError(f"{src} or a header changed while it compiled: run the build again")
    return obj


def build(verbose: bool = True, jobs: int | None = None, defines=(), lib: str = LIB,
          obj_dir: str = OBJ) -> str:
    """defines: extra -D tuning knobs (variant builds go to their own obj_dir/lib)."""
    os.makedirs(obj_dir, exist_ok=True)
    srcs = _sources()
    hm = _headers_mtime()
    jobs = jobs or min(8, os.cpu_count() or 4)
    extra = ["-D" + d for d in defines]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm, extra, obj_dir), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(lib) or os.path.getmtime(lib) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    if verbose:
        print(f"[siril_amd] built {lib}", file=sys.stderr)
    return lib


def build_variant(name: str, defines) -> str:
    """Tuning variant: variants/<name>/libsirilgpu.so (select with SGPU_LIB)."""
    d = os.path.join(ROOT, "variants", name)
    os.makedirs(d, exist_ok=True)
    return build(defines=defines, lib=os.path.join(d, "libsirilgpu.so"),
                 obj_dir=os.path.join(ROOT, "build", "variants", name))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        build_variant(sys.argv[2], sys.argv[3:])
    else:
        build()
