import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    """TEST INFRASTRUCTURE: the CPU restatement (oracle/), built on demand."""
    from oracle import oracle as O
    O.build()
    return O


HOSTSIM_SRC = os.path.join(ROOT, "tests", "hostsim", "sim.hip")
HOSTSIM_LIB = os.path.join(ROOT, "tests", "hostsim", "libsim.so")


@pytest.fixture(scope="session")
def hostsim():
    """Host build of the sorted-path per-pixel logic (G == 1), tests only."""
    import ctypes as C
    csrc = os.path.join(ROOT, "siril_amd", "csrc")
    deps = [HOSTSIM_SRC, os.path.join(csrc, "stack_sorted_impl.h"), os.path.join(csrc, "stack_wz.h"),
            os.path.join(csrc, "sgpu_kparams.h")]
    # SGPU_HOSTSIM_DEFINES="SGPU_WZ_KT=20 SGPU_WZ_KM=8": check a tuning variant's
    # algorithm on the host (own library file)
    defs = os.environ.get("SGPU_HOSTSIM_DEFINES", "").split()
    lib = HOSTSIM_LIB if not defs else HOSTSIM_LIB.replace(".so", "_" + "_".join(defs).replace("=", "") + ".so")
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(map(os.path.getmtime, deps)):
        subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O1", "-std=c++17",
                        "-fPIC", "-shared", "-ffp-contract=off", "-I" + csrc] + ["-D" + d for d in defs] +
                       [HOSTSIM_SRC, "-o", lib], check=True)
    S = C.CDLL(lib)
    fp = C.POINTER(C.c_float)
    S.sim_pixel.restype = C.c_int
    S.sim_pixel.argtypes = [C.c_int, fp, C.c_int, C.c_float, C.c_float, fp, C.c_float, C.c_float,
                            C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    S.sim_pixel_u16.restype = C.c_int
    S.sim_pixel_u16.argtypes = S.sim_pixel.argtypes
    S.sim_pixels.restype = None
    S.sim_pixels.argtypes = [C.c_int, fp, C.c_int, C.c_longlong, C.c_float, C.c_float, fp, C.c_float,
                             C.c_float, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_int),
                             C.POINTER(C.c_int)]
    S.sim_wz_stats.argtypes = [C.POINTER(C.c_longlong)]
    S.sim_wz1_pixels.restype = None
    S.sim_wz1_pixels.argtypes = [fp, C.c_int, C.c_longlong, C.c_float, C.c_float, C.POINTER(C.c_double),
                                 C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    S.sim_wz_stats_reset.argtypes = []
    S.sim_set_roundwise.argtypes = [C.c_int]
    S.sim_set_roundwise.restype = None
    return S
