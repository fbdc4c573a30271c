"""Phase cycles of the one-wave exact kernel on single deferred-like columns
(diagnostic; run with SGPU_LIB=variants/exwprof/libsirilgpu.so, a
-DSGPU_EXW_PROF=1 build whose kernel printf's its phase cycles)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siril_amd import stacking as S, synth  # noqa: E402

ctx = S.Context(0)
ctx.set_exact_only(2)
for n in (100, 400, 1000):
    fr = synth.frames_numpy(n, 1, 1, seed=3)
    for rt in (S.Rejection.SIGMA, S.Rejection.WINSORIZED):
        print(f"-- N={n} {rt.name}", flush=True)
        ctx.stack(fr, S.StackingArgs(rt, (3.0, 3.0)))
        ctx.synchronize() if hasattr(ctx, "synchronize") else None
        sys.stdout.flush()
ctx.close()
