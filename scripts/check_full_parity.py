"""Full-frame consistency check on the GPU box (diagnostic, not a test):
(1) frames_torch is deterministic; (2) the sorted fast path and the exact
sequential kernel (the literal reference algorithm) agree on every pixel of
the BASELINE config-2 stack, bit for bit, including the rejection counts."""
import sys
import time

import torch

sys.path.insert(0, ".")
from siril_amd import stacking as S, synth  # noqa: E402

dev = torch.device("cuda", 0)
n, h, w = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (100, 4000, 6000)))
rname = sys.argv[4] if len(sys.argv) > 4 else "WINSORIZED"
fr = synth.frames_torch(n, h, w, dev)
fr2 = synth.frames_torch(n, h, w, dev)
print("frames deterministic:", bool(torch.equal(fr, fr2)), flush=True)
del fr2
ctx = S.Context(0)
args = S.StackingArgs(S.Rejection[rname], (3.0, 3.0))
out_fast = torch.empty((h, w), dtype=torch.float32, device=dev)
out_exact = torch.empty_like(out_fast)
c_fast = torch.zeros(2, dtype=torch.int64, device=dev)
c_exact = torch.zeros(2, dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream(dev)
ctx.stack_device(fr, args, 0, out=out_fast, counts=c_fast, stream=stream)
torch.cuda.synchronize()
print("fast counts", c_fast.tolist(), "exact pixels", ctx.last_exact_pixels(), flush=True)
ctx.set_exact_only(True)
t0 = time.time()
ctx.stack_device(fr, args, 0, out=out_exact, counts=c_exact, stream=stream)
torch.cuda.synchronize()
print("exact counts", c_exact.tolist(), "time %.1fs" % (time.time() - t0), flush=True)
diff = (out_fast.view(torch.int32) != out_exact.view(torch.int32))
nd = int(diff.sum())
print("pixels differing:", nd, flush=True)
if nd:
    idx = diff.flatten().nonzero()[:10].flatten().tolist()
    for i in idx:
        print(i, float(out_fast.flatten()[i]), float(out_exact.flatten()[i]))
