"""GPU check of the frame-sharded transpose at full size (world-1 RCCL):
is the band that arrives equal to the frames that were sent?  Runs the plain
transpose (both modes) and the pipelined stack, and compares the rejection
totals with the row-band stack of the same frames.
usage: python scripts/fs_check.py N H W"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siril_amd import distributed as D, stacking as S, synth  # noqa: E402

n, h, w = (int(x) for x in sys.argv[1:4])
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
dev = torch.device("cuda", 0)
fr = synth.frames_torch(n, h, w, dev)
torch.cuda.synchronize()
args = S.StackingArgs(S.Rejection.SIGMA, (3.0, 3.0))
ctx = S.Context(0)
_, _, _, c_ref = ctx.stack_device(fr, args)
print("row-band counts", c_ref.tolist(), flush=True)
for mode in ("all_to_all", "p2p"):
    band = D.transpose_frames_to_bands(fr, n, mode=mode)
    torch.cuda.synchronize()
    eq = all(torch.equal(band[f], fr[f]) for f in range(n))
    bad = [f for f in range(n) if not torch.equal(band[f], fr[f])][:8]
    print(mode, "band == frames:", eq, "first bad frames", bad, flush=True)
    _, _, _, c = ctx.stack_device(band, args)
    print(mode, "counts", c.tolist(), flush=True)
    del band
    torch.cuda.empty_cache()
for k in (1, 4):
    full, rej = D.stack_frame_sharded_pipelined(fr, n, args, 0, ctx=ctx, subchunks=k)
    print("pipelined", k, "counts", rej, flush=True)
# raw all_to_all_single of growing sizes
for e in (2**30, 2**31 - 1024, 2**31 + 1024, 3 * 2**30):
    if e > fr.numel():
        break
    src = fr.view(-1)[:e]
    dst = torch.empty_like(src)
    dist.all_to_all_single(dst, src, [e], [e])
    torch.cuda.synchronize()
    print("a2a elements", e, "equal", torch.equal(dst, src), flush=True)
    del dst
ctx.close()
dist.destroy_process_group()
