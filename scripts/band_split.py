"""One rank's row band of a stack, stacked as one launch or as K row
sub-chunks on C contexts / streams (the stack side of the pipelined
frame-sharded transpose), on one GPU, no collective.
usage: python scripts/band_split.py CONFIG ROWS K C [STEPS] [LEAD]
(LEAD 1: the pipeline's lead-half split, sub_bands_lead)
prints one JSON line: ms per band for the split and for one launch."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from siril_amd import distributed as D, stacking as S, synth  # noqa: E402

cfg, rows, K, C = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
lead = len(sys.argv) > 6 and sys.argv[6] == "1"
rname, sig, n, w, h, method = bench.CONFIGS[cfg]
dev = torch.device("cuda", 0)
fr = synth.frames_torch(n, rows, w, dev)
args = S.StackingArgs(S.Rejection[rname], sig)
ctxs = [S.Context(0) for _ in range(C)]
main = torch.cuda.current_stream(dev)
streams = [main] + [torch.cuda.Stream(dev) for _ in range(C - 1)]
out = torch.empty((rows, w), dtype=torch.float32, device=dev)
subs = (D.sub_bands_lead if lead else D.sub_bands)((0, rows), K)


def split():
    # the counters are zeroed on the current stream before the other
    # streams wait on it (a counter zeroed after the wait raced the stack)
    cnts = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in subs]
    for st in streams[1:]:
        st.wait_stream(main)
    for k, (b0, b1) in enumerate(subs):
        j = k % C
        ctxs[j].stack_device(fr[:, b0:b1], args, method, out=out[b0:b1], counts=cnts[k], stream=streams[j])
    for st in streams[1:]:
        main.wait_stream(st)
    return sum(c for c in cnts)


def whole():
    c = torch.zeros(2, dtype=torch.int64, device=dev)
    ctxs[0].stack_device(fr, args, method, out=out, counts=c, stream=main)
    return c


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        c = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, c.tolist()


t_whole, c_whole = timeit(whole)
t_split, c_split = timeit(split)
print(json.dumps({"config": cfg, "rows": rows, "subchunks": K, "contexts": C, "lead": lead,
                  "ms_one_launch": round(t_whole, 3),
                  "ms_split": round(t_split, 3), "counts_equal": c_whole == c_split}), flush=True)
for c in ctxs:
    c.close()
