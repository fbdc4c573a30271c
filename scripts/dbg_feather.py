"""Debug: GPU feather masks vs the oracle on one small frame (prints both)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import feather_ref as F
from siril_amd import feather as Fe
import torch
sys.path.insert(0, "tests")
from test_feather import _feather_frames
np.set_printoptions(linewidth=250, precision=3)
rng = np.random.default_rng(10 + 97 + 123 + 0)
fr = _feather_frames(rng, 3, 97, 123, False)
got = Fe.compute_masks(torch.from_numpy(fr).cuda()).cpu().numpy()
want = F.downscale_blend_mask(fr[0])
print("got\n", got[0]); print("want\n", want)
m8 = np.where(fr[0] != 0, 255, 0).astype(np.uint8)
m8 = F._morph(F._morph(m8, np.maximum, 0), np.minimum, 255)
print("resized u8\n", F.resize_linear_u8(m8, 12, 9))
# all-zero frame and all-white
for v in (0.0, 0.5):
    z = np.full((1, 97, 123), v, np.float32)
    g = Fe.compute_masks(torch.from_numpy(z).cuda()).cpu().numpy()[0]
    print("const", v, "got\n", g, "\nwant\n", F.downscale_blend_mask(z[0]))
