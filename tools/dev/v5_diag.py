"""Dev diagnostic: fused-kernel loss/gradient parts for the selected kernel version (EM_FUSED_V5)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from euromillioner_amd.data.draws import DrawSet  # noqa: E402
from euromillioner_amd.models.mlp import FusedSmallMLP  # noqa: E402
from euromillioner_amd.ops import fused_mlp as FM  # noqa: E402

ds = DrawSet.synthetic(n=6000, seed=11, planted=0.6, calendar=False)
draws = FM.rows_to_masks(torch.from_numpy(ds.numbers).cuda())
out = {}
for loss in ("softmax", "bce"):
    for B, off in ((4096, 0), (37, 100), (256, 0), (32, 0)):
        m = FusedSmallMLP(loss=loss, seed=5)
        lk, g = m.grads(draws, B, offset=off)
        out[f"{loss}_{B}_{off}"] = np.concatenate([[lk], g.cpu().numpy()])
np.savez(sys.argv[1], **out)
