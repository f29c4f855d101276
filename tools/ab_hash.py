#!/usr/bin/env python3
"""Parameter fingerprint of a few fused-MLP training steps (1M-sample batches) under the native
library named by EUROM_NATIVE_LIB: side builds that should be bit-identical to the shipped kernel
print the same hash.  One JSON line."""
from __future__ import annotations

import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from euromillioner_amd.data.device_gen import generate_masks
    from euromillioner_amd.models.mlp import FusedSmallMLP

    B = 1 << 20
    draws = generate_masks(4 * B + 16, seed=11, planted=0.9)
    m = FusedSmallMLP("cuda", lr=1e-3, seed=3)
    for i in range(6):
        loss = m.step(draws, B, offset=(i % 4) * B)
    torch.cuda.synchronize()
    h = hashlib.sha256(m.params.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.path.basename(os.environ.get("EUROM_NATIVE_LIB", "shipped")), "params_sha16": h,
                      "loss": float(loss.item())}))


if __name__ == "__main__":
    main()
