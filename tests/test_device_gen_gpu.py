"""Device draw generator (csrc/datagen.hip) vs its specification, and 64-bit dataset offsets."""
import numpy as np
import pytest
import torch

from euromillioner_amd.data import device_gen as DG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,seg,planted", [(3 * 256 + 37, 256, 0.9), (1000, 4096, 0.0), (4099, 1024, 1.0)])
def test_kernel_matches_spec(n, seg, planted):
    got = DG.generate_masks(n, seed=7, planted=planted, seg_len=seg).cpu().numpy()
    ref = DG.generate_masks_py(n, seed=7, planted=planted, seg_len=seg)
    assert (got == ref).all()


def test_large_fill_domain_rules():
    n = (1 << 26) + 5
    m = DG.generate_masks(n, seed=3, planted=0.9)
    u = m.view(torch.int64)
    main = torch.zeros_like(u)
    star = torch.zeros_like(u)
    for b in range(50):
        main += (u >> b) & 1
    for b in range(50, 62):
        star += (u >> b) & 1
    assert bool((main == 5).all()) and bool((star == 2).all())
    assert bool(((u >> 62) == 0).all())


def test_train_step_at_64bit_offset():
    """A step over samples beyond 2^31 draws (16 GiB of masks) equals the same samples at offset 0."""
    from euromillioner_amd.models.mlp import FusedSmallMLP
    from euromillioner_amd.ops import fused_mlp as FM

    B = 1 << 16
    off = (1 << 31) + 12345
    big = DG.generate_masks(off + B + 1, seed=9, planted=0.9)
    small = big[off:off + B + 1].clone()
    m = FusedSmallMLP("cuda", lr=1e-3)
    outs = []
    for d, o in ((big, off), (small, 0)):
        m.slabs.zero_()
        n = FM.train_partials(d, B, m.img, m.slabs, m.loss_slabs, loss="softmax", offset=o)
        torch.cuda.synchronize()
        outs.append((m.slabs[:n].clone(), m.loss_slabs[:n].clone()))
    del big
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("first,n", [(1024, 2500), (4096 * 3, 4096 + 17)])
def test_kernel_shard_matches_spec(first, n):
    seg = 1024 if first % 4096 else 4096
    got = DG.generate_masks(n, seed=11, planted=0.9, seg_len=seg, first=first).cpu().numpy()
    ref = DG.generate_masks_py(n, seed=11, planted=0.9, seg_len=seg, first=first)
    assert (got == ref).all()
