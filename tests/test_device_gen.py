"""Segmented synthetic-draw specification (euromillioner_amd/data/device_gen.py) on the CPU."""
import numpy as np

from euromillioner_amd.data import device_gen as DG
from euromillioner_amd.data.synthetic import generate_draws


def _popcounts(m):
    u = m.view(np.uint64)
    main = np.array([bin(int(x) & ((1 << 50) - 1)).count("1") for x in u])
    star = np.array([bin(int(x) >> 50).count("1") for x in u])
    return main, star


def test_spec_domain_rules():
    m = DG.generate_masks_py(1500, seed=3, planted=0.9, seg_len=256)
    main, star = _popcounts(m)
    assert (main == 5).all() and (star == 2).all()
    assert (m.view(np.uint64) >> np.uint64(62) == 0).all()  # bits 62/63 (bias / pad) never set


def test_spec_permutations_match_host_generator():
    _, perm = generate_draws(10, seed=11, planted=0.5, native=False)
    assert (DG.permutations(11) == perm).all()


def test_spec_planted_structure():
    seed, seg = 5, 512
    m = DG.generate_masks_py(2048, seed=seed, planted=0.9, seg_len=seg).view(np.uint64)
    pim = DG.permutations(seed)[:50]
    hits = tot = 0
    for t in range(1, len(m)):
        if t % seg == 0:
            continue  # first draw of a segment is unplanted
        prev = [k for k in range(50) if (int(m[t - 1]) >> k) & 1]
        for k in prev:
            tot += 1
            hits += (int(m[t]) >> (int(pim[k]) - 1)) & 1
    assert hits / tot > 0.85  # 0.9 planted + chance refills
    flat = DG.generate_masks_py(2048, seed=seed, planted=0.0, seg_len=seg).view(np.uint64)
    hits0 = sum((int(flat[t]) >> (int(pim[k]) - 1)) & 1 for t in range(1, 2048) if t % seg
                for k in range(50) if (int(flat[t - 1]) >> k) & 1)
    assert hits0 / tot < 0.2  # chance level 0.1


def test_segments_are_independent_streams():
    a = DG.generate_masks_py(600, seed=1, planted=0.9, seg_len=256)
    b = DG.generate_masks_py(600, seed=1, planted=0.9, seg_len=256)
    assert (a == b).all()
    assert not (a[:256] == a[256:512]).all()
    c = DG.generate_masks_py(600, seed=2, planted=0.9, seg_len=256)
    assert not (a == c).all()


def test_gb_to_draws():
    assert DG.gb_to_draws(1) == (1 << 27)


def test_shard_at_offset_equals_slice_of_whole_sequence():
    """A rank's shard generated at ``first`` is bit-identical to that slice of the whole sequence."""
    whole = DG.generate_masks_py(5 * 256 + 40, seed=4, planted=0.9, seg_len=256)
    for first, n in ((256, 300), (3 * 256, 2 * 256 + 40), (0, 100)):
        part = DG.generate_masks_py(n, seed=4, planted=0.9, seg_len=256, first=first)
        assert (part == whole[first:first + n]).all()
    import pytest

    with pytest.raises(ValueError):
        DG.generate_masks_py(10, seed=4, seg_len=256, first=100)


def test_region_cover():
    first, n, skip = DG.region(1000, 3000, seg_len=256)
    assert first == 768 and skip == 232 and first + skip == 1000 and first + n == 3000
