"""CPU checks of the LDS bank-conflict model (tools/lds_conflicts.py) for the fused kernels' layouts:
every modelled per-tile access of v4 and the v6 epilogue's fold image must be conflict-free."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import lds_conflicts as M  # noqa: E402


def test_v6_fold_image_conflict_free():
    c, m = M.v6_epilogue()
    assert c == m, (c, m)


def test_v6_fold_without_swizzle_conflicts():
    # the model must see the 16-way conflict the swizzle removes (guards the model itself)
    c, m = M.v6_epilogue(lambda T, g, L, h: (T * 4 + g) * 64 + h * 32 + L)
    assert c >= 4 * m, (c, m)


def test_v4_image_patterns_conflict_free():
    L = list(M.lanes())
    for rho in (0, 1):
        hb = 8192 + 4096 * rho
        for kind, addr in (
            ("write_b64", [hb + M.swz_v4g(r, 4 * h) for _, r, h, *_ in L]),
            ("read_b64", [hb + M.swz_v4g(r, 4 * h) for _, r, h, *_ in L]),
            ("read_tr", [hb + M.swz_v4g(4 * h + q4, 16 * g1 + 4 * p4) for _, r, h, q4, p4, g1 in L]),
            ("read_b128", [M.w2q_off(32 * 2 * rho + r, 2 + h, swz=False) for _, r, h, *_ in L]),
        ):
            c, m = M.cycles(kind, addr)
            assert c == m, (rho, kind, c, m)


def test_v6_b16_backward_reads_conflict_free():
    # every read of the 16x16x32 backward wave (W2Q fragments, dZ2 A rows, H / dZ2 / X transposes)
    for name, kind, addr in M.v6_b16_patterns():
        c, m = M.cycles(kind, addr)
        assert c == m, (name, c, m)


def test_v6_b16_w2q_needs_swizzle():
    # without csrc/mlp_adam.h w2q_swz the W2Q fragment reads take twice their conflict-free cycles
    c = sum(M.cycles(k, a)[0] for n, k, a in M.v6_b16_patterns(swz=False) if n.startswith("W2Q"))
    m = sum(M.cycles(k, a)[1] for n, k, a in M.v6_b16_patterns(swz=False) if n.startswith("W2Q"))
    assert c == 2 * m, (c, m)
