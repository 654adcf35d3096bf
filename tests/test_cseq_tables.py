"""CPU check of k_co_run's transition-table algebra (siddhi_amd/csrc/cseq_own.h: co_tables, co_comp).

The count-sequence automaton's L (length of e1's chain, 0..M) changes per event by one of three
maps: T0 (f1 false: L -> 0), T10 (f1 alone: 0 -> 1, L -> L + 1, M -> 1), T11 (f1 and f2: 0 -> 1,
M -> 1, else 0) -- the rule tests/test_cseq.py pins against the oracle.  k_co_run composes them
as 8-byte tables (byte i = L after, from L = i) with two byte permutes (v_perm_b32), which is exact
only because every map the three generate sends L = 0 and L = M to the same value, so inputs
0..7 suffice for M <= 7 and every output is a valid permute selector.  This restates v_perm_b32's
selection and checks every composition of random runs of maps against direct evaluation, and
that the identity table composes as an identity on both sides.
"""
import numpy as np
import pytest


def perm(s0, s1, sel):
    """v_perm_b32 for selector bytes 0..7: byte k = byte sel_k of the 8 bytes {s0 (high), s1 (low)}."""
    src = (s0 << 32) | s1
    out = 0
    for k in range(4):
        b = (sel >> (8 * k)) & 0xFF
        assert b < 8
        out |= ((src >> (8 * b)) & 0xFF) << (8 * k)
    return out


def comp(g, f):  # g after f
    gl, gh = g & 0xFFFFFFFF, g >> 32
    return (perm(gh, gl, f >> 32) << 32) | perm(gh, gl, f & 0xFFFFFFFF)


def tables(M):
    t10 = t11 = 0
    for i in range(8):
        t10 |= (1 if (i == 0 or i >= M) else i + 1) << (8 * i)
        t11 |= (1 if (i == 0 or i == M) else 0) << (8 * i)
    return t10, t11


def at(f, i):
    return (f >> (8 * i)) & 0xFF


IDENT = 0x0706050403020100


def step(kind, L, M):
    if kind == 0:
        return 0
    if kind == 1:  # T10
        return 1 if L in (0, M) else L + 1
    return 1 if L in (0, M) else 0  # T11


@pytest.mark.parametrize("M", range(1, 8))
def test_composed_tables_equal_direct_evaluation(M):
    rng = np.random.default_rng(M)
    t10, t11 = tables(M)
    gen = {0: 0, 1: t10, 2: t11}
    for _ in range(400):
        kinds = rng.integers(0, 3, rng.integers(1, 12)).tolist()
        f = IDENT
        for k in kinds:
            f = comp(gen[k], f)
        for L0 in range(M + 1):
            L = L0
            for k in kinds:
                L = step(k, L, M)
            assert at(f, L0) == L, (M, kinds, L0)
        assert at(f, 0) == at(f, M)
        assert comp(IDENT, f) == f and comp(f, IDENT) == f


@pytest.mark.parametrize("M", range(1, 8))
def test_segmented_prefix_with_constants(M):
    """A run start makes the prefix a constant (co_const(at(F, L0))): composing later maps after a
    constant stays a constant, the value the direct walk reaches."""
    rng = np.random.default_rng(100 + M)
    t10, t11 = tables(M)
    gen = {0: 0, 1: t10, 2: t11}
    for _ in range(200):
        L0 = int(rng.integers(0, M + 1))
        kinds = rng.integers(0, 3, 10).tolist()
        g = 0x0101010101010101 * at(gen[kinds[0]], L0)
        L = step(kinds[0], L0, M)
        for k in kinds[1:]:
            g = comp(gen[k], g)
            L = step(k, L, M)
            assert g == 0x0101010101010101 * L
