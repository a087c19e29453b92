"""Signed 32-bit headroom of the transforms that run without reductions (fhe_amd/csrc/bootstrap.hip,
FHE_FWD_TIGHT and the QM classes of K1w), checked for the modulus of every parameter row whose kernel
runs them.

A signed Montgomery product is below |y| |w| 2^-32 + Q/2 with |w| < Q, so a Cooley-Tukey stage takes a bound
B on its inputs to B (1 + Q/2^32) + Q/2.  From signed digits (|d| <= 2^(g-1)) the kernels run:
  - K1 LMKCDEY / AP with 2^27 <= Q < 2^28 (FM 2): ten stages, no reduction;
  - K1 / K1s / K1m with Q < 2^27: ten stages, no reduction;
  - K1w QM 0 / QM 3 (Q < 2^27) and QM 1 (2^27 <= Q < 2^28): eleven stages, no reduction;
  - K1w QM 2 (2^28 <= Q < 2^29): five stages, a reduction (float: < 0.51 Q; signed Montgomery by 2^32 mod Q:
    < B Q/2^32 + Q/2), four stages, a reduction, two stages.
Every intermediate bound must stay below 2^31, and the inverse plans' limits (16 Q / 8 Q / 4 Q) too.
CPU-only: the moduli come from the host parameter table, the kernel choice from Params.kernel."""
from fractions import Fraction

from fhe_amd import binfhe as bf

TWO31 = 1 << 31


def stages(b0, Q, k):
    """bounds after each of k Cooley-Tukey stages from an input bound b0 (exact)"""
    out, b = [], Fraction(b0)
    for _ in range(k):
        b = b * (1 + Fraction(Q, 1 << 32)) + Fraction(Q, 2)
        out.append(b)
    return out


def rows():
    for ps in range(64):
        for m in (bf.GINX, bf.AP, bf.LMKCDEY):
            try:
                p = bf.params(ps, m)
            except Exception:  # noqa: BLE001 -- not a row of the table
                continue
            yield ps, m, p


def test_rows_exist():
    kinds = {p.kernel for _, _, p in rows()}
    assert {1, 2, 4} <= kinds


def test_forward_transforms_stay_in_signed_words():
    checked = 0
    for ps, m, p in rows():
        Q, g = p.Q, (p.baseG.bit_length() - 1)
        d0 = 1 << (g - 1)
        if p.kernel in (1, 2) and p.N == 1024 and Q < (1 << 28):
            if p.kernel == 1 and m == bf.GINX and Q >= (1 << 27):
                continue  # K1 GINX at 2^27 <= Q: the unsigned lazy form, reduced at its transpose
            assert max(stages(d0, Q, 10)) < TWO31, (ps, m)
            checked += 1
        elif p.kernel == 4:
            if Q < (1 << 28):  # QM 0 / QM 3 / QM 1
                assert max(stages(d0, Q, 11)) < TWO31, (ps, m)
            else:  # QM 2: reductions after five and nine stages; the worse of the two reduction forms
                assert Q < (1 << 29)
                s1 = stages(d0, Q, 5)
                r1 = max(Fraction(51, 100) * Q, s1[-1] * Fraction(Q, 1 << 32) + Fraction(Q, 2))
                s2 = stages(r1, Q, 4)
                r2 = max(Fraction(51, 100) * Q, s2[-1] * Fraction(Q, 1 << 32) + Fraction(Q, 2))
                s3 = stages(r2, Q, 2)
                assert max(s1 + s2 + s3) < TWO31, (ps, m)
                assert s3[-1] < 3 * Q, (ps, m)  # the MAC bounds' digit assumption (kW2Bound / kL2AccBound)
            checked += 1
    assert checked >= 20


def test_lmkcdey_accumulator_bound_at_28_bits():
    """K1 LMKCDEY / AP at 2^27 <= Q < 2^28 without the forward reduction: four digits < B10 times keys < Q,
    reduced: |acc| < 4 B10 Q 2^-32 + Q/2 <= 2.2 Q (kLmkAcc 22), and the inverse's 8 Q limit fits 32 bits"""
    for ps, m, p in rows():
        if p.kernel == 1 and m in (bf.LMKCDEY, bf.AP) and (1 << 27) <= p.Q < (1 << 28):
            Q = p.Q
            b10 = stages(1 << (p.baseG.bit_length() - 2), Q, 10)[-1]
            acc = 4 * b10 * Fraction(Q, 1 << 32) + Fraction(Q, 2)
            assert acc <= Fraction(22, 10) * Q, (ps, m, float(acc / Q))
            assert 8 * Q < TWO31


def test_k1w_qm1_accumulator_bound():
    """K1w LMKCDEY at 2^27 <= Q < 2^28 (QM 1) without its forward reduction: own and partner words each
    < ND B11 Q 2^-32 + Q/2, their sum within kL2AccBound (2.9 Q for two digits, 3.9 Q for three)"""
    for ps, m, p in rows():
        if p.kernel == 4 and m == bf.LMKCDEY and (1 << 27) <= p.Q < (1 << 28):
            Q, nd = p.Q, p.digitsG - 1
            b11 = stages(1 << (p.baseG.bit_length() - 2), Q, 11)[-1]
            acc = 2 * (nd * b11 * Fraction(Q, 1 << 32) + Fraction(Q, 2))
            assert acc <= Fraction(29 if nd == 2 else 39, 10) * Q, (ps, m, float(acc / Q))
