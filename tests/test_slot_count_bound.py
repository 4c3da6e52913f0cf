"""The error bound behind the systematic slot counts' exact-recount window
(gen_amd/csrc/gh_kernels.h count_window and k_resample1's
incremental counts), checked in exact rational arithmetic on the host.

count(X) = ceil((X N - o) / S) is taken in floating point and recounted
exactly when v lies within count_window(N) = 2^(ceil(log2 N) + 7 - 53) of an
integer, which is sound if |v - v*| stays below that window.  The kernels'
arithmetic is restated operation by operation with correctly rounded doubles
(float(Fraction) rounds to nearest), 1/S anywhere within 2 ulp of
1/(double)S (recip_est's guarantee), and the claimed bounds are asserted:
one evaluation (sys_count) within 8 N 2^-53 + 2^-53, the incremental marks-
loop counts within (14 + IT) N 2^-53 + 2^-53, both under a quarter of the
window.  Random and adversarial cases (N near 2^31, S near 2^62, weights at
2^52).
"""
import math
import random
from fractions import Fraction

import pytest

EPS = Fraction(1, 2**53)


def rn(x: Fraction) -> float:
    return float(x)  # correctly rounded to nearest


def fma(a: float, b: float, c: float) -> float:
    return rn(Fraction(a) * Fraction(b) + Fraction(c))


def mul(a: float, b: float) -> float:
    return rn(Fraction(a) * Fraction(b))


def ulp(x: float) -> Fraction:
    return Fraction(math.ulp(x))


def window(N: int) -> Fraction:
    lg = 0 if N <= 1 else (N - 1).bit_length()
    return Fraction(2) ** (lg + 7 - 53)


def cases(rng: random.Random, n: int):
    for _ in range(n):
        N = rng.choice([1, 2, 3, 777, 70001, 1 << 20, 1 << 21, (1 << 31) - 1, rng.randrange(1, 1 << 31)])
        shift = min(52, 62 - (0 if N <= 1 else (N - 1).bit_length()))
        IT = rng.choice([4, 8, 16])
        # tile weights: mostly near the top of the scale (peaked) or anything below
        q = [rng.choice([1 << shift, rng.randrange(0, (1 << shift) + 1), 0]) if k < N else 0 for k in range(IT)]
        # S: this tile's weights plus up to 2^shift for each of the other N - IT particles
        S = max(sum(q) + rng.randrange(0, max(N - IT, 0) * (1 << shift) + 1), 1)
        X0 = rng.randrange(0, S - sum(q) + 1)
        o = rng.choice([0, rng.randrange(0, S), S - 1])
        inv_exact = rn(Fraction(1, 1) / Fraction(rn(Fraction(S))))
        d = rng.randrange(-2, 3)  # recip_est: within 2 ulp of 1 / (double)S
        invS = inv_exact + d * math.ulp(inv_exact)
        yield N, S, o, q, X0, invS


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_slot_count_error_within_quarter_window(seed):
    rng = random.Random(seed)
    for N, S, o, q, X0, invS in cases(rng, 400):
        w = window(N)
        Nd = float(N)
        # one evaluation: v = fma((double)X, N, -(double)o) * invS
        def v_once(X):
            return mul(fma(rn(Fraction(X)), Nd, -rn(Fraction(o))), invS)

        bound1 = 8 * N * EPS + EPS
        X = X0
        vs = Fraction(X * N - o, S)
        assert abs(Fraction(v_once(X)) - vs) <= bound1 <= w / 4
        # incremental: v_0 as above, then v += q ns by one FMA per particle
        IT = len(q)
        ns = mul(Nd, invS)
        v = v_once(X0)
        boundk = (14 + IT) * N * EPS + EPS
        assert boundk <= w / 4
        for qk in q:
            X += qk
            v = fma(float(qk), ns, v)  # (double)q is exact: q <= 2^52
            vs = Fraction(X * N - o, S)
            assert abs(Fraction(v) - vs) <= boundk, (N, S, o, q, X0)


def test_window_values():
    assert window(1 << 21) == Fraction(1, 2**25)
    assert window(1 << 20) == Fraction(1, 2**26)
    assert window(1) == Fraction(1, 2**46)
    assert window((1 << 31) - 1) == Fraction(1, 2**15)
