"""R 3.3's default random number stream, restated in Python (TEST INFRASTRUCTURE).

Used only to regenerate the simulated data of the reference's hassan2005
calibration run (hassan2005/main.Rmd:280-285), whose rendered output
(hassan2005/main.html) is the second reference-held result this repo pins
parity to (tests/test_hassan2005.py).  R itself is not in the image; this is
a restatement of the published algorithms R's defaults use:

* RNGkind "Mersenne-Twister" (src/main/RNG.c): set.seed(s) scrambles the
  seed with 50 rounds of the LCG seed = 69069*seed + 1 (mod 2^32), fills the
  625-word state (mti slot + mt[624]) with further LCG steps, then sets
  mti = 624 (FixupSeeds, initial=1), so the first draw regenerates the block.
  MT19937 (Matsumoto & Nishimura 1998), genrand output * 2^-32, and
  unif_rand's fixup keeps the result strictly inside (0, 1).
* normal.kind "Inversion" (src/nmath/snorm.c): u = unif_rand();
  u = (int)(BIG*u) + unif_rand(); qnorm5(u/BIG) with BIG = 134217728 = 2^27.
* qnorm5 is Wichura's AS241 (PPND16, Applied Statistics 37:477, 1988).
* sample(x, 1, prob=p) (src/main/random.c do_sample): FixupProb divides by
  the plain-double sum; size 1 takes the ProbSampleReplace branch (identical
  draws to ProbSampleNoReplace at size 1): revsort (heapsort, descending,
  permutation carried alongside), cumulative sums, first j with
  unif_rand() <= cum[j] (the last slot is never compared).

Checked against values R prints for well-known seeds (tests/test_r_rng.py).
"""
import math

import numpy as np

_N, _M = 624, 397
_MATRIX_A, _UPPER, _LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF
_I2_32M1 = 2.328306437080797e-10  # 1/(2^32 - 1), RNG.c's fixup constant
_BIG = 134217728.0


class RStream:
    """The Mersenne-Twister + Inversion stream after set.seed(seed)."""

    def __init__(self, seed):
        s = seed & 0xFFFFFFFF
        for _ in range(50):
            s = (69069 * s + 1) & 0xFFFFFFFF
        words = []
        for _ in range(_N + 1):
            s = (69069 * s + 1) & 0xFFFFFFFF
            words.append(s)
        self.mt = words[1:]      # dummy[1..624]
        self.mti = _N            # dummy[0], FixupSeeds(initial=1)

    def _regen(self):
        mt = self.mt
        for kk in range(_N):
            y = (mt[kk] & _UPPER) | (mt[(kk + 1) % _N] & _LOWER)
            mt[kk] = mt[(kk + _M) % _N] ^ (y >> 1) ^ (_MATRIX_A if y & 1 else 0)
        self.mti = 0

    def genrand(self):
        if self.mti >= _N:
            self._regen()
        y = self.mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y * 2.3283064365386963e-10

    def unif_rand(self):
        x = self.genrand()
        if x <= 0.0:
            return 0.5 * _I2_32M1
        if 1.0 - x <= 0.0:
            return 1.0 - 0.5 * _I2_32M1
        return x

    def norm_rand(self):
        u = self.unif_rand()
        u = float(int(_BIG * u)) + self.unif_rand()
        return qnorm(u / _BIG)

    def rnorm(self, n, mean=0.0, sd=1.0):
        return [mean + sd * self.norm_rand() for _ in range(n)]

    def runif(self, n):
        return [self.unif_rand() for _ in range(n)]

    def sample1(self, prob):
        """sample(1:len(prob), 1, prob = prob): a 1-based index."""
        p = [float(v) for v in prob]
        tot = 0.0
        for v in p:
            if v > 0.0:
                tot += v
        p = [v / tot for v in p]
        perm = list(range(1, len(p) + 1))
        revsort(p, perm)
        for i in range(1, len(p)):
            p[i] += p[i - 1]
        ru = self.unif_rand()
        j = 0
        while j < len(p) - 1 and not ru <= p[j]:
            j += 1
        return perm[j]


def revsort(a, ib):
    """R's revsort (src/main/sort.c): heapsort a[] into descending order,
    carrying ib[] alongside; in place, 1-based internally."""
    n = len(a)
    if n <= 1:
        return
    a.insert(0, None)
    ib.insert(0, None)
    l_ = (n >> 1) + 1
    ir = n
    while True:
        if l_ > 1:
            l_ -= 1
            ra, ii = a[l_], ib[l_]
        else:
            ra, ii = a[ir], ib[ir]
            a[ir], ib[ir] = a[1], ib[1]
            ir -= 1
            if ir == 1:
                a[1], ib[1] = ra, ii
                break
        i = l_
        j = l_ << 1
        while j <= ir:
            if j < ir and a[j] > a[j + 1]:
                j += 1
            if ra > a[j]:
                a[i], ib[i] = a[j], ib[j]
                i = j
                j += j
            else:
                j = ir + 1
        a[i], ib[i] = ra, ii
    del a[0]
    del ib[0]


def qnorm(p):
    """AS241 PPND16 lower-tail quantile of N(0, 1), as qnorm5(p, 0, 1, 1, 0)."""
    if p <= 0.0:
        return -math.inf
    if p >= 1.0:
        return math.inf
    q = p - 0.5
    if abs(q) <= 0.425:
        r = 0.180625 - q * q
        return (q * (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r
                          + 45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r
                       + 133.14166789178437745) * r + 3.387132872796366608)
                / (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r
                        + 21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r
                     + 42.313330701600911252) * r + 1.0))
    r = p if q < 0 else 1.0 - p
    r = math.sqrt(-math.log(r))
    if r <= 5.0:
        r += -1.6
        val = ((((((((r * 7.7454501427834140764e-4 + 0.0227238449892691845833) * r + 0.24178072517745061177) * r
                    + 1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r
                 + 4.6303378461565452959) * r + 1.42343711074968357734)
               / (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + 0.0151986665636164571966)
                       * r + 0.14810397642748007459) * r + 0.68976733498510000455) * r + 1.6763848301838038494) * r
                    + 2.05319162663775882187) * r + 1.0))
    else:
        r += -5.0
        val = ((((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + 0.0012426609473880784386)
                    * r + 0.026532189526576123093) * r + 0.29656057182850489123) * r + 1.7848265399172913358) * r
                 + 5.4637849111641143699) * r + 6.6579046435011037772)
               / (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5)
                       * r + 7.868691311456132591e-4) * r + 0.0148753612908506148525) * r
                     + 0.13692988092273580531) * r + 0.59983220655588793769) * r + 1.0))
    return -val if q < 0.0 else val


# ---- R arithmetic the simulation uses -------------------------------------------------------
def r_dot(a, b):
    """u[t, ] %*% w[j, ]: R 3.3's matprod -> reference BLAS dgemm, one running sum from 0."""
    s = 0.0
    for x, y in zip(a, b):
        s += x * y
    return s


def r_sum(v):
    """sum() of doubles: rsum accumulates in long double (x86 80-bit)."""
    s = np.longdouble(0.0)
    for x in v:
        s += np.longdouble(x)
    return float(s)


def r_softmax(x):
    """common/R/math.R:1-10: softmax(x) = exp(x - logsumexp(x))."""
    y = max(x)
    lse = y + math.log(r_sum([math.exp(v - y) for v in x]))
    return [math.exp(v - lse) for v in x]
