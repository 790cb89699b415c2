"""Independent pure-Python transcription of the engine's FFBS contract.

TEST INFRASTRUCTURE ONLY.  The reference has no FFBS (techreview/Rmd/hmm.Rmd:193-221
describes it in prose and stops at "= \\dots", :213), so the contract is the
engine's own, written out in oracle/hhmm_oracle.c (ffbs_contract) and
DESIGN.md.  This file restates it from that text, sharing no code with the C
oracle: fma via exact rational arithmetic, and the contract's deterministic
exp / log (gsoc17-hhmm_amd/csrc/hhmm_detmath.h) restated from their
specification (det_exp / det_log below), so it is compared bit-for-bit with
the oracle.  Dot products and the multinomial / Tayal tables come from the
Stan transcription (tests/oracle_numpy.py).
"""
import math
import struct
from fractions import Fraction

import numpy as np

import oracle_numpy as onp

NINF = float("-inf")


def fma(a, b, c):
    """Exactly rounded a * b + c (finite arguments)."""
    if not (math.isfinite(a) and math.isfinite(b) and math.isfinite(c)):
        return a * b + c
    return float(Fraction(a) * Fraction(b) + Fraction(c))


# hhmm_detmath.h constants
_INV_LN2 = float.fromhex("0x1.71547652b82fep+0")
_LN2_HI = float.fromhex("0x1.62e42feep-1")
_LN2_LO = float.fromhex("0x1.a39ef35793c76p-33")
_SQRT2 = float.fromhex("0x1.6a09e667f3bcdp+0")
_LOG_C = [2.0 / (2 * n + 1) for n in range(10, 0, -1)]       # 2/21 .. 2/3
NEG_LOG_SQRT_TWO_PI = onp.NEG_LOG_SQRT_TWO_PI


def _u64(x):
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _f64(u):
    return struct.unpack("<d", struct.pack("<Q", u))[0]


def _exp2_table():
    """2^(j/128) as a double-double (hi = RN(v), lo = RN(v - hi)), from 60-digit decimals."""
    from decimal import Decimal, getcontext
    getcontext().prec = 60
    tab = []
    for j in range(128):
        v = Decimal(2) ** (Decimal(j) / Decimal(128))
        hi = float(v)  # float(Decimal) is correctly rounded
        tab.append((hi, float(v - Decimal(hi))))
    return tab


_EXP2 = _exp2_table()
# hhmm_crlog_table.h: ln2/128 in parts (HI with 35 significant bits) and 128/ln2
_L2_HI = float.fromhex("0x1.62e42fef80000p-8")
_L2_MID = float.fromhex("0x1.1cf79abc80000p-43")
_INV_L2 = float.fromhex("0x1.71547652b82fep+7")
_EXP_P = [1.0 / 120, 1.0 / 24, 1.0 / 6, 0.5, 1.0]  # each correctly rounded


def det_exp(x):
    """k = rint(x 128/ln2), r = x - k ln2/128 (two fma), q = r (1 + r/2 + ... + r^4/120)
    (Horner, fma), 2^(j/128) (T.hi + fma(T.hi, q, T.lo)), times 2^(k >> 7) rounded once."""
    if math.isnan(x):
        return x + x
    xc = -746.0 if x < -746.0 else (710.0 if x > 710.0 else x)
    kd = float(round(xc * _INV_L2))  # round(): ties to even, as rint
    r = fma(-kd, _L2_HI, xc)
    r = fma(-kd, _L2_MID, r)
    p = _EXP_P[0]
    for c in _EXP_P[1:]:
        p = fma(p, r, c)
    q = p * r
    k = int(kd)
    hi, lo = _EXP2[k & 127]
    y0 = hi + fma(hi, q, lo)
    m = k >> 7
    # y0 2^m rounded once: exact scaling in the normal range; where the result is
    # subnormal the exact rational y0 2^m is rounded by float() (correctly rounded
    # int / int division), past the top it overflows to +inf
    if m < -1000:
        v = Fraction(y0) * Fraction(1, 2 ** -m)
        return float(v.numerator / v.denominator) if v.numerator else 0.0
    try:
        return math.ldexp(y0, m)
    except OverflowError:
        return math.inf


def det_log(x):
    """x = 2^e m, m in [sqrt(1/2), sqrt(2)); s = (m-1)/(m+1);
    log m = fma(s^3, q(s^2), 2s); + e ln2 (two fma)."""
    if not (x > 0.0 and x < math.inf):
        return NINF if x == 0.0 else (x if x == math.inf else math.nan)
    sub = x < 2.0 ** -1022
    u = _u64(x * 2.0 ** 54 if sub else x)
    m = _f64((u & 0x000FFFFFFFFFFFFF) | 0x3FF0000000000000)
    hi = m > _SQRT2
    if hi:
        m = m * 0.5
    e = ((u >> 52) & 0x7FF) - 1023 - (54 if sub else 0) + int(hi)
    s = (m - 1.0) / (m + 1.0)
    s2 = s * s
    q = _LOG_C[0]
    for c in _LOG_C[1:]:
        q = fma(q, s2, c)
    lm = fma(s * s2, q, 2.0 * s)
    E = float(e)
    return fma(E, _LN2_HI, fma(E, _LN2_LO, lm))


def fmax(a, b):
    if math.isnan(a):
        return b
    if math.isnan(b):
        return a
    return a if a > b else b


def renorm(v):
    mx = v[0]
    for a in v[1:]:
        mx = fmax(mx, a)
    e = 0
    if math.isfinite(mx) and mx != 0.0:
        e = math.frexp(mx)[1]
    return [math.ldexp(a, -e) for a in v]


def cat(w, u):
    s = w[0]
    for a in w[1:]:
        s = s + a
    if not (s > 0.0) or not math.isfinite(s):
        return 0
    us = u * s
    b = 0
    c = w[0]
    while b < len(w) - 1 and us > c:
        b += 1
        c = c + w[b]
    return b + 1


def _semisup_on(g, j1):
    return (g == 1 and j1 in (1, 4)) or (g == 2 and j1 in (2, 3))


def _tayal_on(s, j1):
    return (s == 1 and j1 in (2, 3)) or (s == 2 and j1 in (1, 4))


def hmm_family(model, T, K, x, p, A, uu, phi=None, mu=None, sigma=None, aux=None):
    """Draws z[0..T) (1-based) for hmm / hmm-multinom / semisup / tayal."""
    def emission(t):
        if model == "hmm":
            lp = [onp.normal_lpdf(float(x[t]), float(mu[j]), float(sigma[j])) for j in range(K)]
            m = NINF
            for a in lp:
                m = fmax(m, a)
            return [det_exp(a - m) for a in lp]
        return [float(phi[j][int(x[t]) - 1]) for j in range(K)]

    def on(t, j1):
        if model == "hmm-multinom-semisup":
            return _semisup_on(int(aux[t]), j1)
        if model == "hhmm-tayal2009":
            return _tayal_on(int(aux[t]), j1)
        return True

    f = [None] * T
    e = emission(0)
    if model == "hmm":
        f0 = [float(p[j]) for j in range(K)]
    elif model == "hhmm-tayal2009":
        f0 = [e[j] * float(p[j]) if ((aux[0] == 1 and j == 2) or (aux[0] == 2 and j == 0)) else e[j]
              for j in range(K)]
    else:
        f0 = [float(p[j]) * e[j] for j in range(K)]
    f[0] = renorm(f0)
    for t in range(1, T):
        e = emission(t)
        fp = f[t - 1]
        tot = fp[0]
        for a in fp[1:]:
            tot = tot + a
        nf = []
        for j in range(K):
            s = fp[0] * float(A[0][j])
            for i in range(1, K):
                s = fma(fp[i], float(A[i][j]), s)
            if not on(t, j + 1):
                s = tot
            nf.append(s * e[j])
        f[t] = renorm(nf)
    z = [0] * T
    z[T - 1] = cat(f[T - 1], float(uu[T - 1]))
    for t in range(T - 2, -1, -1):
        zn = z[t + 1]
        if zn == 0:
            continue
        o = on(t + 1, zn)
        w = [f[t][i] * float(A[i][zn - 1]) if o else f[t][i] for i in range(K)]
        z[t] = cat(w, float(uu[t]))
    return z


def iohmm(T, K, p, E, Arows, uu):
    """Draws for the IOHMM programs; E[t][k] the emission factor e_t(k),
    Arows[t][k] the softmax numerators th_t(k), 0-based (Arows[0] = p filler)."""
    v = []
    for t in range(T):
        e = E[t]
        v.append([float(p[k]) * e[k] for k in range(K)] if t == 0 else e)
    z = []
    for t in range(T):
        w = [v[t][i] * Arows[t + 1][i] for i in range(K)] if t + 1 < T else v[t]
        z.append(cat(w, float(uu[t])))
    return z


def iohmm_det_inputs(model, T, K, u, x, d):
    """The contract's e_t and th_t (th[0] = p filler): the model's emission and
    softmax transition (iohmm-reg.stan:40-57, iohmm-mix.stan:42-65) with
    det_exp / det_log."""
    w = [[float(v) for v in row] for row in np.asarray(d["w_km"])]
    A = [[float(v) for v in d["p_1k"]]]
    for t in range(1, T):
        v = [onp.eigen_dot(u[t], w[j]) for j in range(K)]
        mx = v[0]
        for a in v[1:]:
            if a > mx:
                mx = a
        # the softmax numerators (cat normalises the weights itself)
        A.append([det_exp(a - mx) for a in v])
    E = []
    for t in range(T):
        if model == "iohmm-reg":
            # e_t(j) = det_exp(ob_t(j) - m), m = fmax over j (0 if -inf)
            ob = []
            for j in range(K):
                b = [float(v) for v in np.asarray(d["b_km"])[j]]
                sg = float(d["s_k"][j])
                z = (x[t] - onp.eigen_dot(u[t], b)) * (1.0 / sg)
                ob.append((NEG_LOG_SQRT_TWO_PI - det_log(sg)) + (-0.5 * (z * z)))
            m = ob[0]
            for a in ob[1:]:
                m = fmax(m, a)
            if m == NINF:
                m = 0.0
            E.append([det_exp(a - m) for a in ob])
            continue
        # mixture: e_t(j) = sum_l det_exp(acc_jl - m) over the finite summands of the
        # model's log_sum_exp, m = fmax over j of max_l acc_jl (0 if -inf): no det_log
        accs, m = [], NINF
        for j in range(K):
            lam, mu, sk = (np.asarray(d[k])[j] for k in ("lambda_kl", "mu_kl", "s_kl"))
            acc = []
            for l in range(len(lam)):
                sg = float(sk[l])
                z = (x[t] - float(mu[l])) * (1.0 / sg)
                acc.append(det_log(float(lam[l])) + ((NEG_LOG_SQRT_TWO_PI - det_log(sg)) + (-0.5 * (z * z))))
            mx = NINF
            for a in acc:
                if a > mx:
                    mx = a
            m = mx if j == 0 else fmax(m, mx)
            accs.append(acc)
        if m == NINF:
            m = 0.0
        row = []
        for acc in accs:
            sm = 0.0
            for a in acc:
                if a != NINF:
                    sm += det_exp(a - m)
            row.append(sm)
        E.append(row)
    return E, A


def run(model, data, draws, uniforms):
    """z_ffbs per pair (GRID pairing, p = s + S*n), as lists of length T."""
    xkey = "x_t" if model.startswith("iohmm") else "x"
    x = np.atleast_2d(np.asarray(data[xkey]))
    N, Tm = x.shape
    S = next(np.asarray(v).shape[0] for v in draws.values())
    Ts = np.asarray(data["T"]).reshape(N) if "T" in data else np.full(N, Tm)
    K = int(data["K"])
    out = []
    for p in range(N * S):
        n, s = p // S, p % S
        T = int(Ts[n])
        d = {k: np.asarray(v)[s] for k, v in draws.items()}
        uu = np.asarray(uniforms)[p, :T]
        if model.startswith("iohmm"):
            u = np.asarray(data["u_tm"]).reshape(N, Tm, -1)[n, :T]
            xt = [float(v) for v in np.asarray(data["x_t"]).reshape(N, Tm)[n, :T]]
            E, A = iohmm_det_inputs(model, T, K, [list(map(float, r)) for r in u], xt, d)
            out.append(iohmm(T, K, d["p_1k"], E, A, uu))
        elif model == "hhmm-tayal2009":
            p1, A = onp.tayal_expand(float(d["p_11"]), d["A_row"])
            out.append(hmm_family(model, T, K, x[n], p1, A, uu, phi=d["phi_k"], aux=np.asarray(data["sign"])[n]))
        else:
            aux = np.asarray(data["g"])[n] if "g" in data else None
            out.append(hmm_family(model, T, K, x[n], d["p_1k"], d["A_ij"], uu, phi=d.get("phi_k"),
                                  mu=d.get("mu_k"), sigma=d.get("sigma_k"), aux=aux))
    return out


def exact_marginals(model, T, K, x, p, A, phi=None, mu=None, sigma=None, aux=None, Arows=None, oblik=None):
    """P(z_t = k) under the joint the contract samples from (numpy, normalised
    forward-backward over the forward pass's factors), shape (T, K)."""
    def fac(t):  # K x K transition factor of step t (rows: previous state)
        if Arows is not None:
            return np.tile(np.asarray(Arows[t], dtype=float)[:, None], (1, K))
        F = np.array(A, dtype=float).copy()
        for j in range(K):
            if model == "hmm-multinom-semisup" and not _semisup_on(int(aux[t]), j + 1):
                F[:, j] = 1.0
            if model == "hhmm-tayal2009" and not _tayal_on(int(aux[t]), j + 1):
                F[:, j] = 1.0
        return F

    def emis(t):
        if oblik is not None:
            o = np.asarray(oblik[t], dtype=float)
            return np.exp(o - o.max())
        if model == "hmm":
            lp = np.array([onp.normal_lpdf(float(x[t]), float(mu[j]), float(sigma[j])) for j in range(K)])
            return np.exp(lp - lp.max())
        return np.array([float(phi[j][int(x[t]) - 1]) for j in range(K)])

    e0 = emis(0)
    if model == "hmm":
        a0 = np.array(p, dtype=float)
    elif model == "hhmm-tayal2009":
        a0 = np.array([e0[j] * p[j] if ((aux[0] == 1 and j == 2) or (aux[0] == 2 and j == 0)) else e0[j]
                       for j in range(K)])
    else:
        a0 = np.array(p, dtype=float) * e0
    al = [a0 / a0.sum()]
    for t in range(1, T):
        a = (al[-1] @ fac(t)) * emis(t)
        al.append(a / a.sum())
    be = [None] * T
    be[T - 1] = np.ones(K)
    for t in range(T - 1, 0, -1):
        b = fac(t) @ (emis(t) * be[t])
        be[t - 1] = b / b.sum()
    g = np.array([al[t] * be[t] for t in range(T)])
    return g / g.sum(axis=1, keepdims=True)
