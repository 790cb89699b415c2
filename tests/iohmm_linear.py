"""Test helper: the IOHMM linear-space filter in numpy (the arithmetic of
hhmm_iohmm.h iohmm_sweep, not Stan's), to show which inputs drive it below the
sweeps' underflow check kIoWeak = 2^-960 (gsoc17-hhmm_amd/csrc/hhmm_iolog.hip).
Test infrastructure only: it decides nothing the engine outputs."""
import numpy as np

IO_WEAK = 2.0 ** -960


def _softmax(v):
    v = v - v.max(-1, keepdims=True)
    e = np.exp(v)
    return e / e.sum(-1, keepdims=True)


def reg_linear_floor(data, draws):
    """iohmm-reg, grid pairing: the smallest value the linear filter's check
    sees over every pair and step -- max f_0, then s_t = sum_i f_{t-1}(i) A_t(i)
    of the renormalised filter (iohmm-reg.stan:59-78 in linear space)."""
    x = np.asarray(data["x_t"], dtype=np.float64)
    u = np.asarray(data["u_tm"], dtype=np.float64)
    w, b, s, p1 = (np.asarray(draws[k], dtype=np.float64) for k in ("w_km", "b_km", "s_k", "p_1k"))
    A = _softmax(np.einsum("ntm,skm->nstk", u, w))
    mu = np.einsum("ntm,skm->nstk", u, b)
    sd = s[None, :, None, :]
    o = -0.5 * np.log(2 * np.pi) - np.log(sd) - 0.5 * ((x[:, None, :, None] - mu) / sd) ** 2
    e = np.exp(o - o.max(-1, keepdims=True))
    f = p1[None] * e[:, :, 0, :]
    worst = f.max(-1).min()
    with np.errstate(all="ignore"):
        for t in range(1, x.shape[1]):
            mx = f.max(-1, keepdims=True)
            f = np.where(mx > 0, f / np.where(mx > 0, mx, 1.0), f)
            sv = (f * A[:, :, t, :]).sum(-1)
            worst = min(worst, sv.min())
            f = e[:, :, t, :] * sv[..., None]
    return worst
