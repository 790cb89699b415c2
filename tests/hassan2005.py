"""The hassan2005 calibration run's inputs and printed outputs (TEST INFRASTRUCTURE).

hassan2005/main.Rmd:250-285 simulates one IOHMM-reg series (T=300, K=3,
M=4) with set.seed(9000) and fits iohmm-reg.stan to it; the rendered
hassan2005/main.html prints the posterior summary, the relabelling table and
the "Hard classification" confusion table.  Those printed numbers are data
the reference holds; they are restated here as vectors, with the line each
comes from.  The inputs are regenerated with R's own stream (tests/r_rng.py).
"""
import numpy as np

import r_rng

T, K, M = 300, 3, 4                                        # main.Rmd:252-254
SEED = 9000                                                # main.Rmd:272 (n.seed), :280
W_TRUE = np.array([1.2, 0.5, 0.3, 0.1, 0.5, 1.2, 0.3, 0.1, 0.5, 0.1, 1.2, 0.1]).reshape(K, M)    # :257-259
B_TRUE = np.array([5.0, 6.0, 7.0, 0.5, 1.0, 5.0, 0.1, -0.5, 0.1, -1.0, -5.0, 0.2]).reshape(K, M)  # :260-262
S_TRUE = [0.2, 1.0, 2.5]                                   # :263
P1_TRUE = [0.4, 0.2, 0.4]                                  # :264

# main.html:440-725, column "Mean" of summary(stan.fit, pars = c('p_1k','w_km','b_km','s_k')), 2 decimals.
POSTERIOR_MEAN = {
    "p_1k": [0.24, 0.27, 0.49],
    "w_km": [[-0.23, 0.10, 0.39, -0.18], [-0.09, 0.27, 0.32, -0.53], [-0.28, 0.14, 0.17, -0.37]],
    "b_km": [[0.01, -1.05, -4.91, -0.09], [0.86, 5.00, 0.15, -0.28], [5.04, 6.01, 6.99, 0.46]],
    "s_k": [2.74, 1.00, 0.21],
}
# main.html:440-725, column "Med" (the posterior medians), same rows.
POSTERIOR_MEDIAN = {
    "p_1k": [0.20, 0.23, 0.47],
    "w_km": [[-0.33, 0.47, 0.46, -0.17], [-0.19, 0.64, 0.36, -0.54], [-0.38, 0.56, 0.15, -0.43]],
    "b_km": [[0.00, -1.06, -4.90, -0.09], [0.86, 5.00, 0.15, -0.28], [5.04, 6.01, 6.99, 0.47]],
    "s_k": [2.74, 0.99, 0.21],
}
# main.html:749-753: table(new = zrelab, original = z); rows new 1..3, columns original 1..3.
RELABEL_TABLE = np.array([[0, 0, 102], [0, 108, 0], [90, 0, 0]])
# main.html:1131-1161: table(estimated = which.max(round(median alpha_tk)), real = zrelab).
HARD_TABLE = np.array([[89, 4, 1], [10, 100, 1], [3, 4, 88]])


def simulate():
    """u, z, x of main.Rmd:280-285: u <- matrix(rnorm(T*M), T, M) (column-major),
    then iohmm_sim (:159-189) with obsmodel_reg (:197-218)."""
    st = r_rng.RStream(SEED)
    u = np.array(st.rnorm(T * M)).reshape(M, T).T
    z = [st.sample1(P1_TRUE)]                                          # :175
    for t in range(1, T):
        p = r_rng.r_softmax([r_rng.r_dot(u[t], W_TRUE[j]) for j in range(K)])   # :177
        z.append(st.sample1(p))                                         # :178
    x = [st.rnorm(1, r_rng.r_dot(u[t], B_TRUE[z[t] - 1]), S_TRUE[z[t] - 1])[0] for t in range(T)]  # :214
    return u, np.array(z), np.array(x)


def stan_data(u, x):
    return {"T": T, "K": K, "M": M, "x_t": x[None], "u_tm": u[None]}


def draws(point):
    return {k: np.asarray(v, dtype=np.float64)[None] for k, v in point.items()}


def table(rows, cols):
    """R's table(rows, cols) over labels 1..K."""
    out = np.zeros((K, K), dtype=np.int64)
    for r, c in zip(rows, cols):
        out[r - 1, c - 1] += 1
    return out


def which_max(v):
    """R's which.max: the first maximum, 1-based."""
    return int(np.argmax(v)) + 1


def relabel(alpha, z):
    """main.Rmd:361-374: hard = which.max(alpha_t); zrelab[z == k] = which.max(table(hard, z)[, k])."""
    hard = [which_max(a) for a in alpha]
    tab = table(hard, z)
    zrelab = np.zeros_like(z)
    for k in range(1, K + 1):
        zrelab[z == k] = which_max(tab[:, k - 1])
    return zrelab


def hard_table(alpha, zrelab):
    """main.Rmd:446-453: table(which.max(round(alpha_t)), zrelab).  round() first,
    so a step where no state passes 0.5 counts as state 1 (which.max of zeros)."""
    return table([which_max(np.round(a)) for a in alpha], zrelab)
