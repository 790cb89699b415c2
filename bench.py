#!/usr/bin/env python3
"""Benchmark: series-timesteps/s of forward-backward + gamma + Viterbi (K=4).

Workload (BASELINE.json configs[1], the metric's single-GPU config C2):
hmm/stan/hmm-multinom.stan, K=4, L=9, 1,000,000 (series, draw) pairs
(one posterior draw per series, HHMM_PAIR_ZIP) x T=1000, fp64.  One step =
one pass of the hot path over the whole batch with inputs resident in HBM,
through the C ABI (hhmm_run_device): ONE request for gamma_tk [P,T,K],
loglik [P], zstar_t [P,T] and logp_zstar [P], which the library runs as
fb_kernel on the caller's stream beside viterbi_kernel on a side stream
(forked and joined).  --fused times the same request with HHMM_FLAG_FUSED
(fbv_kernel: one sweep, x read once); both halves alone and the other
schedule are reported after the timed region.

Multi-GPU (one process per GPU): every rank evaluates its own 1M pairs (weak
scaling, no data-path collective); the per-step summed log-likelihood is
all-reduced over RCCL (the path's only exchange).  `--gpus N` with N > 1 and
no WORLD_SIZE in the environment re-launches this script as N ranks under
torch.distributed.run (a child process started before anything touches the
GPU); under a launcher the world size must equal --gpus.  The decoded paths
leave the device after the timed region: each rank copies its zstar_t slice
into a pinned host buffer (the per-rank D2H the R host would do into its
slice of the caller's array), timed on its own (`path_gather`).  `--stub`
rehearses the launcher and the timing harness on CPU ranks over gloo.

Prints ONE JSON line on rank 0 (contract in the task statement), including
`roofline` for the dominant kernel (HIP events on the launch stream) and
`cpu_baseline` (the stanc-faithful CPU oracle, libm log, timed on a bounded
sample of the same workload on the host cores).
"""
import argparse
import ctypes as C
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "gsoc17-hhmm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hhmm_amd  # noqa: E402
import hhmm_amd.api  # noqa: E402
from hhmm_amd import _abi, synth  # noqa: E402

HBM_PEAK = 8.0e12  # B/s, MI355X HBM3E (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=1_000_000, help="pairs per GPU")
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=synth.SEED)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the 64-pair oracle check of the timed data (outside the timed region)")
    ap.add_argument("--check-at", default="after", choices=["after", "before"],
                    help="C2: the oracle check on the last timed step's outputs (after) or between the warmup "
                         "and the timed steps (before: the device idles while the host checks)")
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c2-host", "c3", "c4", "c5", "n1", "n2", "f1"],
                    help="c2 (default, the metric's config) or one of the other BASELINE configs, each "
                         "printed as its own line: c1 hmm Gaussian K=3 T=500, c3 iohmm-reg grid, c4 iohmm-hmix "
                         "+ FFBS, c5 Tayal T=1e6 (parallel scan over T); n1 = hmm-multinom at K=23 (SURVEY §8 N1); "
                         "n2 = hmm-multinom K=23, T=1e6, 250 pairs (the large-K parallel scan, MFMA chunk products); "
                         "f1 = the tick -> leg feature extractor (SURVEY §8 F1); c2-host = the C2 request "
                         "through hhmm_run from pageable host arrays to host arrays (the R .Call path, "
                         "SURVEY §8b; --pairs defaults to 200000 there)")
    ap.add_argument("--ticks", type=int, default=100_000_000, help="f1: ticks per GPU")
    ap.add_argument("--pars", default=None,
                    help="c3-c5 probes: comma-separated outputs instead of the workload's")
    ap.add_argument("--flags", type=int, default=0, help="c3-c5 probes: hhmm_request.flags")
    ap.add_argument("--fused", action="store_true",
                    help="time the one-kernel fused sweep (HHMM_FLAG_FUSED) instead of the two-kernel schedule")
    ap.add_argument("--schedule", default=None, choices=["step", "fused", "split", "vfb", "two"],
                    help="c2: the request's schedule: step (library default), fused (HHMM_FLAG_FUSED), "
                         "split (HHMM_FLAG_FB_SPLIT), vfb (HHMM_FLAG_VFB, phased sweep), two (fb_kernel || "
                         "viterbi_kernel, HHMM_FLAG_VFB_OFF)")
    ap.add_argument("--no-sequential", action="store_true",
                    help="n2: skip the one untimed run on the sequential kernels after the timed region")
    ap.add_argument("--no-path-gather", action="store_true",
                    help="skip the timed D2H of the decoded paths after the timed region")
    ap.add_argument("--stub", action="store_true",
                    help="launcher rehearsal without a GPU: CPU ranks over gloo, a fixed numpy step")
    ap.add_argument("--master-port", type=int, default=0, help="rendezvous port for --gpus N > 1 (0: a free one)")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# Ranks: launch, rendezvous, timing over ranks
# ---------------------------------------------------------------------------

def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv=None):
    """`--gpus N` (N > 1) without a launcher: start N ranks of this script
    under torch.distributed.run as a CHILD process (no exec, and nothing in
    this parent has touched the GPU) and return its exit code."""
    import subprocess
    argv = list(sys.argv[1:] if argv is None else argv)
    port = a.master_port or _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(pathlib.Path(__file__).resolve())] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


class Ranks:
    """World/rank from the launcher's environment; the process group (nccl =
    RCCL on a GPU box, gloo for --stub) and the collectives the timing needs."""

    def __init__(self, a):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={self.world} ranks")
        self.stub = a.stub
        self.dist = None
        # rehearsal knobs for a one-GPU box (never set by the driver): the
        # ranks share the visible devices (local rank modulo their count) and
        # talk over gloo, since RCCL refuses two ranks on one device
        self.backend = os.environ.get("HHMM_BENCH_BACKEND", "gloo" if self.stub else "nccl")
        self.gpu = self.local
        if not self.stub and os.environ.get("HHMM_BENCH_SHARE_DEVICES"):
            self.gpu = self.local % max(1, torch.cuda.device_count())
        if self.world > 1:
            import torch.distributed as dist
            if not self.stub:
                torch.cuda.set_device(self.gpu)
            dist.init_process_group(self.backend)
            self.dist = dist
        self.dev = torch.device("cpu") if self.stub else torch.device("cuda", self.gpu)
        self.cdev = torch.device("cpu") if self.backend == "gloo" else self.dev  # where collectives run

    def sync(self):
        if not self.stub:
            torch.cuda.synchronize()

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def all_reduce_sum(self, t):
        if self.dist:
            if t.device != self.cdev:
                h = t.to(self.cdev)
                self.dist.all_reduce(h)
                t.copy_(h)
            else:
                self.dist.all_reduce(t)
        return t

    def gather(self, values):
        """Per-rank float vectors -> list over ranks (every rank gets it)."""
        t = torch.tensor(values, dtype=torch.float64, device=self.cdev)
        if not self.dist:
            return [t.tolist()]
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.tolist() for o in out]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def timed_region(rk, step, steps, warmup, before_timing=None):
    """W untimed steps, then exactly K steps bracketed by barrier + device
    synchronize on both sides.  Returns the wall time of this rank, the max
    over ranks and the per-rank list."""
    for _ in range(warmup):
        step(None)
    rk.sync()
    if before_timing:
        before_timing()
    rk.barrier()
    rk.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    rk.sync()
    rk.barrier()
    elapsed = time.perf_counter() - t0
    per_rank = [v[0] for v in rk.gather([elapsed])]
    return elapsed, max(per_rank), per_rank


PATH_GATHER_CAP = 512 << 20  # bytes of pinned host buffer per rank for the timed D2H


def path_gather(rk, zs):
    """The decoded paths leave the device: this rank's zstar_t slice is copied
    into a pinned host buffer (a direct D2H per rank into its
    slice of the caller's array), all ranks at once, timed after the timed
    region.  At most PATH_GATHER_CAP bytes (whole time rows) are copied and the
    time is scaled to the whole slice (a 4 GB pinned buffer per rank
    would be 32 GB of pinned memory at 8 GPUs).  Returns bytes per rank and the
    max time over ranks."""
    row = zs[0].numel() * zs.element_size()
    rows = max(1, min(zs.shape[0], PATH_GATHER_CAP // max(row, 1)))
    src = zs[:rows]
    host = torch.empty(src.shape, dtype=zs.dtype, pin_memory=True)
    rk.sync()
    rk.barrier()
    t0 = time.perf_counter()
    host.copy_(src, non_blocking=True)
    rk.sync()
    dt = time.perf_counter() - t0
    rk.barrier()
    nbytes = zs.numel() * zs.element_size()
    sample = src.numel() * src.element_size()
    per_rank = [v[0] * nbytes / sample for v in rk.gather([dt])]
    ok = bool(torch.equal(host[:1], zs[:1].cpu()))
    del host
    return {"bytes_per_rank": nbytes, "ms_max_over_ranks": max(per_rank) * 1e3,
            "ms_per_rank": [x * 1e3 for x in per_rank],
            "GBps_per_rank": nbytes / max(per_rank) / 1e9,
            "GBps_aggregate": rk.world * nbytes / max(per_rank) / 1e9,
            "sample_bytes_per_rank": sample, "scaled_from_sample": sample < nbytes,
            "destination": "pinned host buffer per rank (zstar_t [T, P] int32)", "first_row_verified": ok}


def stub_workload(a, rk):
    """--stub: the launcher, rendezvous and timing harness on CPU ranks (gloo):
    each step is a fixed numpy recursion over this rank's own block."""
    rng = np.random.default_rng(rk.rank)
    P, T = 4096, 64
    x = rng.random((T, P))
    acc = torch.zeros(1, dtype=torch.float64)

    def step(i):
        f = np.ones(P)
        for t in range(T):
            f = f * x[t] + 1e-3
            f /= f.max()
        acc.fill_(float(f.sum()))
        rk.all_reduce_sum(acc)

    elapsed, emax, per_rank = timed_region(rk, step, a.steps, a.warmup)
    if rk.rank == 0:
        print(json.dumps({"metric": "stub (launcher rehearsal)", "value": rk.world * P * T * a.steps / emax,
                          "unit": "series-timesteps/s", "n_gpus": rk.world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": emax / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
                          "rank_ms_per_step": [x / a.steps * 1e3 for x in per_rank],
                          "all_reduce_check": float(acc.item())}), flush=True)


K, L = 4, 9


def make_batch(P, T, seed, dev):
    """Synthetic C2 batch on the device.  x from the true HMM of
    hmm/main-multinom-semisup.R:12-17 with emission rows normalize(1 + 9 e_k);
    one posterior draw per series, jittered as in hhmm_amd.synth."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    A = torch.tensor(synth.A_SEMISUP, device=dev)
    p1 = torch.tensor(synth.P1_SEMISUP, device=dev)
    B = torch.tensor(synth.smoothed_identity(K, L), device=dev)
    cA, cB, cp = A.cumsum(1), B.cumsum(1), p1.cumsum(0)
    # x: [N, T] column-major (series fastest) == torch (T, N) row-major
    x = torch.empty((T, P), dtype=torch.int32, device=dev)
    z = torch.searchsorted(cp, torch.rand(P, generator=g, device=dev, dtype=torch.float64) * cp[-1])
    z = z.clamp_(max=K - 1)
    for t in range(T):
        if t > 0:
            rows = cA[z]
            u = torch.rand(P, 1, generator=g, device=dev, dtype=torch.float64) * rows[:, -1:]
            z = (u >= rows).sum(1).clamp_(max=K - 1)
        rb = cB[z]
        u = torch.rand(P, 1, generator=g, device=dev, dtype=torch.float64) * rb[:, -1:]
        x[t] = ((u >= rb).sum(1).clamp_(max=L - 1) + 1).to(torch.int32)

    def dirichlet_rows(rows, S):
        # rows (R, C) -> F-order [S, R, C] == torch (C, R, S)
        conc = 200.0 * rows + 1.0
        out = torch.empty((rows.shape[1], rows.shape[0], S), dtype=torch.float64, device=dev)
        for r in range(rows.shape[0]):
            gam = torch._standard_gamma(conc[r].expand(S, -1).contiguous(), generator=g)
            out[:, r, :] = (gam / gam.sum(1, keepdim=True)).T
        return out

    draws = {
        "p_1k": dirichlet_rows(p1[None, :], P),          # (K, 1, S)
        "A_ij": dirichlet_rows(A, P),                     # (K, K, S)
        "phi_k": dirichlet_rows(B, P),                    # (L, K, S)
    }
    return x, draws


class DeviceRun:
    """Device buffers and four prepared requests over the same batch and
    outputs: "step" (gamma_tk, loglik, zstar_t, logp_zstar in ONE request:
    the library runs fb_kernel and viterbi_kernel, the latter on a side
    stream forked from and joined into the caller's), "fused" (the same
    request with HHMM_FLAG_FUSED: one fused forward-backward + Viterbi sweep),
    and the two halves alone ("fb", "viterbi")."""

    def __init__(self, lib, x, draws, P, T, dev, share=None):
        """share: another DeviceRun whose output and workspace buffers this one
        reuses (tools/ab_bench.py: every library variant on the same memory)."""
        self.lib = lib
        self.out = share.out if share is not None else {
            "loglik": torch.empty(P, dtype=torch.float64, device=dev),
            "gamma_tk": torch.empty((K, T, P), dtype=torch.float64, device=dev),
            "zstar_t": torch.empty((T, P), dtype=torch.int32, device=dev),
            "logp_zstar": torch.empty(P, dtype=torch.float64, device=dev),
            "pair_status": torch.zeros(P, dtype=torch.int32, device=dev),
        }
        hot = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
        self.reqs = {}
        self._ws = share._ws if share is not None else {}
        for name, outs, flags in (("step", hot, 0), ("fused", hot, _abi.FLAG_FUSED),
                                  ("split", hot, _abi.FLAG_FB_SPLIT), ("vfb", hot, _abi.FLAG_VFB),
                                  ("two", hot, _abi.FLAG_VFB_OFF),
                                  ("fb", ["loglik", "gamma_tk"], 0), ("viterbi", ["zstar_t", "logp_zstar"], 0)):
            r = _abi.Request()
            r.abi_version = _abi.ABI_VERSION
            r.model = _abi.MODELS["hmm-multinom"]
            r.pairing = _abi.PAIR_ZIP
            r.device = -1
            r.flags = flags
            r.data.n_series = P
            r.data.T_max = T
            r.data.K = K
            r.data.L = L
            r.data.x_int = x.data_ptr()
            r.draws.n_draws = P
            for k, v in draws.items():
                setattr(r.draws, k, v.data_ptr())
            res = _abi.Result()
            for o in outs:
                r.outputs |= _abi.OUT[o]
                setattr(res, o, self.out[o].data_ptr())
            res.pair_status = self.out["pair_status"].data_ptr()
            ws = C.c_size_t(0)
            assert lib.hhmm_workspace_size(C.byref(r), C.byref(ws)) == 0
            # one workspace per size (the requests run one at a time on one stream)
            need = max(int(ws.value), 256)
            fit = [k for k in self._ws if k >= need]
            if not fit:
                self._ws[need] = torch.empty(need, dtype=torch.uint8, device=dev)
                fit = [need]
            self.reqs[name] = (r, res, self._ws[min(fit)])

    def launch(self, name):
        r, res, ws = self.reqs[name]
        st = self.lib.hhmm_run_device(C.byref(r), C.byref(res), ws.data_ptr(), ws.numel(),
                                      torch.cuda.current_stream().cuda_stream)
        if st != 0:
            raise RuntimeError(self.lib.hhmm_last_error().decode())


# C2 schedules: the kernel the roofline names, and a description
DEFAULT_SCHEDULE = "vfb"  # what the library runs for the C2 request without flags (HHMM_VFB_DEFAULT)
SCHEDULE_KERNELS = {
    "two": ("fb_kernel+viterbi_kernel", "fb_kernel || viterbi_kernel (library side stream)"),
    "fused": ("fbv_kernel", "fused forward-backward + Viterbi sweep (one kernel, HHMM_FLAG_FUSED)"),
    "split": ("fb_kernel+viterbi_kernel", "forward launch, then backward || packed-symbol Viterbi (HHMM_FLAG_FB_SPLIT)"),
    "vfb": ("vfb_kernel", "phased sweep: Viterbi over x, then forward-backward over its packed symbols "
                          "(one kernel, HHMM_FLAG_VFB)"),
}


def bytes_per_step(T):
    """Algorithmic (compulsory) bytes per series-timestep, SURVEY.md §8d (C2)."""
    params = (K + K * K + K * L) * 8  # p_1k, A_ij, phi_k per pair
    fb = 4 + K * 8 + (params + 8) / T          # x, gamma, params, loglik
    vit = 4 + 4 + (K * K + K * L) * 8 / T + 8 / T  # x, zstar, A/phi, logp
    whole = 4 + K * 8 + 4 + (params + 16) / T  # x once, gamma, zstar, params, loglik+logp
    return fb, vit, whole


def timed_oracle(model, gen, pars, pairing, threads, target_s, n0, cap, uniforms=None):
    """Times the oracle's libm build on a bounded sample: a calibration run of
    n0 units (series or draws, per `gen`), then one sized for ~target_s."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    def run(n, seed_off):
        data, draws, P, T, u = gen(n, seed_off)
        t0 = time.perf_counter()
        pyoracle.gqs(model, data, draws, pars=pars, pairing=pairing, nthreads=threads, variant="libm",
                     uniforms=u)
        return time.perf_counter() - t0, P, T

    run(n0, 0)  # warm (page-in, thread pool)
    dt, P, T = run(n0, 0)
    n = int(max(n0, min(cap, n0 * target_s / max(dt, 1e-3))))
    n = (n // threads) * threads or threads
    dt, P, T = run(n, 1)
    return P * T / dt, P, T, dt


def cpu_baseline(T, target_s, seed):
    """Stanc-faithful CPU oracle (libm log, in-loop log/LSE as Stan) on a
    bounded sample of the same workload (same shapes, host cores): all the
    process's cores (the reported value) and one core beside it."""
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]

    def gen(n, off):
        data, draws = synth.hmm_multinom(N=n, S=n, T=T, K=K, L=L, seed=seed + off)
        return data, draws, n, T, None

    v, P, _, dt = timed_oracle("hmm-multinom", gen, pars, "zip", threads, target_s, 8 * threads, 200_000)
    v1, P1, _, dt1 = timed_oracle("hmm-multinom", gen, pars, "zip", 1, target_s / 3, 8, 20_000)
    return {"value": v, "unit": "series-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{P} pairs x T={T} (hmm-multinom K=4 L=9, zip), FB+gamma+Viterbi, "
                      f"{dt:.1f} s on {threads} threads, oracle libm-log build",
            "single_core": {"value": v1, "cores": 1, "sample": f"{P1} pairs x T={T}, {dt1:.1f} s on 1 thread"},
            "cpu_model": cpu_model()}


def lib_src(lib):
    """The source hash the loaded libhhmm.so was built from (hhmm_version)."""
    return lib.hhmm_version().decode().split(" src ")[-1]


def load_traffic(kernel, P, T, src):
    """HBM bytes per launch of `kernel` from the committed PMC passes
    (profiles/bench_traffic.json, written by tools/prof_summary.py from
    rocprofv3 FETCH_SIZE / WRITE_SIZE, gfx950 correction applied), when they
    were taken on this batch shape AND on the library build now loaded
    (`src`, VERDICT r3: evidence keyed to the build it measured).  Returns
    (bytes or None, source note)."""
    p = ROOT / "profiles" / "bench_traffic.json"
    try:
        bt = json.loads(p.read_text())
    except Exception:
        return None, "no profiles/bench_traffic.json"
    if bt.get("pairs") != P or bt.get("T") != T:
        return None, f"PMC pass taken at pairs={bt.get('pairs')} T={bt.get('T')}, not this shape"
    if bt.get("src") != src:
        return None, f"PMC pass measured build src {bt.get('src')}, the loaded library is src {src}"
    k = bt.get("kernels", {}).get(kernel)
    note = f"{bt.get('source')} (build src {src})"
    return (k.get("hbm_bytes_per_launch") if k else None), note


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    rk = Ranks(a)
    try:
        if a.stub:
            return stub_workload(a, rk)
        torch.cuda.set_device(rk.dev)
        lib = hhmm_amd.load_library()
        assert lib.hhmm_init(1) == 0, lib.hhmm_last_error().decode()
        if a.workload == "f1":
            return features_workload(a, lib, rk)
        if a.workload == "c2-host":
            return c2_host_workload(a, lib, rk)
        if a.workload != "c2":
            return other_workload(a, lib, rk)
        return c2_workload(a, lib, rk)
    finally:
        rk.close()


def c2_workload(a, lib, rk):
    world, rank, dev = rk.world, rk.rank, rk.dev
    P, T = a.pairs, a.T
    x, draws = make_batch(P, T, a.seed + 7919 * rank, dev)
    run = DeviceRun(lib, x, draws, P, T, dev)
    torch.cuda.synchronize()
    s0 = torch.cuda.current_stream()
    name = a.schedule or ("fused" if a.fused else "step")
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(a.steps)]
    total = torch.zeros(1, dtype=torch.float64, device=dev)

    def step(i):
        """One pass of the hot path: one request for gamma_tk, loglik, zstar_t
        and logp_zstar (two kernels, joined on the launch stream; --fused:
        the one-kernel sweep), bracketed by events on the launch stream; then
        the all-reduce of the summed log-likelihood over ranks."""
        if i is not None:
            evs[i][0].record(s0)
        run.launch(name)
        if i is not None:
            evs[i][1].record(s0)
        if world > 1:
            torch.sum(run.out["loglik"], dim=0, keepdim=True, out=total)
            rk.all_reduce_sum(total)

    checked = []

    def check():
        if not a.no_check and rank == 0:
            checked.append(check_slice(run, x, draws, P, T))

    elapsed_rank, elapsed, per_rank = timed_region(rk, step, a.steps, a.warmup,
                                                   before_timing=check if a.check_at == "before" else None)
    if a.check_at == "after":  # the outputs of the last timed step: the same inputs, the same request
        check()
    checked = checked[0] if checked else None
    step_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    rank_step_ms = [v[0] for v in rk.gather([step_ms])]
    bad = int((run.out["pair_status"] != 0).sum().item())
    gather = None if a.no_path_gather else path_gather(rk, run.out["zstar_t"])
    # after the timed region: the other schedules once each (untimed for `value`):
    # the two halves alone (the north star's "batched forward-backward") and the
    # two-kernel schedule
    solo = {}
    others = [nm for nm in ("step", "two", "vfb", "fused", "split") if nm != name]
    for nm in ["fb", "viterbi"] + others:
        ts = []
        for _ in range(3):  # back to back on one stream; median of three launches
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            run.launch(nm)
            e1.record(s0)
            ts.append((e0, e1))
        torch.cuda.synchronize()
        solo[nm] = float(np.median([e0.elapsed_time(e1) for e0, e1 in ts]))

    if rank == 0:
        fb_b, vit_b, whole_b = bytes_per_step(T)
        units = P * T
        sched = SCHEDULE_KERNELS[name if name != "step" else DEFAULT_SCHEDULE]
        dom = sched[0]
        src = lib_src(run.lib)
        if "+" not in dom:
            traffic, pmc_note = load_traffic(dom, P, T, src)
        else:
            (t1, pmc_note), (t2, _) = load_traffic("fb_kernel", P, T, src), load_traffic("viterbi_kernel", P, T, src)
            traffic = (t1 + t2) if (t1 is not None and t2 is not None) else None
        achieved = whole_b * units / (step_ms * 1e-3)
        value = world * units * a.steps / elapsed
        line = {
            "metric": "series-timesteps/sec forward-backward+Viterbi (K=4) at 1/2/4/8 GPU; % HBM roofline",
            "value": value,
            "unit": "series-timesteps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded HMM of hmm/main-multinom-semisup.R, Dirichlet-jittered draws)",
            "config": {"workload": "C2 hmm-multinom K=4 L=9, 1M pairs x T=1000 per GPU (zip pairing)",
                       "pairs_per_gpu": P, "T": T, "outputs": "gamma_tk zstar_t loglik logp_zstar",
                       "parallelism": f"pairs sharded over {world} GPU(s)",
                       "schedule": sched[1]},
            "whole_step_roofline_frac": whole_b * world * units * a.steps / elapsed / (HBM_PEAK * world),
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK,
                         "traffic": traffic, "pmc_source": pmc_note,
                         "algorithmic_bytes_per_series_timestep": whole_b,
                         "duration_ms": step_ms},
            "library": run.lib.hhmm_version().decode(),
            "rank_ms_per_step": [x / a.steps * 1e3 for x in per_rank],
            "rank_kernel_ms": rank_step_ms,
            "path_gather": gather,
            "pair_failures": bad,
            "check": checked,
            "alone_after_timing": {
                "fb_kernel": {"ms": solo["fb"], "algorithmic_bytes_per_series_timestep": fb_b,
                              "roofline_frac": fb_b * units / (solo["fb"] * 1e-3) / HBM_PEAK},
                "viterbi_kernel": {"ms": solo["viterbi"], "algorithmic_bytes_per_series_timestep": vit_b,
                                   "roofline_frac": vit_b * units / (solo["viterbi"] * 1e-3) / HBM_PEAK},
                **{SCHEDULE_KERNELS[nm][1]: {"ms": solo[nm],
                                              "roofline_frac": whole_b * units / (solo[nm] * 1e-3) / HBM_PEAK}
                   for nm in others if nm != "step"}},
        }
        if not a.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(T, a.cpu_seconds, a.seed)
        print(json.dumps(line), flush=True)


def link_rates(dev, nbytes=1 << 30, reps=3):
    """Pinned host <-> device copy rates (B/s) of one nbytes buffer, each way
    alone and both ways at once (PCIe is full duplex)."""
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h2 = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out = {}
    for name in ("h2d", "d2h", "both"):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            if name in ("h2d", "both"):
                with torch.cuda.stream(s1):
                    d.copy_(h, non_blocking=True)
            if name in ("d2h", "both"):
                with torch.cuda.stream(s2):
                    h2.copy_(d2, non_blocking=True)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        out[name] = nbytes / min(ts)
    del h, h2, d, d2
    return out


def c2_host_workload(a, lib, rk):
    """The C2 request (hmm-multinom K=4, gamma_tk + loglik + zstar_t +
    logp_zstar) through hhmm_run: pageable host arrays in, pageable host arrays
    out, as R's .Call hands over REAL() buffers.  The library's
    host pipeline (HHMM_FLAG_HOST_CHUNKS, automatic) overlaps chunk i+1's
    upload and kernels with chunk i's download; the line states the bound the
    host link sets and the one-chunk (no overlap) time beside it."""
    world, rank, dev = rk.world, rk.rank, rk.dev
    P = a.pairs if a.pairs != 1_000_000 else 200_000
    T = a.T
    x_d, draws_d = make_batch(P, T, a.seed + 7919 * rank, dev)
    x = x_d.cpu().numpy()
    draws = {k: v.cpu().numpy() for k, v in draws_d.items()}
    out = {
        "loglik": np.empty(P, dtype=np.float64),
        "gamma_tk": np.empty((K, T, P), dtype=np.float64),
        "zstar_t": np.empty((T, P), dtype=np.int32),
        "logp_zstar": np.empty(P, dtype=np.float64),
    }
    status = np.zeros(P, dtype=np.int32)

    def request(flags):
        r = _abi.Request()
        r.abi_version = _abi.ABI_VERSION
        r.model = _abi.MODELS["hmm-multinom"]
        r.pairing = _abi.PAIR_ZIP
        r.device = -1
        r.flags = flags
        r.data.n_series, r.data.T_max, r.data.K, r.data.L = P, T, K, L
        r.data.x_int = x.ctypes.data
        r.draws.n_draws = P
        for k, v in draws.items():
            setattr(r.draws, k, v.ctypes.data)
        res = _abi.Result()
        for o, arr in out.items():
            r.outputs |= _abi.OUT[o]
            setattr(res, o, arr.ctypes.data)
        res.pair_status = status.ctypes.data
        return r, res

    def call(flags):
        r, res = request(flags)
        st = lib.hhmm_run(C.byref(r), C.byref(res))
        if st < 0:
            raise RuntimeError(lib.hhmm_last_error().decode())

    rates = link_rates(dev)
    fresh_t0 = time.perf_counter()
    call(0)  # first call: pinned staging and device buffers come from the library's pools after this
    first_s = time.perf_counter() - fresh_t0
    for _ in range(max(0, a.warmup - 1)):
        call(0)
    elapsed_rank, elapsed, per_rank = timed_region(rk, lambda i: call(0), a.steps, 0)
    one_chunk = []
    for _ in range(2):
        t0 = time.perf_counter()
        call(_abi.flag_host_chunks(1))
        one_chunk.append(time.perf_counter() - t0)
    # the same request on the device entry: bit-identical outputs
    run = DeviceRun(lib, x_d, draws_d, P, T, dev)
    run.launch("step")
    torch.cuda.synchronize(dev)
    same = {
        "loglik": bool(np.array_equal(run.out["loglik"].cpu().numpy(), out["loglik"])),
        "logp_zstar": bool(np.array_equal(run.out["logp_zstar"].cpu().numpy(), out["logp_zstar"])),
        "zstar_t": bool(np.array_equal(run.out["zstar_t"].cpu().numpy(), out["zstar_t"])),
        "gamma_tk": bool(np.array_equal(run.out["gamma_tk"].cpu().numpy(), out["gamma_tk"])),
        "pair_status": bool(np.array_equal(run.out["pair_status"].cpu().numpy(), status)),
    }
    del run
    up = x.nbytes + sum(v.nbytes for v in draws.values())
    down = sum(v.nbytes for v in out.values()) + status.nbytes
    # each direction alone, and both together (this host link measures about
    # half-duplex: the two copies at once share one aggregate rate)
    t_bound = max(up / rates["h2d"], down / rates["d2h"], (up + down) / (2.0 * rates["both"]))
    if rank == 0:
        value = world * P * T * a.steps / elapsed
        step_s = elapsed / a.steps
        line = {
            "metric": "series-timesteps/sec forward-backward+Viterbi (K=4), host arrays to host arrays "
                      "(hhmm_run, the R .Call path)",
            "value": value,
            "unit": "series-timesteps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": step_s * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded HMM of hmm/main-multinom-semisup.R, Dirichlet-jittered draws), pageable "
                    "numpy arrays",
            "config": {"workload": f"C2-host hmm-multinom K=4 L=9, {P} pairs x T={T} per GPU (zip), "
                                   "gamma_tk zstar_t loglik logp_zstar, host to host",
                       "pairs_per_gpu": P, "T": T, "parallelism": f"pairs sharded over {world} GPU(s)"},
            "host_link": {"bytes_up": up, "bytes_down": down,
                          "pinned_GBps": {k: v / 1e9 for k, v in rates.items()},
                          "bound_ms": t_bound * 1e3,
                          "frac_of_link_bound": t_bound / step_s,
                          "end_to_end_GBps": (up + down) / step_s / 1e9,
                          "bound": "max(bytes_up / pinned H2D rate, bytes_down / pinned D2H rate, (bytes_up + "
                                   "bytes_down) / the aggregate rate of both directions at once): the transfers "
                                   "overlapped, at the rates torch's pinned copies reach on this host"},
            "one_chunk_ms": [t * 1e3 for t in one_chunk],
            "first_call_ms": first_s * 1e3,
            "bit_identical_to_device_entry": same,
            "library": lib.hhmm_version().decode(),
            "rank_ms_per_step": [v / a.steps * 1e3 for v in per_rank],
        }
        print(json.dumps(line), flush=True)


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ---------------------------------------------------------------------------
# The other BASELINE configs (evidence lines; C2 above is the metric)
# ---------------------------------------------------------------------------

WORKLOADS = {
    "c1": ("hmm", dict(N=1, S=1000, T=500, K=3), "grid",
           ["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
           lambda T, S: 3 * 8 + 4 + 8 / S + (8 * (3 + 9 + 3 + 3) + 16) / T,
           "C1 hmm Gaussian K=3 T=500, 1 series x 1000 draws (hmm/main.R), grid"),
    # name: (model, generator kwargs per GPU, pairing, outputs, algorithmic bytes per series-timestep
    #        (SURVEY.md §8d), description)
    "c3": ("iohmm-reg", dict(N=1250, S=4000, T=300, K=4, M=4), "grid",
           ["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
           lambda T, S: 32 + 4 + (8 + 32) / S + 320 / T,
           "C3 iohmm-reg K=4 M=4 T=300, 1250 series x 4000 draws per GPU (10k series / 8 GPUs), grid"),
    "c4": ("iohmm-hmix", dict(N=16, S=4096, T=10_000, K=4, L=3, M=4), "grid",
           ["loglik", "gamma_tk", "z_ffbs"],
           lambda T, S: 32 + 4 + 8 + (8 + 32) / S + 8 * (4 + 4 * 4 + 3 * 4 * 3) / T,
           "C4 iohmm-hmix K=4 L=3 M=4 T=10k, 16 series x 4096 draws, batched FFBS"),
    "n1": ("hmm-multinom", dict(N=1000, S=100, T=1000, K=23, L=9), "grid",
           ["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
           lambda T, S: 23 * 8 + 4 + 4 / S + 8 * (23 + 23 * 23 + 23 * 9) / T,
           "N1 hmm-multinom K=23 L=9 T=1000 (large-K state-parallel kernels), 1000 series x 100 draws, grid"),
    "n2": ("hmm-multinom", dict(N=1, S=250, T=1_000_000, K=23, L=9), "grid",
           ["loglik", "gamma_tk"],
           lambda T, S: 23 * 8 + 4 / S + (8 * (23 + 23 * 23 + 23 * 9) + 8) / T,
           "N2 hmm-multinom K=23 L=9 T=1e6, 1 series x 250 draws (a flattened-HHMM-sized state space over a long "
           "tick series): parallel scan over T with fp64 MFMA chunk products (hhmm_lkscan.h); forward-backward "
           "profile (loglik + gamma)"),
    "c5": ("hhmm-tayal2009", dict(N=1, S=250, T=1_000_000, L=9), "grid",
           ["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
           lambda T, S: 32 + 4 + 8 / S + (8 * (1 + 4 + 36) + 16) / T,
           "C5 tayal K=4 L=9 T=1e6, 1 series x 250 draws per GPU (8 series / 8 GPUs), "
           "parallel scan over T for the forward-backward"),
}


def prepare_other(a, lib, dev, rank):
    """The request of workload a.workload on resident device buffers: returns
    step() (one hhmm_run_device call on the current stream) and the shapes."""
    model, kw, pairing, pars, bps, desc = WORKLOADS[a.workload]
    kw = dict(kw)
    if a.pars:
        pars = a.pars.split(",")
        desc += f" [probe: outputs {a.pars}, flags {a.flags}]"
    data, draws = synth.GENERATORS[model](seed=a.seed + 7919 * rank, **kw)
    T = kw["T"]
    # the request's input pointers from the host mirror (outputs are device-only)
    host = hhmm_amd.api.PreparedRequest(model, data, draws, ["loglik"], pairing)
    req, res = host.req, host.res
    dmap = {}
    for arr in host.keep:
        dmap[arr.ctypes.data] = torch.from_numpy(np.asarray(arr).reshape(-1, order="F").copy()).to(dev)
    for struct in (req.data, req.draws):
        for name, ctype in struct._fields_:
            v = getattr(struct, name)
            if ctype is C.c_void_p and v and v in dmap:
                setattr(struct, name, dmap[v].data_ptr())
    P = host.P
    if "z_ffbs" in pars:
        dmap["u"] = torch.from_numpy(synth.ffbs_uniforms(P, T, seed=a.seed + rank).reshape(-1, order="F")).to(dev)
        req.ffbs_u = dmap["u"].data_ptr()
    req.outputs = 0
    req.flags = a.flags
    outs = {}
    shape = {"P": P, "PTK": P * T * int(data["K"] if "K" in data else 4), "PT": P * T, "PTz": P * T}
    for name in pars:
        dt, code = _abi.RESULT_ARRAYS[name]
        outs[name] = torch.empty(shape[code], dtype=torch.float64 if dt == "f64" else torch.int32, device=dev)
        req.outputs |= _abi.OUT[name]
        setattr(res, name, outs[name].data_ptr())
    status = torch.zeros(P, dtype=torch.int32, device=dev)
    res.pair_status = status.data_ptr()
    ws = C.c_size_t(0)
    assert lib.hhmm_workspace_size(C.byref(req), C.byref(ws)) == 0
    wsbuf = torch.empty(max(int(ws.value), 256), dtype=torch.uint8, device=dev)

    keep = (dmap, outs, status, wsbuf, host)

    def step():
        st = lib.hhmm_run_device(C.byref(req), C.byref(res), wsbuf.data_ptr(), wsbuf.numel(),
                                 torch.cuda.current_stream().cuda_stream)
        if st < 0:
            raise RuntimeError(lib.hhmm_last_error().decode())
        return keep

    return dict(step=step, model=model, kw=kw, pars=pars, bps=bps, desc=desc, data=data, draws=draws, P=P,
                T=T, outs=outs, status=status, req=req)


F64_PEAK = 78.6e12      # FLOP/s, MI355X fp64 vector and fp64 matrix (dense) peak
VALU_ISSUE = 1024 * 2.4e9 / 4.0  # wave-instructions/s: 1024 SIMDs x 2.4 GHz, 4 cycles per fp64-rate VALU op


def load_workload_pmc(name, src):
    """Per-step PMC totals of workload `name` (tools/pmc_workloads.sh ->
    tools/workload_pmc.py -> profiles/bench_traffic.json["workloads"]) when
    they were measured on the library build now loaded (`src`); else {} with
    the reason in "source"."""
    try:
        bt = json.loads((ROOT / "profiles" / "bench_traffic.json").read_text())
        pm = bt.get("workloads", {}).get(name, {}) or {}
    except Exception:
        return {"source": "no profiles/bench_traffic.json"}
    if not pm:
        return {"source": f"no PMC pass of workload {name}"}
    if pm.get("src") != src:
        return {"source": f"{pm.get('source')} measured build src {pm.get('src')}, the loaded library is src {src}"}
    return dict(pm, source=f"{pm.get('source')} (build src {src})")


def compute_rooflines(name, B, units, dev_ms, src, algo_flops=None):
    """HBM roofline of the whole request (algorithmic bytes over the live
    duration) beside the VALU and, where the request uses the matrix cores,
    the f64-MFMA ones: the committed PMC instruction counts per step over the
    same live duration.  `bound` names the larger fraction."""
    t = dev_ms * 1e-3
    pm = load_workload_pmc(name, src)
    hbm_frac = B * units / t / HBM_PEAK
    r = {"kernel": "whole request", "bound": "hbm", "achieved": B * units / t / 1e9, "peak": HBM_PEAK / 1e9,
         "unit": "GB/s", "frac": hbm_frac, "traffic": pm.get("hbm_bytes_per_step"),
         "algorithmic_bytes_per_series_timestep": B, "duration_ms": dev_ms, "pmc_source": pm.get("source")}
    vi = pm.get("valu_insts_per_step")
    if vi:
        r["valu_insts_per_step"] = vi
        r["valu_frac"] = vi / t / VALU_ISSUE
        r["valu_frac_definition"] = ("SQ_INSTS_VALU per step x 4 cycles / (1024 SIMDs x 2.4 GHz x live step "
                                     "time); every VALU op priced at the fp64 issue rate")
    mi = pm.get("mfma_f64_insts_per_step")
    mo = pm.get("mfma_f64_mops_per_step")
    if mo:
        # round 5: the chunk products issue v_mfma_f64_4x4x4_16b (512 FLOP per instruction), so the
        # FLOPs come from the MOPS counter (512 FLOP units) rather than instructions x 2048
        r["mfma_f64_insts_per_step"] = mi
        r["mfma_f64_mops_per_step"] = mo
        r["mfma_frac"] = mo * 512.0 / t / F64_PEAK
        r["mfma_frac_definition"] = ("f64 MFMA work per step (PMC SQ_INSTS_VALU_MFMA_MOPS_F64, units of 512 FLOP) "
                                     "x 512 / live step time / 78.6 TFLOP/s")
    elif mi:
        r["mfma_f64_insts_per_step"] = mi
        r["mfma_frac"] = mi * 2048.0 / t / F64_PEAK
        r["mfma_frac_definition"] = ("v_mfma_f64_16x16x4_f64 instructions per step (PMC SQ_INSTS_VALU_MFMA_F64) x "
                                     "2048 FLOP / live step time / 78.6 TFLOP/s")
    if algo_flops:
        r["algorithmic_flops_per_step"] = algo_flops
        r["algorithmic_mfma_frac"] = algo_flops / t / F64_PEAK
    cands = {"hbm": hbm_frac, "valu": r.get("valu_frac", 0.0), "mfma": r.get("mfma_frac", 0.0)}
    r["bound"] = max(cands, key=cands.get)
    return r


def other_workload(a, lib, rk):
    """C3 / C4 / C5: one request per step through hhmm_run_device on resident
    device buffers (synthetic inputs from hhmm_amd.synth, copied once)."""
    world, rank, dev = rk.world, rk.rank, rk.dev
    w = prepare_other(a, lib, dev, rank)
    run1, model, kw, pars, bps, desc = w["step"], w["model"], w["kw"], w["pars"], w["bps"], w["desc"]
    data, draws, P, T, status = w["data"], w["draws"], w["P"], w["T"], w["status"]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def step(i):
        if i == 0:
            ev[0].record()
        run1()
        if i == a.steps - 1:
            ev[1].record()

    _, elapsed, per_rank = timed_region(rk, step, a.steps, a.warmup)
    dev_ms = ev[0].elapsed_time(ev[1]) / a.steps
    units = P * T
    B = bps(T, kw["S"])
    sequential = None
    if a.workload == "n2" and not a.no_sequential:
        # after the timed region, once: the same request on the sequential
        # state-parallel kernels (HHMM_FLAG_SCAN_OFF), what the scan replaces
        req = w["req"]
        keep_flags = req.flags
        req.flags = keep_flags | _abi.FLAG_SCAN_OFF
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run1()
        e1.record()
        torch.cuda.synchronize()
        req.flags = keep_flags
        sequential = {"ms": e0.elapsed_time(e1), "flags": "HHMM_FLAG_SCAN_OFF (lk_fb_kernel, one 32-lane group per pair)",
                      "scan_speedup": e0.elapsed_time(e1) / dev_ms}
    if rank == 0:
        line = {
            "metric": "series-timesteps/sec (SURVEY §8d config) -- evidence line, not the headline",
            "value": world * units * a.steps / elapsed, "unit": "series-timesteps/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (hhmm_amd.synth generators, seeded)",
            "config": {"workload": desc, "model": model, "pairs_per_gpu": P, "T": T, "outputs": pars},
            "roofline": compute_rooflines(a.workload, B, units, dev_ms, lib_src(lib),
                                          algo_flops=(2.0 * kw["K"] ** 3 * units if a.workload == "n2" else None)),
            "library": lib.hhmm_version().decode(),
            "rank_ms_per_step": [x / a.steps * 1e3 for x in per_rank],
            "pair_failures": int((status != 0).sum().item()),
        }
        if sequential:
            line["sequential_after_timing"] = sequential
        if not a.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline_grid(model, data, draws, pars, T, a.cpu_seconds, a.seed)
        print(json.dumps(line), flush=True)


def cpu_baseline_grid(model, data, draws, pars, T, target_s, seed):
    """The oracle (libm build) on a bounded number of the workload's draws of
    its first series (same T and shapes), all the process's cores."""
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    xkey = "x_t" if model.startswith("iohmm") else "x"
    d1 = {k: (np.asarray(v)[:1] if k in ("x", "x_t", "g", "sign", "u_tm") else v) for k, v in data.items()}
    S = next(np.asarray(v).shape[0] for v in draws.values())
    assert np.asarray(d1[xkey]).shape[0] == 1

    def gen(n, off):
        n = min(n, S)
        dr = {k: np.asarray(v)[:n] for k, v in draws.items()}
        u = synth.ffbs_uniforms(n, T, seed=seed + off) if "z_ffbs" in pars else None
        return d1, dr, n, T, u

    v, P, _, dt = timed_oracle(model, gen, pars, "grid", threads, target_s, threads, S)
    return {"value": v, "unit": "series-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{P} draws x 1 series x T={T} ({model}, outputs {','.join(pars)}), {dt:.1f} s on "
                      f"{threads} threads, oracle libm-log build", "cpu_model": cpu_model()}


def features_workload(a, lib, rk):
    """F1: extract_features (tayal2009/R/feature-extraction.R:8-133) over a
    synthetic tick series resident in HBM; one step = the whole pipeline
    (change points, compaction, per-leg rows and features) through
    hhmm_extract_features_device.  Weak scaling: every rank owns its own ticks."""
    world, rank, dev = rk.world, rk.rank, rk.dev
    from hhmm_amd import features as F
    F.declare(lib)
    n = a.ticks
    price, size, tm = F.synth_ticks(n, seed=a.seed + 7919 * rank)
    dp, ds, dt = (torch.from_numpy(v).to(dev) for v in (price, size, tm))
    cols = {k: torch.empty(n, dtype=torch.float64 if t == "f64" else torch.int32, device=dev)
            for k, t in F.COLUMNS.items()}
    tk = F.Ticks(n, dp.data_ptr(), ds.data_ptr(), dt.data_ptr(), 0.25)
    legs = F.Legs(n, 0, *[cols[k].data_ptr() for k in F.COLUMNS])
    wsb = C.c_size_t(0)
    assert lib.hhmm_features_workspace_size(n, C.byref(wsb)) == 0
    ws = torch.empty(int(wsb.value), dtype=torch.uint8, device=dev)

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def step(i):
        if i == 0:
            ev[0].record()
        st = lib.hhmm_extract_features_device(C.byref(tk), C.byref(legs), ws.data_ptr(), ws.numel(),
                                              torch.cuda.current_stream().cuda_stream)
        if st < 0:
            raise RuntimeError(lib.hhmm_last_error().decode())
        if i == a.steps - 1:
            ev[1].record()

    _, elapsed, per_rank = timed_region(rk, step, a.steps, a.warmup)
    dev_ms = ev[0].elapsed_time(ev[1]) / a.steps
    m = int(legs.n_legs)
    # algorithmic bytes: price + size per tick; per leg the two index times and 52 B of leg columns
    B = 16.0 * n + 68.0 * m
    if rank == 0:
        line = {
            "metric": "ticks/sec, tick -> zig-zag -> leg features (SURVEY §8 F1) -- evidence line, not the headline",
            "value": world * n * a.steps / elapsed, "unit": "ticks/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic ticks (hhmm_amd.features.synth_ticks: 1-cent random walk, board lots, "
                    "exponential gaps)",
            "config": {"workload": f"F1 extract_features alpha=0.25, {n} ticks per GPU", "ticks_per_gpu": n,
                       "legs": m},
            "roofline": {"kernel": "whole pipeline (5 kernels)", "bound": "hbm",
                         "achieved": B / (dev_ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": B / (dev_ms * 1e-3) / HBM_PEAK, "traffic": None,
                         "algorithmic_bytes_per_tick": B / n, "duration_ms": dev_ms},
        }
        if not a.no_cpu_baseline and world == 1:
            sys.path.insert(0, str(ROOT / "oracle"))
            import pyoracle
            ns = min(n, 20_000_000)
            t1 = time.perf_counter()
            pyoracle.extract_features(price[:ns], size[:ns], tm[:ns])
            cs = time.perf_counter() - t1
            line["cpu_baseline"] = {"value": ns / cs, "unit": "ticks/s", "cores": 1, "kind": "port",
                                    "sample": f"first {ns} ticks of the same series, sequential C oracle "
                                              f"(oracle/features_oracle.c), {cs:.1f} s"}
        print(json.dumps(line), flush=True)


def check_slice(run, x, draws, P, T):
    """Compares 64 pairs of the data the timed steps ran on (the first 32 and
    32 spread over the batch) with the oracle, outside the timed region (test
    infrastructure; raises on a mismatch)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import pyoracle
    from tolerances import compare
    idx = np.unique(np.concatenate([np.arange(min(32, P)), np.linspace(0, P - 1, 32).astype(np.int64)]))
    ii = torch.as_tensor(idx, device=x.device)
    data = {"K": K, "L": L, "x": x[:, ii].T.cpu().numpy()}
    dr = {k: v[..., ii].permute(*reversed(range(v.dim()))).cpu().numpy() for k, v in draws.items()}
    dr["p_1k"] = dr["p_1k"][:, 0, :]
    ref = pyoracle.gqs("hmm-multinom", data, dr, pars=["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
                       pairing="zip", nthreads=8)
    got = {
        "loglik": run.out["loglik"][ii].cpu().numpy(),
        "logp_zstar": run.out["logp_zstar"][ii].cpu().numpy(),
        "zstar_t": run.out["zstar_t"][:, ii].T.cpu().numpy(),
        "gamma_tk": run.out["gamma_tk"][:, :, ii].permute(2, 1, 0).cpu().numpy(),
    }
    for k in got:
        compare(k, got[k], ref[k])
    msg = f"{idx.size} pairs of the timed batch match the oracle (loglik, gamma_tk, zstar_t, logp_zstar)"
    print("check:", msg, file=sys.stderr, flush=True)
    return msg


if __name__ == "__main__":
    main()
