"""CPU: bench.py's multi-rank launcher and timing harness (no GPU).

`bench.py --gpus 2 --stub` without a launcher must start two ranks under
torch.distributed.run (gloo), time exactly K steps on each, take the max over
ranks and print one JSON line with n_gpus == 2; a launcher whose world size
differs from --gpus must fail loudly instead of measuring fewer GPUs."""
import json
import os
import pathlib
import subprocess
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_two_launches_two_ranks():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--stub", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["warmup"] == 1
    assert len(line["rank_ms_per_step"]) == 2
    assert abs(line["ms_per_step"] - max(line["rank_ms_per_step"])) < 1e-9
    # the per-step all-reduce ran over both ranks: rank 0 holds the sum of two positive terms
    assert line["all_reduce_check"] > 0


def test_gpus_one_is_a_single_process():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "1", "--stub", "--steps", "2",
                        "--warmup", "0"], capture_output=True, text=True, env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1 and len(line["rank_ms_per_step"]) == 1


def test_world_size_mismatch_fails_loudly():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--stub", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_c2_line_finds_its_pmc_traffic(tmp_path, monkeypatch):
    """The C2 line's roofline.traffic comes from the PMC record of its dominant
    kernel only when that record was taken at the bench shape AND on the
    library build now loaded (evidence keyed to the build); otherwise
    it is null with the reason.  The committed record keeps the shape keys (a
    record without them silently gave traffic = null)."""
    sys.path.insert(0, str(REPO))
    import bench
    dom = bench.SCHEDULE_KERNELS[bench.DEFAULT_SCHEDULE][0]
    committed = json.loads((REPO / "profiles" / "bench_traffic.json").read_text())
    assert committed.get("pairs") == 1_000_000 and committed.get("T") == 1000
    assert dom in committed.get("kernels", {}), dom
    (tmp_path / "profiles").mkdir()
    rec = dict(committed, src="00112233aabbccdd")
    (tmp_path / "profiles" / "bench_traffic.json").write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    t, note = bench.load_traffic(dom, 1_000_000, 1000, "00112233aabbccdd")
    assert t is not None and 40.0e9 < t < 60.0e9, (dom, t, note)
    t, note = bench.load_traffic(dom, 1_000_000, 1000, "ffffffffffffffff")
    assert t is None and "00112233aabbccdd" in note, note
    t, note = bench.load_traffic(dom, 1_000, 1000, "00112233aabbccdd")
    assert t is None and "shape" in note, note


def test_mfma_fraction_counts_flops_not_instructions(monkeypatch):
    """roofline.mfma_frac prices the f64 MFMA work by the MOPS counter (512-FLOP
    units): N2's chunk products issue v_mfma_f64_4x4x4_16b (512 FLOP each), so
    instructions x 2048 -- the 16x16x4 rule -- would report 4x the work."""
    sys.path.insert(0, str(REPO))
    import bench
    pm = {"source": "test", "src": "s", "hbm_bytes_per_step": 1.0e9, "valu_insts_per_step": 1.0e9,
          "mfma_f64_insts_per_step": 1.0e10, "mfma_f64_mops_per_step": 1.0e10}
    monkeypatch.setattr(bench, "load_workload_pmc", lambda name, src: pm)
    r = bench.compute_rooflines("n2", 184.0, 2.5e8, 100.0, "s", algo_flops=5.0e12)
    assert abs(r["mfma_frac"] - 1.0e10 * 512 / 0.1 / bench.F64_PEAK) < 1e-12
    assert r["mfma_frac"] <= 1.0
    # a 16x16x4 build: 4 MOPS per instruction, the same FLOPs either way
    pm.update(mfma_f64_insts_per_step=2.5e9)
    assert abs(bench.compute_rooflines("n2", 184.0, 2.5e8, 100.0, "s")["mfma_frac"] - r["mfma_frac"]) < 1e-12
