"""bench.py driver contract (CPU plumbing preset, 1 and 4 gloo ranks) and the
closed-form quality anchors (rphedge.analytic)."""
import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def test_heston_reduces_to_black_scholes():
    from rphedge.analytic import black_scholes, heston_call

    p, d = heston_call(100.0, 100.0, 0.08, 1.0, 2.0, 0.0225, 1e-4, -0.7, 0.0225)
    bs, bd = black_scholes(100.0, 100.0, 0.08, 0.15, 1.0)
    assert p == pytest.approx(bs, abs=2e-3)
    assert d == pytest.approx(bd, abs=1e-3)


def test_heston_literature_value():
    """Albrecher et al. benchmark: S0=K=100, T=1, r=0, kappa=1.5768, theta=0.0398,
    xi=0.5751, rho=-0.5711, v0=0.0175 -> 5.785155."""
    from rphedge.analytic import heston_call, heston_price

    p, _ = heston_call(100.0, 100.0, 0.0, 1.0, 1.5768, 0.0398, 0.5751, -0.5711, 0.0175)
    assert p == pytest.approx(5.785155, abs=1e-4)
    put, _ = heston_price(100.0, 110.0, 0.05, 1.0, 2.0, 0.04, 0.5, -0.7, 0.04, "PUT")
    call, _ = heston_call(100.0, 110.0, 0.05, 1.0, 2.0, 0.04, 0.5, -0.7, 0.04)
    assert put == pytest.approx(call - 100.0 + 110.0 * math.exp(-0.05), abs=1e-9)  # put-call parity


def _bench(args, env=None, nproc=1, bare=False):
    e = dict(os.environ, **(env or {}))
    e.setdefault("OMP_NUM_THREADS", "1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    if nproc == 1 or bare:
        cmd = [sys.executable, "bench.py"] + (["--gpus", str(nproc)] if bare else []) + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(29531 + nproc), "bench.py", "--gpus", str(nproc)] + args
    out = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_cpu_preset_contract():
    r = _bench(["--preset", "euro1_cpu", "--steps", "1", "--warmup", "0", "--epochs-first", "20"])
    assert KEYS <= set(r)
    assert r["n_gpus"] == 1 and r["steps"] == 1 and r["higher_is_better"] is True and r["scaling"] == "weak"
    assert r["config"]["preset"] == "euro1_cpu" and r["config"]["parallelism"] == "dp1"
    assert r["value"] > 0 and r["vs_baseline"] == pytest.approx(r["value"] / (4096.0 / ((500 + 29 * 904 / 51) * 0.048)))
    assert r["path_samples_per_s"] == pytest.approx(r["value"] * r["full_passes_per_run"])
    assert r["quality"]["anchor"]["analytic"] == "black_scholes"


@pytest.mark.parametrize("nproc", [4, 8])
def test_bench_cpu_multi_rank(nproc):
    """--gpus N under torch.distributed.run (gloo on CPU; N=8 is the driver's
    scaling-node world size): weak scaling, the global batch and path count
    grow with the world size; rank 0 prints once."""
    r = _bench(["--preset", "euro1_cpu", "--steps", "1", "--warmup", "0", "--epochs-first", "10",
                "--paths-log2", "12", "--batch-log2", "10", "--cpu"], nproc=nproc)
    assert r["n_gpus"] == nproc and r["config"]["parallelism"] == f"dp{nproc}"
    assert r["config"]["paths_global"] == nproc * (1 << 12) and r["config"]["global_batch"] == nproc * (1 << 10)
    assert r["config"]["dist_world"] == nproc
    assert math.isfinite(r["quality"]["V0"]) and abs(r["quality"]["V0"] - 10.39) < 1.5


@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_bench_bare_gpus_self_launches(nproc):
    """``python bench.py --gpus N`` with no torch.distributed environment (the
    driver's scaling invocation) spawns the N ranks itself; the JSON line and
    its keys are the same as under an external torch.distributed.run."""
    args = ["--preset", "euro1_cpu", "--steps", "1", "--warmup", "0", "--epochs-first", "6",
            "--paths-log2", "11", "--batch-log2", "9", "--cpu"]
    r = _bench(args, nproc=nproc, bare=True)
    assert r["n_gpus"] == nproc and r["config"]["dist_world"] == nproc
    assert r["config"]["paths_global"] == nproc * (1 << 11)
    if nproc == 4:
        t = _bench(args, nproc=nproc)
        assert set(r) == set(t) and set(r["config"]) == set(t["config"]) and set(r["quality"]) == set(t["quality"])
        assert r["quality"]["V0"] == t["quality"]["V0"]  # same global paths, same ranks: same result


@pytest.mark.gpu
def test_bench_bare_two_ranks_one_gpu_lm():
    """The driver's scaling invocation on the GPU path, rehearsed with two
    ranks sharing one card: self-launch, the transport probe (Adam packet AND
    LM reduced-block exchanges over the IPC mailboxes) picks xgmi, the default
    LM preset runs data parallel, and the result is the 2-rank fit of the
    doubled global path set (V0 on the BS price)."""
    r = _bench(["--steps", "1", "--warmup", "1", "--paths-log2", "16", "--lm-passes-first", "30"],
               nproc=2, bare=True)
    c = r["config"]
    assert r["n_gpus"] == 2 and c["dist_world"] == 2 and c["optimizer"] == "lm" and c["backend"] == "hip"
    clean = {"local_ok": True, "all_ok": True, "bitwise_equal_weights": True, "chosen": "xgmi", "clean": True}
    pk, lm = c["dp_probe"]["packet"], c["dp_probe"]["lm"]
    assert {k: pk.get(k) for k in clean} == clean and {k: lm.get(k) for k in clean} == clean, c["dp_probe"]
    # the LM probe ran the production exchange (summed inside k_lm_reduce) and
    # matched the same fit over an independent all-reduce
    assert lm["fused"] is True and lm["max_rel_dev_vs_allreduce"] <= lm["rtol"], lm
    assert c["dp_transport"] == "xgmi" and c["lm_dp_transport"] == "xgmi" and c["paths_global"] == 2 << 16
    assert abs(r["quality"]["V0"] - 10.3896) < 0.1, r["quality"]
    assert math.isfinite(r["quality"]["terminal_pnl_std"]) and r["quality"]["terminal_pnl_std"] < 3.5  # 2^17 paths, 30 passes: 2.57 measured


def test_heston_greeks_match_quadrature_and_finite_differences():
    """Per-path Heston greeks (the hedge anchor's engine) vs the scalar
    quadrature price / delta at ordinary points and a central finite
    difference of the price in v; near maturity at small variance vs a
    high-resolution quadrature (umax 20000)."""
    import torch

    from rphedge import analytic as A

    k = dict(kappa=2.0, theta=0.04, xi=0.5, rho=-0.7)
    r = 0.05
    for S, v, tau in [(1.0, 0.04, 1.0), (0.9, 0.09, 0.5), (0.97, 0.04, 1 / 30)]:
        p_ref, d_ref = A.heston_call(S, 1.0, r, tau, k["kappa"], k["theta"], k["xi"], k["rho"], v)
        h = 1e-5
        up = A.heston_call(S, 1.0, r, tau, k["kappa"], k["theta"], k["xi"], k["rho"], v + h)[0]
        dn = A.heston_call(S, 1.0, r, tau, k["kappa"], k["theta"], k["xi"], k["rho"], v - h)[0]
        p, d, cv = A.heston_greeks(torch.tensor([S]), torch.tensor([v]), 1.0, r, tau, **k)
        assert p.item() == pytest.approx(p_ref, abs=2e-8)
        assert d.item() == pytest.approx(d_ref, abs=2e-6)
        assert cv.item() == pytest.approx((up - dn) / (2 * h), rel=1e-3)
    # short maturity, tiny variance: the per-path scaled quadrature
    S, v, tau = 1.02, 5e-4, 1 / 30
    p1 = A._heston_p(1, S, 1.0, tau, k["kappa"], k["theta"], k["xi"], k["rho"], v, r, umax=20000, n=400001)
    _, d, _ = A.heston_greeks(torch.tensor([S]), torch.tensor([v]), 1.0, r, tau, **k)
    assert d.item() == pytest.approx(p1, abs=1e-5)


def test_heston_min_variance_hedge_beats_delta_on_paths():
    """On simulated Heston paths (rho = -0.7) the minimum-variance hedge
    Delta + (rho xi / S) dC/dv has a smaller self-financing P&L spread than
    the Heston delta hedge, both far below the unhedged payoff spread."""
    import torch

    from rphedge import analytic as A
    from rphedge.ops import paths as P

    T, nd, sub = 1.0, 12, 8
    g = P.Grid(T=T, dt=T / (nd * sub), rebalancing=T / nd)
    p = P.simulate_sv(g, 4096, 1.0, 0.05, 0.04, model="heston", kappa=2.0, theta=0.04, xi=0.5, rho=-0.7,
                      device="cpu")
    p.bond = g.bond(0.05)
    a = A.heston_hedge_anchor(p.S, p.vol, p.bond, 1.0, 0.05, T, g.times(), 2.0, 0.04, 0.5, -0.7, max_paths=4096)
    pay = (p.S[-1].double() - 1.0).clamp_min(0)
    assert a["min_variance"]["pnl_std"] < a["delta"]["pnl_std"] < 0.5 * float(pay.std())
    assert a["price"] == pytest.approx(A.heston_call(1.0, 1.0, 0.05, T, 2.0, 0.04, 0.5, -0.7, 0.04)[0], rel=1e-6)


def test_levy_basket_anchor():
    """Levy basket: a one-asset basket is Black-Scholes (price and delta);
    on a simulated 5-asset basket the per-asset delta hedge cuts the payoff
    spread by an order of magnitude."""
    import torch

    from rphedge import analytic as A
    from rphedge.ops import paths as P

    S = torch.tensor([[1.0, 1.1, 0.9]], dtype=torch.float64)
    c = A.levy_basket_call(S, [1.0], 1.0, 0.05, 0.2, 0.5, 0.5)
    for i, s in enumerate([1.0, 1.1, 0.9]):
        bs, _ = A.black_scholes(s, 1.0, 0.05, 0.2, 0.5, "CALL")
        assert c[i].item() == pytest.approx(bs, rel=1e-9)
    T, nd = 1.0, 24
    g = P.Grid(T=T, dt=T / nd, rebalancing=T / nd)
    na, rho = 5, 0.5
    corr = np.full((na, na), rho) + np.eye(na) * (1 - rho)
    p = P.simulate_basket(g, 4096, [1.0] * na, [0.05] * na, [0.2] * na, corr, device="cpu")
    p.bond = g.bond(0.05)
    w = [1.0 / na] * na
    a = A.basket_hedge_anchor(p.S, p.bond, w, 1.0, 0.05, 0.2, rho, T, g.times(), max_paths=4096)
    pay = ((torch.tensor(w, dtype=torch.float64)[:, None] * p.S[-1].double()).sum(0) - 1.0).clamp_min(0)
    assert a["levy_delta"]["pnl_std"] < 0.1 * float(pay.std())
    assert a["price"] == pytest.approx(float(pay.mean()) * math.exp(-0.05), rel=0.03)


def test_bench_lm_knobs_reach_the_backend():
    """--lm-ridge / --lm-out-mu travel bench -> TrainingParams -> the backend's
    TrainConfig (the defaults are the engine's: 1e-10 / 1e-5)."""
    sys.path.insert(0, ROOT)
    import bench
    from rphedge.api import HedgeRun

    a = bench.parse(["--preset", "euro1_cpu"])
    assert a.lm_ridge == 1e-10 and a.lm_out_mu == 1e-5
    a = bench.parse(["--preset", "euro1_cpu", "--optimizer", "lm", "--lm-ridge", "1e-6", "--lm-out-mu", "1e-3"])
    cfg = bench.build_run(a, 1)
    assert cfg.train.lm_ridge == 1e-6 and cfg.train.lm_out_mu == 1e-3
    run = HedgeRun(cfg).build()
    assert run.backend.tcfg.lm_ridge == 1e-6 and run.backend.tcfg.lm_out_mu == 1e-3
