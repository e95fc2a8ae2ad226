"""Data-parallel path sharding/reduction on CPU (gloo, 2 ranks) — the same code
paths as RCCL on MI355X, minus the device."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from rphedge.config import ParityFlags, RunConfig, TrainingParams

    tr = TrainingParams(batch_size=2048, epochs_first=6, epochs_rest=3, early_stopping=True, patience_first=3,
                        patience_rest=2, q99=True, lr_schedule_first=False, shuffle=False, lr=5e-3)
    return RunConfig(Y=1.0, K=1.0, T=2.0, mu=0.08, r=0.03, sigma=0.15, rebalancing=0.5, dt=0.05, n_paths=11,
                     N=10000, P=100, verbose=False, train=tr, parity=ParityFlags(), device="cpu", backend="torch")


def _worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from rphedge import risk
    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    di = D.init(device="cpu")
    run = HedgeRun(_cfg(), dist_info=di)
    res = run.run()
    q = risk.quantile(res.induction.residuals, (0.5, 0.99), world)
    vals = res.induction.values.detach().numpy()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"phi": res.phi, "psi": res.psi, "v0": res.v0, "q": q.tolist(),
                       "epochs": res.summary["epochs_mse"], "pnl": res.terminal_pnl}, f)
    np.save(out + f".values{rank}.npy", vals)
    D.shutdown()


def test_dp_two_ranks_matches_single_process():
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res.json")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
            assert p.exitcode == 0
        dp = json.load(open(out))
        v_dp = np.concatenate([np.load(out + f".values{r}.npy") for r in range(world)], axis=1)

    from rphedge import risk
    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    run = HedgeRun(_cfg(), dist_info=D.DistInfo(device=torch.device("cpu")))
    ref = run.run()
    v_ref = ref.induction.values.detach().numpy()
    # batch=2048 of 2048 paths: full-batch GD, so the DP gradient is the 1-rank gradient
    assert dp["epochs"] == ref.summary["epochs_mse"]          # identical early-stop decisions on all ranks
    np.testing.assert_allclose(v_dp, v_ref, rtol=2e-4, atol=2e-5)
    assert dp["phi"] == pytest.approx(ref.phi, rel=1e-3)
    assert dp["psi"] == pytest.approx(ref.psi, rel=1e-3)
    q_ref = risk.quantile(ref.induction.residuals, (0.5, 0.99))
    np.testing.assert_allclose(dp["q"], q_ref, rtol=1e-3, atol=1e-6)


def test_shard_ranges():
    from rphedge.parallel.dist import shard

    assert [shard(1 << 20, 8, r) for r in (0, 7)] == [(0, 131072), (917504, 131072)]
    with pytest.raises(ValueError):
        shard(10, 3, 0)


def _dying_worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import time

    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    di = D.init(device="cpu", timeout_s=20.0)
    if rank == 1:
        os._exit(3)  # fault injection: a rank dies before the first collective of the run
    t0 = time.time()
    try:
        HedgeRun(_cfg(), dist_info=di).run()
        status = "completed"
    except Exception as e:  # gloo: peer closed / timeout
        status = "raised: " + type(e).__name__
    with open(out, "w") as f:
        json.dump({"status": status, "elapsed": time.time() - t0}, f)
    os._exit(0)  # (the process group cannot be shut down cleanly without its peer)


def test_dead_rank_errors_out_cleanly():
    """SURVEY §5.3 fault injection: a rank killed before a collective makes the
    surviving rank raise (bounded by the process-group timeout) instead of
    hanging or returning a silently wrong result."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "dead.json")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_dying_worker, args=(r, world, port, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        assert procs[1].exitcode == 3
        assert procs[0].exitcode == 0
        res = json.load(open(out))
    assert res["status"].startswith("raised"), res
    assert res["elapsed"] < 60


def _params(save_dir):
    from rphedge.experiments import mts_parameters

    return mts_parameters(n_paths=10, dt=0.1, rebalancing=1.0, epochs_first=8, epochs_rest=3, verbose=True,
                          device="cpu", save_dir=save_dir, batch_size=1024, shuffle=False)


def _verbose_save_resume_worker(rank, world, port, out, save_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from rphedge.api import HedgeRun, run_params
    from rphedge.config import parse_params
    from rphedge.parallel import dist as D

    D.init(device="cpu", timeout_s=60.0)
    res = run_params(_params(save_dir))          # verbose: per-date quantiles are collectives on every rank
    run = HedgeRun(parse_params(_params(None)))
    r2 = run.resume(save_dir, 5)                 # restart at date 4 from the gathered values.npy
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"phi": res.phi, "psi": res.psi, "resumed_phi": r2.phi}, f)
    D.shutdown()


def test_dp_verbose_save_and_resume_two_ranks():
    """verbose per-date reports run their distributed quantiles on
    every rank (no rank-0-only collective), values.npy holds every rank's
    shard, and a data-parallel resume trains each rank on its own shard: the
    2-rank resume equals the 1-process resume of the same saved run."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res.json")
        save = os.path.join(td, "run")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_verbose_save_resume_worker, args=(r, world, port, out, save))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
            assert p.exitcode == 0
        dp = json.load(open(out))
        vals = np.load(os.path.join(save, "values.npy"))
        assert vals.shape[1] == 1 << 10            # gathered: both shards
        from rphedge.api import HedgeRun
        from rphedge.config import parse_params
        from rphedge.parallel import dist as D

        run = HedgeRun(parse_params(_params(None)), dist_info=D.DistInfo(device=torch.device("cpu")))
        r1 = run.resume(save, 5)
    assert dp["resumed_phi"] == pytest.approx(r1.phi, rel=2e-3)


def _lm_cfg(out_fix=False):
    from rphedge.config import ParityFlags, RunConfig, TrainingParams

    tr = TrainingParams(batch_size=2048, early_stopping=False, q99=False, optimizer="lm", lm_passes_first=15,
                        lm_passes_rest=2, lm_gram_paths=2048, lm_out_fix=out_fix)
    return RunConfig(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=0.25, dt=0.25, n_paths=11,
                     payoff="call", option_type="CALL", model="gbm_log", mortality=False, N=1, P=1.0,
                     verbose=False, train=tr, parity=ParityFlags(), device="cpu", backend="torch")


def _lm_worker(rank, world, port, out, out_fix=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    di = D.init(device="cpu")
    run = HedgeRun(_lm_cfg(out_fix), dist_info=di)
    res = run.run()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"phi": res.phi, "v0": res.v0, "pnl": res.terminal_pnl["std"],
                       "out_dl": float(getattr(run.backend, "lm_out_dl", 0.0))}, f)
    D.shutdown()


@pytest.mark.parametrize("out_fix", [False, True])
def test_dp_lm_two_ranks_matches_single_process(out_fix):
    """Levenberg-Marquardt fits data parallel: the per-pass reduced block
    [G | g | stats] is all-reduced, and with the Gram subsample covering every
    path the 2-rank fit is the 1-process fit.  out_fix: the final
    output-layer Newton step's full-batch output Gram matrix is all-reduced
    too (its step predicts the same loss drop on both sides)."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "lm.json")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_lm_worker, args=(r, world, port, out, out_fix)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
            assert p.exitcode == 0
        dp = json.load(open(out))
    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    run = HedgeRun(_lm_cfg(out_fix), dist_info=D.DistInfo(device=torch.device("cpu")))
    ref = run.run()
    if out_fix:
        assert dp["out_dl"] == pytest.approx(run.backend.lm_out_dl, rel=1e-4, abs=1e-12)
    assert dp["phi"] == pytest.approx(ref.phi, rel=1e-5)
    assert dp["v0"] == pytest.approx(ref.v0, rel=1e-5)
    assert dp["pnl"] == pytest.approx(ref.terminal_pnl["std"], rel=1e-4)


def _ms_cfg():
    c = _lm_cfg()
    c.train.lm_starts, c.train.lm_explore_passes, c.train.lm_explore_log2 = 3, 6, 9
    c.train.lm_passes_first, c.train.lm_lam_carry = 4, 3.0
    return c


def _ms_worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    di = D.init(device="cpu")
    run = HedgeRun(_ms_cfg(), dist_info=di)
    res = run.run()
    x = run.backend.lm_explore_last
    with open(out + f".{rank}", "w") as f:
        json.dump({"phi": res.phi, "v0": res.v0, "losses": x["losses"], "pick": x["pick"]}, f)
    D.shutdown()


def test_dp_lm_multistart_two_ranks():
    """Multi-start exploration data parallel: every rank explores the SAME
    starts on the same global path prefix (simulated on every rank, no
    exchange) and continues from the same winner - the candidates, their
    losses and the pick are exactly those of the one-process run (the
    exploration does not depend on the world size)."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "ms.json")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_ms_worker, args=(r, world, port, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
            assert p.exitcode == 0
        r0, r1 = (json.load(open(out + f".{r}")) for r in range(world))
    assert r0 == r1                                  # same candidates, same pick, same result on both ranks
    assert len(r0["losses"]) == 3
    ls = np.where(np.isnan(r0["losses"]), np.inf, r0["losses"])
    assert r0["pick"] == int(np.argmin(ls))
    from rphedge.api import HedgeRun
    from rphedge.parallel import dist as D

    run = HedgeRun(_ms_cfg(), dist_info=D.DistInfo(device=torch.device("cpu")))
    res = run.run()
    x = run.backend.lm_explore_last
    assert x["losses"] == r0["losses"] and x["pick"] == r0["pick"]
    assert res.v0 == pytest.approx(r0["v0"], rel=1e-5)


def _pin_params():
    from rphedge import experiments

    return experiments.mts_lm_parameters(n_paths=11, dt=0.25, rebalancing=1.0, T=4, device="cpu", backend="torch",
                                         verbose=False, lm_starts=1, lm_explore_passes=0, lm_passes_first=10,
                                         lm_passes_rest=2, lm_q_passes_first=8, lm_q_passes_rest=3,
                                         lm_gram_paths=1024, concurrent_q99=False)


def _pin_worker(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.parallel import dist as D

    di = D.init(device="cpu")
    run = HedgeRun(parse_params(_pin_params()), dist_info=di)
    res = run.run()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"phi": res.phi, "psi": res.psi, "v0": res.v0}, f)
    D.shutdown()


def test_dp_pinball_lm_two_ranks_matches_single_process():
    """Both fits on LM (pension, two networks) on 2 gloo ranks: the pinball
    fits' IRLS Gram is built on the simulated global subsample with its own
    targets (DateData.gram_target, evaluated at every date boundary), so only
    the gradient region is all-reduced and the 2-rank run is the 1-process
    run (torch oracle; RP:138-145, :217-221)."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "pin.json")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_pin_worker, args=(r, world, port, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        dp = json.load(open(out))
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.parallel import dist as D

    run = HedgeRun(parse_params(_pin_params()), dist_info=D.DistInfo(device=torch.device("cpu")))
    assert run.build().induction.gvalues is not None   # the subsample carries its targets
    ref = run.run()
    for k in ("phi", "psi", "v0"):
        assert dp[k] == pytest.approx(getattr(ref, k), rel=1e-5), (k, dp[k], getattr(ref, k))
