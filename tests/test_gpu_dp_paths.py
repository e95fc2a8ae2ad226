"""Every data-parallel LM code path runs in a test on ONE GPU:

* the split LM sequence (pass + reduce -> RCCL all-reduce of the reduced
  [G | g | stats] block -> solve) with a 1-rank RCCL communicator, eager and
  hipGraph-captured, is bitwise the fused one-rank fit (engine.HipBackend._lm_fit;
  TrainConfig.lm_split is the hook);
* select_transport with an injected probe failure (RPH_PROBE_FAIL = packet |
  lm | both) picks the RCCL fallback for exactly that exchange and creates its
  communicator before any capture; the fallback sequence then reproduces the
  one-process fit (two ranks sharing the card: RCCL refuses two ranks on one
  GPU, so the communicator is a gloo stand-in with RCCL's allreduce_ contract);
* the 32-unit (MFMA) nets' mean refit is graph-capturable (no allocation
  inside the capture) and the captured run equals the eager one.

The reference has no parallelism at all (Replicating_Portfolio.py:61 holds
every path in one array); SURVEY §2.3 / §5.8."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(n, dev, lo=0, cnt=None):
    g = torch.Generator().manual_seed(17)
    x = torch.rand(n, generator=g) * 0.6 + 0.7
    cnt = n if cnt is None else cnt
    f = x[lo:lo + cnt].to(dev)
    return f, f * 1.01, torch.relu(f * 1.01 - 1.0) + 0.02 * torch.sin(9 * f)


def _lm_fit(be, spec, f, p1, y, passes, graph=False):
    from rphedge.engine import DateData, FitConfig, current_weights
    from rphedge.models.hedge_mlp import init_weights
    from rphedge.ops.native import Graph

    data = DateData(feats=[f], prices_next=[p1], bond_next=1.0, target=y, prices_now=[f])
    fc = FitConfig(epochs=passes, optimizer="lm", early_stopping=False)
    w0 = init_weights(spec, [0.5, 0.0])
    w, o, fs = be.new_weights(w0), be.new_opt(), be.new_fit()
    if not graph:
        be.fit(w, o, fs, data, fc, seed=0)
        torch.cuda.synchronize()
        return current_weights(spec, w), fs[2048 + 16:2048 + 16 + passes + 1].cpu().numpy()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        be.fit(w, o, fs, data, fc, seed=0)  # eager pass: caches every device constant
        s.synchronize()
        w.copy_(be.new_weights(w0))
        g = Graph()
        g.capture_begin(s)
        try:
            be.fit(w, o, fs, data, fc, seed=0)
        finally:
            g.capture_end()
        w.copy_(be.new_weights(w0))
        g.replay(s)
        s.synchronize()
    return current_weights(spec, w), fs[2048 + 16:2048 + 16 + passes + 1].cpu().numpy()


@pytest.mark.parametrize("graph", [False, True])
def test_lm_split_sequence_with_rccl_is_bitwise_fused(graph):
    """world = 1: lm_eval -> comm.allreduce_ (1-rank RCCL) -> lm_solve per
    pass == the fused rph_lm_fit, bit for bit, eager and captured."""
    import torch.distributed as dist  # noqa: F401
    from torch.distributed import HashStore

    from rphedge.engine import HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops.native import NcclComm

    dev = torch.device("cuda", 0)
    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 1 << 15
    f, p1, y = _problem(n, dev)
    comm = NcclComm(0, 1, HashStore(), tag="t_lm_split")
    try:
        tc = TrainConfig(batch_size=n, lm_gram_paths=2048)
        ref = _lm_fit(HipBackend(spec, n, tc, device=dev), spec, f, p1, y, 12, graph=graph)
        tcs = TrainConfig(batch_size=n, lm_gram_paths=2048, lm_split=True)
        got = _lm_fit(HipBackend(spec, n, tcs, device=dev, lm_comm=comm), spec, f, p1, y, 12, graph=graph)
    finally:
        comm.close()
    np.testing.assert_array_equal(got[0], ref[0])
    np.testing.assert_array_equal(got[1], ref[1])


def test_lm_split_without_transport_raises():
    """A split / data-parallel LM fit with neither a mailbox nor a communicator
    is refused before any launch (never a lazily created communicator)."""
    from rphedge.engine import HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec

    dev = torch.device("cuda", 0)
    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    n = 1 << 12
    f, p1, y = _problem(n, dev)
    be = HipBackend(spec, n, TrainConfig(batch_size=n, lm_split=True), device=dev)
    with pytest.raises(RuntimeError, match="select_transport"):
        _lm_fit(be, spec, f, p1, y, 2)


class _GlooComm:
    """Stand-in for the RCCL fallback communicator when two ranks share one
    GPU (RCCL refuses that): the same allreduce_(tensor, stream) contract,
    summed over gloo on the host (eager only)."""

    def __init__(self, rank, world, store, tag=""):
        self.rank, self.world = rank, world

    def allreduce_(self, t, stream=None):
        import torch.distributed as dist

        torch.cuda.synchronize()
        h = t.detach().cpu()
        dist.all_reduce(h)
        t.copy_(h.to(t.device))

    def close(self):
        pass


def _inject_worker(rank, world, port, inject, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world), RPH_PROBE_FAIL=inject)
    from rphedge.engine import HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops import native
    from rphedge.parallel import dist as D

    native.NcclComm = _GlooComm  # select_transport's fallback constructor
    info = D.init(device="cuda:0")
    D.select_transport(info)
    res = {"dp_mode": info.dp_mode, "lm_dp_mode": info.lm_dp_mode, "comm": info.comm is not None,
           "lm_comm": info.lm_comm is not None, "probe": {k: v["chosen"] for k, v in info.probe.items()}}
    dev = info.device
    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    per = n // world
    f, p1, y = _problem(n, dev, rank * per, per)
    from rphedge.ops import layout as L

    # the mailboxes api.HedgeRun.build would create for these transports
    mb = D.make_mailbox(info, spec.red_width, tag="t_inj_pk", mode=info.dp_mode)
    lmb = D.make_mailbox(info, L.LM_DP_PITCH, tag="t_inj_lm", mode=info.lm_dp_mode)
    be = HipBackend(spec, per, TrainConfig(batch_size=n, lm_gram_paths=2048), device=dev, world=world, rank=rank,
                    comm=info.comm, mailbox=mb, lm_mailbox=lmb, lm_comm=info.lm_comm)
    w, hist = _lm_fit(be, spec, f, p1, y, 8)
    np.save(out + f".{rank}.npy", w)
    import json

    with open(out + f".{rank}.json", "w") as fh:
        json.dump(res, fh)
    D.barrier()
    for m in (mb, lmb):
        if m is not None:
            m.close()
    D.shutdown()


@pytest.mark.parametrize("inject", ["packet", "lm", "both"])
def test_injected_probe_failure_selects_rccl_fallback(inject):
    import json

    from rphedge.engine import HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec

    n, world = 1 << 14, 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w")
        ctx = mp.get_context("spawn")
        port = _port()
        env_keep = dict(os.environ)
        procs = [ctx.Process(target=_inject_worker, args=(r, world, port, inject, n, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
        os.environ.clear()
        os.environ.update(env_keep)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res = [json.load(open(out + f".{r}.json")) for r in range(world)]
        ws = [np.load(out + f".{r}.npy") for r in range(world)]
    for r in res:
        assert r["probe"]["packet"] == ("rccl" if inject in ("packet", "both") else "xgmi"), r
        assert r["probe"]["lm"] == ("rccl" if inject in ("lm", "both") else "xgmi"), r
        if inject in ("packet", "both"):   # one communicator serves both exchanges
            assert r["dp_mode"] == "rccl" and r["comm"], r
        else:
            assert r["dp_mode"] == "xgmi" and r["lm_dp_mode"] == "rccl" and r["lm_comm"], r
    np.testing.assert_array_equal(ws[0], ws[1])
    # the same global path set on one process
    dev = torch.device("cuda", 0)
    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    f, p1, y = _problem(n, dev)
    w1, _ = _lm_fit(HipBackend(spec, n, TrainConfig(batch_size=n, lm_gram_paths=2048), device=dev), spec, f, p1,
                    y, 8)
    np.testing.assert_allclose(ws[0], w1, rtol=2e-4, atol=2e-6)


def test_mfma_net_mean_refit_graph_capture_matches_eager():
    """hidden = 32 (no LM solver): the mean refit after each Adam fit runs from
    preallocated buffers, so the whole induction captures into one hipGraph
    (round-2 advisor: it used to fall back to eager launches silently); the
    replay reproduces the eager run (float-atomic step kernels: to rounding)."""
    import bench
    from rphedge.api import HedgeRun

    a = bench.parse(["--preset", "euro30_mfma", "--paths-log2", "15", "--batch-log2", "13", "--dates", "6",
                     "--epochs-first", "16", "--epochs-rest", "2"])
    cfg = bench.build_run(a, 1)
    assert cfg.train.hidden == 32 and cfg.train.optimizer == "adam"
    run = HedgeRun(cfg)
    run.build()
    run.enqueue()
    torch.cuda.synchronize()
    r_eager = run.collect()
    run.capture(include_simulation=True)  # raises if anything allocates inside the capture
    run.replay()
    torch.cuda.synchronize()
    r_graph = run.collect()
    run.close()
    assert r_eager.v0 == pytest.approx(r_graph.v0, rel=2e-3)
    assert r_eager.terminal_pnl["std"] == pytest.approx(r_graph.terminal_pnl["std"], rel=2e-2)
