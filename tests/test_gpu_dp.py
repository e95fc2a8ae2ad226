"""Data parallelism on ONE MI355X: two processes share the card and run the
fused xGMI/IPC all-reduce inside the step kernel (the 8-GPU path minus the
links).  Full-batch GD makes the DP result comparable with one process."""
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


def _data(n, dev, lo=0, cnt=None):
    g = torch.Generator().manual_seed(11)
    x = torch.rand(n, generator=g) * 0.6 + 0.7
    cnt = n if cnt is None else cnt
    f = x[lo:lo + cnt].to(dev)
    return f, f * 1.01, torch.relu(f * 1.01 - 1.0)


def _fit(rank, world, n, epochs, dev, mailbox=None, deterministic=True, mode=None):
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig, current_weights
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    per = n // world
    f, p1, y = _data(n, dev, rank * per, per)
    mode = mode or ("ticket" if deterministic else "lag")
    tc = TrainConfig(batch_size=n, chunk_log2=6, lr=1e-2, shuffle=False, deterministic=mode == "ticket",
                     step_mode=mode)
    be = HipBackend(spec, per, tc, device=dev, world=world, rank=rank, mailbox=mailbox)
    data = DateData(feats=[f], prices_next=[p1], bond_next=1.0, target=y, prices_now=[f])
    w, o, fs = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
    be.fit(w, o, fs, data, FitConfig(epochs=epochs, patience=10 ** 6, early_stopping=False), seed=3)
    torch.cuda.synchronize()
    return current_weights(spec, w), fs.cpu().numpy()


def _worker(rank, world, port, n, epochs, out, mode="ticket"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.ops.native import IpcMailbox

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mb = IpcMailbox(rank, world, 128, c10d._get_default_store(), dev, tag="t_dp")
    dist.barrier()
    w, fs = _fit(rank, world, n, epochs, dev, mailbox=mb, mode=mode)
    mb.check()
    np.save(out + f".{rank}.npy", w)
    dist.barrier()
    mb.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ticket", "lag", "persistent"])
def test_fused_xgmi_allreduce_two_ranks_one_gpu(mode):
    """ticket: per-step kernels, deterministic slab, exchange in the last
    arriver; lag: exchange in every kernel's prologue; persistent: in-kernel
    exchange of the one-launch-per-fit kernel."""
    n, epochs, world = 1 << 15, 6, 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, n, epochs, out, mode))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        w0, w1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert np.array_equal(w0, w1)                      # bitwise-identical replicas
    ref, _ = _fit(0, 1, n, epochs, torch.device("cuda", 0), mode=mode)
    tol = 1e-4 if mode == "ticket" else 1e-3   # float-atomic summation order in lag / persistent
    np.testing.assert_allclose(w0, ref, rtol=tol, atol=1e-5)


def _worker_missing_peer(rank, world, port, out):
    """Rank 1 never trains: rank 0's in-kernel exchange must time out (bounded
    spin), raise dp_error, fail fast in the later steps and surface as an error
    on the host (SURVEY §5.3 fault injection: a rank lost mid-all-reduce)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.ops.native import IpcMailbox

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mb = IpcMailbox(rank, world, 128, c10d._get_default_store(), dev, tag="t_dp_fail")
    dist.barrier()
    status = "idle"
    if rank == 0:
        _fit(0, world, 1 << 13, 2, dev, mailbox=mb, mode="ticket")
        try:
            mb.check()
            status = "no-error"
        except RuntimeError as e:
            status = "error:" + str(e)
    with open(out + f".{rank}.txt", "w") as f:
        f.write(status)
    dist.barrier()
    mb.close()
    dist.destroy_process_group()


def test_missing_peer_times_out_cleanly():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "s")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_missing_peer, args=(r, world, port, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        status = open(out + ".0.txt").read()
    assert status.startswith("error:") and "did not arrive" in status, status


def _ms_starts(spec, k):
    from rphedge.models.hedge_mlp import init_weights

    return np.stack([init_weights(spec, [0.5, 0.0], seed=1234 + 1000 * c) for c in range(k)])


def _lm_fit(rank, world, n, passes, dev, mailbox=None, lm_mailbox=None, starts=0, n_total=None, side=False,
            leaf=0, out_fix=False):
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig, current_weights, gram_subsample
    from rphedge.models.hedge_mlp import NetSpec, init_weights
    from rphedge.ops.paths import path_indices

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    per = n // world
    f, p1, y = _data(n if n_total is None else n_total, dev, rank * per, per)
    y = y + 0.02 * torch.sin(9 * f)
    be = HipBackend(spec, per, TrainConfig(batch_size=per, lm_gram_paths=2048, lm_leaf_paths=leaf, lm_out_fix=out_fix),
                    device=dev, world=world, rank=rank, mailbox=mailbox, lm_mailbox=lm_mailbox)
    gk = {}
    if side:  # the global Gram subsample, identical on every rank (engine.gram_subsample)
        ns, blk, stride = gram_subsample(n, 2048)
        fa, pa, _ = _data(n, dev)
        idx = torch.as_tensor(path_indices(ns, 0, (blk, stride)).astype(np.int64), device=dev)
        gk = dict(gram_feats=[fa[idx].contiguous()], gram_prices_next=[pa[idx].contiguous()])
    data = DateData(feats=[f], prices_next=[p1], bond_next=1.0, target=y, prices_now=[f], **gk)
    w, o, fs = be.new_weights(init_weights(spec, [0.5, 0.0])), be.new_opt(), be.new_fit()
    fc = FitConfig(epochs=passes, optimizer="lm", early_stopping=False)
    if starts:  # multi-start exploration: the same starts on the global 2^12-path prefix on every rank
        fc.lm_starts, fc.lm_explore_passes, fc.lm_explore_paths = starts, 6, 1 << 12
        fc.lm_w0s = _ms_starts(spec, starts)
        fa, pa, ya = _data(n if n_total is None else n_total, dev)
        ya = ya + 0.02 * torch.sin(9 * fa)
        nx = 1 << 12
        fc.lm_explore_data = DateData(feats=[fa[:nx].contiguous()], prices_next=[pa[:nx].contiguous()], bond_next=1.0,
                                      target=ya[:nx].contiguous(), prices_now=[fa[:nx].contiguous()])
    be.fit(w, o, fs, data, fc, seed=3)
    torch.cuda.synchronize()
    if starts:
        from rphedge.ops import layout as L
        st = be.lm_explore_last["state"].cpu().numpy()
        return current_weights(spec, w), [float(st[k, L.LMS_LFIN]) for k in range(starts)]
    return current_weights(spec, w), be.lm_state()


def _worker_lm(rank, world, port, n, passes, out, side=False, leaf=0, out_fix=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.ops import layout as L
    from rphedge.ops.native import IpcMailbox

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = c10d._get_default_store()
    mb = IpcMailbox(rank, world, 128, store, dev, tag=f"t_lm_a{world}")
    lmb = IpcMailbox(rank, world, L.LM_DP_PITCH, store, dev, tag=f"t_lm_b{world}")
    dist.barrier()
    w, st = _lm_fit(rank, world, n, passes, dev, mailbox=mb, lm_mailbox=lmb, side=side, leaf=leaf, out_fix=out_fix)
    lmb.check()
    np.save(out + f".{rank}.npy", w)
    with open(out + f".{rank}.txt", "w") as fh:
        fh.write(f"{st['accepted']} {st['chol_failures']}")
    dist.barrier()
    mb.close()
    lmb.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("side", [False, True])
def test_lm_mailbox_exchange_two_ranks_one_gpu(side):
    """Levenberg-Marquardt fit over 2 ranks over the IPC mailboxes (the xGMI
    transport): bitwise-identical replicas, and the 1-rank fit of the same
    global paths.  side=True: every rank builds the same Gram matrix from the
    global subsample (LmDesc.gram_side) and k_lm_dp_exchange_g carries only
    the 2.1 KB gradient region; side=False: each rank's part of the subsample,
    the whole [G | g | stats] block exchanged (only the fp64 summation order
    differs from one rank)."""
    n, passes, world = 1 << 15, 12, 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_lm, args=(r, world, port, n, passes, out, side))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        w0, w1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
        s0, s1 = open(out + ".0.txt").read(), open(out + ".1.txt").read()
    assert np.array_equal(w0, w1) and s0 == s1
    ref, st = _lm_fit(0, 1, n, passes, torch.device("cuda", 0), side=side)
    assert s0 == f"{st['accepted']} {st['chol_failures']}"
    if side:
        # the shared Gram, the gradient region summed in k_lm_reduce (fused
        # exchange) and W-invariant leaves / reduction trees: the one-rank fit
        # bit for bit (2^15 paths: the auto leaf is one 128-path block at both
        # world sizes)
        assert np.array_equal(w0, ref), np.abs(w0 - ref).max()
    else:
        np.testing.assert_allclose(w0, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_lm_strong_scaling_rehearsal_is_bitwise(world):
    """The same 2^18 global paths fitted by 1, 2, 4 or 8 ranks on one GPU (shared
    Gram subsample, gradient region summed inside k_lm_reduce over the IPC
    mailboxes, output-layer Newton step): with the same contiguous 256-path
    leaves at every world size (TrainConfig.lm_leaf_paths) and the
    contiguous-halves reduction trees, every rank's weights are bit for bit
    those of the one-rank fit.  W = 8 runs every level of the 8-way rank tree
    in lm_dp_sum_wave, 7 peers' flags per row and the DP_SLOTS rotation."""
    n, passes, leaf = 1 << 18, 10, 256
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_lm, args=(r, world, port, n, passes, out, True, leaf, True))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        ws = [np.load(out + f".{r}.npy") for r in range(world)]
        ss = [open(out + f".{r}.txt").read() for r in range(world)]
    ref, st = _lm_fit(0, 1, n, passes, torch.device("cuda", 0), side=True, leaf=leaf, out_fix=True)
    for r in range(world):
        assert np.array_equal(ws[r], ref), (r, np.abs(ws[r] - ref).max())
        assert ss[r] == f"{st['accepted']} {st['chol_failures']}"


@pytest.mark.parametrize("leaf", [0, 256])
def test_lm_512_pass_workgroups_two_ranks(leaf):
    """The two-workgroups-per-CU pass grid under data parallelism: 2^19 global
    paths, so one rank runs 512 pass workgroups (512-row packet reduce; in
    leaf mode also the 512-row output-Gram reduce) and each of two ranks 512
    (cyclic) or 256 (256-path leaves).  The replicas agree bit for bit; in
    leaf mode they are the one-rank fit bit for bit (the 512-row trees are the
    contiguous-halves trees the rank tree completes), cyclic to 1e-4."""
    from rphedge.engine import lm_pass_schedule

    n, passes, world = 1 << 19, 6, 2
    assert lm_pass_schedule(n, leaf, 2)[0] == 512
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_lm, args=(r, world, port, n, passes, out, True, leaf, True))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        w0, w1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
        s0, s1 = open(out + ".0.txt").read(), open(out + ".1.txt").read()
    assert np.array_equal(w0, w1) and s0 == s1
    ref, st = _lm_fit(0, 1, n, passes, torch.device("cuda", 0), side=True, leaf=leaf, out_fix=True)
    if leaf:
        assert np.array_equal(w0, ref), np.abs(w0 - ref).max()
        assert s0 == f"{st['accepted']} {st['chol_failures']}"
    else:
        np.testing.assert_allclose(w0, ref, rtol=1e-4, atol=1e-6)


def test_lm_gram_side_one_rank_is_bitwise_the_shard_gram():
    """One rank: the Gram subsample read from simulated subsample data
    (LmDesc.gram_side) or from the shard (the same global paths) gives the
    bitwise-identical fit."""
    dev = torch.device("cuda", 0)
    w_a, st_a = _lm_fit(0, 1, 1 << 15, 10, dev, side=False)
    w_b, st_b = _lm_fit(0, 1, 1 << 15, 10, dev, side=True)
    assert np.array_equal(w_a, w_b) and st_a == st_b


def _worker_ms(rank, world, port, n, passes, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.ops import layout as L
    from rphedge.ops.native import IpcMailbox

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = c10d._get_default_store()
    mb = IpcMailbox(rank, world, 128, store, dev, tag="t_ms_a")
    lmb = IpcMailbox(rank, world, L.LM_DP_PITCH, store, dev, tag="t_ms_b")
    dist.barrier()
    w, losses = _lm_fit(rank, world, n, passes, dev, mailbox=mb, lm_mailbox=lmb, starts=3)
    lmb.check()
    np.save(out + f".{rank}.npy", w)
    np.save(out + f".{rank}.losses.npy", np.asarray(losses))
    dist.barrier()
    mb.close()
    lmb.close()
    dist.destroy_process_group()


def test_lm_multistart_two_ranks_one_gpu():
    """Multi-start exploration over 2 ranks: every rank explores the same 3
    starts on the same global 2^12-path prefix (no exchange) and both polish
    the same winner: bitwise-identical replicas, and the candidates' losses
    are bitwise those of the 1-rank run over the same global paths."""
    n, passes, world = 1 << 15, 4, 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "w")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_ms, args=(r, world, port, n, passes, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        w0, w1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
        l0, l1 = np.load(out + ".0.losses.npy"), np.load(out + ".1.losses.npy")
    assert np.array_equal(w0, w1) and np.array_equal(l0, l1) and len(l0) == 3
    # 1 rank, the same global paths [0, n): the same exploration, bit for bit
    _, l_ref = _lm_fit(0, 1, n, passes, torch.device("cuda", 0), starts=3)
    np.testing.assert_array_equal(l0, np.asarray(l_ref))


def _worker_probe(rank, world, port, out, fault):
    """One rank of a torchrun-style job on a shared card: rphedge.parallel.dist
    init + select_transport, the probe record written as JSON."""
    import json

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    if fault:
        os.environ["RPH_PROBE_FAULT"] = fault
    from rphedge.parallel import dist as D

    info = D.init()
    D.select_transport(info)
    with open(out + f".{rank}.json", "w") as fh:
        json.dump({"probe": info.probe, "lm_dp_mode": info.lm_dp_mode, "dp_mode": info.dp_mode,
                   "lm_comm": type(info.lm_comm).__name__}, fh)
    D.barrier()
    D.shutdown()


def _run_probe(world, fault=""):
    import json

    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "p")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_probe, args=(r, world, port, out, fault)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        return [json.load(open(out + f".{r}.json")) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
def test_transport_probe_runs_the_fused_lm_exchange(world):
    """select_transport's LM probe runs the exchange the runs use (global Gram
    subsample -> LmDesc.dp_fused, the gradient region and the output-Gram rows
    summed inside k_lm_reduce) and checks it against the same fit over an
    independent torch.distributed all-reduce."""
    recs = _run_probe(world)
    for r in recs:
        lm = r["probe"]["lm"]
        assert lm["fused"] is True and lm["clean"] is True, lm
        assert lm["chosen"] == "xgmi" and r["lm_dp_mode"] == "xgmi", lm
        assert lm["max_rel_dev_vs_allreduce"] <= lm["rtol"], lm
        assert r["probe"]["packet"]["chosen"] == "xgmi"


def test_transport_probe_catches_a_symmetric_wrong_sum():
    """Fault injection into the fused path itself (LmDpDesc.fault: rank W-1's
    contribution dropped on EVERY rank): the replicas still agree bit for bit,
    so only the comparison with the independent all-reduce catches it - and
    the LM exchange falls back (on a shared card: the process group)."""
    recs = _run_probe(2, fault="lm_drop")
    for r in recs:
        lm = r["probe"]["lm"]
        assert lm["fused"] is True and lm["fault_injected"] is True, lm
        assert lm["bitwise_equal_weights"] is True, lm          # symmetric: the old probe passed it
        assert lm["max_rel_dev_vs_allreduce"] > lm["rtol"], lm
        assert r["lm_dp_mode"] == "rccl" and r["lm_comm"] == "TorchComm", r
        assert r["probe"]["packet"]["chosen"] == "xgmi"


def _mts_lm_run(di, leaf, graph):
    """experiments.mts_lm_parameters (both fits of every date on LM, 2^16
    paths, 40 quarterly dates) in leaf mode: (result, snapshots, graph nodes,
    k_lm_dp_exchange launches, whether the last pinball fit ran fused)."""
    from rphedge import experiments
    from rphedge.api import HedgeRun
    from rphedge.config import parse_params
    from rphedge.ops import native

    calls = [0]
    orig = native.lm_dp_exchange

    def counted(*a, **kw):
        calls[0] += 1
        return orig(*a, **kw)

    native.lm_dp_exchange = counted
    try:
        cfg = parse_params(experiments.mts_lm_parameters(n_paths=16, verbose=False, device="cuda:0",
                                                         lm_leaf_paths=leaf, concurrent_q99=False,
                                                         keep_paths=False))
        run = HedgeRun(cfg, dist_info=di) if di is not None else HedgeRun(cfg)
        res = run.run()
        torch.cuda.synchronize()
        fused = bool(run.backend.lm_last_fused)
        nodes = None
        if graph:
            run.capture(include_simulation=True)
            nodes = int(run.graph.num_nodes)
        snap = run.induction.snap.cpu().numpy().copy()
        out = dict(phi=res.phi, psi=res.psi, v0=res.v0, nodes=nodes, exchanges=calls[0], fused=fused)
        run.close()
        return out, snap
    finally:
        native.lm_dp_exchange = orig


def _worker_mts(rank, world, port, out, leaf):
    import json

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    from rphedge.parallel import dist as D

    di = D.init()
    rec, snap = _mts_lm_run(di, leaf, graph=True)
    np.save(out + f".{rank}.npy", snap)
    with open(out + f".{rank}.json", "w") as fh:
        json.dump(rec, fh)
    D.barrier()
    D.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_pension_both_fits_lm_world_invariant(world):
    """The pension run with BOTH fits on LM, data parallel on one card: the
    pinball (Q99) fits build their IRLS Gram on the simulated global subsample
    with its own targets (V_{t+1} evaluated on the subsample at every date
    boundary: DateData.gram_target), so every rank builds the same Gram and
    the gradient region is summed inside k_lm_reduce - no k_lm_dp_exchange
    launch at all, the same graph node count as one rank, and in leaf mode
    every date's weights are bit for bit those of the one-rank run
    (Replicating_Portfolio.py:138-145, :217-221)."""
    import json

    leaf = 256
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "m")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_worker_mts, args=(r, world, port, out, leaf)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        recs = [json.load(open(out + f".{r}.json")) for r in range(world)]
        snaps = [np.load(out + f".{r}.npy") for r in range(world)]
    ref, snap1 = _mts_lm_run(None, leaf, graph=True)
    for r in range(world):
        assert recs[r]["exchanges"] == 0 and recs[r]["fused"] is True, recs[r]
        assert np.array_equal(snaps[r], snap1), np.abs(snaps[r] - snap1).max()
        for k in ("phi", "psi", "v0"):   # (per-rank eval statistics: summed in another order)
            assert recs[r][k] == pytest.approx(ref[k], rel=1e-9), (k, recs[r][k], ref[k])
        # no node per pass or per date: the only extra nodes are the 3 kernels
        # simulating the multi-start's global path prefix once per run (path
        # scan, mortality, payoff), which one rank reads from its own shard
        assert recs[r]["nodes"] == ref["nodes"] + 3, (recs[r]["nodes"], ref["nodes"])
