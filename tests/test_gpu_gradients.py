"""Gradient EXACTNESS of the fused training kernels.

Adam's update is invariant to a constant gradient scale, so weight-trajectory
comparisons cannot see a mis-scaled gradient packet.  These tests read the raw
summed packet [P grads | loss sum | |e| sum | ape sum | count] the kernels
hand to the optimiser and compare it with fp64 autograd of the SAME minibatch:

* one ticketed step with the split update (the RCCL data-parallel path) for
  every 8-unit shape and the 32-unit shapes (fp32 and bf16 MFMA), MSE and
  pinball losses;
* the lagged schedule's exchanged packet (finalize, ``expose_packet``);
* data parallel on one GPU (2 processes): the in-kernel xGMI exchange of the
  lagged schedule, and the split-update path with the packet all-reduced by
  an external communicator (the RCCL call pattern; gloo transport here because
  RCCL refuses two ranks on one device) - both equal the 1-rank full-batch
  gradient.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SHAPES = [(1, 8, 2, 0), (1, 8, 1, 1), (2, 8, 2, 0), (3, 8, 2, 0), (4, 8, 2, 0), (5, 8, 6, 0), (6, 8, 7, 0),
          (1, 32, 2, 0), (2, 32, 2, 0), (3, 32, 2, 0), (5, 32, 6, 0)]


def _problem(spec, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    feats = [torch.rand(n, generator=g) * 0.5 + 0.75 for _ in range(spec.nin)]
    prices = [f.clone() * (1 + 0.05 * torch.randn(n, generator=g)) for f in feats[: spec.nhold - 1]]
    target = torch.relu(prices[0] - 1.0) + 0.05 * torch.rand(n, generator=g)
    return feats, prices, target


def _w0(spec):
    from rphedge.models.hedge_mlp import init_weights

    return init_weights(spec, ([0.5] + [-0.4] * (spec.nout - 1)) if spec.head == 0 else [0.1])


def autograd_packet(spec, w0, feats, prices, target, idx, loss, q=0.99, bond=1.02, world_batch=None, norm=None):
    """fp64 autograd of the mean loss over the minibatch ``idx`` + the packet's
    loss statistics (sums over idx)."""
    from rphedge.models.hedge_mlp import torch_forward
    from rphedge.ops import layout as L

    X = torch.stack([f[idx].double() for f in feats], dim=1)
    if norm is not None:
        X = (X - torch.tensor(norm[0], dtype=torch.float64)) * torch.tensor(norm[1], dtype=torch.float64)
    pr = torch.stack([p[idx].double() for p in prices] + [torch.full((len(idx),), bond, dtype=torch.float64)], 1)
    y = target[idx].double()
    w = torch.tensor(np.asarray(w0, np.float64), requires_grad=True)
    V = (torch_forward(spec, w, X) * pr).sum(1)
    e = V - y
    lv = torch.maximum(q * -e, (q - 1) * -e) if loss == L.LOSS_PINBALL else e * e
    B = world_batch or len(idx)
    (lv.sum() / B).backward()
    lv, e = lv.detach(), e.detach()
    stats = [float(lv.sum()), float(e.abs().sum()), float((e.abs() / y.abs().clamp_min(1e-7)).sum()), float(len(idx))]
    return w.grad.numpy(), np.asarray(stats)


def _check(pkt, P, g_ref, s_ref, gtol, stol=1e-5):
    g = pkt[:P].astype(np.float64)
    # relative L2 error of the whole gradient plus an entrywise bound scaled
    # by the gradient norm (a constant scale error of 1e-3 fails both)
    rel = np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref)
    assert rel < gtol, rel
    np.testing.assert_allclose(g, g_ref, rtol=0, atol=gtol * np.abs(g_ref).max())
    np.testing.assert_allclose(pkt[P:P + 4], s_ref, rtol=stol)


@pytest.mark.parametrize("loss", [0, 1])
@pytest.mark.parametrize("shape", SHAPES)
def test_split_update_packet_matches_fp64_autograd(shape, loss):
    """Ticketed step 1 (paths [batch, 2*batch), no shuffle) with the split
    update: HipBackend.grad holds the summed packet the update kernel (or the
    RCCL all-reduce) receives."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec

    nin, h, nout, head = shape
    spec = NetSpec(nin=nin, hidden=h, nout=nout, head=head)
    n, batch = 1 << 14, 1 << 12
    feats, prices, target = _problem(spec, n)
    dev = torch.device("cuda", 0)
    fp32_mfma = h == 32 and shape != (1, 32, 2, 0)
    tc = TrainConfig(batch_size=batch, shuffle=False, split_update=True, step_mode="ticket",
                     mfma_fp32=fp32_mfma)
    be = HipBackend(spec, n, tc, device=dev)
    data = DateData(feats=[f.to(dev) for f in feats], prices_next=[p.to(dev) for p in prices], bond_next=1.02,
                    target=target.to(dev), prices_now=[f.to(dev) for f in feats[: spec.nhold - 1]])
    w0 = _w0(spec)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    fc = FitConfig(epochs=1, patience=10 ** 6, loss=loss, early_stopping=False)
    d = be._train_desc(w, o, f, data, fc, seed=1, lr_t=None)
    assert d.fused_update == 0
    be.native.train_step(d, 1, 0, None)
    torch.cuda.synchronize()
    pkt = be.grad.cpu().numpy()
    g_ref, s_ref = autograd_packet(spec, w0, feats, prices, target, torch.arange(batch, 2 * batch), loss)
    # fp32 VALU / fp32 MFMA: 1e-5 relative; bf16 MFMA operands: 1e-2 (cosine-level agreement)
    bf16 = h == 32 and not fp32_mfma
    _check(pkt, spec.nparams, g_ref, s_ref, gtol=2e-2 if bf16 else 2e-5, stol=2e-3 if bf16 else 1e-5)


@pytest.mark.parametrize("shape", [(1, 8, 2, 0), (3, 8, 2, 0), (5, 8, 6, 0), (1, 32, 2, 0), (2, 32, 2, 0)])
def test_lag_finalize_packet_full_batch(shape):
    """Lagged schedule, one full-batch step: the packet summed from the
    float-atomic replica rows (finalize, expose_packet) is the full-batch
    gradient; the standardised-input path is included."""
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec

    nin, h, nout, head = shape
    spec = NetSpec(nin=nin, hidden=h, nout=nout, head=head)
    n = 1 << 15
    feats, prices, target = _problem(spec, n, seed=3)
    norm = (tuple(1.0 - 0.01 * k for k in range(nin)), tuple(7.0 + k for k in range(nin)))
    dev = torch.device("cuda", 0)
    tc = TrainConfig(batch_size=n, shuffle=False, step_mode="lag", expose_packet=True, mfma_fp32=h == 32)
    be = HipBackend(spec, n, tc, device=dev)
    data = DateData(feats=[f.to(dev) for f in feats], prices_next=[p.to(dev) for p in prices], bond_next=1.02,
                    target=target.to(dev), prices_now=[f.to(dev) for f in feats[: spec.nhold - 1]],
                    fmu=norm[0], fisd=norm[1])
    w0 = _w0(spec)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=1, patience=10 ** 6, early_stopping=False), seed=1)
    torch.cuda.synchronize()
    assert be.step_mode() == "lag" and be.num_wgs > 1
    g_ref, s_ref = autograd_packet(spec, w0, feats, prices, target, torch.arange(n), 0, norm=norm)
    _check(be.grad.cpu().numpy(), spec.nparams, g_ref, s_ref, gtol=2e-5)


def test_misscaled_gradient_is_detected():
    """Guard for the check itself: a packet off by 0.1 % fails it."""
    g = np.linspace(-1.0, 1.0, 106)
    pkt = np.concatenate([g * 1.001, [1.0, 1.0, 1.0, 4.0]])
    with pytest.raises(AssertionError):
        _check(pkt, 106, g, np.array([1.0, 1.0, 1.0, 4.0]), gtol=2e-5)


# ---------------------------------------------------------------------------
# data parallel on one GPU (2 processes)
# ---------------------------------------------------------------------------
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _GlooPacketComm:
    """The RCCL communicator's interface (allreduce_ of the packet on the
    compute stream), with the sum done by gloo through the host: the same
    split-update kernels and call pattern as RPH_DP=rccl."""

    def allreduce_(self, t, stream=None):
        import torch.distributed as dist

        torch.cuda.synchronize()
        h = t.detach().cpu()
        dist.all_reduce(h)
        t.copy_(h)


def _dp_worker(rank, world, port, n, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d

    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec
    from rphedge.ops.native import IpcMailbox

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    feats, prices, target = _problem(spec, n, seed=5)
    per = n // world
    sl = slice(rank * per, (rank + 1) * per)
    data = DateData(feats=[feats[0][sl].to(dev)], prices_next=[prices[0][sl].to(dev)], bond_next=1.02,
                    target=target[sl].to(dev), prices_now=[feats[0][sl].to(dev)])
    mb = None
    if mode == "xgmi_lag":
        mb = IpcMailbox(rank, world, spec.red_width, c10d._get_default_store(), dev, tag="t_gradpkt")
        dist.barrier()
        tc = TrainConfig(batch_size=n, shuffle=False, step_mode="lag", expose_packet=True)
        be = HipBackend(spec, per, tc, device=dev, world=world, rank=rank, mailbox=mb)
    else:
        tc = TrainConfig(batch_size=n, shuffle=False, step_mode="ticket", split_update=True)
        be = HipBackend(spec, per, tc, device=dev, world=world, rank=rank, comm=_GlooPacketComm())
    w, o, f = be.new_weights(_w0(spec)), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, FitConfig(epochs=1, patience=10 ** 6, early_stopping=False), seed=1)
    torch.cuda.synchronize()
    if mb is not None:
        mb.check()
    np.save(out + f".{rank}.npy", be.grad.cpu().numpy())
    dist.barrier()
    if mb is not None:
        mb.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["xgmi_lag", "split_update_comm"])
def test_dp_exchanged_packet_equals_full_batch_gradient(mode):
    n, world = 1 << 15, 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "g")
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_dp_worker, args=(r, world, port, n, mode, out)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
            assert p.exitcode == 0
        p0, p1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    from rphedge.models.hedge_mlp import NetSpec

    spec = NetSpec(nin=1, hidden=8, nout=2, head=0)
    assert np.array_equal(p0, p1)  # every rank applies the identical packet
    feats, prices, target = _problem(spec, n, seed=5)
    g_ref, s_ref = autograd_packet(spec, _w0(spec), feats, prices, target, torch.arange(n), 0)
    _check(p0, spec.nparams, g_ref, s_ref, gtol=2e-5)
