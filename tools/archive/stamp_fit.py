"""Phase breakdown of the persistent one-launch-per-fit kernel (csrc/hedge_fit.h)
from in-kernel s_memrealtime stamps of the LAST step (100 MHz), plus the
event-timed per-step cost of whole fits.  Diagnostic only.

usage: python tools/archive/stamp_fit.py '[{"batch_log2": 18}, {"batch_log2": 18, "hidden": 32}]'
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig  # noqa: E402
from rphedge.models.hedge_mlp import NetSpec, init_weights  # noqa: E402


def run(batch_log2=18, n_log2=20, nin=1, nout=2, hidden=8, epochs=64, max_wgs=256, mode="persistent",
        mfma_fp32=False, variant=0):
    dev = torch.device("cuda", 0)
    spec = NetSpec(nin=nin, hidden=hidden, nout=nout, head=0)
    n = 1 << n_log2
    g = torch.Generator(device="cpu").manual_seed(0)
    feats = [(torch.rand(n, generator=g) * 0.5 + 0.75).to(dev) for _ in range(nin)]
    prices = [f * 1.01 for f in feats[: spec.nhold - 1]]
    target = torch.relu(prices[0] - 1.0)
    tc = TrainConfig(batch_size=1 << batch_log2, chunk_log2=6, max_wgs=max_wgs, step_mode=mode,
                     mfma_fp32=mfma_fp32, variant=variant)
    be = HipBackend(spec, n, tc, device=dev)
    data = DateData(feats=feats, prices_next=prices, bond_next=1.0, target=target, prices_now=feats[:1])
    w0 = init_weights(spec, [0.5] + [0.0] * (nout - 1))
    fc = FitConfig(epochs=epochs, patience=10 ** 6, early_stopping=False)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, fc, seed=1)  # warm
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        be.fit(w, o, f, data, fc, seed=1)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e3 / (epochs * be.steps_per_epoch))
    out = {"batch_log2": batch_log2, "hidden": hidden, "mode": be.step_mode(), "variant": variant,
           "num_wgs": be.num_wgs,
           "steps_per_fit": epochs * be.steps_per_epoch, "us_per_step": float(np.median(times))}
    if be.step_mode() == "persistent":
        be.stamps = torch.zeros(be.num_wgs, 8, dtype=torch.int64, device=dev)
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, fc, seed=1)
        torch.cuda.synchronize()
        be.check()
        s = be.stamps.cpu().numpy().astype(np.int64)
        s = s[s[:, 0] > 0]
        us = lambda x: float(x) * 0.01  # noqa: E731
        med = lambda a, b: us(np.median(s[:, b] - s[:, a]))  # noqa: E731
        t0 = s[:, 0].min()
        out.update({
            "start_spread_us": us(s[:, 0].max() - t0),
            "partial_us": med(0, 1), "partial_max_us": us((s[:, 1] - s[:, 0]).max()),
            "drain_us": med(1, 2),
            "last_drained_after_start_us": us(s[:, 2].max() - t0),
            "arrive_wait_us": med(2, 3),
            "release_seen_after_last_drain_us": us(np.median(s[:, 3]) - s[:, 2].max()),
            "sums_us": med(3, 4), "update_us": med(4, 5),
            "step_us_stamped": us(np.median(s[:, 5]) - t0),
        })
        be.stamps = None
    if be.step_mode() == "lag":
        be.stamps = torch.zeros(be.num_wgs, 8, dtype=torch.int64, device=dev)
        w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
        be.fit(w, o, f, data, fc, seed=1)
        torch.cuda.synchronize()
        s = be.stamps.cpu().numpy().astype(np.int64)
        us = lambda x: float(x) * 0.01  # noqa: E731
        med = lambda a, b: us(np.median(s[:, b] - s[:, a]))  # noqa: E731
        t0 = s[:, 0].min()
        out.update({"start_spread_us": us(s[:, 0].max() - t0), "prologue_us": med(0, 1), "update_us": med(1, 2),
                    "paths_us": med(2, 5), "reduce_us": med(5, 3), "publish_us": med(3, 4),
                    "last_end_after_start_us": us(s[:, 4].max() - t0)})
        be.stamps = None
    return out


if __name__ == "__main__":
    grid = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [
        dict(batch_log2=18, mode=m) for m in ("lag", "ticket", "persistent")] + [
        dict(batch_log2=16, mode=m) for m in ("lag", "ticket")] + [
        dict(batch_log2=18, hidden=32, mode=m) for m in ("lag", "ticket")]
    for gcfg in grid:
        print(json.dumps(run(**gcfg)), flush=True)
