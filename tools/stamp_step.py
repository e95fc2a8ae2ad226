"""Phase breakdown of ONE fused training step from in-kernel s_memrealtime
stamps (100 MHz).  Diagnostic only (production launches pass stamps=null)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig  # noqa: E402
from rphedge.models.hedge_mlp import NetSpec, init_weights  # noqa: E402
from rphedge.ops import layout as L  # noqa: E402
from rphedge.ops import native  # noqa: E402


def run(batch_log2=16, n_log2=20, nin=1, nout=2, reps=20, det=False, max_wgs=256, ppt=1):
    dev = torch.device("cuda", 0)
    spec = NetSpec(nin=nin, hidden=8, nout=nout, head=0)
    n = 1 << n_log2
    g = torch.Generator(device="cpu").manual_seed(0)
    feats = [(torch.rand(n, generator=g) * 0.5 + 0.75).to(dev) for _ in range(nin)]
    prices = [f * 1.01 for f in feats[: spec.nhold - 1]]
    target = torch.relu(prices[0] - 1.0)
    be = HipBackend(spec, n, TrainConfig(batch_size=1 << batch_log2, chunk_log2=6, deterministic=det, max_wgs=max_wgs,
                                         paths_per_thread=ppt), device=dev)
    data = DateData(feats=feats, prices_next=prices, bond_next=1.0, target=target, prices_now=feats[:1])
    w, o, f = be.new_weights(init_weights(spec, [0.5] + [0.0] * (nout - 1))), be.new_opt(), be.new_fit()
    fc = FitConfig(epochs=1000, patience=10 ** 6, early_stopping=False)
    be.fit(w, o, f, data, fc, seed=1)  # warm
    torch.cuda.synchronize()
    be.stamps = torch.zeros(be.num_wgs, 8, dtype=torch.int64, device=dev)
    d = be._train_desc(w, o, f, data, fc, 1, None)
    f.copy_(be._template(fc))
    rows = []
    for r in range(reps):
        be.stamps.zero_()
        torch.cuda.synchronize()
        native.train_step(d, r % be.steps_per_epoch, r // be.steps_per_epoch)
        torch.cuda.synchronize()
        s = be.stamps.cpu().numpy().astype(np.int64)
        t0 = s[:, 0].min()
        last = int(np.argmax(s[:, 6]))
        ph = lambda a, b: np.median(s[:, b] - s[:, a]) * 10.0 / 1000.0  # noqa: E731  (us)
        rows.append({
            "dispatch_spread_us": float((s[:, 0].max() - t0) * 0.01),
            "prologue_us": float(ph(0, 1)), "paths_reduce_us": float(ph(1, 3)),
            "publish_drain_us": float(ph(3, 4)), "ticket_us": float(ph(4, 5)),
            "last_fetch_us": float((s[last, 6] - s[last, 5]) * 0.01),
            "last_update_us": float((s[last, 7] - s[last, 6]) * 0.01),
            "last_arrival_after_start_us": float((s[last, 5] - t0) * 0.01),
            "total_us": float((s[last, 7] - t0) * 0.01)})
    med = {k: float(np.median([r[k] for r in rows[2:]])) for k in rows[0]}
    med.update({"batch_log2": batch_log2, "num_wgs": be.num_wgs, "det": det})
    return med


if __name__ == "__main__":
    import sys as _s
    grid = json.loads(_s.argv[1]) if len(_s.argv) > 1 else (
        [dict(batch_log2=bl) for bl in (14, 16, 18)] + [dict(batch_log2=18, max_wgs=512), dict(batch_log2=17, max_wgs=512),
                                                       dict(batch_log2=18, max_wgs=1024)])
    for g in grid:
        print(json.dumps(run(**g)), flush=True)
