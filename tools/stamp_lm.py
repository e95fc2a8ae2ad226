"""Phase breakdown of the Levenberg-Marquardt solve kernel (k_lm_solve,
csrc/hedge_lm.hip) from in-kernel s_memrealtime stamps (100 MHz), plus the
event-timed cost per LM pass of whole fits.  Diagnostic only.

usage: python tools/stamp_lm.py [n_log2] [nin] [og]

og: lm_out_fix fits (the last LM_OUTG_TAIL passes build the full-batch output
Gram, k_lm_pass<BodyOG>; the stamped pass is the last one).
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig  # noqa: E402
from rphedge.models.hedge_mlp import NetSpec, init_weights  # noqa: E402


def run(n_log2=20, nin=1, passes=40, og=False):
    dev = torch.device("cuda", 0)
    nout = 2 if nin <= 4 else nin + 1
    spec = NetSpec(nin=nin, hidden=8, nout=nout, head=0)
    n = 1 << n_log2
    g = torch.Generator(device="cpu").manual_seed(0)
    feats = [(torch.rand(n, generator=g) * 0.5 + 0.75).to(dev) for _ in range(nin)]
    prices = [f * 1.01 for f in feats[: spec.nhold - 1]]
    target = torch.relu(prices[0] - 1.0)
    be = HipBackend(spec, n, TrainConfig(batch_size=n, lm_out_fix=og), device=dev)
    be.stamps = torch.zeros(1024, 8, dtype=torch.int64, device=dev)
    data = DateData(feats=feats, prices_next=prices, bond_next=1.0, target=target, prices_now=feats[:1])
    w0 = init_weights(spec, [0.5] + [0.0] * (nout - 1))
    fc = FitConfig(epochs=passes, optimizer="lm", early_stopping=False)
    w, o, f = be.new_weights(w0), be.new_opt(), be.new_fit()
    be.fit(w, o, f, data, fc, seed=0)  # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w = be.new_weights(w0)
    e0.record()
    be.fit(w, o, f, data, fc, seed=0)
    e1.record()
    torch.cuda.synchronize()
    st = be.stamps[0].cpu().tolist()
    order = [k for k in (0, 1, 2, 6, 7, 3, 4, 5) if st[k]]
    ph = {f"solve_phase_{a}_{b}_us": (st[b] - st[a]) / 100.0 for a, b in zip(order, order[1:])}
    s1 = be.stamps[1].cpu().tolist()
    if all(s1[k] for k in range(6)) and st[2]:
        # row 0 = the last FULL solve (k_lm_solve writes it only then), row 1 = its
        # panel wave (csrc/lm_chol.h: 0/1 panel 0 wait passed / done, 2/3 panel 1, 4/5 last)
        ph["tile_solver_us"] = {"setup_to_panel0_ready": (s1[0] - st[2]) / 100.0,
                                "panel0": (s1[1] - s1[0]) / 100.0, "wait_panel1": (s1[2] - s1[1]) / 100.0,
                                "panel1": (s1[3] - s1[2]) / 100.0, "wait_last": (s1[4] - s1[3]) / 100.0,
                                "last_panel": (s1[5] - s1[4]) / 100.0,
                                "last_panel_load": (s1[6] - s1[4]) / 100.0 if s1[6] else None,
                                "last_panel_columns": (s1[7] - s1[6]) / 100.0 if s1[6] and s1[7] else None,
                                "last_panel_writeback": (s1[5] - s1[7]) / 100.0 if s1[7] else None,
                                "factor_total": (s1[5] - s1[0]) / 100.0,
                                "backward": (st[7] - st[6]) / 100.0 if st[6] and st[7] else None,
                                "total_kernel": (st[5] - st[0]) / 100.0 if st[5] else None}
    # k_lm_pass phases of the last pass over all workgroups >= 2 (rows 0/1 are the solve's)
    import numpy as np
    lmd = be._lm_buffers()["desc"]
    S = be.stamps[2:lmd.num_wgs].cpu().numpy().astype(np.int64)
    t0 = S[:, 0].min()
    gram = np.arange(2, 2 + len(S)) < lmd.gram_wgs
    end = np.where(gram, S[:, 4], S[:, 2])
    q = lambda v: [round(float(np.percentile(v, x)) / 100.0, 2) for x in (0, 50, 100)]
    ph["pass_wg_us_min_med_max"] = {"start": q(S[:, 0] - t0), "prologue": q(S[:, 1] - S[:, 0]),
                                     "paths_gram_wgs": q((S[:, 2] - S[:, 1])[gram]),
                                     "paths_other_wgs": q((S[:, 2] - S[:, 1])[~gram]),
                                     "j_build": q((S[:, 3] - S[:, 2])[gram]), "gram_mfma": q((S[:, 4] - S[:, 3])[gram]),
                                     "end_gram_wgs": q((end - t0)[gram]), "end_other_wgs": q((end - t0)[~gram])}
    wg = np.arange(2, 2 + len(S))
    pth = (S[:, 2] - S[:, 1]) / 100.0
    ph["pass_paths_us_by_group"] = {f"{'second' if b else 'first'}_half_xcd{x}": round(float(pth[(wg % 8 == x) & ((wg >= len(S) // 2) == b)].mean()), 2)
                                    for b in (False, True) for x in range(8)}
    return {"n_log2": n_log2, "nin": nin, "passes": passes, "og": og, "us_per_pass": 1000.0 * e0.elapsed_time(e1) / (passes + 1),
            **ph, "lm": be.lm_state()}


if __name__ == "__main__":
    n_log2 = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    nin = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    og = len(sys.argv) > 3 and sys.argv[3] == "og"
    print(json.dumps(run(n_log2, nin, og=og)))
