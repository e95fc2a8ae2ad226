import json, sys
sys.path.insert(0, ".")
from rphedge.api import HedgeRun
from rphedge.config import ParityFlags, RunConfig, TrainingParams
out = []
for mode in ("lag", "ticket"):
    for prec in ("bf16", "fp32"):
        for lr in (5e-3, 2e-3):
            tr = TrainingParams(batch_size=1 << 14, epochs_first=60, epochs_rest=15, early_stopping=False, q99=False,
                                lr_schedule_first=False, chunk_log2=6, lr=lr, hidden=32, step_mode=mode,
                                mfma_precision=prec)
            cfg = RunConfig(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=1 / 12, dt=1 / 12,
                            n_paths=18, payoff="call", option_type="CALL", model="gbm_log", mortality=False, N=1,
                            P=1.0, keep_paths=True, verbose=False, train=tr, parity=ParityFlags())
            res = HedgeRun(cfg).run()
            print(json.dumps({"mode": mode, "prec": prec, "lr": lr, "V0": res.v0, "phi": res.phi,
                              "pnl_std": res.terminal_pnl["std"]}), flush=True)
