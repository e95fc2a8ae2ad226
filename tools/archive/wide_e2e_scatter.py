"""Run-to-run scatter of the wide (1-32-32-2) European end-to-end test
configuration (tests/test_gpu_wide.py::test_wide_european_end_to_end), per
input-standardisation mode."""
import json
import sys

sys.path.insert(0, ".")
from rphedge.api import HedgeRun  # noqa: E402
from rphedge.config import ParityFlags, RunConfig, TrainingParams  # noqa: E402

for fn in ("date", "none"):
    for rep in range(3):
        tr = TrainingParams(batch_size=1 << 14, epochs_first=60, epochs_rest=15, early_stopping=False, q99=False,
                            lr_schedule_first=False, chunk_log2=6, lr=5e-3, hidden=32, feature_norm=fn)
        cfg = RunConfig(Y=100.0, K=100.0, T=1.0, mu=0.08, r=0.08, sigma=0.15, rebalancing=1 / 12, dt=1 / 12,
                        n_paths=18, payoff="call", option_type="CALL", model="gbm_log", mortality=False, N=1, P=1.0,
                        keep_paths=True, verbose=False, train=tr, parity=ParityFlags())
        res = HedgeRun(cfg).run()
        print(json.dumps({"feature_norm": fn, "rep": rep, "V0": res.v0, "phi": res.phi,
                          "pnl_std": res.terminal_pnl["std"]}), flush=True)
