"""Phase breakdown of ONE full k_lm_solve (tile-store Cholesky, csrc/lm_chol.h)
from in-kernel s_memrealtime stamps (100 MHz ticks), per net shape, median
over repeats.  Diagnostic build of nothing: the production kernel writes the
stamps only when TrainDesc.stamps is set.

usage: python tools/archive/solve_stamps.py > out.jsonl
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")

from test_gpu_lm_solve import SHAPES, _backend, gram, make_block, run_solve  # noqa: E402

from rphedge.ops import layout as L  # noqa: E402


def one(shape, P, reps=20):
    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev)
    st = torch.zeros(1024, 8, dtype=torch.int64, device=dev)
    d.stamps = st.data_ptr()
    rng = np.random.default_rng(1)
    G = gram("spd", P, rng)
    g = rng.standard_normal(P) * 1e-2
    rows = []
    for _ in range(reps):
        st.zero_()
        run_solve(L, be, d, b, P=P, best=0, w_best=np.zeros(P), w_trial=np.zeros(P),
                  red_best=make_block(L, G, g, 1e-4), red_new=make_block(L, G, g, 2e-4), lam=1e-3)
        s0, s1 = st[0].cpu().numpy().astype(np.int64), st[1].cpu().numpy().astype(np.int64)
        t = lambda a, b_: (float(b_ - a) / 100.0) if (a and b_) else None  # noqa: E731
        rows.append({"decision": t(s0[0], s0[1]), "setup": t(s0[1], s0[2]), "tiles_loaded": t(s0[2], s1[0]),
                     "panel0": t(s1[0], s1[1]), "wait_panel1": t(s1[1], s1[2]), "panel1": t(s1[2], s1[3]),
                     "panels_2_to_last": t(s1[3], s1[5]), "last_panel": t(s1[4], s1[5]),
                     "factor": t(s1[0], s1[5]), "backward": t(s0[6], s0[7]), "join": t(s0[7], s0[3]),
                     "publish": t(s0[3], s0[5]), "total": t(s0[0], s0[5])})
    keys = rows[0].keys()
    return {"P": P, **{k: float(np.median([r[k] for r in rows if r[k] is not None] or [np.nan])) for k in keys}}


if __name__ == "__main__":
    for shape, P in SHAPES:
        print(json.dumps(one(shape, P)), flush=True)
