"""Diagnostic: factor one LM system with the RPH_DUMP_T library and compare
the tile store (L of the augmented matrix, tile by tile) with numpy's
Cholesky factor.  usage: RPH_NATIVE_LIB=... python tools/archive/dump_tiles.py [P_index]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_gpu_lm_solve import SHAPES, _backend, gram, make_block, run_solve  # noqa: E402

from rphedge.ops import layout as L  # noqa: E402


def main(k=0):
    shape, P = SHAPES[k]
    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev)
    st = torch.zeros(1024, 8, dtype=torch.int64, device=dev)
    d.stamps = st.data_ptr()
    rng = np.random.default_rng(1)
    G = gram("spd", P, rng)
    g = rng.standard_normal(P) * 1e-2
    lam = 1e-3
    run_solve(L, be, d, b, P=P, best=0, w_best=np.zeros(P), w_trial=np.zeros(P),
              red_best=make_block(L, G, g, 1e-4), red_new=make_block(L, G, g, 2e-4), lam=lam)
    raw = st.view(torch.float64).flatten().cpu().numpy()
    NT = (P + 1 + 15) // 16
    PT = 16 * NT
    lam2 = min(lam * 4.0, 1e10)  # reject branch
    A = 2.0 * G
    dg = np.diag(A).copy()
    A = A + np.diag(dg * lam2 + tc.lm_ridge * dg.mean())
    M = np.eye(PT)
    M[:P, :P] = A
    M[P, :P] = -g
    # Cholesky of the augmented lower matrix: rows < P as A, row P = b^T
    Lr = np.zeros((PT, PT))
    Lr[:P, :P] = np.linalg.cholesky(A)
    Lr[P, :P] = np.linalg.solve(Lr[:P, :P], -g)
    out = []
    t = 0
    for jb in range(NT):
        for ib in range(jb, NT):
            tile = raw[t * 256:(t + 1) * 256]
            got = np.zeros((16, 16))
            for r in range(16):
                for c in range(16):
                    got[r, c] = tile[r * 16 + (c ^ ((r >> 1) << 1))]
            ref = Lr[16 * ib:16 * ib + 16, 16 * jb:16 * jb + 16].copy()
            rows = [r for r in range(16) if 16 * ib + r <= P]
            cols = [c for c in range(16) if 16 * jb + c < P]
            if rows and cols:
                e = np.abs(got[np.ix_(rows, cols)] - ref[np.ix_(rows, cols)])
                i, j = np.unravel_index(np.argmax(e), e.shape)
                bad = e > 1e-9 * max(1.0, np.abs(ref).max())
                out.append({"tile": [ib, jb], "err": float(e.max()), "at": [16 * ib + rows[i], 16 * jb + cols[j]],
                             "nbad": int(bad.sum()), "bad_cols": [cols[c] - 16 * jb for c in range(len(cols)) if bad[:, c].any()],
                             "bad_rows": [rows[r] for r in range(len(rows)) if bad[r].any()]})
            t += 1
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
