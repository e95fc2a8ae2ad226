"""Direct tests of the Levenberg-Marquardt solve kernel (k_lm_solve,
csrc/hedge_lm.hip): on a synthetic reduced block and solver state, one call
must take the accept / reject decision, update the damping, and write the
trial point theta + d with d the fp64 solution of

    (2 G + lam' diag(2 G) + ridge * mean(diag(2 G)) I) d = -g

for every supported parameter count (97, 106, 114, 122, 130, 174, 191), on
well-conditioned, ill-conditioned and rank-deficient Gram matrices; an
indefinite system must take the failure branch (damping raised, FAIL counter
bumped, trial := best).  The fit this replaces is the Keras fit of
Replicating_Portfolio.py:211."""
import json

import numpy as np
import pytest
import torch

from rphedge.engine import lm_tpack_image

pytestmark = pytest.mark.gpu

# (shape, P)
SHAPES = [((1, 8, 1, 1), 97), ((1, 8, 2, 0), 106), ((2, 8, 2, 0), 114), ((3, 8, 2, 0), 122),
          ((4, 8, 2, 0), 130), ((5, 8, 6, 0), 174), ((6, 8, 7, 0), 191)]


def _lm_row(q, h):
    return (q & 3) + 8 * (q >> 2) + 4 * h


def encode_gram(G):
    """Dense symmetric G -> upper-triangular 32x32 blocks in MFMA register order
    (the layout k_lm_reduce writes; inverse of test_gpu_lm.decode_gram)."""
    P = G.shape[0]
    NP = (P + 31) // 32 * 32
    NB = NP // 32
    Gp = np.zeros((NP, NP))
    Gp[:P, :P] = G
    out = []
    q = np.arange(16)[:, None]
    lane = np.arange(64)[None, :]
    for mb in range(NB):
        for nb in range(mb, NB):
            i = mb * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5)
            j = nb * 32 + (lane & 31)
            out.append(Gp[i, j].reshape(-1))
    return np.concatenate(out)


def make_block(L, G, g, loss_mean, count=1000.0):
    """Reduced LM block [G | g | stats] (layout of rph_types.h LM_RED)."""
    red = np.zeros(L.LM_RED)
    enc = encode_gram(G)
    red[:enc.size] = enc
    P = G.shape[0]
    img = lm_tpack_image(enc, P, enc.size // 1024)  # what k_lm_reduce writes beside the blocks
    if img is not None:
        red[enc.size:enc.size + img.size] = img
    red[L.LM_GBLK_MAX:L.LM_GBLK_MAX + P] = g
    s = L.LM_GBLK_MAX + L.LM_NPMAX
    red[s:s + 4] = [loss_mean * count, 0.5, 0.25, count]
    return red


def gram(kind, P, rng):
    if kind == "spd":
        J = rng.standard_normal((4 * P, P)) * rng.uniform(0.2, 3.0, P)
        return J.T @ J / (4 * P)
    if kind == "illcond":
        Q, _ = np.linalg.qr(rng.standard_normal((P, P)))
        ev = np.logspace(0, -9, P)
        return (Q * ev) @ Q.T
    if kind == "rankdef":  # duplicated Jacobian columns: singular G, PD only through the damping
        J = rng.standard_normal((3 * P, P - P // 2))
        J = np.concatenate([J, J[:, : P // 2] * 0.5], axis=1)
        return J.T @ J / (3 * P)
    if kind == "indefinite":
        G = np.diag(rng.uniform(1.0, 2.0, P))
        G[3, 4] = G[4, 3] = 10.0 * np.sqrt(G[3, 3] * G[4, 4])
        return G
    raise ValueError(kind)


def _backend(shape, dev, damping="simple"):
    from rphedge.engine import DateData, FitConfig, HipBackend, TrainConfig
    from rphedge.models.hedge_mlp import NetSpec, init_weights

    spec = NetSpec(*shape)
    n = 1 << 12
    feats = [torch.rand(n, device=dev) for _ in range(spec.nin)]
    pr = [torch.rand(n, device=dev) + 0.5 for _ in range(spec.nhold - 1)]
    data = DateData(feats=feats, prices_next=pr, bond_next=1.0, target=torch.rand(n, device=dev), prices_now=pr)
    tc = TrainConfig(batch_size=n, lm_ridge=1e-10, lm_damping=damping)
    be = HipBackend(spec, n, tc, device=dev)
    w = be.new_weights(init_weights(spec, [0.5] * spec.nout, seed=1))
    # the descriptor holds raw pointers: keep every buffer it names alive (a
    # freed FitState block can be handed to the LM state allocated next, and
    # the solve's loss-history writes then land in the best point's Gram block)
    be._keep = (w, be.new_opt(), be.new_fit(), data)
    d = be._train_desc(w, be._keep[1], be._keep[2], data, FitConfig(optimizer="lm"), 0, None)
    d.batch, d.steps_per_epoch, d.shuffle = n, 1, 0
    b = be._lm_buffers()
    b["desc"].passes = 4
    return spec, be, d, b, tc


def slot(L, pass_):
    """Offset of the scalar slot pass `pass_` reads (the solve of pass p writes
    the slot of p + 1)."""
    return L.LMS_SLOTS + L.LM_SLOT * (pass_ & 1)


def run_solve(L, be, d, b, *, P, best, w_best, w_trial, red_best, red_new, lam, pass_=1):
    """One solve of pass `pass_`; returns (state, offset of the slot it wrote)."""
    st = np.zeros(L.LMS_FLOATS)
    st[L.LMS_W + best * L.LM_NPMAX:L.LMS_W + best * L.LM_NPMAX + P] = w_best
    st[L.LMS_W + (1 - best) * L.LM_NPMAX:L.LMS_W + (1 - best) * L.LM_NPMAX + P] = w_trial
    st[L.LMS_RED:L.LMS_RED + L.LM_RED] = red_best
    s = L.LMS_RED + L.LM_GBLK_MAX + L.LM_NPMAX
    si = slot(L, pass_)
    st[si + L.LSS_LBEST] = red_best[L.LM_GBLK_MAX + L.LM_NPMAX] / red_best[L.LM_GBLK_MAX + L.LM_NPMAX + 3]
    st[si + L.LSS_BEST] = best
    st[si + L.LSS_LAM] = lam
    st[si + L.LSS_NU] = 2.0
    st[si + L.LSS_SPEC_IDX] = float(L.LM_SPEC)
    b["state"].copy_(torch.from_numpy(st))
    red = torch.from_numpy(red_new).to(b["red"].device)
    be.native.lm_solve(d, b["desc"], red, pass_, None)
    torch.cuda.synchronize()
    return b["state"].cpu().numpy(), slot(L, pass_ + 1)


def expected_step(G, g, lam, ridge):
    A = 2.0 * G
    dg = np.diag(A).copy()
    dmp = dg * lam + ridge * dg.mean()
    A = A + np.diag(dmp)
    try:
        np.linalg.cholesky(A)
    except np.linalg.LinAlgError:
        return None, None, A
    dv = np.linalg.solve(A, -g)
    pred = 0.5 * (np.sum(dmp * dv * dv) - g @ dv)
    return dv, pred, A


@pytest.mark.parametrize("shape,P", SHAPES)
@pytest.mark.parametrize("kind", ["spd", "illcond", "rankdef"])
@pytest.mark.parametrize("accept", [True, False])
def test_lm_solve_step_matches_fp64(shape, P, kind, accept):
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev)
    assert spec.nparams == P
    rng = np.random.default_rng(P * 7 + len(kind) + accept)
    lm = b["desc"]
    for it, lam in enumerate([1e-3, 0.7, 30.0]):
        Gb, Gt = gram(kind, P, rng), gram(kind, P, rng)
        gb, gt = rng.standard_normal(P) * 1e-2, rng.standard_normal(P) * 1e-2
        Lb = 1.0e-4
        Lt = Lb * (0.5 if accept else 2.0)
        # small weights: trial - base then carries the step at full precision
        w_best, w_trial = rng.standard_normal(P) * 2.0 ** -20, rng.standard_normal(P) * 2.0 ** -20
        best = it % 2
        st, so = run_solve(L, be, d, b, P=P, best=best, w_best=w_best, w_trial=w_trial,
                           red_best=make_block(L, Gb, gb, Lb), red_new=make_block(L, Gt, gt, Lt), lam=lam)
        if accept:
            G, g, base = Gt, gt, w_trial
            lam2, best2 = max(lam * lm.lam_down, lm.lam_min), 1 - best
        else:
            G, g, base = Gb, gb, w_best
            lam2, best2 = min(lam * lm.lam_up, lm.lam_max), best
        dv, pred, A = expected_step(G, g, lam2, tc.lm_ridge)
        assert dv is not None
        assert int(st[L.LMS_BEST]) == best2
        assert st[L.LMS_LAM] == pytest.approx(lam2, rel=1e-15)
        assert int(st[so + L.LSS_BEST]) == best2 and st[so + L.LSS_LAM] == st[L.LMS_LAM]
        assert st[so + L.LSS_COPY] == (1.0 if accept else 0.0)
        assert st[so + L.LSS_LBEST] == (Lt if accept else Lb)
        assert st[L.LMS_FAIL] == 0.0
        tr = 1 - best2
        got = st[L.LMS_W + tr * L.LM_NPMAX:L.LMS_W + tr * L.LM_NPMAX + P] - base
        # backward stable: small residual of the computed step in the system it solves
        res = np.linalg.norm(A @ got + g) / (np.linalg.norm(A, 2) * np.linalg.norm(got) + np.linalg.norm(g))
        assert res < 1e-13, (lam, res)
        # forward error within the conditioning of the damped system
        cond = np.linalg.cond(A)
        err = np.linalg.norm(got - dv) / np.linalg.norm(dv)
        assert err < max(1e-9, 1e-14 * cond), (lam, err, cond)
        assert st[so + L.LSS_PRED] == pytest.approx(pred, rel=max(1e-9, 1e-14 * cond))
        # the best slot's weights are untouched
        bw = st[L.LMS_W + best2 * L.LM_NPMAX:L.LMS_W + best2 * L.LM_NPMAX + P]
        np.testing.assert_array_equal(bw, w_trial if accept else w_best)


@pytest.mark.parametrize("shape,P", [SHAPES[0], SHAPES[1], SHAPES[5]])
@pytest.mark.parametrize("accept", [True, False])
def test_lm_solve_indefinite_takes_failure_branch(shape, P, accept):
    """A system that is not positive definite at the new damping: no step,
    trial := best, damping x lam_up^2 on top of the accept / reject update,
    FAIL counter + 1."""
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev)
    rng = np.random.default_rng(11 + P)
    lm = b["desc"]
    G = gram("indefinite", P, rng)
    g = rng.standard_normal(P)
    lam = 1e-3
    Lb = 1e-4
    Lt = Lb * (0.5 if accept else 2.0)
    w_best, w_trial = rng.standard_normal(P), rng.standard_normal(P)
    best = 0
    st, so = run_solve(L, be, d, b, P=P, best=best, w_best=w_best, w_trial=w_trial,
                       red_best=make_block(L, G, g, Lb), red_new=make_block(L, G, g, Lt), lam=lam)
    lam2 = max(lam * lm.lam_down, lm.lam_min) if accept else min(lam * lm.lam_up, lm.lam_max)
    dv, _, _ = expected_step(G, g, lam2, tc.lm_ridge)
    assert dv is None  # numpy agrees the damped system is indefinite
    best2 = 1 - best if accept else best
    assert st[L.LMS_FAIL] == 1.0
    assert int(st[L.LMS_BEST]) == best2
    assert st[L.LMS_LAM] == pytest.approx(min(lam2 * lm.lam_up * lm.lam_up, lm.lam_max), rel=1e-15)
    assert st[so + L.LSS_LAM] == st[L.LMS_LAM] and st[so + L.LSS_SPEC_IDX] == float(L.LM_SPEC)
    keep = w_trial if accept else w_best
    for slot in (0, 1):
        np.testing.assert_array_equal(st[L.LMS_W + slot * L.LM_NPMAX:L.LMS_W + slot * L.LM_NPMAX + P], keep)


@pytest.mark.parametrize("shape,P", [SHAPES[1], SHAPES[5]])
@pytest.mark.parametrize("damping", ["simple", "nielsen"])
def test_lm_solve_speculative_chain_is_bitwise_serial(shape, P, damping):
    """A full solve also factorises the systems of the next LM_SPEC - 1
    consecutive rejections (one workgroup each); the solves of those
    rejections only publish the precomputed steps.  The trial sequence must be
    bitwise the one-full-solve-per-pass sequence (LSS_SPEC_IDX invalidated
    before every call), including a rejection chain longer than LM_SPEC - 1."""
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev, damping)
    b["desc"].passes = 8
    rng = np.random.default_rng(3 + P)
    G = gram("spd", P, rng)
    Gt = gram("spd", P, rng)
    g, gt = rng.standard_normal(P) * 1e-2, rng.standard_normal(P) * 1e-2
    # pass 1 accepted (full solve), passes 2..6 rejected
    losses = [0.5e-4] + [9e-4] * 5
    runs = []
    for serial in (False, True):
        st0 = np.zeros(L.LMS_FLOATS)
        st0[L.LMS_W:L.LMS_W + P] = rng.standard_normal(P) if not runs else runs[0]["w0"]
        w0 = st0[L.LMS_W:L.LMS_W + P].copy()
        st0[L.LMS_RED:L.LMS_RED + L.LM_RED] = make_block(L, G, g, 1e-4)
        s1 = slot(L, 1)
        st0[s1 + L.LSS_LBEST] = 1e-4
        st0[s1 + L.LSS_BEST] = 0
        st0[s1 + L.LSS_LAM] = 1e-3
        st0[s1 + L.LSS_NU] = 2.0
        st0[s1 + L.LSS_PRED] = 1e-5
        st0[s1 + L.LSS_SPEC_IDX] = float(L.LM_SPEC)
        b["state"].copy_(torch.from_numpy(st0))
        trials, lams, idx = [], [], []
        for k, Lt in enumerate(losses):
            if serial:
                b["state"][slot(L, k + 1) + L.LSS_SPEC_IDX] = float(L.LM_SPEC)
            red = torch.from_numpy(make_block(L, Gt, gt, Lt)).to(dev)
            be.native.lm_solve(d, b["desc"], red, k + 1, None)
            torch.cuda.synchronize()
            st = b["state"].cpu().numpy()
            so = slot(L, k + 2)
            if st[so + L.LSS_COPY] != 0.0:  # what the next pass kernel does: best block := the accepted trial's
                n_cp = L.LM_GBLK_MAX + L.LM_NPMAX + 4
                b["state"][L.LMS_RED:L.LMS_RED + n_cp] = red[:n_cp]
            tr = 1 - int(st[L.LMS_BEST])
            trials.append(st[L.LMS_W + tr * L.LM_NPMAX:L.LMS_W + tr * L.LM_NPMAX + P].copy())
            lams.append(st[L.LMS_LAM])
            idx.append(st[so + L.LSS_SPEC_IDX])
            assert st[L.LMS_FAIL] == 0.0
        blk = make_block(L, Gt, gt, losses[0])
        stf = b["state"].cpu().numpy()
        n_cp = L.LM_GBLK_MAX + L.LM_NPMAX + 4
        dd = np.abs(stf[L.LMS_RED:L.LMS_RED + n_cp] - blk[:n_cp])
        runs.append(dict(bestred=(float(dd.max()), [int(i) for i in np.nonzero(dd)[0][:12]]),
                         w0=w0, trials=trials, lams=lams, idx=idx,
                         best=b["state"][L.LMS_W + L.LM_NPMAX:L.LMS_W + L.LM_NPMAX + P].cpu().numpy()))
    spec_run, ser = runs
    # the speculative run used precomputed steps for rejections 1..3, then a full solve
    assert spec_run["idx"][:5] == [1.0, 2.0, 3.0, 4.0, 1.0], spec_run["idx"]
    assert spec_run["lams"] == ser["lams"]
    bad = [k for k, (a_, b_) in enumerate(zip(spec_run["trials"], ser["trials"])) if not np.array_equal(a_, b_)]
    if bad:  # which run is off: each trial vs the fp64 step from the best point (the pass-1 trial)
        base = ser["best"]
        errs = {}
        for name, r in (("spec", spec_run), ("serial", ser)):
            e = []
            for k, lam_k in enumerate(r["lams"]):
                dv, _, _ = expected_step(Gt, gt, lam_k, tc.lm_ridge)
                e.append(float(np.linalg.norm(r["trials"][k] - base - dv) / np.linalg.norm(dv)))
            errs[name] = e
            errs[name + "_bestred"] = r["bestred"]
        raise AssertionError((bad, [float(np.abs(spec_run["trials"][k] - ser["trials"][k]).max()) for k in bad], errs))


@pytest.mark.parametrize("shape,P", [SHAPES[1], SHAPES[5]])
@pytest.mark.parametrize("accept", [True, False])
def test_lm_solve_speculative_steps_match_fp64(shape, P, accept):
    """Workgroup m of a full solve writes the step of m further rejections:
    best + d(lam_m), lam_m = min(lam' x lam_up^m, lam_max), to LMS_SPEC_W[m];
    each must solve its damped system like workgroup 0's own step."""
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev)
    b["desc"].passes = 8
    lm = b["desc"]
    rng = np.random.default_rng(5 + P + accept)
    G = gram("spd", P, rng)
    g = rng.standard_normal(P) * 1e-2
    w_best, w_trial = rng.standard_normal(P) * 2.0 ** -20, rng.standard_normal(P) * 2.0 ** -20
    lam = 1e-3
    st, so = run_solve(L, be, d, b, P=P, best=0, w_best=w_best, w_trial=w_trial, red_best=make_block(L, G, g, 1e-4),
                       red_new=make_block(L, G, g, 0.5e-4 if accept else 2e-4), lam=lam)
    lam_m = max(lam * lm.lam_down, lm.lam_min) if accept else min(lam * lm.lam_up, lm.lam_max)
    base = w_trial if accept else w_best
    assert st[so + L.LSS_SPEC_IDX] == 1.0
    for m in range(4):
        if m > 0:
            lam_m = min(lam_m * lm.lam_up, lm.lam_max)
            assert st[L.LMS_SPEC_LAM + m] == lam_m and st[L.LMS_SPEC_OK + m] == 1.0
            got = st[L.LMS_SPEC_W + m * L.LM_NPMAX:L.LMS_SPEC_W + m * L.LM_NPMAX + P] - base
        else:
            tr = 1 - int(st[L.LMS_BEST])
            got = st[L.LMS_W + tr * L.LM_NPMAX:L.LMS_W + tr * L.LM_NPMAX + P] - base
        dv, pred, A = expected_step(G, g, lam_m, tc.lm_ridge)
        res = np.linalg.norm(A @ got + g) / (np.linalg.norm(A, 2) * np.linalg.norm(got) + np.linalg.norm(g))
        err = np.linalg.norm(got - dv) / np.linalg.norm(dv)
        assert res < 1e-13 and err < 1e-9, (m, res, err)


@pytest.mark.parametrize("shape,P", [SHAPES[1], SHAPES[5]])
def test_lm_solve_is_deterministic(shape, P):
    """The same full solve twice (same state, same block): bitwise equal trial
    weights (no timing-dependent order inside the workgroup hand-offs)."""
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    spec, be, d, b, tc = _backend(shape, dev)
    rng = np.random.default_rng(21 + P)
    G = gram("illcond", P, rng)
    g = rng.standard_normal(P) * 1e-2
    outs = []
    for _ in range(6):
        st, _ = run_solve(L, be, d, b, P=P, best=0, w_best=np.zeros(P), w_trial=np.zeros(P),
                          red_best=make_block(L, G, g, 1e-4), red_new=make_block(L, G, g, 2e-4), lam=1e-3)
        outs.append(st[L.LMS_W + L.LM_NPMAX:L.LMS_W + L.LM_NPMAX + P].copy())
    for o in outs[1:]:
        np.testing.assert_array_equal(o, outs[0])


def test_lm_solve_time_per_shape(capsys):
    """Per-call time of the solve (eager launches, GPU-bound); printed for the
    record (profiles/), asserted only loosely so a regression shows up."""
    from rphedge.ops import layout as L

    dev = torch.device("cuda", 0)
    out = {}
    for shape, P in SHAPES:
        try:
            spec, be, d, b, tc = _backend(shape, dev)
        except ValueError:  # an A/B library without this shape's solver
            continue
        rng = np.random.default_rng(5)
        G = gram("spd", P, rng)
        g = rng.standard_normal(P) * 1e-2
        blk = make_block(L, G, g, 1e-4)
        run_solve(L, be, d, b, P=P, best=0, w_best=np.zeros(P), w_trial=np.zeros(P),
                  red_best=blk, red_new=make_block(L, G, g, 2e-4), lam=1e-3)
        red = torch.from_numpy(make_block(L, G, g, 2e-4)).to(dev)
        n = 400
        s1 = slot(L, 1)
        slot1 = b["state"][s1:s1 + L.LM_SLOT].clone()  # pass 1's inputs (a pass-2 solve overwrites them)
        sin = b["state"][s1:s1 + L.LM_SLOT]

        def loop(solve):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                sin.copy_(slot1)  # no precomputed step: a full solve every call
                if solve:
                    be.native.lm_solve(d, b["desc"], red, 1, None)  # reject branch
            e1.record()
            torch.cuda.synchronize()
            return 1000.0 * e0.elapsed_time(e1) / n

        loop(True)
        out[P] = loop(True) - loop(False)
        # the speculative (published) rejection: precomputed step available
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        cheap = []
        for _ in range(50):
            sin.copy_(slot1)
            be.native.lm_solve(d, b["desc"], red, 1, None)  # full: precomputes steps 1..3
            e0.record()
            be.native.lm_solve(d, b["desc"], red, 2, None)  # rejection 1: published
            e1.record()
            torch.cuda.synchronize()
            cheap.append(1000.0 * e0.elapsed_time(e1))
        out[f"{P}_published"] = float(np.median(cheap))
    with capsys.disabled():
        print("\nk_lm_solve us/call:", json.dumps({str(k): round(v, 2) for k, v in out.items()}))
    assert all(v < 200.0 for v in out.values()), out
