"""Hedge quality of the GPU presets at their BASELINE sizes against analytic
hedges on the SAME paths (bench.py's hedge_anchor): Black-Scholes delta
(euro30, euro252), the Heston minimum-variance hedge (heston30;
rphedge.analytic.heston_hedge_anchor) and the Levy moment-matched basket delta
(basket5).

Seeds: at least four per long-horizon preset, always including the worst seeds
of the 16-seed measurements - a first-date local minimum or a later-date
blow-up shows on a minority of seeds, so two good seeds cannot guard it.
Bounds: the 16-seed worst of the current presets (round 6, the final build:
profiles/r6/final3/seeds/, BENCHMARKS.md) + a small margin; the P&L ratio is
the learnt hedge's self-financing P&L std / the analytic hedge's.

  preset    16 seeds: mean / worst ratio (worst seed)   seeds tested   bound
  euro30    1.0087 / 1.0297 (14)                        1 2 13 14      1.035
  heston30  1.0071 / 1.0132 (5)                         1 2 5 13       1.015
  euro252   1.0412 / 1.0984 (4), residual <= 0.0749     1 2 4 12       1.12, residual 0.08
  basket5   1.071 / 1.131 (3)                           1 3 4 13       1.15

basket5 meets the round-5 verdict's target (16 seeds: mean <= 1.08 x, worst
<= 1.15 x the Levy hedge) since the round-6 preset (4 passes per later date,
damping carry x2, 80 first-date polish passes, output-step trust region):
its bound IS the target."""
import json
import math
import os
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seeds(preset, seeds, extra=()):
    """Every seed of a preset in ONE process (tools/seeds.py): per-seed records."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "s.jsonl")
        e = dict(os.environ)
        e.setdefault("OMP_NUM_THREADS", "1")
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            e.pop(k, None)
        cmd = [sys.executable, "tools/seeds.py", out, ",".join(str(s) for s in seeds), "--preset", preset,
               "--steps", "1", "--warmup", "1", *extra]
        r = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-3000:]
        recs = [json.loads(ln) for ln in open(out) if ln.startswith("{")]
    assert [x["seed"] for x in recs] == list(seeds)
    return recs


@pytest.mark.parametrize("preset,seeds,ratio,resid_max,price_tol", [
    ("euro30", (1, 2, 13, 14), 1.035, None, 0.01),
    ("heston30", (1, 2, 5, 13), 1.015, None, 0.02),
    ("euro252", (1, 2, 4, 12), 1.12, 0.08, 0.01),
    ("basket5", (1, 3, 4, 13), 1.15, None, None),
])
def test_preset_pnl_within_anchor(preset, seeds, ratio, resid_max, price_tol):
    for r in _seeds(preset, seeds):
        s, pnl, a = r["seed"], r["pnl"], r["anchor_pnl"]
        assert a and math.isfinite(pnl), r
        assert pnl <= ratio * a, (preset, s, pnl / a)
        if resid_max is not None:
            assert r["resid"] <= resid_max, (preset, s, r["resid"])
        if price_tol is not None:
            assert abs(r["V0"] - r["anchor_price"]) < price_tol, (preset, s, r["V0"], r["anchor_price"])
        else:  # basket: no closed form; the moment-matched anchor's price
            assert abs(r["V0"] - r["hedge_price"]) < 0.02 * r["hedge_price"], (preset, s, r["V0"], r["hedge_price"])


def test_basket5_verdict_target():
    """The round-5 verdict's basket target on its worst seed of the 16 (seed 3)."""
    r = _seeds("basket5", (3,))[0]
    assert r["pnl"] <= 1.15 * r["anchor_pnl"], r["pnl"] / r["anchor_pnl"]
