"""Command line interface: ``python -m rphedge <command>``.

  run        --config cfg.json [--set key=value ...]   any params dict (pension, SV, European, basket)
  european   [--paths N] [--parity] ...                  European Options notebook driver
  sts                                                    Single Time Step notebook driver
  sweep      [--sigmas .05,.1,...]                       volatility sweep (Multi Time Step)
  calibrate  --csv prices.csv | --synthetic               CIR calibration (Extra: Stochastic Volatility)
  sanity     --config cfg.json                           notebook sanity checks
  info                                                   device + native library info
Multi-GPU: launch with ``python -m torch.distributed.run --nproc-per-node N -m rphedge run ...``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def _coerce(v: str):
    for f in (int, float):
        try:
            return f(v)
        except ValueError:
            pass
    if v.lower() in ("true", "false"):
        return v.lower() == "true"
    return v


def _summary(res) -> dict:
    return {"phi0": res.phi, "psi0": res.psi, "V0": res.v0, "terminal_pnl": res.terminal_pnl, "VaR": res.var,
            "summary": {k: v for k, v in res.summary.items() if not isinstance(v, list)},
            "timings": res.timings}


def _plots(res, out_dir):
    if not out_dir:
        return
    from .utils.reports import plot_run

    os.makedirs(out_dir, exist_ok=True)
    res.summary["figures"] = plot_run(res, out_prefix=os.path.join(out_dir, "rphedge"))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="rphedge", description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--config", required=True)
    r.add_argument("--set", nargs="*", default=[])
    r.add_argument("--sv", action="store_true")
    r.add_argument("--out", default=None)
    r.add_argument("--plots", default=None, help="directory for the report figures (C26-C32)")
    e = sub.add_parser("european")
    e.add_argument("--paths", type=int, default=3000)
    e.add_argument("--rebalancing", type=float, default=1 / 52)
    e.add_argument("--parity", action="store_true")
    e.add_argument("--set", nargs="*", default=[])
    e.add_argument("--plots", default=None, help="directory for the report figures (C26-C32)")
    sub.add_parser("sts").add_argument("--no-parity", action="store_true")
    s = sub.add_parser("sweep")
    s.add_argument("--sigmas", default="0.05,0.10,0.15,0.20,0.30")
    s.add_argument("--set", nargs="*", default=[])
    c = sub.add_parser("calibrate")
    c.add_argument("--csv", default=None)
    c.add_argument("--synthetic", action="store_true")
    c.add_argument("--window", type=int, default=40)
    sa = sub.add_parser("sanity")
    sa.add_argument("--config", required=True)
    sub.add_parser("info")
    a = ap.parse_args(argv)

    if a.cmd == "run":
        from .api import run_params

        with open(a.config) as f:
            params = json.load(f)
        params.update({k: _coerce(v) for k, v in (kv.split("=", 1) for kv in a.set)})
        if a.out:
            params["save_dir"] = a.out
        res = run_params(params, sv=a.sv)
        _plots(res, a.plots)
        print(json.dumps(_summary(res), default=float, indent=1))
    elif a.cmd == "european":
        from .api import european_option

        extra = {k: _coerce(v) for k, v in (kv.split("=", 1) for kv in a.set)}
        res = european_option(N_paths=a.paths, rebalancing_frequency=a.rebalancing, parity=a.parity, **extra)
        _plots(res, a.plots)
        print(json.dumps(_summary(res), default=float, indent=1))
    elif a.cmd == "sts":
        from .experiments import single_time_step

        out = single_time_step(parity=not a.no_parity)
        out.pop("result")
        print(json.dumps(out, default=float, indent=1))
    elif a.cmd == "sweep":
        from .experiments import volatility_sweep

        extra = {k: _coerce(v) for k, v in (kv.split("=", 1) for kv in a.set)}
        rows = volatility_sweep(sigmas=[float(x) for x in a.sigmas.split(",")], **extra)
        print(json.dumps(rows, default=float, indent=1))
    elif a.cmd == "calibrate":
        from . import calib

        prices = calib.load_prices(a.csv) if a.csv else calib.synthetic_prices()
        out = calib.calibrate(prices, window=a.window)
        out.pop("volatility")
        print(json.dumps(out, indent=1))
    elif a.cmd == "sanity":
        from .experiments import sanity_checks

        with open(a.config) as f:
            print(json.dumps(sanity_checks(json.load(f)), default=float, indent=1))
    elif a.cmd == "info":
        import torch

        from .ops import native

        info = {"torch": torch.__version__, "hip": torch.version.hip, "gpu": torch.cuda.is_available(),
                "native": str(native._LIB_PATH), "native_loaded": native.available()}
        if torch.cuda.is_available():
            info.update(native.device_info(0))
        print(json.dumps(info, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
