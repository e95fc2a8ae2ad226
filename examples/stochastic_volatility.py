"""'Extra: Stochastic Volatility.ipynb' offline: HV40D, drift and CIR OLS.

    python examples/stochastic_volatility.py [--csv prices.csv]
(no network: without --csv a synthetic CIR-on-sigma price history is used)"""
import argparse
import json

from rphedge import calib

ap = argparse.ArgumentParser()
ap.add_argument("--csv", default=None, help="CSV with a 'Close' column (e.g. an exported ^GSPC history)")
a = ap.parse_args()
prices = calib.load_prices(a.csv) if a.csv else calib.synthetic_prices()
out = calib.calibrate(prices)
vol = out.pop("volatility")
print(json.dumps(out, indent=1))
print("acf(returns)[:5]", calib.acf(calib.log_returns(prices), 4).round(4).tolist())
print("reference (S&P500 10y): a=0.0033566 b=0.15431 c=0.015833 mu=0.09464 vol0=0.15965")
