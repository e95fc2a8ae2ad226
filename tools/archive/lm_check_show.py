"""Summarise tools/archive/lm_check.sh outputs (host side)."""
import csv
import json
import re

print(open("gpurun_out/pytest.log").read().strip().splitlines()[-1])
log = open("gpurun_out/prof.log").read()
line = [ln for ln in log.splitlines() if ln.startswith("{")][0]
r = json.loads(line)
q = r["quality"]
print("ms/run", round(r["ms_per_step"], 3), "pnl", q["terminal_pnl_std"], "resid", q["terminal_residual_std"], "V0", q["V0"])
for row in list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))[:4]:
    print(" ", re.sub(r"\(.*", "", row["Name"])[:50], row["Calls"], row["AverageNs"], row["Percentage"])
st = [ln for ln in open("gpurun_out/stamp.log").read().splitlines() if ln.startswith("{")]
for ln in st:
    print(ln[:900])
