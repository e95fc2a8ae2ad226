import json, subprocess, sys, os
# usage: run.py variant seed log2 [extra bench args...]
v, s, n = sys.argv[1], sys.argv[2], sys.argv[3]
extra = " ".join(["--seed", s] + sys.argv[4:])
env = dict(os.environ, OMP_NUM_THREADS="1")
out = subprocess.run([sys.executable, "tools/lm_lab.py", "--variants", v, "--paths-log2", n, "--extra", extra],
                     capture_output=True, text=True, env=env, timeout=3600).stdout
for l in out.splitlines():
    if not l.startswith("{"):
        continue
    r = json.loads(l)
    h = r["first"]["hist"]
    best, b = [], 1e9
    for x in h:
        b = min(b, x)
        best.append(b)
    tgt = [1e-4, 3e-5, 1.5e-5, 1.2e-5, 1e-5]
    print(json.dumps(dict(v=v, seed=int(s), ex=" ".join(sys.argv[4:]), n=int(n), pnl=r["pnl_std"], res=r["resid_std"],
                          V0=r["V0"], L=r["first"]["L"], acc=r["first"]["acc"],
                          reach={str(t): next((i for i, x in enumerate(best) if x <= t), None) for t in tgt},
                          acc_rest=r["acc_rest"], passes_rest=r["passes_rest"])), flush=True)
