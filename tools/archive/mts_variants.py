"""Which reference semantic moves the GBM pension parity runs' phi0 / psi0?
The "Multi Time Step.ipynb" headline run (mts_notebook, parity mode) under
candidate explanations of the phi0 +5 % / psi0 -10 % offset of the multi-seed
bands: LeakyReLU slope 0.2 (Keras 3) instead of 0.3 (Keras 2),
Keras-3 EarlyStopping restore at the end of every fit, and the Adam state
reset per date instead of carried (Q18).  One JSON line per (variant, seed).

usage: python tools/archive/mts_variants.py [--backend torch] [--seeds 4] [variants...] > out.jsonl
"""
import argparse
import json
import sys
import time

sys.path.insert(0, ".")

VARIANTS = {
    "base": {},
    "alpha02": {"leaky_alpha": 0.2},
    "restore_end": {"parity_flags": {"restore_best_at_end": True}},
    "adam_reset": {"parity_flags": {"carry_optimizer": False}},
    "alpha02_restore_end": {"leaky_alpha": 0.2, "parity_flags": {"restore_best_at_end": True}},
    "unshared_q99": {"parity_flags": {"shared_q99_model": False}},
    "blend_sign_corrected": {"parity_flags": {"holdings_blend_sign_rp": False}},
    # round 4: one seeded initializer instance reused for every kernel (RP:149, :154-156)
    "shared_init": {"parity_flags": {"shared_initializer": True}},
    "shared_init_alpha02": {"leaky_alpha": 0.2, "parity_flags": {"shared_initializer": True}},
    # round 5: the remaining pairwise / triple combinations of the Keras candidates
    "shared_init_restore_end": {"parity_flags": {"shared_initializer": True, "restore_best_at_end": True}},
    "shared_init_adam_reset": {"parity_flags": {"shared_initializer": True, "carry_optimizer": False}},
    "alpha02_adam_reset": {"leaky_alpha": 0.2, "parity_flags": {"carry_optimizer": False}},
    "restore_end_adam_reset": {"parity_flags": {"restore_best_at_end": True, "carry_optimizer": False}},
    "shared_init_alpha02_restore_end": {"leaky_alpha": 0.2,
                                        "parity_flags": {"shared_initializer": True, "restore_best_at_end": True}},
    "shared_init_alpha02_adam_reset": {"leaky_alpha": 0.2,
                                       "parity_flags": {"shared_initializer": True, "carry_optimizer": False}},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default=None, help="torch = CPU oracle")
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--seed0", type=int, default=1234)
    ap.add_argument("variants", nargs="*", default=list(VARIANTS))
    a = ap.parse_args()
    from rphedge.experiments import mts_notebook

    for v in a.variants:
        for k in range(a.seeds):
            over = dict(VARIANTS[v], seed=a.seed0 + k, verbose=False)
            if a.backend:
                over.update(backend=a.backend, device="cpu")
            else:
                over.update(poll_every=10)
            t0 = time.perf_counter()
            o = mts_notebook(**over)
            print(json.dumps({"variant": v, "seed": a.seed0 + k, "V0": o["V0"], "phi0": o["phi0"], "psi0": o["psi0"],
                              "VaR": o.get("VaR"), "s": time.perf_counter() - t0}), flush=True)


if __name__ == "__main__":
    main()
