"""Build-time cost of driver.feature_norms on the basket5 shape (252 dates x 5 assets x 2^23 paths)."""
import time, torch, sys
sys.path.insert(0, '.')
from rphedge.ops import paths as P
from rphedge.driver import feature_norms
g = P.Grid(1.0, 1/252, 1/252)
import rphedge.ops.paths as PP
import numpy as np
corr = np.full((5, 5), 0.5) + 0.5 * np.eye(5)
p = PP.simulate_basket(g, 1 << 23, [1.0] * 5, [0.05] * 5, [0.2] * 5, corr, device="cuda")
torch.cuda.synchronize()
for mode in ("date",):
    t0 = time.time(); n = feature_norms(p, mode); torch.cuda.synchronize(); print(mode, time.time() - t0, n[10])
