"""rphedge — MI355X-native neural replicating portfolios / deep hedging.

Same capabilities and dict API as ithakis/Option-Replicating-Portfolio-with-
Neural-Networks (``Replicating_Portfolio``, ``Replicating_Portfolio_SV``), with
Sobol-QMC path generation, the hedge-MLP training step, Adam, residual/VaR
reductions as hand-written HIP kernels for gfx950 and RCCL data parallelism.
"""
__version__ = "0.1.0"

from .api import HedgeRun, Replicating_Portfolio, Replicating_Portfolio_SV, RunResult, european_option  # noqa: F401
from .config import ParityFlags, RunConfig, TrainingParams, parse_params  # noqa: F401
from .ops.sobol import sobol_norm  # noqa: F401
