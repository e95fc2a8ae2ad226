"""Hedge network family (SURVEY C14–C16)."""
from .hedge_mlp import EUROPEAN, EUROPEAN_REF, HESTON, PENSION, HedgeNet, NetSpec, basket_spec, init_weights  # noqa: F401
