"""Flow layers on the hot path (mirrors src/flows/__init__.py for the in-scope symbols)."""
from .flow import Flow, SequentialFlow, HipFlow, STATS, reset_stats, drop_pack_caches, drop_layer_pack_caches
from .coupling import CouplingLayer
from .spline import SplineCouplingLayer, rational_quadratic_spline
from .arqs import ARQS
from .autoregressive import (MaskedLinear, MADE, MaskedAutoregressiveFlow,
                             InverseAutoregressiveFlow, made_degrees)

__all__ = ["Flow", "SequentialFlow", "HipFlow", "CouplingLayer", "SplineCouplingLayer",
           "rational_quadratic_spline", "ARQS", "MaskedLinear", "MADE", "MaskedAutoregressiveFlow",
           "InverseAutoregressiveFlow", "made_degrees", "STATS", "reset_stats", "drop_pack_caches",
           "drop_layer_pack_caches"]
