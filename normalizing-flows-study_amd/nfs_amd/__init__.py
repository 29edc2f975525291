"""nfs_amd — MI355X-native (gfx950) flow-transform hot path of itxtx/normalizing-flows-study.

Drop-in nn.Modules for the reference's per-layer transform + log|det| path (src/flows/* and
src/models/*), backed by hand-written HIP kernels in libnfx.so (C-ABI: include/nfx.h).
"""
from . import _lib
from .flows import (Flow, SequentialFlow, CouplingLayer, SplineCouplingLayer,
                    rational_quadratic_spline, ARQS, MaskedLinear, MADE, MaskedAutoregressiveFlow,
                    InverseAutoregressiveFlow, made_degrees, STATS, reset_stats)
from .models import NormalizingFlowModel, RealNVP, RealNVPSpline, gauss_logprob
from .graphs import GraphedFlow, GraphedTrainStep

__all__ = ["Flow", "SequentialFlow", "CouplingLayer", "SplineCouplingLayer",
           "rational_quadratic_spline", "ARQS", "MaskedLinear", "MADE", "MaskedAutoregressiveFlow",
           "InverseAutoregressiveFlow", "NormalizingFlowModel", "RealNVP", "RealNVPSpline",
           "gauss_logprob", "made_degrees", "STATS", "reset_stats", "GraphedFlow", "GraphedTrainStep"]
