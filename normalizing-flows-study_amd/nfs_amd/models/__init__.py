from .normalizing_flow_model import NormalizingFlowModel, gauss_logprob
from .real_nvp import RealNVP
from .real_nvp_spline import RealNVPSpline

__all__ = ["NormalizingFlowModel", "RealNVP", "RealNVPSpline", "gauss_logprob"]
