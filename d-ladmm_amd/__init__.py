"""d-ladmm_amd: MI355X-native fused D-LADMM forward and backward (drop-in for DLADMMNet).

Import with ``importlib.import_module("d-ladmm_amd")`` (the directory name is not a Python
identifier) or put the repo root on sys.path and use the same call.
"""
from . import _lib  # noqa: F401
from . import dist  # noqa: F401
from .model import (DLADMMNet, DLADMMNetFull, DLADMMNetLasso, DLADMMNetLTheta,  # noqa: F401
                    DLADMMNetScalar, DLADMMNetScalarSl2, DLADMMNetScalarTied,
                    DLADMMNetScalarZ0, VARIANTS, load_checkpoint)
from .model import DLADMMNetNewS, DLADMMNetPTiedNewS, DLADMMNetTiedNewS  # noqa: F401
from .lskm import DLADMMNetLSKM  # noqa: F401
from .ops import (BackwardResult, ForwardResult, dladmm_backward, dladmm_forward,  # noqa: F401
                  plan_flags)

__all__ = ["DLADMMNet", "DLADMMNetLTheta", "DLADMMNetFull", "DLADMMNetScalar",
           "DLADMMNetScalarSl2", "DLADMMNetScalarZ0",
           "DLADMMNetScalarTied", "DLADMMNetLasso", "DLADMMNetNewS", "DLADMMNetTiedNewS",
           "DLADMMNetPTiedNewS", "DLADMMNetLSKM", "VARIANTS", "load_checkpoint",
           "dladmm_forward", "dladmm_backward", "ForwardResult", "BackwardResult"]
