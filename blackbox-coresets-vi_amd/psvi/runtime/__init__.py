"""MI355X runtime of the coreset-ELBO inner loop: ctypes boundary to libpsvi_hip.so."""
from ._lib import PsviError, load  # noqa: F401
from .engine import (InnerLoopPlan, adam_adjoint_, adam_update_, make_adam, nonfinite_,  # noqa: F401
                     randn_)
