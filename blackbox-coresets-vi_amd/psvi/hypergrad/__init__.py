"""psvi.hypergrad: the reference's hypergradient package
(psvi/hypergrad/{hypergradients,diff_optimizers,CG_torch}.py) on the HIP
inner objective -- the names PSVI.hyper_step's body binds
(psvi_classes.py:602-687): DifferentiableAdam, GradientDescent,
CG_normaleq, fixed_point, ..."""
from .diff_optimizers import *  # noqa: F401,F403
from .hypergradients import *  # noqa: F401,F403
from . import CG_torch  # noqa: F401
