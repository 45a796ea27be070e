"""Model API of the reference's psvi.models (variational layers, builders)."""
from .neural_net import (MultivariateNormalVIMixin, VILinear, VILinearMultivariateNormal,  # noqa: F401
                         VIMixin, categorical_fn, gaussian_fn, inverse_softplus, make_fc2net,
                         make_fcnet, make_logreg, model_spec, set_mc_samples, vi_layers,
                         VIConv2d, BatchMaxPool2d, make_lenet, LENET_LAYERS)
