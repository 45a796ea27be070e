"""Inner-loop surface of the reference's psvi.inference (PSVI classes)."""
from .psvi_classes import (PSVI, PSVIAV, PSVIAFixedU, PSVIFixedU, PSVIFreeV,  # noqa: F401
                           PSVILearnV, PSVI_Ablated, PSVI_No_IW, PSVI_No_Rescaling, HipInnerELBO)
from .baselines import run_mfvi, run_mfvi_subset  # noqa: F401,E402
