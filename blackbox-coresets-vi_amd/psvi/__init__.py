"""psvi (MI355X-native): coreset-weighted ELBO inner loop on hand-written HIP kernels.

Mirrors the reference package layout (psvi.models, psvi.inference,
psvi.robust_higher, psvi.hypergrad, psvi.experiments) for the hot path; the
arithmetic of the inner loop runs in blackbox-coresets-vi_amd/csrc (gfx950).
"""
