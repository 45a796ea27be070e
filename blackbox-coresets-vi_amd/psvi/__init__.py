"""psvi (MI355X-native): the coreset-weighted ELBO inner loop of
souravc83/Blackbox-Coresets-VI on hand-written HIP kernels (gfx950).

  psvi.models     variational layers with the reference's parameter layout
                  (VILinear, VILinearMultivariateNormal, make_fcnet, make_fc2net)
  psvi.inference  PSVI classes: inner_elbo / inner_loop on the HIP library
  psvi.runtime    ctypes boundary to libpsvi_hip.so (C ABI: include/psvi_hip.h),
                  single-GPU plans and the multi-GPU sharded driver
"""
