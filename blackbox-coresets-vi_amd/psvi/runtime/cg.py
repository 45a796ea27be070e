"""hyper_step's conjugate-gradient solve on the device (psvi_cg_*).

CG_normaleq (reference psvi/hypergrad/hypergradients.py:199-244) runs
CG_torch.cg (psvi/hypergrad/CG_torch.py:9-45) on the normal-equation operator
A(p) = vmj - J vmj, vmj = lr H_A p, J y = y - lr H_B y: H_A is the inner
objective's Hessian at the draw of w_mapped, H_B at a fresh draw per call
(fp_map draws its noise).  Per iteration the two Hessian-vector products run
on psvi_hvp; the vector work around them -- the fp32 <-> fp64 promotions, p.Ap,
the residual and its norm, the x / r / p updates -- is three fused passes
(csrc/kernels_cg.hip) with the step lengths and the stopping flag kept on the
device."""
import ctypes

import torch

from . import _lib
from ._lib import check


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class DeviceCG:
    """Buffers of one solve size n (float64 vectors on `device`)."""

    def __init__(self, n, device):
        self.lib = _lib.load()
        self.n = int(n)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("DeviceCG runs on the HIP device (psvi_cg_*)")
        self.state = torch.zeros(7, dtype=torch.float64, device=dev)
        self.ws = torch.zeros(int(self.lib.psvi_cg_ws_bytes()), dtype=torch.uint8, device=dev)
        self.p32 = torch.empty(self.n, dtype=torch.float32, device=dev)
        self.vmj32 = torch.empty(self.n, dtype=torch.float32, device=dev)

    def solve(self, hv_a, hv_b, b, lr, K, tol=1e-10, sync_every=1):
        """x after at most K iterations of the reference's cg(A, b) (the
        iterate before ||r|| < tol, as the reference's break returns it).
        hv_a(p32) / hv_b(v32): the fp32 products H_A p32 and H_B v32 (hv_b
        draws H_B's noise as fp_map would); the host reads the stopping flag
        every sync_every iterations (1: exactly the reference's number of
        operator calls, hence of draws)."""
        n, lib = self.n, self.lib
        if b.numel() != n or b.dtype != torch.float64 or not b.is_contiguous():
            raise ValueError("b: contiguous float64 of the solve size expected")
        x = torch.zeros_like(b)
        r = b.clone()
        p = b.clone()
        self.p32.copy_(b)
        self.state.zero_()
        self.state[0] = torch.dot(r, r)
        lr = float(lr)
        wsb = self.ws.numel()
        sync_every = max(1, int(sync_every))
        for it in range(int(K)):
            hv1 = hv_a(self.p32)
            check(lib.psvi_cg_scale(n, _p(hv1), lr, _p(self.vmj32), _s()), "psvi_cg_scale")
            hv2 = hv_b(self.vmj32)
            check(lib.psvi_cg_pap(n, _p(hv1), _p(hv2), lr, _p(p), _p(self.state), _p(self.ws),
                                  wsb, _s()), "psvi_cg_pap")
            check(lib.psvi_cg_residual(n, _p(hv1), _p(hv2), lr, _p(r), _p(self.state),
                                       float(tol), _p(self.ws), wsb, _s()), "psvi_cg_residual")
            check(lib.psvi_cg_update(n, _p(x), _p(p), _p(self.p32), _p(r), _p(self.state), _s()),
                  "psvi_cg_update")
            if (it + 1) % sync_every == 0 and bool(self.state[3].item()):
                break
        return x
