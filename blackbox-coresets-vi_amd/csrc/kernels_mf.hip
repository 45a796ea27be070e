// kernels_mf.hip -- mean-field (VILinear) KL + gradient assembly + Adam, the
// generic fused Adam, and the Philox normal generator.
//
// Reference (/root/reference):
//   VIMixin.kl              psvi/models/neural_net.py:101-108 (-> torch
//                           _kl_normal_normal: 0.5(vr + t1 - 1 - log vr))
//   softplus sigma          neural_net.py:133-135, 150-153
//   DifferentiableAdam      psvi/robust_higher/optim.py:299-367
//   hypergrad adam_step     psvi/hypergrad/diff_optimizers.py:184-213
// Gradient: d mu = sum_s dW_s + mu/s0^2,
//   d rho = (sum_s dW_s*eps_s + sp/s0^2 - 1/sp) * sigmoid(rho).
#include <cstdio>
#include <cstdlib>

#include "psvi_internal.hpp"

namespace psvi {

// The shortest decimal that rounds to f (what Python's repr shows): the
// hyperparameters reach the ABI as floats, but the reference forms 1 - beta
// and the bias corrections 1 - beta^t from the Python doubles (0.999, not
// 0.999f = 0.99900001287): 1.f - 0.999f = 0.00099998713 would put a 1.3e-5
// relative error on every (1 - beta2) g^2 term of the second moment.
static double decimal_of(float f) {
    char buf[40];
    for (int digits = 6; digits <= 9; ++digits) {
        std::snprintf(buf, sizeof buf, "%.*g", digits, (double)f);
        const double d = std::strtod(buf, nullptr);
        if ((float)d == f) return d;
    }
    return (double)f;
}

AdamC make_adam(const psvi_adam_hp* hp) {
    AdamC a{};
    const double b1 = decimal_of(hp->beta1), b2 = decimal_of(hp->beta2), lr = decimal_of(hp->lr);
    a.lr = hp->lr;
    a.b1 = hp->beta1;
    a.b2 = hp->beta2;
    a.eps = hp->eps;
    a.omb1 = (float)(1.0 - b1);
    a.omb2 = (float)(1.0 - b2);
    const double bc1 = 1.0 - std::pow(b1, (double)hp->step);
    const double bc2 = 1.0 - std::pow(b2, (double)hp->step);
    a.inv_bc1 = (float)(1.0 / bc1);
    a.inv_sqrt_bc2 = (float)(1.0 / std::sqrt(bc2));
    a.lr_bc1 = (float)(lr / bc1);
    a.inv_bc2 = (float)(1.0 / bc2);
    a.kind = hp->kind;
    return a;
}

struct MfUpdArgs {
    int L;
    int woff[kMaxL + 1];
    int64_t poff[kMaxL];
    int n[kMaxL];
    const float* acc;   // [sum_s dW (n_tot) | sum_s dW*eps (n_tot)]
    int n_tot;
    float* params;
    float* m;
    float* v;
    float* grad_out;
    double* kl_out;
    int include_kl;
    unsigned kl_mask;  // layers carrying a KL term (LeNet: the VILinear layers only)
    float inv_s0sq, log_s0;
    AdamC adam;
    // SLOTS: acc from the plan's gradient slots [S_loc][nz][n_tot] and the
    // step's eps (layer l: weights [S_total][nw], then biases [S_total][dout])
    const float* slots;
    const float* seps;
    int S_loc, nz, s_goff, S_total;
    int64_t eoff[kMaxL];
    int nw[kMaxL], dout[kMaxL];
};

// Fixed-order slot sums for parameter e (layer l, element idx) over the samples
// s = s0, s0 + sstep, ...: g = sum_s sum_c slot[s][c][e], ge = sum_s (sum_c
// slot[s][c][e]) eps_s[idx] -- the net kernel's per-(sample, chunk) gradients
// (VIMixin sampling, neural_net.py:155-162: d mu = sum_s dW_s, d rho via
// sum_s dW_s eps_s).
__device__ __forceinline__ void mf_slot_sums(const MfUpdArgs& a, int l, int idx, int e, int s0,
                                             int sstep, float& g, float& ge) {
    const int nw = a.nw[l];
    const bool wt = idx < nw;
    const float* ep = a.seps + a.eoff[l] + (wt ? idx : (int64_t)a.S_total * nw + (idx - nw));
    const int64_t es = wt ? nw : a.dout[l];
    const size_t ss = (size_t)a.nz * a.n_tot;
    // two samples x the first kC chunks per round as unconditional loads at
    // clamped indices (all in flight together); the sums run in the order
    // s, then c = 0, 1, ... whatever the unroll
    constexpr int kC = 4;
    const int ncl = a.nz < kC ? a.nz : kC;
    g = 0.f;
    ge = 0.f;
    for (int s = s0; s < a.S_loc; s += 2 * sstep) {
        const int sb = s + sstep < a.S_loc ? s + sstep : s;
        float v[2][kC], ev[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int su = u ? sb : s;
            const float* q = a.slots + (size_t)su * ss + e;
#pragma unroll
            for (int c = 0; c < kC; ++c) v[u][c] = q[(size_t)min(c, a.nz - 1) * a.n_tot];
            ev[u] = ep[(int64_t)(a.s_goff + su) * es];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (u && s + sstep >= a.S_loc) break;
            const float* q = a.slots + (size_t)(u ? sb : s) * ss + e;
            float gs = 0.f;
#pragma unroll
            for (int c = 0; c < kC; ++c)
                if (c < ncl) gs += v[u][c];
            for (int c = kC; c < a.nz; ++c) gs += q[(size_t)c * a.n_tot];
            g += gs;
            ge += gs * ev[u];
        }
    }
}

constexpr int kSlotGroups = 16;  // SLOTS: 16 parameters x 16 sample groups per block

template <bool GRAD>
__device__ __forceinline__ void mf_upd(const MfUpdArgs& a, int64_t pidx, float g) {
    if (GRAD) {
        a.grad_out[pidx] = g;
    } else {
        float mm = a.m[pidx], vv = a.v[pidx];
        a.params[pidx] = adam_apply(a.adam, a.params[pidx], g, mm, vv);
        a.m[pidx] = mm;
        a.v[pidx] = vv;
    }
}

// SLOTS: thread (group q, parameter lane) sums samples s = q (mod 16); the
// group partials meet in LDS and group 0 adds them in order q = 0..15.
template <bool GRAD, bool SLOTS>
__global__ __launch_bounds__(256) void mf_update_kernel(MfUpdArgs a) {
    __shared__ float red[8];
    __shared__ float sred[SLOTS ? 2 * 256 : 1];
    const int e = SLOTS ? blockIdx.x * kSlotGroups + (threadIdx.x & (kSlotGroups - 1))
                        : blockIdx.x * blockDim.x + threadIdx.x;
    const int grp = SLOTS ? threadIdx.x / kSlotGroups : 0;
    int l = 0;
    while (l + 1 < a.L && e >= a.woff[l + 1]) ++l;
    const int idx = e - a.woff[l];
    float sg_acc = 0.f, sge_acc = 0.f;
    if (SLOTS) {
        if (e < a.n_tot) mf_slot_sums(a, l, idx, e, grp, kSlotGroups, sg_acc, sge_acc);
        sred[threadIdx.x] = sg_acc;
        sred[256 + threadIdx.x] = sge_acc;
        __syncthreads();
        if (grp == 0) {
            sg_acc = 0.f;
            sge_acc = 0.f;
            for (int q = 0; q < kSlotGroups; ++q) {
                sg_acc += sred[q * kSlotGroups + threadIdx.x];
                sge_acc += sred[256 + q * kSlotGroups + threadIdx.x];
            }
        }
    }
    float klp = 0.f;
    if (e < a.n_tot && grp == 0) {
        const int64_t pmu = a.poff[l] + idx, prho = pmu + a.n[l];
        const float mu = a.params[pmu], rho = a.params[prho];
        const float sp = softplus_f(rho), sg = sigmoid_f(rho);
        float gmu, grho;
        if (SLOTS) {
            gmu = sg_acc;
            grho = sge_acc * sg;
        } else {
            gmu = a.acc[e];
            grho = a.acc[a.n_tot + e] * sg;
        }
        if (a.include_kl && ((a.kl_mask >> l) & 1u)) {
            gmu += mu * a.inv_s0sq;
            grho += (sp * a.inv_s0sq - 1.f / sp) * sg;
            // _kl_normal_normal with q = N(0, s0): 0.5(vr + mu^2/s0^2 - 1 - log vr)
            const float vr = sp * sp * a.inv_s0sq;
            klp = 0.5f * (vr + mu * mu * a.inv_s0sq - 1.f - logf(vr));
        }
        mf_upd<GRAD>(a, pmu, gmu);
        mf_upd<GRAD>(a, prho, grho);
    }
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, red);
        if (threadIdx.x == 0) atomicAdd(a.kl_out, (double)tot);
    }
}

// Reverse of one Adam step (nested trainer: reverse-mode through the unrolled
// inner loop, psvi_classes.py:549-560 differentiated by psvi_elbo.backward()).
// Forward (either variant, adam_apply):  m' = b1 m + (1-b1) g,
//   higher:    v' = b2 v + (1-b2) g^2,          p' = p - lr/bc1 m' / (sqrt(v'+1e-8)/sqrt(bc2) + eps)
//   hypergrad: v' = b2 v + (1-b2) g^2 + 1e-12,  p' = p - lr (m'/bc1) / (sqrt(v'/bc2) + eps)
// Given the adjoints lt, lm, lv of (p', m', v') and the step's m', v', g:
//   lg <- adjoint of g;  lm <- adjoint of m;  lv <- adjoint of v
// (p's adjoint is lt + H^T lg: psvi_hvp).
__global__ __launch_bounds__(256) void adam_adjoint_kernel(int64_t n, const float* lt, float* lm,
                                                           float* lv, const float* m,
                                                           const float* v, const float* g,
                                                           float* lg, AdamC a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float mm = m[i], vv = v[i], t = lt[i];
    float dm, dv;
    if (a.kind == PSVI_ADAM_HIGHER) {
        const float sq = sqrtf(vv + 1e-8f), D = sq * a.inv_sqrt_bc2 + a.eps;
        dm = -t * a.lr_bc1 / D;
        dv = t * a.lr_bc1 * mm / (D * D) * (0.5f * a.inv_sqrt_bc2 / sq);
    } else {
        const float q = sqrtf(vv * a.inv_bc2), D = q + a.eps;
        dm = -t * a.lr * a.inv_bc1 / D;
        dv = t * a.lr * mm * a.inv_bc1 / (D * D) * (0.5f * a.inv_bc2 / fmaxf(q, 1e-30f));
    }
    const float lm2 = lm[i] + dm, lv2 = lv[i] + dv;
    lg[i] = lm2 * a.omb1 + lv2 * 2.f * a.omb2 * g[i];
    lm[i] = a.b1 * lm2;
    lv[i] = a.b2 * lv2;
}

hipError_t launch_adam_adjoint(int64_t n, const float* lt, float* lm, float* lv, const float* m,
                               const float* v, const float* g, float* lg,
                               const psvi_adam_hp* hp, hipStream_t st) {
    const AdamC a = make_adam(hp);
    hipLaunchKernelGGL(adam_adjoint_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n,
                       lt, lm, lv, m, v, g, lg, a);
    return hipGetLastError();
}

static void mf_slot_args(const psvi_plan& p, const float* eps, MfUpdArgs& a) {
    a.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        a.woff[l] = p.lay[l].woff;
        a.poff[l] = p.lay[l].poff;
        a.n[l] = p.lay[l].n;
        a.eoff[l] = p.lay[l].eoff;
        a.nw[l] = p.lay[l].din * p.lay[l].dout;
        a.dout[l] = p.lay[l].dout;
    }
    a.woff[p.L] = p.n_tot;
    a.n_tot = p.n_tot;
    a.slots = p.d_mf_slots;
    a.seps = eps;
    a.S_loc = p.s_cnt[p.rank];
    a.nz = p.mchunks;
    a.s_goff = p.s_off[p.rank];
    a.S_total = p.d.S;
}

// acc = [sum_s dW_s | sum_s dW_s eps_s] from the slots (psvi_mf_phase_accumulate:
// the all-reduced accumulator of the sample-sharded mean-field step)
__global__ __launch_bounds__(256) void mf_slot_acc_kernel(MfUpdArgs a, float* acc) {
    __shared__ float sred[2 * 256];
    const int e = blockIdx.x * kSlotGroups + (threadIdx.x & (kSlotGroups - 1));
    const int grp = threadIdx.x / kSlotGroups;
    int l = 0;
    while (l + 1 < a.L && e >= a.woff[l + 1]) ++l;
    float g = 0.f, ge = 0.f;
    if (e < a.n_tot) mf_slot_sums(a, l, e - a.woff[l], e, grp, kSlotGroups, g, ge);
    sred[threadIdx.x] = g;
    sred[256 + threadIdx.x] = ge;
    __syncthreads();
    if (grp == 0 && e < a.n_tot) {
        g = 0.f;
        ge = 0.f;
        for (int q = 0; q < kSlotGroups; ++q) {
            g += sred[q * kSlotGroups + threadIdx.x];
            ge += sred[256 + q * kSlotGroups + threadIdx.x];
        }
        acc[e] = g;
        acc[a.n_tot + e] = ge;
    }
}

hipError_t launch_mf_slot_acc(const psvi_plan& p, const float* eps, float* acc, hipStream_t st) {
    if (!p.d_mf_slots) return hipErrorInvalidValue;
    MfUpdArgs a{};
    mf_slot_args(p, eps, a);
    hipLaunchKernelGGL(mf_slot_acc_kernel, dim3((p.n_tot + kSlotGroups - 1) / kSlotGroups),
                       dim3(256), 0, st, a, acc);
    return hipGetLastError();
}

hipError_t launch_mf_update(const psvi_plan& p, const float* acc, float* params, float* m,
                            float* v, const psvi_adam_hp* hp, double* kl_out,
                            float* grad_out, int include_kl, hipStream_t st,
                            const float* slot_eps) {
    const bool slots = acc == nullptr;
    if (slots && (!p.d_mf_slots || !slot_eps)) return hipErrorInvalidValue;
    MfUpdArgs a{};
    mf_slot_args(p, slot_eps, a);
    a.woff[p.L] = p.n_tot;
    a.acc = acc;
    a.n_tot = p.n_tot;
    a.params = params;
    a.m = m;
    a.v = v;
    a.grad_out = grad_out;
    a.kl_out = kl_out;
    a.include_kl = include_kl;
    a.kl_mask = p.family == PSVI_FAMILY_LENET ? 0x1Cu : 0xFFu;
    const float s0 = p.d.prior_sd;
    a.inv_s0sq = 1.f / (s0 * s0);
    a.log_s0 = logf(s0);
    if (hp) a.adam = make_adam(hp);
    const int nb = slots ? (p.n_tot + kSlotGroups - 1) / kSlotGroups : (p.n_tot + 255) / 256;
    if (grad_out && slots)
        hipLaunchKernelGGL((mf_update_kernel<true, true>), dim3(nb), dim3(256), 0, st, a);
    else if (grad_out)
        hipLaunchKernelGGL((mf_update_kernel<true, false>), dim3(nb), dim3(256), 0, st, a);
    else if (slots)
        hipLaunchKernelGGL((mf_update_kernel<false, true>), dim3(nb), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((mf_update_kernel<false, false>), dim3(nb), dim3(256), 0, st, a);
    return hipGetLastError();
}

// ------------------------------------------------------------ generic Adam
__global__ __launch_bounds__(256) void adam_kernel(int64_t n, float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m,
                                                   float* __restrict__ v, AdamC a) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        float mm = m[i], vv = v[i];
        p[i] = adam_apply(a, p[i], g[i], mm, vv);
        m[i] = mm;
        v[i] = vv;
    }
}

hipError_t launch_adam(int64_t n, float* p, const float* g, float* m, float* v,
                       const psvi_adam_hp* hp, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nb), dim3(256), 0, st, n, p, g, m, v,
                       make_adam(hp));
    return hipGetLastError();
}

// ----------------------------------------------------- Philox4x32-10 randn
// zero != nullptr: the same launch also clears zero[0, nzero) (the inner
// loop's per-step ELBO accumulators, which the first network launch adds into)
template <bool VEC>
__global__ __launch_bounds__(256) void randn_kernel(float* __restrict__ out, int64_t n,
                                                    uint64_t seed, uint64_t offset,
                                                    double* __restrict__ zero, int64_t nzero) {
    const int64_t nq = (n + 3) / 4;
    const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = gid; i < nzero; i += gs) zero[i] = 0.0;
    for (int64_t q = gid; q < nq; q += gs)
        randn_quad<VEC>(out, n, seed, offset, q);
}

// the same stream, also as the full-cov draw's three bf16 planes (EpsPlanes)
__global__ __launch_bounds__(256) void randn_planes_kernel(float* __restrict__ out, int64_t n,
                                                           uint64_t seed, uint64_t offset,
                                                           double* __restrict__ zero, int64_t nzero,
                                                           EpsPlanes P, uint16_t* __restrict__ planes) {
    const int64_t nq = (n + 3) / 4;
    const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = gid; i < nzero; i += gs) zero[i] = 0.0;
    for (int64_t q = gid; q < nq; q += gs) randn_quad_planes(out, n, seed, offset, q, P, planes);
}

hipError_t launch_randn(float* out, int64_t n, uint64_t seed, uint64_t offset, hipStream_t st,
                        double* zero, int64_t nzero, const EpsPlanes* planes_desc, uint16_t* planes) {
    if (n <= 0 && nzero <= 0) return hipSuccess;
    if (!zero) nzero = 0;
    const int64_t nb = std::max<int64_t>(
        1, std::min<int64_t>(std::max((n + 3) / 4, nzero) / 256 + 1, 4096));
    if (planes && planes_desc) {
        if ((uintptr_t)out & 15) return hipErrorInvalidValue;
        hipLaunchKernelGGL(randn_planes_kernel, dim3((unsigned)nb), dim3(256), 0, st, out, n, seed,
                           offset, zero, nzero, *planes_desc, planes);
        return hipGetLastError();
    }
    if (((uintptr_t)out & 15) == 0)
        hipLaunchKernelGGL(randn_kernel<true>, dim3((unsigned)nb), dim3(256), 0, st, out, n, seed,
                           offset, zero, nzero);
    else
        hipLaunchKernelGGL(randn_kernel<false>, dim3((unsigned)nb), dim3(256), 0, st, out, n,
                           seed, offset, zero, nzero);
    return hipGetLastError();
}

// ------------------------------------------------- non-finite values flag
// flag[0] |= 1 when any of the n values is NaN or +-inf: the device-side check
// that stands in for torch.autograd.set_detect_anomaly (flow_psvi.py:50) on the
// HIP path; one int32 for the host to read once per outer step.
template <typename T>
__global__ __launch_bounds__(256) void nonfinite_kernel(const T* __restrict__ x, int64_t n,
                                                        int32_t* __restrict__ flag) {
    bool bad = false;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        bad |= !isfinite(x[i]);
    if (__any(bad) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(flag, 1);
}

hipError_t launch_nonfinite(const void* x, int64_t n, int dtype, int32_t* flag, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t nb = std::min<int64_t>((n + 255) / 256, 1024);
    if (dtype == 1)
        hipLaunchKernelGGL(nonfinite_kernel<double>, dim3((unsigned)nb), dim3(256), 0, st,
                           (const double*)x, n, flag);
    else
        hipLaunchKernelGGL(nonfinite_kernel<float>, dim3((unsigned)nb), dim3(256), 0, st,
                           (const float*)x, n, flag);
    return hipGetLastError();
}

}  // namespace psvi
