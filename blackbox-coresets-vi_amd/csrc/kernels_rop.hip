// kernels_rop.hip -- Hessian-vector products of the inner ELBO (psvi_hvp) for
// hypergrad's CG_normaleq (the `hyper` trainer's implicit hypergradient).
//
// Reference (/root/reference):
//   PSVI.hyper_step            psvi/inference/psvi_classes.py:602-687
//   CG_normaleq / jvp / grd    psvi/hypergrad/hypergradients.py:199-244, 300-311
//   GradientDescent fp_map     psvi/hypergrad/diff_optimizers.py:51-60, 157-159
// The reference differentiates autograd's gradient graph a second time; here
// the product is forward-over-reverse (Pearlmutter's R-op) at fixed eps:
//   tangent sample    x_dot_s = J_s vec  (full-cov: v_mean + Lv eps_s with
//                     Lv = diag(sigmoid(sd) v_sd) + lower(v_corr); mean-field:
//                     v_mu + sigmoid(rho) v_rho eps_s)
//   tangent forward   a_dot = h_dot W^T + h W_dot^T + b_dot, h_dot = 1[a>0] a_dot
//   head              delta = w_m (p - onehot), delta_dot = w_m p (a_dot - p.a_dot),
//                     NLL_dot = (p - onehot).a_dot
//   R-backward        dW_dot = delta_dot^T h + delta^T h_dot,
//                     delta_dot' = (delta_dot W + delta W_dot) 1[a>0]
// (net_rop_kernel: one workgroup per sample, rows in chunks, VALU), then the
// reparameterised backward of G_dot (the update kernel's gradient mode for
// full-cov), the softplus curvature sum_s (G_s . eps_s) sigmoid'(sd) v_sd and
// the KL Hessian (hvp_assemble_kernel).  The mixed products the hypergradient
// needs come out of the same pass: d/du (vec . grad) = sum_s delta_dot_0 W +
// delta_0 W_dot, d/dw_m (vec . grad) = sum_s NLL_dot_sm.
#include <algorithm>

#include "psvi_internal.hpp"

namespace psvi {

struct RopArgs {
    int L, M, S, n_tot, family, rc, maxd;
    int nsplit;  // workgroups per sample (row halves); 2: G / G_dot added onto zeroed buffers,
                 // two addends, so the sum is exact-order independent
    int din[kMaxL], dout[kMaxL], woff[kMaxL];
    int64_t poff[kMaxL], eoff[kMaxL];
    int lx, lxd, lg, lgd, lh[kMaxL + 1], lhd[kMaxL + 1], ld0, ld1, ldd0, ldd1;  // LDS carve
    // W_l / W_dot_l in LDS: rows of an odd stride ldw[l] (a lane per output row
    // then hits its own bank), layer l at xo[l] of the X / XD regions, b after W
    int ldw[kMaxL], xo[kMaxL];
    const float* u;
    const int32_t* z;
    const float* w;
    const float* x;    // full-cov: x_s   [S][n_tot]
    const float* xd;   // full-cov: x_dot [S][n_tot]
    const float* params;
    const float* vec;
    const float* eps;
    float* G;          // [S][n_tot]
    float* Gd;         // [S][n_tot]
    float* du;         // [S][M][D]
    float* nlld;       // [S][M]
};

__global__ __launch_bounds__(512) void net_rop_kernel(RopArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const int L = a.L, D = a.din[0], C = a.dout[L - 1];
    float* X = sm + a.lx;
    float* XD = sm + a.lxd;
    float* GA = sm + a.lg;
    float* GDA = sm + a.lgd;
    // sampled weights and their tangents, in the per-sample weight layout
    // (layer l at woff_l: W row-major [dout][din], then b)
    for (int l = 0; l < L; ++l) {
        const int din = a.din[l], dout = a.dout[l], n = din * dout + dout, nw = din * dout;
        for (int i = tid; i < n; i += nt) {
            const int o = a.woff[l] + i;
            float xv, xdv;
            if (a.family == PSVI_FAMILY_FULLCOV) {
                xv = a.x[(int64_t)s * a.n_tot + o];
                xdv = a.xd[(int64_t)s * a.n_tot + o];
            } else {
                const float e = i < nw ? a.eps[a.eoff[l] + (int64_t)s * nw + i]
                                       : a.eps[a.eoff[l] + (int64_t)a.S * nw + (int64_t)s * dout + i - nw];
                const int64_t pm = a.poff[l] + i, pr = pm + n;
                const float rho = a.params[pr];
                xv = a.params[pm] + softplus_f(rho) * e;
                xdv = a.vec[pm] + sigmoid_f(rho) * a.vec[pr] * e;
            }
            const int dst = a.xo[l] + (i < nw ? (i / din) * a.ldw[l] + i % din
                                              : dout * a.ldw[l] + (i - nw));
            X[dst] = xv;
            XD[dst] = xdv;
            GA[o] = 0.f;
            GDA[o] = 0.f;
        }
    }
    __syncthreads();
    const int rows_per = (a.M + a.nsplit - 1) / a.nsplit;
    const int m_lo = blockIdx.y * rows_per, m_hi = min(a.M, m_lo + rows_per);
    for (int m0 = m_lo; m0 < m_hi; m0 += a.rc) {
        const int rc = min(a.rc, m_hi - m0);
        // inputs: h_0 = u rows, h_dot_0 = 0
        for (int i = tid; i < rc * D; i += nt) {
            sm[a.lh[0] + i] = a.u[(int64_t)m0 * D + i];
            sm[a.lhd[0] + i] = 0.f;
        }
        __syncthreads();
        // forward + tangent forward
        for (int l = 0; l < L; ++l) {
            const int din = a.din[l], dout = a.dout[l], ldw = a.ldw[l];
            const float* W = X + a.xo[l];
            const float* Wd = XD + a.xo[l];
            const float* b = W + dout * ldw;
            const float* bd = Wd + dout * ldw;
            const float* H = sm + a.lh[l];
            const float* HD = sm + a.lhd[l];
            float* Hn = sm + a.lh[l + 1];
            float* HDn = sm + a.lhd[l + 1];
            for (int q = tid; q < rc * dout; q += nt) {
                const int m = q / dout, o = q - m * dout;
                float acc = b[o], accd = bd[o];
                for (int i = 0; i < din; ++i) {
                    const float h = H[m * din + i], hd = HD[m * din + i];
                    const float wv = W[o * ldw + i];
                    acc = fmaf(h, wv, acc);
                    accd = fmaf(hd, wv, fmaf(h, Wd[o * ldw + i], accd));
                }
                if (l < L - 1) {
                    Hn[q] = acc > 0.f ? acc : 0.f;
                    HDn[q] = acc > 0.f ? accd : 0.f;
                } else {
                    Hn[q] = acc;
                    HDn[q] = accd;
                }
            }
            __syncthreads();
        }
        // head: delta = w (p - onehot), delta_dot = w p (a_dot - p.a_dot)
        float* Dl = sm + a.ld0;
        float* DDl = sm + a.ldd0;
        float* Dn = sm + a.ld1;
        float* DDn = sm + a.ldd1;
        for (int m = tid; m < rc; m += nt) {
            const float* lg = sm + a.lh[L] + m * C;
            const float* ld = sm + a.lhd[L] + m * C;
            const int zm = a.z[m0 + m];
            const float wm = a.w[m0 + m];
            float mx = -INFINITY;
            for (int c = 0; c < C; ++c) mx = fmaxf(mx, lg[c]);
            float se = 0.f;
            for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
            const float lse = mx + logf(se);
            float pad = 0.f, nd = 0.f;
            for (int c = 0; c < C; ++c) pad += expf(lg[c] - lse) * ld[c];
            for (int c = 0; c < C; ++c) {
                const float p = expf(lg[c] - lse);
                const float pmo = p - (c == zm ? 1.f : 0.f);
                nd = fmaf(pmo, ld[c], nd);
                Dl[m * a.maxd + c] = wm * pmo;
                DDl[m * a.maxd + c] = wm * p * (ld[c] - pad);
            }
            if (a.nlld) a.nlld[(int64_t)s * a.M + m0 + m] = nd;
        }
        __syncthreads();
        // R-backward
        for (int l = L - 1; l >= 0; --l) {
            const int din = a.din[l], dout = a.dout[l], nw = din * dout, ldw = a.ldw[l];
            const float* W = X + a.xo[l];
            const float* Wd = XD + a.xo[l];
            const float* H = sm + a.lh[l];
            const float* HD = sm + a.lhd[l];
            float* GW = GA + a.woff[l];
            float* GDW = GDA + a.woff[l];
            for (int q = tid; q < nw + dout; q += nt) {
                if (q < nw) {
                    const int o = q / din, i = q - o * din;
                    float g = 0.f, gd = 0.f;
                    for (int m = 0; m < rc; ++m) {
                        const float dl = Dl[m * a.maxd + o], ddl = DDl[m * a.maxd + o];
                        const float h = H[m * din + i];
                        g = fmaf(dl, h, g);
                        gd = fmaf(ddl, h, fmaf(dl, HD[m * din + i], gd));
                    }
                    GW[q] += g;
                    GDW[q] += gd;
                } else {
                    const int o = q - nw;
                    float g = 0.f, gd = 0.f;
                    for (int m = 0; m < rc; ++m) {
                        g += Dl[m * a.maxd + o];
                        gd += DDl[m * a.maxd + o];
                    }
                    GW[q] += g;
                    GDW[q] += gd;
                }
            }
            if (l > 0 || a.du) {
                // delta' = (delta W) 1[h > 0]   (h = relu(a_{l-1}); none at the input)
                for (int q = tid; q < rc * din; q += nt) {
                    const int m = q / din, i = q - m * din;
                    float t = 0.f, td = 0.f;
                    for (int o = 0; o < dout; ++o) {
                        const float dl = Dl[m * a.maxd + o], ddl = DDl[m * a.maxd + o];
                        const float wv = W[o * ldw + i];
                        t = fmaf(dl, wv, t);
                        td = fmaf(ddl, wv, fmaf(dl, Wd[o * ldw + i], td));
                    }
                    if (l > 0) {
                        const bool on = H[q] > 0.f;
                        Dn[m * a.maxd + i] = on ? t : 0.f;
                        DDn[m * a.maxd + i] = on ? td : 0.f;
                    } else {
                        a.du[((int64_t)s * a.M + m0 + m) * D + i] = td;
                    }
                }
            }
            __syncthreads();
            float* t0 = Dl; Dl = Dn; Dn = t0;
            float* t1 = DDl; DDl = DDn; DDn = t1;
        }
    }
    for (int o = tid; o < a.n_tot; o += nt) {
        if (a.nsplit == 1) {
            a.G[(int64_t)s * a.n_tot + o] = GA[o];
            a.Gd[(int64_t)s * a.n_tot + o] = GDA[o];
        } else {
            atomicAdd(a.G + (int64_t)s * a.n_tot + o, GA[o]);
            atomicAdd(a.Gd + (int64_t)s * a.n_tot + o, GDA[o]);
        }
    }
}

// full-cov tangent parameters: vec with the sd slots scaled by sigmoid(sd),
// so the sample phase (raw diagonal) yields x_dot = v_mean + Lv eps
__global__ __launch_bounds__(256) void hvp_tangent_kernel(RopArgs a, float* T) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.n_tot) return;
    int l = 0;
    while (l + 1 < a.L && e >= a.woff[l + 1]) ++l;
    const int n = a.din[l] * a.dout[l] + a.dout[l];
    const int64_t ps = a.poff[l] + n + (e - a.woff[l]);
    T[ps] = sigmoid_f(a.params[ps]) * a.vec[ps];
}

// Hv assembly.  Index space: [0, n_tot) mean / sd terms, then (full-cov) the
// corr prior terms, then d_u (M x D), then d_w (M).
__global__ __launch_bounds__(256) void hvp_assemble_kernel(RopArgs a, float* hv, float* d_u,
                                                           float* d_w, int64_t ncorr_tot,
                                                           float inv_s0sq, float klw) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int D = a.din[0];
    // klw = 0: a sample shard's partial product without the KL Hessian
    const float kls = klw * inv_s0sq;
    if (i < a.n_tot) {
        const int e = (int)i;
        int l = 0;
        while (l + 1 < a.L && e >= a.woff[l + 1]) ++l;
        const int n = a.din[l] * a.dout[l] + a.dout[l], k = e - a.woff[l], nw = n - a.dout[l];
        const int64_t pm = a.poff[l] + k, ps = pm + n;
        float gd = 0.f, gde = 0.f, ge = 0.f;
        for (int s = 0; s < a.S; ++s) {
            float ev;
            if (a.family == PSVI_FAMILY_FULLCOV)
                ev = a.eps[a.eoff[l] + (int64_t)s * n + k];
            else
                ev = k < nw ? a.eps[a.eoff[l] + (int64_t)s * nw + k]
                            : a.eps[a.eoff[l] + (int64_t)a.S * nw + (int64_t)s * a.dout[l] + k - nw];
            const float g = a.G[(int64_t)s * a.n_tot + e], gdv = a.Gd[(int64_t)s * a.n_tot + e];
            ge = fmaf(g, ev, ge);
            gd += gdv;
            gde = fmaf(gdv, ev, gde);
        }
        const float r = a.params[ps], sp = softplus_f(r), sg = sigmoid_f(r);
        const float vsd = a.vec[ps];
        const float kl2 = klw * ((1.f / (sp * sp) + inv_s0sq) * sg * sg + (sp * inv_s0sq - 1.f / sp) * sg * (1.f - sg));
        const float curv = ge * sg * (1.f - sg) * vsd + kl2 * vsd;
        if (a.family == PSVI_FAMILY_FULLCOV) {
            // the update kernel's gradient mode already wrote sum G_dot, diag(G_dot^T E) sg
            hv[pm] += a.vec[pm] * kls;
            hv[ps] += curv;
        } else {
            hv[pm] = gd + a.vec[pm] * kls;
            hv[ps] = gde * sg + curv;
        }
        return;
    }
    int64_t j = i - a.n_tot;
    if (j < ncorr_tot) {
        // corr prior: + v_corr / s0^2 (layers' corr blocks in order)
        int64_t base = 0;
        for (int l = 0; l < a.L; ++l) {
            const int n = a.din[l] * a.dout[l] + a.dout[l];
            const int64_t nc = (int64_t)(n - 1) * (n - 2) / 2;
            if (j < base + nc) {
                const int64_t pc = a.poff[l] + 2 * n + (j - base);
                hv[pc] += a.vec[pc] * kls;
                return;
            }
            base += nc;
        }
        return;
    }
    j -= ncorr_tot;
    if (j < (int64_t)a.M * D) {
        if (d_u) {
            float t = 0.f;
            for (int s = 0; s < a.S; ++s) t += a.du[(int64_t)s * a.M * D + j];
            d_u[j] = t;
        }
        return;
    }
    j -= (int64_t)a.M * D;
    if (j < a.M && d_w) {
        float t = 0.f;
        for (int s = 0; s < a.S; ++s) t += a.nlld[(int64_t)s * a.M + j];
        d_w[j] = t;
    }
}

static int rup4(int x) { return (x + 3) & ~3; }

// LDS carve for rows in chunks of rc; returns floats
static size_t rop_carve(const psvi_plan& p, int rc, RopArgs* a) {
    size_t off = 0;
    auto take = [&](size_t nfl) {
        const size_t o = off;
        off += (nfl + 3) & ~size_t(3);
        return (int)o;
    };
    int maxd = 0;
    for (int l = 0; l < p.L; ++l) maxd = std::max(maxd, std::max(p.lay[l].din, p.lay[l].dout));
    maxd = rup4(maxd) | 1;  // odd row stride of the delta buffers
    int xo[kMaxL], ldw[kMaxL], xtot = 0;
    for (int l = 0; l < p.L; ++l) {
        ldw[l] = p.lay[l].din | 1;
        xo[l] = xtot;
        xtot += p.lay[l].dout * ldw[l] + p.lay[l].dout;
    }
    const int lx = take(xtot), lxd = take(xtot), lg = take(p.n_tot), lgd = take(p.n_tot);
    int lh[kMaxL + 1], lhd[kMaxL + 1];
    for (int l = 0; l <= p.L; ++l) {
        const int d = l < p.L ? p.lay[l].din : p.lay[p.L - 1].dout;
        lh[l] = take((size_t)rc * d);
        lhd[l] = take((size_t)rc * d);
    }
    const int ld0 = take((size_t)rc * maxd), ld1 = take((size_t)rc * maxd);
    const int ldd0 = take((size_t)rc * maxd), ldd1 = take((size_t)rc * maxd);
    if (a) {
        a->lx = lx; a->lxd = lxd; a->lg = lg; a->lgd = lgd;
        for (int l = 0; l < p.L; ++l) { a->xo[l] = xo[l]; a->ldw[l] = ldw[l]; }
        for (int l = 0; l <= p.L; ++l) { a->lh[l] = lh[l]; a->lhd[l] = lhd[l]; }
        a->ld0 = ld0; a->ld1 = ld1; a->ldd0 = ldd0; a->ldd1 = ldd1;
        a->maxd = maxd;
        a->rc = rc;
    }
    return off;
}

constexpr size_t kRopLds = 160 * 1024;

// rows per chunk that fit the LDS (0: the model's weights alone do not fit)
int rop_rows(const psvi_plan& p) {
    for (int rc = 64; rc >= 1; rc >>= 1)
        if (rop_carve(p, rc, nullptr) * 4 <= kRopLds) return rc;
    return 0;
}

static void rop_fill(const psvi_plan& p, RopArgs& a) {
    a.L = p.L;
    a.M = p.d.M;
    a.S = p.d.S;
    a.n_tot = p.n_tot;
    a.family = p.family;
    for (int l = 0; l < p.L; ++l) {
        a.din[l] = p.lay[l].din;
        a.dout[l] = p.lay[l].dout;
        a.woff[l] = p.lay[l].woff;
        a.poff[l] = p.lay[l].poff;
        a.eoff[l] = p.lay[l].eoff;
    }
}

hipError_t launch_hvp_tangent(const psvi_plan& p, const float* params, const float* vec,
                              float* T, hipStream_t st) {
    RopArgs a{};
    rop_fill(p, a);
    a.params = params;
    a.vec = vec;
    hipError_t e = hipMemcpyAsync(T, vec, sizeof(float) * (size_t)p.P, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(hvp_tangent_kernel, dim3((p.n_tot + 255) / 256), dim3(256), 0, st, a, T);
    return hipGetLastError();
}

hipError_t launch_net_rop(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                          const float* x, const float* xd, const float* params, const float* vec,
                          const float* eps, float* G, float* Gd, float* du, float* nlld,
                          hipStream_t st) {
    static bool once = [] {
        (void)hipFuncSetAttribute((const void*)net_rop_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRopLds);
        return true;
    }();
    (void)once;
    RopArgs a{};
    rop_fill(p, a);
    const int rc = rop_rows(p);
    if (rc == 0) return hipErrorInvalidValue;
    const size_t lds = rop_carve(p, rc, &a) * 4;
    a.u = u; a.z = z; a.w = w; a.x = x; a.xd = xd;
    a.params = params; a.vec = vec; a.eps = eps;
    a.G = G; a.Gd = Gd; a.du = du; a.nlld = nlld;
    // two workgroups per sample while the samples alone leave CUs idle
    a.nsplit = (p.d.S < 256 && p.d.M > 1) ? 2 : 1;
    if (a.nsplit > 1) {
        const size_t bytes = sizeof(float) * (size_t)p.d.S * p.n_tot;
        hipError_t e = hipMemsetAsync(G, 0, bytes, st);
        if (e == hipSuccess) e = hipMemsetAsync(Gd, 0, bytes, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(net_rop_kernel, dim3(p.d.S, a.nsplit), dim3(512), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_hvp_assemble(const psvi_plan& p, const float* params, const float* vec,
                               const float* eps, const float* G, const float* Gd, const float* du,
                               const float* nlld, float* hv, float* d_u, float* d_w,
                               hipStream_t st, bool include_kl) {
    RopArgs a{};
    rop_fill(p, a);
    a.params = params; a.vec = vec; a.eps = eps;
    a.G = const_cast<float*>(G);
    a.Gd = const_cast<float*>(Gd);
    a.du = const_cast<float*>(du);
    a.nlld = const_cast<float*>(nlld);
    int64_t nct = 0;
    if (p.family == PSVI_FAMILY_FULLCOV)
        for (int l = 0; l < p.L; ++l) nct += p.lay[l].nc;
    const int64_t total = p.n_tot + nct + (int64_t)p.d.M * p.lay[0].din + p.d.M;
    const float s0 = p.d.prior_sd;
    hipLaunchKernelGGL(hvp_assemble_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       st, a, hv, d_u, d_w, nct, 1.f / (s0 * s0), include_kl ? 1.f : 0.f);
    return hipGetLastError();
}

}  // namespace psvi
