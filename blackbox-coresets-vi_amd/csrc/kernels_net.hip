// kernels_net.hip -- per-(sample, pseudopoint-chunk) MLP forward + weighted NLL
// + hand-derived backward, for both VI families.
//
// Reference (psvi/..., /root/reference):
//   VILinear.forward        models/neural_net.py:176-179   a = h W_s^T + b_s
//   VILinearMultivariateNormal.forward  neural_net.py:485-491 (W_s, b_s split of x_s)
//   ReLU                    make_fcnet 288 / make_fc2net 515
//   Categorical(logits).log_prob(z) .matmul(N f(v))  inference/psvi_classes.py:496-505
// Backward: g = w_m (softmax - onehot); dW_s = g^T h;
// db_s = sum_m g; g <- (g W_s) * 1[a > 0].
//
// One workgroup = one MC sample x one chunk of pseudopoints.  Everything the
// sample needs (its weights, the pseudo-input chunk, every layer's
// activations) is staged in LDS with odd row strides (conflict-free b32
// column walks); the contractions are 4x4 register-tiled VALU FMA chains.
//  MEANFIELD: W_s = mu + softplus(rho) * eps formed in LDS; per-sample dW and
//             dW*eps go to the [sum_s dW | sum_s dW*eps] accumulators
//             (fp32 atomics, S adders per address).
//  FULLCOV:   W_s gathered from x_recv (blocked by source rank); dW written
//             to g_send in the same blocked layout (atomics when the sample's
//             pseudopoints are split over several workgroups).
#include "psvi_internal.hpp"

namespace psvi {

struct NetArgs {
    int L, M, mc, S_total, s_goff, atomic_g;
    int din[kMaxL], dout[kMaxL], woff[kMaxL];
    // LDS carve (float offsets) and row strides
    int lw[kMaxL], ldw[kMaxL], lb[kMaxL], le[kMaxL], leb[kMaxL], la[kMaxL], lda[kMaxL];
    int lu, ldu, lred;
    const float* u;
    const int32_t* z;
    const float* w;
    float* nll_out;
    // MEANFIELD
    const float* params;
    const float* eps;
    int64_t poff[kMaxL], eoff[kMaxL];
    float* accMu;
    float* accRho;
    // FULLCOV (blocked by source rank)
    const float* xrecv;
    float* gsend;
    int nsrc;
    int64_t src_base[kMaxWorld];
    int src_stride[kMaxWorld];
    int src_lo[kMaxWorld][kMaxL], src_hi[kMaxWorld][kMaxL], src_col[kMaxWorld][kMaxL];
};

// C[p][q] = sum_k A(p,k) B(q,k), A(p,k)=A[p*sap+k*sak], B(q,k)=B[q*sbq+k*sbk].
// Thread t owns p in {pt + i*tp}, q in {qt + j*tq}: consecutive lanes walk
// consecutive q, so unit-stride operands are conflict-free.
template <bool RELU_A, bool RELU_B, class Epi>
__device__ __forceinline__ void lds_gemm(int P, int Q, int K, const float* __restrict__ A,
                                         int sap, int sak, const float* __restrict__ B,
                                         int sbq, int sbk, Epi epi) {
    const int tp = (P + 3) >> 2, tq = (Q + 3) >> 2;
    for (int t = threadIdx.x; t < tp * tq; t += blockDim.x) {
        const int pt = t / tq, qt = t - pt * tq;
        const float* Ap[4];
        const float* Bp[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            Ap[i] = A + min(pt + i * tp, P - 1) * sap;
            Bp[i] = B + min(qt + i * tq, Q - 1) * sbq;
        }
        float acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
        for (int k = 0; k < K; ++k) {
            float av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                av[i] = Ap[i][k * sak];
                if (RELU_A) av[i] = fmaxf(av[i], 0.f);
                bv[i] = Bp[i][k * sbk];
                if (RELU_B) bv[i] = fmaxf(bv[i], 0.f);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int p = pt + i * tp, q = qt + j * tq;
                if (p < P && q < Q) epi(p, q, acc[i][j]);
            }
    }
}

// FULLCOV: address in x_recv / g_send of row r of layer l for local sample s.
__device__ __forceinline__ int64_t fc_addr(const NetArgs& a, int l, int r, int s) {
    int p = 0;
    while (p + 1 < a.nsrc && r >= a.src_hi[p][l]) ++p;
    return a.src_base[p] + (int64_t)s * a.src_stride[p] + a.src_col[p][l] + (r - a.src_lo[p][l]);
}

template <int FAM>
__global__ __launch_bounds__(256) void net_kernel(NetArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int s = blockIdx.x;                 // local sample
    const int sg = a.s_goff + s;              // global sample (eps indexing)
    const int m0 = blockIdx.y * a.mc;
    const int mcnt = min(a.mc, a.M - m0);
    const int L = a.L;

    // ---- 1. this sample's weights into LDS ------------------------------
    for (int l = 0; l < L; ++l) {
        const int din = a.din[l], dout = a.dout[l], nw = din * dout, n = nw + dout;
        float* W = sm + a.lw[l];
        float* Bv = sm + a.lb[l];
        if (FAM == PSVI_FAMILY_MEANFIELD) {
            const float* mu = a.params + a.poff[l];
            const float* rho = mu + n;
            const float* eW = a.eps + a.eoff[l] + (int64_t)sg * nw;
            const float* eB = a.eps + a.eoff[l] + (int64_t)a.S_total * nw + (int64_t)sg * dout;
            float* E = sm + a.le[l];
            float* EB = sm + a.leb[l];
            for (int idx = threadIdx.x; idx < n; idx += blockDim.x) {
                const float e = idx < nw ? eW[idx] : eB[idx - nw];
                // Normal.rsample: loc + eps * scale (torch/distributions/normal.py)
                const float val = mu[idx] + e * softplus_f(rho[idx]);
                if (idx < nw) {
                    const int j = idx / din, i = idx - j * din;
                    W[j * a.ldw[l] + i] = val;
                    E[j * a.ldw[l] + i] = e;
                } else {
                    Bv[idx - nw] = val;
                    EB[idx - nw] = e;
                }
            }
        } else {
            for (int p = 0; p < a.nsrc; ++p) {
                const int lo = a.src_lo[p][l], hi = a.src_hi[p][l];
                const float* src = a.xrecv + a.src_base[p] + (int64_t)s * a.src_stride[p] +
                                   a.src_col[p][l] - lo;
                for (int r = lo + threadIdx.x; r < hi; r += blockDim.x) {
                    const float val = src[r];
                    if (r < nw) {
                        const int j = r / din, i = r - j * din;
                        W[j * a.ldw[l] + i] = val;
                    } else {
                        Bv[r - nw] = val;
                    }
                }
            }
        }
    }
    // ---- 2. pseudo-input chunk -------------------------------------------
    {
        const int D = a.din[0];
        float* U = sm + a.lu;
        for (int idx = threadIdx.x; idx < mcnt * D; idx += blockDim.x) {
            const int m = idx / D, i = idx - m * D;
            U[m * a.ldu + i] = a.u[(int64_t)(m0 + m) * D + i];
        }
    }
    __syncthreads();

    // ---- 3. forward --------------------------------------------------------
    for (int l = 0; l < L; ++l) {
        const float* H = l == 0 ? sm + a.lu : sm + a.la[l - 1];
        const int ldh = l == 0 ? a.ldu : a.lda[l - 1];
        float* Aout = sm + a.la[l];
        const int ldo = a.lda[l];
        const float* Bv = sm + a.lb[l];
        auto epi = [&](int m, int j, float acc) { Aout[m * ldo + j] = acc + Bv[j]; };
        if (l == 0)
            lds_gemm<false, false>(mcnt, a.dout[l], a.din[l], H, ldh, 1, sm + a.lw[l], a.ldw[l],
                                   1, epi);
        else
            lds_gemm<true, false>(mcnt, a.dout[l], a.din[l], H, ldh, 1, sm + a.lw[l], a.ldw[l],
                                  1, epi);
        __syncthreads();
    }

    // ---- 4. weighted NLL, dlogits ------------------------------------------
    {
        const int C = a.dout[L - 1];
        float* G = sm + a.la[L - 1];
        const int ldg = a.lda[L - 1];
        float part = 0.f;
        for (int m = threadIdx.x; m < mcnt; m += blockDim.x) {
            float* row = G + m * ldg;
            float mx = row[0];
            for (int k = 1; k < C; ++k) mx = fmaxf(mx, row[k]);
            float se = 0.f;
            for (int k = 0; k < C; ++k) se += __expf(row[k] - mx);
            const float lse = mx + __logf(se);
            const int zm = a.z[m0 + m];
            const float wm = a.w[m0 + m];
            part += wm * (lse - row[zm]);
            for (int k = 0; k < C; ++k) {
                const float pk = __expf(row[k] - lse);
                row[k] = wm * (pk - (k == zm ? 1.f : 0.f));
            }
        }
        const float tot = block_sum(part, sm + a.lred);
        if (threadIdx.x == 0) atomicAdd(a.nll_out, tot);
        __syncthreads();
    }

    // ---- 5. backward -------------------------------------------------------
    for (int l = L - 1; l >= 0; --l) {
        const int din = a.din[l], dout = a.dout[l], nw = din * dout;
        const float* G = sm + a.la[l];
        const int ldg = a.lda[l];
        const float* H = l == 0 ? sm + a.lu : sm + a.la[l - 1];
        const int ldh = l == 0 ? a.ldu : a.lda[l - 1];
        // dW[j][i] = sum_m g[m][j] h[m][i]
        if (FAM == PSVI_FAMILY_MEANFIELD) {
            float* accMu = a.accMu + a.woff[l];
            float* accRho = a.accRho + a.woff[l];
            const float* E = sm + a.le[l];
            const int ldw = a.ldw[l];
            auto epi = [&](int j, int i, float dw) {
                atomicAdd(accMu + j * din + i, dw);
                atomicAdd(accRho + j * din + i, dw * E[j * ldw + i]);
            };
            if (l == 0)
                lds_gemm<false, false>(dout, din, mcnt, G, 1, ldg, H, 1, ldh, epi);
            else
                lds_gemm<false, true>(dout, din, mcnt, G, 1, ldg, H, 1, ldh, epi);
            const float* EB = sm + a.leb[l];
            for (int j = threadIdx.x; j < dout; j += blockDim.x) {
                float db = 0.f;
                for (int m = 0; m < mcnt; ++m) db += G[m * ldg + j];
                atomicAdd(accMu + nw + j, db);
                atomicAdd(accRho + nw + j, db * EB[j]);
            }
        } else {
            const bool at = a.atomic_g != 0;
            auto epi = [&](int j, int i, float dw) {
                float* dst = a.gsend + fc_addr(a, l, j * din + i, s);
                if (at) atomicAdd(dst, dw); else *dst = dw;
            };
            if (l == 0)
                lds_gemm<false, false>(dout, din, mcnt, G, 1, ldg, H, 1, ldh, epi);
            else
                lds_gemm<false, true>(dout, din, mcnt, G, 1, ldg, H, 1, ldh, epi);
            for (int j = threadIdx.x; j < dout; j += blockDim.x) {
                float db = 0.f;
                for (int m = 0; m < mcnt; ++m) db += G[m * ldg + j];
                float* dst = a.gsend + fc_addr(a, l, nw + j, s);
                if (at) atomicAdd(dst, db); else *dst = db;
            }
        }
        if (l == 0) break;
        __syncthreads();  // dW read h_{l-1}; g_{l-1} overwrites it in place
        {
            float* Hp = sm + a.la[l - 1];
            const int ldp = a.lda[l - 1];
            auto epi = [&](int m, int i, float acc) {
                float* e = Hp + m * ldp + i;
                *e = *e > 0.f ? acc : 0.f;
            };
            // g_{l-1}[m][i] = sum_j g[m][j] W[j][i]
            lds_gemm<false, false>(mcnt, din, dout, G, ldg, 1, sm + a.lw[l], 1, a.ldw[l], epi);
        }
        __syncthreads();
    }
}

static inline int odd_ld(int x) { return (x & 1) ? x : x + 1; }

// LDS floats needed for a chunk of `mc` points.
static size_t net_lds_floats(const psvi_plan& p, int mc, NetArgs* a) {
    size_t off = 0;
    auto take = [&](size_t nfl) {
        size_t o = off;
        off += (nfl + 3) & ~size_t(3);  // keep 16-B alignment of every region
        return (int)o;
    };
    for (int l = 0; l < p.L; ++l) {
        const int din = p.lay[l].din, dout = p.lay[l].dout;
        const int ldw = odd_ld(din);
        if (a) a->ldw[l] = ldw;
        int lw = take((size_t)dout * ldw), lb = take(dout);
        int le = 0, leb = 0;
        if (p.family == PSVI_FAMILY_MEANFIELD) {
            le = take((size_t)dout * ldw);
            leb = take(dout);
        }
        const int lda = odd_ld(dout);
        int la = take((size_t)mc * lda);
        if (a) {
            a->lw[l] = lw; a->lb[l] = lb; a->le[l] = le; a->leb[l] = leb;
            a->la[l] = la; a->lda[l] = lda;
        }
    }
    const int ldu = odd_ld(p.lay[0].din);
    int lu = take((size_t)mc * ldu);
    int lred = take(16);
    if (a) { a->lu = lu; a->ldu = ldu; a->lred = lred; }
    return off;
}

size_t net_plan_geometry(psvi_plan& p) {
    // Enough workgroups to cover the CUs, and LDS <= 80 KiB (2 WGs / CU)
    // when possible, <= 160 KiB always.
    const int S_local = p.s_cnt[p.rank];
    const int M = p.d.M;
    int mchunks = 1;
    while (S_local * mchunks < 256 && (M + mchunks) / (mchunks + 1) >= 16) ++mchunks;
    for (;;) {
        const int mc = (M + mchunks - 1) / mchunks;
        const size_t bytes = net_lds_floats(p, mc, nullptr) * 4;
        if (bytes <= 80 * 1024 || (bytes <= 160 * 1024 && mc <= 16) || mc == 1) {
            p.mchunks = (M + mc - 1) / mc;
            p.mc = mc;
            p.net_lds = bytes;
            return bytes;
        }
        ++mchunks;
    }
}

void net_set_lds_limit() {
    // gfx950: up to 160 KiB of LDS per workgroup
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_MEANFIELD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

hipError_t launch_net(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                      const float* params, const float* eps, float* accMu, float* accRho,
                      const float* xrecv, float* gsend, float* nll_out, hipStream_t st) {
    NetArgs a{};
    a.L = p.L;
    a.M = p.d.M;
    a.mc = p.mc;
    a.S_total = p.d.S;
    a.s_goff = p.s_off[p.rank];
    a.atomic_g = p.mchunks > 1;
    for (int l = 0; l < p.L; ++l) {
        a.din[l] = p.lay[l].din;
        a.dout[l] = p.lay[l].dout;
        a.woff[l] = p.lay[l].woff;
        a.poff[l] = p.lay[l].poff;
        a.eoff[l] = p.lay[l].eoff;
    }
    net_lds_floats(p, p.mc, &a);
    a.u = u; a.z = z; a.w = w; a.nll_out = nll_out;
    a.params = params; a.eps = eps; a.accMu = accMu; a.accRho = accRho;
    a.xrecv = xrecv; a.gsend = gsend;
    if (p.family == PSVI_FAMILY_FULLCOV) {
        const int S_local = p.s_cnt[p.rank];
        a.nsrc = p.world;
        int64_t base = 0;
        for (int q = 0; q < p.world; ++q) {
            a.src_base[q] = base;
            a.src_stride[q] = p.rows_tot[q];
            for (int l = 0; l < p.L; ++l) {
                a.src_lo[q][l] = p.row_lo[q][l];
                a.src_hi[q][l] = p.row_hi[q][l];
                a.src_col[q][l] = p.xcol_l[q][l];
            }
            base += (int64_t)S_local * p.rows_tot[q];
        }
    }
    dim3 grid(p.s_cnt[p.rank], p.mchunks), block(256);
    if (p.s_cnt[p.rank] == 0) return hipSuccess;
    if (p.family == PSVI_FAMILY_MEANFIELD)
        hipLaunchKernelGGL(net_kernel<PSVI_FAMILY_MEANFIELD>, grid, block, p.net_lds, st, a);
    else
        hipLaunchKernelGGL(net_kernel<PSVI_FAMILY_FULLCOV>, grid, block, p.net_lds, st, a);
    return hipGetLastError();
}

}  // namespace psvi
