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
// activations) is staged in LDS with odd row strides; the per-sample
// contractions run on fp32 MFMA (16x16x4) tiles.
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
    double* nll_out;   // fp64 accumulator (many similar-size adds)
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

typedef float floatx4 __attribute__((ext_vector_type(4)));

// C[p][q] = sum_k A(p,k) B(q,k), A(p,k)=A[p*sap+k*sak], B(q,k)=B[q*sbq+k*sbk],
// all operands in LDS.  16x16 output tiles on v_mfma_f32_16x16x4_f32 (exact
// fp32), dealt round-robin to the workgroup's waves; lane l feeds
// A[p0 + (l&15)][k + (l>>4)] and B[q0 + (l&15)][k + (l>>4)] and holds
// D[p0 + 4(l>>4) + r][q0 + (l&15)], r = 0..3.  Out-of-range rows / k read 0.
// (LDS reads are predicated selects, not branches: LDS, unlike VMEM, has no
// in-order counter to drain.)
template <bool RELU_A, bool RELU_B, class Epi>
__device__ __forceinline__ void lds_gemm(int P, int Q, int K, const float* __restrict__ A,
                                         int sap, int sak, const float* __restrict__ B,
                                         int sbq, int sbk, Epi epi) {
    // Work unit = one 16-row block of P x TWO adjacent 16-column blocks of Q:
    // two independent accumulator chains (hides the 40-cycle dependent
    // latency of 16x16x4) sharing the A fragment (3 LDS reads per 2 MFMAs).
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const int i16 = lane & 15, k4 = lane >> 4;
    const int tp = (P + 15) >> 4, tq2 = (Q + 31) >> 5;
    for (int t = wid; t < tp * tq2; t += nwv) {
        const int p0 = (t / tq2) << 4, q0 = (t - (t / tq2) * tq2) << 5;
        const int p = p0 + i16, qa = q0 + i16, qb = qa + 16;
        const bool pv = p < P, qav = qa < Q, qbv = qb < Q;
        const float* Ap = A + (pv ? p : 0) * sap;
        const float* Ba = B + (qav ? qa : 0) * sbq;
        const float* Bb = B + (qbv ? qb : 0) * sbq;
        floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        int kb = 0;  // wave-uniform k base
        for (; kb + 16 <= K; kb += 16) {
            float av[4], b0[4], b1[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int kk = kb + 4 * u + k4;
                av[u] = pv ? Ap[kk * sak] : 0.f;
                b0[u] = qav ? Ba[kk * sbk] : 0.f;
                b1[u] = qbv ? Bb[kk * sbk] : 0.f;
                if (RELU_A) av[u] = fmaxf(av[u], 0.f);
                if (RELU_B) { b0[u] = fmaxf(b0[u], 0.f); b1[u] = fmaxf(b1[u], 0.f); }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b0[u], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b1[u], acc1, 0, 0, 0);
            }
        }
        for (; kb < K; kb += 4) {
            const int kk = kb + k4;
            const bool kv = kk < K;
            float av = (pv && kv) ? Ap[kk * sak] : 0.f;
            float b0 = (qav && kv) ? Ba[kk * sbk] : 0.f;
            float b1 = (qbv && kv) ? Bb[kk * sbk] : 0.f;
            if (RELU_A) av = fmaxf(av, 0.f);
            if (RELU_B) { b0 = fmaxf(b0, 0.f); b1 = fmaxf(b1, 0.f); }
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc1, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int pp = p0 + 4 * k4 + r;
            if (pp < P) {
                if (qav) epi(pp, qa, acc0[r]);
                if (qbv) epi(pp, qb, acc1[r]);
            }
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
    // Global -> LDS copies issue kB independent loads per thread before any
    // LDS store (a load-then-store loop would expose one memory latency per
    // element); indices are clamped so every load is unconditional.
    constexpr int kB = 8;
    for (int l = 0; l < L; ++l) {
        const int din = a.din[l], dout = a.dout[l], nw = din * dout, n = nw + dout;
        float* W = sm + a.lw[l];
        float* Bv = sm + a.lb[l];
        const int ldw = a.ldw[l];
        if (FAM == PSVI_FAMILY_MEANFIELD) {
            const float* mu = a.params + a.poff[l];
            const float* rho = mu + n;
            const float* eW = a.eps + a.eoff[l] + (int64_t)sg * nw;
            const float* eB = a.eps + a.eoff[l] + (int64_t)a.S_total * nw + (int64_t)sg * dout;
            float* E = sm + a.le[l];
            float* EB = sm + a.leb[l];
            for (int base = threadIdx.x; base < n; base += kB * blockDim.x) {
                float vm[kB], vr[kB], ve[kB];
#pragma unroll
                for (int k = 0; k < kB; ++k) {
                    const int idx = min(base + k * (int)blockDim.x, n - 1);
                    vm[k] = mu[idx];
                    vr[k] = rho[idx];
                    ve[k] = idx < nw ? eW[idx] : eB[idx - nw];
                }
#pragma unroll
                for (int k = 0; k < kB; ++k) {
                    const int idx = base + k * (int)blockDim.x;
                    if (idx >= n) break;
                    // Normal.rsample: loc + eps * scale (torch/distributions/normal.py)
                    const float val = vm[k] + ve[k] * softplus_f(vr[k]);
                    if (idx < nw) {
                        const int j = idx / din, i = idx - j * din;
                        W[j * ldw + i] = val;
                        E[j * ldw + i] = ve[k];
                    } else {
                        Bv[idx - nw] = val;
                        EB[idx - nw] = ve[k];
                    }
                }
            }
        } else {
            for (int p = 0; p < a.nsrc; ++p) {
                const int lo = a.src_lo[p][l], hi = a.src_hi[p][l];
                if (hi <= lo) continue;
                const float* src = a.xrecv + a.src_base[p] + (int64_t)s * a.src_stride[p] +
                                   a.src_col[p][l] - lo;
                for (int base = lo + threadIdx.x; base < hi; base += kB * blockDim.x) {
                    float v[kB];
#pragma unroll
                    for (int k = 0; k < kB; ++k) v[k] = src[min(base + k * (int)blockDim.x, hi - 1)];
#pragma unroll
                    for (int k = 0; k < kB; ++k) {
                        const int r = base + k * (int)blockDim.x;
                        if (r >= hi) break;
                        if (r < nw) {
                            const int j = r / din, i = r - j * din;
                            W[j * ldw + i] = v[k];
                        } else {
                            Bv[r - nw] = v[k];
                        }
                    }
                }
            }
        }
    }
    // ---- 2. pseudo-input chunk -------------------------------------------
    {
        const int D = a.din[0], nU = mcnt * D;
        float* U = sm + a.lu;
        const float* src = a.u + (int64_t)m0 * D;
        for (int base = threadIdx.x; base < nU; base += kB * blockDim.x) {
            float v[kB];
#pragma unroll
            for (int k = 0; k < kB; ++k) v[k] = src[min(base + k * (int)blockDim.x, nU - 1)];
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                const int idx = base + k * (int)blockDim.x;
                if (idx >= nU) break;
                const int m = idx / D, i = idx - m * D;
                U[m * a.ldu + i] = v[k];
            }
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
            for (int k = 0; k < C; ++k) se += expf(row[k] - mx);
            const float lse = mx + logf(se);
            const int zm = a.z[m0 + m];
            const float wm = a.w[m0 + m];
            part += wm * (lse - row[zm]);
            for (int k = 0; k < C; ++k) {
                const float pk = expf(row[k] - lse);
                row[k] = wm * (pk - (k == zm ? 1.f : 0.f));
            }
        }
        const float tot = block_sum(part, sm + a.lred);
        if (threadIdx.x == 0) atomicAdd(a.nll_out, (double)tot);
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
                      const float* xrecv, float* gsend, double* nll_out, hipStream_t st) {
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
