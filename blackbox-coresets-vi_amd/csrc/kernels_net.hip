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
// activations, two gradient buffers, one dW accumulation tile) lives in LDS
// with odd row strides.  The contractions run on fp32 MFMA (16x16x4) "units"
// of 16 rows x 32 columns with software-pipelined operand loads; units are
// dealt round-robin to the waves.  Backward, per layer, in ONE phase:
//   dW_l = g_l^T [h_{l-1} | 1]  (the ones column makes the last output column
//          the bias gradient), K = pseudopoints split over waves, partial
//          tiles summed with LDS float atomics into the dW tile;
//   g_{l-1} = (g_l W_l) * 1[a_{l-1} > 0]  into the other gradient buffer;
// then the dW tile leaves LDS as contiguous rows:
//  MEANFIELD: [sum_s dW | sum_s dW*eps] accumulators (fp32 atomics, S adders);
//  FULLCOV:   g_send in the blocked-by-source-rank layout (plain stores, or
//             atomics when a sample's pseudopoints span several workgroups).
#include <algorithm>

#include "psvi_internal.hpp"

namespace psvi {

struct NetArgs {
    int L, M, mc, S_total, s_goff, atomic_g;
    int abl;  // diagnostics ablation mask (0 in production): 1 loads, 2 fwd
              // GEMMs, 4 NLL, 8 bwd GEMMs, 16 global dW writes,
              // 128 g-propagation GEMMs
    unsigned long long* stamps;  // diagnostics: s_memtime per phase (nullptr in production)
    int din[kMaxL], dout[kMaxL], woff[kMaxL];
    // LDS carve (float offsets) and row strides
    int lw[kMaxL], ldw[kMaxL], lb[kMaxL], le[kMaxL], leb[kMaxL], la[kMaxL], lda[kMaxL];
    int lu, ldu, lred, lg0, lg1, ldgb, ldwt, lds_f4;
    int lstage_f4;                // float4 index where the late regions (and the DMA stage) start
    int stage_off[kMaxWorld], stage_u;  // DMA stage: per-source x rows, then the u chunk
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

// One MFMA work unit of C[p][q] = sum_k A(p,k) B(q,k) with
// A(p,k) = A[p*sap + k*sak], B(q,k) = B[q*sbq + k*sbk] in LDS: rows
// [p0, p0+16) x columns [q0, q0+32) (two 16x16 tiles on v_mfma_f32_16x16x4_f32,
// exact fp32, two independent accumulator chains sharing the A fragment),
// k in [k0, k0 + 16*ceil((k1-k0)/16)).  Lane l feeds A[p0+(l&15)][k+(l>>4)],
// B[q+(l&15)][k+(l>>4)] and holds D[p0+4(l>>4)+r][q+(l&15)].
// No masks: the LDS layout (net_lds_floats) zero-fills and pads every
// operand so that any k >= k1 meets a zero in A or B, and rows / columns
// past P / Q only feed outputs the epilogue drops.  The next 16-k group's
// operands are read before the current group's MFMAs.
template <int NQ, bool RELU_A, bool RELU_B, class Epi>
__device__ __forceinline__ void gemm_unit(int P, int Q, int k0, int k1, int p0, int q0,
                                          const float* __restrict__ A, int sap, int sak,
                                          const float* __restrict__ B, int sbq, int sbk,
                                          Epi epi) {
    const int lane = threadIdx.x & 63, i16 = lane & 15, k4 = lane >> 4;
    const float* Ap = A + (p0 + i16) * sap + k4 * sak;
    const float* Bp = B + (q0 + i16) * sbq + k4 * sbk;
    floatx4 acc[NQ];
#pragma unroll
    for (int c = 0; c < NQ; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    float a[4], b[NQ][4];
    auto load = [&](int kb, float (&x)[4], float (&y)[NQ][4]) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int kk = kb + 4 * u;
            x[u] = Ap[kk * sak];
            if (RELU_A) x[u] = fmaxf(x[u], 0.f);
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                y[c][u] = Bp[16 * c * sbq + kk * sbk];
                if (RELU_B) y[c][u] = fmaxf(y[c][u], 0.f);
            }
        }
    };
    if (k0 < k1) load(k0, a, b);
    for (int kb = k0; kb < k1; kb += 16) {  // wave-uniform
        float na[4], nb[NQ][4];
        if (kb + 16 < k1) load(kb + 16, na, nb);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < NQ; ++c)
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[c][u], acc[c], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = na[u];
#pragma unroll
            for (int c = 0; c < NQ; ++c) b[c][u] = nb[c][u];
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int pp = p0 + 4 * k4 + r;
        if (pp < P) {
#pragma unroll
            for (int c = 0; c < NQ; ++c) {
                const int q = q0 + 16 * c + i16;
                if (q < Q) epi(pp, q, acc[c][r]);
            }
        }
    }
}

// Degenerate shapes (a side < 8, or K <= 4: the classifier layer) on VALU.
// K >= 16: one output per 16-lane group, lanes split k, xor-shuffle reduce;
// short K: one output per thread.
template <bool RELU_A, bool RELU_B, class Epi>
__device__ __forceinline__ void valu_gemm(int P, int Q, int K, const float* A, int sap, int sak,
                                          const float* B, int sbq, int sbk, Epi epi) {
    const int PQ = P * Q;
    if (K >= 16) {
        const int g = threadIdx.x >> 4, ng = blockDim.x >> 4, l16 = threadIdx.x & 15;
        for (int base = 0; base < PQ; base += ng) {  // uniform trip count: shuffles converge
            const int idx = min(base + g, PQ - 1);
            const int p = idx / Q, q = idx - p * Q;
            const float* Ap = A + p * sap;
            const float* Bp = B + q * sbq;
            float acc = 0.f;
            for (int k = l16; k < K; k += 16) {
                float x = Ap[k * sak], y = Bp[k * sbk];
                if (RELU_A) x = fmaxf(x, 0.f);
                if (RELU_B) y = fmaxf(y, 0.f);
                acc = fmaf(x, y, acc);
            }
            acc += __shfl_xor(acc, 8, 16);
            acc += __shfl_xor(acc, 4, 16);
            acc += __shfl_xor(acc, 2, 16);
            acc += __shfl_xor(acc, 1, 16);
            if (l16 == 0 && base + g < PQ) epi(p, q, acc);
        }
        return;
    }
    for (int idx = threadIdx.x; idx < PQ; idx += blockDim.x) {
        const int p = idx / Q, q = idx - p * Q;
        const float* Ap = A + p * sap;
        const float* Bp = B + q * sbq;
        float acc = 0.f;
        for (int k = 0; k < K; ++k) {
            float x = Ap[k * sak], y = Bp[k * sbk];
            if (RELU_A) x = fmaxf(x, 0.f);
            if (RELU_B) y = fmaxf(y, 0.f);
            acc = fmaf(x, y, acc);
        }
        epi(p, q, acc);
    }
}

// Whole GEMM: VALU for degenerate shapes, else MFMA units of 16 rows x
// 16*NQ columns (NQ matched to Q) dealt round-robin to the waves.
template <bool RELU_A, bool RELU_B, class Epi>
__device__ __forceinline__ void lds_gemm(int P, int Q, int K, const float* A, int sap, int sak,
                                         const float* B, int sbq, int sbk, Epi epi) {
    if (P < 8 || Q < 8 || K <= 4) {
        valu_gemm<RELU_A, RELU_B>(P, Q, K, A, sap, sak, B, sbq, sbk, epi);
        return;
    }
    const int wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const int tp = (P + 15) >> 4;
    if (Q <= 16) {
        for (int t = wid; t < tp; t += nwv)
            gemm_unit<1, RELU_A, RELU_B>(P, Q, 0, K, t << 4, 0, A, sap, sak, B, sbq, sbk, epi);
    } else if (Q <= 32 || (Q > 48 && Q <= 64)) {
        const int tq = (Q + 31) >> 5;
        for (int t = wid; t < tp * tq; t += nwv) {
            const int pt = t / tq;
            gemm_unit<2, RELU_A, RELU_B>(P, Q, 0, K, pt << 4, (t - pt * tq) << 5, A, sap, sak, B,
                                         sbq, sbk, epi);
        }
    } else {
        const int tq = (Q + 47) / 48;
        for (int t = wid; t < tp * tq; t += nwv) {
            const int pt = t / tq;
            gemm_unit<3, RELU_A, RELU_B>(P, Q, 0, K, pt << 4, (t - pt * tq) * 48, A, sap, sak, B,
                                         sbq, sbk, epi);
        }
    }
}

// FULLCOV: address in x_recv / g_send of row r of layer l for local sample s.
__device__ __forceinline__ int64_t fc_addr(const NetArgs& a, int l, int r, int s) {
    int p = 0;
    while (p + 1 < a.nsrc && r >= a.src_hi[p][l]) ++p;
    return a.src_base[p] + (int64_t)s * a.src_stride[p] + a.src_col[p][l] + (r - a.src_lo[p][l]);
}

// diagnostics: one wave-0 lane of every workgroup records the shader clock at
// phase boundaries (slot k of its row); costs nothing when stamps == nullptr
#define NET_STAMP(k)                                                                   \
    do {                                                                               \
        if (a.stamps && threadIdx.x == 0)                                              \
            a.stamps[(blockIdx.x + blockIdx.y * gridDim.x) * 16 + (k)] =               \
                __builtin_amdgcn_s_memtime();                                          \
    } while (0)

template <int FAM>
__global__ __launch_bounds__(512) void net_kernel(NetArgs a) {
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
    NET_STAMP(0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    float4* z4 = reinterpret_cast<float4*>(sm);
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float* dWt = sm + a.lg0 - a.ldwt;  // dW tile [dout][din + 1]
    const int D = a.din[0], nU = mcnt * D;
    float* U = sm + a.lu;
    if constexpr (FAM == PSVI_FAMILY_FULLCOV) {
        // LDS-DMA (global_load_lds_dword): this sample's x rows (one contiguous
        // run per source rank) and the u chunk land in the stage with no VGPR
        // round trip; the resident regions are zeroed while they are in flight.
        float* stage = sm + 4 * a.lstage_f4;
        if (!(a.abl & 1)) {
            for (int p = 0; p < a.nsrc; ++p) {
                const int len = a.src_stride[p];
                const float* src = a.xrecv + a.src_base[p] + (int64_t)s * len;
                float* dst = stage + a.stage_off[p];
                for (int c = wid; c * 64 < len; c += nwv)
                    __builtin_amdgcn_global_load_lds(
                        (const void*)(src + min(c * 64 + lane, len - 1)),
                        (__attribute__((address_space(3))) void*)(dst + c * 64), 4, 0, 0);
            }
            const float* usrc = a.u + (int64_t)m0 * D;
            float* udst = stage + a.stage_u;
            for (int c = wid; c * 64 < nU; c += nwv)
                __builtin_amdgcn_global_load_lds(
                    (const void*)(usrc + min(c * 64 + lane, nU - 1)),
                    (__attribute__((address_space(3))) void*)(udst + c * 64), 4, 0, 0);
        }
        for (int i = threadIdx.x; i < a.lstage_f4; i += blockDim.x) z4[i] = zero4;
        __syncthreads();  // drains the DMA (vmcnt(0)) and the zeroing
        if (!(a.abl & 1)) {
            for (int p = 0; p < a.nsrc; ++p) {
                const float* st = stage + a.stage_off[p];
                for (int l = 0; l < L; ++l) {
                    const int lo = a.src_lo[p][l], hi = a.src_hi[p][l];
                    const int din = a.din[l], nw = din * a.dout[l], ldw = a.ldw[l];
                    const float rdin = 1.f / (float)din;
                    const float* sl = st + a.src_col[p][l] - lo;
                    float* W = sm + a.lw[l];
                    float* Bv = sm + a.lb[l];
                    for (int r = lo + threadIdx.x; r < hi; r += blockDim.x) {
                        const float v = sl[r];
                        if (r < nw) {
                            // exact for r < 2^21: (r + 0.5) / din is >= 0.5/din from an integer
                            const int j = (int)(((float)r + 0.5f) * rdin), i = r - j * din;
                            W[j * ldw + i] = v;
                        } else {
                            Bv[r - nw] = v;
                        }
                    }
                }
            }
            const float* us = stage + a.stage_u;
            const float rD = 1.f / (float)D;
            for (int idx = threadIdx.x; idx < nU; idx += blockDim.x) {
                const int m = (int)(((float)idx + 0.5f) * rD), i = idx - m * D;
                U[m * a.ldu + i] = us[idx];
            }
        }
        for (int m = threadIdx.x; m < mcnt; m += blockDim.x) U[m * a.ldu + D] = 1.f;
        __syncthreads();
        for (int i = a.lstage_f4 + threadIdx.x; i < a.lds_f4; i += blockDim.x) z4[i] = zero4;
        __syncthreads();
        // ones column of every hidden activation (read from fwd layer 1 on,
        // past the barrier that ends fwd layer 0)
        for (int m = threadIdx.x; m < mcnt; m += blockDim.x)
            for (int l = 0; l + 1 < L; ++l) sm[a.la[l] + m * a.lda[l] + a.dout[l]] = 1.f;
    } else {
        for (int i = threadIdx.x; i < a.lds_f4; i += blockDim.x) z4[i] = zero4;
        __syncthreads();
        constexpr int kB = 16;
        for (int l = 0; l < L && !(a.abl & 1); ++l) {
            const int din = a.din[l], dout = a.dout[l], nw = din * dout, n = nw + dout;
            float* W = sm + a.lw[l];
            float* Bv = sm + a.lb[l];
            const int ldw = a.ldw[l];
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
        }
        if (!(a.abl & 1)) {
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
        // ones column (index dim) of u and of every hidden activation: the dW
        // GEMM over [h | 1] then yields the bias gradient as its last column.
        for (int m = threadIdx.x; m < mcnt; m += blockDim.x) {
            U[m * a.ldu + D] = 1.f;
            for (int l = 0; l + 1 < L; ++l) sm[a.la[l] + m * a.lda[l] + a.dout[l]] = 1.f;
        }
    }
    __syncthreads();
    NET_STAMP(1);

    // ---- 3. forward --------------------------------------------------------
    for (int l = 0; l < L && !(a.abl & 2); ++l) {
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

    NET_STAMP(2);
    // ---- 4. weighted NLL, dlogits ------------------------------------------
    {
        const int C = a.dout[L - 1];
        float* G = sm + a.la[L - 1];
        const int ldg = a.lda[L - 1];
        float part = 0.f;
        for (int m = threadIdx.x; m < mcnt && !(a.abl & 4); m += blockDim.x) {
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

    NET_STAMP(3);
    // ---- 5. backward -------------------------------------------------------
    float sink = 0.f;
    for (int l = L - 1; l >= 0 && !(a.abl & 8); --l) {
        const int din = a.din[l], dout = a.dout[l], nw = din * dout, qw = din + 1;
        // g_l: dlogits in the last activation buffer, else a ping-pong buffer
        const float* G = l == L - 1 ? sm + a.la[L - 1] : sm + (((L - 1 - l) & 1) ? a.lg0 : a.lg1);
        const int ldg = l == L - 1 ? a.lda[L - 1] : a.ldgb;
        float* Gn = sm + (((L - l) & 1) ? a.lg0 : a.lg1);  // g_{l-1}
        const float* H = l == 0 ? sm + a.lu : sm + a.la[l - 1];
        const int ldh = l == 0 ? a.ldu : a.lda[l - 1];
        // dW_l = g_l^T [h_{l-1} | 1] into the LDS dW tile, and
        // g_{l-1} = (g_l W_l) * 1[a_{l-1} > 0] into the other gradient buffer
        {
            auto epi = [&](int j, int i, float v) { dWt[j * qw + i] = v; };
            if (l == 0)
                lds_gemm<false, false>(dout, qw, mcnt, G, 1, ldg, H, 1, ldh, epi);
            else
                lds_gemm<false, true>(dout, qw, mcnt, G, 1, ldg, H, 1, ldh, epi);
        }
        if (l > 0 && !(a.abl & 128)) {
            const float* Ap = sm + a.la[l - 1];
            const int ldp = a.lda[l - 1];
            auto epi = [&](int m, int i, float v) {
                Gn[m * a.ldgb + i] = Ap[m * ldp + i] > 0.f ? v : 0.f;
            };
            lds_gemm<false, false>(mcnt, din, dout, G, ldg, 1, sm + a.lw[l], 1, a.ldw[l], epi);
        }
        __syncthreads();
        NET_STAMP(4 + 2 * (L - 1 - l));
        // dW tile -> global as contiguous rows; re-zero the tile
        const int nt = dout * qw;
        if (FAM == PSVI_FAMILY_MEANFIELD) {
            float* accMu = a.accMu + a.woff[l];
            float* accRho = a.accRho + a.woff[l];
            const float* E = sm + a.le[l];
            const float* EB = sm + a.leb[l];
            for (int idx = threadIdx.x; idx < nt; idx += blockDim.x) {
                const int j = idx / qw, i = idx - j * qw;
                const float dw = dWt[idx];
                const int o = i < din ? j * din + i : nw + j;
                const float e = i < din ? E[j * a.ldw[l] + i] : EB[j];
                if (a.abl & 16) { sink += dw; continue; }
                atomicAdd(accMu + o, dw);
                atomicAdd(accRho + o, dw * e);
            }
        } else {
            const bool at = a.atomic_g != 0;
            for (int idx = threadIdx.x; idx < nt; idx += blockDim.x) {
                const int j = idx / qw, i = idx - j * qw;
                const float dw = dWt[idx];
                if (a.abl & 16) { sink += dw; continue; }
                // column din of [h | 1] is the bias gradient
                float* dst = a.gsend + fc_addr(a, l, i < din ? j * din + i : nw + j, s);
                if (at) atomicAdd(dst, dw); else *dst = dw;
            }
        }
        __syncthreads();
        NET_STAMP(5 + 2 * (L - 1 - l));
    }
    asm volatile("" ::"v"(sink));
}

static inline int odd_ld(int x) { return (x & 1) ? x : x + 1; }
static inline int rup(int x, int m) { return (x + m - 1) / m * m; }

// LDS floats needed for a chunk of `mc` points.  Padding contract of
// gemm_unit (everything zero-filled at kernel start):
//   W_l: rup(dout,32) rows (rows >= dout stay 0), odd stride >= rup(din,16)
//        (columns din.. stay 0): k past din / dout meets zeros;
//   h buffers (u, activations, gradients): rup(mc,16) rows (rows >= mcnt
//        stay 0: k past the pseudopoint count meets zeros), odd stride with a
//        ones column at index dim for u / hidden activations;
//   every region is followed by 64 floats of zero slack for the row-wrap
//   reads of out-of-range rows / columns (whose outputs are dropped).
//   Resident regions (weights, u) come first; the late regions (activations,
//   dW tile, gradient buffers) follow from lstage and double as the landing
//   area of the full-cov LDS-DMA loads before they are zeroed.
static size_t net_lds_floats(const psvi_plan& p, int mc, NetArgs* a) {
    size_t off = 0;
    auto take = [&](size_t nfl) {
        size_t o = off;
        off += ((nfl + 3) & ~size_t(3)) + 64;
        return (int)o;
    };
    const int mcr = rup(mc, 16);
    int maxh = 1, wt = 1;
    for (int l = 0; l < p.L; ++l) {
        const int din = p.lay[l].din, dout = p.lay[l].dout;
        if (l > 0) maxh = std::max(maxh, din);
        wt = std::max(wt, dout * (din + 1));
        const int ldw = odd_ld(rup(din, 16));
        int lw = take((size_t)rup(dout, 32) * ldw), lb = take(dout);
        int le = 0, leb = 0;
        if (p.family == PSVI_FAMILY_MEANFIELD) {
            le = take((size_t)dout * ldw);
            leb = take(dout);
        }
        if (a) {
            a->ldw[l] = ldw; a->lw[l] = lw; a->lb[l] = lb; a->le[l] = le; a->leb[l] = leb;
        }
    }
    const int ldu = odd_ld(p.lay[0].din + 1);
    int lu = take((size_t)mcr * ldu);
    int lred = take(16);
    const size_t lstage = off;
    for (int l = 0; l < p.L; ++l) {
        const int lda = odd_ld(p.lay[l].dout + 1);
        int la = take((size_t)mcr * lda);
        if (a) { a->la[l] = la; a->lda[l] = lda; }
    }
    const int wt4 = (wt + 3) & ~3;
    const int ldgb = odd_ld(maxh);
    // the dW tile sits directly in front of the first gradient buffer
    off += wt4;
    int lg0 = take((size_t)mcr * ldgb);
    int lg1 = take((size_t)mcr * ldgb);
    if (p.family == PSVI_FAMILY_FULLCOV) {
        // DMA stage: whole-wave (64-float) pieces per source, then u
        size_t st = lstage;
        for (int q = 0; q < p.world; ++q) {
            if (a) a->stage_off[q] = (int)(st - lstage);
            st += (size_t)rup(p.rows_tot[q], 64);
        }
        if (a) a->stage_u = (int)(st - lstage);
        st += (size_t)rup(mc * p.lay[0].din, 64);
        off = std::max(off, st);
    }
    off = (off + 3) & ~size_t(3);
    if (a) {
        a->lu = lu; a->ldu = ldu; a->lred = lred;
        a->lg0 = lg0; a->lg1 = lg1; a->ldgb = ldgb; a->ldwt = wt4;
        a->lds_f4 = (int)(off / 4);
        a->lstage_f4 = (int)(lstage / 4);
    }
    return off;
}

int g_net_split_below = 256;  // split when a rank has fewer samples than CUs (psvi_debug_set(PSVI_DBG_NET_SPLIT_BELOW, n))

size_t net_plan_geometry(psvi_plan& p) {
    // One workgroup per sample and all M pseudopoints when the samples alone
    // fill the chip (G gets plain stores: no memset, no atomics); otherwise
    // split the pseudopoints over workgroups (partial dW summed with atomics).
    // LDS <= 160 KiB per workgroup.
    const int S_local = std::max(1, p.s_cnt[p.rank]);
    const int M = p.d.M;
    int mchunks = 1;
    if (S_local < g_net_split_below)
        while (S_local * mchunks < 256 && (M + mchunks) / (mchunks + 1) >= 16) ++mchunks;
    for (;;) {
        const int mc = (M + mchunks - 1) / mchunks;
        const size_t bytes = net_lds_floats(p, mc, nullptr) * 4;
        if (bytes <= 160 * 1024 || mc == 1) {
            p.mchunks = (M + mc - 1) / mc;
            p.mc = mc;
            p.net_lds = bytes;
            p.net_threads = mc > 32 ? 512 : 256;
            return bytes;
        }
        ++mchunks;
    }
}

int g_net_ablation = 0;  // psvi_debug_set(PSVI_DBG_NET_ABLATION, mask)
unsigned long long* g_net_stamps = nullptr;  // psvi_debug_set_ptr(PSVI_DBG_NET_STAMPS, buf)

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
    a.abl = g_net_ablation;
    a.stamps = g_net_stamps;
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
    dim3 grid(p.s_cnt[p.rank], p.mchunks), block(p.net_threads);
    if (p.s_cnt[p.rank] == 0) return hipSuccess;
    if (p.family == PSVI_FAMILY_MEANFIELD)
        hipLaunchKernelGGL(net_kernel<PSVI_FAMILY_MEANFIELD>, grid, block, p.net_lds, st, a);
    else
        hipLaunchKernelGGL(net_kernel<PSVI_FAMILY_FULLCOV>, grid, block, p.net_lds, st, a);
    return hipGetLastError();
}

}  // namespace psvi
