// kernels_mvn.hip -- full-covariance (VILinearMultivariateNormal) layers.
//
// Reference (/root/reference):
//   scale_tril  psvi/models/neural_net.py:452-461  L = diag(softplus(sd)) + corr
//               scattered row-major into the strict lower (n-1)x(n-1) block
//   rsample     neural_net.py:467-476  x_s = mean + L eps_s  (torch _batch_mv)
//   kl          neural_net.py:435-436  KL(N(mean, LL^T) || N(0, s0^2 I)); torch
//               evaluates it with an O(n^3) triangular solve, here it is the
//               exactly equal O(n^2) sum  n log s0 - sum log diag L
//               + (|L|_F^2 + |mean|^2) / (2 s0^2) - n/2
// Backward: G (S x n) = per-sample grads of x_s;
//   d mean = sum_s G_s + mean/s0^2,  dL = G^T eps (lower triangle only),
//   d sd = diag(dL) sigmoid(sd) + (sp/s0^2 - 1/sp) sigmoid(sd),
//   d corr = dL[tril] + corr/s0^2.
//
// L is never materialised: both GEMMs read the packed corr vector directly
// (row r starts at r(r-1)/2) and run on v_mfma_f32_32x32x2_f32 (exact fp32,
// gfx950 has no xf32).  The backward never writes dL to HBM: the Adam update
// of corr (p, m, v read + written once) is the GEMM epilogue.
#include "psvi_internal.hpp"

namespace psvi {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct MvnLayerArgs {
    int n;
    int64_t poff, eoff;
};

// ----------------------------------------------------------------- forward
constexpr int FBK = 64;    // k (columns of L) per LDS stage
constexpr int FST = 128;   // samples per pass: 4 waves x 32

struct FwdArgs {
    const FwdItem* items;
    const float* params;
    const float* eps;
    float* x;         // x_shard [S][ldx]
    int ldx, S;
    MvnLayerArgs lay[kMaxL];
};

__global__ __launch_bounds__(256) void mvn_fwd_kernel(FwdArgs a) {
    __shared__ float Es[FST][FBK + 1];  // eps  [s][k]
    __shared__ float Ls[32][FBK + 1];   // corr [r][k]
    const FwdItem it = a.items[blockIdx.x];
    const int n = a.lay[it.layer].n;
    const float* mean = a.params + a.lay[it.layer].poff;
    const float* sd = mean + n;
    const float* corr = mean + 2 * n;
    const float* E = a.eps + a.lay[it.layer].eoff;   // [S][n]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l32 = lane & 31;
    const rsrc_t rsL = make_rsrc(corr, ((int64_t)(n - 1) * (n - 2) / 2) * 4);
    const rsrc_t rsE = make_rsrc(E, (int64_t)a.S * n * 4);

    for (int sb = 0; sb < a.S; sb += FST) {
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        const bool wave_live = sb + 32 * wv < a.S;
        // register prefetch of stage kb
        float lreg[FBK / 8], ereg[FBK / 2];
        // L rows of this item and eps rows of this pass; loads outside the
        // triangle / past S read 0 through the buffer range check.  eps
        // columns past k1 need no mask: they meet zero L entries.
        const int kk = tid % FBK, rq = tid / FBK;
        auto fetch = [&](int kb) {
            const int c = kb + kk;
#pragma unroll
            for (int j = 0; j < FBK / 8; ++j) {
                const int r = it.r0 + rq + 4 * j;
                const bool ok = r < it.r1 && c < r && c < it.k1 && r <= n - 2;
                lreg[j] = bload(rsL, ok ? (uint32_t)(((int64_t)r * (r - 1) / 2 + c) * 4) : kOOB);
            }
#pragma unroll
            for (int j = 0; j < FBK / 2; ++j) {
                const int srow = sb + rq + 4 * j;
                ereg[j] = bload(rsE, (uint32_t)(((int64_t)srow * n + c) * 4));
            }
        };
        if (it.k0 < it.k1) fetch(it.k0);
        for (int kb = it.k0; kb < it.k1; kb += FBK) {
            __syncthreads();
#pragma unroll
            for (int j = 0; j < FBK / 8; ++j) Ls[rq + 4 * j][kk] = lreg[j];
#pragma unroll
            for (int j = 0; j < FBK / 2; ++j) Es[rq + 4 * j][kk] = ereg[j];
            __syncthreads();
            if (kb + FBK < it.k1) fetch(kb + FBK);
            if (wave_live) {
#pragma unroll
                for (int kk = 0; kk < FBK; kk += 2) {
                    const float av = Es[32 * wv + l32][kk + h];
                    const float bv = Ls[l32][kk + h];
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
                }
            }
        }
        // D[i = s][j = r]: j = lane&31, i = (q&3) + 8(q>>2) + 4h
        const int r = it.r0 + l32;
        if (wave_live && r < it.r1) {
            float base_m = 0.f, base_sd = 0.f;
            if (it.k0 == 0) {
                base_m = mean[r];
                base_sd = softplus_f(sd[r]);
            }
            float* xrow = a.x + it.xcol + l32;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int s = sb + 32 * wv + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (s < a.S) {
                    float val = acc[q];
                    if (it.k0 == 0) val += base_m + base_sd * E[(int64_t)s * n + r];
                    atomicAdd(xrow + (int64_t)s * a.ldx, val);
                }
            }
        }
    }
}

// ---------------------------------------------------------------- backward
constexpr int BT = 64;    // output tile 64 (rows r) x 64 (cols c)
constexpr int BKS = 128;  // samples staged per pass (K of the dL GEMM); S <= 128: one pass

struct UpdArgs {
    const BwdTile* tiles;
    const DiagBlock* diag;
    int n_tiles, n_diag;
    const float* eps;
    const float* g;    // g_shard [S][ldg]
    int ldg, S;
    float* params;
    float* m;
    float* v;
    float* grad_out;   // GRAD mode output
    double* kl_out;    // nullable
    int64_t pcount;    // parameter vector length
    int include_kl;
    float inv_s0sq, log_s0;
    AdamC adam;
    MvnLayerArgs lay[kMaxL];
};

template <bool GRAD>
__device__ __forceinline__ void upd_elem(const UpdArgs& a, int64_t pidx, float gval) {
    if (GRAD) {
        a.grad_out[pidx] = gval;
    } else {
        float mm = a.m[pidx], vv = a.v[pidx];
        const float pn = adam_apply(a.adam, a.params[pidx], gval, mm, vv);
        a.params[pidx] = pn;
        a.m[pidx] = mm;
        a.v[pidx] = vv;
    }
}

// Tiles: dL[r0:r0+64, c0:c0+64] = G^T eps over all S samples (4 waves, 32x32
// each), then the fused corr update.  Memory schedule per tile: issue the
// G / eps loads of the first sample chunk, THEN the epilogue's corr/m/v loads
// (vmcnt retires in order, so the GEMM operands are not held behind them),
// stage the chunk in LDS, run the MFMAs while the corr/m/v loads land, update.
// Diag blocks (blockIdx < n_diag, scheduled first): mean and sd of 64 rows each.
template <bool GRAD>
__global__ __launch_bounds__(256) void mvn_update_kernel(UpdArgs a) {
    __shared__ float Gs[BKS][BT + 1];
    __shared__ float Xs[BKS][BT + 1];
    __shared__ float red[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l32 = lane & 31;
    float klp = 0.f;
    if ((int)blockIdx.x >= a.n_diag) {
        const BwdTile t = a.tiles[(int)blockIdx.x - a.n_diag];
        const int n = a.lay[t.layer].n;
        const float* E = a.eps + a.lay[t.layer].eoff;
        const int64_t corr_off = a.lay[t.layer].poff + 2 * n;
        const int wr = wv >> 1, wc = wv & 1;
        const int c = t.c0 + 32 * wc + l32;
        const int rb = t.r0 + 32 * wr + 4 * h;
        const int cc = tid & 63, s0 = tid >> 6;   // staging: column, first sample row
        // Out-of-tile rows / columns of G and eps only feed dL entries the
        // epilogue masks, so staging needs no predicate; rows past S read 0.
        const rsrc_t rsG = make_rsrc(a.g, (int64_t)a.S * a.ldg * 4);
        const rsrc_t rsE = make_rsrc(E, (int64_t)a.S * n * 4);
        const rsrc_t rsP = make_rsrc(a.params, a.pcount * 4);
        const rsrc_t rsM = make_rsrc(a.m, GRAD ? 0 : a.pcount * 4);
        const rsrc_t rsV = make_rsrc(a.v, GRAD ? 0 : a.pcount * 4);
        const uint32_t gcol = (uint32_t)(t.xcol + t.r0 + cc) * 4;
        const uint32_t xcol = (uint32_t)(t.c0 + cc) * 4;
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        float pq[16], mq[16], vq[16];
        for (int sb = 0; sb < a.S; sb += BKS) {
            float greg[BKS / 4], xreg[BKS / 4];
#pragma unroll
            for (int j = 0; j < BKS / 4; ++j) {
                const uint32_t s = sb + s0 + 4 * j;
                greg[j] = bload(rsG, gcol + s * (uint32_t)a.ldg * 4);
                xreg[j] = bload(rsE, xcol + s * (uint32_t)n * 4);
            }
            if (sb == 0) {
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int r = rb + (q & 3) + 8 * (q >> 2);
                    const bool ok = r >= t.rlo && r < t.rhi && c < r;
                    const uint32_t off =
                        ok ? (uint32_t)((corr_off + (int64_t)r * (r - 1) / 2 + c) * 4) : kOOB;
                    pq[q] = bload(rsP, off);
                    if (!GRAD) {
                        mq[q] = bload(rsM, off);
                        vq[q] = bload(rsV, off);
                    }
                }
            } else {
                __syncthreads();  // previous chunk fully consumed
            }
#pragma unroll
            for (int j = 0; j < BKS / 4; ++j) {
                Gs[s0 + 4 * j][cc] = greg[j];
                Xs[s0 + 4 * j][cc] = xreg[j];
            }
            __syncthreads();
            const int kend = min(BKS, a.S - sb);
            for (int kk = 0; kk < kend; kk += 2) {
                const float av = Gs[kk + h][32 * wr + l32];
                const float bv = Xs[kk + h][32 * wc + l32];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
            }
        }
        // D[i = r][j = c]: j = lane&31, i = (q&3) + 8(q>>2) + 4h
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int r = rb + (q & 3) + 8 * (q >> 2);
            if (r >= t.rlo && r < t.rhi && c < r) {
                const int64_t pidx = corr_off + (int64_t)r * (r - 1) / 2 + c;
                const float p = pq[q];
                klp += p * p;
                const float gval = a.include_kl ? acc[q] + p * a.inv_s0sq : acc[q];
                if (GRAD) {
                    a.grad_out[pidx] = gval;
                } else {
                    float mm = mq[q], vv = vq[q];
                    a.params[pidx] = adam_apply(a.adam, p, gval, mm, vv);
                    a.m[pidx] = mm;
                    a.v[pidx] = vv;
                }
            }
        }
        klp *= 0.5f * a.inv_s0sq;
    } else {
        // 64 rows per block; the 4 waves split the samples, partial sums meet
        // in LDS (reusing the staging arrays); loads batched 8 deep.
        const DiagBlock db = a.diag[blockIdx.x];
        const int n = a.lay[db.layer].n;
        const float* E = a.eps + a.lay[db.layer].eoff;
        const int r = db.r0 + (tid & 63);
        const bool rv = r < db.rhi;
        const int rr = rv ? r : db.r0;
        const rsrc_t rsG = make_rsrc(a.g, (int64_t)a.S * a.ldg * 4);
        const rsrc_t rsE = make_rsrc(E, (int64_t)a.S * n * 4);
        const uint32_t gofs = (uint32_t)(db.xcol + rr) * 4, eofs = (uint32_t)rr * 4;
        float gm = 0.f, gs = 0.f;
        for (int s0 = wv; s0 < a.S; s0 += 32) {
            float gv[8], ev[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t s = s0 + 4 * k;   // past S: range check -> 0
                gv[k] = bload(rsG, gofs + s * (uint32_t)a.ldg * 4);
                ev[k] = bload(rsE, eofs + s * (uint32_t)n * 4);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                gm += gv[k];
                gs = fmaf(gv[k], ev[k], gs);
            }
        }
        Gs[wv][tid & 63] = gm;
        Xs[wv][tid & 63] = gs;
        __syncthreads();
        if (tid < 64 && rv) {
            gm = Gs[0][tid] + Gs[1][tid] + Gs[2][tid] + Gs[3][tid];
            gs = Xs[0][tid] + Xs[1][tid] + Xs[2][tid] + Xs[3][tid];
            const int64_t pm = a.lay[db.layer].poff + r, ps = pm + n;
            const float mu = a.params[pm], sdr = a.params[ps];
            const float sp = softplus_f(sdr), sg = sigmoid_f(sdr);
            float gmean = gm, gsd = gs * sg;
            if (a.include_kl) {
                gmean += mu * a.inv_s0sq;
                gsd += (sp * a.inv_s0sq - 1.f / sp) * sg;
                klp = a.log_s0 - logf(sp) + 0.5f * ((sp * sp + mu * mu) * a.inv_s0sq - 1.f);
            }
            upd_elem<GRAD>(a, pm, gmean);
            upd_elem<GRAD>(a, ps, gsd);
        }
    }
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, red);
        if (tid == 0) atomicAdd(a.kl_out, (double)tot);
    }
}

static void fill_layers(const psvi_plan& p, MvnLayerArgs* la) {
    for (int l = 0; l < p.L; ++l) {
        la[l].n = p.lay[l].n;
        la[l].poff = p.lay[l].poff;
        la[l].eoff = p.lay[l].eoff;
    }
}

hipError_t launch_mvn_fwd(const psvi_plan& p, const float* eps, const float* params,
                          float* x_shard, hipStream_t st) {
    FwdArgs a{};
    a.items = p.d_fwd;
    a.params = params;
    a.eps = eps;
    a.x = x_shard;
    a.ldx = p.rows_tot[p.rank];
    a.S = p.d.S;
    fill_layers(p, a.lay);
    hipError_t e = hipMemsetAsync(x_shard, 0, sizeof(float) * (size_t)a.S * a.ldx, st);
    if (e != hipSuccess) return e;
    if (p.n_fwd == 0) return hipSuccess;
    hipLaunchKernelGGL(mvn_fwd_kernel, dim3(p.n_fwd), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_mvn_update(const psvi_plan& p, const float* eps, const float* g_shard,
                             float* params, float* m, float* v, const psvi_adam_hp* hp,
                             double* kl_out, float* grad_out, int include_kl, hipStream_t st) {
    UpdArgs a{};
    a.tiles = p.d_bwd;
    a.diag = p.d_diag;
    a.n_tiles = p.n_bwd;
    a.n_diag = p.n_diag;
    a.eps = eps;
    a.g = g_shard;
    a.ldg = p.rows_tot[p.rank];
    a.S = p.d.S;
    a.params = params;
    a.m = m;
    a.v = v;
    a.grad_out = grad_out;
    a.kl_out = kl_out;
    a.include_kl = include_kl;
    a.pcount = p.P;
    const float s0 = p.d.prior_sd;
    a.inv_s0sq = 1.f / (s0 * s0);
    a.log_s0 = logf(s0);
    if (hp) a.adam = make_adam(hp);
    fill_layers(p, a.lay);
    const int nb = p.n_bwd + p.n_diag;
    if (nb == 0) return hipSuccess;
    if (grad_out)
        hipLaunchKernelGGL(mvn_update_kernel<true>, dim3(nb), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(mvn_update_kernel<false>, dim3(nb), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace psvi
