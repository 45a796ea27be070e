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
constexpr int FBK = 32;    // k (columns of L) per LDS stage
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

    for (int sb = 0; sb < a.S; sb += FST) {
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        const bool wave_live = sb + 32 * wv < a.S;
        // register prefetch of stage kb
        float lreg[4], ereg[16];
        auto fetch = [&](int kb) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int e = tid + 256 * j, rr = e >> 5, kk = e & 31;
                const int r = it.r0 + rr, c = kb + kk;
                lreg[j] = (r < it.r1 && c < r && c < it.k1 && r <= n - 2)
                              ? corr[(int64_t)r * (r - 1) / 2 + c] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int e = tid + 256 * j, ss = e >> 5, kk = e & 31;
                const int s = sb + ss, c = kb + kk;
                ereg[j] = (s < a.S && c < it.k1) ? E[(int64_t)s * n + c] : 0.f;
            }
        };
        if (it.k0 < it.k1) fetch(it.k0);
        for (int kb = it.k0; kb < it.k1; kb += FBK) {
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int e = tid + 256 * j;
                Ls[e >> 5][e & 31] = lreg[j];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int e = tid + 256 * j;
                Es[e >> 5][e & 31] = ereg[j];
            }
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
constexpr int BKS = 32;   // samples per LDS stage

struct UpdArgs {
    const BwdTile* tiles;
    const DiagBlock* diag;
    int n_tiles;
    const float* eps;
    const float* g;    // g_shard [S][ldg]
    int ldg, S;
    float* params;
    float* m;
    float* v;
    float* grad_out;   // nullable
    float* kl_out;     // nullable
    int include_kl;
    float inv_s0sq, log_s0;
    AdamC adam;
    MvnLayerArgs lay[kMaxL];
};

__device__ __forceinline__ void upd_elem(const UpdArgs& a, int64_t pidx, float gval) {
    if (a.grad_out) {
        a.grad_out[pidx] = gval;
    } else {
        float mm = a.m[pidx], vv = a.v[pidx];
        const float pn = adam_apply(a.adam, a.params[pidx], gval, mm, vv);
        a.params[pidx] = pn;
        a.m[pidx] = mm;
        a.v[pidx] = vv;
    }
}

__global__ __launch_bounds__(256) void mvn_update_kernel(UpdArgs a) {
    __shared__ float Gs[BKS][BT + 1];
    __shared__ float Xs[BKS][BT + 1];
    __shared__ float red[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l32 = lane & 31;
    float klp = 0.f;
    if ((int)blockIdx.x < a.n_tiles) {
        const BwdTile t = a.tiles[blockIdx.x];
        const int n = a.lay[t.layer].n;
        const float* E = a.eps + a.lay[t.layer].eoff;
        const int64_t corr_off = a.lay[t.layer].poff + 2 * n;
        const int wr = wv >> 1, wc = wv & 1;
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        float greg[8], xreg[8];
        auto fetch = [&](int sb) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int e = tid + 256 * j, ss = e >> 6, cc = e & 63;
                const int s = sb + ss;
                const int r = t.r0 + cc, c = t.c0 + cc;
                greg[j] = (s < a.S && r < t.rhi) ? a.g[(int64_t)s * a.ldg + t.xcol + r] : 0.f;
                xreg[j] = (s < a.S && c < n) ? E[(int64_t)s * n + c] : 0.f;
            }
        };
        fetch(0);
        for (int sb = 0; sb < a.S; sb += BKS) {
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int e = tid + 256 * j;
                Gs[e >> 6][e & 63] = greg[j];
                Xs[e >> 6][e & 63] = xreg[j];
            }
            __syncthreads();
            if (sb + BKS < a.S) fetch(sb + BKS);
#pragma unroll
            for (int kk = 0; kk < BKS; kk += 2) {
                const float av = Gs[kk + h][32 * wr + l32];
                const float bv = Xs[kk + h][32 * wc + l32];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
            }
        }
        // D[i = r][j = c]: j = lane&31, i = (q&3) + 8(q>>2) + 4h
        const int c = t.c0 + 32 * wc + l32;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int r = t.r0 + 32 * wr + (q & 3) + 8 * (q >> 2) + 4 * h;
            if (r >= t.rlo && r < t.rhi && c < r) {
                const int64_t pidx = corr_off + (int64_t)r * (r - 1) / 2 + c;
                const float p = a.params[pidx];
                klp += p * p;
                upd_elem(a, pidx, a.include_kl ? acc[q] + p * a.inv_s0sq : acc[q]);
            }
        }
        klp *= 0.5f * a.inv_s0sq;
    } else {
        const DiagBlock db = a.diag[blockIdx.x - a.n_tiles];
        const int n = a.lay[db.layer].n;
        const float* E = a.eps + a.lay[db.layer].eoff;
        const int r = db.r0 + tid;
        if (r < db.rhi) {
            float gm = 0.f, gs = 0.f;
            const float* gcol = a.g + db.xcol + r;
            for (int s = 0; s < a.S; ++s) {
                const float gv = gcol[(int64_t)s * a.ldg];
                gm += gv;
                gs = fmaf(gv, E[(int64_t)s * n + r], gs);
            }
            const int64_t pm = a.lay[db.layer].poff + r, ps = pm + n;
            const float mu = a.params[pm], sdr = a.params[ps];
            const float sp = softplus_f(sdr), sg = sigmoid_f(sdr);
            float gmean = gm, gsd = gs * sg;
            if (a.include_kl) {
                gmean += mu * a.inv_s0sq;
                gsd += (sp * a.inv_s0sq - 1.f / sp) * sg;
                klp = a.log_s0 - logf(sp) + 0.5f * ((sp * sp + mu * mu) * a.inv_s0sq - 1.f);
            }
            upd_elem(a, pm, gmean);
            upd_elem(a, ps, gsd);
        }
    }
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, red);
        if (tid == 0) atomicAdd(a.kl_out, tot);
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
                             float* kl_out, float* grad_out, int include_kl, hipStream_t st) {
    UpdArgs a{};
    a.tiles = p.d_bwd;
    a.diag = p.d_diag;
    a.n_tiles = p.n_bwd;
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
    const float s0 = p.d.prior_sd;
    a.inv_s0sq = 1.f / (s0 * s0);
    a.log_s0 = logf(s0);
    if (hp) a.adam = make_adam(hp);
    fill_layers(p, a.lay);
    const int nb = p.n_bwd + p.n_diag;
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(mvn_update_kernel, dim3(nb), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace psvi
