// kernels_outer.hip -- the outer objective PSVI.psvi_elbo around the network
// kernel's two outer passes (psvi_outer_elbo_grad, capi.cpp).
//
// Reference (/root/reference):
//   PSVI.psvi_elbo            psvi/inference/psvi_classes.py:445-486
//   VIMixin.sampled_nkl       psvi/models/neural_net.py:110-115
//   MultivariateNormalVIMixin.sampled_nkl   neural_net.py:438-442
//
//   pseudo_s = sum_{m<Mu} w_m NLL_sm        data_s = sum_{m>=Mu} w_m NLL_sm (w = N/Nx)
//   nkl_s    = sum_i [-x_si^2 / (2 s0^2) - log s0 + eps_si^2 / 2 + log sigma_i]
//   lw_s = -pseudo_s + nkl_s,  W = softmax_s(lw),  a_s = data_s - pseudo_s
//   loss = sum_s W_s a_s - mean_s lw_s
// The reference evaluates log q(x_s) with a triangular solve of L against
// x_s - mean; x_s = mean + L eps_s makes that solve eps_s, whose square is
// taken directly here (the fp32 solve overflows at fn2 sizes, SURVEY.md
// Appendix B #16).  Backward coefficients, all per sample:
//   ck_s = d loss / d nkl_s = W_s (a_s - abar) - 1/S
//   cd_s = d loss / d data_s = W_s,   cp_s = d loss / d pseudo_s = -W_s - ck_s
// The network kernel's backward pass takes coef_sm = w_m c{p,d}_s per row and
// adds the pathwise sampled-KL gradient -ck_s x_s / s0^2; the explicit
// +sum_s ck_s / sigma_i on every scale is added here after the reparameterised
// backward (outer_finish_kernel).
#include "psvi_internal.hpp"

namespace psvi {

struct OuterArgs {
    int L, S, M, n_pseudo, n_tot, family;
    unsigned nkl_mask;     // layers in the sampled KL (plan_nkl_mask)
    int nkl_n;             // their sampled elements per sample
    int in_dim;            // input features per row (plan_in_dim)
    int batched[kMaxL];    // LeNet: the last layer is one shared sample
    int n[kMaxL], woff[kMaxL];
    int64_t poff[kMaxL], eoff[kMaxL];
    int din[kMaxL], dout[kMaxL];
    float s0;
    int ablated;           // PSVI_Ablated.psvi_elbo: mean data - mean nkl (no softmax)
    const float* params;
    const float* eps;
    const float* x;        // full-cov: x_shard [S][n_tot] (world 1)
    const float* w;        // [M] row weights
    const float* nll;      // [S][M]
    double* stats;         // [S][2]: sum x^2, sum eps^2
    double* loss;          // [1]
    float* rowcoef;        // [S][2]
    float* ck;             // [S]
    float* sck;            // [1] sum_s ck_s
    float* grad_w;         // [n_pseudo] nullable
    double* sample_out;    // [S][4] nullable: pseudo, data, nkl, weight
    float* grad;           // [P] nullable
    const float* du_part;  // [S][n_pseudo][D] nullable
    float* grad_u;         // [n_pseudo][D] nullable
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// block-wide double sum, result in every thread; `red` >= 16 doubles of LDS
__device__ __forceinline__ double block_sum_all(double v, double* red) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, wid = wave_id(), nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < nw; ++i) t += red[i];
    return t;
}
__device__ __forceinline__ double block_max_all(double v, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
    const int lane = threadIdx.x & 63, wid = wave_id(), nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = -INFINITY;
    for (int i = 0; i < nw; ++i) t = fmax(t, red[i]);
    return t;
}

// one workgroup per sample: sum_i x_si^2 and sum_i eps_si^2 over every layer
// (mean-field: x = mu + softplus(rho) eps, as the network kernel samples it)
__global__ __launch_bounds__(256) void outer_stats_kernel(OuterArgs a) {
    __shared__ double red[16];
    const int s = blockIdx.x;
    double sx = 0.0, se = 0.0;
    for (int l = 0; l < a.L; ++l) {
        if (!((a.nkl_mask >> l) & 1u)) continue;
        const int n = a.n[l];
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            float e, x;
            if (a.family != PSVI_FAMILY_FULLCOV) {
                const int dout = a.dout[l], nwl = a.din[l] * dout;
                e = !a.batched[l] ? a.eps[a.eoff[l] + i]
                    : i < nwl ? a.eps[a.eoff[l] + (int64_t)s * nwl + i]
                              : a.eps[a.eoff[l] + (int64_t)a.S * nwl + (int64_t)s * dout + i - nwl];
                const float mu = a.params[a.poff[l] + i], rho = a.params[a.poff[l] + n + i];
                x = mu + e * softplus_f(rho);
            } else {
                e = a.eps[a.eoff[l] + (int64_t)s * n + i];
                x = a.x[(int64_t)s * a.n_tot + a.woff[l] + i];
            }
            sx += (double)x * x;
            se += (double)e * e;
        }
    }
    sx = block_sum_all(sx, red);
    se = block_sum_all(se, red);
    if (threadIdx.x == 0) {
        a.stats[2 * s] = sx;
        a.stats[2 * s + 1] = se;
    }
}

// one workgroup: per-sample terms, the softmax over samples, the loss and the
// backward coefficients
constexpr int kOuterMaxS = 2048;  // samples the combine keeps in LDS
__global__ __launch_bounds__(1024) void outer_combine_kernel(OuterArgs a) {
    __shared__ double red[16];
    __shared__ double lw[kOuterMaxS], av[kOuterMaxS];
    __shared__ float cps[kOuterMaxS];
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wid = wave_id(), nwv = nthr >> 6;
    // sum_i log sigma_i: the scales sit at poff + n .. poff + 2n in both families
    double sl = 0.0;
    for (int l = 0; l < a.L; ++l)
        if ((a.nkl_mask >> l) & 1u)
            for (int i = tid; i < a.n[l]; i += nthr)
                sl += log((double)softplus_f(a.params[a.poff[l] + a.n[l] + i]));
    sl = block_sum_all(sl, red);
    const double s0 = a.s0, inv2 = 0.5 / (s0 * s0);
    const double nlog = a.nkl_n * log(s0);
    // per sample (one wave each): pseudo_s, data_s
    for (int s = wid; s < a.S; s += nwv) {
        double ps = 0.0, ds = 0.0;
        const float* row = a.nll + (size_t)s * a.M;
        for (int m = lane; m < a.M; m += 64) {
            const double t = (double)a.w[m] * row[m];
            if (m < a.n_pseudo) ps += t; else ds += t;
        }
        ps = wave_sum_d(ps);
        ds = wave_sum_d(ds);
        if (lane == 0) {
            const double nkl = -a.stats[2 * s] * inv2 - nlog + 0.5 * a.stats[2 * s + 1] + sl;
            lw[s] = a.ablated ? nkl : -ps + nkl;
            av[s] = a.ablated ? ds : ds - ps;
            if (a.sample_out) {
                a.sample_out[4 * s] = ps;
                a.sample_out[4 * s + 1] = ds;
                a.sample_out[4 * s + 2] = nkl;
            }
        }
    }
    __syncthreads();
    if (a.ablated) {
        // PSVI_Ablated.psvi_elbo (psvi_classes.py:1397-1408): data rows only,
        // loss = mean_s data_s - mean_s nkl_s; constant coefficients
        double dsum = 0.0, ksum = 0.0;
        for (int s = tid; s < a.S; s += nthr) {
            dsum += av[s];
            ksum += lw[s];
            a.rowcoef[2 * s] = 0.f;
            a.rowcoef[2 * s + 1] = 1.f / a.S;
            a.ck[s] = -1.f / a.S;
            if (a.sample_out) a.sample_out[4 * s + 3] = 1.0 / a.S;
        }
        dsum = block_sum_all(dsum, red);
        ksum = block_sum_all(ksum, red);
        if (tid == 0) {
            a.loss[0] = (dsum - ksum) / a.S;
            a.sck[0] = -1.f;
        }
        return;
    }
    double mx = -INFINITY, sm = 0.0;
    for (int s = tid; s < a.S; s += nthr) mx = fmax(mx, lw[s]);
    mx = block_max_all(mx, red);
    for (int s = tid; s < a.S; s += nthr) sm += exp(lw[s] - mx);
    sm = block_sum_all(sm, red);
    double abar = 0.0, lwsum = 0.0;
    for (int s = tid; s < a.S; s += nthr) {
        abar += exp(lw[s] - mx) / sm * av[s];
        lwsum += lw[s];
    }
    abar = block_sum_all(abar, red);
    lwsum = block_sum_all(lwsum, red);
    if (tid == 0) a.loss[0] = abar - lwsum / a.S;
    double cks = 0.0;
    for (int s = tid; s < a.S; s += nthr) {
        const double W = exp(lw[s] - mx) / sm;
        const double ck = W * (av[s] - abar) - 1.0 / a.S;
        const double cp = -W - ck;
        a.rowcoef[2 * s] = (float)cp;
        a.rowcoef[2 * s + 1] = (float)W;
        a.ck[s] = (float)ck;
        cps[s] = (float)cp;
        cks += ck;
        if (a.sample_out) a.sample_out[4 * s + 3] = W;
    }
    cks = block_sum_all(cks, red);
    if (tid == 0) a.sck[0] = (float)cks;
    __syncthreads();
    // d loss / d w_m = sum_s cp_s NLL_sm for the pseudopoints
    if (a.grad_w)
        for (int m = tid; m < a.n_pseudo; m += nthr) {
            double g = 0.0;
            for (int s = 0; s < a.S; ++s) g += (double)cps[s] * a.nll[(size_t)s * a.M + m];
            a.grad_w[m] = (float)g;
        }
}

// evaluate (psvi_classes.py:1031-1108) / pred_on_grid (1130-1175): importance
// weights over samples, then the predictive distribution of every test row.
// The reference's weights there use pseudo_nll = log_prob(z).matmul(N f(v)),
// the pseudopoints' weighted LOG-LIKELIHOOD (psvi_elbo's is the negative), so
//   lw_s = -pseudo_nll + nkl_s = +sum_m w_m NLL_sm + nkl_s;
// that sign is reproduced.  correction == 0: uniform weights (mean over s).
// out[4] (double): [0] entropy of the softmax weights over W > 0, [1] normalised
// ESS (sum W)^2 / sum W^2 / S, [2] correct predictions, [3] summed test NLL
// ([2], [3] added by eval_predict_kernel).
__global__ __launch_bounds__(1024) void eval_weights_kernel(OuterArgs a, int correction,
                                                            float* W, double* out) {
    __shared__ double red[16];
    __shared__ double lw[kOuterMaxS];
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int lane = tid & 63, wid = wave_id(), nwv = nthr >> 6;
    double sl = 0.0;
    for (int l = 0; l < a.L; ++l)
        if ((a.nkl_mask >> l) & 1u)
            for (int i = tid; i < a.n[l]; i += nthr)
                sl += log((double)softplus_f(a.params[a.poff[l] + a.n[l] + i]));
    sl = block_sum_all(sl, red);
    const double s0 = a.s0, inv2 = 0.5 / (s0 * s0), nlog = a.nkl_n * log(s0);
    for (int s = wid; s < a.S; s += nwv) {
        double ps = 0.0;
        const float* row = a.nll + (size_t)s * a.M;
        for (int m = lane; m < a.n_pseudo; m += 64) ps += (double)a.w[m] * row[m];
        ps = wave_sum_d(ps);
        if (lane == 0)
            lw[s] = ps + (-a.stats[2 * s] * inv2 - nlog + 0.5 * a.stats[2 * s + 1] + sl);
    }
    __syncthreads();
    double mx = -INFINITY, sm = 0.0;
    for (int s = tid; s < a.S; s += nthr) mx = fmax(mx, lw[s]);
    mx = block_max_all(mx, red);
    for (int s = tid; s < a.S; s += nthr) sm += exp(lw[s] - mx);
    sm = block_sum_all(sm, red);
    double ent = 0.0, s1 = 0.0, s2 = 0.0;
    for (int s = tid; s < a.S; s += nthr) {
        const double Wsoft = exp(lw[s] - mx) / sm;
        if (Wsoft > 0.0) ent -= Wsoft * log(Wsoft);
        s1 += Wsoft;
        s2 += Wsoft * Wsoft;
        W[s] = correction ? (float)Wsoft : 1.f / a.S;
    }
    ent = block_sum_all(ent, red);
    s1 = block_sum_all(s1, red);
    s2 = block_sum_all(s2, red);
    if (tid == 0) {
        out[0] = ent;
        out[1] = s1 * s1 / s2 / a.S;
        out[2] = 0.0;
        out[3] = 0.0;
    }
}

// one thread per test row: p = sum_s W_s softmax(logits_s), argmax against the
// label, and Categorical(probs=p).log_prob(y) (normalised, clamped to
// [eps, 1 - eps] with fp32 eps as torch's probs_to_logits)
__global__ __launch_bounds__(256) void eval_predict_kernel(OuterArgs a, const float* W,
                                                           const float* prob, const int32_t* z,
                                                           float* probs_out, double* out) {
    __shared__ double red[16];
    const int nt = a.M - a.n_pseudo, C = a.n_tot;  // n_tot carries C here
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    double correct = 0.0, nll = 0.0;
    if (j < nt) {
        float best = -1.f, tot = 0.f, py = 0.f;
        int arg = 0;
        const int y = z[a.n_pseudo + j];
        for (int c = 0; c < C; ++c) {
            float p = 0.f;
            for (int s = 0; s < a.S; ++s) p = fmaf(W[s], prob[((size_t)s * nt + j) * C + c], p);
            if (probs_out) probs_out[(size_t)j * C + c] = p;
            if (p > best) { best = p; arg = c; }
            tot += p;
            if (c == y) py = p;
        }
        correct = arg == y ? 1.0 : 0.0;
        const float q = fminf(fmaxf(py / tot, 1.1920929e-07f), 1.f - 1.1920929e-07f);
        nll = -(double)logf(q);
    }
    correct = block_sum_all(correct, red);
    nll = block_sum_all(nll, red);
    if (threadIdx.x == 0) {
        atomicAdd(out + 2, correct);
        atomicAdd(out + 3, nll);
    }
}

static void fill(const psvi_plan& p, OuterArgs& a);

hipError_t launch_eval(const psvi_plan& p, int n_pseudo, const float* params, const float* w,
                       const int32_t* z, const float* nll, const double* stats,
                       const float* prob, int correction, float* W, float* probs_out,
                       double* out, hipStream_t st) {
    if (p.d.S > kOuterMaxS) return hipErrorInvalidValue;
    OuterArgs a{};
    fill(p, a);
    a.n_pseudo = n_pseudo;
    a.params = params;
    a.w = w;
    a.nll = nll;
    a.stats = const_cast<double*>(stats);
    hipLaunchKernelGGL(eval_weights_kernel, dim3(1), dim3(1024), 0, st, a, correction, W, out);
    const int nt = p.d.M - n_pseudo;
    if (nt > 0) {
        OuterArgs b = a;
        b.n_tot = p.lay[p.L - 1].dout;
        hipLaunchKernelGGL(eval_predict_kernel, dim3((nt + 255) / 256), dim3(256), 0, st, b, W,
                           prob, z, probs_out, out);
    }
    return hipGetLastError();
}

// after the reparameterised backward: + sum_s ck_s sigmoid(sd_i) / softplus(sd_i)
// on every scale, and d loss / d u = sum_s du_part[s]
__global__ __launch_bounds__(256) void outer_finish_kernel(OuterArgs a, int nu) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < a.n_tot && a.grad) {
        int l = 0;
        while (l + 1 < a.L && i >= a.woff[l + 1]) ++l;
        if ((a.nkl_mask >> l) & 1u) {
            const int64_t ps = a.poff[l] + a.n[l] + (i - a.woff[l]);
            const float r = a.params[ps];
            a.grad[ps] += a.sck[0] * sigmoid_f(r) / softplus_f(r);
        }
    }
    const int j = i - a.n_tot;
    if (j >= 0 && j < nu && a.grad_u) {
        float g = 0.f;
        for (int s = 0; s < a.S; ++s) g += a.du_part[(size_t)s * nu + j];
        a.grad_u[j] = g;
    }
}

static void fill(const psvi_plan& p, OuterArgs& a) {
    a.L = p.L;
    a.S = p.d.S;
    a.M = p.d.M;
    a.n_tot = p.n_tot;
    a.family = p.family;
    a.s0 = p.d.prior_sd;
    a.nkl_mask = plan_nkl_mask(p);
    a.in_dim = plan_in_dim(p);
    a.nkl_n = 0;
    for (int l = 0; l < p.L; ++l) {
        a.batched[l] = !(p.family == PSVI_FAMILY_LENET && l == p.L - 1);
        if ((a.nkl_mask >> l) & 1u) a.nkl_n += p.lay[l].n;
    }
    for (int l = 0; l < p.L; ++l) {
        a.n[l] = p.lay[l].n;
        a.woff[l] = p.lay[l].woff;
        a.poff[l] = p.lay[l].poff;
        a.eoff[l] = p.lay[l].eoff;
        a.din[l] = p.lay[l].din;
        a.dout[l] = p.lay[l].dout;
    }
}

hipError_t launch_outer_stats(const psvi_plan& p, const float* params, const float* eps,
                              const float* x, double* stats, hipStream_t st) {
    OuterArgs a{};
    fill(p, a);
    a.params = params;
    a.eps = eps;
    a.x = x;
    a.stats = stats;
    hipLaunchKernelGGL(outer_stats_kernel, dim3(p.d.S), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_outer_combine(const psvi_plan& p, int n_pseudo, const float* params,
                                const float* w, const float* nll, const double* stats,
                                double* loss, float* rowcoef, float* ck, float* sck,
                                float* grad_w, double* sample_out, int ablated,
                                hipStream_t st) {
    if (p.d.S > kOuterMaxS) return hipErrorInvalidValue;
    OuterArgs a{};
    fill(p, a);
    a.ablated = ablated;
    a.n_pseudo = n_pseudo;
    a.params = params;
    a.w = w;
    a.nll = nll;
    a.stats = const_cast<double*>(stats);
    a.loss = loss;
    a.rowcoef = rowcoef;
    a.ck = ck;
    a.sck = sck;
    a.grad_w = grad_w;
    a.sample_out = sample_out;
    hipLaunchKernelGGL(outer_combine_kernel, dim3(1), dim3(1024), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_outer_finish(const psvi_plan& p, int n_pseudo, const float* params,
                               const float* sck, float* grad, const float* du_part,
                               float* grad_u, hipStream_t st) {
    OuterArgs a{};
    fill(p, a);
    a.n_pseudo = n_pseudo;
    a.params = params;
    a.sck = const_cast<float*>(sck);
    a.grad = grad;
    a.du_part = du_part;
    a.grad_u = grad_u;
    const int nu = grad_u ? n_pseudo * plan_in_dim(p) : 0;
    const int n = p.n_tot + nu;
    hipLaunchKernelGGL(outer_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, st, a, nu);
    return hipGetLastError();
}

// d loss / d w_m = sum_s cp_s NLL_sm (the combine kernel's last loop) for
// caller-given coefficients (psvi_outer_elbo_grad_coef)
__global__ __launch_bounds__(256) void outer_gradw_kernel(int S, int M, int n_pseudo,
                                                          const float* __restrict__ nll,
                                                          const float* __restrict__ rowcoef,
                                                          float* __restrict__ grad_w) {
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= n_pseudo) return;
    double g = 0.0;
    for (int s = 0; s < S; ++s) g += (double)rowcoef[2 * s] * nll[(size_t)s * M + m];
    grad_w[m] = (float)g;
}

hipError_t launch_outer_gradw(const psvi_plan& p, int n_pseudo, const float* nll,
                              const float* rowcoef, float* grad_w, hipStream_t st) {
    if (n_pseudo <= 0) return hipSuccess;
    hipLaunchKernelGGL(outer_gradw_kernel, dim3((n_pseudo + 255) / 256), dim3(256), 0, st,
                       p.d.S, p.d.M, n_pseudo, nll, rowcoef, grad_w);
    return hipGetLastError();
}

}  // namespace psvi
