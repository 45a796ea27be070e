// kernels_lenet.hip -- the coreset-ELBO inner step of make_lenet (config C5):
// per-sample VIConv2d + BatchMaxPool2d towers, the VILinear head as batched
// GEMMs, weighted NLL, and the hand-derived backward down to the per-sample
// weight gradients.  The parameter update (KL on the VILinear layers only,
// Adam) is the mean-field mf_update_kernel with a layer mask.
//
// Reference (/root/reference):
//   make_lenet            psvi/models/neural_net.py:334-359
//   VIConv2d.forward      neural_net.py:202-246 (grouped conv over the S-repeated
//                         input == one conv per sample with its own weights)
//   BatchMaxPool2d        neural_net.py:249-255 (2x2/2 max-pool per (s, m) map)
//   VILinear.forward      neural_net.py:176-179; the last layer's mc_samples=1
//                         gives ONE shared weight sample (neural_net.py:164-170)
//   inner_elbo            psvi/inference/psvi_classes.py:488-511
//
// Layout (per sample s, floats, the plan's woff order = parameter order):
//   conv1 W [6][1][5][5] b[6] | conv2 W [16][6][5][5] b[16] | fc1 W [120][400]
//   b[120] | fc2 W [84][120] b[84] | fc3 W [10][84] b[10]        (n_tot = 61706)
// Activations, row (s, m) major: P1 [S][M][6][14][14] (pooled conv1, kept for
// conv2's weight gradient), route1/route2 int8 (pool window index of the first
// maximum, -1 where relu zeroes it), X2 [S][M][400], H1 [S][M][120],
// H2 [S][M][84], D [S][M][10] (logits, then d logits).
#include <type_traits>

#include "psvi_internal.hpp"

namespace psvi {

int g_lenet_abl = 0;        // psvi_debug_set(PSVI_DBG_LENET_ABLATION, mask): backward parts skipped

namespace {

constexpr int kThreads = 256;
constexpr int kNConv = 2572;  // conv1 W+b, conv2 W+b: the per-sample conv block
constexpr int kP1 = 1176;     // 6 x 14 x 14
constexpr int kX2 = 400;      // 16 x 5 x 5

// ------------------------------------------------------------ weight draw
struct SampleArgs {
    int L, n_tot, S_loc, s_off, S_tot;
    int woff[kMaxL + 1], nw[kMaxL], n[kMaxL], batched[kMaxL];
    int64_t poff[kMaxL], eoff[kMaxL];
};

__device__ __forceinline__ int64_t lenet_eps_index(const SampleArgs& a, int l, int idx, int sg) {
    if (!a.batched[l]) return a.eoff[l] + idx;
    const int nw = a.nw[l];
    return idx < nw ? a.eoff[l] + (int64_t)sg * nw + idx
                    : a.eoff[l] + (int64_t)a.S_tot * nw + (int64_t)sg * (a.n[l] - nw) + (idx - nw);
}

__device__ __forceinline__ int lenet_layer(const SampleArgs& a, int j) {
    int l = 0;
    while (l + 1 < a.L && j >= a.woff[l + 1]) ++l;
    return l;
}

// Wsamp[s][j] = mu_j + softplus(rho_j) eps_(s, j)   (VIMixin.rsample, neural_net.py:155-162)
constexpr int kSampleRun = 16;  // samples per block row of lenet_sample_kernel
__global__ __launch_bounds__(kThreads) void lenet_sample_kernel(SampleArgs a,
                                                                const float* __restrict__ params,
                                                                const float* __restrict__ eps,
                                                                float* __restrict__ wsamp) {
    // thread = parameter j, block row = kSampleRun consecutive samples: mu and
    // softplus(rho) once, the eps index branches hoisted, 8 draws in flight
    const int j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.n_tot) return;
    const int l = lenet_layer(a, j);
    const int idx = j - a.woff[l];
    const float mu = params[a.poff[l] + idx], sp = softplus_f(params[a.poff[l] + a.n[l] + idx]);
    const int s0 = blockIdx.y * kSampleRun, s1 = min(a.S_loc, s0 + kSampleRun);
    const float* ep = eps + lenet_eps_index(a, l, idx, a.s_off + s0);
    const int64_t es = !a.batched[l] ? 0 : idx < a.nw[l] ? a.nw[l] : a.n[l] - a.nw[l];
    float* out = wsamp + (int64_t)s0 * a.n_tot + j;
#pragma unroll 8
    for (int s = 0; s < s1 - s0; ++s) out[(int64_t)s * a.n_tot] = mu + sp * ep[(int64_t)s * es];
}

// acc[j] = sum_s dW[s][j],  acc[n_tot + j] = sum_s dW[s][j] eps_(s, j)
// ck (outer backward, nullable): the pathwise sampled-KL gradient
// -ck_s W_s / s0^2 joins every VILinear-layer weight gradient
__global__ __launch_bounds__(kThreads) void lenet_acc_kernel(SampleArgs a,
                                                             const float* __restrict__ eps,
                                                             const float* __restrict__ dws,
                                                             float* __restrict__ acc,
                                                             const float* __restrict__ ck,
                                                             const float* __restrict__ wsamp,
                                                             float inv_s0sq) {
    const int j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= a.n_tot) return;
    const int l = lenet_layer(a, j);
    const int idx = j - a.woff[l];
    const bool path = ck != nullptr && l >= 2;
    // eps of sample s at ep[s * es] (lenet_eps_index with the branches hoisted)
    const float* ep = eps + lenet_eps_index(a, l, idx, a.s_off);
    const int64_t es = !a.batched[l] ? 0 : idx < a.nw[l] ? a.nw[l] : a.n[l] - a.nw[l];
    float g = 0.f, ge = 0.f;
    // 8 samples' loads issued together, then added in sample order
    constexpr int kU = 8;
    int s = 0;
    for (; s + kU <= a.S_loc; s += kU) {
        float d[kU], e[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            d[u] = dws[(int64_t)(s + u) * a.n_tot + j];
            e[u] = ep[(int64_t)(s + u) * es];
        }
        if (path) {
#pragma unroll
            for (int u = 0; u < kU; ++u) d[u] -= ck[s + u] * wsamp[(int64_t)(s + u) * a.n_tot + j] * inv_s0sq;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            g += d[u];
            ge += d[u] * e[u];
        }
    }
    for (; s < a.S_loc; ++s) {
        float d = dws[(int64_t)s * a.n_tot + j];
        if (path) d -= ck[s] * wsamp[(int64_t)s * a.n_tot + j] * inv_s0sq;
        g += d;
        ge += d * ep[(int64_t)s * es];
    }
    acc[j] = g;
    acc[a.n_tot + j] = ge;
}

// ------------------------------------------------------- conv towers, fwd
struct ConvArgs {
    int M, n_tot, nchunk, chunk;
    const float* u;       // [M][28][28]
    const float* wsamp;   // [S][n_tot]
    float* p1;            // [S][M][1176]
    int8_t* r1;           // [S][M][1176]
    float* x2;            // [S][M][400]
    int8_t* r2;           // [S][M][400]
    const float* dx2;     // bwd: [S][M][400]
    float* part;          // bwd: [S][nchunk][2572]
    float* du;            // bwd <DU>: [S][n_pseudo][784] input gradient of the pseudo rows
    int n_pseudo;
    int abl;              // diagnostics (PSVI_DBG_LENET_ABLATION): parts of the backward skipped
    float* g1g;           // MFMA bwd: [S][M][1176] routed d P1 (0 where relu / pool drop it)
    float* part1;         // conv1 weight-gradient partials [S][nch1][156]
    int nch1;
    const float* wdot;    // tangent forward <TAN>: [S][n_tot] W_dot
    float* p1dot;         // tangent forward <TAN>: [S][M][1176] P1_dot (conv1 out, conv2 in)
};

// relu + first-max 2x2 pool of four conv values in window order (0,0) (0,1)
// (1,0) (1,1): torch's max_pool2d keeps the first maximum; the gradient of a
// window whose maximum is <= 0 dies in relu's backward (route -1).
__device__ __forceinline__ float relu_pool4(float a0, float a1, float a2, float a3, int8_t& r) {
    float m = a0;
    int k = 0;
    if (a1 > m) { m = a1; k = 1; }
    if (a2 > m) { m = a2; k = 2; }
    if (a3 > m) { m = a3; k = 3; }
    r = m > 0.f ? (int8_t)k : (int8_t)-1;
    return m > 0.f ? m : 0.f;
}

// One workgroup per (image chunk, sample): the sample's conv weights stay in
// LDS while the chunk's images stream through.  320 threads (5 waves): the
// bwd kernel's 294 transposed-conv blocks fit in one pass.
constexpr int kConvThreads = 320;

// ------------------------------------- conv towers, fwd, on the matrix cores
// Both convolutions as implicit GEMMs on v_mfma_f32_16x16x4_f32 (fp32 in,
// fp32 accumulate: an ordered fmaf chain per output, bias in the accumulator).
// Fragment maps (16x16x4 f32): A[row l & 15][k l >> 4], B[k l >> 4][col l & 15],
// C/D col l & 15, rows 4 (l >> 4) + i (i = 0..3).  Rows are ordered (pool
// window, window offset q = 2 dy + dx), so a lane's four accumulators are the
// four conv values of ONE 2x2 pool window: relu + first-max pool run in the
// epilogue on registers (window order (0,0) (0,1) (1,0) (1,1), as relu_pool4).
typedef float f32x4 __attribute__((ext_vector_type(4)));

// the conv value at the primal's routed pool offset r (0 where relu / pool drop it)
__device__ __forceinline__ float routed4(const f32x4& v, int r) {
    return r == 0 ? v[0] : r == 1 ? v[1] : r == 2 ? v[2] : r == 3 ? v[3] : 0.f;
}

// conv1 (1 -> 6, 5x5, pad 2) of one image for 8 samples at once: the image's
// im2col [784 conv positions x 25 taps] (padded image in LDS) times the 8
// samples' filters [25 taps x 48 (sample, channel) columns] -- the image is
// shared by every sample (VIConv2d's grouped conv over the S-repeated input,
// neural_net.py:202-246), so one A fragment feeds three column tiles.  K = 25
// padded to 28 (B rows 25..27 are zero).  49 row tiles of 16 (4 windows x 4
// offsets) per image, dealt to the 4 waves.
constexpr int kC1S = 8;           // samples per workgroup (48 columns)
constexpr int kC1RS = 38;         // padded-image row stride (ds_read_b32 banks: tools/lds_banks)
constexpr int kC1Img = 32 * kC1RS;
// TAN: the tangent forward -- W_dot's filters and bias, and instead of relu +
// pool the value at the primal's routed offset (0 where relu / pool drop it)
// into a.p1dot, a.r1 read.
template <bool TAN>
__global__ __launch_bounds__(256) void lenet_conv1_mfma_kernel(ConvArgs a, int S_loc) {
    __shared__ float img[2][kC1Img];
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    const int s0 = blockIdx.y * kC1S;
    const int r16 = lane & 15, kq = lane >> 4;
    // B fragments and the accumulators' bias: column n = 16 nt + r16 is
    // (sample s0 + n / 6, channel n % 6)
    float bf[3][7], bias[3];
    bool col_ok[3];
    int64_t col_out[3];
#pragma unroll
    for (int nt = 0; nt < 3; ++nt) {
        const int n = 16 * nt + r16, sl = n / 6, c = n % 6;
        col_ok[nt] = s0 + sl < S_loc;
        const float* ws = (TAN ? a.wdot : a.wsamp) + (int64_t)min(s0 + sl, S_loc - 1) * a.n_tot;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const int k = 4 * t + kq;
            bf[nt][t] = (k < 25 && col_ok[nt]) ? ws[c * 25 + k] : 0.f;
        }
        bias[nt] = ws[150 + c];
        col_out[nt] = (int64_t)(s0 + sl) * a.M * kP1 + c * 196;
    }
    // A fragment: tap k = 4 t + kq -> (i, j) offset in the padded image
    int koff[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        const int k = min(4 * t + kq, 24);
        koff[t] = (k / 5) * kC1RS + k % 5;
    }
    const int m0 = blockIdx.x * a.chunk, m1 = min(a.M, m0 + a.chunk);
    auto load_img = [&](int m, float* dst) __attribute__((always_inline)) {
        const float* um = a.u + (int64_t)m * 784;
        for (int i = tid; i < 1024; i += 256) {
            const int y = (i >> 5) - 2, x = (i & 31) - 2;
            dst[(i >> 5) * kC1RS + (i & 31)] =
                (y >= 0 && y < 28 && x >= 0 && x < 28) ? um[y * 28 + x] : 0.f;
        }
    };
    if (m0 < m1) load_img(m0, img[0]);
    int buf = 0;
    for (int m = m0; m < m1; ++m, buf ^= 1) {
        __syncthreads();  // img[buf] complete; img[buf ^ 1] free
        if (m + 1 < m1) load_img(m + 1, img[buf ^ 1]);
        const float* im = img[buf];
        for (int mt = wv; mt < 49; mt += 4) {
            // this lane's A row: window g = 4 mt + r16 / 4, offset q = r16 % 4
            const int g = 4 * mt + (r16 >> 2), q = r16 & 3;
            const int rowoff = (2 * (g / 14) + (q >> 1)) * kC1RS + 2 * (g % 14) + (q & 1);
            f32x4 acc[3];
#pragma unroll
            for (int nt = 0; nt < 3; ++nt) acc[nt] = f32x4{bias[nt], bias[nt], bias[nt], bias[nt]};
            float av[7];
#pragma unroll
            for (int t = 0; t < 7; ++t) av[t] = im[rowoff + koff[t]];
#pragma unroll
            for (int t = 0; t < 7; ++t)
#pragma unroll
                for (int nt = 0; nt < 3; ++nt)
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bf[nt][t], acc[nt], 0, 0, 0);
            // epilogue: lane holds window 4 mt + kq of column r16 (4 offsets)
            const int gw = 4 * mt + kq;
#pragma unroll
            for (int nt = 0; nt < 3; ++nt) {
                if (!col_ok[nt]) continue;
                const int64_t o = col_out[nt] + (int64_t)m * kP1 + gw;
                if (TAN) {
                    a.p1dot[o] = routed4(acc[nt], a.r1[o]);
                } else {
                    int8_t r;
                    a.p1[o] = relu_pool4(acc[nt][0], acc[nt][1], acc[nt][2], acc[nt][3], r);
                    a.r1[o] = r;
                }
            }
        }
    }
}

// conv2 (6 -> 16, 5x5) of one sample: per image the im2col of the pooled
// conv1 map [100 conv positions x 150 taps (c, i, j)] times the sample's
// filters [150 x 16 output channels].  One wave per workgroup, two images per
// pass: 200 rows = 13 row tiles of 16 (4 windows x 4 offsets; windows 25..49
// are the second image's), two tiles in flight (two accumulator chains against
// the 40-cycle MFMA latency).  The pair's P1 maps sit in LDS as they lie in
// HBM (rows 14 floats, channel planes 196: a straight float4 copy; the reads
// below average ~3 LDS cycles against the MFMA's 32); 4 waves per SIMD (LDS
// bound) hide each other's copies (a register prefetch of the next pair cost
// 40 VGPRs and a wave of occupancy).  K = 150 in 38 steps, ordered
// so every lane's A address is (row offset) + (its kq times a stride) + an
// immediate: steps 0..29 tap (c, i, j = kq) for (c, i) = (t / 5, t % 5);
// steps 30..35 tap (t - 30, i = kq, 4); steps 36, 37 tap (4 (t - 36) + kq, 4,
// 4), channels 6 and 7 zero in B (their A reads clamped to channel 5).
constexpr int kC2Pair = 2 * kP1;
constexpr int kC2Q = kC2Pair / 4 / 64 + 1;  // float4 per lane per pair (588 / 64 -> 10)
//
// TAN: the tangent forward, X2_dot = conv(P1_dot, W2) + conv(P1, W2_dot) +
// b2_dot at the primal's routed offsets (a.r2 read, a.x2 written): K = 2 x 150
// over the pair's P1 | P1_dot maps in LDS (two waves per SIMD).
template <bool TAN>
__global__ __launch_bounds__(64) void lenet_conv2_mfma_kernel(ConvArgs a) {
    __shared__ __attribute__((aligned(16))) float pm[TAN ? 2 * kC2Pair : kC2Pair];
    const int lane = threadIdx.x, r16 = lane & 15, kq = lane >> 4;
    const int s = blockIdx.y;
    const float* ws = a.wsamp + (int64_t)s * a.n_tot;
    auto load_b = [&](const float* w2, float (&b)[38]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 30; ++t) b[t] = w2[(t / 5) * 25 + (t % 5) * 5 + kq];
#pragma unroll
        for (int t = 30; t < 36; ++t) b[t] = w2[(t - 30) * 25 + kq * 5 + 4];
        b[36] = w2[kq * 25 + 24];
        b[37] = kq < 2 ? w2[(4 + kq) * 25 + 24] : 0.f;
    };
    float bf[38], bfd[38];
    load_b(ws + 156 + r16 * 150, bf);
    const float* wds = TAN ? a.wdot + (int64_t)s * a.n_tot : ws;
    if (TAN) load_b(wds + 156 + r16 * 150, bfd);
    const float bias = wds[2556 + r16];
    const int oj = kq, oi = kq * 14, oc = kq * 196, oc2 = min(kq, 1) * 196;
    const int npair = (a.M + 1) >> 1;
    const int p0 = blockIdx.x * a.chunk, p1 = min(npair, p0 + a.chunk);
    if (p0 >= p1) return;
    // the pair's maps HBM -> LDS (float4 loads in flight together, then stored;
    // one function-local array, so it stays in registers)
    auto copy_pair = [&](const float* base, int p, float* d) __attribute__((always_inline)) {
        const int n4 = (min(a.M, 2 * p + 2) - 2 * p) * (kP1 / 4);
        const float4* sp = reinterpret_cast<const float4*>(base + (int64_t)s * a.M * kP1) +
                           (int64_t)p * (kC2Pair / 4);
        float4 pf[kC2Q];
#pragma unroll
        for (int q = 0; q < kC2Q; ++q) pf[q] = sp[min(lane + 64 * q, n4 - 1)];
#pragma unroll
        for (int q = 0; q < kC2Q; ++q) {
            const int i = lane + 64 * q;
            if (i < kC2Pair / 4) reinterpret_cast<float4*>(d)[i] = pf[q];
        }
    };
    for (int p = p0; p < p1; ++p) {
        __syncthreads();  // the previous pair's reads are done
        copy_pair(a.p1, p, pm);
        if (TAN) copy_pair(a.p1dot, p, pm + kC2Pair);
        __syncthreads();
        const bool two_img = 2 * p + 1 < a.M;  // uniform
        // NT row tiles from tile mt on: 38 MFMA steps each, then relu + pool
        auto tiles = [&](int mt, auto nt_c) __attribute__((always_inline)) {
            constexpr int NT = decltype(nt_c)::value;
            int ro[NT];
            f32x4 acc[NT];
#pragma unroll
            for (int h = 0; h < NT; ++h) {
                const int g = min(4 * (mt + h) + (r16 >> 2), 49), q = r16 & 3;
                const int im = g >= 25, w = g - 25 * im;
                ro[h] = im * kP1 + (2 * (w / 5) + (q >> 1)) * 14 + 2 * (w % 5) + (q & 1);
                acc[h] = f32x4{bias, bias, bias, bias};
            }
            // primal: P1 x W2; tangent: P1_dot x W2, then P1 x W2_dot
            const float* am = TAN ? pm + kC2Pair : pm;
#pragma unroll
            for (int t = 0; t < 38; ++t) {
                const int off = t < 30 ? oj + (t / 5) * 196 + (t % 5) * 14
                              : t < 36 ? oi + (t - 30) * 196 + 4
                              : t == 36 ? oc + 60 : oc2 + 4 * 196 + 60;
#pragma unroll
                for (int h = 0; h < NT; ++h)
                    acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(am[ro[h] + off], bf[t], acc[h], 0, 0, 0);
            }
            if (TAN) {
#pragma unroll
                for (int t = 0; t < 38; ++t) {
                    const int off = t < 30 ? oj + (t / 5) * 196 + (t % 5) * 14
                                  : t < 36 ? oi + (t - 30) * 196 + 4
                                  : t == 36 ? oc + 60 : oc2 + 4 * 196 + 60;
#pragma unroll
                    for (int h = 0; h < NT; ++h)
                        acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(pm[ro[h] + off], bfd[t], acc[h], 0, 0, 0);
                }
            }
#pragma unroll
            for (int h = 0; h < NT; ++h) {
                const int g = 4 * (mt + h) + kq;
                if (g >= 50 || (g >= 25 && !two_img)) continue;
                const int im = g >= 25, w = g - 25 * im;
                const int64_t o = ((int64_t)s * a.M + 2 * p + im) * kX2 + r16 * 25 + w;
                if (TAN) {
                    a.x2[o] = routed4(acc[h], a.r2[o]);
                } else {
                    int8_t r;
                    a.x2[o] = relu_pool4(acc[h][0], acc[h][1], acc[h][2], acc[h][3], r);
                    a.r2[o] = r;
                }
            }
        };
#pragma unroll 1
        for (int mt = 0; mt < 12; mt += 2) tiles(mt, std::integral_constant<int, 2>{});
        tiles(12, std::integral_constant<int, 1>{});  // windows 48, 49 (rows 50, 51 clamped)
    }
}

// ------------------------------------------------------- conv towers, bwd
// Given d X2 (the head's input gradient) per (s, m): route through pool2/relu
// (one conv2 position per pooled output), accumulate conv2's weight gradient
// against P1 (25 routed terms per weight), form d P1 as the transposed conv
// of the routed map (dense, zero-padded in LDS, 2x2 output blocks per thread),
// route through pool1/relu, accumulate conv1's weight gradient against the
// padded image.  Per-(s, chunk) partial sums, reduced over chunks in fixed
// order by lenet_conv_reduce_kernel: bitwise run-to-run reproducible.
// The backward's LDS layouts, against ds_read_b32 bank conflicts: the padded
// image with 37-word rows, so the 25 taps (i, j) of one conv1 weight row
// block sit on 25 banks.
constexpr int kBS = 37;               // padded-image row stride in the backward
// the pooled conv1 map P1 likewise: 37-word rows, channel planes 537 words
// apart, so the 25 taps of a conv2 weight block and the next channel's first
// taps fall on distinct banks
constexpr int kP1S = 37, kP1C = 14 * kP1S + 19;
// DU (outer backward): also d u = the transposed conv1 of the routed conv1
// gradient (dense, zero-bordered LDS plane, 2x2 pixel blocks per thread) for
// the pseudopoint rows m < n_pseudo.
// The same backward with d P1 on the matrix cores.  Each pool2 window w
// (5x5 per channel) routes its gradient g2[k][w] to ONE of its four conv2
// positions q = 2 dy + dx, so the transposed conv2 of the routed map is, per
// window, a 6x6 patch per input channel:
//   U[w][(c, ay, ax)] = sum_(k, q) A[w][(k, q)] B[(k, q)][(c, ay, ax)],
//   A[w][(k, q)] = g2[k][w] if window (k, w) routes to q else 0,
//   B[(k, q)][(c, ay, ax)] = W2[k][c][ay - dy][ax - dx] (0 outside the 5x5),
// a [25 windows x 64] x [64 x 216] GEMM per image (v_mfma_f32_16x16x4_f32: 2
// row tiles, 14 column tiles dealt to the 5 waves, k-step = output channel
// k, lane group = q); then d P1[c][y][x] = the sum, in window order, of the
// (<= 9) patches covering (y, x) (stride 2: window (wy, wx) covers rows
// 2 wy .. 2 wy + 5).  Per (image chunk, sample) partials as the other conv
// kernels (fixed-order chunk sums).
constexpr int kUS = 217;  // LDS row stride of U (216 patch columns)
constexpr int kGK = 33, kGQ = 16 * kGK;  // routed-map rows / offset planes (ga below)
template <bool DU>
__global__ __launch_bounds__(kConvThreads, DU ? 2 : 3) void lenet_conv_bwd_mfma_kernel(ConvArgs a) {
    __shared__ float w1[DU ? 150 : 1];
    __shared__ float da1[DU ? 6 * 1024 : 1];  // routed conv1 gradient, 28x28 + 2-wide zero border
    __shared__ float in[DU ? 32 * kBS : 1];
    __shared__ float p1[6 * kP1C];   // [c][y * kP1S + x]
    __shared__ float g2[kX2];        // routed gradient of each pooled conv2 output
    // the routed map expanded by window offset: ga[q][k][w] = g2[k][w] if
    // window (k, w) routes to q else 0 (w 25..32 zero): the A operand of both
    // GEMMs below, read unconditionally (rows 33 apart, offset planes 528:
    // both read patterns hit 32 distinct banks per half-wave)
    __shared__ float ga[4 * kGQ];
    __shared__ float U[25 * kUS + 1];  // per-window 6x6 d P1 patches, then one zero
    float* w2 = U;  // conv2's filters until the B fragments are loaded (U is first written
                    // after the image loop's first barrier)
    __shared__ float g1[DU ? kP1 : 1];   // DU: routed gradient of each pooled conv1 output
    __shared__ int off1[DU ? kP1 : 1];   // DU: its conv1 position y * kBS + x (padded image)
    __shared__ int8_t r1s[kP1];      // the image's pool1 routes
    const int tid = threadIdx.x, s = blockIdx.y;
    const int lane = tid & 63, wv = wave_id(), r16 = lane & 15, kq = lane >> 4;
    const float* ws = a.wsamp + (int64_t)s * a.n_tot;
    for (int i = tid; i < 2400; i += kConvThreads) w2[i] = ws[156 + i];
    if (DU) {
        for (int i = tid; i < 150; i += kConvThreads) w1[i] = ws[i];
        for (int i = tid; i < 6 * 1024; i += kConvThreads) da1[i] = 0.f;
    }
    __syncthreads();
    // B fragments of this wave's column tiles nt = wv + 5 j (< 14): k-step t =
    // output channel k, lane group kq = q = (dy, dx), column n = (c, ay, ax)
    constexpr int kNT = 3;
    const int ntw = wv < 4 ? 3 : 2;  // wave-uniform
    float bf[kNT][16];
#pragma unroll
    for (int j = 0; j < kNT; ++j) {
        const int n = 16 * (wv + 5 * j) + r16;
        const int c = n / 36, ay = (n % 36) / 6 - (kq >> 1), ax = n % 6 - (kq & 1);
        const bool ok = j < ntw && n < 216 && ay >= 0 && ay < 5 && ax >= 0 && ax < 5;
        const int wo = ok ? c * 25 + ay * 5 + ax : 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) bf[j][t] = ok ? w2[t * 150 + wo] : 0.f;
    }
    if (tid == 0) U[25 * kUS] = 0.f;
    for (int i = tid; i < 4 * kGQ; i += kConvThreads) ga[i] = 0.f;
    // conv2 weight gradient on the matrix cores, accumulated over the chunk's
    // images in registers: dW2[k][(c, i, j)] += sum_(w, q) A[k][(w, q)]
    // P1[c][2 wy + dy + i][2 wx + dx + j] (the routed map as A, k-step = pool
    // window w, lane group = offset q; the im2col of P1 as B, one LDS read per
    // MFMA).  Wave wv owns column tiles 2 wv, 2 wv + 1 of the 150 (c, i, j).
    int nb2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int n = min(16 * (2 * wv + h) + r16, 149);
        nb2[h] = (n / 25) * kP1C + ((n % 25) / 5) * kP1S + n % 5;
    }
    const int kqoff = (kq >> 1) * kP1S + (kq & 1);
    f32x4 accw2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    float accb2 = 0.f;
    // DU: the padded image's zero border, once (the interior is rewritten per image)
    for (int i = tid; i < 1024 && DU; i += kConvThreads) {
        const int y = (i >> 5) - 2, x = (i & 31) - 2;
        if (!(y >= 0 && y < 28 && x >= 0 && x < 28)) in[(i >> 5) * kBS + (i & 31)] = 0.f;
    }
    // Per-image inputs in registers, loaded one image ahead (the next image's
    // global loads are in flight behind this image's compute): u interior 784,
    // P1 1176, pool1 routes 1176 bytes, pool2 routes and d X2 400 each
    constexpr int kLU = (784 + kConvThreads - 1) / kConvThreads;   // 3
    constexpr int kLP = (kP1 + kConvThreads - 1) / kConvThreads;   // 4
    constexpr int kLX = (kX2 + kConvThreads - 1) / kConvThreads;   // 2
    float pu[kLU], pp[kLP], pg[kLX];
    int8_t pr1[kLP], pr2[kLX];
    const int m0 = blockIdx.x * a.chunk, m1 = min(a.M, m0 + a.chunk);
    auto fetch = [&](int m) __attribute__((always_inline)) {
        const int64_t row = (int64_t)s * a.M + m;
        const float* um = a.u + (int64_t)m * 784;
#pragma unroll
        for (int k = 0; k < kLU; ++k) pu[k] = DU ? um[min(tid + k * kConvThreads, 783)] : 0.f;
#pragma unroll
        for (int k = 0; k < kLP; ++k) {
            const int i = min(tid + k * kConvThreads, kP1 - 1);
            pp[k] = a.p1[row * kP1 + i];
            pr1[k] = a.r1[row * kP1 + i];
        }
#pragma unroll
        for (int k = 0; k < kLX; ++k) {
            const int o = min(tid + k * kConvThreads, kX2 - 1);
            pg[k] = a.dx2[row * kX2 + o];
            pr2[k] = a.r2[row * kX2 + o];
        }
    };
    if (m0 < m1) fetch(m0);
    for (int m = m0; m < m1; ++m) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kLU; ++k) {
            const int i = tid + k * kConvThreads;
            if (DU && i < 784 && !(a.abl & 16)) in[(i / 28 + 2) * kBS + i % 28 + 2] = pu[k];
        }
#pragma unroll
        for (int k = 0; k < kLP; ++k) {
            const int i = tid + k * kConvThreads;
            if (i < kP1 && !(a.abl & 32)) {
                p1[(i / 196) * kP1C + ((i % 196) / 14) * kP1S + i % 14] = pp[k];
                r1s[i] = pr1[k];
            }
        }
#pragma unroll
        for (int k = 0; k < kLX; ++k) {
            const int o = tid + k * kConvThreads;
            if (o < kX2) {
                const int r = pr2[k], kk = o / 25, w = o % 25;
                const float g = r >= 0 ? pg[k] : 0.f;
                g2[o] = g;
#pragma unroll
                for (int q = 0; q < 4; ++q) ga[q * kGQ + kk * kGK + w] = r == q ? g : 0.f;
            }
        }
        if (m + 1 < m1) fetch(m + 1);
        __syncthreads();
        // d P1 patches on the matrix cores (U), two row tiles of windows; the
        // wave's column-tile count as a template constant (no branch per MFMA)
        auto dp1 = [&](auto nt_c) __attribute__((always_inline)) {
            constexpr int NT = decltype(nt_c)::value;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const float* ar = ga + kq * kGQ + 16 * mt + r16;
                f32x4 acc[NT];
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const float av = ar[t * kGK];
#pragma unroll
                    for (int j = 0; j < NT; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bf[j][t], acc[j], 0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const int n = 16 * (wv + 5 * j) + r16;
                    if (n >= 216) continue;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int wr = 16 * mt + 4 * kq + i;
                        if (wr < 25) U[wr * kUS + n] = acc[j][i];
                    }
                }
            }
        };
        if (!(a.abl & 1)) {
            if (ntw == 3)
                dp1(std::integral_constant<int, 3>{});
            else
                dp1(std::integral_constant<int, 2>{});
        }
        // conv2 weight gradient (MFMA, see above)
        if (!(a.abl & 2)) {
            const float* ar = ga + kq * kGQ + r16 * kGK;
#pragma unroll 5
            for (int t = 0; t < 25; ++t) {
                const float av = ar[t];
                const int po = kqoff + 2 * (t / 5) * kP1S + 2 * (t % 5);
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    accw2[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, p1[nb2[h] + po], accw2[h],
                                                                    0, 0, 0);
            }
        }
        if (tid < 16) {
            float acc = 0.f;
            for (int p = 0; p < 25; ++p) acc += g2[tid * 25 + p];
            accb2 += acc;
        }
        __syncthreads();
        // d P1 = the covering patches in window order (windows wy = y / 2 - 2
        // .. y / 2, the ones off the map read the zero slot), routed through
        // pool1 / relu; the 9 reads of an output issued together
#pragma unroll 2
        for (int k = 0; k < 4; ++k) {
            const int o = tid + k * kConvThreads;
            if (o >= kP1 || (a.abl & 4)) break;
            const int c = o / 196, y = (o % 196) / 14, x = o % 14;
            const int by = (y >> 1) - 2, bx = (x >> 1) - 2;
            int uo[9];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int wy = by + dy, wx = bx + dx;
                    const bool in_map = wy >= 0 && wy < 5 && wx >= 0 && wx < 5;
                    uo[dy * 3 + dx] = in_map ? (wy * 5 + wx) * kUS + c * 36 +
                                                   ((y & 1) + 4 - 2 * dy) * 6 + (x & 1) + 4 - 2 * dx
                                             : 25 * kUS;
                }
            float uv[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) uv[q] = U[uo[q]];
            float v = 0.f;
#pragma unroll
            for (int q = 0; q < 9; ++q) v += uv[q];
            const int r = r1s[o];
            a.g1g[((int64_t)s * a.M + m) * kP1 + o] = r >= 0 ? v : 0.f;
            if (DU) {
                const int rr = r >= 0 ? r : 0;
                g1[o] = r >= 0 ? v : 0.f;
                off1[o] = (2 * y + (rr >> 1)) * kBS + 2 * x + (rr & 1);
            }
        }
        if (DU && m < a.n_pseudo) {
            __syncthreads();
            for (int o = tid; o < kP1; o += kConvThreads)
                da1[(o / 196) * 1024 + (off1[o] / kBS + 2) * 32 + off1[o] % kBS + 2] = g1[o];
            __syncthreads();
            if (tid < 196) {
                const int yy = 2 * (tid / 14), xx = 2 * (tid % 14);
                float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
                for (int c = 0; c < 6; ++c) {
                    const float* q = da1 + c * 1024 + yy * 32 + xx;
                    float Q[6][6];
#pragma unroll
                    for (int i = 0; i < 6; ++i)
#pragma unroll
                        for (int j = 0; j < 6; ++j) Q[i][j] = q[i * 32 + j];
#pragma unroll
                    for (int i = 0; i < 5; ++i)
#pragma unroll
                        for (int j = 0; j < 5; ++j) {
                            const float wv1 = w1[c * 25 + i * 5 + j];
                            acc[0] += wv1 * Q[4 - i][4 - j];
                            acc[1] += wv1 * Q[4 - i][5 - j];
                            acc[2] += wv1 * Q[5 - i][4 - j];
                            acc[3] += wv1 * Q[5 - i][5 - j];
                        }
                }
                float* out = a.du + ((int64_t)s * a.n_pseudo + m) * 784 + yy * 28 + xx;
                out[0] = acc[0];
                out[1] = acc[1];
                out[28] = acc[2];
                out[29] = acc[3];
            }
            __syncthreads();
            for (int o = tid; o < kP1; o += kConvThreads)
                da1[(o / 196) * 1024 + (off1[o] / kBS + 2) * 32 + off1[o] % kBS + 2] = 0.f;
        }
    }
    float* out = a.part + ((int64_t)s * a.nchunk + blockIdx.x) * kNConv;
    if (tid < 16) out[2556 + tid] = accb2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int n = 16 * (2 * wv + h) + r16;
        if (n < 150) {
#pragma unroll
            for (int i = 0; i < 4; ++i) out[156 + (4 * kq + i) * 150 + n] = accw2[h][i];
        }
    }
}

// conv1's weight and bias gradients on the matrix cores, 8 samples per
// workgroup (the image im2col is shared by every sample, as in the forward):
//   dW1[s][c][(i, j)] = sum over images m, pooled positions p, offsets q of
//     A[(s, c)][(p, q)] B[(p, q)][(i, j)],
//   A = g1[s][m][c][p] if the pool1 window (s, m, c, p) routes to q else 0
//     (g1: the routed d P1 the backward wrote),
//   B = img_m[2 py + dy + i][2 px + dx + j] (padded image), plus a column of
//     ones for the bias.
// Rows (sample, channel) 48 = 3 tiles, columns 25 taps + bias = 2 tiles,
// k-step = pooled position p, lane group = q.  Wave w takes p in [49 w, 49 w
// + 49) of every image; its six accumulators live across the chunk's images
// and the four waves' partials are added in wave order at the end.
constexpr int kW1S = 8;
__global__ __launch_bounds__(256) void lenet_conv1_wgrad_mfma_kernel(ConvArgs a, int S_loc) {
    __shared__ float img[kC1Img];
    __shared__ __attribute__((aligned(16))) float gs[kW1S * kP1];
    __shared__ __attribute__((aligned(16))) int8_t rs[kW1S * kP1];
    __shared__ float red[3][48 * 26];
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), r16 = lane & 15, kq = lane >> 4;
    const int s0 = blockIdx.y * kW1S;
    const int ns = min(kW1S, S_loc - s0);
    for (int i = tid; i < kC1Img; i += 256) img[i] = 0.f;
    // A rows of this lane: (sample, channel) = row / 6, row % 6; B columns:
    // taps n < 25 at (n / 5) * kC1RS + n % 5, n = 25 the bias (B = 1)
    int aoff[3];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
        const int row = 16 * mt + r16;
        aoff[mt] = (row / 6) * kP1 + (row % 6) * 196;
    }
    int boff[2];
    bool btap[2], bone[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int n = 16 * nt + r16;
        btap[nt] = n < 25;
        bone[nt] = n == 25;
        boff[nt] = btap[nt] ? (n / 5) * kC1RS + n % 5 : 0;
    }
    const int qoff = (kq >> 1) * kC1RS + (kq & 1);
    f32x4 acc[3][2];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int p0 = 49 * wv;
    const int m0 = blockIdx.x * a.chunk, m1 = min(a.M, m0 + a.chunk);
    // the next image's inputs in registers (loads in flight behind this
    // image's MFMAs): the 8 samples' routed d P1 as float4, their routes as
    // 4-byte words, the image as float4 (196 per image)
    constexpr int kQ = kP1 / 4;                        // 294 quads per (s, m)
    constexpr int kNQ = (kW1S * kQ + 255) / 256;       // 10 per thread
    float4 pg[kNQ];
    int pr[kNQ];
    float4 pu;
    const bool u16 = ((uintptr_t)a.u & 15) == 0;  // the caller's u: float4 loads when aligned
    auto fetch = [&](int m) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < kNQ; ++k) {
            const int i = min(tid + 256 * k, kW1S * kQ - 1), sl = i / kQ;
            const int64_t src = ((int64_t)(s0 + min(sl, ns - 1)) * a.M + m) * kQ + i % kQ;
            pg[k] = reinterpret_cast<const float4*>(a.g1g)[src];
            pr[k] = reinterpret_cast<const int*>(a.r1)[src];
        }
        const float* uq = a.u + (int64_t)m * 784 + 4 * min(tid, 195);
        if (u16)
            pu = *reinterpret_cast<const float4*>(uq);
        else
            pu = make_float4(uq[0], uq[1], uq[2], uq[3]);
    };
    if (m0 < m1) fetch(m0);
    for (int m = m0; m < m1; ++m) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kNQ; ++k) {
            const int i = tid + 256 * k;
            if (i < kW1S * kQ) {
                const bool live = i / kQ < ns;
                reinterpret_cast<float4*>(gs)[i] = live ? pg[k] : make_float4(0.f, 0.f, 0.f, 0.f);
                reinterpret_cast<int*>(rs)[i] = pr[k];
            }
        }
        if (tid < 196) {
            const int y = (4 * tid) / 28, x = (4 * tid) % 28;
            float* d = img + (y + 2) * kC1RS + x + 2;
            d[0] = pu.x; d[1] = pu.y; d[2] = pu.z; d[3] = pu.w;
        }
        if (m + 1 < m1) fetch(m + 1);
        __syncthreads();
#pragma unroll 7
        for (int pp = 0; pp < 49; ++pp) {
            const int p = p0 + pp;
            float av[3], bv[2];
#pragma unroll
            for (int mt = 0; mt < 3; ++mt) av[mt] = rs[aoff[mt] + p] == kq ? gs[aoff[mt] + p] : 0.f;
            const int po = 2 * (p / 14) * kC1RS + 2 * (p % 14) + qoff;
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
                bv[nt] = btap[nt] ? img[po + boff[nt]] : (bone[nt] ? 1.f : 0.f);
#pragma unroll
            for (int mt = 0; mt < 3; ++mt)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], bv[nt], acc[mt][nt],
                                                                       0, 0, 0);
        }
    }
    // the four waves' partials, added in wave order (red holds waves 1..3)
    __syncthreads();
    if (wv > 0) {
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int n = 16 * nt + r16;
                if (n < 26)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        red[wv - 1][(16 * mt + 4 * kq + i) * 26 + n] = acc[mt][nt][i];
            }
    }
    __syncthreads();
    if (wv == 0) {
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int n = 16 * nt + r16;
                if (n >= 26) continue;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = 16 * mt + 4 * kq + i, sl = row / 6, c = row % 6;
                    if (sl >= ns) continue;
                    float v = acc[mt][nt][i];
#pragma unroll
                    for (int w = 0; w < 3; ++w) v += red[w][row * 26 + n];
                    float* out = a.part1 + ((int64_t)(s0 + sl) * a.nch1 + blockIdx.x) * 156;
                    out[n < 25 ? c * 25 + n : 150 + c] = v;
                }
            }
    }
}

// dws[s][e] = sum over chunks of the conv weight-gradient partials (fixed
// order); part1 (nullable): conv1's entries e < 156 from its own partials
__global__ __launch_bounds__(kThreads) void lenet_conv_reduce_kernel(int S_loc, int nchunk,
                                                                     int n_tot,
                                                                     const float* __restrict__ part,
                                                                     float* __restrict__ dws,
                                                                     const float* __restrict__ part1,
                                                                     int nch1) {
    const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (i >= (int64_t)S_loc * kNConv) return;
    const int s = (int)(i / kNConv), e = (int)(i % kNConv);
    float g = 0.f;
    if (part1 && e < 156) {
        const float* p = part1 + (int64_t)s * nch1 * 156 + e;
        for (int c = 0; c < nch1; ++c) g += p[(int64_t)c * 156];
    } else {
        const float* p = part + (int64_t)s * nchunk * kNConv + e;
        for (int c = 0; c < nchunk; ++c) g += p[(int64_t)c * kNConv];
    }
    dws[(int64_t)s * n_tot + e] = g;
}

// ---------------------------------------------------------- head GEMMs
// C[b](m, n) = sum_k A[b](m, k) B[b](k, n) with arbitrary element strides,
// on the matrix cores (the head is 1/7 of the step's flops).  Epilogue flags, in order: 8 add the
// existing C (a second product of a tangent), 1 add bias[b][n], 2 relu, 4
// multiply by (mask[b](m, n) > 0) (relu's backward).  GemmArgs:
struct GemmArgs {
    int M, N, K;
    const float* A; int64_t sAb; int sAm, sAk;
    const float* B; int64_t sBb; int sBk, sBn;
    float* C; int64_t sCb; int sCm;
    int epi;
    const float* bias; int64_t sbias;
    const float* mask; int64_t sMb; int sMm;
};

// 64x64 tiles, four waves of one 32x32 v_mfma_f32_32x32x2_f32 accumulator each, k-steps of 16 staged through
// two LDS buffers (the next step's operands are loaded into registers before
// this step's MFMAs and written to the other buffer after them: one barrier
// per step).  Operand reads: lane l takes A(m0 + 32 wr + l % 32, k + l / 32)
// and B(k + l / 32, n0 + 32 wc + l % 32) -- 68-word LDS rows, conflict free.
// Accumulator element q of lane l is C(32 wr + 8 (q / 4) + 4 (l / 32) + q % 4,
// 32 wc + l % 32).
typedef float gemm_f32x16 __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(kThreads) void lenet_gemm_mfma_kernel(GemmArgs g) {
    __shared__ float As[2][16][68];
    __shared__ float Bs[2][16][68];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1, h = lane >> 5, l32 = lane & 31;
    const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64, b = blockIdx.z;
    const float* A = g.A + b * g.sAb;
    const float* B = g.B + b * g.sBb;
    const bool a_kfast = g.sAk == 1, b_nfast = g.sBn == 1;
    float ra[4], rb[4];
    auto gload = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = tid + r * kThreads;
            int mm, kk;
            if (a_kfast) { kk = e & 15; mm = e >> 4; } else { mm = e & 63; kk = e >> 6; }
            const int gm = m0 + mm, gk = k0 + kk;
            ra[r] = (gm < g.M && gk < g.K) ? A[(int64_t)gm * g.sAm + (int64_t)gk * g.sAk] : 0.f;
            int nn, kb;
            if (b_nfast) { nn = e & 63; kb = e >> 6; } else { kb = e & 15; nn = e >> 4; }
            const int gn = n0 + nn, gkb = k0 + kb;
            rb[r] = (gn < g.N && gkb < g.K) ? B[(int64_t)gkb * g.sBk + (int64_t)gn * g.sBn] : 0.f;
        }
    };
    auto sstore = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int e = tid + r * kThreads;
            int mm, kk;
            if (a_kfast) { kk = e & 15; mm = e >> 4; } else { mm = e & 63; kk = e >> 6; }
            As[buf][kk][mm] = ra[r];
            int nn, kb;
            if (b_nfast) { nn = e & 63; kb = e >> 6; } else { kb = e & 15; nn = e >> 4; }
            Bs[buf][kb][nn] = rb[r];
        }
    };
    gemm_f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    gload(0);
    sstore(0);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < g.K; k0 += 16) {
        const bool more = k0 + 16 < g.K;
        if (more) gload(k0 + 16);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[buf][2 * kk + h][32 * wr + l32],
                                                       Bs[buf][2 * kk + h][32 * wc + l32], acc,
                                                       0, 0, 0);
        if (more) sstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    float* C = g.C + b * g.sCb;
    const int n = n0 + 32 * wc + l32;
    if (n >= g.N) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int m = m0 + 32 * wr + 8 * (q >> 2) + 4 * h + (q & 3);
        if (m >= g.M) continue;
        float v = acc[q];
        if (g.epi & 8) v += C[(int64_t)m * g.sCm + n];  // accumulate onto C
        if (g.epi & 1) v += g.bias[b * g.sbias + n];
        if (g.epi & 2) v = fmaxf(v, 0.f);
        if (g.epi & 4) v = g.mask[b * g.sMb + (int64_t)m * g.sMm + n] > 0.f ? v : 0.f;
        C[(int64_t)m * g.sCm + n] = v;
    }
}

// out[b * sOb + n] = sum_m X[b][m][n]  (bias gradients): one workgroup per
// (b, 64 columns), four row groups (m = g mod 4) summed in a fixed order
__global__ __launch_bounds__(kThreads) void lenet_colsum_kernel(const float* __restrict__ X,
                                                                int M, int N,
                                                                float* __restrict__ out,
                                                                int64_t sOb) {
    __shared__ float red[4][64];
    const int b = blockIdx.x, c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int n = blockIdx.y * 64 + c;
    const float* x = X + (int64_t)b * M * N;
    float acc = 0.f;
    if (n < N) {
        // 8 rows' loads in flight, added in row order
        int m = g;
        for (; m + 28 < M; m += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = x[(int64_t)(m + 4 * u) * N + n];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
        for (; m < M; m += 4) acc += x[(int64_t)m * N + n];
    }
    red[g][c] = acc;
    __syncthreads();
    if (g == 0 && n < N) out[b * sOb + n] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

// weighted NLL of each (s, m) row and d logits in place: w_m (softmax - onehot)
// mode 0 (inner step): nll_out += sum w_m NLL, D <- w_m (softmax - onehot);
// mode 1 (outer forward): nll_rows[s][m] <- NLL, prob_rows <- softmax of the
// data rows (m >= n_pseudo), D untouched; mode 2 (outer backward): D <-
// coef_sm (softmax - onehot), coef_sm = w_m rowcoef[s][m >= n_pseudo]
struct LossOuter {
    int mode, n_pseudo;
    float* nll_rows;
    float* prob_rows;
    const float* rowcoef;
    float* prob_all;  // mode 0, nullable: softmax of every row [S][M][10] (HVP)
};

__global__ __launch_bounds__(kThreads) void lenet_loss_kernel(int rows, int M,
                                                              const int32_t* __restrict__ z,
                                                              const float* __restrict__ w,
                                                              float* __restrict__ D,
                                                              double* __restrict__ nll_out,
                                                              LossOuter o) {
    __shared__ float red[kThreads / kWave];
    const int r = blockIdx.x * kThreads + threadIdx.x;
    float contrib = 0.f;
    if (o.mode != 0) {
        if (r >= rows) return;
        const int m = r % M, s = r / M;
        float* d = D + (int64_t)r * 10;
        float l[10];
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < 10; ++c) { l[c] = d[c]; mx = fmaxf(mx, l[c]); }
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) { l[c] = expf(l[c] - mx); se += l[c]; }
        const int zc = min(max(z[m], 0), 9);
        const float inv = 1.f / se;
        if (o.mode == 1) {
            o.nll_rows[r] = mx + logf(se) - d[zc];
            if (o.prob_rows && m >= o.n_pseudo) {
                float* pr = o.prob_rows + ((int64_t)s * (M - o.n_pseudo) + (m - o.n_pseudo)) * 10;
#pragma unroll
                for (int c = 0; c < 10; ++c) pr[c] = l[c] * inv;
            }
        } else {
            const float cf = w[m] * o.rowcoef[2 * s + (m >= o.n_pseudo ? 1 : 0)];
#pragma unroll
            for (int c = 0; c < 10; ++c) d[c] = cf * (l[c] * inv - (c == zc ? 1.f : 0.f));
        }
        return;
    }
    if (r < rows) {
        const int m = r % M;
        float* d = D + (int64_t)r * 10;
        float l[10];
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < 10; ++c) { l[c] = d[c]; mx = fmaxf(mx, l[c]); }
        float se = 0.f;
#pragma unroll
        for (int c = 0; c < 10; ++c) { l[c] = expf(l[c] - mx); se += l[c]; }
        const int zc = min(max(z[m], 0), 9);  // ids are validated by the host
        const float wm = w[m];
        const float lse = mx + logf(se);
        contrib = wm * (lse - d[zc]);
        const float inv = 1.f / se;
        if (o.prob_all)
#pragma unroll
            for (int c = 0; c < 10; ++c) o.prob_all[(int64_t)r * 10 + c] = l[c] * inv;
#pragma unroll
        for (int c = 0; c < 10; ++c) d[c] = wm * (l[c] * inv - (c == zc ? 1.f : 0.f));
    }
    const float tot = block_sum(contrib, red);
    if (threadIdx.x == 0) atomicAdd(nll_out, (double)tot);
}

// ------------------------------------------------------ HVP (R-op) kernels
// psvi_hvp for LeNet: forward-over-reverse at fixed eps with the relu masks
// and pool routes of the primal pass held constant (oracle lenet_inner_hvp).

// W_dot[s][j] = v_mu + sigmoid(rho) v_rho eps_(s, j)
__global__ __launch_bounds__(kThreads) void lenet_tangent_kernel(SampleArgs a,
                                                                 const float* __restrict__ params,
                                                                 const float* __restrict__ vec,
                                                                 const float* __restrict__ eps,
                                                                 float* __restrict__ wdot) {
    const int64_t total = (int64_t)a.S_loc * a.n_tot;
    for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * kThreads) {
        const int s = (int)(i / a.n_tot), j = (int)(i - (int64_t)s * a.n_tot);
        const int l = lenet_layer(a, j);
        const int idx = j - a.woff[l];
        const int64_t pm = a.poff[l] + idx, pr = pm + a.n[l];
        wdot[i] = vec[pm] + sigmoid_f(params[pr]) * vec[pr] *
                                eps[lenet_eps_index(a, l, idx, a.s_off + s)];
    }
}

struct TanArgs {
    int M, n_tot, nchunk, chunk;
    const float* u;
    const float* wsamp;
    const float* wdot;
    const float* p1;
    const int8_t* r1;
    const int8_t* r2;
    const float* dx2;    // primal d X2
    const float* dx2d;   // tangent d X2
    float* p1d;          // fwd out: tangent pooled conv1 [S][M][1176]
    float* x2d;          // fwd out: tangent X2 [S][M][400]
    float* part;         // bwd out: tangent conv weight gradients [S][nchunk][2572]
    float* du;           // bwd out, nullable: [S][M][784] tangent of d u
    float* g1g;          // MFMA bwd out: [S][M][1176] routed d P1_dot
};

// tangent of d logits and of each row's NLL:
//   dd = w (P . l_dot - P (P . l_dot)),  nll_dot = (P - onehot) . l_dot
__global__ __launch_bounds__(kThreads) void lenet_loss_tan_kernel(int rows, int M,
                                                                  const int32_t* __restrict__ z,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ P,
                                                                  float* __restrict__ LD,
                                                                  float* __restrict__ nlld) {
    const int r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= rows) return;
    const int m = r % M;
    const int zc = min(max(z[m], 0), 9);
    const float* p = P + (int64_t)r * 10;
    float* ld = LD + (int64_t)r * 10;
    float pl = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) pl += p[c] * ld[c];
    nlld[r] = pl - ld[zc];
    const float wm = w[m];
    float out[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) out[c] = wm * p[c] * (ld[c] - pl);
#pragma unroll
    for (int c = 0; c < 10; ++c) ld[c] = out[c];
}

// The tangent backward on the matrix cores (d/du, when asked for, by
// lenet_du_tan_kernel afterwards).  Per image, as lenet_conv_bwd_mfma_kernel:
//   d P1_dot patches  U_dot = [A_dot | A] [B(W2) ; B(W2_dot)]   (K = 2 x 64),
//     A / A_dot: the routed primal / tangent conv2 gradients expanded by window
//     offset (ga / gad), B(.): the filters shifted by offset, as there;
//   G_dot conv2 = sum_(w, q) A_dot P1 + A P1_dot   (K = 2 x 100),
//   d P1_dot = the covering U_dot patches in window order, routed through pool1
//     / relu, written to HBM for lenet_conv1_wgrad_mfma_kernel (conv1's G_dot).
// Eight waves: waves 0..5 own d P1 column tiles wv, wv + 8 and conv2 weight
// tile wv; waves 6, 7 own d P1 tile wv and conv2 weight tiles 6 + 2 (wv - 6)
// + {0, 1} (178 / 164 MFMAs per image).  LDS: P1 | P1_dot, then U_dot (the
// weight-gradient GEMM is done before the patches are written); W2's and
// W2_dot's B fragments in registers (122 VGPRs: four waves per SIMD, two
// workgroups per CU; W2_dot's read from LDS per k-step took 2 % longer).
constexpr int kTW = 8, kTThreads = 64 * kTW;
constexpr int kTPP = 2 * 6 * kP1C;
static_assert(kTPP >= 25 * kUS + 1, "P1 | P1_dot region holds U_dot");
__global__ __launch_bounds__(kTThreads, 4) void lenet_conv_bwd_tan_mfma_kernel(TanArgs a) {
    __shared__ float pp[kTPP];
    __shared__ float ga[4 * kGQ], gad[4 * kGQ];
    __shared__ float g2d[kX2];
    __shared__ int8_t r1s[kP1];
    __shared__ float wd2[2400];  // W2_dot: its B fragments are read per k-step
    float* const p1 = pp;
    float* const p1d = pp + 6 * kP1C;
    float* const U = pp;
    const int tid = threadIdx.x, s = blockIdx.y;
    const int lane = tid & 63, wv = wave_id(), r16 = lane & 15, kq = lane >> 4;
    const float* ws = a.wsamp + (int64_t)s * a.n_tot;
    const float* wds = a.wdot + (int64_t)s * a.n_tot;
    for (int i = tid; i < 2400; i += kTThreads) {
        pp[i] = ws[156 + i];
        wd2[i] = wds[156 + i];
    }
    for (int i = tid; i < 4 * kGQ; i += kTThreads) ga[i] = gad[i] = 0.f;
    __syncthreads();
    // B fragments of the d P1 column tiles wv + 8 j: k-steps 0..15 W2,
    // 16..31 W2_dot (both in registers, 0 off the tile)
    float bf[2][16], bfd[2][16];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int tile = wv + 8 * j, n = 16 * tile + r16;
        const int c = n / 36, ay = (n % 36) / 6 - (kq >> 1), ax = n % 6 - (kq & 1);
        const bool ok = tile < 14 && n < 216 && ay >= 0 && ay < 5 && ax >= 0 && ax < 5;
        const int wo = ok ? c * 25 + ay * 5 + ax : 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            bf[j][t] = ok ? pp[t * 150 + wo] : 0.f;
            bfd[j][t] = ok ? wd2[t * 150 + wo] : 0.f;
        }
    }
    const bool hi = wv >= 6;  // wave-uniform
    int nb2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int tile = hi ? 6 + 2 * (wv - 6) + h : wv;
        const int n = min(16 * tile + r16, 149);
        nb2[h] = (n / 25) * kP1C + ((n % 25) / 5) * kP1S + n % 5;
    }
    const int kqoff = (kq >> 1) * kP1S + (kq & 1);
    f32x4 accw2[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    float accb2 = 0.f;
    constexpr int kLP = (kP1 + kTThreads - 1) / kTThreads;  // 3
    const int m0 = blockIdx.x * a.chunk, m1 = min(a.M, m0 + a.chunk);
    // conv2 weight tangent for NW column tiles (k-steps: 25 windows x A_dot P1,
    // then 25 x A P1_dot)
    auto wgrad2 = [&](auto nw_c) __attribute__((always_inline)) {
        constexpr int NW = decltype(nw_c)::value;
        const float* ad = gad + kq * kGQ + r16 * kGK;
        const float* ap = ga + kq * kGQ + r16 * kGK;
#pragma unroll 5
        for (int t = 0; t < 25; ++t) {
            const float av = ad[t];
            const int po = kqoff + 2 * (t / 5) * kP1S + 2 * (t % 5);
#pragma unroll
            for (int h = 0; h < NW; ++h)
                accw2[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, p1[nb2[h] + po], accw2[h], 0, 0, 0);
        }
#pragma unroll 5
        for (int t = 0; t < 25; ++t) {
            const float av = ap[t];
            const int po = kqoff + 2 * (t / 5) * kP1S + 2 * (t % 5);
#pragma unroll
            for (int h = 0; h < NW; ++h)
                accw2[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, p1d[nb2[h] + po], accw2[h], 0, 0, 0);
        }
    };
    // U_dot for NT column tiles, two row tiles of windows
    auto dp1 = [&](auto nt_c) __attribute__((always_inline)) {
        constexpr int NT = decltype(nt_c)::value;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const float* ad = gad + kq * kGQ + 16 * mt + r16;
            const float* ap = ga + kq * kGQ + 16 * mt + r16;
            f32x4 acc[NT];
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const float av = ad[t * kGK];
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bf[j][t], acc[j], 0, 0, 0);
            }
#pragma unroll 4
            for (int t = 0; t < 16; ++t) {
                const float av = ap[t * kGK];
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bfd[j][t], acc[j], 0, 0, 0);
            }
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n = 16 * (wv + 8 * j) + r16;
                if (n >= 216) continue;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int wr = 16 * mt + 4 * kq + i;
                    if (wr < 25) U[wr * kUS + n] = acc[j][i];
                }
            }
        }
    };
    for (int m = m0; m < m1; ++m) {
        // this image's inputs (no register prefetch: 128 VGPRs hold 4 waves per
        // SIMD, two workgroups per CU, one staging while the other multiplies)
        const int64_t row = (int64_t)s * a.M + m;
        float pv[kLP], pvd[kLP];
        int8_t pr1[kLP];
#pragma unroll
        for (int k = 0; k < kLP; ++k) {
            const int i = min(tid + k * kTThreads, kP1 - 1);
            pv[k] = a.p1[row * kP1 + i];
            pvd[k] = a.p1d[row * kP1 + i];
            pr1[k] = a.r1[row * kP1 + i];
        }
        const int o2 = min(tid, kX2 - 1);
        const float pg = a.dx2[row * kX2 + o2], pgd = a.dx2d[row * kX2 + o2];
        const int pr2 = a.r2[row * kX2 + o2];
        __syncthreads();  // the previous image's patch reads are done
#pragma unroll
        for (int k = 0; k < kLP; ++k) {
            const int i = tid + k * kTThreads;
            if (i < kP1) {
                const int q = (i / 196) * kP1C + ((i % 196) / 14) * kP1S + i % 14;
                p1[q] = pv[k];
                p1d[q] = pvd[k];
                r1s[i] = pr1[k];
            }
        }
        if (tid < kX2) {
            const int r = pr2, kk = tid / 25, w = tid % 25;
            const float g = r >= 0 ? pg : 0.f, gd = r >= 0 ? pgd : 0.f;
            g2d[tid] = gd;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                ga[q * kGQ + kk * kGK + w] = r == q ? g : 0.f;
                gad[q * kGQ + kk * kGK + w] = r == q ? gd : 0.f;
            }
        }
        __syncthreads();
        if (hi)
            wgrad2(std::integral_constant<int, 2>{});
        else
            wgrad2(std::integral_constant<int, 1>{});
        if (tid < 16) {
            float acc = 0.f;
            for (int p = 0; p < 25; ++p) acc += g2d[tid * 25 + p];
            accb2 += acc;
        }
        __syncthreads();  // P1 | P1_dot reads are done: U_dot overwrites them
        if (tid == 0) U[25 * kUS] = 0.f;
        if (hi)
            dp1(std::integral_constant<int, 1>{});
        else
            dp1(std::integral_constant<int, 2>{});
        __syncthreads();
        // d P1_dot = the covering patches in window order, routed
#pragma unroll 1
        for (int k = 0; k < kLP; ++k) {
            const int o = tid + k * kTThreads;
            if (o >= kP1) break;
            const int c = o / 196, y = (o % 196) / 14, x = o % 14;
            const int by = (y >> 1) - 2, bx = (x >> 1) - 2;
            int uo[9];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int wy = by + dy, wx = bx + dx;
                    const bool in_map = wy >= 0 && wy < 5 && wx >= 0 && wx < 5;
                    uo[dy * 3 + dx] = in_map ? (wy * 5 + wx) * kUS + c * 36 +
                                                   ((y & 1) + 4 - 2 * dy) * 6 + (x & 1) + 4 - 2 * dx
                                             : 25 * kUS;
                }
            float uv[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) uv[q] = U[uo[q]];
            float v = 0.f;
#pragma unroll
            for (int q = 0; q < 9; ++q) v += uv[q];
            a.g1g[((int64_t)s * a.M + m) * kP1 + o] = r1s[o] >= 0 ? v : 0.f;
        }
    }
    float* out = a.part + ((int64_t)s * a.nchunk + blockIdx.x) * kNConv;
    if (tid < 16) out[2556 + tid] = accb2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h == 1 && !hi) break;
        const int tile = hi ? 6 + 2 * (wv - 6) + h : wv;
        const int n = 16 * tile + r16;
        if (n < 150) {
#pragma unroll
            for (int i = 0; i < 4; ++i) out[156 + (4 * kq + i) * 150 + n] = accw2[h][i];
        }
    }
}

// The tangent of d u (the mixed product d/du) for every row, from the routed
// primal and tangent d P1 the backward kernels left in HBM:
//   du_dot = convT(routed d P1_dot, W1) + convT(routed d P1, W1_dot)
// (each routed value placed at its conv1 position of a zero-bordered 32 x 32
// plane per channel, 2x2 output blocks per thread).  Each pooled value
// writes its whole 2x2 conv1 block (the routed position, zeros elsewhere),
// so the planes need no clearing between images, and the next image's
// routes and values are loaded into registers behind this image's
// convolution.  Planes with 46-float rows, read as float2: a wave's 16-lane
// groups (2x2 blocks of rows yy = 0, 2, 4, ... at even columns) then cover
// distinct banks (2 x 46 = 28 mod 32) -- the 32-float rows put every block
// row on the same banks (3-way conflicts at ds_read_b32).  C5 (rocprof,
// tools/gpu_g32.sh): 3.39 ms -> 3.08 (prefetch, no clearing) -> 2.41 (the
// planes) -> 1.77 (packed fma); a second pair of accumulators: no change.
constexpr int kDuLd = 46, kDuPlane = 32 * kDuLd;
// 2x2 block of a transposed 5x5 conv: acc[q] += sum_ij w[i][j] Q[4 - i + dy][4 - j + dx]
// over a 6x6 patch at q (row stride kDuLd, q 8-byte aligned) of a zero-bordered plane
// (acc as two column pairs: each update one packed fma, v_pk_fma_f32 -- the
// same per-element fma as the scalar form)
typedef float duf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void convT_block2(const float* q, const float* wk, duf2 (&acc)[2]) {
    float Q[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 6; j += 2) {
            const float2 v = *reinterpret_cast<const float2*>(q + i * kDuLd + j);
            Q[i][j] = v.x;
            Q[i][j + 1] = v.y;
        }
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const float wv = wk[i * 5 + j];
            acc[0] = __builtin_elementwise_fma(duf2{wv, wv}, duf2{Q[4 - i][4 - j], Q[4 - i][5 - j]}, acc[0]);
            acc[1] = __builtin_elementwise_fma(duf2{wv, wv}, duf2{Q[5 - i][4 - j], Q[5 - i][5 - j]}, acc[1]);
        }
}
__global__ __launch_bounds__(kThreads) void lenet_du_tan_kernel(TanArgs a, const float* __restrict__ g1p,
                                                               const float* __restrict__ g1t) {
    __shared__ float w1[150], wd1[150];
    __shared__ __attribute__((aligned(16))) float da1[6 * kDuPlane], da1d[6 * kDuPlane];
    const int tid = threadIdx.x, s = blockIdx.y;
    const float* ws = a.wsamp + (int64_t)s * a.n_tot;
    const float* wds = a.wdot + (int64_t)s * a.n_tot;
    for (int i = tid; i < 150; i += kThreads) {
        w1[i] = ws[i];
        wd1[i] = wds[i];
    }
    for (int i = tid; i < 6 * kDuPlane; i += kThreads) da1[i] = da1d[i] = 0.f;  // the borders stay 0
    const int m0 = blockIdx.x * a.chunk, m1 = min(a.M, m0 + a.chunk);
    constexpr int kLP = (kP1 + kThreads - 1) / kThreads;
    int pr[kLP];
    float pg[kLP], pt[kLP];
    auto fetch = [&](int m) __attribute__((always_inline)) {
        const int64_t row = (int64_t)s * a.M + m;
#pragma unroll
        for (int k = 0; k < kLP; ++k) {
            const int o = min(tid + k * kThreads, kP1 - 1);
            pr[k] = a.r1[row * kP1 + o];
            pg[k] = g1p[row * kP1 + o];
            pt[k] = g1t[row * kP1 + o];
        }
    };
    if (m0 < m1) fetch(m0);
    for (int m = m0; m < m1; ++m) {
        const int64_t row = (int64_t)s * a.M + m;
        __syncthreads();  // the previous image's convolution is done with the planes
#pragma unroll
        for (int k = 0; k < kLP; ++k) {
            const int o = tid + k * kThreads;
            if (o < kP1) {
                const int rr = pr[k] >= 0 ? pr[k] : 0;  // a dropped value (0) at offset 0
                const int c = o / 196, py = (o % 196) / 14, px = o % 14;
                const int q = c * kDuPlane + (2 * py + 2) * kDuLd + 2 * px + 2;
                const float g = pg[k], t = pt[k];
                *reinterpret_cast<float2*>(da1 + q) = make_float2(rr == 0 ? g : 0.f, rr == 1 ? g : 0.f);
                *reinterpret_cast<float2*>(da1 + q + kDuLd) = make_float2(rr == 2 ? g : 0.f, rr == 3 ? g : 0.f);
                *reinterpret_cast<float2*>(da1d + q) = make_float2(rr == 0 ? t : 0.f, rr == 1 ? t : 0.f);
                *reinterpret_cast<float2*>(da1d + q + kDuLd) = make_float2(rr == 2 ? t : 0.f, rr == 3 ? t : 0.f);
            }
        }
        if (m + 1 < m1) fetch(m + 1);
        __syncthreads();
        if (tid < 196) {
            const int yy = 2 * (tid / 14), xx = 2 * (tid % 14);
            duf2 acc[2] = {duf2{0.f, 0.f}, duf2{0.f, 0.f}};
#pragma unroll 1
            for (int c = 0; c < 6; ++c) {
                convT_block2(da1d + c * kDuPlane + yy * kDuLd + xx, w1 + c * 25, acc);
                convT_block2(da1 + c * kDuPlane + yy * kDuLd + xx, wd1 + c * 25, acc);
            }
            float* out = a.du + row * 784 + yy * 28 + xx;
            *reinterpret_cast<float2*>(out) = make_float2(acc[0].x, acc[0].y);
            *reinterpret_cast<float2*>(out + 28) = make_float2(acc[1].x, acc[1].y);
        }
    }
}

// H vec: sum_s G_dot (+ eps) through the reparameterisation, the softplus
// curvature sum_s (G_s eps_s) sigmoid'(rho) v_rho, the KL Hessian on the
// VILinear layers; then d_u = sum_s du_dot, d_w = sum_s nll_dot.
__global__ __launch_bounds__(kThreads) void lenet_hvp_assemble_kernel(
    SampleArgs a, const float* __restrict__ params, const float* __restrict__ vec,
    const float* __restrict__ eps, const float* __restrict__ G, const float* __restrict__ Gd,
    const float* __restrict__ dud, const float* __restrict__ nlld, float* __restrict__ hv,
    float* __restrict__ d_u, float* __restrict__ d_w, int M, float inv_s0sq, int include_kl) {
    const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
    if (i < a.n_tot) {
        const int j = (int)i;
        const int l = lenet_layer(a, j);
        const int idx = j - a.woff[l];
        float gd = 0.f, gde = 0.f, ge = 0.f;
        for (int s = 0; s < a.S_loc; ++s) {
            const float e = eps[lenet_eps_index(a, l, idx, a.s_off + s)];
            const float g = G[(int64_t)s * a.n_tot + j], gdv = Gd[(int64_t)s * a.n_tot + j];
            ge = fmaf(g, e, ge);
            gd += gdv;
            gde = fmaf(gdv, e, gde);
        }
        const int64_t pm = a.poff[l] + idx, pr = pm + a.n[l];
        const float r = params[pr], sp = softplus_f(r), sg = sigmoid_f(r);
        const float vr = vec[pr];
        float hm = gd, hr = gde * sg + ge * sg * (1.f - sg) * vr;
        if (l >= 2 && include_kl) {  // KL on the VILinear layers (not in a shard's partial)
            hm += vec[pm] * inv_s0sq;
            hr += ((1.f / (sp * sp) + inv_s0sq) * sg * sg + (sp * inv_s0sq - 1.f / sp) * sg * (1.f - sg)) * vr;
        }
        hv[pm] = hm;
        hv[pr] = hr;
        return;
    }
    const int64_t j = i - a.n_tot;
    if (d_u && j < (int64_t)M * 784) {
        float g = 0.f;
        for (int s = 0; s < a.S_loc; ++s) g += dud[(int64_t)s * M * 784 + j];
        d_u[j] = g;
        return;
    }
    const int64_t k = j - (d_u ? (int64_t)M * 784 : 0);
    if (d_w && k >= 0 && k < M) {
        float g = 0.f;
        for (int s = 0; s < a.S_loc; ++s) g += nlld[(int64_t)s * M + k];
        d_w[k] = g;
    }
}

hipError_t gemm(const GemmArgs& g, int batch, hipStream_t st) {
    dim3 grid((g.N + 63) / 64, (g.M + 63) / 64, batch);
    hipLaunchKernelGGL(lenet_gemm_mfma_kernel, grid, dim3(kThreads), 0, st, g);
    return hipGetLastError();
}

GemmArgs gemm_args(int M, int N, int K, const float* A, int64_t sAb, int sAm, int sAk,
                   const float* B, int64_t sBb, int sBk, int sBn, float* C, int64_t sCb,
                   int sCm) {
    GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.sAb = sAb; g.sAm = sAm; g.sAk = sAk;
    g.B = B; g.sBb = sBb; g.sBk = sBk; g.sBn = sBn;
    g.C = C; g.sCb = sCb; g.sCm = sCm;
    return g;
}

}  // namespace

LenetWs lenet_ws(const psvi_plan& p, void* base) {
    const int64_t S = p.s_cnt[p.rank], M = p.d.M;
    LenetWs w{};
    w.nchunk = lenet_nchunk(p);
    size_t off = 0;
    char* b = (char*)base;
    auto take = [&](size_t bytes) -> void* {
        void* r = b ? (void*)(b + off) : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return r;
    };
    w.wsamp = (float*)take(sizeof(float) * S * p.n_tot);
    w.dws = (float*)take(sizeof(float) * S * p.n_tot);
    w.p1 = (float*)take(sizeof(float) * S * M * kP1);
    w.r1 = (int8_t*)take(S * M * kP1);
    w.x2 = (float*)take(sizeof(float) * S * M * kX2);
    w.r2 = (int8_t*)take(S * M * kX2);
    w.h1 = (float*)take(sizeof(float) * S * M * 120);
    w.h2 = (float*)take(sizeof(float) * S * M * 84);
    w.d = (float*)take(sizeof(float) * S * M * 10);
    w.dh2 = (float*)take(sizeof(float) * S * M * 84);
    w.dh1 = (float*)take(sizeof(float) * S * M * 120);
    w.dx2 = (float*)take(sizeof(float) * S * M * kX2);
    w.part = (float*)take(sizeof(float) * S * w.nchunk * kNConv);
    // MFMA backward: the routed d P1 and conv1's weight-gradient partials
    // (8 samples per workgroup, >= ~1024 workgroups)
    w.g1 = (float*)take(sizeof(float) * S * M * kP1);
    w.nch1 = (int)std::max<int64_t>(1, std::min<int64_t>(M, 1024 / ((S + kW1S - 1) / kW1S)));
    w.part1 = (float*)take(sizeof(float) * S * w.nch1 * 156);
    w.bytes = off;
    return w;
}

int lenet_nchunk(const psvi_plan& p) {
    // >= ~2048 workgroups over the chip (256 CUs), at most one image per chunk
    const int S = p.s_cnt[p.rank], M = p.d.M;
    const int want = (2048 + S - 1) / S;
    return std::max(1, std::min(M, want));
}

static SampleArgs sample_args(const psvi_plan& p) {
    SampleArgs a{};
    a.L = p.L;
    a.n_tot = p.n_tot;
    a.S_loc = p.s_cnt[p.rank];
    a.s_off = p.s_off[p.rank];
    a.S_tot = p.d.S;
    for (int l = 0; l < p.L; ++l) {
        a.woff[l] = p.lay[l].woff;
        a.n[l] = p.lay[l].n;
        a.nw[l] = p.lay[l].din * p.lay[l].dout;
        a.batched[l] = l < p.L - 1;
        a.poff[l] = p.lay[l].poff;
        a.eoff[l] = p.lay[l].eoff;
    }
    a.woff[p.L] = p.n_tot;
    return a;
}

// conv1 on the matrix cores, 8 samples per workgroup; then conv2, one wave per
// workgroup over a chunk of image pairs (>= ~2048 workgroups / ~8192 waves)
template <bool TAN>
static void conv_fwd_mfma(const ConvArgs& ca, int S, int M, hipStream_t st) {
    ConvArgs c1 = ca;
    const int sg = (S + kC1S - 1) / kC1S;
    const int n1 = std::max(1, std::min(M, 2048 / sg));
    c1.chunk = (M + n1 - 1) / n1;
    hipLaunchKernelGGL(lenet_conv1_mfma_kernel<TAN>, dim3((M + c1.chunk - 1) / c1.chunk, sg),
                       dim3(256), 0, st, c1, S);
    ConvArgs c2 = ca;
    const int np = (M + 1) / 2;
    const int n2 = std::max(1, std::min(np, 8192 / S));
    c2.chunk = (np + n2 - 1) / n2;
    hipLaunchKernelGGL(lenet_conv2_mfma_kernel<TAN>, dim3((np + c2.chunk - 1) / c2.chunk, S),
                       dim3(64), 0, st, c2);
}

hipError_t launch_lenet(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                        const float* params, const float* eps, float* acc, double* nll_out,
                        void* ws, hipStream_t st, const NetOuter* outer) {
    const LenetWs W = lenet_ws(p, ws);
    LossOuter lo{};
    if (outer) {
        lo.mode = outer->mode;
        lo.n_pseudo = outer->n_pseudo;
        lo.nll_rows = outer->nll_rows;
        lo.prob_rows = outer->mode == 0 ? nullptr : outer->prob_rows;
        lo.rowcoef = outer->rowcoef;
        lo.prob_all = outer->mode == 0 ? outer->prob_rows : nullptr;
    }
    const SampleArgs sa = sample_args(p);
    const int S = sa.S_loc, M = p.d.M, nt = p.n_tot;
    if (S == 0) return hipMemsetAsync(acc, 0, sizeof(float) * 2 * nt, st);
    const int64_t rows = (int64_t)S * M;
    {
        const dim3 grid((unsigned)((nt + kThreads - 1) / kThreads),
                        (unsigned)((S + kSampleRun - 1) / kSampleRun));
        hipLaunchKernelGGL(lenet_sample_kernel, grid, dim3(kThreads), 0, st, sa, params, eps,
                           W.wsamp);
    }
    ConvArgs ca{};
    ca.M = M;
    ca.n_tot = nt;
    ca.nchunk = W.nchunk;
    ca.chunk = (M + W.nchunk - 1) / W.nchunk;
    ca.u = u;
    ca.wsamp = W.wsamp;
    ca.p1 = W.p1;
    ca.r1 = W.r1;
    ca.x2 = W.x2;
    ca.r2 = W.r2;
    ca.dx2 = W.dx2;
    ca.part = W.part;
    ca.abl = g_lenet_abl;
    conv_fwd_mfma<false>(ca, S, M, st);
    const int w3 = p.lay[2].woff, w4 = p.lay[3].woff, w5 = p.lay[4].woff;
    const float* Ws = W.wsamp;
    // head forward: H1 = relu(X2 W1^T + b1), H2 = relu(H1 W2^T + b2), D = H2 W3^T + b3
    GemmArgs g = gemm_args(M, 120, 400, W.x2, (int64_t)M * 400, 400, 1, Ws + w3, nt, 1, 400,
                           W.h1, (int64_t)M * 120, 120);
    g.epi = 3; g.bias = Ws + w3 + 48000; g.sbias = nt;
    if (hipError_t e = gemm(g, S, st)) return e;
    g = gemm_args(M, 84, 120, W.h1, (int64_t)M * 120, 120, 1, Ws + w4, nt, 1, 120, W.h2,
                  (int64_t)M * 84, 84);
    g.epi = 3; g.bias = Ws + w4 + 10080; g.sbias = nt;
    if (hipError_t e = gemm(g, S, st)) return e;
    g = gemm_args(M, 10, 84, W.h2, (int64_t)M * 84, 84, 1, Ws + w5, nt, 1, 84, W.d,
                  (int64_t)M * 10, 10);
    g.epi = 1; g.bias = Ws + w5 + 840; g.sbias = nt;
    if (hipError_t e = gemm(g, S, st)) return e;
    hipLaunchKernelGGL(lenet_loss_kernel, dim3((unsigned)((rows + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, (int)rows, M, z, w, W.d, nll_out, lo);
    if (lo.mode == 1) return hipGetLastError();
    // head backward
    float* dW = W.dws;
    g = gemm_args(10, 84, M, W.d, (int64_t)M * 10, 1, 10, W.h2, (int64_t)M * 84, 84, 1,
                  dW + w5, nt, 84);
    if (hipError_t e = gemm(g, S, st)) return e;
    hipLaunchKernelGGL(lenet_colsum_kernel, dim3(S, (10 + 63) / 64), dim3(kThreads), 0, st, W.d, M, 10,
                       dW + w5 + 840, (int64_t)nt);
    g = gemm_args(M, 84, 10, W.d, (int64_t)M * 10, 10, 1, Ws + w5, nt, 84, 1, W.dh2,
                  (int64_t)M * 84, 84);
    g.epi = 4; g.mask = W.h2; g.sMb = (int64_t)M * 84; g.sMm = 84;
    if (hipError_t e = gemm(g, S, st)) return e;
    g = gemm_args(84, 120, M, W.dh2, (int64_t)M * 84, 1, 84, W.h1, (int64_t)M * 120, 120, 1,
                  dW + w4, nt, 120);
    if (hipError_t e = gemm(g, S, st)) return e;
    hipLaunchKernelGGL(lenet_colsum_kernel, dim3(S, (84 + 63) / 64), dim3(kThreads), 0, st, W.dh2, M, 84,
                       dW + w4 + 10080, (int64_t)nt);
    g = gemm_args(M, 120, 84, W.dh2, (int64_t)M * 84, 84, 1, Ws + w4, nt, 120, 1, W.dh1,
                  (int64_t)M * 120, 120);
    g.epi = 4; g.mask = W.h1; g.sMb = (int64_t)M * 120; g.sMm = 120;
    if (hipError_t e = gemm(g, S, st)) return e;
    g = gemm_args(120, 400, M, W.dh1, (int64_t)M * 120, 1, 120, W.x2, (int64_t)M * 400, 400, 1,
                  dW + w3, nt, 400);
    if (hipError_t e = gemm(g, S, st)) return e;
    hipLaunchKernelGGL(lenet_colsum_kernel, dim3(S, (120 + 63) / 64), dim3(kThreads), 0, st, W.dh1, M, 120,
                       dW + w3 + 48000, (int64_t)nt);
    g = gemm_args(M, 400, 120, W.dh1, (int64_t)M * 120, 120, 1, Ws + w3, nt, 400, 1, W.dx2,
                  (int64_t)M * 400, 400);
    if (hipError_t e = gemm(g, S, st)) return e;
    // conv towers backward, then the per-sample sums with eps
    const bool du = outer && outer->du_part;
    if (du) {
        ca.du = outer->du_part;
        ca.n_pseudo = outer->n_pseudo;
    }
    const dim3 bgrid(W.nchunk, S), bblk(kConvThreads);
    const float* part1 = nullptr;
    {
        ca.g1g = W.g1;
        if (du) hipLaunchKernelGGL(lenet_conv_bwd_mfma_kernel<true>, bgrid, bblk, 0, st, ca);
        else hipLaunchKernelGGL(lenet_conv_bwd_mfma_kernel<false>, bgrid, bblk, 0, st, ca);
        // conv1's weight gradient from the routed d P1: 8 samples per workgroup
        ConvArgs c1 = ca;
        c1.part1 = W.part1;
        c1.nch1 = W.nch1;
        c1.chunk = (M + W.nch1 - 1) / W.nch1;
        hipLaunchKernelGGL(lenet_conv1_wgrad_mfma_kernel, dim3(W.nch1, (S + kW1S - 1) / kW1S),
                           dim3(256), 0, st, c1, S);
        part1 = W.part1;
    }
    hipLaunchKernelGGL(lenet_conv_reduce_kernel,
                       dim3((unsigned)(((int64_t)S * kNConv + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, S, W.nchunk, nt, W.part, dW, part1, W.nch1);
    hipLaunchKernelGGL(lenet_acc_kernel, dim3((nt + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       st, sa, eps, dW, acc, outer ? outer->ck : nullptr, W.wsamp,
                       1.f / (p.d.prior_sd * p.d.prior_sd));
    return hipGetLastError();
}

LenetTanWs lenet_tan_ws(const psvi_plan& p, void* base) {
    const int64_t S = p.s_cnt[p.rank], M = p.d.M;
    LenetTanWs w{};
    size_t off = 0;
    char* b = (char*)base;
    auto take = [&](size_t bytes) -> void* {
        void* r = b ? (void*)(b + off) : nullptr;
        off += (bytes + 255) & ~size_t(255);
        return r;
    };
    w.nll = (double*)take(sizeof(double));
    w.acc = (float*)take(sizeof(float) * 2 * p.n_tot);
    w.wdot = (float*)take(sizeof(float) * S * p.n_tot);
    w.gd = (float*)take(sizeof(float) * S * p.n_tot);
    w.p1d = (float*)take(sizeof(float) * S * M * kP1);
    w.x2d = (float*)take(sizeof(float) * S * M * kX2);
    w.h1d = (float*)take(sizeof(float) * S * M * 120);
    w.h2d = (float*)take(sizeof(float) * S * M * 84);
    w.ld = (float*)take(sizeof(float) * S * M * 10);
    w.prob = (float*)take(sizeof(float) * S * M * 10);
    w.dh2d = (float*)take(sizeof(float) * S * M * 84);
    w.dh1d = (float*)take(sizeof(float) * S * M * 120);
    w.dx2d = (float*)take(sizeof(float) * S * M * kX2);
    w.part = (float*)take(sizeof(float) * S * lenet_nchunk(p) * kNConv);
    w.du = (float*)take(sizeof(float) * S * M * 784);
    w.nlld = (float*)take(sizeof(float) * S * M);
    w.bytes = off;
    return w;
}

hipError_t launch_lenet_hvp(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                            const float* eps, const float* params, const float* vec, float* hv,
                            float* d_u, float* d_w, void* tws, hipStream_t st, bool include_kl) {
    const LenetWs W = lenet_ws(p, p.d_lenet_ws);
    const LenetTanWs T = lenet_tan_ws(p, tws);
    const SampleArgs sa = sample_args(p);
    const int S = sa.S_loc, M = p.d.M, nt = p.n_tot;
    const int64_t rows = (int64_t)S * M;
    // primal pass: activations, routes, per-sample G, row probabilities
    if (hipError_t e = hipMemsetAsync(T.nll, 0, sizeof(double), st)) return e;
    NetOuter keep{0, 0, nullptr, nullptr, nullptr, nullptr, T.prob};
    if (hipError_t e = launch_lenet(p, u, z, w, params, eps, T.acc, T.nll, p.d_lenet_ws, st, &keep))
        return e;
    {
        const int64_t nb = std::min<int64_t>(((int64_t)S * nt + kThreads - 1) / kThreads, 8192);
        hipLaunchKernelGGL(lenet_tangent_kernel, dim3((unsigned)nb), dim3(kThreads), 0, st, sa,
                           params, vec, eps, T.wdot);
    }
    TanArgs ta{};
    ta.M = M;
    ta.n_tot = nt;
    ta.nchunk = W.nchunk;
    ta.chunk = (M + W.nchunk - 1) / W.nchunk;
    ta.u = u;
    ta.wsamp = W.wsamp;
    ta.wdot = T.wdot;
    ta.p1 = W.p1;
    ta.r1 = W.r1;
    ta.r2 = W.r2;
    ta.dx2 = W.dx2;
    ta.dx2d = T.dx2d;
    ta.p1d = T.p1d;
    ta.x2d = T.x2d;
    ta.part = T.part;
    ta.du = d_u ? T.du : nullptr;
    {
        // the forward's kernels in tangent mode: P1_dot from W_dot at conv1's
        // routed offsets, then X2_dot from [P1_dot | P1] x [W2; W2_dot]
        ConvArgs ct{};
        ct.M = M;
        ct.n_tot = nt;
        ct.u = u;
        ct.wsamp = W.wsamp;
        ct.wdot = T.wdot;
        ct.p1 = W.p1;
        ct.p1dot = T.p1d;
        ct.r1 = W.r1;
        ct.r2 = W.r2;
        ct.x2 = T.x2d;
        conv_fwd_mfma<true>(ct, S, M, st);
    }
    const int w3 = p.lay[2].woff, w4 = p.lay[3].woff, w5 = p.lay[4].woff;
    const float* Ws = W.wsamp;
    const float* Wd = T.wdot;
    // head tangent forward: h1_dot = 1[h1>0] (x2_dot W1^T + x2 W1_dot^T + b1_dot), ...
    auto fwd2 = [&](int K, int N, const float* Ad, const float* A, int lw, int lb, float* C,
                    const float* mask) -> hipError_t {
        GemmArgs g = gemm_args(M, N, K, Ad, (int64_t)M * K, K, 1, Ws + lw, nt, 1, K, C,
                               (int64_t)M * N, N);
        if (hipError_t e = gemm(g, S, st)) return e;
        g = gemm_args(M, N, K, A, (int64_t)M * K, K, 1, Wd + lw, nt, 1, K, C, (int64_t)M * N, N);
        g.epi = 8 | 1 | (mask ? 4 : 0);
        g.bias = Wd + lb;
        g.sbias = nt;
        g.mask = mask;
        g.sMb = (int64_t)M * N;
        g.sMm = N;
        return gemm(g, S, st);
    };
    if (hipError_t e = fwd2(400, 120, T.x2d, W.x2, w3, w3 + 48000, T.h1d, W.h1)) return e;
    if (hipError_t e = fwd2(120, 84, T.h1d, W.h1, w4, w4 + 10080, T.h2d, W.h2)) return e;
    if (hipError_t e = fwd2(84, 10, T.h2d, W.h2, w5, w5 + 840, T.ld, nullptr)) return e;
    hipLaunchKernelGGL(lenet_loss_tan_kernel, dim3((unsigned)((rows + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, (int)rows, M, z, w, T.prob, T.ld, T.nlld);
    // head tangent backward (T.ld now holds d logits_dot)
    auto dW2 = [&](int O, int I, const float* Dd, const float* Hp, const float* Dp,
                   const float* Hd, int lw) -> hipError_t {
        GemmArgs g = gemm_args(O, I, M, Dd, (int64_t)M * O, 1, O, Hp, (int64_t)M * I, I, 1,
                               T.gd + lw, nt, I);
        if (hipError_t e = gemm(g, S, st)) return e;
        g = gemm_args(O, I, M, Dp, (int64_t)M * O, 1, O, Hd, (int64_t)M * I, I, 1, T.gd + lw, nt,
                      I);
        g.epi = 8;
        if (hipError_t e = gemm(g, S, st)) return e;
        hipLaunchKernelGGL(lenet_colsum_kernel, dim3(S, (O + 63) / 64), dim3(kThreads), 0, st, Dd, M, O,
                           T.gd + lw + O * I, (int64_t)nt);
        return hipGetLastError();
    };
    auto dX2 = [&](int O, int I, const float* Dd, const float* Dp, int lw, float* C,
                   const float* mask) -> hipError_t {
        GemmArgs g = gemm_args(M, I, O, Dd, (int64_t)M * O, O, 1, Ws + lw, nt, I, 1, C,
                               (int64_t)M * I, I);
        if (hipError_t e = gemm(g, S, st)) return e;
        g = gemm_args(M, I, O, Dp, (int64_t)M * O, O, 1, Wd + lw, nt, I, 1, C, (int64_t)M * I, I);
        g.epi = 8 | (mask ? 4 : 0);
        g.mask = mask;
        g.sMb = (int64_t)M * I;
        g.sMm = I;
        return gemm(g, S, st);
    };
    if (hipError_t e = dW2(10, 84, T.ld, W.h2, W.d, T.h2d, w5)) return e;
    if (hipError_t e = dX2(10, 84, T.ld, W.d, w5, T.dh2d, W.h2)) return e;
    if (hipError_t e = dW2(84, 120, T.dh2d, W.h1, W.dh2, T.h1d, w4)) return e;
    if (hipError_t e = dX2(84, 120, T.dh2d, W.dh2, w4, T.dh1d, W.h1)) return e;
    if (hipError_t e = dW2(120, 400, T.dh1d, W.x2, W.dh1, T.x2d, w3)) return e;
    if (hipError_t e = dX2(120, 400, T.dh1d, W.dh1, w3, T.dx2d, nullptr)) return e;
    const float* part1 = nullptr;
    {
        // conv2's G_dot and the routed d P1_dot (over P1_dot: each row is read
        // by its workgroup before its d P1_dot is written), then conv1's G_dot
        // by the primal's weight-gradient kernel, then d/du from the routed
        // primal d P1 (the primal backward's, still in W.g1) and its tangent
        ta.g1g = T.p1d;
        hipLaunchKernelGGL(lenet_conv_bwd_tan_mfma_kernel, dim3(W.nchunk, S), dim3(kTThreads), 0, st,
                           ta);
        ConvArgs c1{};
        c1.M = M;
        c1.u = u;
        c1.r1 = W.r1;
        c1.g1g = T.p1d;
        c1.part1 = W.part1;
        c1.nch1 = W.nch1;
        c1.chunk = (M + W.nch1 - 1) / W.nch1;
        hipLaunchKernelGGL(lenet_conv1_wgrad_mfma_kernel, dim3(W.nch1, (S + kW1S - 1) / kW1S),
                           dim3(256), 0, st, c1, S);
        part1 = W.part1;
        if (d_u)
            hipLaunchKernelGGL(lenet_du_tan_kernel, dim3(W.nchunk, S), dim3(kThreads), 0, st, ta,
                               (const float*)W.g1, (const float*)T.p1d);
    }
    hipLaunchKernelGGL(lenet_conv_reduce_kernel,
                       dim3((unsigned)(((int64_t)S * kNConv + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, S, W.nchunk, nt, T.part, T.gd, part1, W.nch1);
    const int64_t n = nt + (d_u ? (int64_t)M * 784 : 0) + (d_w ? M : 0);
    hipLaunchKernelGGL(lenet_hvp_assemble_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, sa, params, vec, eps, W.dws, T.gd, T.du, T.nlld, hv,
                       d_u, d_w, M, 1.f / (p.d.prior_sd * p.d.prior_sd),
                       include_kl ? 1 : 0);
    return hipGetLastError();
}

}  // namespace psvi
