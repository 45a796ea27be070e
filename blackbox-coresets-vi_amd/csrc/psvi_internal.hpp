// psvi_internal.hpp -- shared host/device definitions of libpsvi_hip.so.
// Written for gfx950 (CDNA4, wave64) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "psvi_hip.h"

namespace psvi {

constexpr int kMaxL = PSVI_MAX_LAYERS;
constexpr int kMaxWorld = 8;      // ranks per node (xGMI)
constexpr int kWave = 64;

// ---------------------------------------------------------------- numerics
// a * b rounded on its own: never fused into an fma with the add that uses it
// (hipcc contracts a * b + c across statements and through __fmul_rn), for
// two kernels that must give the same bits from the same operands
__device__ __forceinline__ float mul_unfused(float a, float b) {
    float r;
    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// torch.nn.functional.softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplus_f(float x) {
    return x > 20.f ? x : log1pf(expf(x));
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

// The wave's index in its workgroup, in an SGPR: the compiler cannot prove
// threadIdx.x >> 6 wave-uniform, and treats loops and branches on it as
// divergent (exec-masked, with conservative s_waitcnt that drain every
// outstanding load at the branch).
__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// sum over each 16-lane row (DPP row rotations; every lane of the row active)
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dppf<0x128>(v));
    v = fmaxf(v, dppf<0x124>(v));
    v = fmaxf(v, dppf<0x122>(v));
    v = fmaxf(v, dppf<0x121>(v));
    return v;
}
// max / sum over the first W lanes of each aligned group of W (W = 2, 4:
// quad permutes; 16: the row reductions above); the result is valid on those
// lanes
template <int W>
__device__ __forceinline__ float lanes_max(float v) {
    static_assert(W == 2 || W == 4 || W == 16, "2, 4 or 16 lanes");
    if constexpr (W == 16) {
        v = fmaxf(v, dppf<0x128>(v));
        v = fmaxf(v, dppf<0x124>(v));
        v = fmaxf(v, dppf<0x122>(v));
        return fmaxf(v, dppf<0x121>(v));
    } else {
        v = fmaxf(v, dppf<0xB1>(v));              // quad_perm [1, 0, 3, 2]: lane ^ 1
        if constexpr (W == 4) v = fmaxf(v, dppf<0x4E>(v));  // quad_perm [2, 3, 0, 1]: lane ^ 2
        return v;
    }
}
template <int W>
__device__ __forceinline__ float lanes_sum(float v) {
    static_assert(W == 2 || W == 4 || W == 16, "2, 4 or 16 lanes");
    if constexpr (W == 16) {
        v += dppf<0x128>(v);
        v += dppf<0x124>(v);
        v += dppf<0x122>(v);
        return v + dppf<0x121>(v);
    } else {
        v += dppf<0xB1>(v);
        if constexpr (W == 4) v += dppf<0x4E>(v);
        return v;
    }
}
__device__ __forceinline__ float row16_sum(float v) {
    v += dppf<0x128>(v);  // row_ror:8
    v += dppf<0x124>(v);  // row_ror:4
    v += dppf<0x122>(v);  // row_ror:2
    v += dppf<0x121>(v);  // row_ror:1
    return v;
}

// Block-wide sum; `red` is >= blockDim/64 floats of LDS.  All threads call.
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = wave_id();
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x == 0)
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    return t;  // valid in thread 0
}

// ------------------------------------------------------- buffer loads (T8)
// 128-bit SRD in SGPRs + 32-bit per-lane byte offset; the hardware range
// check returns 0 for any offset >= `bytes`, which is how the kernels mask
// ragged / triangular tiles without exec-mask branches around the loads.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;  // byte offset past every buffer we map

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, int64_t bytes) {
    const uint32_t nb = bytes > 0x7fffffff ? 0x7fffffffu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nb,
                                             0x00020000);
}
// A 16-byte buffer store whose data registers stay untouched for the two wait
// states after it.  hipcc (ROCm 7.2) does not pad the VMEM-store data hazard
// for __builtin_amdgcn_raw_buffer_store_b128 (it does for global stores): a
// VALU write of a data VGPR in the next instruction can reach memory instead
// of the stored value -- seen as LDS-offset bit patterns in the streaming
// update's tiled Adam state.  The asm reads the data after the store, so no
// instruction in between may redefine those registers, and pads two states.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
#define BSTORE128(v, r, voff, soff, aux)                                    \
    do {                                                                    \
        const u32x4_t bst_v_ = (v);                                         \
        __builtin_amdgcn_raw_buffer_store_b128(bst_v_, r, voff, soff, aux); \
        asm volatile("s_nop 1" ::"v"(bst_v_));                              \
    } while (0)
__device__ __forceinline__ float bload(rsrc_t r, uint32_t off) {
    // the builtin returns the raw 32 bits as an integer
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// ------------------------------------------------- Philox4x32-10 normals
// psvi_randn's stream: normal i of (seed, offset) is element i % 4 of
// Philox4x32-10(counter = offset / 4 + i / 4, key = seed) through Box-Muller.
// Shared by randn_kernel and the network kernel's fused next-step draw.
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    c[0] = hi1 ^ c[1] ^ k0;
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k1;
    c[3] = lo0;
}

__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        philox_round(c, k0, k1);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// normals 4q .. 4q+3 of the stream into out[0, n)
template <bool VEC>
__device__ __forceinline__ void randn_quad(float* __restrict__ out, int64_t n, uint64_t seed,
                                           uint64_t offset, int64_t q) {
    const uint64_t ctr = offset / 4 + (uint64_t)q;
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float r[4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        // Box-Muller on the native transcendentals: u1 in (0, 1], u2 in [0, 1);
        // v_log_f32 is log2, v_sin/v_cos_f32 take revolutions (sin(2 pi u2))
        const float u1 = ((float)(c[2 * j] >> 8) + 1.0f) * (1.0f / 16777216.0f);
        const float u2 = (float)(c[2 * j + 1] >> 8) * (1.0f / 16777216.0f);
        const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
        r[2 * j] = rad * __builtin_amdgcn_cosf(u2);
        r[2 * j + 1] = rad * __builtin_amdgcn_sinf(u2);
    }
    const int64_t base = q * 4;
    if (VEC && base + 3 < n) {
        *reinterpret_cast<float4*>(out + base) = make_float4(r[0], r[1], r[2], r[3]);
    } else {
        for (int j = 0; j < 4 && base + j < n; ++j) out[base + j] = r[j];
    }
}

// ------------------------------------------- bf16 planes of a full-cov draw
// fp32-faithful products on the bf16 matrix cores: x = x0 + x1 + x2, each
// piece bf16 (round to nearest even) and the sum exact for normal fp32 (the
// second residual has <= 8 significant bits); a product of two split operands
// is the six piece products down to 2^-27 relative, below fp32's rounding.
__device__ __forceinline__ uint16_t bf_bits(float x) {
    return __builtin_bit_cast(uint16_t, (__bf16)x);
}
__device__ __forceinline__ float bf_val(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ void split3(float x, uint16_t& x0, uint16_t& x1, uint16_t& x2) {
    x0 = bf_bits(x);
    const float r1 = x - bf_val(x0);
    x1 = bf_bits(r1);
    x2 = bf_bits(r1 - bf_val(x1));
}

// A full-cov eps draw also as three bf16 planes (the streaming update's MFMA
// operands): plane p holds piece p of element (l, s, c) at poff[l] + s npad[l]
// + c, rows padded to npad[l] = a 64-multiple with zeros (the pads are never
// drawn).  eoff: the layers' [S][n] blocks in the fp32 draw order (eoff[L] =
// the draw's length).
struct EpsPlanes {
    int L;
    int64_t pl;  // elements per plane; planes back to back
    int64_t eoff[kMaxL + 1];
    int n[kMaxL], npad[kMaxL];
    int64_t poff[kMaxL];
};

// normals 4q .. 4q+3 of the stream into out[0, n) and, with planes, their
// three bf16 pieces (randn_quad's values)
__device__ __forceinline__ void randn_quad_planes(float* __restrict__ out, int64_t n, uint64_t seed,
                                                  uint64_t offset, int64_t q, const EpsPlanes& P,
                                                  uint16_t* __restrict__ planes) {
    const uint64_t ctr = offset / 4 + (uint64_t)q;
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    float r[4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const float u1 = ((float)(c[2 * j] >> 8) + 1.0f) * (1.0f / 16777216.0f);
        const float u2 = (float)(c[2 * j + 1] >> 8) * (1.0f / 16777216.0f);
        const float rad = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
        r[2 * j] = rad * __builtin_amdgcn_cosf(u2);
        r[2 * j + 1] = rad * __builtin_amdgcn_sinf(u2);
    }
    const int64_t base = q * 4;
    if (base + 3 < n) {
        *reinterpret_cast<float4*>(out + base) = make_float4(r[0], r[1], r[2], r[3]);
    } else {
        for (int j = 0; j < 4 && base + j < n; ++j) out[base + j] = r[j];
    }
    if (!planes) return;
    // element i's place in the planes (selects over the layers: a dynamic
    // index into P would put it in scratch)
    auto place = [&](int64_t i, int& c, int& nl) -> int64_t {
        int64_t e0 = P.eoff[0], po = P.poff[0];
        int np = P.npad[0];
        nl = P.n[0];
#pragma unroll
        for (int k = 1; k < kMaxL; ++k)
            if (k < P.L && i >= P.eoff[k]) {
                e0 = P.eoff[k];
                po = P.poff[k];
                np = P.npad[k];
                nl = P.n[k];
            }
        const int64_t rem = i - e0;
        const int s = (int)(rem / nl);
        c = (int)(rem - (int64_t)s * nl);
        return po + (int64_t)s * np + c;
    };
    uint16_t pc[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split3(r[j], pc[0][j], pc[1][j], pc[2][j]);
    int c0, nl;
    const int64_t o = place(base, c0, nl);
    if (c0 + 3 < nl && base + 3 < n && (o & 3) == 0) {  // the quad in one row
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<u16x4*>(planes + p * P.pl + o) = u16x4{pc[p][0], pc[p][1], pc[p][2], pc[p][3]};
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (base + j >= n) break;
        int cj, nj;
        const int64_t oj = place(base + j, cj, nj);
#pragma unroll
        for (int p = 0; p < 3; ++p) planes[p * P.pl + oj] = pc[p][j];
    }
}

// Adam, both reference variants; returns new p, updates m, v in place.
struct AdamC {
    float lr, b1, b2, eps, omb1, omb2;
    float inv_bc1, inv_sqrt_bc2;  // 1/(1-b1^t), 1/sqrt(1-b2^t)
    float lr_bc1;                 // lr/(1-b1^t)
    float inv_bc2;                // 1/(1-b2^t)
    int kind;
};

__device__ __forceinline__ float adam_apply(const AdamC& a, float p, float g, float& m,
                                            float& v) {
    m = a.b1 * m + a.omb1 * g;
    if (a.kind == PSVI_ADAM_HIGHER) {
        // optim.py:339-367: v stored without the 1e-8; denom = sqrt(v+1e-8)/sqrt(bc2)+eps
        v = a.b2 * v + a.omb2 * g * g;
        const float denom = sqrtf(v + 1e-8f) * a.inv_sqrt_bc2 + a.eps;
        return p - a.lr_bc1 * (m / denom);
    } else if (a.kind == PSVI_ADAM_TORCH) {
        // torch.optim.Adam (single-tensor path): denom = sqrt(v)/sqrt(bc2) + eps
        v = a.b2 * v + a.omb2 * g * g;
        const float denom = sqrtf(v) * a.inv_sqrt_bc2 + a.eps;
        return p - a.lr_bc1 * (m / denom);
    } else {
        // diff_optimizers.py:197-213: v += 1e-12 stored; denom = sqrt(v/bc2)+eps
        v = a.b2 * v + a.omb2 * g * g + 1e-12f;
        const float denom = sqrtf(v * a.inv_bc2) + a.eps;
        return p - a.lr * ((m * a.inv_bc1) / denom);
    }
}

// Same update with the raw v_sqrt_f32 / v_rcp_f32 (1 ulp each) instead of the
// IEEE-exact expansions: the full-cov update runs it on 4.7 M entries per step.
__device__ __forceinline__ float adam_apply_fast(const AdamC& a, float p, float g, float& m,
                                                 float& v) {
    m = a.b1 * m + a.omb1 * g;
    if (a.kind == PSVI_ADAM_HIGHER) {
        v = a.b2 * v + a.omb2 * g * g;
        const float denom = __builtin_amdgcn_sqrtf(v + 1e-8f) * a.inv_sqrt_bc2 + a.eps;
        return p - a.lr_bc1 * m * __builtin_amdgcn_rcpf(denom);
    } else if (a.kind == PSVI_ADAM_TORCH) {
        v = a.b2 * v + a.omb2 * g * g;
        const float denom = __builtin_amdgcn_sqrtf(v) * a.inv_sqrt_bc2 + a.eps;
        return p - a.lr_bc1 * m * __builtin_amdgcn_rcpf(denom);
    } else {
        v = a.b2 * v + a.omb2 * g * g + 1e-12f;
        const float denom = __builtin_amdgcn_sqrtf(v * a.inv_bc2) + a.eps;
        return p - a.lr * (m * a.inv_bc1) * __builtin_amdgcn_rcpf(denom);
    }
}

// ------------------------------------------------------------- plan layout
struct LayerInfo {
    int din, dout;
    int n;          // out*in + out (sampled elements per layer and sample)
    int64_t nc;     // full-cov: packed corr count (n-1)(n-2)/2
    int64_t poff;   // offset of the layer in the flat parameter vector
    int64_t eoff;   // offset of the layer in the flat eps vector (all S)
    int woff;       // offset of the layer in the per-sample weight space [0, n_tot)
    int64_t tbase;  // full-cov tiled layout: first 64x64 tile of the layer
    int nb;         // full-cov: 64-row bands covering rows 0 .. n-1
};

// Full-cov forward work item: rows [r0, r1) (<= kFwdRows) of layer `layer`
// (global row ids, clipped to the rank's row range), columns c in [k0, k1) of L.
constexpr int kFwdRows = 64;
struct FwdItem {
    int layer, r0, r1, k0, k1, xcol;  // xcol: x_shard column of row r0
    int slot;                         // partial-sum slot ([S][kFwdRows] floats) of this item
};
// Rows [r0, r0 + R) (R <= kFwdRows) of one layer: their x = sum of the nk partial
// slots slot0 .. slot0 + nk - 1 (split-K over the columns of L, no atomics).
struct FwdRowBlock {
    int slot0, nk, R, xcol;
    int layer, r0;  // absolute first row (the reduce adds mean + softplus(sd) eps)
    int s0;         // first sample of the block's slots (segmented sample: a pass's 128)
};
// Segmented sample (mvn_fwd_seg_kernel, K = S > 128): units (row block,
// 128-sample pass, 64-column block of L), row block-major then pass then
// column block, cut into equal contiguous runs, one per workgroup; a run's
// piece of one (row block, pass) is a segment with its own partial slot
// ([128][kFwdRows] floats), and the reduce adds a (row block, pass)'s slots.
struct FsSeg {
    int layer, r0, r1, pass;  // rows [r0, r1) of layer, samples [128 pass, 128 pass + 128)
    int k0, k1, slot, pad;    // columns [k0, k1) of L (64-column blocks)
};
// Full-cov update work item: the 64-row band [r0, r0+64) of layer `layer`
// (r0 a multiple of 64; the rank owns rows [rlo, rhi)) against the c-blocks
// [k0, k1) (columns [64 k0, 64 k1)).  The band's G slice is staged once and
// reused across the chunk's c-blocks; the chunk holding c-block r0/64 (diag)
// also updates the band's mean and sd.  xcol: g_shard column of row r is xcol + r.
struct UpdChunk {
    int layer, r0, k0, k1, rlo, rhi, xcol, diag;
    int slot;  // fused next-step sample: partial-sum slot ([S][64] floats), -1 if none
};

// K-split streaming update (mvn_kstream_kernel; Adam, packed state, K = S >
// 128): the rank's 64 x 64 tiles, each K = S samples cut in passes of 128;
// the (tile, pass) units, tile-major, are cut into equal contiguous runs, one
// per workgroup.  A tile whose passes span several runs is "split": each
// contributor writes its partial dL (and diagonal sums) to its slot, and the
// contributor whose count comes last adds the partials in pass order and
// runs the tile's Adam epilogue.
struct KsTile {
    int layer, r0, k, diag;  // band rows [r0, r0 + 64), c-block k, k == band
    int rlo, rhi, xcol;      // rows of the band that exist (< n); g_shard column of row r: xcol + r
    int cnt;                 // counter index of a split tile (-1: never split)
};
constexpr int kKsPass = 128;               // samples per pass (the kernel's LDS stage)
constexpr int kKsSlotFloats = 4096 + 512;  // a split tile's partial: dL fragments, diagonal sums
struct KsSeg {
    int tile, p0, p1;  // passes [p0, p1) of the tile
    int slot, nc, ci;  // split tiles: first slot, contributors, this one's index (slot -1: whole tile)
};

// Streaming fused update (mvn_stream_kernel): workgroup w walks tiles
// [t0, t1) of the layer-major, band-major tile list; its x' partial of each
// band it touches goes to slots slot0, slot0 + 1, ... (a band's slots are
// consecutive over the workgroups).
struct StreamRange {
    int t0, t1, slot0;
    uint32_t lbk0;  // tile t0 as layer << 28 | b << 14 | k
};

// A rank's full-cov rows: rows [lo, hi) of `layer` sit at x-shard columns
// col .. col + hi - lo (world > 1: runs of whole 64-row bands; world 1 and the
// replicated families: one run per layer)
struct ShardRun {
    int layer, lo, hi, col;
};

// world > 1 full-cov network kernel: g_send offset of a 64-row band's first
// row for local sample 0 (owner block + column - first row) and the owner's
// row stride (its rows_total)
struct NetBand {
    int64_t base;
    int32_t stride, pad;
};

struct NetArgs;  // kernels_net.hip

// Outer-objective passes of the network kernel (psvi_outer_elbo_grad).
struct NetOuter {
    int mode;             // 1 forward (per-row NLL), 2 backward (row coefficients)
    int n_pseudo;         // rows [0, n_pseudo) are pseudopoints, the rest data
    float* nll_rows;      // mode 1: [S][M] unweighted NLL
    const float* rowcoef; // mode 2: [S][2] d loss / d pseudo_s, d loss / d data_s
    const float* ck;      // mode 2: [S] d loss / d nkl_s
    float* du_part;       // mode 2, nullable: [S][n_pseudo][D] input gradient
    float* prob_rows;     // mode 1, nullable: [S][M - n_pseudo][C] softmax of the data rows
};

}  // namespace psvi

struct psvi_plan {
    int family = 0;
    psvi_net_desc d{};
    int world = 1, rank = 0;
    int L = 0;
    psvi::LayerInfo lay[psvi::kMaxL];
    int64_t P = 0;        // parameter count
    int64_t Peps = 0;     // eps floats for all S
    int n_tot = 0;        // per-sample weight-space size (sum n)
    // sample shards
    int s_off[psvi::kMaxWorld], s_cnt[psvi::kMaxWorld];
    // full-cov row shards: each rank's runs of rows (whole 64-row bands at
    // world > 1, dealt largest first to the least-loaded rank), its x-shard
    // columns layer-major in row order
    std::vector<psvi::ShardRun> runs[psvi::kMaxWorld];
    int rows_tot[psvi::kMaxWorld];
    int xcol_l[psvi::kMaxWorld][psvi::kMaxL];  // column of layer l's first row in a shard
    // world > 1 full-cov: owner rank and (x-shard column - first row) of every
    // 64-row band, bands numbered layer by layer from band_base[l]
    std::vector<int> band_owner, band_coloff;
    int band_base[psvi::kMaxL + 1] = {0};
    // network kernel: LDS destination of every x element the workgroup loads
    // (stage position -> W_l / b_l offset | W_l^T offset << 16, 0xFFFF = none)
    // and, world > 1, the band table (owner, column offset)
    uint32_t* d_net_xmap = nullptr;
    psvi::NetBand* d_net_bands = nullptr;
    // work lists (host copies, then device)
    std::vector<psvi::FwdItem> h_fwd;
    std::vector<psvi::UpdChunk> h_upd;
    bool on_device = false;
    psvi::FwdItem* d_fwd = nullptr;
    int n_fwd = 0;
    std::vector<psvi::FwdRowBlock> h_frb;
    psvi::FwdRowBlock* d_frb = nullptr;
    int n_frb = 0;
    float* d_fwd_part = nullptr;  // split-K partial slots: n_fwd x S x 32 floats (plan-owned)
    psvi::UpdChunk* d_upd = nullptr;
    // fused update + next-step sample (world == 1, S <= 128): one row block
    // per 64-row band, one partial slot per chunk
    bool fuse_sample = false;
    // tiled corr/m/v (world == 1, S <= 128 inner loops): 64x64 tiles (b, k <= b)
    // per layer in MFMA fragment order, tiles_total * 4096 floats per array
    int64_t tiles_total = 0;
    std::vector<psvi::FwdRowBlock> h_ufrb;
    psvi::FwdRowBlock* d_ufrb = nullptr;
    int n_ufrb = 0, n_uslots = 0;
    float* d_upd_part = nullptr;
    // streaming fused update (fuse_sample plans with S % 32 == 0): one
    // workgroup per range, tile map, band row blocks over its slots
    std::vector<psvi::StreamRange> h_str;
    std::vector<psvi::FwdRowBlock> h_sfrb;
    psvi::StreamRange* d_str = nullptr;
    psvi::FwdRowBlock* d_sfrb = nullptr;
    float* d_str_part = nullptr;
    int* d_str_cnt = nullptr;  // the in-kernel band combine's arrival counters (n_sfrb)
    float* d_str_bms = nullptr;  // per band: new mean + softplus(sd), 128 floats (n_sfrb)
    int str_max_ends = 0;      // most band ends (slots) in one run of the stream
    int n_str = 0, n_sfrb = 0, n_sslots = 0;
    int n_upd = 0;
    int upd_tiles = 0;  // c-blocks over all chunks (work measure)
    // K-split streaming update (full-cov Adam steps with S > 128): tiles, the
    // workgroups' segment lists (offsets [n_kwg + 1]), split-tile partial slots
    // (kKsSlotFloats each) and their arrival counters (zeroed, reset by use)
    std::vector<psvi::KsTile> h_ks_tiles;
    std::vector<psvi::KsSeg> h_ks_segs;
    std::vector<int> h_ks_off;
    psvi::KsTile* d_ks_tiles = nullptr;
    psvi::KsSeg* d_ks_segs = nullptr;
    int* d_ks_off = nullptr;
    float* d_ks_slots = nullptr;
    int* d_ks_cnt = nullptr;
    int n_kwg = 0, n_ks_slots = 0, n_ks_cnt = 0;
    // segmented sample (S > 128): segments, per-workgroup offsets, (row block,
    // pass) reduce blocks, partial slots ([n_fs_slots][128][kFwdRows])
    std::vector<psvi::FsSeg> h_fs_segs;
    std::vector<int> h_fs_off;
    std::vector<psvi::FwdRowBlock> h_fs_rb;
    psvi::FsSeg* d_fs_segs = nullptr;
    int* d_fs_off = nullptr;
    psvi::FwdRowBlock* d_fs_rb = nullptr;
    float* d_fs_part = nullptr;
    int n_fswg = 0, n_fs_slots = 0, n_fs_rb = 0;
    // psvi_hvp's sample pair (one eight-wave workgroup per CU): the same units
    // over 256 workgroups, slots in d_fs_part (sized for both tables)
    std::vector<psvi::FsSeg> h_fp_segs;
    std::vector<int> h_fp_off;
    std::vector<psvi::FwdRowBlock> h_fp_rb;
    psvi::FsSeg* d_fp_segs = nullptr;
    int* d_fp_off = nullptr;
    psvi::FwdRowBlock* d_fp_rb = nullptr;
    int n_fpwg = 0, n_fp_slots = 0, n_fp_rb = 0;
    // net kernel geometry
    int mchunks = 1, mc = 0, net_threads = 256, net_roles = 1;
    bool net_mloop = false;  // full-cov inner objective: the LDS-forced chunks looped in a workgroup
    size_t net_lds = 0;
    size_t ws_bytes = 0;
    int64_t acc_count = 0;
    // LeNet: plan-owned activation / gradient scratch (kernels_lenet.hip)
    void* d_lenet_ws = nullptr;
    // mean-field: plan-owned per-(sample, pseudopoint chunk) gradient slots
    // [s_cnt[rank]][mchunks][n_tot]; one writer per element, summed in a fixed
    // order by the update (run-to-run bitwise reproducible, no float atomics)
    float* d_mf_slots = nullptr;
    // full-cov with pseudopoint chunks: per-chunk dW slots [mchunks][s_cnt[rank]][n_tot],
    // added in chunk order into g_send (no float atomics)
    float* d_net_slots = nullptr;
    // tiled-state inner loops: the packed -> tiled conversion runs on aux_st,
    // forked from / joined to the caller's stream by the two events, behind the
    // first sample and network step (not re-entrant across host threads)
    hipStream_t aux_st = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // bf16-plane streaming update (tiled S = 128 loops): every eps draw of
    // the loop also as three bf16 planes (EpsPlanes; device copy for the
    // network kernel's fused draw), two plane buffers in the loop workspace
    bool bf_stream = false;
    psvi::EpsPlanes eps_planes{};
    psvi::EpsPlanes* d_eps_planes = nullptr;
    // psvi_inner_loop_ex(PSVI_LOOP_KEEP): what the last call left in its
    // workspace -- the tiled corr / m / v, the draw at `offset` (eps buffer
    // `ebuf`, and its planes) and the sample x from it -- and for which
    // arrays; any loop call clears it first (mutable: the API's plans are const)
    struct Resident {
        bool valid = false;
        const void* ws = nullptr;
        const float *params = nullptr, *m = nullptr, *v = nullptr;
        uint64_t seed = 0, offset = 0;
        int ebuf = 0;
    };
    mutable Resident resident{};
};

namespace psvi {
// input features per row: D, or 1x28x28 for LeNet
inline int plan_in_dim(const psvi_plan& p) {
    return p.family == PSVI_FAMILY_LENET ? 784 : p.lay[0].din;
}
// layers whose sampled KL enters psvi_elbo (LeNet: the VILinear layers only,
// psvi_classes.py:455-459 sums sampled_nkl over VILinear modules)
inline unsigned plan_nkl_mask(const psvi_plan& p) {
    return p.family == PSVI_FAMILY_LENET ? 0x1Cu : 0xFFu;
}
// the full-cov network kernel's x map and band table (kernels_net.hip)
void net_xmap(const psvi_plan& p, std::vector<uint32_t>& xmap, std::vector<NetBand>& bands);
// launchers (defined in the .hip translation units)
hipError_t launch_net(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                      const float* params, const float* eps, float* mf_slots,
                      const float* xrecv, float* gsend, double* nll_out, hipStream_t st,
                      float* rn_out = nullptr, int64_t rn_n = 0, uint64_t rn_seed = 0,
                      uint64_t rn_off = 0, const NetOuter* outer = nullptr,
                      uint16_t* rn_planes = nullptr, int s_begin = 0, int s_count = -1,
                      int rn_part = 0, int rn_nparts = 1);
// acc == nullptr: the accumulators come from the plan's mean-field gradient
// slots, reduced in a fixed order against slot_eps (the step's eps)
hipError_t launch_mf_update(const psvi_plan& p, const float* acc, float* params,
                            float* m, float* v, const psvi_adam_hp* hp, double* kl_out,
                            float* grad_out, int include_kl, hipStream_t st,
                            const float* slot_eps = nullptr);
// acc = [sum_s dW_s | sum_s dW_s eps_s] from the plan's mean-field gradient slots
hipError_t launch_mf_slot_acc(const psvi_plan& p, const float* eps, float* acc, hipStream_t st);
// diag_of (HVP tangent sample): params is the direction, the diagonal
// sigmoid(diag_of's sd) * its sd slot
hipError_t launch_mvn_fwd(const psvi_plan& p, const float* eps, const float* params,
                          float* x_shard, hipStream_t st, const float* diag_of = nullptr);
hipError_t launch_mvn_fwd_pair(const psvi_plan& p, const float* eps, const float* params,
                               float* x, const float* vec, float* x2, float* part2,
                               hipStream_t st);
hipError_t launch_mvn_update(const psvi_plan& p, const float* eps, const float* g_shard,
                             float* params, float* m, float* v, const psvi_adam_hp* hp,
                             double* kl_out, float* grad_out, int include_kl,
                             const float* eps_next, float* x_next, hipStream_t st,
                             float* tstate = nullptr, bool packed_out = false,
                             const float* kl_vec = nullptr, bool padded = false,
                             const uint16_t* eps_planes = nullptr,
                             const uint16_t* eps_next_planes = nullptr,
                             const float* g_shard2 = nullptr);
// the gradient-mode update takes a second G slot (g_shard2: added to g_shard at
// staging, the R-op's row-block slots unsummed) when this holds
bool mvn_grad_takes_slots(const psvi_plan& p);
// pads (to_tiled, nullable): three 64-float regions the first workgroup zeroes
hipError_t launch_mvn_tile_convert(const psvi_plan& p, float* params, float* m, float* v,
                                   float* tstate, bool to_tiled, hipStream_t st,
                                   float* const* pads = nullptr);
hipError_t launch_randn(float* out, int64_t n, uint64_t seed, uint64_t offset, hipStream_t st,
                        double* zero = nullptr, int64_t nzero = 0,
                        const EpsPlanes* planes_desc = nullptr, uint16_t* planes = nullptr);
hipError_t launch_adam(int64_t n, float* p, const float* g, float* m, float* v,
                       const psvi_adam_hp* hp, hipStream_t st);
AdamC make_adam(const psvi_adam_hp* hp);
hipError_t launch_adam_adjoint(int64_t n, const float* lt, float* lm, float* lv, const float* m,
                               const float* v, const float* g, float* lg,
                               const psvi_adam_hp* hp, hipStream_t st);
// outer objective (kernels_outer.hip)
hipError_t launch_outer_stats(const psvi_plan& p, const float* params, const float* eps,
                              const float* x, double* stats, hipStream_t st);
hipError_t launch_outer_combine(const psvi_plan& p, int n_pseudo, const float* params,
                                const float* w, const float* nll, const double* stats,
                                double* loss, float* rowcoef, float* ck, float* sck,
                                float* grad_w, double* sample_out, int ablated,
                                hipStream_t st);
hipError_t launch_eval(const psvi_plan& p, int n_pseudo, const float* params, const float* w,
                       const int32_t* z, const float* nll, const double* stats,
                       const float* prob, int correction, float* W, float* probs_out,
                       double* out, hipStream_t st);
hipError_t launch_outer_gradw(const psvi_plan& p, int n_pseudo, const float* nll,
                              const float* rowcoef, float* grad_w, hipStream_t st);
hipError_t launch_outer_finish(const psvi_plan& p, int n_pseudo, const float* params,
                               const float* sck, float* grad, const float* du_part,
                               float* grad_u, hipStream_t st);
// LeNet (kernels_lenet.hip): scratch carve of the plan-owned buffer
struct LenetWs {
    float *wsamp, *dws, *p1, *x2, *h1, *h2, *d, *dh2, *dh1, *dx2, *part;
    int8_t *r1, *r2;
    int nchunk;
    float *g1, *part1;  // MFMA backward: routed d P1 [S][M][1176], conv1 partials [S][nch1][156]
    int nch1;
    size_t bytes;
};
int lenet_nchunk(const psvi_plan& p);
LenetWs lenet_ws(const psvi_plan& p, void* base);  // base nullptr: sizes only
// per-sample weight draw, forward, weighted NLL (+= nll_out), backward, and
// acc = [sum_s dW | sum_s dW eps] over the rank's samples (acc fully written)
// outer (psvi_outer_elbo_grad / psvi_evaluate): mode 1 forward only (per-row
// NLL, softmax of the data rows), mode 2 backward of the row coefficients with
// the pathwise sampled-KL term on the VILinear layers and d u of the pseudo rows
hipError_t launch_lenet(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                        const float* params, const float* eps, float* acc, double* nll_out,
                        void* ws, hipStream_t st, const NetOuter* outer = nullptr);
// LeNet HVP (kernels_lenet.hip): tangent scratch in the caller's workspace;
// the primal pass uses the plan-owned scratch
struct LenetTanWs {
    double* nll;
    float *acc, *wdot, *gd, *p1d, *x2d, *h1d, *h2d, *ld, *prob, *dh2d, *dh1d, *dx2d, *part, *du,
        *nlld;
    size_t bytes;
};
LenetTanWs lenet_tan_ws(const psvi_plan& p, void* base);
hipError_t launch_lenet_hvp(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                            const float* eps, const float* params, const float* vec, float* hv,
                            float* d_u, float* d_w, void* tws, hipStream_t st,
                            bool include_kl = true);
hipError_t launch_nonfinite(const void* x, int64_t n, int dtype, int32_t* flag, hipStream_t st);
// hyper_step's conjugate-gradient iteration (kernels_cg.hip)
size_t cg_ws_bytes();
hipError_t launch_cg_scale(int64_t n, const float* hv, double lr, float* out, hipStream_t st);
hipError_t launch_cg_pap(int64_t n, const float* hv1, const float* hv2, double lr, const double* p,
                         double* state, void* ws, hipStream_t st);
hipError_t launch_cg_residual(int64_t n, const float* hv1, const float* hv2, double lr, double* r,
                              double* state, double tol, void* ws, hipStream_t st);
hipError_t launch_cg_update(int64_t n, double* x, double* p, float* p32, const double* r,
                            const double* state, hipStream_t st);
// Hessian-vector products (kernels_rop.hip)
int rop_rows(const psvi_plan& p);
int rop_splits(const psvi_plan& p);  // row blocks per sample: G / G_dot slots
hipError_t launch_net_rop(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                          const float* x, const float* xd, const float* params, const float* vec,
                          const float* eps, float* G, float* Gd, float* du, float* nlld,
                          hipStream_t st, bool sum_slots = true);
hipError_t launch_hvp_assemble(const psvi_plan& p, const float* params, const float* vec,
                               const float* eps, const float* G, const float* Gd, const float* du,
                               const float* nlld, float* hv, float* d_u, float* d_w,
                               hipStream_t st, bool include_kl = true, int64_t slot2 = 0);
}  // namespace psvi
