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
#include <type_traits>

#include "psvi_internal.hpp"

namespace psvi {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct MvnLayerArgs {
    int n;
    int64_t poff, eoff;
    int64_t tbase;  // tiled layout: first tile of the layer
};

// Tiled corr/m/v (world == 1 inner loops): tile (b, k <= b) of a layer holds
// rows [64b, 64b+64) x columns [64k, 64k+64) of L's strict lower part (0
// elsewhere) in the update MFMA's fragment order: wave w = 2 wr + wc, column
// group g, lane = 32 h + l32 hold the float4 of row 64b + 32 wr + l32, columns
// 64k + 32 wc + 8 g + 4 h .. +3, at ((w * 4 + g) * 64 + lane) * 4.  Every
// wave instruction of the update then moves 1 KB of contiguous memory.
__device__ __forceinline__ int64_t tile_index(const MvnLayerArgs& l, int b, int k) {
    return l.tbase + (int64_t)b * (b + 1) / 2 + k;
}

// ----------------------------------------------------------------- forward
constexpr int FBK = 64;    // k (columns of L) per LDS stage
constexpr int FST = 128;   // samples per pass: 4 waves x 32
constexpr int FLD = FBK + 4;  // LDS row stride: 16-byte rows (float4 stores, ds_read_b128)

// bf16 pieces (fp32-faithful products on v_mfma_f32_32x32x16_bf16): the
// cache policy of mvn_stream_bf2_kernel's tiled-state loads: read once per
// launch, so nt (2) -- the L2 keeps the eps planes, which every tile of a
// column re-reads.  C3 (tools/gpu_g25.sh): 180.8 -> 175.7 MB per launch
// (FETCH_SIZE x 2 + WRITE_SIZE), kernel time unchanged (38.3 us); sc1 nt (18)
// the same.  Other values: A/B builds only.
#ifndef PSVI_STATE_LOAD_AUX
#define PSVI_STATE_LOAD_AUX 2
#endif

// helpers of mvn_stream_bf2_kernel, mvn_fwd_seg_bf_kernel and the bf16 K-split update
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short bf8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx16 mfma6(const bf8v (&x)[3], const bf8v (&y)[3], floatx16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[2], y[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[1], y[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[1], y[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[0], y[0], c, 0, 0, 0);
    return c;
}
__device__ __forceinline__ bf8v cat44(s4v lo, s4v hi) {
    return bf8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// LDS images of a 128 x 64 bf16 block, 128-byte rows.  Column image (the
// transposed reads): 16-byte chunk c / 8 XORed with 4 on rows 2, 3 (mod 4), so
// a 32-lane half's four rows of one 64-byte run fall on four bank ranges.  Row
// image (x''s A operand, 8 columns per lane: c0 .. c0 + 3 and c0 + 8 .. c0 +
// 11 for c0 = 16 m + 4 h): each 16-column group stored in the order 0-3, 8-11,
// 4-7, 12-15, so a lane's 8 columns are one 16-byte chunk 2 m + h, and the
// chunk XORed with (s / 2) mod 8, so a ds_read_b128 lane group's 16 rows fall
// on 16 distinct (bank half, chunk) pairs.
// split3 on two entries at once: packed conversions (v_cvt_pk_bf16_f32) and
// packed subtractions; word p holds piece p of both entries (entry 0 low)
__device__ __forceinline__ void split3_pk(f32x2 x, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
    typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
    auto cvt = [](f32x2 v) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf2v)); };
    auto val = [](uint32_t w) { return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)}; };
    w0 = cvt(x);
    const f32x2 r1 = x - val(w0);
    w1 = cvt(r1);
    w2 = cvt(r1 - val(w1));
}
// entries j, j + 1 of a fragment as fp32 (the pieces' values)
__device__ __forceinline__ f32x2 bf_pair(bf8v v, int j) {
    const uint32_t w = (uint32_t)(uint16_t)v[j] | ((uint32_t)(uint16_t)v[j + 1] << 16);
    return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
constexpr int kBfImg = 128 * 128;  // bytes per plane image
__device__ __forceinline__ int img_col(int s, int c) {
    return s * 128 + (((c >> 3) ^ (((s >> 1) & 1) << 2)) << 4) + ((c & 7) << 1);
}
__device__ __forceinline__ int img_row(int s, int c) {
    // column c: group m = c / 16, quarter q = (c / 4) % 4 -> chunk 2 m + (q & 1),
    // half q >> 1 of the chunk
    const int q = (c >> 2) & 3;
    return s * 128 + ((((c >> 4) * 2 + (q & 1)) ^ ((s >> 1) & 7)) << 4) + ((q >> 1) << 3) + ((c & 3) << 1);
}

struct FwdArgs {
    const FwdItem* items;
    const float* params;
    const float* eps;
    float* part;      // split-K partial slots [n_items][S][32]
    int ldx, S;
    int64_t e_total;  // floats in eps (load guards)
    const float* diag_of;  // HVP tangent sample: params is the direction vec, and the
                           // diagonal is sigmoid(diag_of's sd) vec_sd (nullptr: softplus(sd))
    // pair launches (launch_mvn_fwd_pair, blockIdx.y / .z = 1): the second
    // sample's parameters, split-K slots and diagonal source
    const float* params2;
    float* part2;
    const float* diag_of2;
    int abl;                     // diagnostics ablation mask (0 in production):
                                 // 1 loads, 2 MFMAs, 4 x atomics
    unsigned long long* stamps;  // diagnostics: 16 slots per workgroup
    // segmented sample (mvn_fwd_seg_kernel): segments, per-workgroup offsets,
    // parameter count (buffer range), sample rows per slot (0: S, one slot spans
    // all samples -- the item grid and the fused updates' slots)
    const FsSeg* segs;
    const int* seg_off;
    int64_t pcount;
    int slot_rows;
    int slot_frag;  // slots in MFMA fragment order (the segmented sample)
    int seg_nrun;  // runs in seg_off (one per workgroup)
    MvnLayerArgs lay[kMaxL];
};

// Branch-free 16-byte loads (see the update kernel below for the rationale):
// clamp the offset into the buffer for the load, shift back at consumption.
__device__ __forceinline__ int fclamp4(int off, int lo, int hi) {
    return off < lo ? lo : (off > hi - 4 ? hi - 4 : off);
}
__device__ __forceinline__ float4 fld4(const float* base, int off, int lo, int hi) {
    return *reinterpret_cast<const float4*>(base + fclamp4(off, lo, hi));
}
__device__ __forceinline__ float4 ffix4(float4 v, int off, int lo, int hi) {
    const int d = off - fclamp4(off, lo, hi);
    if (d == 0) return v;  // VALU-only branch
    const float x[4] = {v.x, v.y, v.z, v.w};
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = i + d;
        r[i] = k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : k == 3 ? x[3] : 0.f;
    }
    return make_float4(r[0], r[1], r[2], r[3]);
}

#define FWD_STAMP(k, val)                                                          \
    do {                                                                           \
        if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 16 + (k)] = (val); \
    } while (0)

// One item: rows [r0, r1) (<= kFwdRows) of L against columns [k0, k1) for all
// samples: D[s][r] = sum_c eps[s][c] L[r][c] on v_mfma_f32_32x32x2_f32; wave w
// owns 32 samples x all kFwdRows rows (FT = kFwdRows/32 accumulators), so one
// eps fragment feeds FT MFMAs and the eps block (L2-resident, shared by every
// item of the column range) is read once per kFwdRows rows.  Stages of 64 columns:
// L rows (packed triangle, 256-byte runs) and eps rows go global -> registers
// (float4) -> LDS, the next stage's loads in flight during this stage's
// MFMAs.  k-permuted operand feed: one ds_read_b128 per operand per 4 MFMAs.
// Each item stores its partial sums in its own slot; mvn_fwd_reduce_kernel
// adds a row block's slots and mean + softplus(sd) eps into x (split-K
// without atomics; float atomics from the k-chunks of a row block contend on
// the same addresses).
__global__ __launch_bounds__(256, 2) void mvn_fwd_kernel(FwdArgs a) {
    __shared__ __attribute__((aligned(16))) float Es[FST * FLD];       // eps  [s][k]
    __shared__ __attribute__((aligned(16))) float Ls[kFwdRows * FLD];  // corr [r][k]
    FWD_STAMP(0, __builtin_amdgcn_s_memtime());
    FWD_STAMP(6, __builtin_amdgcn_s_memrealtime());  // chip-wide 100 MHz clock
    FWD_STAMP(4, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4));
    FWD_STAMP(5, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20));
    const FwdItem it = a.items[blockIdx.x];
    const int n = a.lay[it.layer].n;
    const bool second = blockIdx.y == 1;  // pair launch: the second sample
    const float* corr = (second ? a.params2 : a.params) + a.lay[it.layer].poff + 2 * n;
    float* const part = second ? a.part2 : a.part;
    const int corr_len = (int)((int64_t)(n - 1) * (n - 2) / 2);
    const int eoff = (int)a.lay[it.layer].eoff;
    const rsrc_t re = make_rsrc(a.eps, 4 * a.e_total);
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int col4 = tid & 15, srow = tid >> 4;
    constexpr int FT = kFwdRows / 32, LJ = kFwdRows / 16;
    // this thread's staged L rows
    int lrp[LJ];
#pragma unroll
    for (int j = 0; j < LJ; ++j) {
        const int r = it.r0 + srow + 16 * j;
        lrp[j] = r >= 1 ? (int)((int64_t)r * (r - 1) / 2) : 0;
    }
    const int klast = it.k0 + ((it.k1 - it.k0 - 1) / FBK) * FBK;  // last stage start

    // sample blocks: gridDim.z workgroups share an item's FST-sample passes
    // (launch_mvn_fwd spreads them when the items alone leave CUs idle)
    for (int sb = blockIdx.z * FST; sb < a.S; sb += FST * gridDim.z) {
        floatx16 acc[FT];
#pragma unroll
        for (int t = 0; t < FT; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        const bool wave_live = sb + 32 * wv < a.S;
        float4 lreg[LJ], ereg[8];
        // eps through buffer loads: the per-dword range check returns 0 past
        // the buffer's end, and rows past S go to offset kOOB (zeros) -- no
        // clamp, fix-up or select at staging
        auto eofs = [&](int j, int kb) {
            const int sr = sb + srow + 16 * j;
            return sr < a.S ? (uint32_t)(eoff + sr * n + kb + 4 * col4) * 4u : kOOB;
        };
        auto fetch = [&](int kb) {
#pragma unroll
            for (int j = 0; j < LJ; ++j)
                lreg[j] = fld4(corr, (a.abl & 1) ? 0 : lrp[j] + kb + 4 * col4, 0, corr_len);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                ereg[j] = __builtin_bit_cast(
                    float4, __builtin_amdgcn_raw_buffer_load_b128(re, (a.abl & 1) ? 0u : eofs(j, kb), 0, 0));
        };
        auto stage = [&](int kb) {
            const int c = kb + 4 * col4;
#pragma unroll
            for (int j = 0; j < LJ; ++j) {
                // entries outside the item / triangle / column range are 0
                const int r = it.r0 + srow + 16 * j;
                const float4 v = ffix4(lreg[j], lrp[j] + c, 0, corr_len);
                const bool rok = r < it.r1 && r <= n - 2;
                float4 o;
                o.x = rok && c + 0 < r && c + 0 < it.k1 ? v.x : 0.f;
                o.y = rok && c + 1 < r && c + 1 < it.k1 ? v.y : 0.f;
                o.z = rok && c + 2 < r && c + 2 < it.k1 ? v.z : 0.f;
                o.w = rok && c + 3 < r && c + 3 < it.k1 ? v.w : 0.f;
                *reinterpret_cast<float4*>(&Ls[(srow + 16 * j) * FLD + 4 * col4]) = o;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) *reinterpret_cast<float4*>(&Es[(srow + 16 * j) * FLD + 4 * col4]) = ereg[j];
        };
        if (it.k0 < it.k1) fetch(it.k0);
        for (int kb = it.k0; kb < it.k1; kb += FBK) {
            __syncthreads();  // previous stage's MFMAs done with the LDS
            stage(kb);
            __syncthreads();
            fetch(min(kb + FBK, klast));  // unconditional: keeps the vmcnt bookkeeping exact
            if (kb == it.k0 && sb == 0) FWD_STAMP(1, __builtin_amdgcn_s_memtime());
            if (wave_live && !(a.abl & 2)) {
                // k permutation: per 8 columns, lane half h feeds k = kk + 4h + j to
                // MFMA j (j = 0..3) for BOTH operands -- the same sum over k
                const float* Ea = Es + (32 * wv + l32) * FLD + 4 * h;
                const float* Lb = Ls + l32 * FLD + 4 * h;
#pragma unroll
                for (int kk = 0; kk < FBK; kk += 8) {
                    const float4 av = *reinterpret_cast<const float4*>(Ea + kk);
                    float4 bv[FT];
#pragma unroll
                    for (int t = 0; t < FT; ++t)
                        bv[t] = *reinterpret_cast<const float4*>(Lb + 32 * t * FLD + kk);
#pragma unroll
                    for (int t = 0; t < FT; ++t) {
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[t].x, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[t].y, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[t].z, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[t].w, acc[t], 0, 0, 0);
                    }
                }
            }
        }
        FWD_STAMP(2, __builtin_amdgcn_s_memtime());
        // D[i = s][j = r]: j = lane&31, i = (q&3) + 8(q>>2) + 4h
        if (wave_live && !(a.abl & 4)) {
#pragma unroll
            for (int t = 0; t < FT; ++t) {
                if (it.r0 + 32 * t + l32 >= it.r1) continue;
                float* slot = part + (size_t)it.slot * a.S * kFwdRows + 32 * t + l32;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int s = sb + 32 * wv + (q & 3) + 8 * (q >> 2) + 4 * h;
                    if (s < a.S) slot[(size_t)s * kFwdRows] = acc[t][q];
                }
            }
        }
    }
    FWD_STAMP(3, __builtin_amdgcn_s_memtime());
    FWD_STAMP(7, __builtin_amdgcn_s_memrealtime());
}

// x[s][xcol + rr] = mean[r] + softplus(sd[r]) eps[s][r] + sum over the row
// block's slots (r = r0 + rr); one workgroup per (row block, 256/kFwdRows
// samples), coalesced along the rows.
// Two samples per thread (s and s + 4 of the block's 8): the row block's
// descriptor, mean and softplus(sd) serve both, and twice the loads are in
// flight.
constexpr int kRedSpb = 2 * 256 / kFwdRows;  // samples per reduce block
__global__ __launch_bounds__(256) void mvn_fwd_reduce_kernel(const FwdRowBlock* rbs,
                                                             const float* part, FwdArgs a,
                                                             float* x, float* x2 = nullptr) {
    const FwdRowBlock rb = rbs[blockIdx.x];
    // pair launch: the second sample (locals -- writing into the by-value
    // argument copies the whole struct to scratch)
    const bool second = blockIdx.z == 1;
    if (second) {
        part = a.part2;
        x = x2;
    }
    const float* const prm = second ? a.params2 : a.params;
    const float* const dof = second ? a.diag_of2 : a.diag_of;
    const int rr = threadIdx.x & (kFwdRows - 1);
    // slots of slot_rows samples from sample rb.s0 (0 / S: one slot spans all)
    const int srows = a.slot_rows > 0 ? a.slot_rows : a.S;
    const int l0 = blockIdx.y * kRedSpb + threadIdx.x / kFwdRows, l1 = l0 + kRedSpb / 2;
    const int s0 = rb.s0 + l0, s1 = rb.s0 + l1, s_end = min(a.S, rb.s0 + srows);
    if (s0 >= s_end || rr >= rb.R) return;
    const bool two = s1 < s_end;
    const int n = a.lay[rb.layer].n, r = rb.r0 + rr;
    const float* mean = prm + a.lay[rb.layer].poff;
    const float* eps = a.eps + a.lay[rb.layer].eoff + r;
    const float e0 = eps[(int64_t)s0 * n], e1 = eps[(int64_t)(two ? s1 : s0) * n];
    const float mu = mean[r], sdr = mean[n + r];
    const size_t st = (size_t)srows * kFwdRows;
    // slot element (sample l, row rr): row-major [l][rr], or (a.slot_frag, the
    // segmented sample) the MFMA fragment order of mvn_fwd_seg_kernel
    auto so = [&](int l) -> size_t {
        if (!a.slot_frag) return (size_t)l * kFwdRows + rr;
        const int i = l & 31, hh = (i >> 2) & 1, q = (i & 3) + 4 * (i >> 3);
        return ((size_t)((l >> 5) * (kFwdRows / 32) + (rr >> 5)) * 16 + q) * 64 + (rr & 31) + 32 * hh;
    };
    const float* p0 = part + (size_t)rb.slot0 * st + so(l0);
    const float* p1 = part + (size_t)rb.slot0 * st + so(two ? l1 : l0);
    // The first 8 slots as unconditional loads at clamped indices (all in
    // flight at once; a row block of C3's streaming update has 1-10 slots),
    // any further ones 4 at a time.  Partial sums s4[k % 4] in slot order k =
    // 0, 1, ..., so the result does not depend on the unroll.
    float a4[4] = {0.f, 0.f, 0.f, 0.f}, b4[4] = {0.f, 0.f, 0.f, 0.f};
    {
        float va[8], vb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const size_t o = (size_t)max(min(i, rb.nk - 1), 0) * st;
            va[i] = p0[o];
            vb[i] = p1[o];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            a4[i & 3] += i < rb.nk ? va[i] : 0.f;
            b4[i & 3] += i < rb.nk ? vb[i] : 0.f;
        }
    }
    int k = 8;
    for (; k + 4 <= rb.nk; k += 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            a4[i] += p0[(k + i) * st];
            b4[i] += p1[(k + i) * st];
        }
    }
    for (int i = 0; k + i < rb.nk; ++i) {
        a4[i] += p0[(k + i) * st];
        b4[i] += p1[(k + i) * st];
    }
    const float dg = dof ? sigmoid_f(dof[a.lay[rb.layer].poff + n + r]) * sdr
                               : softplus_f(sdr);
    // mean + (softplus(sd) eps, rounded) + the slots: the product never fused
    // into an fma, here and in the streaming update's in-kernel combine, so
    // the two give the same bits
    x[(int64_t)s0 * a.ldx + rb.xcol + rr] = (mu + mul_unfused(dg, e0)) + ((a4[0] + a4[1]) + (a4[2] + a4[3]));
    if (two)
        x[(int64_t)s1 * a.ldx + rb.xcol + rr] = (mu + mul_unfused(dg, e1)) + ((b4[0] + b4[1]) + (b4[2] + b4[3]));
}

// Segmented sample (K = S > 128): one persistent workgroup run of the
// (row block, pass, column block) unit list (build_fseg), two per CU.  Per
// segment -- consecutive column blocks of one (row block, 128-sample pass) --
// D[s][r] = sum_c eps[s][c] L[r][c] accumulates over its column blocks as in
// mvn_fwd_kernel (64-column LDS stages, k-permuted ds_read_b128 feed, wave w
// = 32 samples x 64 rows), then goes to the segment's slot ([128][64]); the
// reduce adds a (row block, pass)'s slots.  The next stage -- the next
// segment's first after a segment's last -- is loaded behind the MFMAs.  corr
// and eps through buffer loads: the range check returns 0 past the end (rows
// past S to offset kOOB); the triangle / row masks are applied at staging.
__global__ __launch_bounds__(256, 2) void mvn_fwd_seg_kernel(FwdArgs a) {
    __shared__ __attribute__((aligned(16))) float Es[FST * FLD];       // eps  [s][k]
    __shared__ __attribute__((aligned(16))) float Ls[kFwdRows * FLD];  // corr [r][k]
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int col4 = tid & 15, srow = tid >> 4;
    constexpr int FT = kFwdRows / 32, LJ = kFwdRows / 16;
    const rsrc_t re = make_rsrc(a.eps, 4 * a.e_total);
    const rsrc_t rp = make_rsrc(a.params, 4 * a.pcount);
    const int sbeg = a.seg_off[blockIdx.x], send = a.seg_off[blockIdx.x + 1];
    if (sbeg >= send) return;  // uniform, before any barrier
    struct D {
        int n, corr, eoff, r0, r1, s0;
    };
    auto desc = [&](const FsSeg& g) __attribute__((always_inline)) {
        D d;
        int poff = (int)a.lay[0].poff;
        d.n = a.lay[0].n;
        d.eoff = (int)a.lay[0].eoff;
#pragma unroll
        for (int l = 1; l < kMaxL; ++l)  // select: a dynamic index into the arguments goes to scratch
            if (g.layer == l) {
                d.n = a.lay[l].n;
                d.eoff = (int)a.lay[l].eoff;
                poff = (int)a.lay[l].poff;
            }
        d.corr = poff + 2 * d.n;
        d.r0 = g.r0;
        d.r1 = g.r1;
        d.s0 = g.pass * FST;
        return d;
    };
    float4 lreg[LJ], ereg[8];
    auto fetch = [&](const D& d, int kb) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < LJ; ++j) {
            const int r = d.r0 + srow + 16 * j;
            const int ro = r >= 1 ? (int)((int64_t)r * (r - 1) / 2) : 0;
            lreg[j] = __builtin_bit_cast(
                float4, __builtin_amdgcn_raw_buffer_load_b128(rp, (uint32_t)(d.corr + ro + kb + 4 * col4) * 4u, 0, 0));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int sr = d.s0 + srow + 16 * j;
            const uint32_t eo = sr < a.S ? (uint32_t)(d.eoff + sr * d.n + kb + 4 * col4) * 4u : kOOB;
            ereg[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(re, eo, 0, 0));
        }
    };
    auto stage = [&](const D& d, int kb) __attribute__((always_inline)) {
        const int c = kb + 4 * col4;
#pragma unroll
        for (int j = 0; j < LJ; ++j) {
            // entries outside the block's rows / the strict lower triangle are 0
            const int r = d.r0 + srow + 16 * j;
            const bool rok = r < d.r1 && r <= d.n - 2;
            const float4 v = lreg[j];
            float4 o;
            o.x = rok && c + 0 < r ? v.x : 0.f;
            o.y = rok && c + 1 < r ? v.y : 0.f;
            o.z = rok && c + 2 < r ? v.z : 0.f;
            o.w = rok && c + 3 < r ? v.w : 0.f;
            *reinterpret_cast<float4*>(&Ls[(srow + 16 * j) * FLD + 4 * col4]) = o;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) *reinterpret_cast<float4*>(&Es[(srow + 16 * j) * FLD + 4 * col4]) = ereg[j];
    };
    // diagnostics (a.stamps): shader clocks -- 1 until the first stage is in
    // LDS, 2 stages + MFMAs, 3 slot writes (summed over segments); 6 stages;
    // 0 / 12 start / end, 13 / 14 the 100 MHz clock at start / end
    const bool dgn = a.stamps != nullptr;
    unsigned long long ph[4] = {0ull, 0ull, 0ull, 0ull}, tprev = dgn ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long t_start = tprev, rt_start = dgn ? __builtin_amdgcn_s_memrealtime() : 0ull;
    int nst = 0;
    auto mark = [&](int q) __attribute__((always_inline)) {
        if (dgn) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            ph[q] += t - tprev;
            tprev = t;
        }
    };
    FsSeg gn = a.segs[sbeg];
    D dn = desc(gn);
    fetch(dn, gn.k0);
    for (int si = sbeg; si < send; ++si) {  // uniform
        const FsSeg g = gn;
        const D d = dn;
        const bool more = si + 1 < send;
        if (more) {
            gn = a.segs[si + 1];
            dn = desc(gn);
        }
        floatx16 acc[FT];
#pragma unroll
        for (int t = 0; t < FT; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        const bool wave_live = d.s0 + 32 * wv < a.S;
        for (int kb = g.k0; kb < g.k1; kb += FBK) {  // uniform
            __syncthreads();  // previous stage's MFMAs done with the LDS
            stage(d, kb);
            __syncthreads();
            if (si == sbeg && kb == g.k0) mark(1);
            ++nst;
            {
                const bool inseg = kb + FBK < g.k1;
                if (inseg || more) fetch(inseg ? d : dn, inseg ? kb + FBK : gn.k0);
            }
            if (wave_live) {
                // k permutation: per 8 columns, lane half h feeds k = kk + 4h + j to
                // MFMA j (j = 0..3) for BOTH operands -- the same sum over k
                const float* Ea = Es + (32 * wv + l32) * FLD + 4 * h;
                const float* Lb = Ls + l32 * FLD + 4 * h;
#pragma unroll
                for (int kk = 0; kk < FBK; kk += 8) {
                    const float4 av = *reinterpret_cast<const float4*>(Ea + kk);
                    float4 bv[FT];
#pragma unroll
                    for (int t = 0; t < FT; ++t) bv[t] = *reinterpret_cast<const float4*>(Lb + 32 * t * FLD + kk);
#pragma unroll
                    for (int t = 0; t < FT; ++t) {
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[t].x, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[t].y, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[t].z, acc[t], 0, 0, 0);
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[t].w, acc[t], 0, 0, 0);
                    }
                }
            }
        }
        mark(2);
        // the accumulators in fragment order ((wave FT + t) 16 + q) 64 + lane: every
        // store a contiguous 256-byte wave run (the reduce reads the order back)
        if (wave_live) {
            float* slot = a.part + (size_t)g.slot * FST * kFwdRows + (size_t)wv * FT * 16 * 64 + lane;
#pragma unroll
            for (int t = 0; t < FT; ++t)
#pragma unroll
                for (int q = 0; q < 16; ++q) slot[(t * 16 + q) * 64] = acc[t][q];
        }
        mark(3);
    }
    if (dgn && threadIdx.x == 0) {
        unsigned long long* o = a.stamps + (size_t)blockIdx.x * 16;
        o[0] = t_start;
        for (int q = 1; q < 4; ++q) o[q] = ph[q];
        o[6] = (unsigned long long)nst;
        o[12] = __builtin_amdgcn_s_memtime();
        o[13] = rt_start;
        o[14] = __builtin_amdgcn_s_memrealtime();
    }
}


int g_fwd_ablation = 0;                      // psvi_debug_set(PSVI_DBG_FWD_ABLATION, mask)
unsigned long long* g_fwd_stamps = nullptr;  // psvi_debug_set_ptr(PSVI_DBG_FWD_STAMPS, buf)

// ---------------------------------------------------------------- backward
constexpr int UB = 64;    // band rows = c-block columns
constexpr int USB = 128;  // samples staged per pass (K of the dL GEMM)
constexpr int ULD = 68;   // LDS row stride: 16-byte aligned rows for float4 stores

struct UpdArgs {
    const UpdChunk* chunks;
    const float* eps;
    const float* g;    // g_shard [S][ldg]
    int ldg, S;
    int64_t g_total, e_total;  // floats in g_shard / eps (load guards)
    float* params;
    float* m;
    float* v;
    float* grad_out;   // GRAD mode output
    const float* kl_vec;  // GRAD mode, nullable: + kl_vec / s0^2 on the corr entries (the
                          // KL Hessian's corr block in an HVP: kl_vec = the direction)
    double* kl_out;    // nullable
    int64_t pcount;    // parameter vector length
    int include_kl;
    int abl;                       // diagnostics ablation mask (0 in production)
    unsigned long long* stamps;    // diagnostics: 16 slots per workgroup (nullptr in production)
    float inv_s0sq, log_s0;
    AdamC adam;
    // fused next-step sample (FUSE kernels): partial x_next per chunk slot
    const float* eps_next;
    float* part;
    // tiled corr / m / v (TILED kernels)
    float* tp;
    float* tm;
    float* tv;
    MvnLayerArgs lay[kMaxL];
};

// Branch-free 16-byte loads.  gfx950 global loads need only 4-byte
// alignment, so a float4 may start at any float offset; the offset is clamped
// into the buffer [lo, hi) (hi - lo >= 4) so the load is unconditional (loads
// under divergent branches make the compiler's vmcnt bookkeeping fall back to
// vmcnt(0), which would drain every prefetch), and fix4 -- applied where the
// value is consumed -- shifts the clamped vector back, zeroing elements
// outside [lo, hi).  Offsets are 32-bit (the plan rejects larger buffers).
__device__ __forceinline__ int clamp4(int off, int lo, int hi) {
    return off < lo ? lo : (off > hi - 4 ? hi - 4 : off);
}
__device__ __forceinline__ float4 ld4u(const float* base, int off, int lo, int hi) {
    return *reinterpret_cast<const float4*>(base + clamp4(off, lo, hi));
}
__device__ __forceinline__ float4 fix4(float4 v, int off, int lo, int hi) {
    const int d = off - clamp4(off, lo, hi);
    if (d == 0) return v;  // VALU-only branch
    const float x[4] = {v.x, v.y, v.z, v.w};
    float r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = i + d;
        r[i] = k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : k == 3 ? x[3] : 0.f;
    }
    return make_float4(r[0], r[1], r[2], r[3]);
}
__device__ __forceinline__ float f4get(const float4& v, int i) {
    return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

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

#define UPD_STAMP(k, val)                                                          \
    do {                                                                           \
        if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 16 + (k)] = (val); \
    } while (0)

// One chunk: for each of its c-blocks, dL^T[c][r] = sum_s eps[s][c] G[s][r]
// (v_mfma_f32_32x32x2_f32, 4 waves = 2 x 2 sub-tiles of 32 x 32), then
//   corr <- Adam(corr, dL + corr/s0^2)         (or grad_out in GRAD mode).
// The accumulator tile goes through LDS (into the eps stage, free after the
// MFMAs) so the corr / m / v / grad traffic moves in 256-byte row runs, four
// rows per wave instruction.
// Pipeline: after each staging barrier the next step's operand loads (eps,
// and G when S > 128; clamped to the last step rather than skipped) and, on a
// c-block's last sample pass, its corr/m/v loads are issued; the MFMAs run
// while they land.  Every global load is unconditional: a load under a
// branch makes the compiler's vmcnt bookkeeping fall back to vmcnt(0).
// The diagonal c-block (columns = the band's rows) also yields sum_s G and
// sum_s G*eps per row: the mean / sd update.
constexpr int TLD = 68;   // LDS stride of the transposed accumulator tile
// S <= 128: G resident (all samples), eps staged in halves of UEH samples
// (52 KB of LDS: three workgroups per CU); S > 128: both staged per pass.
constexpr int UEH = 64;
template <bool MULTI>
struct UpdShared {
    float Gs[USB * ULD];
    float Es[(MULTI ? USB : UEH) * ULD];
    float red[2 * 4 * 64];
};

// MODE: 0 = S <= 64 (one eps half), 1 = S <= 128 (two halves), 2 = S > 128.
// FUSE (Adam, MODE < 2): also the next step's sample from the updated L --
// per c-block, x_next[s][r] += sum_c eps_next[s][c] L_new[r][c] on a second
// MFMA GEMM (L_new tile through the LDS tile region, eps_next fragments
// straight from L2 into registers), partial sums to the chunk's slot.
// PKO (tiled state, no fused sample: an inner loop's last step): corr / m / v
// read from the tiled state, written back to the packed arrays
template <bool GRAD, int MODE, bool FUSE, bool TILED, bool PKO = false>
__device__ __forceinline__ void upd_chunk(const UpdArgs& a, const UpdChunk& ch,
                                          UpdShared<MODE == 2>& sh) {
    constexpr bool MULTI = MODE == 2, TWOH = MODE == 1;
    static_assert(!FUSE || (!GRAD && !MULTI), "fused sample: Adam mode, S <= 128");
    static_assert(!TILED || (!GRAD && !MULTI), "tiled state: Adam mode, S <= 128");
    float* Gs = sh.Gs;
    float* Es = sh.Es;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int wr = wv >> 1, wc = wv & 1;
    const int n = a.lay[ch.layer].n;
    const int eoff = (int)a.lay[ch.layer].eoff;
    const float* E = a.eps + eoff;  // [S][n]; the whole eps buffer is [-eoff, e_rem)
    const int e_rem = (int)a.e_total - eoff;
    const int g_total = (int)a.g_total, pcount = (int)a.pcount;
    const int poff = (int)a.lay[ch.layer].poff, corr_off = poff + 2 * n;
    const int np = MULTI ? (a.S + USB - 1) / USB : 1;
    const int nt = ch.k1 - ch.k0;
    const int kd = ch.diag ? ch.r0 / UB - ch.k0 : -1;  // diagonal c-block index in the chunk

    // staging / epilogue map: 16 lanes x float4 = one 64-column row, rows srow + 16 j
    const int col4 = tid & 15, srow = tid >> 4;
    const int gcol = ch.xcol + ch.r0 + 4 * col4;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 greg[8], ereg[8];
    // sample row s is clamped to S-1 (rows >= S are zeroed at the LDS write)
    // (ablation 1: every G / eps load from one cached address)
    const int ab1 = (a.abl & 1) ? 0 : 1;
    auto goff = [&](int s) { return ab1 * (min(s, a.S - 1) * a.ldg + gcol); };
    auto eofs = [&](int s, int ti) {
        return ab1 * (min(s, a.S - 1) * n + (ch.k0 + ti) * UB + 4 * col4);
    };
    auto load_G = [&](int pi) {
#pragma unroll
        for (int j = 0; j < 8; ++j) greg[j] = ld4u(a.g, goff(pi * USB + srow + 16 * j), 0, g_total);
    };
    auto load_E = [&](int ti, int pi) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            ereg[j] = ld4u(E, eofs(pi * USB + srow + 16 * j, ti), -eoff, e_rem);
    };
    auto stage = [&](bool withG, int ti, int pi) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int o = (srow + 16 * j) * ULD + 4 * col4;
            const int sr = pi * USB + srow + 16 * j;
            const bool live = sr < a.S && !(a.abl & 1);
            if (withG)
                *reinterpret_cast<float4*>(&Gs[o]) = live ? fix4(greg[j], goff(sr), 0, g_total) : z4;
            *reinterpret_cast<float4*>(&Es[o]) =
                live ? fix4(ereg[j], eofs(sr, ti), -eoff, e_rem) : z4;
        }
    };

    // S <= 128: eps halves of UEH samples (4 float4 per thread)
    float4 ehreg[4];
    auto load_Eh = [&](int ti, int hh) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            ehreg[j] = ld4u(E, eofs(hh * UEH + srow + 16 * j, ti), -eoff, e_rem);
    };
    auto stage_Eh = [&](int ti, int hh) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int sr = hh * UEH + srow + 16 * j;
            const bool live = sr < a.S && !(a.abl & 1);
            *reinterpret_cast<float4*>(&Es[(srow + 16 * j) * ULD + 4 * col4]) =
                live ? fix4(ehreg[j], eofs(sr, ti), -eoff, e_rem) : z4;
        }
    };

    // epilogue rows: r_j = r0 + srow + 16 j, columns c0 + 4 col4 + (0..3)
    int rowp[4];
    bool rown[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int r = ch.r0 + srow + 16 * j;
        rown[j] = r >= ch.rlo && r < ch.rhi && r >= 1 && r <= n - 2;
        rowp[j] = corr_off + (int)((int64_t)r * (r - 1) / 2);
    }
    float4 pq[4], mq[4], vq[4];
    // tiled state: this lane's 4 fragment float4s of a tile (contiguous per wave)
    auto tile_off = [&](int ti, int g) {
        return tile_index(a.lay[ch.layer], ch.r0 / UB, ch.k0 + ti) * 4096 +
               (int64_t)((wv * 4 + g) * 64 + lane) * 4;
    };
    const int64_t ab4 = (a.abl & 4) ? 0 : 1;  // ablation 4: corr/m/v loads from one address
    auto load_pmv = [&](int ti) {
        if (TILED) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t o = ab4 * tile_off(ti, g);
                pq[g] = *reinterpret_cast<const float4*>(a.tp + o);
                mq[g] = *reinterpret_cast<const float4*>(a.tm + o);
                vq[g] = *reinterpret_cast<const float4*>(a.tv + o);
            }
            return;
        }
        const int cl = (ch.k0 + ti) * UB + 4 * col4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // rows off the band's corr rows load something valid, never stored
            pq[j] = ld4u(a.params, rowp[j] + cl, 0, pcount);
            if (!GRAD) {
                mq[j] = ld4u(a.m, rowp[j] + cl, 0, pcount);
                vq[j] = ld4u(a.v, rowp[j] + cl, 0, pcount);
            }
        }
    };

    floatx16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    float dgm = 0.f, dgs = 0.f, klp = 0.f;

    // ---- fused next-step sample state
    floatx16 acc2[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc2[t][q] = 0.f;
    float4 enreg[FUSE ? 8 : 1];
    const bool wave_s = 32 * wv < a.S;  // this wave owns samples of the fused GEMM
    const int es = min(32 * wv + l32, a.S - 1);
    const int ab32 = (a.abl & 32) ? 0 : 1;  // ablation 32: eps_next loads from one address
    auto enofs = [&](int ti, int g) { return ab32 * (es * n + (ch.k0 + ti) * UB + 8 * g + 4 * h); };
    auto load_En = [&](int ti) {
        if (FUSE) {
#pragma unroll
            for (int g = 0; g < 8; ++g) enreg[g] = ld4u(a.eps_next + eoff, enofs(ti, g), -eoff, e_rem);
        }
    };
    // x_next partial over one c-block: A = eps_next[s][c] (registers, k-permuted:
    // lane half h holds c = 8g + 4h + j for MFMA j), B = L_new[r][c] from the tile
    auto gemm2 = [&](int ti) {
        if (FUSE && wave_s && !(a.abl & 16)) {
            const float* Lb = Es + l32 * TLD + 4 * h;
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const float4 av = fix4(enreg[g], enofs(ti, g), -eoff, e_rem);
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const float4 bv = *reinterpret_cast<const float4*>(Lb + 32 * t * TLD + 8 * g);
                    acc2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc2[t], 0, 0, 0);
                    acc2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc2[t], 0, 0, 0);
                    acc2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc2[t], 0, 0, 0);
                    acc2[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc2[t], 0, 0, 0);
                }
            }
        }
    };

    auto compute = [&](int ti, int pi) {
        const int kend = (a.abl & 2) ? 0 : min(USB, a.S - pi * USB);
        if (ti == kd) {
            // diagonal c-block: column j of Es is row r0 + j of the band
            for (int s = 32 * wv; s < 32 * wv + 32 && s < kend; ++s) {
                const float gv = Gs[s * ULD + lane];
                dgm += gv;
                dgs = fmaf(gv, Es[s * ULD + lane], dgs);
            }
        }
        // 16 samples per group (rows past S are staged as zeros up to USB)
        const float* Ea = Es + h * ULD + 32 * wc + l32;
        const float* Gb = Gs + h * ULD + 32 * wr + l32;
        for (int kk = 0; kk < kend; kk += 16) {
            float av[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                av[u] = Ea[(kk + 2 * u) * ULD];
                bv[u] = Gb[(kk + 2 * u) * ULD];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
        }
    };

    // one eps half against the resident G (rows hh*UEH ..)
    auto compute_h = [&](int ti, int hh) {
        const int kend = (a.abl & 2) ? 0 : min(UEH, a.S - hh * UEH);
        if (ti == kd) {
            for (int s = 16 * wv; s < 16 * wv + 16 && s < kend; ++s) {
                const float gv = Gs[(hh * UEH + s) * ULD + lane];
                dgm += gv;
                dgs = fmaf(gv, Es[s * ULD + lane], dgs);
            }
        }
        const float* Ea = Es + h * ULD + 32 * wc + l32;
        const float* Gb = Gs + (hh * UEH + h) * ULD + 32 * wr + l32;
        for (int kk = 0; kk < kend; kk += 16) {
            float av[8], bv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                av[u] = Ea[(kk + 2 * u) * ULD];
                bv[u] = Gb[(kk + 2 * u) * ULD];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
        }
    };

    // call after a barrier that ends every wave's reads of Es
    auto epilogue = [&](int ti) {
        if (TILED) {
            // D[i = c][j = r] (j = lane & 31, i = (q&3) + 8(q>>2) + 4h) is already the
            // tile's fragment order: Adam on the accumulators, float4 in / out
            static_assert(!PKO || !FUSE, "packed-out: the last step samples nothing");
            const int r = ch.r0 + 32 * wr + l32;
            const bool rv = r >= 1 && r <= n - 2 && !(a.abl & 8);
            float kp[PKO ? 16 : 1], km[PKO ? 16 : 1], kv[PKO ? 16 : 1];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int cb = (ch.k0 + ti) * UB + 32 * wc + 8 * g + 4 * h;
                const int64_t o = tile_off(ti, g);
                float pn[4], mn[4], vn[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    // entries outside the strict lower part stay exactly 0: zero
                    // gradient, zero state (both Adam variants keep p = 0)
                    const float p = f4get(pq[g], i);
                    klp += p * p;
                    const bool ok = rv && cb + i < r;
                    const float gval = ok ? (a.include_kl ? acc[4 * g + i] + p * a.inv_s0sq
                                                          : acc[4 * g + i])
                                          : 0.f;
                    float mm = f4get(mq[g], i), vv = f4get(vq[g], i);
                    pn[i] = (a.abl & 64) ? p + gval + mm + vv
                                         : adam_apply_fast(a.adam, p, gval, mm, vv);
                    mn[i] = mm;
                    vn[i] = vv;
                }
                if (PKO) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        kp[4 * g + i] = pn[i];
                        km[4 * g + i] = mn[i];
                        kv[4 * g + i] = vn[i];
                    }
                } else if (!(a.abl & 8)) {
                    // write-through (sc1): the state leaves the XCD's L2, which keeps
                    // the eps / G blocks other chunks re-read (as the stream kernel)
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    const rsrc_t rs_t = make_rsrc(a.tp, 0x7fffffff);
                    const int tmb = __builtin_amdgcn_readfirstlane((int)((a.tm - a.tp) * 4));
                    const int tvb = __builtin_amdgcn_readfirstlane((int)((a.tv - a.tp) * 4));
                    const uint32_t ob = (uint32_t)(o * 4);
                    BSTORE128(
                        __builtin_bit_cast(u32x4, make_float4(pn[0], pn[1], pn[2], pn[3])), rs_t, ob, 0, 16);
                    BSTORE128(
                        __builtin_bit_cast(u32x4, make_float4(mn[0], mn[1], mn[2], mn[3])), rs_t, ob, tmb, 16);
                    BSTORE128(
                        __builtin_bit_cast(u32x4, make_float4(vn[0], vn[1], vn[2], vn[3])), rs_t, ob, tvb, 16);
                }
                if (FUSE)  // L_new fragment -> the [r][c] tile for the sample GEMM
                    *reinterpret_cast<float4*>(&Es[(32 * wr + l32) * TLD + 32 * wc + 8 * g + 4 * h]) =
                        make_float4(pn[0], pn[1], pn[2], pn[3]);
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.f;
            if (PKO) {
                // fragment -> [r][c] through LDS, then the rows' float4 segments
                // to the packed triangle (as the packed epilogue below)
                float* T = Es;
                const int cb = (ch.k0 + ti) * UB + 4 * col4;
#pragma unroll
                for (int ai = 0; ai < 3; ++ai) {
                    const float* kk = ai == 0 ? kp : ai == 1 ? km : kv;
                    float* dst = ai == 0 ? a.params : ai == 1 ? a.m : a.v;
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        *reinterpret_cast<float4*>(&T[(32 * wr + l32) * TLD + 32 * wc + 8 * g + 4 * h]) =
                            make_float4(kk[4 * g], kk[4 * g + 1], kk[4 * g + 2], kk[4 * g + 3]);
                    __syncthreads();
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int rr = ch.r0 + srow + 16 * j;
                        if (!rown[j] || cb >= rr) continue;
                        const int o = rowp[j] + cb;
                        const float4 d4 = *reinterpret_cast<const float4*>(&T[(srow + 16 * j) * TLD + 4 * col4]);
                        if (cb + 3 < rr) {
                            *reinterpret_cast<float4*>(dst + o) = d4;
                        } else {
#pragma unroll
                            for (int i = 0; i < 3; ++i)
                                if (cb + i < rr) dst[o + i] = f4get(d4, i);
                        }
                    }
                    __syncthreads();
                }
            }
            return;
        }
        // D[i = c][j = r]: j = lane & 31, i = (q & 3) + 8 (q >> 2) + 4 h  ->  T[r][c] in Es
        float* T = Es;
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(&T[(32 * wr + l32) * TLD + 32 * wc + 8 * g + 4 * h]) =
                make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        __syncthreads();
        const int cb = (ch.k0 + ti) * UB + 4 * col4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = ch.r0 + srow + 16 * j;
            if (!rown[j] || cb >= r || (a.abl & 8)) {
                if (FUSE)  // no L entries here: zeros for the fused sample GEMM
                    *reinterpret_cast<float4*>(&T[(srow + 16 * j) * TLD + 4 * col4]) = z4;
                continue;
            }
            const int o = rowp[j] + cb;
            const float4 d4 = *reinterpret_cast<const float4*>(&T[(srow + 16 * j) * TLD + 4 * col4]);
            const float4 p4 = (a.abl & 4) ? z4 : fix4(pq[j], o, 0, pcount);
            const float4 kv4 = (GRAD && a.kl_vec) ? fix4(ld4u(a.kl_vec, o, 0, pcount), o, 0, pcount) : z4;
            float4 m4 = z4, v4 = z4;
            if (!GRAD) {
                m4 = (a.abl & 4) ? z4 : fix4(mq[j], o, 0, pcount);
                v4 = (a.abl & 4) ? z4 : fix4(vq[j], o, 0, pcount);
            }
            float pn[4], mn[4], vn[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = f4get(p4, i);
                klp += cb + i < r ? p * p : 0.f;
                float gval = a.include_kl ? f4get(d4, i) + p * a.inv_s0sq : f4get(d4, i);
                if (GRAD && a.kl_vec) gval += f4get(kv4, i) * a.inv_s0sq;
                if (GRAD) {
                    pn[i] = gval;
                } else {
                    float mm = f4get(m4, i), vv = f4get(v4, i);
                    pn[i] = adam_apply_fast(a.adam, p, gval, mm, vv);
                    mn[i] = mm;
                    vn[i] = vv;
                }
            }
            float* dp = GRAD ? a.grad_out : a.params;
            if (FUSE) {  // L_new row segment (strict lower part only)
                float4 lv;
                lv.x = cb + 0 < r ? pn[0] : 0.f;
                lv.y = cb + 1 < r ? pn[1] : 0.f;
                lv.z = cb + 2 < r ? pn[2] : 0.f;
                lv.w = cb + 3 < r ? pn[3] : 0.f;
                *reinterpret_cast<float4*>(&T[(srow + 16 * j) * TLD + 4 * col4]) = lv;
            }
            if (cb + 3 < r) {
                *reinterpret_cast<float4*>(dp + o) = make_float4(pn[0], pn[1], pn[2], pn[3]);
                if (!GRAD) {
                    *reinterpret_cast<float4*>(a.m + o) = make_float4(mn[0], mn[1], mn[2], mn[3]);
                    *reinterpret_cast<float4*>(a.v + o) = make_float4(vn[0], vn[1], vn[2], vn[3]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    if (cb + i < r) {
                        dp[o + i] = pn[i];
                        if (!GRAD) {
                            a.m[o + i] = mn[i];
                            a.v[o + i] = vn[i];
                        }
                    }
                }
            }
        }
    };

    if (!MULTI) {
        // all samples in one pass: the band's G slice stays in LDS, eps
        // comes in halves.  Loads are issued in the order they are consumed
        // (vmcnt retires in order): second eps half, this c-block's corr/m/v,
        // next c-block's first eps half -- the corr/m/v get both MFMA halves
        // to land.
        load_G(0);
        load_Eh(0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // G slice once (its registers die here)
            const int sr = srow + 16 * j;
            *reinterpret_cast<float4*>(&Gs[sr * ULD + 4 * col4]) =
                sr < a.S && !(a.abl & 1) ? fix4(greg[j], goff(sr), 0, g_total) : z4;
        }
        // diagnostics: shader-clock time per loop phase, summed over c-blocks
        // (slots 6..11: stage 1, MFMA half 1, stage 2, MFMA half 2, epilogue, gemm2)
        unsigned long long tph[6] = {0, 0, 0, 0, 0, 0}, tlast = 0;
        auto ph = [&](int k) {
            if (a.stamps && tid == 0) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                if (k >= 0) tph[k] += t - tlast;
                tlast = t;
            }
        };
        ph(-1);
        for (int ti = 0; ti < nt; ++ti) {
            stage_Eh(ti, 0);
            __syncthreads();
            if (ti == 0) UPD_STAMP(1, __builtin_amdgcn_s_memtime());
            ph(0);
            if (TWOH) {
                load_Eh(ti, 1);
                load_pmv(ti);
                load_En(ti);
                compute_h(ti, 0);
                __syncthreads();
                ph(1);
                stage_Eh(ti, 1);
                __syncthreads();
                ph(2);
                load_Eh(min(ti + 1, nt - 1), 0);
                compute_h(ti, 1);
            } else {
                load_pmv(ti);
                load_En(ti);
                load_Eh(min(ti + 1, nt - 1), 0);
                compute_h(ti, 0);
            }
            __syncthreads();  // every wave done with Es: it takes the accumulator tile
            ph(3);
            epilogue(ti);
            if (FUSE) {
                __syncthreads();  // L_new tile complete
                ph(4);
                gemm2(ti);
            }
            __syncthreads();  // tile read before the next staging overwrites Es
            ph(FUSE ? 5 : 4);
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) UPD_STAMP(6 + k, tph[k]);
    } else {
        load_G(0);
        load_E(0, 0);
        for (int ti = 0; ti < nt; ++ti) {
            for (int pi = 0; pi < np - 1; ++pi) {
                stage(true, ti, pi);
                __syncthreads();
                load_G(pi + 1);
                load_E(ti, pi + 1);
                compute(ti, pi);
                __syncthreads();
            }
            stage(true, ti, np - 1);
            __syncthreads();
            load_G(0);
            load_E(min(ti + 1, nt - 1), 0);
            load_pmv(ti);
            compute(ti, np - 1);
            __syncthreads();
            epilogue(ti);
            __syncthreads();
        }
    }
    UPD_STAMP(2, __builtin_amdgcn_s_memtime());
    if (FUSE && wave_s && ch.slot >= 0) {
        // D2[i = s][j = r]: j = lane & 31, i = (q & 3) + 8 (q >> 2) + 4 h
        float* slot = a.part + (size_t)ch.slot * a.S * 64 + l32;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int s = 32 * wv + (q & 3) + 8 * (q >> 2) + 4 * h;
                if (s < a.S) slot[(size_t)s * 64 + 32 * t] = acc2[t][q];
            }
    }
    klp *= 0.5f * a.inv_s0sq;
    if (ch.diag) {
        sh.red[wv * 64 + lane] = dgm;
        sh.red[256 + wv * 64 + lane] = dgs;
        __syncthreads();
        const int rr = ch.r0 + tid;
        if (tid < 64 && rr >= ch.rlo && rr < ch.rhi && rr < n) {
            const float* red = sh.red;
            const float gm = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];
            const float gs = red[256 + tid] + red[320 + tid] + red[384 + tid] + red[448 + tid];
            const int pm = poff + rr, ps = pm + n;
            const float mu = a.params[pm], sdr = a.params[ps];
            const float sp = softplus_f(sdr), sg = sigmoid_f(sdr);
            float gmean = gm, gsd = gs * sg;
            if (a.include_kl) {
                gmean += mu * a.inv_s0sq;
                gsd += (sp * a.inv_s0sq - 1.f / sp) * sg;
                klp += a.log_s0 - logf(sp) + 0.5f * ((sp * sp + mu * mu) * a.inv_s0sq - 1.f);
            }
            upd_elem<GRAD>(a, pm, gmean);
            upd_elem<GRAD>(a, ps, gsd);
        }
        __syncthreads();
    }
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, sh.red);
        if (tid == 0) atomicAdd(a.kl_out, (double)tot);
    }
}

template <bool GRAD, int MODE, bool FUSE = false, bool TILED = false, bool PKO = false>
__global__ __launch_bounds__(256, MODE == 2 || FUSE ? 2 : 3) void mvn_update_kernel(UpdArgs a) {
    __shared__ __attribute__((aligned(16))) UpdShared<MODE == 2> sh;
    UPD_STAMP(0, __builtin_amdgcn_s_memtime());
    UPD_STAMP(12, __builtin_amdgcn_s_memrealtime());  // chip-wide 100 MHz clock
    UPD_STAMP(4, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4));
    UPD_STAMP(5, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20));
    const UpdChunk ch = a.chunks[blockIdx.x];
    if (ch.k1 > ch.k0) upd_chunk<GRAD, MODE, FUSE, TILED, PKO>(a, ch, sh);  // XCD padding chunks are empty
    UPD_STAMP(3, __builtin_amdgcn_s_memtime());
    UPD_STAMP(13, __builtin_amdgcn_s_memrealtime());
}

// ------------------------------------------------ K-split streaming update
// The full-cov Adam update at K = S > 128 (every rank of the row-sharded step,
// where a rank's rows take all S samples; C4 on one GPU): the rank's 64 x 64
// tiles with their K cut in 128-sample passes, units (tile, pass) dealt as
// equal contiguous runs to persistent workgroups (two per CU; build_kstream).
// Per pass: the band's G rows and the tile's eps column block staged into LDS
// (register prefetch of the next pass during the MFMAs), dL^T[c][r] +=
// sum_s eps[s][c] G[s][r] on v_mfma_f32_32x32x2_f32 (4 waves = 2 x 2 of 32 x
// 32), the diagonal tile also sum_s G and sum_s G eps per row.  A tile whose
// passes all sit in one run goes straight to the Adam epilogue (the chunked
// kernel's packed epilogue: accumulators transposed through LDS, corr / m / v
// as 256-byte row runs).  A split tile's contributors write their partials to
// their slots with write-through (sc1) stores, drain them (vmcnt 0), and one
// lane adds to the tile's counter (relaxed, agent scope); the contributor that
// draws the last ticket reads every partial with sc1 loads, adds them in pass
// order (the result does not depend on who arrives last) and runs the
// epilogue -- the in-launch split-K combine of cdna_hip_programming.md (§6
// Guideline 16, counter form), correct for any placement of the contributors.
// No workgroup ever waits on another: the kernel cannot hang on the hand-off.
// The ticket stays relaxed on purpose: sc1 stores + the vmcnt(0) drain before
// the add is the first row of MI355X_MICROARCH.md's hand-off table (release by
// drain, acquire by sc1 loads); an acq_rel atomic would add an L2 writeback /
// invalidate per contributor (1.7 - 3.5 us per launch at C4 W = 8) for no
// ordering the drain does not give.  The last arriver resets the counter in
// the same launch; an aborted launch ends the process, so no half-counted
// ticket reaches a later launch.
struct KsArgs {
    const KsTile* tiles;
    const KsSeg* segs;
    const int* seg_off;
    float* slots;
    int* cnt;
    int64_t slot_bytes;
    const float* eps;
    const float* g;
    int ldg, S;
    int64_t g_total, e_total;
    float* params;
    float* m;
    float* v;
    double* kl_out;
    int64_t pcount;
    int include_kl;
    float inv_s0sq, log_s0;
    AdamC adam;
    unsigned long long* stamps;  // diagnostics: 16 slots per workgroup (nullptr in production)
    MvnLayerArgs lay[kMaxL];
    // GRAD: the reparameterised gradient into grad_out instead of Adam (the
    // HVP's J^T G_dot), + kl_vec / s0^2 on the corr entries when kl_vec is set
    float* grad_out;
    const float* kl_vec;
    const float* g2;  // GRAD: a second G slot added at staging (slot 0 + slot 1, as slot_sum_kernel)
};

// G / eps / corr / m / v through buffer loads whose per-dword range check
// returns 0 past the end (rows past S are sent to offset kOOB): no clamped
// addresses, fix-ups or zero selects at staging.  The first pass of the next
// segment is loaded behind the last pass of this one (its latency overlaps the
// hand-off and the epilogue).
// BF: the dL GEMM on bf16 pieces (fp32-faithful, mvn_stream_bf2_kernel's
// products): a pass's G and eps blocks are split at staging into three bf16
// planes each, in two halves of 64 samples (column images of 8 KB per plane,
// read with ds_read_b64_tr_b16; 48 KB of LDS, two workgroups per CU), each
// half's next loads issued as soon as it is staged.  The diagonal tile's row
// sums come from the planes (their sum is the fp32 value exactly).
constexpr int kKsBfImg = 64 * 128;  // bytes per plane image (64 samples x 64 columns)
struct KsBfShared {
    uint8_t img[6 * kKsBfImg];  // eps planes, then G planes; the epilogue's T tile after the passes
    float red[2 * 4 * 64];
};
template <bool BF, bool GRAD = false>
__global__ __launch_bounds__(256, 2) void mvn_kstream_kernel(KsArgs a) {
    __shared__ __attribute__((aligned(16))) std::conditional_t<BF, KsBfShared, UpdShared<true>> sh;
    static_assert(kKsPass == USB, "one LDS stage per pass");
    static_assert(64 * TLD * 4 <= 6 * kKsBfImg, "the epilogue tile fits the images");
    float* Gs = nullptr;
    float* Es = nullptr;
    if constexpr (!BF) {
        Gs = sh.Gs;
        Es = sh.Es;
    }
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int wr = wv >> 1, wc = wv & 1;
    const int col4 = tid & 15, srow = tid >> 4;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const rsrc_t rs = make_rsrc(a.slots, a.slot_bytes);
    const rsrc_t rg = make_rsrc(a.g, 4 * a.g_total), re = make_rsrc(a.eps, 4 * a.e_total);
    const rsrc_t rg2 = make_rsrc(a.g2, GRAD && a.g2 ? 4 * a.g_total : 0);
    // GRAD: m reads kl_vec (0 when none: an empty range), v is not read
    const rsrc_t rpar = make_rsrc(a.params, 4 * a.pcount),
                 rm = make_rsrc(GRAD ? a.kl_vec : a.m, GRAD && !a.kl_vec ? 0 : 4 * a.pcount),
                 rv = make_rsrc(a.v, 4 * a.pcount);
    float klp = 0.f;
    // diagnostics (a.stamps): shader clocks per phase summed over the segments
    // -- 1 first-pass load wait, 2 passes (MFMAs + later loads), 3 hand-off,
    // 4 partial sums, 5 epilogue; 6 segments, 7 combines; 0 / 12 start / end,
    // 13 / 14 the 100 MHz clock at start / end
    const bool dg = a.stamps != nullptr;
    unsigned long long ph[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
    unsigned long long tprev = dg ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long t_start = tprev, rt_start = dg ? __builtin_amdgcn_s_memrealtime() : 0ull;
    int ncomb = 0;
    auto mark = [&](int k) __attribute__((always_inline)) {
        if (dg) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            ph[k] += t - tprev;
            tprev = t;
        }
    };
    // a segment's pass operands: G columns gcol.., eps [S][n] at eoff, columns ecol..
    struct Ld {
        int gcol, eoff, n, ecol;
    };
    auto desc = [&](const KsTile& t) __attribute__((always_inline)) {
        Ld d;
        d.n = a.lay[0].n;
        d.eoff = (int)a.lay[0].eoff;
#pragma unroll
        for (int l = 1; l < kMaxL; ++l)  // select: a dynamic index into the arguments goes to scratch
            if (t.layer == l) {
                d.n = a.lay[l].n;
                d.eoff = (int)a.lay[l].eoff;
            }
        d.gcol = t.xcol + t.r0 + 4 * col4;
        d.ecol = t.k * UB + 4 * col4;
        return d;
    };
    float4 greg[8], ereg[8], greg2[GRAD ? 8 : 1];
    auto load = [&](const Ld& d, int pi) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int s = pi * USB + srow + 16 * j;
            const bool live = s < a.S;
            const uint32_t go = live ? (uint32_t)(s * a.ldg + d.gcol) * 4u : kOOB;
            const uint32_t eo = live ? (uint32_t)(d.eoff + s * d.n + d.ecol) * 4u : kOOB;
            greg[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rg, go, 0, 0));
            ereg[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(re, eo, 0, 0));
        }
    };
    auto stage = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int o = (srow + 16 * j) * ULD + 4 * col4;
            *reinterpret_cast<float4*>(&Gs[o]) = greg[j];
            *reinterpret_cast<float4*>(&Es[o]) = ereg[j];
        }
    };
    // BF: half hp of a pass (samples 64 hp + srow + 16 j', registers j = 4 hp + j')
    uint8_t* const Eb = BF ? reinterpret_cast<uint8_t*>(&sh) : nullptr;
    uint8_t* const Gb = BF ? reinterpret_cast<uint8_t*>(&sh) + 3 * kKsBfImg : nullptr;
    auto load_half = [&](const Ld& d, int pi, int hp) __attribute__((always_inline)) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * hp + jj;
            const int s = pi * USB + srow + 16 * j;
            const bool live = s < a.S;
            const uint32_t go = live ? (uint32_t)(s * a.ldg + d.gcol) * 4u : kOOB;
            const uint32_t eo = live ? (uint32_t)(d.eoff + s * d.n + d.ecol) * 4u : kOOB;
            greg[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rg, go, 0, 0));
            ereg[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(re, eo, 0, 0));
            if (GRAD) greg2[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rg2, go, 0, 0));
        }
    };
    auto stage_half = [&](int hp) __attribute__((always_inline)) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = 4 * hp + jj, sl = srow + 16 * jj;
            if (GRAD && a.g2) {
                greg[j].x += greg2[j].x;
                greg[j].y += greg2[j].y;
                greg[j].z += greg2[j].z;
                greg[j].w += greg2[j].w;
            }
            uint32_t x[3][2], y[3][2];
            split3_pk(f32x2{greg[j].x, greg[j].y}, x[0][0], x[1][0], x[2][0]);
            split3_pk(f32x2{greg[j].z, greg[j].w}, x[0][1], x[1][1], x[2][1]);
            split3_pk(f32x2{ereg[j].x, ereg[j].y}, y[0][0], y[1][0], y[2][0]);
            split3_pk(f32x2{ereg[j].z, ereg[j].w}, y[0][1], y[1][1], y[2][1]);
            const int o = img_col(sl, 4 * col4);
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                *reinterpret_cast<u32x2*>(Gb + p * kKsBfImg + o) = u32x2{x[p][0], x[p][1]};
                *reinterpret_cast<u32x2*>(Eb + p * kKsBfImg + o) = u32x2{y[p][0], y[p][1]};
            }
        }
    };
    // the transposed reads (mvn_stream_bf2_kernel's): lane 4 qq + pp of its
    // 16-lane group takes sample row qq, columns 4 pp .. + 3 of its 16
    const int g16 = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const uint8_t* const rda = BF ? Eb + img_col(8 * h + qq, 32 * wc + 16 * (g16 & 1) + 4 * pp) : nullptr;
    const uint8_t* const rdb = BF ? Gb + img_col(8 * h + qq, 32 * wr + 16 * (g16 & 1) + 4 * pp) : nullptr;
    auto read_ab = [&](int t, bf8v (&av)[3], bf8v (&bv)[3]) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            typedef __attribute__((address_space(3))) s4v* lds_s4;
            const int o = p * kKsBfImg + 2048 * t;  // sample rows 16 t + 8 h + qq (+ 4)
            av[p] = cat44(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rda + o)),
                          __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rda + o + 512)));
            bv[p] = cat44(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rdb + o)),
                          __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rdb + o + 512)));
        }
    };
    const int sbeg = a.seg_off[blockIdx.x], send = a.seg_off[blockIdx.x + 1];
    KsSeg sg_next = a.segs[sbeg < send ? sbeg : 0];
    if (sbeg < send) {
        if constexpr (BF) {
            load_half(desc(a.tiles[sg_next.tile]), sg_next.p0, 0);
            load_half(desc(a.tiles[sg_next.tile]), sg_next.p0, 1);
        } else {
            load(desc(a.tiles[sg_next.tile]), sg_next.p0);
        }
    }
    for (int si = sbeg; si < send; ++si) {  // uniform
        if (dg) tprev = __builtin_amdgcn_s_memtime();
        const KsSeg sg = sg_next;
        const KsTile tl = a.tiles[sg.tile];
        const Ld cur = desc(tl);
        const int n = cur.n;
        int poff = (int)a.lay[0].poff;
#pragma unroll
        for (int l = 1; l < kMaxL; ++l)
            if (tl.layer == l) poff = (int)a.lay[l].poff;
        const int corr_off = poff + 2 * n;
        // the segment after this one: its first pass loads behind our last
        const bool more = si + 1 < send;
        if (more) sg_next = a.segs[si + 1];
        const Ld nxt = desc(a.tiles[sg_next.tile]);
        // epilogue rows: r_j = r0 + srow + 16 j, columns 64 k + 4 col4 + (0..3)
        int rowp[4];
        bool rown[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = tl.r0 + srow + 16 * j;
            rown[j] = r >= tl.rlo && r < tl.rhi && r >= 1 && r <= n - 2;
            rowp[j] = corr_off + (int)((int64_t)r * (r - 1) / 2);
        }
        float4 pq[4], mq[4], vq[4];
        // the diagonal tile's mean / sd rows (thread tid & 63 -> row r0 + (tid & 63)):
        // value, m, v of both, loaded with corr / m / v (not one round trip each)
        float dmu = 0.f, dsd = 0.f, dmm = 0.f, dmv = 0.f, dsm = 0.f, dsv = 0.f;
        const int pm_d = poff + tl.r0 + (tid & 63), ps_d = pm_d + n;
        auto load_pmv = [&]() {
            if (tl.diag) {  // uniform
                const uint32_t om = (uint32_t)pm_d * 4u, os = (uint32_t)ps_d * 4u;
                dmu = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rpar, om, 0, 0));
                dsd = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rpar, os, 0, 0));
                if (!GRAD) {
                    dmm = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rm, om, 0, 0));
                    dmv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rv, om, 0, 0));
                    dsm = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rm, os, 0, 0));
                    dsv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rv, os, 0, 0));
                }
            }
            const int cl = tl.k * UB + 4 * col4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // rows off the band's corr rows load something valid, never stored
                const uint32_t o = (uint32_t)(rowp[j] + cl) * 4u;
                pq[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rpar, o, 0, 0));
                mq[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rm, o, 0, 0));
                if (!GRAD) vq[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rv, o, 0, 0));
            }
        };
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
        float dgm = 0.f, dgs = 0.f;
        const bool whole = sg.slot < 0;
        for (int pi = sg.p0; pi < sg.p1; ++pi) {  // uniform
            const bool inseg = pi + 1 < sg.p1;
            if constexpr (BF) {
#pragma unroll
                for (int hp = 0; hp < 2; ++hp) {
                    __syncthreads();  // every wave done with the images
                    stage_half(hp);
                    __syncthreads();
                    if (pi == sg.p0 && hp == 0) mark(1);
                    // this half's registers refilled at once: the next pass's
                    // half (after the segment's last pass, the next segment's)
                    if (inseg || more) load_half(inseg ? cur : nxt, inseg ? pi + 1 : sg_next.p0, hp);
                    if (pi * USB + 64 * hp >= a.S) continue;  // uniform: a ragged last pass
                    // one K-step of fragments at a time (the other workgroup on
                    // the CU covers the LDS latency; a second set spills)
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        bf8v fa[3], fb[3];
                        read_ab(t, fa, fb);
                        acc = mfma6(fa, fb, acc);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (tl.diag && wc == wr) {
                        // the diagonal quadrants: lane (c = r, h) reads eps and G of
                        // the same row for its samples -- sum_s G, sum_s G eps
#pragma unroll 1
                        for (int t = 0; t < 4; ++t) {
                            bf8v av[3], bv[3];
                            read_ab(t, av, bv);
#pragma unroll
                            for (int j = 0; j < 8; j += 2) {
                                const f32x2 e = (bf_pair(av[0], j) + bf_pair(av[1], j)) + bf_pair(av[2], j);
                                const f32x2 gg = (bf_pair(bv[0], j) + bf_pair(bv[1], j)) + bf_pair(bv[2], j);
                                dgm += gg[0] + gg[1];
                                dgs = fmaf(gg[1], e[1], fmaf(gg[0], e[0], dgs));
                            }
                        }
                    }
                }
                continue;
            }
            stage();
            __syncthreads();
            if (pi == sg.p0) mark(1);
            // the next pass's operands behind this pass's MFMAs -- after the
            // segment's last pass, the next segment's first (corr / m / v are
            // loaded at the epilogue: prefetched here they keep 48 more
            // registers live across the MFMAs and the kernel takes scratch)
            if (inseg || more) load(inseg ? cur : nxt, inseg ? pi + 1 : sg_next.p0);
            const int kend = min(USB, a.S - pi * USB);
            if (tl.diag) {
                // column j of Es is row r0 + j of the band
                for (int s = 32 * wv; s < 32 * wv + 32 && s < kend; ++s) {
                    const float gv = Gs[s * ULD + lane];
                    dgm += gv;
                    dgs = fmaf(gv, Es[s * ULD + lane], dgs);
                }
            }
            const float* Ea = Es + h * ULD + 32 * wc + l32;
            const float* Gb = Gs + h * ULD + 32 * wr + l32;
            for (int kk = 0; kk < kend; kk += 16) {
                float av[8], bv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    av[u] = Ea[(kk + 2 * u) * ULD];
                    bv[u] = Gb[(kk + 2 * u) * ULD];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
            }
            __syncthreads();  // every wave done with Gs / Es
        }
        if (BF && tl.diag) {
            // the two halves' sums; row 32 wr + l32 of the band kept by wave 0
            // in lanes 0..31 and by wave 3 in lanes 32..63, so that the
            // epilogue's wave sum red[w 64 + j] sees row j once
            dgm += __shfl_xor(dgm, 32, kWave);
            dgs += __shfl_xor(dgs, 32, kWave);
            if (!((wv == 0 && h == 0) || (wv == 3 && h == 1))) dgm = dgs = 0.f;
        }
        mark(2);
        if (!whole) {
            // ---- split tile: publish this contributor's partial (fragment order:
            // float4 (w * 4 + g) * 64 + lane; then 2 floats of diagonal sums per thread)
            const uint32_t sbase = (uint32_t)((sg.slot + sg.ci) * kKsSlotFloats) * 4u;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                BSTORE128(
                    __builtin_bit_cast(u32x4, make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2],
                                                          acc[4 * g + 3])),
                    rs, sbase + (uint32_t)(((wv * 4 + g) * 64 + lane) * 16), 0, 16);
            if (tl.diag)
                __builtin_amdgcn_raw_buffer_store_b64(
                    __builtin_bit_cast(u32x2, f32x2{dgm, dgs}), rs,
                    sbase + (uint32_t)(4096 * 4 + tid * 8), 0, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const int old = __hip_atomic_fetch_add(a.cnt + tl.cnt, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                sh.red[0] = __int_as_float(old);
            }
            __syncthreads();
            const int old = __float_as_int(sh.red[0]);
            __syncthreads();  // everyone has read the ticket before red is reused
            mark(3);
            if (old != sg.nc - 1) continue;  // uniform: another contributor finishes the tile
            ++ncomb;
            // the last arriver: every partial, in pass order, through sc1 loads
            if (tid == 0)
                __hip_atomic_store(a.cnt + tl.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            load_pmv();
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.f;
            dgm = dgs = 0.f;
            // the partials KP at a time (all their loads in flight together),
            // added in pass order; past nc the last one is loaded again, not added
            constexpr int KP = BF ? 2 : 4;  // BF: fewer registers beside the image bases
            for (int c0 = 0; c0 < sg.nc; c0 += KP) {  // uniform
                float4 part[KP][4];
                f32x2 pd[KP];
#pragma unroll
                for (int i = 0; i < KP; ++i) {
                    const int c = min(c0 + i, sg.nc - 1);
                    const uint32_t cb = (uint32_t)((sg.slot + c) * kKsSlotFloats) * 4u;
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        part[i][g] = __builtin_bit_cast(
                            float4, __builtin_amdgcn_raw_buffer_load_b128(
                                        rs, cb + (uint32_t)(((wv * 4 + g) * 64 + lane) * 16), 0, 16));
                    pd[i] = tl.diag ? __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                                                   rs, cb + (uint32_t)(4096 * 4 + tid * 8), 0, 16))
                                    : f32x2{0.f, 0.f};
                }
#pragma unroll
                for (int i = 0; i < KP; ++i) {
                    if (c0 + i >= sg.nc) break;  // uniform
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        acc[4 * g] += part[i][g].x;
                        acc[4 * g + 1] += part[i][g].y;
                        acc[4 * g + 2] += part[i][g].z;
                        acc[4 * g + 3] += part[i][g].w;
                    }
                    dgm += pd[i][0];
                    dgs += pd[i][1];
                }
            }
            mark(4);
        }
        if (whole) load_pmv();
        // ---- Adam epilogue: D[i = c][j = r] (j = lane & 31, i = (q & 3) + 8 (q >> 2) + 4 h)
        // -> T[r][c] in Es, then the rows' 256-byte runs of corr / m / v
        float* T = BF ? reinterpret_cast<float*>(&sh) : Es;
        if constexpr (BF) __syncthreads();  // the images are T now: every wave past its last reads
#pragma unroll
        for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(&T[(32 * wr + l32) * TLD + 32 * wc + 8 * g + 4 * h]) =
                make_float4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]);
        __syncthreads();
        const int cb = tl.k * UB + 4 * col4;
        float klt = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = tl.r0 + srow + 16 * j;
            if (!rown[j] || cb >= r) continue;
            const int o = rowp[j] + cb;
            const float4 d4 = *reinterpret_cast<const float4*>(&T[(srow + 16 * j) * TLD + 4 * col4]);
            const float4 p4 = pq[j], m4 = mq[j], v4 = GRAD ? float4{} : vq[j];
            float pn[4], mn[4], vn[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float p = f4get(p4, i);
                klt += cb + i < r ? p * p : 0.f;
                float gval = a.include_kl ? f4get(d4, i) + p * a.inv_s0sq : f4get(d4, i);
                if (GRAD) {
                    // the chunked kernel's gradient mode (upd_chunk): + kl_vec / s0^2
                    if (a.kl_vec) gval += f4get(m4, i) * a.inv_s0sq;
                    pn[i] = gval;
                    continue;
                }
                float mm = f4get(m4, i), vv = f4get(v4, i);
                pn[i] = adam_apply_fast(a.adam, p, gval, mm, vv);
                mn[i] = mm;
                vn[i] = vv;
            }
            if (GRAD) {
                if (cb + 3 < r) {
                    *reinterpret_cast<float4*>(a.grad_out + o) = make_float4(pn[0], pn[1], pn[2], pn[3]);
                } else {
#pragma unroll
                    for (int i = 0; i < 3; ++i)
                        if (cb + i < r) a.grad_out[o + i] = pn[i];
                }
                continue;
            }
            if (cb + 3 < r) {
                *reinterpret_cast<float4*>(a.params + o) = make_float4(pn[0], pn[1], pn[2], pn[3]);
                *reinterpret_cast<float4*>(a.m + o) = make_float4(mn[0], mn[1], mn[2], mn[3]);
                *reinterpret_cast<float4*>(a.v + o) = make_float4(vn[0], vn[1], vn[2], vn[3]);
            } else {
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    if (cb + i < r) {
                        a.params[o + i] = pn[i];
                        a.m[o + i] = mn[i];
                        a.v[o + i] = vn[i];
                    }
            }
        }
        klp += klt * (0.5f * a.inv_s0sq);
        if (tl.diag) {
            // the band's mean / sd from the four waves' row sums, added in wave order
            sh.red[wv * 64 + lane] = dgm;
            sh.red[256 + wv * 64 + lane] = dgs;
            __syncthreads();
            const int rr = tl.r0 + tid;
            if (tid < 64 && rr >= tl.rlo && rr < tl.rhi) {
                const float* red = sh.red;
                const float gm = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];
                const float gs = red[256 + tid] + red[320 + tid] + red[384 + tid] + red[448 + tid];
                const int pm = pm_d, ps = ps_d;  // rr = r0 + tid
                const float mu = dmu, sdr = dsd;
                const float sp = softplus_f(sdr), sgm = sigmoid_f(sdr);
                float gmean = gm, gsd = gs * sgm;
                if (a.include_kl) {
                    gmean += mu * a.inv_s0sq;
                    gsd += (sp * a.inv_s0sq - 1.f / sp) * sgm;
                    klp += a.log_s0 - logf(sp) + 0.5f * ((sp * sp + mu * mu) * a.inv_s0sq - 1.f);
                }
                if (GRAD) {
                    a.grad_out[pm] = gmean;
                    a.grad_out[ps] = gsd;
                } else {
                float mm = dmm, vv = dmv;
                a.params[pm] = adam_apply(a.adam, mu, gmean, mm, vv);
                a.m[pm] = mm;
                a.v[pm] = vv;
                mm = dsm;
                vv = dsv;
                a.params[ps] = adam_apply(a.adam, sdr, gsd, mm, vv);
                a.m[ps] = mm;
                a.v[ps] = vv;
                }
            }
        }
        __syncthreads();  // T / red reads done before the next segment stages
        mark(5);
    }
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, sh.red);
        if (tid == 0) atomicAdd(a.kl_out, (double)tot);
    }
    if (dg && tid == 0) {
        unsigned long long* o = a.stamps + (size_t)blockIdx.x * 16;
        o[0] = t_start;
        for (int k = 1; k < 6; ++k) o[k] = ph[k];
        o[6] = (unsigned long long)(send - sbeg);
        o[7] = (unsigned long long)ncomb;
        o[12] = __builtin_amdgcn_s_memtime();
        o[13] = rt_start;
        o[14] = __builtin_amdgcn_s_memrealtime();
    }
}

// ------------------------------------------------- streaming fused update
// The inner loop's steady-state update (Adam, tiled corr/m/v state, world 1,
// S a multiple of 32 up to 128) fused with the next step's sample, as one
// persistent workgroup per CU walking a contiguous run of the layer-major,
// band-major tile list (band b: tiles k = 0 .. b, the diagonal last).
// Per 64x64 tile (l, b, k), wave (wr, wc) owns rows 64b + 32wr + [0, 32) x
// columns 64k + 32wc + [0, 32):
//   dL^T[c][r] = sum_s eps[s][c] G[s][r]      v_mfma_f32_32x32x2_f32, K = S;
//       A = eps (the tile's column block), B = G (the band's slice), both
//       from LDS with ds_read_b32 (the band's slice is staged once per band);
//   corr/m/v <- Adam on the accumulators (tiled state: the fragment order, 1 KB
//       per wave instruction); the new L entries stay in registers;
//   x'[s][r] += sum_c eps'[s][c] L'[r][c]     K = the wave's 32 columns:
//       B = L' straight from the registers (K permuted to the fragment
//       order), A = eps' from LDS, one ds_read_b128 per 4 MFMAs.
// x' accumulates in registers over the run's tiles of one band; at the band's
// end the two column-half waves add their partials through LDS and write the
// segment's slot ([S][64]); mvn_fwd_reduce_kernel adds a band's slots.
// Prefetch: tile i+1's corr/m/v and eps / eps' blocks are loaded behind tile
// i's x' GEMM (eps blocks into the other LDS buffer after it), the next
// band's G slice too.  LDS rows of the eps blocks are 16 float4 slots, slot
// c4 stored at c4 ^ (s & 15): the dL reads (one row, 32 columns) and the x'
// reads (16 rows, one float4 column) are both bank-conflict free.
// One barrier per tile (three at a band's end).
struct StrArgs {
    const StreamRange* ranges;
    int nb[kMaxL];         // bands per layer
    const float* eps;
    const float* eps_next;
    const float* g;
    int ldg, S;
    int64_t g_total, e_total;
    float* params;
    float* m;
    float* v;
    float* tp;
    float* tm;
    float* tv;
    float* part;
    double* kl_out;
    int include_kl;
    unsigned long long* stamps;    // diagnostics: 16 slots per workgroup (DIAG build only)
    float inv_s0sq, log_s0;
    AdamC adam;
    int xcol[kMaxL];
    MvnLayerArgs lay[kMaxL];
    // mvn_stream_bf2_kernel: the bf16 planes of eps / eps_next (EpsPlanes layout)
    const uint16_t* ep;
    const uint16_t* enp;
    int64_t pl;
    int64_t ppoff[kMaxL];
    int npad[kMaxL];
    // mvn_stream_bf2_kernel<FOLD>: the band combine in the kernel (the
    // stream's row-block table, one arrival counter per band, x' and its row
    // stride)
    const FwdRowBlock* rbs;
    int* bcnt;
    float* bms;  // per band: the new mean (64) and softplus(sd) (64)
    float* x;
    int ldx;
};

struct StrTile {
    int l, b, k, n, eoff, xc;
    int64_t tb, poff;
    int64_t pe;  // bf16 planes: element of (layer l, sample 0, column 64 k)
    int npad;    // bf16 planes: row length of layer l
};

__device__ __forceinline__ StrTile str_tile(const StrArgs& a, int l, int b, int k) {
    StrTile T;
    T.l = l;
    T.b = b;
    T.k = k;
    T.n = a.lay[l].n;
    T.eoff = (int)a.lay[l].eoff;
    T.xc = a.xcol[l];
    T.poff = a.lay[l].poff;
    T.tb = tile_index(a.lay[l], b, k) * 4096;
    T.pe = a.ppoff[l] + 64 * k;
    T.npad = a.npad[l];
    return T;
}

// Adam with the variant fixed at compile time (adam_apply_fast's arithmetic)
template <int KIND>
__device__ __forceinline__ float adam_fast_k(const AdamC& a, float p, float g, float& m, float& v) {
    m = a.b1 * m + a.omb1 * g;
    if (KIND == PSVI_ADAM_HIGHER) {
        v = a.b2 * v + a.omb2 * g * g;
        const float denom = __builtin_amdgcn_sqrtf(v + 1e-8f) * a.inv_sqrt_bc2 + a.eps;
        return p - a.lr_bc1 * m * __builtin_amdgcn_rcpf(denom);
    } else if (KIND == PSVI_ADAM_TORCH) {
        v = a.b2 * v + a.omb2 * g * g;
        const float denom = __builtin_amdgcn_sqrtf(v) * a.inv_sqrt_bc2 + a.eps;
        return p - a.lr_bc1 * m * __builtin_amdgcn_rcpf(denom);
    } else {
        v = a.b2 * v + a.omb2 * g * g + 1e-12f;
        const float denom = __builtin_amdgcn_sqrtf(v * a.inv_bc2) + a.eps;
        return p - a.lr * (m * a.inv_bc1) * __builtin_amdgcn_rcpf(denom);
    }
}

constexpr int kFoldMax = 64;  // band ends per run the in-kernel combine can take (FOLD)
constexpr int kStrBuf = 128 * 16;  // float4 per eps block buffer ([128 samples][16 slots])
typedef float f32x4 __attribute__((ext_vector_type(4)));  // plain vector loads / stores (no memcpy)

// adam_fast_k on two entries at once: the arithmetic as v_pk_mul_f32 /
// v_pk_fma_f32 / v_pk_add_f32 (two fp32 lanes per instruction on gfx950),
// the square root and reciprocal per entry
template <int KIND>
__device__ __forceinline__ f32x2 adam_fast_k2(const AdamC& a, f32x2 p, f32x2 g, f32x2& m, f32x2& v) {
    const f32x2 b1 = {a.b1, a.b1}, omb1 = {a.omb1, a.omb1}, b2 = {a.b2, a.b2}, omb2 = {a.omb2, a.omb2};
    m = __builtin_elementwise_fma(b1, m, omb1 * g);
    f32x2 d;
    if (KIND == PSVI_ADAM_HIGHER || KIND == PSVI_ADAM_TORCH) {
        v = __builtin_elementwise_fma(b2, v, (omb2 * g) * g);
        const f32x2 vv = KIND == PSVI_ADAM_HIGHER ? v + f32x2{1e-8f, 1e-8f} : v;
        const f32x2 sq = {__builtin_amdgcn_sqrtf(vv[0]), __builtin_amdgcn_sqrtf(vv[1])};
        d = __builtin_elementwise_fma(sq, f32x2{a.inv_sqrt_bc2, a.inv_sqrt_bc2}, f32x2{a.eps, a.eps});
        const f32x2 r = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
        return p - (f32x2{a.lr_bc1, a.lr_bc1} * m) * r;
    } else {
        v = __builtin_elementwise_fma(b2, v, (omb2 * g) * g) + f32x2{1e-12f, 1e-12f};
        const f32x2 vb = v * f32x2{a.inv_bc2, a.inv_bc2};
        d = f32x2{__builtin_amdgcn_sqrtf(vb[0]), __builtin_amdgcn_sqrtf(vb[1])} + f32x2{a.eps, a.eps};
        const f32x2 r = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
        return p - f32x2{a.lr, a.lr} * (m * f32x2{a.inv_bc1, a.inv_bc1}) * r;
    }
}

// NS = S / 32; KIND: Adam variant; DIAG: the diagnostics build (phase stamps);
// SC1: corr / m / v stores write-through with sc1, which drops the lines from
// the XCD's L2 (MI355X_MICROARCH.md, store flavours): the 60 MB of state written
// per launch then no longer evicts the eps / eps' blocks and G slices that
// later tiles re-read from L2 (false: plain stores, A/B)
template <int NS, int KIND, bool DIAG = false, bool SC1 = true, bool PAD = false>
__global__ __launch_bounds__(256, 1) void mvn_stream_kernel(StrArgs a) {
    constexpr int KT = 16 * NS;  // K steps of the dL GEMM (2 samples each)
    // [0, 4 kStrBuf): eps / eps' blocks, two buffers; then the band's G slice [128][64]
    __shared__ __attribute__((aligned(16))) f32x4 sm[4 * kStrBuf + 2048];
    f32x4* const Gl4 = sm + 4 * kStrBuf;
    const float* const Gl = reinterpret_cast<const float*>(Gl4);
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    const int wr = wv >> 1, wc = wv & 1, h = lane >> 5, l32 = lane & 31;
    const StreamRange R = a.ranges[blockIdx.x];
    const int t0 = __builtin_amdgcn_readfirstlane(R.t0);
    const int t1 = __builtin_amdgcn_readfirstlane(R.t1);
    int slot = __builtin_amdgcn_readfirstlane(R.slot0);
    const int S = a.S;
    // diagnostics: shader clocks per phase summed over the run's tiles (thread 0)
    unsigned long long tph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
    auto ph = [&](int q) __attribute__((always_inline)) {
        if (DIAG && tid == 0) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            if (q >= 0) tph[q] += tt - tlast;
            tlast = tt;
        }
    };
    // PAD (psvi_inner_loop's own eps / G buffers, each followed by 64 zeroed
    // floats): the loads past a layer's last column block run into the pad,
    // so they need no clamp at the buffer's end and no fix-up at use
    const int e_hi = PAD ? 0x7fffffff : (int)a.e_total - 4;
    const int g_hi = PAD ? 0x7fffffff : (int)a.g_total - 4;
    constexpr int SMAX = 32 * NS - 1;  // the staged sample rows: f >> 4 <= 127 needs no clamp at NS = 4

    // eps / eps' block of a tile: 8 + 8 float4 per thread, registers then LDS
    f32x4 ereg[8], enreg[8];
    auto load_E = [&](const StrTile& T) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + 256 * j, s = min(f >> 4, SMAX), c4 = f & 15;
            const int off = min(T.eoff + s * T.n + 64 * T.k + 4 * c4, e_hi);
            ereg[j] = *reinterpret_cast<const f32x4*>(a.eps + off);
            enreg[j] = *reinterpret_cast<const f32x4*>(a.eps_next + off);
        }
    };
    // the float4 clamped at the buffer's end holds columns shifted by d: move
    // them back (applied where the registers are consumed, after the loads land)
    auto fix_E = [&](const StrTile& T) __attribute__((always_inline)) {
        if constexpr (PAD) return;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + 256 * j, s = min(f >> 4, SMAX), c4 = f & 15;
            const int o = T.eoff + s * T.n + 64 * T.k + 4 * c4, d = o - min(o, e_hi);
            if (d > 0) {  // VALU-only: the loads are already unconditional
                ereg[j] = f32x4{d < 4 ? ereg[j][min(d, 3)] : 0.f, d < 3 ? ereg[j][min(d + 1, 3)] : 0.f,
                                d < 2 ? ereg[j][min(d + 2, 3)] : 0.f, d < 1 ? ereg[j][3] : 0.f};
                enreg[j] = f32x4{d < 4 ? enreg[j][min(d, 3)] : 0.f, d < 3 ? enreg[j][min(d + 1, 3)] : 0.f,
                                 d < 2 ? enreg[j][min(d + 2, 3)] : 0.f, d < 1 ? enreg[j][3] : 0.f};
            }
        }
    };
    auto store_E = [&](int bi, const StrTile& T) __attribute__((always_inline)) {
        fix_E(T);
        f32x4* E = sm + 2 * bi * kStrBuf;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + 256 * j, s = f >> 4, c4 = f & 15;
            const int o = s * 16 + (c4 ^ (s & 15));
            E[o] = ereg[j];
            E[kStrBuf + o] = enreg[j];
        }
    };
    // the band's G slice [s][64 rows]: 8 float4 per thread
    f32x4 greg[8];
    auto load_G = [&](const StrTile& T) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + 256 * j, s = min(f >> 4, SMAX), c4 = f & 15;
            greg[j] = *reinterpret_cast<const f32x4*>(
                a.g + min(s * a.ldg + T.xc + 64 * T.b + 4 * c4, g_hi));
        }
    };
    auto store_G = [&](const StrTile& T) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int f = tid + 256 * j, s = min(f >> 4, SMAX), c4 = f & 15;
            const int o = s * a.ldg + T.xc + 64 * T.b + 4 * c4, d = o - min(o, g_hi);
            f32x4 gv = greg[j];
            if (!PAD && d > 0)  // clamped at the buffer's end (see fix_E)
                gv = f32x4{d < 4 ? gv[min(d, 3)] : 0.f, d < 3 ? gv[min(d + 1, 3)] : 0.f,
                           d < 2 ? gv[min(d + 2, 3)] : 0.f, 0.f};
            Gl4[tid + 256 * j] = gv;
        }
    };
    f32x4 P[4], M4[4], V4[4];
    auto frag_off = [&](const StrTile& T, int g) __attribute__((always_inline)) {
        return T.tb + (int64_t)((wv * 4 + g) * 64 + lane) * 4;
    };
    // tm / tv follow tp in one allocation (tstate) of < 2 GB: one descriptor,
    // the m / v arrays at a scalar byte offset
    const rsrc_t rs_t = make_rsrc(a.tp, 0x7fffffff);
    const int tmb = __builtin_amdgcn_readfirstlane((int)((a.tm - a.tp) * 4));
    const int tvb = __builtin_amdgcn_readfirstlane((int)((a.tv - a.tp) * 4));
    auto load_pmv = [&](const StrTile& T) __attribute__((always_inline)) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int64_t o = frag_off(T, g);
            P[g] = *reinterpret_cast<const f32x4*>(a.tp + o);
            M4[g] = *reinterpret_cast<const f32x4*>(a.tm + o);
            V4[g] = *reinterpret_cast<const f32x4*>(a.tv + o);
        }
    };

    floatx16 xacc[NS];
#pragma unroll
    for (int sb = 0; sb < NS; ++sb)
#pragma unroll
        for (int q = 0; q < 16; ++q) xacc[sb][q] = 0.f;
    float klp = 0.f, kld = 0.f;  // sum corr^2 (scaled at the end), diagonal KL terms
    f32x2 kl2 = {0.f, 0.f};      // sum corr^2, two lanes (packed with the Adam arithmetic)

    // per-lane LDS offsets of the XOR-swizzled reads
    int okd[8];  // dL A operand (floats): row s = 2t + h, column 32wc + l32; index t & 7
    {
        const int c = 32 * wc + l32, c4 = c >> 2;
#pragma unroll
        for (int k = 0; k < 8; ++k) okd[k] = h * 64 + 4 * ((c4 ^ h) ^ (2 * k)) + (c & 3);
    }
    int okx[4];  // x' A operand (float4): row l32 (+ 32 sb), slot 8wc + 2g + h
#pragma unroll
    for (int g = 0; g < 4; ++g) okx[g] = l32 * 16 + ((8 * wc + 2 * g + h) ^ (l32 & 15));
    const int ogb = h * 64 + 32 * wr + l32;  // G[2t + h][32wr + l32] at ogb + 128 t

    if (DIAG && tid == 0) {
        a.stamps[(size_t)blockIdx.x * 16 + 12] = __builtin_amdgcn_s_memtime();
        a.stamps[(size_t)blockIdx.x * 16 + 13] = __builtin_amdgcn_s_memrealtime();
    }
    // prologue: tile t0
    // tile (l, b, k) of t0, then walked in list order with scalar arithmetic
    int tl = __builtin_amdgcn_readfirstlane(R.lbk0 >> 28);
    int tb_ = __builtin_amdgcn_readfirstlane((R.lbk0 >> 14) & 0x3fff);
    int tk = __builtin_amdgcn_readfirstlane(R.lbk0 & 0x3fff);
    StrTile cur = str_tile(a, tl, tb_, tk);
    load_E(cur);
    load_G(cur);
    store_E(0, cur);
    store_G(cur);
    __syncthreads();

    // one tile; HAS_NEXT / NEWBAND compile-time so that every load is unconditional
    auto tile = [&](int i, const StrTile& nxt, auto has_next_c, auto newband_c) __attribute__((always_inline)) {
        constexpr bool has_next = decltype(has_next_c)::value;
        constexpr bool newband = decltype(newband_c)::value;
        const int bi = (i - t0) & 1;
        ph(-1);
        const float* Ef = reinterpret_cast<const float*>(sm + 2 * bi * kStrBuf);
        const f32x4* En = sm + (2 * bi + 1) * kStrBuf;
        // ---- this tile's corr/m/v: in flight behind the dL GEMM
        load_pmv(cur);
        // ---- dL^T = eps^T G over the samples
        floatx16 acc;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
        for (int t = 0; t < KT; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ef[okd[t & 7] + 128 * t], Gl[ogb + 128 * t],
                                                       acc, 0, 0, 0);
        ph(0);
        const int n = cur.n, r = 64 * cur.b + 32 * wr + l32;
        // ---- diagonal tile: sum_s G and sum_s G eps of the band's rows -> mean / sd
        if (cur.k == cur.b && wc == 0) {
            // row c of the band per lane pair; the sums run in the chunked
            // kernel's order (four partials over sample groups 16w + [0, 16)
            // (+ 64), added left to right), so both kernels agree bit for bit
            const int c = 32 * wr + l32;
            float pm2[2], ps2[2];
#pragma unroll
            for (int ww = 0; ww < 2; ++ww) {
                const int w = 2 * h + ww;
                float gm = 0.f, gsum = 0.f;
#pragma unroll
                for (int hh = 0; hh < (NS > 2 ? 2 : 1); ++hh)
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const int sm_ = hh * 64 + 16 * w + j;
                        if (sm_ < 32 * NS) {
                            const float gv = Gl[sm_ * 64 + c];
                            gm += gv;
                            gsum = fmaf(gv, Ef[sm_ * 64 + 4 * ((c >> 2) ^ (sm_ & 15)) + (c & 3)],
                                        gsum);
                        }
                    }
                pm2[ww] = gm;
                ps2[ww] = gsum;
            }
            const float m2 = __shfl_xor(pm2[0], 32, kWave), m3 = __shfl_xor(pm2[1], 32, kWave);
            const float s2 = __shfl_xor(ps2[0], 32, kWave), s3 = __shfl_xor(ps2[1], 32, kWave);
            const float dgm = ((pm2[0] + pm2[1]) + m2) + m3;
            const float dgs = ((ps2[0] + ps2[1]) + s2) + s3;
            if (h == 0 && r < n) {
                const int pm = (int)cur.poff + r, ps = pm + n;
                const float mu = a.params[pm], sdr = a.params[ps];
                const float sp = softplus_f(sdr), sg = sigmoid_f(sdr);
                float gmean = dgm, gsd = dgs * sg;
                if (a.include_kl) {
                    gmean += mu * a.inv_s0sq;
                    gsd += (sp * a.inv_s0sq - 1.f / sp) * sg;
                    kld += a.log_s0 - logf(sp) + 0.5f * ((sp * sp + mu * mu) * a.inv_s0sq - 1.f);
                }
                float mm = a.m[pm], vv = a.v[pm];
                a.params[pm] = adam_apply(a.adam, mu, gmean, mm, vv);
                a.m[pm] = mm;
                a.v[pm] = vv;
                mm = a.m[ps];
                vv = a.v[ps];
                a.params[ps] = adam_apply(a.adam, sdr, gsd, mm, vv);
                a.m[ps] = mm;
                a.v[ps] = vv;
            }
        }
        ph(1);
        // ---- per column group g: Adam on the accumulators (fragment order =
        // tiled order), the stores, then g's share of the x' GEMM with the next
        // tile's loads spread between its MFMAs (a burst of them stalls the
        // in-order wave on the memory queue)
        const bool rv = r >= 1 && r <= n - 2;
        const float kls = a.include_kl ? a.inv_s0sq : 0.f;
        float Lf[16];
        auto issue_load = [&](int q) __attribute__((always_inline)) {
            // q < 16: the next tile's eps blocks (8 + 8); then (NEWBAND) the
            // next band's G slice (8)
            if constexpr (has_next) {
                if (q < 16) {
                    const int j = q >> 1;
                    const int f = tid + 256 * j, s = min(f >> 4, SMAX), c4 = f & 15;
                    const int off = min(nxt.eoff + s * nxt.n + 64 * nxt.k + 4 * c4, e_hi);
                    if ((q & 1) == 0) ereg[j] = *reinterpret_cast<const f32x4*>(a.eps + off);
                    else enreg[j] = *reinterpret_cast<const f32x4*>(a.eps_next + off);
                } else if constexpr (newband) {
                    const int j = q - 16;
                    const int f = tid + 256 * j, s = min(f >> 4, SMAX), c4 = f & 15;
                    greg[j] = *reinterpret_cast<const f32x4*>(
                        a.g + min(s * a.ldg + nxt.xc + 64 * nxt.b + 4 * c4, g_hi));
                }
            }
        };
        constexpr int NLOAD = has_next ? (newband ? 24 : 16) : 0;
        f32x4 avn = En[okx[0]];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int cb = 64 * cur.k + 32 * wc + 8 * g + 4 * h;
            float pn[4], mn[4], vn[4];
            // two entries per packed instruction (entries e, e + 1)
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                const f32x2 p = {P[g][e], P[g][e + 1]};
                kl2 = __builtin_elementwise_fma(p, p, kl2);
                const f32x2 gv = __builtin_elementwise_fma(p, f32x2{kls, kls},
                                                           f32x2{acc[4 * g + e], acc[4 * g + e + 1]});
                const f32x2 gm = {rv && cb + e < r ? gv[0] : 0.f, rv && cb + e + 1 < r ? gv[1] : 0.f};
                f32x2 mm = {M4[g][e], M4[g][e + 1]}, vv = {V4[g][e], V4[g][e + 1]};
                const f32x2 pv = adam_fast_k2<KIND>(a.adam, p, gm, mm, vv);
                pn[e] = pv[0];
                pn[e + 1] = pv[1];
                mn[e] = mm[0];
                mn[e + 1] = mm[1];
                vn[e] = vv[0];
                vn[e + 1] = vv[1];
                Lf[4 * g + e] = pn[e];
                Lf[4 * g + e + 1] = pn[e + 1];
            }
            const int64_t o = frag_off(cur, g);
            if constexpr (SC1) {
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                const uint32_t ob = (uint32_t)(o * 4);
                BSTORE128(
                    __builtin_bit_cast(u32x4, f32x4{pn[0], pn[1], pn[2], pn[3]}), rs_t, ob, 0, 16);
                BSTORE128(
                    __builtin_bit_cast(u32x4, f32x4{mn[0], mn[1], mn[2], mn[3]}), rs_t, ob, tmb, 16);
                BSTORE128(
                    __builtin_bit_cast(u32x4, f32x4{vn[0], vn[1], vn[2], vn[3]}), rs_t, ob, tvb, 16);
            } else {
                *reinterpret_cast<f32x4*>(a.tp + o) = f32x4{pn[0], pn[1], pn[2], pn[3]};
                *reinterpret_cast<f32x4*>(a.tm + o) = f32x4{mn[0], mn[1], mn[2], mn[3]};
                *reinterpret_cast<f32x4*>(a.tv + o) = f32x4{vn[0], vn[1], vn[2], vn[3]};
            }
            // x' += eps' L'^T over this group's 8 columns, all sample blocks; the
            // A fragments are read one slot ahead, and each slot is pinned
            // (sched_barrier) so the loads stay spread between the MFMAs
#pragma unroll
            for (int sb = 0; sb < NS; ++sb) {
                const int k = g * NS + sb;
                const f32x4 av = avn;
                if (k + 1 < 4 * NS) avn = En[okx[(k + 1) / NS] + 512 * ((k + 1) % NS)];
                xacc[sb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0], Lf[4 * g + 0], xacc[sb], 0, 0, 0);
                xacc[sb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1], Lf[4 * g + 1], xacc[sb], 0, 0, 0);
                xacc[sb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[2], Lf[4 * g + 2], xacc[sb], 0, 0, 0);
                xacc[sb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[3], Lf[4 * g + 3], xacc[sb], 0, 0, 0);
                // this slot's share of the next tile's loads (slot k of 4 NS)
                constexpr int NSLOT = 4 * NS;
#pragma unroll
                for (int q = 0; q < NLOAD; ++q)
                    if ((q * NSLOT) / (NLOAD > 0 ? NLOAD : 1) == k) issue_load(q);
                __builtin_amdgcn_sched_barrier(0x6);  // VALU / SALU may cross, memory and MFMA may not
            }
        }
        ph(2);
        ph(3);
        ph(4);
        if constexpr (has_next) store_E(bi ^ 1, nxt);
        ph(5);
        // ---- band end (or run end): the two column halves' x' partials -> the slot
        if constexpr (!has_next || newband) {
            __syncthreads();  // every wave done reading buffer bi and the G slice
            float* X = reinterpret_cast<float*>(sm + 2 * bi * kStrBuf);
            if (wc == 1) {
#pragma unroll
                for (int sb = 0; sb < NS; ++sb)
#pragma unroll
                    for (int q = 0; q < 16; ++q) X[((wr * NS + sb) * 16 + q) * 64 + lane] = xacc[sb][q];
            }
            if constexpr (newband) store_G(nxt);
            __syncthreads();
            if (wc == 0) {
                float* dst = a.part + (size_t)slot * S * 64 + 32 * wr + l32;
#pragma unroll
                for (int sb = 0; sb < NS; ++sb)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int s = 32 * sb + (q & 3) + 8 * (q >> 2) + 4 * h;
                        dst[(size_t)s * 64] = xacc[sb][q] + X[((wr * NS + sb) * 16 + q) * 64 + lane];
                    }
            }
#pragma unroll
            for (int sb = 0; sb < NS; ++sb)
#pragma unroll
                for (int q = 0; q < 16; ++q) xacc[sb][q] = 0.f;
            ++slot;
        }
        ph(6);
        __syncthreads();  // buffer bi ^ 1 complete; buffer bi free
        ph(7);
        if (DIAG && tid == 0) ++tph[9];
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    for (int i = t0; i + 1 < t1; ++i) {
        if (++tk > tb_) {
            tk = 0;
            int nbl = a.nb[0];  // select: a dynamic index into the argument copies it to scratch
#pragma unroll
            for (int l = 1; l < kMaxL; ++l)
                if (tl == l) nbl = a.nb[l];
            if (++tb_ == nbl) {
                tb_ = 0;
                ++tl;
            }
        }
        const StrTile nxt = str_tile(a, tl, tb_, tk);
        if (nxt.l != cur.l || nxt.b != cur.b)
            tile(i, nxt, T_{}, T_{});
        else
            tile(i, nxt, T_{}, F_{});
        cur = nxt;
    }
    tile(t1 - 1, cur, F_{}, F_{});
    if (DIAG && tid == 0) {
        unsigned long long* o = a.stamps + (size_t)blockIdx.x * 16;
#pragma unroll
        for (int q = 0; q < 10; ++q) o[q] = tph[q];
        o[10] = __builtin_amdgcn_s_memtime();
        o[11] = __builtin_amdgcn_s_memrealtime();
    }
    klp = (klp + (kl2[0] + kl2[1])) * (0.5f * a.inv_s0sq) + kld;
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, reinterpret_cast<float*>(sm));
        if (tid == 0) atomicAdd(a.kl_out, (double)tot);
    }
}


// ---------------------------------------------------------------------------
// The bf16-piece streaming update: mvn_stream_kernel's tile walk with both
// products on the bf16 matrix cores, fp32-faithful.  Every operand is split into three bf16
// pieces (split3: exact) and each product is the six piece products that
// matter (the dropped ones are below 2^-26 of the product, under fp32's own
// rounding); the matrix cores accumulate in fp32.  v_mfma_f32_32x32x16_bf16
// does 16 K per 32 cycles against v_mfma_f32_32x32x2_f32's 2 per 64, so the
// six products take 3/8 of the fp32 MFMA time, and the vector unit keeps
// issuing beside a bf16 MFMA (it holds the SIMD for 8 of its 32 cycles;
// MI355X_MICROARCH.md, cycle constants), where the fp32 form serialises
// with the Adam epilogue.
//   eps  (dL's A operand, K = samples): the draw's planes staged into an
//        LDS image [s][64 columns] per plane, read column-wise with
//        ds_read_b64_tr_b16;
//   G    (dL's B operand): the band's slice split once per band into a
//        second column image;
//   eps' (x''s A operand, K = columns): the next draw's planes in a row image;
//   L'   (x''s B operand): the new corr entries, split in the accumulators'
//        registers (the accumulator-as-operand order of the 32x32x16 form).
// Tiled state, slots, the diagonal's mean / sd and the KL as mvn_stream_kernel.
//
// mvn_stream_bf2_kernel: that tile walk with two waves per SIMD (the round-5
// four-wave form, one wave per SIMD, ran 37.6 us against 33.8 at C3).  Eight
// waves per workgroup: wave (q, hk) with quadrant q = wv & 3 -- rows 32 wr,
// columns 32 wc of the 64 x 64 tile, (wr, wc) = (q >> 1, q & 1) -- and sample
// half hk = wv >> 2 (samples 64 hk .. 64 hk + 63).  The two waves of a
// quadrant sit on one SIMD (waves w and w + 4), so one's vector work, LDS
// waits and stores run beside the other's MFMAs:
//   dL: each wave its samples' half of K (4 K-steps), the halves exchanged
//       through LDS -- each wave gets the partner's partial of its own two
//       column groups g = 2 hk, 2 hk + 1 and adds it (hk 0's + hk 1's, the
//       same sum in both orders);
//   Adam: each wave its two groups (corr / m / v fragments loaded, stored),
//       and their L' pieces -- K-half st = hk of x''s B operand -- swapped
//       with the partner through LDS;
//   x': each wave its samples' two 32-row blocks over both K-halves (x'
//       accumulators: 32 registers per wave);
//   band end: the wc = 1 waves' x' partials added by the wc = 0 waves (per
//       sample half) and written to the segment's slot, as before.
// The exchanges use the eps column image after the dL reads (16 + 24 KB); the
// next tile's eps planes are stored after them.  Images, pieces, swizzles and
// the slot layout as described above.  DIAG: per-phase shader clocks summed
// over the run's tiles (thread 0) into the stamp buffer (tools/bf_stamps.py).
//
// FOLD: the band's x' rows are finished in the kernel instead of by
// mvn_fwd_reduce_kernel.  At a band's end each segment stores its slot
// write-through (sc1), drains (vmcnt 0), and one lane adds to the band's
// counter (relaxed, agent scope); the segment that draws the last ticket
// reads the band's slots with sc1 loads and writes x' = mean + softplus(sd)
// eps' + the slots' sum, in the reduce's order (slot k into partial k mod 4),
// so the result is the reduce's bit for bit.  The band's new mean / sd come
// from its diagonal tile, the band's last: stored write-through by that
// segment before its own drain and ticket, read with agent-scope loads.  The
// hand-off is the K-split update's (MI355X_MICROARCH.md hand-off table, first
// row); no workgroup waits on another.
template <int KIND, bool DIAG = false, bool FOLD = false>
__global__ __launch_bounds__(512, 1) void mvn_stream_bf2_kernel(StrArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t smb[9 * kBfImg];
    uint8_t* const Eb = smb;
    uint8_t* const Gb = smb + 3 * kBfImg;
    uint8_t* const En = smb + 6 * kBfImg;
    float* const Xs = reinterpret_cast<float*>(En);
    float* const Xd = reinterpret_cast<float*>(Eb);                  // dL partials: 8 waves x 8 x 64 (16 KB)
    uint32_t* const Xl = reinterpret_cast<uint32_t*>(Eb + 16384);    // L' pieces: 8 waves x 12 x 64 (24 KB)
    float* const Xg = reinterpret_cast<float*>(Eb + 40960);          // diagonal sums: 8 waves x 2 x 64 (4 KB)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    const int q = wv & 3, hk = wv >> 2, wr = q >> 1, wc = q & 1, h = lane >> 5, l32 = lane & 31;
    const int pw = wv ^ 4;  // the partner wave (same quadrant, other sample half)
    const StreamRange R = a.ranges[blockIdx.x];
    const int t0 = __builtin_amdgcn_readfirstlane(R.t0);
    const int t1 = __builtin_amdgcn_readfirstlane(R.t1);
    int slot = __builtin_amdgcn_readfirstlane(R.slot0);
    const int S = a.S;  // 128
    unsigned long long tph[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
    // (wave 0 as a whole: the stamps stay wave-uniform, in scalar registers)
    if (DIAG && tid == 0) a.stamps[(size_t)blockIdx.x * 16 + 13] = __builtin_amdgcn_s_memtime();
    auto ph = [&](int qq) __attribute__((always_inline)) {
        if (DIAG && wv == 0) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            if (qq >= 0) tph[qq] += tt - tlast;
            tlast = tt;
        }
    };

    // ---- staging: 6 chunks of 16 bytes per thread: chunk j = plane j >> 1, row
    // (tid >> 3) + 64 (j & 1), chunk tid % 8 of the tile's 64 columns
    u32x4 stg[6];
    const int srow0 = tid >> 3, ch = tid & 7;
    const int st_col = srow0 * 128 + ((ch ^ (((srow0 >> 1) & 1) << 2)) << 4);
    const int st_row0 = img_row(srow0, 8 * ch), st_row1 = img_row(srow0, 8 * ch + 4);
    auto store_col = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 6; ++j)
            *reinterpret_cast<u32x4*>(Eb + st_col + (j >> 1) * kBfImg + 8192 * (j & 1)) = stg[j];
    };
    auto store_row = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            uint8_t* img = En + (j >> 1) * kBfImg + 8192 * (j & 1);
            *reinterpret_cast<u32x2*>(img + st_row0) = u32x2{stg[j][0], stg[j][1]};
            *reinterpret_cast<u32x2*>(img + st_row1) = u32x2{stg[j][2], stg[j][3]};
        }
    };
    // ---- the band's G slice [128 samples][64 rows]: 4 float4 per thread
    f32x4 greg[4];
    auto split_G = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int f = tid + 512 * j, s = f >> 4, c4 = f & 15;
            uint32_t x[3][2];
            split3_pk(f32x2{greg[j][0], greg[j][1]}, x[0][0], x[1][0], x[2][0]);
            split3_pk(f32x2{greg[j][2], greg[j][3]}, x[0][1], x[1][1], x[2][1]);
#pragma unroll
            for (int p = 0; p < 3; ++p)
                *reinterpret_cast<u32x2*>(Gb + p * kBfImg + img_col(s, 4 * c4)) = u32x2{x[p][0], x[p][1]};
        }
    };
    // this wave's two fragment groups g = 2 hk + gi of its quadrant (tiled order)
    f32x4 P[2], M4[2], V4[2];
    const rsrc_t rs_t = make_rsrc(a.tp, 0x7fffffff);
    const rsrc_t rs_e = make_rsrc(a.ep, 0x7fffffff), rs_en = make_rsrc(a.enp, 0x7fffffff);
    const rsrc_t rs_g = make_rsrc(a.g, 0x7fffffff);
    const int tmb = __builtin_amdgcn_readfirstlane((int)((a.tm - a.tp) * 4));
    const int tvb = __builtin_amdgcn_readfirstlane((int)((a.tv - a.tp) * 4));
    const uint32_t vo_f = (uint32_t)(((q * 4 + 2 * hk) * 64 + lane) * 16);  // + 1024 gi
    const uint32_t vo_g = (uint32_t)(4 * ((tid >> 4) * a.ldg + 4 * (tid & 15)));  // G rows tid / 16 (+ 32 j)
    auto vo_planes = [&](const StrTile& T) __attribute__((always_inline)) {
        return (uint32_t)(2 * (srow0 * T.npad + 8 * ch));
    };
    auto so_planes = [&](const StrTile& T, int j) __attribute__((always_inline)) {
        return __builtin_amdgcn_readfirstlane((int)(2 * (T.pe + (j >> 1) * a.pl + (int64_t)(64 * (j & 1)) * T.npad)));
    };
    auto ldb = [&](rsrc_t r, uint32_t vo, int so) __attribute__((always_inline)) {
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
    };
    auto load_G = [&](const StrTile& T, int j) __attribute__((always_inline)) {
        const int so = __builtin_amdgcn_readfirstlane(4 * (32 * j * a.ldg + T.xc + 64 * T.b));
        greg[j] = __builtin_bit_cast(f32x4, ldb(rs_g, vo_g, so));
    };
    floatx16 xacc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int qq = 0; qq < 16; ++qq) xacc[j][qq] = 0.f;
    float kld = 0.f;
    f32x2 kl2 = {0.f, 0.f};
    const int g16 = lane >> 4, qq4 = (lane >> 2) & 3, pp = lane & 3;
    const int ca = 32 * wc + 16 * (g16 & 1) + 4 * pp;  // eps column (dL's A)
    const int cg = 32 * wr + 16 * (g16 & 1) + 4 * pp;  // G column (dL's B)
    const uint8_t* const rda = Eb + img_col(8 * h + qq4, ca);
    const uint8_t* const rdb = Gb + img_col(8 * h + qq4, cg);
    const int xsw = (l32 >> 1) & 7;

    int tl = __builtin_amdgcn_readfirstlane(R.lbk0 >> 28);
    int tb_ = __builtin_amdgcn_readfirstlane((R.lbk0 >> 14) & 0x3fff);
    int tk = __builtin_amdgcn_readfirstlane(R.lbk0 & 0x3fff);
    StrTile cur = str_tile(a, tl, tb_, tk);
    {
        const uint32_t vo = vo_planes(cur);
#pragma unroll
        for (int j = 0; j < 4; ++j) load_G(cur, j);
#pragma unroll
        for (int j = 0; j < 6; ++j) stg[j] = ldb(rs_e, vo, so_planes(cur, j));
        store_col();
#pragma unroll
        for (int j = 0; j < 6; ++j) stg[j] = ldb(rs_en, vo, so_planes(cur, j));
        store_row();
        split_G();
    }
    __syncthreads();

    // phase A's loads: 0..5 this tile's corr / m / v fragments (2 groups x 3),
    // 6..11 the next tile's eps planes
    auto issue_a = [&](int qi, const StrTile& nxt, bool has_next, uint32_t vo_n) __attribute__((always_inline)) {
        if (qi < 6) {
            const int gi = qi / 3, which = qi % 3;
            const int so = __builtin_amdgcn_readfirstlane((int)(cur.tb * 4));
            const u32x4 x = __builtin_bit_cast(
                u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_t, vo_f + 1024 * gi,
                                                             which == 0 ? so : which == 1 ? so + tmb : so + tvb,
                                                             PSVI_STATE_LOAD_AUX));
            if (which == 0) P[gi] = __builtin_bit_cast(f32x4, x);
            else if (which == 1) M4[gi] = __builtin_bit_cast(f32x4, x);
            else V4[gi] = __builtin_bit_cast(f32x4, x);
        } else if (has_next) {
            stg[qi - 6] = ldb(rs_e, vo_n, so_planes(nxt, qi - 6));
        }
    };
    // phase B's loads: 0..5 the next tile's eps' planes, 6..9 the next band's G
    auto issue_b = [&](int qi, const StrTile& nxt, bool has_next, bool newband, uint32_t vo_n) __attribute__((always_inline)) {
        if (qi < 6) {
            if (has_next) stg[qi] = ldb(rs_en, vo_n, so_planes(nxt, qi));
        } else if (newband) {
            load_G(nxt, qi - 6);
        }
    };

    // the band's index in the stream's row-block table (layer-major)
    auto band_id = [&](const StrTile& T) __attribute__((always_inline)) {
        int bid = T.b;
#pragma unroll
        for (int l = 0; l < kMaxL - 1; ++l)
            if (l < T.l) bid += a.nb[l];
        return __builtin_amdgcn_readfirstlane(bid);
    };
    // FOLD: the band's arrival after its slot is stored; the last arriver
    // notes the band and finishes its x' rows after the walk, where the tile
    // walk's prefetch registers are free (see above)
    __shared__ int fold_list[kFoldMax];
    int nfold = 0;
    auto band_arrive = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slot (and mean / sd) stores
        __syncthreads();                                 // ... and every other wave's
        const int bid = band_id(cur);
        const int nk = __builtin_amdgcn_readfirstlane(a.rbs[bid].nk);
        if (nk > 1) {
            if (tid == 0)
                Xs[0] = __int_as_float(
                    __hip_atomic_fetch_add(a.bcnt + bid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            __syncthreads();
            const int old = __builtin_amdgcn_readfirstlane(__float_as_int(Xs[0]));
            if (old != nk - 1) return;  // uniform: another segment finishes the band
            if (tid == 0) __hip_atomic_store(a.bcnt + bid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0) fold_list[nfold] = bid;  // read after the walk's later barriers
        ++nfold;
    };
    // x' rows of band bid from its slots (fragment order, see the band end):
    // thread t takes float4 f = t + 512 m (m = 0..3) of every slot -- row 32
    // (m >> 1) + (t & 31) of the band, samples 64 (m & 1) + 32 j + 4 h + 8 qg +
    // e (e = 0..3) with (j, qg) = ((t >> 8) & 1, (t >> 6) & 3), h = (t >> 5) & 1.
    // Runs after the walk, where the walk's registers are free: mean / sd, eps'
    // and the first four slots' loads in flight together.
    auto band_combine = [&](int bid) __attribute__((always_inline)) {
        const FwdRowBlock rb = a.rbs[bid];
        const int nk = __builtin_amdgcn_readfirstlane(rb.nk), slot0 = __builtin_amdgcn_readfirstlane(rb.slot0);
        const int R = __builtin_amdgcn_readfirstlane(rb.R), xcol = __builtin_amdgcn_readfirstlane(rb.xcol);
        const int l = __builtin_amdgcn_readfirstlane(rb.layer), r0 = __builtin_amdgcn_readfirstlane(rb.r0);
        const int n = a.lay[l].n;
        const float* const bm = a.bms + 128 * (int64_t)bid;
        const int lt = tid & 31, hh = (tid >> 5) & 1, qg = (tid >> 6) & 3, jj = (tid >> 8) & 1;
        // rows rr[w] = 32 w + lt (w = m >> 1): the band's new mean and softplus(sd)
        float mu[2], dg[2], ev[4][4];
#pragma unroll
        for (int w = 0; w < 2; ++w) {
            mu[w] = __hip_atomic_load(bm + 32 * w + lt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            dg[w] = __hip_atomic_load(bm + 64 + 32 * w + lt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        auto smp = [&](int m, int e) { return 64 * (m & 1) + 32 * jj + 4 * hh + 8 * qg + e; };
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float* ec = a.eps_next + a.lay[l].eoff + r0 + min(32 * (m >> 1) + lt, R - 1);
#pragma unroll
            for (int e = 0; e < 4; ++e) ev[m][e] = ec[(int64_t)smp(m, e) * n];
        }
        const rsrc_t rs_p = make_rsrc(a.part, 0x7fffffff);
        f32x4 A[4][4];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) A[m][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        // slot k into partial k mod 4, in slot order (mvn_fwd_reduce_kernel's
        // sum); eight slots' loads in flight per round (the walk's registers
        // are free here): a round trip of sc1 loads is the combine's cost
        // (four in the stamps build, whose stamp registers would spill)
        constexpr int KR = DIAG ? 4 : 8;
        for (int k0 = 0; k0 < nk; k0 += KR) {  // uniform
            f32x4 v[4][KR];
#pragma unroll
            for (int i = 0; i < KR; ++i) {
                const int so = __builtin_amdgcn_readfirstlane((slot0 + min(k0 + i, nk - 1)) * S * 64 * 4);
                if (k0 + i < nk || i == 0) {  // uniform
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        v[m][i] = __builtin_bit_cast(
                            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_p, (uint32_t)((tid + 512 * m) * 16), so, 16));
                }
            }
#pragma unroll
            for (int i = 0; i < KR; ++i)
                if (k0 + i < nk)  // uniform
#pragma unroll
                    for (int m = 0; m < 4; ++m) A[m][i & 3] += v[m][i];
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const f32x4 t = (A[m][0] + A[m][1]) + (A[m][2] + A[m][3]);
            const int rr = 32 * (m >> 1) + lt;
            if (rr < R) {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    a.x[(int64_t)smp(m, e) * a.ldx + xcol + rr] =
                        (mu[m >> 1] + mul_unfused(dg[m >> 1], ev[m][e])) + t[e];  // mvn_fwd_reduce_kernel's rounding
            }
        }
    };

    auto tile = [&](const StrTile& nxt, auto has_next_c, auto newband_c) __attribute__((always_inline)) {
        constexpr bool has_next = decltype(has_next_c)::value;
        constexpr bool newband = decltype(newband_c)::value;
        ph(-1);
        const bool diag = cur.k == cur.b && wc == wr;  // wave-uniform
        const uint32_t vo_n = vo_planes(nxt);
        // ---- phase A: this wave's half of K (sample rows 64 hk + 16 t')
        floatx16 acc;
#pragma unroll
        for (int qq = 0; qq < 16; ++qq) acc[qq] = 0.f;
        float dgm = 0.f, dgs = 0.f;
        auto read_ab = [&](int t, bf8v (&av)[3], bf8v (&bv)[3]) __attribute__((always_inline)) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                typedef __attribute__((address_space(3))) s4v* lds_s4;
                const int o = p * kBfImg + 2048 * t;
                av[p] = cat44(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rda + o)),
                              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rda + o + 512)));
                bv[p] = cat44(__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rdb + o)),
                              __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(rdb + o + 512)));
            }
        };
        // one K-step of fragments at a time: the SIMD's other wave covers the
        // LDS latency (a second set would spill)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            bf8v fa[3], fb[3];
            read_ab(4 * hk + t, fa, fb);
#pragma unroll
            for (int qi = 3 * t; qi < 3 * t + 3; ++qi) issue_a(qi, nxt, has_next, vo_n);
            acc = mfma6(fa, fb, acc);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (diag) {
#pragma unroll 1
            for (int t = 0; t < 4; ++t) {
                bf8v av[3], bv[3];
                read_ab(4 * hk + t, av, bv);
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const f32x2 e = (bf_pair(av[0], j) + bf_pair(av[1], j)) + bf_pair(av[2], j);
                    const f32x2 gg = (bf_pair(bv[0], j) + bf_pair(bv[1], j)) + bf_pair(bv[2], j);
                    dgm += gg[0] + gg[1];
                    dgs = fmaf(gg[1], e[1], fmaf(gg[0], e[0], dgs));
                }
            }
        }
        ph(1);
        __syncthreads();  // B1: every wave done with the eps and G images of this tile
        ph(2);
        // ---- the partner's partial of this wave's groups: send the other two
        // (wave-uniform selects between constant accumulator indices: a
        // run-time index into the accumulators would go through scratch)
        auto accg = [&](int gsel, int e) __attribute__((always_inline)) {
            return hk == 0 ? acc[4 * (gsel + 2) + e] : acc[4 * gsel + e];  // gsel of the OTHER half
        };
        auto accown = [&](int gi, int e) __attribute__((always_inline)) {
            return hk == 0 ? acc[4 * gi + e] : acc[4 * (gi + 2) + e];
        };
        {
#pragma unroll
            for (int gi = 0; gi < 2; ++gi)
                *reinterpret_cast<f32x4*>(Xd + ((wv * 2 + gi) * 64 + lane) * 4) =
                    f32x4{accg(gi, 0), accg(gi, 1), accg(gi, 2), accg(gi, 3)};
            if (diag && hk == 1) {
                // the diagonal sums of this half for the partner (hk 0 runs the mean / sd Adam)
                Xg[wv * 128 + lane] = dgm;
                Xg[wv * 128 + 64 + lane] = dgs;
            }
        }
        __syncthreads();  // B2
        float dv[8];
        {
#pragma unroll
            for (int gi = 0; gi < 2; ++gi) {
                const f32x4 o4 = *reinterpret_cast<const f32x4*>(Xd + ((pw * 2 + gi) * 64 + lane) * 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) dv[4 * gi + e] = accown(gi, e) + o4[e];
            }
            if (diag && hk == 0) {
                dgm += Xg[pw * 128 + lane];
                dgs += Xg[pw * 128 + 64 + lane];
            }
        }
        const int n = cur.n, r = 64 * cur.b + 32 * wr + l32;
        // ---- diagonal tile: mean / sd of the band's rows (the hk = 0 wave)
        if (diag && hk == 0) {
            dgm += __shfl_xor(dgm, 32, kWave);
            dgs += __shfl_xor(dgs, 32, kWave);
            if (h == 0 && r < n) {
                const int pm = (int)cur.poff + r, ps = pm + n;
                const float mu = a.params[pm], sdr = a.params[ps];
                const float sp = softplus_f(sdr), sg = sigmoid_f(sdr);
                float gmean = dgm, gsd = dgs * sg;
                if (a.include_kl) {
                    gmean += mu * a.inv_s0sq;
                    gsd += (sp * a.inv_s0sq - 1.f / sp) * sg;
                    kld += a.log_s0 - logf(sp) + 0.5f * ((sp * sp + mu * mu) * a.inv_s0sq - 1.f);
                }
                float mm = a.m[pm], vv = a.v[pm];
                const float mun = adam_apply(a.adam, mu, gmean, mm, vv);
                a.m[pm] = mm;
                a.v[pm] = vv;
                mm = a.m[ps];
                vv = a.v[ps];
                const float sdn = adam_apply(a.adam, sdr, gsd, mm, vv);
                a.m[ps] = mm;
                a.v[ps] = vv;
                a.params[pm] = mun;
                a.params[ps] = sdn;
                if constexpr (FOLD) {
                    // the band's new mean and softplus(sd) for its combine, on
                    // lines of the band's own, write-through: the combine may
                    // run on another XCD, and the params lines are shared with
                    // the neighbouring bands, whose diagonal tiles and combines
                    // load them (an sc1 load is served by the reader's L2, so a
                    // line another band's reader brought there would be stale)
                    float* const bm = a.bms + 128 * (int64_t)band_id(cur);
                    __hip_atomic_store(bm + 32 * wr + l32, mun, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(bm + 64 + 32 * wr + l32, softplus_f(sdn), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        ph(3);
        // ---- Adam on this wave's two groups, their stores and L' pieces
        const bool rv = r >= 1 && r <= n - 2;
        const float kls = a.include_kl ? a.inv_s0sq : 0.f;
        uint32_t lwo[3][4], lwp[3][4];  // L' pieces [plane][element pair]: K-half hk, the partner's
#pragma unroll
        for (int gi = 0; gi < 2; ++gi) {
            const int g = 2 * hk + gi;
            const int cb = 64 * cur.k + 32 * wc + 8 * g + 4 * h;
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
                const f32x2 pv0 = {P[gi][e], P[gi][e + 1]};
                kl2 = __builtin_elementwise_fma(pv0, pv0, kl2);
                const f32x2 gvv = __builtin_elementwise_fma(pv0, f32x2{kls, kls}, f32x2{dv[4 * gi + e], dv[4 * gi + e + 1]});
                const f32x2 gm = {rv && cb + e < r ? gvv[0] : 0.f, rv && cb + e + 1 < r ? gvv[1] : 0.f};
                f32x2 mm = {M4[gi][e], M4[gi][e + 1]}, vv = {V4[gi][e], V4[gi][e + 1]};
                const f32x2 pv = adam_fast_k2<KIND>(a.adam, pv0, gm, mm, vv);
                P[gi][e] = pv[0];
                P[gi][e + 1] = pv[1];
                M4[gi][e] = mm[0];
                M4[gi][e + 1] = mm[1];
                V4[gi][e] = vv[0];
                V4[gi][e + 1] = vv[1];
                uint32_t w0, w1, w2;
                split3_pk(pv, w0, w1, w2);
                const int jp = (4 * gi + e) >> 1;  // g & 1 == gi
                lwo[0][jp] = w0;
                lwo[1][jp] = w1;
                lwo[2][jp] = w2;
            }
            const uint32_t ob = (uint32_t)((cur.tb + (int64_t)((q * 4 + g) * 64 + lane) * 4) * 4);
            BSTORE128(__builtin_bit_cast(u32x4, P[gi]), rs_t, ob, 0, 16);
            BSTORE128(__builtin_bit_cast(u32x4, M4[gi]), rs_t, ob, tmb, 16);
            BSTORE128(__builtin_bit_cast(u32x4, V4[gi]), rs_t, ob, tvb, 16);
        }
        // the pieces of K-half hk to the partner, its K-half back
#pragma unroll
        for (int p = 0; p < 3; ++p)
            *reinterpret_cast<u32x4*>(Xl + ((wv * 3 + p) * 64 + lane) * 4) =
                u32x4{lwo[p][0], lwo[p][1], lwo[p][2], lwo[p][3]};
        // ---- x' += eps' L'^T for this wave's sample blocks sb = 2 hk + j: its own
        // K-half (st = hk) first, before the partner's pieces are waited for --
        // the SIMD's other wave may still be in its Adam
        auto xprime = [&](int ss, const uint32_t (&lwx)[3][4]) __attribute__((always_inline)) {
            const int st = ss == 0 ? hk : 1 - hk;
            const uint8_t* const rx = En + l32 * 128 + (((2 * (2 * wc + st) + h) ^ xsw) << 4);
            bf8v lb[3];
#pragma unroll
            for (int p = 0; p < 3; ++p)
                lb[p] = __builtin_bit_cast(bf8v, u32x4{lwx[p][0], lwx[p][1], lwx[p][2], lwx[p][3]});
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int sb = 2 * hk + j;
                bf8v fx[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) fx[p] = *reinterpret_cast<const bf8v*>(rx + p * kBfImg + 4096 * sb);
                xacc[j] = mfma6(fx, lb, xacc[j]);
                // the own half issues the next band's G (6..9), the partner's half
                // the next tile's eps' planes (0..5: stg holds the next eps planes
                // until store_col, between the halves)
                {
                    const int q0 = ss == 0 ? 6 + 2 * j : 3 * j, q1 = ss == 0 ? 8 + 2 * j : 3 * j + 3;
#pragma unroll
                    for (int qi = q0; qi < q1; ++qi) issue_b(qi, nxt, has_next, newband, vo_n);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        ph(4);
        xprime(0, lwo);
        __syncthreads();  // B3
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const u32x4 o4 = *reinterpret_cast<const u32x4*>(Xl + ((pw * 3 + p) * 64 + lane) * 4);
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) lwp[p][jp] = o4[jp];
        }
        __syncthreads();  // B4: the exchange scratch read; the eps image is free
        if constexpr (has_next) store_col();  // the next tile's eps image
        xprime(1, lwp);
        ph(5);
        // ---- band end (or run end): the two column halves' x' partials -> the slot
        if constexpr (!has_next || newband) {
            __syncthreads();  // every wave done reading the eps' image (the scratch)
            if (wc == 1) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int qq = 0; qq < 16; ++qq)
                        Xs[(((wr * 2 + hk) * 2 + j) * 16 + qq) * 64 + lane] = xacc[j][qq];
            }
            __syncthreads();
            if (wc == 0) {
                // buffer stores: a scalar slot base, a per-lane 32-bit offset
                const rsrc_t rs_p = make_rsrc(a.part, 0x7fffffff);
                const int sob = __builtin_amdgcn_readfirstlane(slot * S * 64 * 4);
                if constexpr (FOLD) {
                    // fragment order, 16-byte write-through stores (a 4-byte sc1
                    // store is one fabric write each): float4 ((((wr 2 + hk) 2 +
                    // j) 4 + qg) 64 + lane) holds accumulators 4 qg .. 4 qg + 3
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int qg = 0; qg < 4; ++qg) {
                            u32x4 v4;
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                v4[e] = __float_as_uint(xacc[j][4 * qg + e] +
                                                        Xs[(((wr * 2 + hk) * 2 + j) * 16 + 4 * qg + e) * 64 + lane]);
                            BSTORE128(v4, rs_p, (uint32_t)((((((wr * 2 + hk) * 2 + j) * 4 + qg) * 64 + lane)) * 16),
                                      sob, 16);
                        }
                } else {
                    const uint32_t vb = (uint32_t)((32 * wr + l32 + 64 * (64 * hk + 4 * h)) * 4);
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int qq = 0; qq < 16; ++qq) {
                            const int sl = 32 * j + (qq & 3) + 8 * (qq >> 2);  // sample - 64 hk - 4 h
                            const float v = xacc[j][qq] + Xs[(((wr * 2 + hk) * 2 + j) * 16 + qq) * 64 + lane];
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rs_p,
                                                                  vb + (uint32_t)(sl * 256), sob, 0);
                        }
                }
            }
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int qq = 0; qq < 16; ++qq) xacc[j][qq] = 0.f;
            ++slot;
            if constexpr (FOLD) band_arrive();
        }
        ph(6);
        __syncthreads();  // every wave done with the eps' image
        ph(7);
        if constexpr (has_next) store_row();
        if constexpr (newband) {
            split_G();
            __syncthreads();  // the new band's G image written before any wave's dL reads it
        }
        ph(8);
        if (DIAG && wv == 0) ++tph[9];
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    for (int i = t0; i + 1 < t1; ++i) {
        if (++tk > tb_) {
            tk = 0;
            int nbl = a.nb[0];
#pragma unroll
            for (int l = 1; l < kMaxL; ++l)
                if (tl == l) nbl = a.nb[l];
            if (++tb_ == nbl) {
                tb_ = 0;
                ++tl;
            }
        }
        const StrTile nxt = str_tile(a, tl, tb_, tk);
        if (nxt.l != cur.l || nxt.b != cur.b)
            tile(nxt, T_{}, T_{});
        else
            tile(nxt, T_{}, F_{});
        cur = nxt;
    }
    tile(cur, F_{}, F_{});
    if constexpr (FOLD) {
        ph(-1);
        for (int i = 0; i < nfold; ++i) band_combine(__builtin_amdgcn_readfirstlane(fold_list[i]));
        ph(10);  // DIAG: the combines' clocks (stamp slot 12)
    }
    if (DIAG && tid == 0) {
        unsigned long long* o = a.stamps + (size_t)blockIdx.x * 16;
#pragma unroll
        for (int qq = 0; qq < 10; ++qq) o[qq] = tph[qq];
        o[10] = __builtin_amdgcn_s_memtime();
        o[11] = __builtin_amdgcn_s_memrealtime();
        o[12] = tph[10];
    }
    float klp = (kl2[0] + kl2[1]) * (0.5f * a.inv_s0sq) + kld;
    if (a.kl_out && a.include_kl) {
        const float tot = block_sum(klp, Xs);
        if (tid == 0) atomicAdd(a.kl_out, (double)tot);
    }
}

int g_stream_off = 0;  // psvi_debug_set(PSVI_DBG_UPD_STREAM_OFF, 1): the chunked kernel (A/B)
int g_stream_bf_off = 0;  // psvi_debug_set(PSVI_DBG_STREAM_BF_OFF, 1): the fp32-MFMA streaming kernel (A/B)
unsigned long long* g_bf_stamps = nullptr;  // psvi_debug_set_ptr(PSVI_DBG_BF_STAMPS, buf)
int g_ks_off = 0;      // psvi_debug_set(PSVI_DBG_KSTREAM_OFF, 1): the chunked kernel at S > 128 (A/B)
int g_fs_off = 0;      // psvi_debug_set(PSVI_DBG_FWD_SEG_OFF, 1): the item-grid sample kernel at S > 128 (A/B)
int g_ks_bf_off = 0;   // psvi_debug_set(PSVI_DBG_KSTREAM_BF_OFF, 1): the fp32 K-split update (A/B)
int g_fs_bf_off = 0;   // psvi_debug_set(PSVI_DBG_FWD_SEG_BF_OFF, 1): the fp32 segmented sample (A/B)
int g_fwd_pair_bf = 1;  // psvi_debug_set(PSVI_DBG_FWD_PAIR_BF, 0): the HVP's sample pair on the fp32 item grid (A/B)
int g_stream_fold_off = 0;  // psvi_debug_set(PSVI_DBG_STREAM_FOLD_OFF, 1): the band combine as mvn_fwd_reduce_kernel (A/B)

int g_upd_ablation = 0;                      // psvi_debug_set(PSVI_DBG_UPD_ABLATION, mask)
unsigned long long* g_upd_stamps = nullptr;  // psvi_debug_set_ptr(PSVI_DBG_UPD_STAMPS, buf)

static void fill_layers(const psvi_plan& p, MvnLayerArgs* la) {
    for (int l = 0; l < p.L; ++l) {
        la[l].n = p.lay[l].n;
        la[l].poff = p.lay[l].poff;
        la[l].eoff = p.lay[l].eoff;
        la[l].tbase = p.lay[l].tbase;
    }
}

// mvn_fwd_seg_bf_kernel: mvn_fwd_seg_kernel with the GEMM on the bf16 matrix
// cores, fp32-faithful (the pieces of mvn_stream_bf2_kernel): each stage's eps
// block [128 s][64 k] and masked L block [64 r][64 k] are split at staging
// into three bf16 planes each, stored as row images (128-byte rows, 16-byte
// chunk c of row s at c ^ ((s >> 1) & 7)), and both operands read with one
// ds_read_b128 per plane: lane (l32, h) of K-step t takes k = 16 t + 8 h ..
// + 7 of row l32 -- the same k order for A (eps, M = samples) and B (L, N =
// rows), so the accumulators, slots and reduce are mvn_fwd_seg_kernel's.
// 72 KB of LDS: two workgroups per CU, as the fp32 kernel.
//
// PAIR (psvi_hvp's sample pair, launch_mvn_fwd_pair): x = L eps and the
// tangent x2 = Lv eps in one launch on the same segments.  Eight waves: wave
// group g = wv >> 2 stages and multiplies group g's matrix (g 0: params, 1:
// params2) into its own L image and writes its own slots (part / part2); the
// eps stage is shared, each group staging half of its rows.  96 KB of LDS, one
// workgroup per CU (the same eight waves per CU as two single workgroups).
constexpr int kSegEImg = FST * 128;       // bytes per eps plane image
constexpr int kSegLImg = kFwdRows * 128;  // bytes per L plane image
__device__ __forceinline__ int seg_img(int s, int chunk) {
    return s * 128 + ((chunk ^ ((s >> 1) & 7)) << 4);
}
template <bool PAIR>
__global__ __launch_bounds__(PAIR ? 512 : 256, PAIR ? 1 : 2) void mvn_fwd_seg_bf_kernel(FwdArgs a) {
    constexpr int NG = PAIR ? 2 : 1;  // matrices (wave groups)
    __shared__ __attribute__((aligned(16))) uint8_t smb[3 * kSegEImg + NG * 3 * kSegLImg];
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int gw = PAIR ? __builtin_amdgcn_readfirstlane(wave_id() >> 2) : 0;  // wave group
    const int wv = wave_id() & 3, tl = tid & 255;
    const int col4 = tl & 15, srow = tl >> 4;
    uint8_t* const Eb = smb;
    uint8_t* const Lb = smb + 3 * kSegEImg + gw * 3 * kSegLImg;
    constexpr int FT = kFwdRows / 32, LJ = kFwdRows / 16;
    constexpr int EJ = 8 / NG;  // eps rows staged per thread: rows srow + 16 (EJ gw + j)
    const rsrc_t re = make_rsrc(a.eps, 4 * a.e_total);
    const rsrc_t rp = make_rsrc(gw ? a.params2 : a.params, 4 * a.pcount);
    const int sbeg = a.seg_off[blockIdx.x], send = a.seg_off[min((int)blockIdx.x + 1, a.seg_nrun)];
    if (sbeg >= send) return;  // uniform, before any barrier
    // a stage: column block kb of segment si (si == send: past the run's end)
    struct St {
        int si, kb, n, corr, eoff, r0, r1, s0, k1;
    };
    auto stage_at = [&](int si, int kb) __attribute__((always_inline)) {
        St d;
        d.si = si;
        d.kb = kb;
        if (si >= send) return d;
        const FsSeg g = a.segs[si];
        int poff = (int)a.lay[0].poff;
        d.n = a.lay[0].n;
        d.eoff = (int)a.lay[0].eoff;
#pragma unroll
        for (int l = 1; l < kMaxL; ++l)  // select: a dynamic index into the arguments goes to scratch
            if (g.layer == l) {
                d.n = a.lay[l].n;
                d.eoff = (int)a.lay[l].eoff;
                poff = (int)a.lay[l].poff;
            }
        d.corr = poff + 2 * d.n;
        d.r0 = g.r0;
        d.r1 = g.r1;
        d.s0 = g.pass * FST;
        d.k1 = g.k1;
        if (kb < 0) d.kb = g.k0;
        return d;
    };
    auto next = [&](const St& d) __attribute__((always_inline)) {
        return d.kb + FBK < d.k1 ? stage_at(d.si, d.kb + FBK) : stage_at(d.si + 1, -1);
    };
    // two register sets: stage i + 2 is loaded behind stage i's MFMAs
    float4 lreg[2][LJ], ereg[2][EJ];
    auto fetch = [&](const St& d, float4 (&lr)[LJ], float4 (&er)[EJ]) __attribute__((always_inline)) {
        if (d.si >= send) return;  // uniform
#pragma unroll
        for (int j = 0; j < LJ; ++j) {
            const int r = d.r0 + srow + 16 * j;
            const int ro = r >= 1 ? (int)((int64_t)r * (r - 1) / 2) : 0;
            lr[j] = __builtin_bit_cast(
                float4, __builtin_amdgcn_raw_buffer_load_b128(rp, (uint32_t)(d.corr + ro + d.kb + 4 * col4) * 4u, 0, 0));
        }
#pragma unroll
        for (int j = 0; j < EJ; ++j) {
            const int sr = d.s0 + srow + 16 * (EJ * gw + j);
            const uint32_t eo = sr < a.S ? (uint32_t)(d.eoff + sr * d.n + d.kb + 4 * col4) * 4u : kOOB;
            er[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(re, eo, 0, 0));
        }
    };
    // a thread's 4 columns 4 col4 .. + 3: half (col4 & 1) of chunk col4 >> 1
    const int cw = (col4 & 1) * 8;
    auto put = [&](uint8_t* img, int pbytes, int row, float4 v) __attribute__((always_inline)) {
        uint32_t x0[2], x1[2], x2[2];
        split3_pk(f32x2{v.x, v.y}, x0[0], x1[0], x2[0]);
        split3_pk(f32x2{v.z, v.w}, x0[1], x1[1], x2[1]);
        uint8_t* q = img + seg_img(row, col4 >> 1) + cw;
        *reinterpret_cast<u32x2*>(q) = u32x2{x0[0], x0[1]};
        *reinterpret_cast<u32x2*>(q + pbytes) = u32x2{x1[0], x1[1]};
        *reinterpret_cast<u32x2*>(q + 2 * pbytes) = u32x2{x2[0], x2[1]};
    };
    auto stage = [&](const St& d, const float4 (&lr)[LJ], const float4 (&er)[EJ]) __attribute__((always_inline)) {
        const int c = d.kb + 4 * col4;
#pragma unroll
        for (int j = 0; j < LJ; ++j) {
            // entries outside the block's rows / the strict lower triangle are 0
            const int r = d.r0 + srow + 16 * j;
            const bool rok = r < d.r1 && r <= d.n - 2;
            const float4 v = lr[j];
            float4 o;
            o.x = rok && c + 0 < r ? v.x : 0.f;
            o.y = rok && c + 1 < r ? v.y : 0.f;
            o.z = rok && c + 2 < r ? v.z : 0.f;
            o.w = rok && c + 3 < r ? v.w : 0.f;
            put(Lb, kSegLImg, srow + 16 * j, o);
        }
#pragma unroll
        for (int j = 0; j < EJ; ++j) put(Eb, kSegEImg, srow + 16 * (EJ * gw + j), er[j]);
    };
    // operand bases: A row 32 wv + l32 of the eps image, B rows 32 t + l32 of
    // the L image; K-step t, half h -> chunk 2 t + h (the swizzle of row s
    // depends on s alone: (s >> 1) & 7 = (l32 >> 1) & 7 for both)
    const int sw = (l32 >> 1) & 7;
    const uint8_t* const ra = Eb + (32 * wv + l32) * 128;
    const uint8_t* const rb = Lb + l32 * 128;
    floatx16 acc[FT];
#pragma unroll
    for (int t = 0; t < FT; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
    St cur = stage_at(sbeg, -1);
    St nx1 = next(cur);
    fetch(cur, lreg[0], ereg[0]);
    fetch(nx1, lreg[1], ereg[1]);
    // one stage with register set P: stage, load the stage after next into P,
    // the MFMAs; at a segment's last stage its slot is written
    auto body = [&](auto P_c) __attribute__((always_inline)) {
        constexpr int P = decltype(P_c)::value;
        __syncthreads();  // previous stage's MFMAs done with the LDS
        stage(cur, lreg[P], ereg[P]);
        __syncthreads();
        const St nx2 = next(nx1);
        fetch(nx2, lreg[P], ereg[P]);
        const bool wave_live = cur.s0 + 32 * wv < a.S;
        if (wave_live) {
#pragma unroll
            for (int t = 0; t < FBK / 16; ++t) {
                const int co = ((2 * t + h) ^ sw) << 4;
                bf8v av[3], bv[FT][3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    av[p] = *reinterpret_cast<const bf8v*>(ra + p * kSegEImg + co);
#pragma unroll
                    for (int u = 0; u < FT; ++u)
                        bv[u][p] = *reinterpret_cast<const bf8v*>(rb + p * kSegLImg + 32 * 128 * u + co);
                }
#pragma unroll
                for (int u = 0; u < FT; ++u) acc[u] = mfma6(av, bv[u], acc[u]);
            }
        }
        if (nx1.si != cur.si) {  // uniform: the segment's last stage
            // the accumulators in fragment order, as mvn_fwd_seg_kernel
            if (wave_live) {
                const FsSeg g = a.segs[cur.si];
                float* slot = (gw ? a.part2 : a.part) + (size_t)g.slot * FST * kFwdRows + (size_t)wv * FT * 16 * 64 + lane;
#pragma unroll
                for (int t = 0; t < FT; ++t)
#pragma unroll
                    for (int q = 0; q < 16; ++q) slot[(t * 16 + q) * 64] = acc[t][q];
            }
#pragma unroll
            for (int t = 0; t < FT; ++t)
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
        }
        cur = nx1;
        nx1 = nx2;
    };
    for (;;) {  // uniform
        body(std::integral_constant<int, 0>{});
        if (cur.si >= send) break;
        body(std::integral_constant<int, 1>{});
        if (cur.si >= send) break;
    }
}

// packed <-> tiled corr / m / v: one workgroup per 64 x 64 tile.  The tile's
// 64 row segments are contiguous in the packed triangle (row r from poff + 2n +
// r (r - 1) / 2, columns c < r): they go through LDS (row stride 65) between
// row-major packed accesses and float4 fragment-order tiled accesses
// (fragment float4 q = (w * 4 + g) * 64 + lane holds row 32 (w >> 1) + (lane
// & 31), columns 32 (w & 1) + 8 g + 4 (lane >> 5) + 0..3).  Entries outside
// the triangle (or rows 0, n - 1) are zero in the tiled copy.
struct ConvArgs {
    float* pad[3];      // nullable: 64 floats to zero each (the inner loop's eps / G pads)
    float* params;
    float* m;
    float* v;
    float* tstate;      // [3][tiles_total * 4096]: p, m, v
    int64_t tfloats;    // tiles_total * 4096
    int L;
    MvnLayerArgs lay[kMaxL];
};

template <bool TO_TILED>
__global__ __launch_bounds__(256) void mvn_tile_convert_kernel(ConvArgs c) {
    __shared__ float T[64 * 65];
    const int tid = threadIdx.x;
    const int64_t tile = blockIdx.x;
    if (TO_TILED && tile == 0 && tid < 192 && c.pad[tid >> 6]) c.pad[tid >> 6][tid & 63] = 0.f;
    int l = 0;
#pragma unroll
    for (int j = 1; j < kMaxL; ++j)
        if (j < c.L && tile >= c.lay[j].tbase) l = j;
    int n = c.lay[0].n;
    int64_t poff = c.lay[0].poff, tbase = c.lay[0].tbase;
#pragma unroll
    for (int j = 1; j < kMaxL; ++j)
        if (j == l) {
            n = c.lay[j].n;
            poff = c.lay[j].poff;
            tbase = c.lay[j].tbase;
        }
    const int64_t tb = tile - tbase;
    int b = (int)((sqrtf(8.f * (float)tb + 1.f) - 1.f) * 0.5f);
    while ((int64_t)(b + 1) * (b + 2) / 2 <= tb) ++b;
    while ((int64_t)b * (b + 1) / 2 > tb) --b;
    const int k = (int)(tb - (int64_t)b * (b + 1) / 2);
    // row-major side: thread -> (row 16 pass + tid / 16, columns 4 (tid % 16) + 0..3)
    const int cq = 4 * (tid & 15);
    // fragment side: thread -> float4 q = tid + 256 j
    float* arr[3] = {c.params, c.m, c.v};
#pragma unroll 1
    for (int ai = 0; ai < 3; ++ai) {
        float* A = arr[ai];
        float4* tt = reinterpret_cast<float4*>(c.tstate + ai * c.tfloats + tile * 4096);
        if (TO_TILED) {
#pragma unroll
            for (int ps = 0; ps < 4; ++ps) {
                const int i = 16 * ps + (tid >> 4), r = 64 * b + i;
                const bool rv = r >= 1 && r <= n - 2;
                const int64_t rowp = poff + 2 * (int64_t)n + (int64_t)r * (r - 1) / 2 + 64 * k;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int cc = 64 * k + cq + e;
                    T[i * 65 + cq + e] = rv && cc < r ? A[rowp + cq + e] : 0.f;
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int q = tid + 256 * j, w = q >> 8, g = (q >> 6) & 3, lane = q & 63;
                const int i = 32 * (w >> 1) + (lane & 31), c0 = 32 * (w & 1) + 8 * g + 4 * (lane >> 5);
                tt[q] = make_float4(T[i * 65 + c0], T[i * 65 + c0 + 1], T[i * 65 + c0 + 2],
                                    T[i * 65 + c0 + 3]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int q = tid + 256 * j, w = q >> 8, g = (q >> 6) & 3, lane = q & 63;
                const int i = 32 * (w >> 1) + (lane & 31), c0 = 32 * (w & 1) + 8 * g + 4 * (lane >> 5);
                const float4 v4 = tt[q];
                T[i * 65 + c0] = v4.x;
                T[i * 65 + c0 + 1] = v4.y;
                T[i * 65 + c0 + 2] = v4.z;
                T[i * 65 + c0 + 3] = v4.w;
            }
            __syncthreads();
#pragma unroll
            for (int ps = 0; ps < 4; ++ps) {
                const int i = 16 * ps + (tid >> 4), r = 64 * b + i;
                const bool rv = r >= 1 && r <= n - 2;
                const int64_t rowp = poff + 2 * (int64_t)n + (int64_t)r * (r - 1) / 2 + 64 * k;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (rv && 64 * k + cq + e < r) A[rowp + cq + e] = T[i * 65 + cq + e];
            }
        }
        __syncthreads();  // T reused by the next array
    }
}

hipError_t launch_mvn_tile_convert(const psvi_plan& p, float* params, float* m, float* v,
                                   float* tstate, bool to_tiled, hipStream_t st, float* const* pads) {
    ConvArgs c{};
    for (int i = 0; i < 3; ++i) c.pad[i] = pads ? pads[i] : nullptr;
    c.params = params;
    c.m = m;
    c.v = v;
    c.tstate = tstate;
    c.tfloats = p.tiles_total * 4096;
    c.L = p.L;
    fill_layers(p, c.lay);
    if (c.tfloats == 0) return hipSuccess;
    const dim3 grid((unsigned)p.tiles_total);
    if (to_tiled)
        hipLaunchKernelGGL(mvn_tile_convert_kernel<true>, grid, dim3(256), 0, st, c);
    else
        hipLaunchKernelGGL(mvn_tile_convert_kernel<false>, grid, dim3(256), 0, st, c);
    return hipGetLastError();
}

// Workgroups per forward item along the samples: the items (row blocks x
// column chunks of the rank's rows) run their FST-sample passes in parallel
// when they alone would leave the chip's 2 x 256 workgroup slots idle -- the
// K = S >> 128 shapes (a rank's rows for all S = 1024 samples at 8 ranks, C4
// on one GPU); every (item, sample) partial still has one writer.
static int fwd_sample_blocks(const psvi_plan& p, int pairs = 1) {
    const int nsb = (p.d.S + FST - 1) / FST;
    const int want = (512 + p.n_fwd * pairs - 1) / (p.n_fwd * pairs);
    return std::max(1, std::min(nsb, want));
}

hipError_t launch_mvn_fwd(const psvi_plan& p, const float* eps, const float* params,
                          float* x_shard, hipStream_t st, const float* diag_of) {
    FwdArgs a{};
    a.diag_of = diag_of;
    a.items = p.d_fwd;
    a.params = params;
    a.eps = eps;
    a.part = p.d_fwd_part;
    a.ldx = p.rows_tot[p.rank];
    a.S = p.d.S;
    a.e_total = p.Peps;
    a.abl = g_fwd_ablation;
    a.stamps = g_fwd_stamps;
    fill_layers(p, a.lay);
    if (p.n_fswg > 0 && !g_fs_off) {
        // K = S > 128: the segmented sample, then the (row block, pass) reduce
        a.segs = p.d_fs_segs;
        a.seg_off = p.d_fs_off;
        a.pcount = p.P;
        a.part = p.d_fs_part;
        a.slot_rows = FST;
        a.slot_frag = 1;
        a.seg_nrun = p.n_fswg;
        a.abl = 0;
        if (g_fs_bf_off || a.stamps)
            hipLaunchKernelGGL(mvn_fwd_seg_kernel, dim3(p.n_fswg), dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL(mvn_fwd_seg_bf_kernel<false>, dim3(p.n_fswg), dim3(256), 0, st, a);
        hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_fs_rb, FST / kRedSpb), dim3(256), 0, st,
                           p.d_fs_rb, p.d_fs_part, a, x_shard);
        return hipGetLastError();
    }
    if (p.n_fwd == 0) return hipSuccess;
    // every x element is written by exactly one reduce thread: no memset
    hipLaunchKernelGGL(mvn_fwd_kernel, dim3(p.n_fwd, 1, fwd_sample_blocks(p)), dim3(256), 0, st, a);
    constexpr int spb = kRedSpb;  // samples per reduce workgroup
    hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_frb, (a.S + spb - 1) / spb), dim3(256), 0,
                       st, p.d_frb, p.d_fwd_part, a, x_shard);
    return hipGetLastError();
}

// x = mean + L eps (params) and x2 = its HVP tangent, v_mean + Lv eps with the
// diagonal from params (vec), in one launch of each kernel: the items of the
// two GEMMs share eps through L2 and fill the chip together (psvi_hvp)
hipError_t launch_mvn_fwd_pair(const psvi_plan& p, const float* eps, const float* params,
                               float* x, const float* vec, float* x2, float* part2,
                               hipStream_t st) {
    if (p.n_fpwg > 0 && !g_fs_off && !g_fs_bf_off && g_fwd_pair_bf) {
        // the segmented sample's units over the pair table (256 workgroups of
        // eight waves), both matrices per unit (the eps stage shared), then the
        // pair reduce over the two slot sets.  Measured at C3: 25.4 + 7.5 us
        // against the fp32 item grid's 39.2 + 7.9 (psvi_hvp 0.120 -> 0.107 ms);
        // the two bf16-piece samples one after the other took 2 x (20.1 + 6.8),
        // the pair on the sample's 512-run table (two runs per workgroup) 29.5 + 9.3
        FwdArgs a{};
        a.params = params;
        a.eps = eps;
        a.params2 = vec;
        a.diag_of2 = params;
        a.part = p.d_fs_part;
        a.part2 = part2;
        a.ldx = p.rows_tot[p.rank];
        a.S = p.d.S;
        a.e_total = p.Peps;
        a.segs = p.d_fp_segs;
        a.seg_off = p.d_fp_off;
        a.pcount = p.P;
        a.slot_rows = FST;
        a.slot_frag = 1;
        a.seg_nrun = p.n_fpwg;
        fill_layers(p, a.lay);
        hipLaunchKernelGGL(mvn_fwd_seg_bf_kernel<true>, dim3(p.n_fpwg), dim3(512), 0, st, a);
        hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_fp_rb, FST / kRedSpb, 2), dim3(256), 0, st, p.d_fp_rb,
                           p.d_fs_part, a, x, x2);
        return hipGetLastError();
    }
    FwdArgs a{};
    a.items = p.d_fwd;
    a.params = params;
    a.eps = eps;
    a.part = p.d_fwd_part;
    a.params2 = vec;
    a.part2 = part2;
    a.diag_of2 = params;
    a.ldx = p.rows_tot[p.rank];
    a.S = p.d.S;
    a.e_total = p.Peps;
    a.abl = g_fwd_ablation;
    fill_layers(p, a.lay);
    if (p.n_fwd == 0) return hipSuccess;
    hipLaunchKernelGGL(mvn_fwd_kernel, dim3(p.n_fwd, 2, fwd_sample_blocks(p, 2)), dim3(256), 0, st, a);
    constexpr int spb = kRedSpb;
    hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_frb, (a.S + spb - 1) / spb, 2), dim3(256),
                       0, st, p.d_frb, p.d_fwd_part, a, x, x2);
    return hipGetLastError();
}

template <int NS>
static void launch_stream_ns(int kind, dim3 g, dim3 bl, hipStream_t st, const StrArgs& b, bool pad) {
    if (pad && kind == PSVI_ADAM_HIGHER)
        hipLaunchKernelGGL((mvn_stream_kernel<NS, PSVI_ADAM_HIGHER, false, true, true>), g, bl, 0, st, b);
    else if (pad)
        hipLaunchKernelGGL((mvn_stream_kernel<NS, PSVI_ADAM_HYPERGRAD, false, true, true>), g, bl, 0, st, b);
    else if (kind == PSVI_ADAM_HIGHER)
        hipLaunchKernelGGL((mvn_stream_kernel<NS, PSVI_ADAM_HIGHER>), g, bl, 0, st, b);
    else
        hipLaunchKernelGGL((mvn_stream_kernel<NS, PSVI_ADAM_HYPERGRAD>), g, bl, 0, st, b);
}
// the trainers' variants (higher / hypergrad Adam) at S = 128 (C3 and the
// sharded C4 per-GPU count); other S take the chunked kernel (the stream
// kernel's narrower instantiations spilled their scalar registers to scratch)
static bool stream_ok(int S, int kind) {
    return S == 128 && (kind == PSVI_ADAM_HIGHER || kind == PSVI_ADAM_HYPERGRAD);
}
static void launch_stream(int ns, int kind, dim3 g, dim3 bl, hipStream_t st, const StrArgs& b,
                          bool pad) {
    (void)ns;
    launch_stream_ns<4>(kind, g, bl, st, b, pad);
}

bool mvn_grad_takes_slots(const psvi_plan& p) {
    return p.n_kwg > 0 && !g_ks_off && !g_ks_bf_off;
}

hipError_t launch_mvn_update(const psvi_plan& p, const float* eps, const float* g_shard,
                             float* params, float* m, float* v, const psvi_adam_hp* hp,
                             double* kl_out, float* grad_out, int include_kl,
                             const float* eps_next, float* x_next, hipStream_t st,
                             float* tstate, bool packed_out, const float* kl_vec, bool padded,
                             const uint16_t* eps_planes, const uint16_t* eps_next_planes,
                             const float* g_shard2) {
    UpdArgs a{};
    a.kl_vec = kl_vec;
    a.chunks = p.d_upd;
    a.eps = eps;
    a.g = g_shard;
    a.ldg = p.rows_tot[p.rank];
    a.S = p.d.S;
    a.g_total = (int64_t)p.d.S * p.rows_tot[p.rank];
    a.e_total = p.Peps;
    a.params = params;
    a.m = m;
    a.v = v;
    a.grad_out = grad_out;
    a.kl_out = kl_out;
    a.include_kl = include_kl;
    a.abl = g_upd_ablation;
    a.stamps = g_upd_stamps;
    a.pcount = p.P;
    const float s0 = p.d.prior_sd;
    a.inv_s0sq = 1.f / (s0 * s0);
    a.log_s0 = logf(s0);
    if (hp) a.adam = make_adam(hp);
    fill_layers(p, a.lay);
    if (p.n_upd == 0) return hipSuccess;
    const dim3 grid(p.n_upd), block(256);
    const int mode = a.S > USB ? 2 : a.S > UEH ? 1 : 0;  // samples per LDS pass
    if (tstate) {
        // tiled state (psvi_inner_loop on a fusable plan): corr / m / v in tstate
        const int64_t tf = p.tiles_total * 4096;
        a.tp = tstate;
        a.tm = tstate + tf;
        a.tv = tstate + 2 * tf;
        if (eps_next && p.n_str > 0 && g_stream_off != 1 && stream_ok(a.S, a.adam.kind)) {
            StrArgs b{};
            b.ranges = p.d_str;
            b.eps = eps;
            b.eps_next = eps_next;
            b.g = g_shard;
            b.ldg = a.ldg;
            b.S = a.S;
            b.g_total = a.g_total;
            b.e_total = a.e_total;
            b.params = params;
            b.m = m;
            b.v = v;
            b.tp = a.tp;
            b.tm = a.tm;
            b.tv = a.tv;
            b.part = p.d_str_part;
            b.kl_out = kl_out;
            b.include_kl = include_kl;
            b.stamps = g_upd_stamps;
            b.inv_s0sq = a.inv_s0sq;
            b.log_s0 = a.log_s0;
            b.adam = a.adam;
            for (int l = 0; l < p.L; ++l) {
                b.xcol[l] = p.xcol_l[p.rank][l];
                b.nb[l] = p.lay[l].nb;
            }
            fill_layers(p, b.lay);
            const dim3 sg(p.n_str);
            const bool bf = eps_planes && eps_next_planes && p.bf_stream && padded && !g_stream_bf_off;
            if (bf) {
                b.stamps = g_bf_stamps;
                // both products on the bf16 matrix cores (fp32-faithful pieces)
                b.ep = eps_planes;
                b.enp = eps_next_planes;
                b.pl = p.eps_planes.pl;
                for (int l = 0; l < p.L; ++l) {
                    b.ppoff[l] = p.eps_planes.poff[l];
                    b.npad[l] = p.eps_planes.npad[l];
                }
                const dim3 b8(512);
                const bool fold = p.d_str_cnt && p.d_str_bms && p.str_max_ends <= kFoldMax && !g_stream_fold_off;
                b.rbs = p.d_sfrb;
                b.bcnt = p.d_str_cnt;
                b.bms = p.d_str_bms;
                b.x = x_next;
                b.ldx = p.rows_tot[p.rank];
                if (fold && b.stamps && b.adam.kind == PSVI_ADAM_HIGHER)
                    hipLaunchKernelGGL((mvn_stream_bf2_kernel<PSVI_ADAM_HIGHER, true, true>), sg, b8, 0, st, b);
                else if (fold && b.adam.kind == PSVI_ADAM_HIGHER)
                    hipLaunchKernelGGL((mvn_stream_bf2_kernel<PSVI_ADAM_HIGHER, false, true>), sg, b8, 0, st, b);
                else if (fold)
                    hipLaunchKernelGGL((mvn_stream_bf2_kernel<PSVI_ADAM_HYPERGRAD, false, true>), sg, b8, 0, st, b);
                else if (b.adam.kind == PSVI_ADAM_HIGHER)
                    hipLaunchKernelGGL(mvn_stream_bf2_kernel<PSVI_ADAM_HIGHER>, sg, b8, 0, st, b);
                else
                    hipLaunchKernelGGL(mvn_stream_bf2_kernel<PSVI_ADAM_HYPERGRAD>, sg, b8, 0, st, b);
                if (fold) return hipGetLastError();
            } else if (b.stamps && a.S == 128 && b.adam.kind == PSVI_ADAM_HIGHER)
                hipLaunchKernelGGL((mvn_stream_kernel<4, PSVI_ADAM_HIGHER, true>), sg, block, 0, st, b);
            else
                launch_stream(a.S / 32, b.adam.kind, sg, block, st, b, padded);
            FwdArgs f{};
            f.params = params;
            f.eps = eps_next;
            f.ldx = p.rows_tot[p.rank];
            f.S = p.d.S;
            fill_layers(p, f.lay);
            constexpr int spb = kRedSpb;
            hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_sfrb, (f.S + spb - 1) / spb),
                               dim3(256), 0, st, p.d_sfrb, p.d_str_part, f, x_next);
            return hipGetLastError();
        }
        if (eps_next) {
            a.eps_next = eps_next;
            a.part = p.d_upd_part;
            if (mode == 1) hipLaunchKernelGGL((mvn_update_kernel<false, 1, true, true>), grid, block, 0, st, a);
            else hipLaunchKernelGGL((mvn_update_kernel<false, 0, true, true>), grid, block, 0, st, a);
            FwdArgs f{};
            f.params = params;
            f.eps = eps_next;
            f.ldx = p.rows_tot[p.rank];
            f.S = p.d.S;
            fill_layers(p, f.lay);
            constexpr int spb = kRedSpb;
            hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_ufrb, (f.S + spb - 1) / spb),
                               dim3(256), 0, st, p.d_ufrb, p.d_upd_part, f, x_next);
        } else if (packed_out) {
            if (mode == 1) hipLaunchKernelGGL((mvn_update_kernel<false, 1, false, true, true>), grid, block, 0, st, a);
            else hipLaunchKernelGGL((mvn_update_kernel<false, 0, false, true, true>), grid, block, 0, st, a);
        } else {
            if (mode == 1) hipLaunchKernelGGL((mvn_update_kernel<false, 1, false, true>), grid, block, 0, st, a);
            else hipLaunchKernelGGL((mvn_update_kernel<false, 0, false, true>), grid, block, 0, st, a);
        }
        return hipGetLastError();
    }
    // gradient mode (the HVP's J^T G_dot) at any S on the bf16-piece K-split kernel
    const bool ks_grad = grad_out && mvn_grad_takes_slots(p);
    if (g_shard2 && !ks_grad) return hipErrorInvalidValue;
    if ((mode == 2 && !grad_out && p.n_kwg > 0 && g_ks_off != 1) || ks_grad) {
        // K = S > 128: the K-split streaming update (then the next step's
        // sample from the new parameters when asked)
        KsArgs k{};
        k.tiles = p.d_ks_tiles;
        k.segs = p.d_ks_segs;
        k.seg_off = p.d_ks_off;
        k.slots = p.d_ks_slots;
        k.cnt = p.d_ks_cnt;
        k.slot_bytes = (int64_t)sizeof(float) * std::max(1, p.n_ks_slots) * kKsSlotFloats;
        k.eps = eps;
        k.g = g_shard;
        k.ldg = a.ldg;
        k.S = a.S;
        k.g_total = a.g_total;
        k.e_total = a.e_total;
        k.params = params;
        k.m = m;
        k.v = v;
        k.kl_out = kl_out;
        k.pcount = p.P;
        k.include_kl = include_kl;
        k.inv_s0sq = a.inv_s0sq;
        k.log_s0 = a.log_s0;
        k.adam = a.adam;
        k.stamps = g_upd_stamps;
        k.grad_out = grad_out;
        k.kl_vec = kl_vec;
        k.g2 = g_shard2;
        fill_layers(p, k.lay);
        if (ks_grad)
            hipLaunchKernelGGL((mvn_kstream_kernel<true, true>), dim3(p.n_kwg), block, 0, st, k);
        else if (g_ks_bf_off || k.stamps)
            hipLaunchKernelGGL(mvn_kstream_kernel<false>, dim3(p.n_kwg), block, 0, st, k);
        else
            hipLaunchKernelGGL(mvn_kstream_kernel<true>, dim3(p.n_kwg), block, 0, st, k);
        if (eps_next) {
            const hipError_t e = hipGetLastError();
            return e != hipSuccess ? e : launch_mvn_fwd(p, eps_next, params, x_next, st);
        }
        return hipGetLastError();
    }
    if (eps_next && !grad_out) {
        if (!(p.fuse_sample && mode < 2)) {
            // no fusion for this plan: update, then sample from the new params
            hipError_t e = launch_mvn_update(p, eps, g_shard, params, m, v, hp, kl_out, nullptr,
                                             include_kl, nullptr, nullptr, st, nullptr);
            return e != hipSuccess ? e : launch_mvn_fwd(p, eps_next, params, x_next, st);
        }
        a.eps_next = eps_next;
        a.part = p.d_upd_part;
        if (mode == 1) hipLaunchKernelGGL((mvn_update_kernel<false, 1, true>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((mvn_update_kernel<false, 0, true>), grid, block, 0, st, a);
        // x_next = mean' + softplus(sd') eps_next + sum of the band's chunk slots
        FwdArgs f{};
        f.params = params;
        f.eps = eps_next;
        f.ldx = p.rows_tot[p.rank];
        f.S = p.d.S;
        fill_layers(p, f.lay);
        constexpr int spb = kRedSpb;
        hipLaunchKernelGGL(mvn_fwd_reduce_kernel, dim3(p.n_ufrb, (f.S + spb - 1) / spb), dim3(256),
                           0, st, p.d_ufrb, p.d_upd_part, f, x_next);
        return hipGetLastError();
    }
    if (grad_out) {
        if (mode == 2) hipLaunchKernelGGL((mvn_update_kernel<true, 2>), grid, block, 0, st, a);
        else if (mode == 1) hipLaunchKernelGGL((mvn_update_kernel<true, 1>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((mvn_update_kernel<true, 0>), grid, block, 0, st, a);
    } else {
        if (mode == 2) hipLaunchKernelGGL((mvn_update_kernel<false, 2>), grid, block, 0, st, a);
        else if (mode == 1) hipLaunchKernelGGL((mvn_update_kernel<false, 1>), grid, block, 0, st, a);
        else hipLaunchKernelGGL((mvn_update_kernel<false, 0>), grid, block, 0, st, a);
    }
    return hipGetLastError();
}

}  // namespace psvi
