// kernels_net.hip -- per-(sample, role, pseudopoint-chunk) MLP forward + weighted
// NLL + hand-derived backward, for both VI families.
//
// Reference (psvi/..., /root/reference):
//   VILinear.forward        models/neural_net.py:176-179   a = h W_s^T + b_s
//   VILinearMultivariateNormal.forward  neural_net.py:485-491 (W_s, b_s split of x_s)
//   ReLU                    make_fcnet 288 / make_fc2net 515
//   Categorical(logits).log_prob(z) .matmul(N f(v))  inference/psvi_classes.py:496-505
// Backward: g = w_m (softmax - onehot); dW_s = g^T h;
// db_s = sum_m g; g <- (g W_s) * 1[a > 0].
//
// One workgroup = one MC sample x one ROLE x one chunk of pseudopoints.
// When a rank has fewer samples than CUs, each sample gets two workgroups
// with different roles instead of a split of its pseudopoints: both run the
// forward pass and the loss head; role 0 then produces layer 0's weight
// gradient (and the gradient chain down to it), role 1 every other layer's.
// Each gradient element has exactly one writer -- plain stores into g_send,
// no zeroing pass, no atomics, deterministic.  (Full-cov pseudopoint chunks --
// shapes whose buffers exceed the LDS, ranks with very few samples -- store
// their partial dW into per-chunk slots of the plan, added in chunk order.)
// Mean-field: every (sample, chunk) stores its gradient into its own slot of
// the plan's d_mf_slots; mf_update_kernel sums the slots in a fixed order
// (against eps for the rho accumulator), so the step is bitwise reproducible.
//
// LDS holds everything a workgroup touches.  Every matrix is row-major with
// a row stride == 8 (mod 16) floats, and every GEMM operand is read without
// bank conflicts: a k-contiguous operand as one ds_read_b128 per lane (the
// 16-lane groups of ds_read_b128 then cover 16 distinct 16-byte slots), a
// k-strided one as ds_read_b32 with the k order of kbase/kstep (the two
// lane-groups of a 32-lane half two rows apart).  The forward GEMM reads X_l
// and W_l along k; the propagation GEMM reads G_l along k and a transposed
// copy W_l^T (written with W_l); the weight-gradient GEMM reads G_l and X_l
// down k.  Contractions run on v_mfma_f32_16x16x4_f32 tiles (exact fp32)
// with double-buffered operand reads, tiles dealt round-robin to the waves
// (wave w sits on SIMD w % 4).
// Padding contract: W rows / columns past dout / din are zero; activation and
// gradient rows past the chunk's pseudopoints are zero and their columns up
// to the next multiple of 16 (within the row stride) too (epilogues write
// them); a k-loop that runs past a row's end reads the next row's (finite)
// values against zero weights; every region is followed by zeroed slack.
// Forward, loss head and gradient propagation are row-local: each wave
// carries whole 16-row tiles through them with no workgroup barrier (the
// row chain), and the weight gradients -- sums over every row -- follow one
// barrier.  The loss head runs in the head GEMM's epilogue (C <= 16: a row's
// logits on a DPP row), else on VALU, one lane per row.  Weight gradients
// leave straight from the MFMA accumulators.
#include <algorithm>

#include "mfma_tiles.hpp"
#include "psvi_internal.hpp"

namespace psvi {

struct NetArgs {
    int L, M, mc, S_total, s_goff, nroles, Mp;
    float* gslot;   // full-cov, pseudopoint chunks > 1: chunk z's partial dW into slot z
    int64_t gsz;    // floats per slot (= the g_send buffer)
    int abl;  // diagnostics ablation mask (0 in production): 1 loads, 2 fwd
              // GEMMs, 4 loss head, 8 bwd GEMMs, 16 global gradient writes
    unsigned long long* stamps;  // diagnostics: s_memtime per phase (nullptr in production)
    int din[kMaxL], dout[kMaxL], woff[kMaxL];
    // LDS carve (float offsets) and row strides: W_l, b_l, X_l (input of layer l:
    // X_0 = u chunk, X_l = relu(a_{l-1})), two gradient buffers, dlogits
    int lw[kMaxL], ldw[kMaxL], lb[kMaxL], lx[kMaxL], ldx[kMaxL];
    int lwt[kMaxL], ldwt[kMaxL];  // W_l^T (l >= 1: the propagation GEMM's k-contiguous operand)
    int lg[kMaxL], ldl, lddl, lred, lsrc, lzw, lstamp, lds_f4;  // lg[l]: G_l (l < L-1); ldl: dlogits [Mp][lddl]; lzw: z, w
    int nslack, nslack_early, slack[5 * kMaxL + 8];  // kNetSlack  // float offsets of the 64-float zero slacks
    int stage_len, stage_off[kMaxWorld + 1];  // FULLCOV: this sample's x row, source blocks back to back
    const float* u;
    const int32_t* z;
    const float* w;
    double* nll_out;   // fp64 accumulator (many similar-size adds)
    // MEANFIELD
    const float* params;
    const float* eps;
    int64_t poff[kMaxL], eoff[kMaxL];
    // per-(sample, pseudopoint chunk) gradient slots [S_loc][gridDim.z][slot_ld]
    // (the plan's d_mf_slots): one plain store per element, summed by the update
    float* mf_slots;
    int slot_ld;
    // fused next-step draw (psvi_inner_loop): normals [0, rn_n) of the Philox
    // stream (rn_seed, rn_off) into rn_out, split over the grid's workgroups
    float* rn_out;
    int64_t rn_n;
    uint64_t rn_seed, rn_off;
    // FULLCOV (blocked by source rank)
    const float* xrecv;
    float* gsend;
    // outer objective (psvi_outer_elbo_grad, world 1): 0 = the inner ELBO;
    // 1 = forward only, NLL of every row -> nll_rows [S][M] (no weighting, no
    // backward); 2 = backward of sum_{s,m} coef_sm NLL_sm with coef_sm =
    // w_m * rowcoef[s][m >= n_pseudo], plus the sampled-KL path term
    // -ck_s x_s / s0^2 on every weight gradient, and (du_part) the input
    // gradient of the pseudopoint rows [S][n_pseudo][D]
    int outer, n_pseudo;
    float inv_s0sq;
    float* nll_rows;
    const float* rowcoef;
    const float* ck;
    float* du_part;
    float* prob_rows;  // outer forward (evaluate): softmax of the data rows [S][M - n_pseudo][C]
    int nsrc;
    int64_t src_base[kMaxWorld];
    int src_stride[kMaxWorld];
    int xcol0[kMaxL];         // one source: x / g column of layer l's row 0
    int src_chunk0[kMaxWorld + 1];  // several sources, float4 loads: first chunk of each source block
    // FULLCOV: LDS destination of x row position r (stage order: source blocks
    // back to back, each in its x-shard column order): W_l / b_l float offset
    // in the low 16 bits, W_l^T offset (0xFFFF: none) in the high 16
    const uint32_t* xmap;
    // several sources: the gradient of row r of layer l goes to
    // bands[bbase[l] + r / 64].base + s * .stride + r in g_send
    const NetBand* bands;
    int nbands, bbase[kMaxL];
    int mloop;  // pseudopoint chunks looped inside one workgroup (1: none)
    // this launch's local samples [s_begin, s_begin + gridDim.x) (the sharded
    // loop's sample halves); the fused draw's part rn_part of rn_nparts
    // contiguous quad ranges
    int s_begin, rn_part, rn_nparts;
    // the fused draw also as bf16 planes (the bf16-plane streaming update)
    const EpsPlanes* rn_P;
    uint16_t* rn_planes;
};

// ---- LDS carve (float offsets, row strides) of the network kernel.  Row
// strides are 4 x odd (== 8 mod 16): a 16-lane float4 read along k (rows i16
// = 0..15) and a 64-lane float read down k (lanes 16 k4 + i16, rows 4 k4
// apart) both hit distinct banks.  Regions read before the forward pass come
// first; every region is followed by a 64-float zero slack.
constexpr int kNetSlack = 5 * kMaxL + 8;
struct NetDims {
    int L;
    int din[kMaxL], dout[kMaxL];
};
struct NetCarve {
    int lw[kMaxL], ldw[kMaxL], lb[kMaxL], lx[kMaxL], ldx[kMaxL], lwt[kMaxL], ldwt[kMaxL],
        lg[kMaxL];
    int ldl, lddl, lred, lsrc, lzw, lstamp, lds_f4, Mp, nslack, nslack_early;
    int slack[kNetSlack];
};
constexpr int net_rup(int x, int m) { return (x + m - 1) / m * m; }
constexpr int net_ld8o(int x) { return x + (24 - x % 16) % 16; }  // >= x, == 8 (mod 16)
// nbands: world > 1 full-cov plans, the band table's entries (per-workgroup
// source tables in LDS); 0 otherwise
constexpr NetCarve net_carve(const NetDims& d, int mc, int nbands) {
    NetCarve c{};
    int off = 0, ns = 0;
    auto take = [&](int nfl) {
        const int o = off;
        off += (nfl + 3) & ~3;
        c.slack[ns] = off;
        ++ns;
        off += 64;
        return o;
    };
    const int Mp = net_rup(mc, 16);
    for (int l = 0; l < d.L; ++l) {
        const int din = d.din[l], dout = d.dout[l];
        const int ldw = net_ld8o(net_rup(din, 16));
        c.lw[l] = take(net_rup(dout, 16) * ldw);
        c.ldw[l] = ldw;
        c.lb[l] = take(dout);
        if (l > 0) {  // W^T: rows i < din (16-multiple), columns j < dout (16-multiple)
            const int ldwt = net_ld8o(net_rup(dout, 16));
            c.lwt[l] = take(net_rup(din, 16) * ldwt);
            c.ldwt[l] = ldwt;
        } else {
            c.lwt[0] = c.lw[0];  // unused (no propagation below layer 0)
            c.ldwt[0] = ldw;
        }
    }
    const int ldx0 = net_ld8o(d.din[0]);
    const int lx0 = take(Mp * ldx0);
    c.lred = take(16);
    c.lzw = take(2 * Mp);
    c.lstamp = take(48);  // 16 x uint64 diagnostics stamps + 8 wave starts
    // per-workgroup tables (world > 1): every band's int64 g_send offset
    // (8-byte aligned), the x row's per-source int64 bases and int starts,
    // the layers' first band index
    c.lsrc = take(2 * nbands + 3 * kMaxWorld + kMaxL + 2 * kMaxWorld + 1);
    c.nslack_early = ns;
    for (int l = 1; l < d.L; ++l) {
        c.ldx[l] = net_ld8o(d.din[l]);
        c.lx[l] = take(Mp * c.ldx[l]);
    }
    // G_l (l < L - 1, the gradient of layer l's output, stride of X_{l+1}):
    // every one stays until the weight-gradient phase
    for (int l = 0; l + 1 < d.L; ++l) c.lg[l] = take(Mp * net_ld8o(d.din[l + 1]));
    c.lddl = net_ld8o(d.dout[d.L - 1]);
    c.ldl = take(Mp * c.lddl);
    off = (off + 3) & ~3;
    c.lx[0] = lx0;
    c.ldx[0] = ldx0;
    c.Mp = Mp;
    c.nslack = ns;
    c.lds_f4 = off / 4;
    return c;
}

// Geometry the kernel reads: GEO 0 the plan's (NetArgs, any stack, at run
// time); GEO 1 / 2 the fn2 stack of configs C3 / C4 (64 -> 40 -> 40 -> 2,
// 100-row pseudopoint chunks: Mp = 112), one source rank / several (the
// band table's 69 entries) -- every layer size, row stride and LDS offset a
// compile-time constant, so layer loops unroll, LDS addresses become
// instruction offsets and no kernel argument is loaded for them.
constexpr NetDims kFn2Dims{3, {64, 40, 40}, {40, 40, 2}};
constexpr int kFn2Mp = 112, kFn2Bands = 41 + 26 + 2;
template <int GEO>
struct NetGeo {
    static constexpr bool kFixed = true;
    static constexpr int kUnroll = kMaxL;
    static constexpr NetCarve C = net_carve(kFn2Dims, kFn2Mp, GEO == 2 ? kFn2Bands : 0);
    // lanes of the loss head's reductions: the smallest power of two >= C
    static constexpr int kHeadLanes = kFn2Dims.dout[kFn2Dims.L - 1] <= 2   ? 2
                                      : kFn2Dims.dout[kFn2Dims.L - 1] <= 4 ? 4
                                                                          : 16;
    __device__ explicit NetGeo(const NetArgs&) {}
    __device__ static constexpr int L() { return kFn2Dims.L; }
    __device__ static constexpr int din(int l) { return kFn2Dims.din[l]; }
    __device__ static constexpr int dout(int l) { return kFn2Dims.dout[l]; }
    __device__ static constexpr int lw(int l) { return C.lw[l]; }
    __device__ static constexpr int ldw(int l) { return C.ldw[l]; }
    __device__ static constexpr int lb(int l) { return C.lb[l]; }
    __device__ static constexpr int lx(int l) { return C.lx[l]; }
    __device__ static constexpr int ldx(int l) { return C.ldx[l]; }
    __device__ static constexpr int lwt(int l) { return C.lwt[l]; }
    __device__ static constexpr int ldwt(int l) { return C.ldwt[l]; }
    __device__ static constexpr int lg(int l) { return C.lg[l]; }
    __device__ static constexpr int slack(int k) { return C.slack[k]; }
    __device__ static constexpr int ldl() { return C.ldl; }
    __device__ static constexpr int lddl() { return C.lddl; }
    __device__ static constexpr int lred() { return C.lred; }
    __device__ static constexpr int lsrc() { return C.lsrc; }
    __device__ static constexpr int lzw() { return C.lzw; }
    __device__ static constexpr int lstamp() { return C.lstamp; }
    __device__ static constexpr int lds_f4() { return C.lds_f4; }
    __device__ static constexpr int Mp() { return C.Mp; }
    __device__ static constexpr int nslack() { return C.nslack; }
};
template <>
struct NetGeo<0> {
    static constexpr bool kFixed = false;
    static constexpr int kUnroll = 1;
    static constexpr int kHeadLanes = 16;
    const NetArgs& a;
    __device__ explicit NetGeo(const NetArgs& args) : a(args) {}
    __device__ int L() const { return a.L; }
    __device__ int din(int l) const { return a.din[l]; }
    __device__ int dout(int l) const { return a.dout[l]; }
    __device__ int lw(int l) const { return a.lw[l]; }
    __device__ int ldw(int l) const { return a.ldw[l]; }
    __device__ int lb(int l) const { return a.lb[l]; }
    __device__ int lx(int l) const { return a.lx[l]; }
    __device__ int ldx(int l) const { return a.ldx[l]; }
    __device__ int lwt(int l) const { return a.lwt[l]; }
    __device__ int ldwt(int l) const { return a.ldwt[l]; }
    __device__ int lg(int l) const { return a.lg[l]; }
    __device__ int slack(int k) const { return a.slack[k]; }
    __device__ int ldl() const { return a.ldl; }
    __device__ int lddl() const { return a.lddl; }
    __device__ int lred() const { return a.lred; }
    __device__ int lsrc() const { return a.lsrc; }
    __device__ int lzw() const { return a.lzw; }
    __device__ int lstamp() const { return a.lstamp; }
    __device__ int lds_f4() const { return a.lds_f4; }
    __device__ int Mp() const { return a.Mp; }
    __device__ int nslack() const { return a.nslack; }
};

// One GEMM's tiles (P x Q outputs rounded up to 16-tiles): units of one
// 16-row tile x NQ column tiles -- a whole row of column tiles (NQ = tq <= 3:
// one A read per NQ MFMAs) when that still gives every SIMD a unit, else
// single tiles.  Unit u goes to wave (u + first) % nwaves, so two GEMMs of
// one phase share the round-robin.  Per unit: the operand pointers are
// formed once, the k-groups run as a two-deep register pipeline (the next
// group's LDS reads issued before the current group's MFMAs) with constant
// pointer steps, and the next unit's first group is read before this unit's
// epilogue.
__device__ __forceinline__ int gemm_nq(int tp, int tq) {
    return (tq <= 3 && tp >= 4) ? tq : 1;
}
__device__ __forceinline__ int gemm_units(int P, int Q) {
    const int tp = (P + 15) >> 4, tq = (Q + 15) >> 4;
    return tp * (tq / gemm_nq(tp, tq));
}
template <bool ACONT, bool BCONT, int NQ, int CARRY = 0, class Epi>
__device__ __forceinline__ void gemm_steps(int nu, int tqu, int K16, int u0, const float* A, int lda,
                                           const float* B, int ldb, Epi epi, int ustep = 0,
                                           int K = 0, floatx4 (*carry)[NQ] = nullptr,
                                           int cmode = 0) {
    // K (row GEMMs, k-contiguous A): the true contraction length, masked in
    // the last k-group; 0 = K16 (no mask)
    // CARRY > 0 (looped pseudopoint chunks, fixed geometry): the wave's units
    // k = 0 .. CARRY - 1 (u = u0 + k nwaves) keep their sums in carry[k]
    // across the chunks -- cmode 1 (first chunk): store the chunk's sums
    // there, no epilogue; 3 (a middle chunk): add them; 2 (the last): the
    // epilogue gets carry[k] + the chunk's sums (the chunks added in chunk
    // order, as the run-time geometry's read-modify-write of g_send does)
    const bool kmask = ACONT && K > 0 && K < K16;  // uniform
    const int nwv = ustep ? ustep : (int)(blockDim.x >> 6), lane = threadIdx.x & 63, i16 = lane & 15,
              k4 = lane >> 4;
    const int nk = K16 >> 4;
    if (u0 >= nu) return;  // wave-uniform
    const int da = ACONT ? 16 : 16 * lda, db = BCONT ? 16 : 16 * ldb;  // one k-group
    const int rot = (k4 & 1) << 1;  // epilogue row rotation: v[r] is row 4 k4 + ((r + rot) & 3)
    auto ptrs = [&](int u, const float*& pa, const float*& pb, int& p0, int& q0) {
        const int pt = u / tqu, qt = (u - pt * tqu) * NQ;
        p0 = pt << 4;
        q0 = qt << 4;
        constexpr bool PERM = !ACONT && !BCONT;
        pa = ACONT ? A + (p0 + i16) * lda + 4 * k4 : A + kbase<PERM>(k4) * lda + p0 + i16;
        pb = BCONT ? B + (q0 + i16) * ldb + 4 * k4 : B + kbase<PERM>(k4) * ldb + q0 + i16;
    };
    const float *pa, *pb;
    int p0, q0;
    ptrs(u0, pa, pb, p0, q0);
    TileOps<ACONT, BCONT, NQ> x0, x1;
    x0.load(pa, lda, pb, ldb);
    // one unit: the k-groups into acc, then the next unit's first group read
    // before the epilogue; returns the unit's first row / column
    auto unit = [&](int u, floatx4 (&acc)[NQ], int& pe, int& qe) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NQ; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
        // x0 holds group 0; two groups per trip with fixed registers (no
        // copies at the back edge, so the reads of the group after next stay
        // in flight across the current group's MFMAs), then a 1- or 2-group tail
        int kg = 0;
        for (; kg + 2 < nk; kg += 2) {
            pa += da;
            pb += db;
            x1.load(pa, lda, pb, ldb);
            x0.mma(acc);
            pa += da;
            pb += db;
            x0.load(pa, lda, pb, ldb);
            x1.mma(acc);
        }
        if (kg + 1 < nk) {
            pa += da;
            pb += db;
            x1.load(pa, lda, pb, ldb);
            x0.mma(acc);
            if (kmask) x1.mask_a(16 * (nk - 1), K);
            x1.mma(acc);
        } else {
            if (kmask) x0.mask_a(16 * (nk - 1), K);
            x0.mma(acc);
        }
        pe = p0;
        qe = q0;
        if (u + nwv < nu) {
            ptrs(u + nwv, pa, pb, p0, q0);
            x0.load(pa, lda, pb, ldb);
        }
    };
    // odd lane-groups hand over their four rows rotated by two: the
    // epilogue's row-wise LDS accesses of the two groups of a 32-lane half
    // are then 2 or 6 rows apart (16 banks at strides == 8 mod 16), not 4
    auto out = [&](const floatx4 (&acc)[NQ], int pe, int qe) __attribute__((always_inline)) {
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            const floatx4 v = acc[c];
            epi(pe + 4 * k4, qe + 16 * c + i16, rot ? floatx4{v[2], v[3], v[0], v[1]} : v, rot);
        }
    };
    if constexpr (CARRY == 0) {
        for (int u = u0; u < nu; u += nwv) {  // wave-uniform
            floatx4 acc[NQ];
            int pe, qe;
            unit(u, acc, pe, qe);
            out(acc, pe, qe);
        }
    } else {
#pragma unroll
        for (int k = 0; k < CARRY; ++k) {
            const int u = u0 + k * nwv;
            if (u >= nu) break;  // wave-uniform
            floatx4 acc[NQ];
            int pe, qe;
            unit(u, acc, pe, qe);
            if (cmode == 1 || cmode == 3) {
#pragma unroll
                for (int c = 0; c < NQ; ++c) carry[k][c] = cmode == 3 ? carry[k][c] + acc[c] : acc[c];
            } else {
                if (cmode == 2) {
#pragma unroll
                    for (int c = 0; c < NQ; ++c) acc[c] = carry[k][c] + acc[c];
                }
                out(acc, pe, qe);
            }
        }
    }
}
template <bool ACONT, bool BCONT, class Epi>
__device__ __forceinline__ void mfma_gemm(int P, int Q, int K, int first, const float* A, int lda,
                                          const float* B, int ldb, Epi epi, int nwaves = 0) {
    // nwaves: the workgroup's waves when known at compile time (0: blockDim)
    const int wid = wave_id(), nwv = nwaves ? nwaves : (int)(blockDim.x >> 6);
    const int tp = (P + 15) >> 4, tq = (Q + 15) >> 4, K16 = (K + 15) & ~15;
    const int u0 = ((wid - first) % nwv + nwv) % nwv;
    switch (gemm_nq(tp, tq)) {
        case 3: gemm_steps<ACONT, BCONT, 3>(tp, 1, K16, u0, A, lda, B, ldb, epi, nwv); break;
        case 2: gemm_steps<ACONT, BCONT, 2>(tp, 1, K16, u0, A, lda, B, ldb, epi, nwv); break;
        default: gemm_steps<ACONT, BCONT, 1>(tp * tq, tq, K16, u0, A, lda, B, ldb, epi, nwv); break;
    }
}

// mfma_gemm with the units' sums carried across looped pseudopoint chunks
// (gemm_steps CARRY): the fixed fn2 geometry's weight gradients, one column
// tile per unit (NQ = 1) and at most CARRY units per wave and layer
template <int CARRY, class Epi>
__device__ __forceinline__ void mfma_gemm_carry(int P, int Q, int K, int first, const float* A,
                                                int lda, const float* B, int ldb, Epi epi,
                                                floatx4 (*carry)[1], int cmode, int nwaves = 0) {
    const int wid = wave_id(), nwv = nwaves ? nwaves : (int)(blockDim.x >> 6);
    const int tp = (P + 15) >> 4, tq = (Q + 15) >> 4, K16 = (K + 15) & ~15;
    const int u0 = ((wid - first) % nwv + nwv) % nwv;
    // (the host gates the fixed geometry to 512 threads: tp tq <= CARRY nwaves
    // for every fn2 layer, and gemm_nq is 1 for all of them)
    gemm_steps<false, false, 1, CARRY>(tp * tq, tq, K16, u0, A, lda, B, ldb, epi, nwv, 0, carry, cmode);
}

// One 16-row tile by ONE wave: C[p][q] for p < 16, q < Q (every column tile:
// NQ = all of them up to 3 per unit, so one A read feeds them), K = the
// contraction.  A / B as mfma_gemm (A at the tile's first row); the epilogue
// gets rows relative to the tile.
template <bool ACONT, bool BCONT, class Epi>
__device__ __forceinline__ void row_gemm(int Q, int K, const float* A, int lda, const float* B, int ldb,
                                         Epi epi) {
    const int tq = (Q + 15) >> 4, K16 = (K + 15) & ~15;
    switch (tq) {
        case 3: gemm_steps<ACONT, BCONT, 3>(1, 1, K16, 0, A, lda, B, ldb, epi, 1, K); break;
        case 2: gemm_steps<ACONT, BCONT, 2>(1, 1, K16, 0, A, lda, B, ldb, epi, 1, K); break;
        default: gemm_steps<ACONT, BCONT, 1>(tq, tq, K16, 0, A, lda, B, ldb, epi, 1, K); break;
    }
}

// FULLCOV: address in g_send of row r of layer l (wave-uniform) for local
// sample s.  One source rank: one contiguous row per sample.  Several: the
// row's 64-row band names its owner; the per-workgroup table srct in LDS holds
// every band's int64 offset for this sample ([nbands]), then the layers'
// first band index ([L] ints, after the stage's source bases), built at
// kernel start.
__device__ __forceinline__ int64_t fc_addr(const NetArgs& a, int nsrc, const int* srct, int l, int r,
                                           int s) {
    if (nsrc == 1) return (int64_t)s * a.src_stride[0] + a.xcol0[l] + r;
    const int64_t* boff = reinterpret_cast<const int64_t*>(srct);
    const int* bb = srct + 2 * a.nbands + 3 * kMaxWorld;
    return boff[bb[l] + (r >> 6)] + r;
}

// diagnostics: one wave-0 lane of every workgroup records a clock at phase
// boundaries into LDS (slot k), flushed to the stamp buffer at the end -- a
// global store per stamp would make the next barrier wait for it; costs
// nothing when stamps == nullptr
#define NET_STAMP(k, val)                                                  \
    do {                                                                   \
        if (a.stamps && threadIdx.x == 0) stl[(k)] = (val);                \
    } while (0)

// MSRC: full-cov rows from several source ranks (world > 1).  The single-source
// instantiation has straight-line x loads: with the run-table path in the
// same kernel the register allocator shares registers across the two paths
// and the waitcnt pass then serialises the u and x loads (seen in the ISA).
template <int FAM, bool MSRC, bool VEC = false, bool MLOOP = false, int GEO = 0>
__global__ __launch_bounds__(512) void net_kernel(NetArgs a) {
    using Geo = NetGeo<GEO>;
    const Geo g(a);
    constexpr int kUL = Geo::kUnroll;  // layer loops: fully unrolled for a fixed geometry
    // threads per workgroup: the fixed geometry runs 512 (the host gates it),
    // so no implicit-argument load for blockDim
    const int nthr = Geo::kFixed ? 512 : (int)blockDim.x;
    static_assert(!VEC || FAM == PSVI_FAMILY_FULLCOV, "float4 loads: the full-cov x row");
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int s = blockIdx.x + a.s_begin;     // local sample
    const int sg = a.s_goff + s;              // global sample (eps indexing)
    const int role = blockIdx.y;
    const int L = g.L(), Mp = g.Mp();
    const int tid = threadIdx.x;
    unsigned long long* stl = reinterpret_cast<unsigned long long*>(sm + g.lstamp());
    if constexpr (Geo::kFixed) {
        // the load phase's kernel arguments in one batch of scalar loads: the
        // diagnostics branches below would otherwise each wait for their own
        // before the first global load is issued
        asm volatile("" ::"s"(a.u), "s"(a.xrecv), "s"(a.xmap), "s"(a.z), "s"(a.w), "s"(a.abl),
                     "s"(a.stamps), "s"(a.mc), "s"(a.M), "s"(a.stage_len), "s"(a.src_stride[0]),
                     "s"(a.rn_P));  // (rn_P: the cache line of the implicit arguments)
    }
    if (a.abl & 128) {
        // diagnostics: poison the LDS with NaN first -- every word the kernel
        // reads must have been written by it (the padding contract).  abl >> 8
        // picks one region (0: all; 1 weights, 2 X_0, 3 red / zw / stamps /
        // tables, 4 X_l (l >= 1), 5 G_l, 6 dlogits and the rest)
        const int reg = a.abl >> 8;
        int lo = 0, hi = 4 * g.lds_f4();
        if (reg == 1) { lo = 0; hi = g.lx(0); }
        else if (reg == 2) { lo = g.lx(0); hi = g.lred(); }
        else if (reg == 3) { lo = g.lred(); hi = g.L() > 1 ? g.lx(1) : g.ldl(); }
        else if (reg == 4) { lo = g.L() > 1 ? g.lx(1) : g.ldl(); hi = g.L() > 1 ? g.lg(0) : g.ldl(); }
        else if (reg == 5) { lo = g.L() > 1 ? g.lg(0) : g.ldl(); hi = g.ldl(); }
        else if (reg == 6) { lo = g.ldl(); }
        for (int i = lo + (int)threadIdx.x; i < hi; i += nthr) sm[i] = __builtin_nanf("");
        __syncthreads();
    }
    if (a.stamps && threadIdx.x < 16) stl[threadIdx.x] = 0;
    NET_STAMP(0, __builtin_amdgcn_s_memtime());
    // diagnostics: each wave's start, for the launch skew in slot 15
    const unsigned long long wstart = a.stamps ? __builtin_amdgcn_s_memtime() : 0ull;
    NET_STAMP(13, __builtin_amdgcn_s_memrealtime());  // chip-wide 100 MHz clock

    // layers whose weight gradients this workgroup produces: [own_lo, own_hi)
    const int own_lo = (a.nroles == 1 || role == 0) ? 0 : 1;
    // W_l^T (the propagation GEMM's k-contiguous operand) is written with W_l
    // for the layers this workgroup propagates through: l > own_lo
    const int wt_lo = (a.outer == 1 || FAM != PSVI_FAMILY_FULLCOV) ? L : max(1, own_lo + 1);
    const int own_hi = (a.nroles == 1 || role == 1) ? L : 1;

    // ---- 1. loads --------------------------------------------------------
    int* srct = reinterpret_cast<int*>(sm + g.lsrc());
    const int nsrc = MSRC ? a.nsrc : 1;
    if (FAM == PSVI_FAMILY_FULLCOV && MSRC) {
        // uniform loops: a per-lane index into the by-value kernel arguments
        // would make the compiler copy the whole argument block to scratch
        // (the band table -- global loads -- is filled after the load phase: a
        // global load here would hold the x loads behind its latency)
        int64_t* xb = reinterpret_cast<int64_t*>(srct) + a.nbands;
        int* xs0 = srct + 2 * a.nbands + 2 * kMaxWorld;
        int* bb = xs0 + kMaxWorld;
        // constant trip counts: the argument reads are scalar loads at constant
        // offsets, issued together (a run-time bound made each iteration wait for
        // its own scalar load: ~4 k clocks for 8 sources)
        if (tid == 0) {
#pragma unroll
            for (int p = 0; p < kMaxWorld; ++p)
                if (p < nsrc) {  // the stage: source p's block at stage_off[p]
                    xs0[p] = a.stage_off[p];
                    xb[p] = a.src_base[p] + (int64_t)s * a.src_stride[p] - a.stage_off[p];
                }
#pragma unroll
            for (int l = 0; l < kMaxL; ++l)
                if (l < L) bb[l] = a.bbase[l];
            if constexpr (VEC) {
                int* cs = bb + kMaxL;
                int* rq = cs + kMaxWorld + 1;
#pragma unroll
                for (int p = 0; p <= kMaxWorld; ++p)
                    if (p <= nsrc) {
                        cs[p] = a.src_chunk0[p];
                        if (p < nsrc) rq[p] = a.src_stride[p];
                    }
            }
        }
        __syncthreads();
    }
    float part = 0.f;  // this thread's share of the weighted NLL
    // Pseudopoint chunks: blockIdx.z picks a run of a.mloop chunks, looped
    // inside the workgroup (full-cov inner objective, buffers past the LDS: the
    // sample's weights are loaded once, the weight gradients of chunk > 0 are
    // added to the first chunk's -- by the same lane, in chunk order, so the
    // sums equal the per-chunk slots added in chunk order)
    const int nloop = MLOOP ? a.mloop : 1;
    // looped chunks under the fixed geometry: the weight-gradient sums of the
    // chunks stay in registers (wc: two 16x16 units per wave and layer; bc:
    // the bias column sums) and leave once, after the last chunk, instead of
    // each chunk's read-modify-write of g_send
    constexpr bool kCarry = MLOOP && Geo::kFixed;
    constexpr int kWcUnits = 2;
    floatx4 wc[kMaxL][kWcUnits][1];
    float bc[kMaxL];
    int ch = 0;
chunk_top:  // a backward jump only when MLOOP (no loop at all in the other instantiations)
    {
    const int m0 = (blockIdx.z * nloop + ch) * a.mc;
    const int mcnt = min(a.mc, a.M - m0);
    const bool first = !MLOOP || ch == 0;
    NET_STAMP(4, __builtin_amdgcn_s_memtime());
    // Every global load of the phase is issued before its first LDS store:
    // the u chunk (float4 per lane when rows are float4-sized), the labels and
    // weights, and (full-cov) this sample's x row -- the source ranks' blocks
    // back to back -- with each element's LDS destination from the plan's x
    // map (W_l[j][i] or b_l[j], and W_l^T[i][j]): the elements go straight
    // into the padded W_l, b_l, W_l^T, no stage, no index arithmetic behind
    // the loads (LDS-DMA of the rows measured several times slower).
    const int D = g.din(0);
    const int r16 = tid >> 4, c16 = tid & 15, nr16 = nthr >> 4;
    float* zw = sm + g.lzw();  // the chunk's labels (as int bits) and weights
    float* X0 = sm + g.lx(0);
    const int ldx0 = g.ldx(0);
    if constexpr (VEC) {
        // one source, D % 4 == 0: the u chunk and the x row as float4 runs (a
        // quarter of the load instructions), x's < 4 trailing elements by
        // scalar loads at clamped indices; every load unconditional
        constexpr int kU4 = 4, kX4 = 3;
        // ext vectors (a HIP float4 array here went to scratch: SROA gives up
        // on the struct type)
        typedef float f4 __attribute__((ext_vector_type(4)));
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const int nu4 = (mcnt * D) >> 2;
        const float rdu = 1.f / (float)D;
        const f4* usrc = reinterpret_cast<const f4*>(a.u + (int64_t)m0 * D);
        const int nx = first ? a.stage_len : 0, nxt = MSRC ? 0 : nx & 3;
        // float4 chunks of the x row: one source -- the row's whole float4s;
        // several -- every source block's ceil(rows / 4) chunks (the last one
        // loaded at rows - 4 and shifted), chunk prefix per source in LDS
        const int nx4 = MSRC ? (first ? a.src_chunk0[a.nsrc] : 0) : nx >> 2;
        const float* xr = a.xrecv + (int64_t)s * a.src_stride[0];
        const u4* xm4 = reinterpret_cast<const u4*>(a.xmap);
        const int bd = nthr;
        int xsh[kX4];  // MSRC: this lane's shift of each chunk (0: all four valid)
        for (int pass = 0; pass * kU4 * bd < nu4 || pass * kX4 * bd < nx4 || pass == 0; ++pass) {  // uniform
            const int bu = pass * kU4 * bd + tid, bx = pass * kX4 * bd + tid;
            f4 uv[kU4], xv[kX4];
            u4 xm[kX4];
            float xt = 0.f;
            uint32_t xmt = 0xFFFFFFFFu;
            int zi = 0;
            float wv = 0.f;
            if (!(a.abl & 1)) {
#pragma unroll
                for (int k = 0; k < kU4; ++k) uv[k] = usrc[max(min(bu + k * bd, nu4 - 1), 0)];
                if constexpr (!MSRC) {
#pragma unroll
                    for (int k = 0; k < kX4; ++k) {
                        const int c = max(min(bx + k * bd, nx4 - 1), 0);
                        xv[k] = *reinterpret_cast<const f4*>(xr + 4 * c);
                        xm[k] = xm4[c];
                    }
                    const int rt = max(min(4 * nx4 + (tid & 3), nx - 1), 0);
                    xt = xr[rt];
                    xmt = a.xmap[rt];
                } else {
                    const int64_t* xb = reinterpret_cast<const int64_t*>(srct) + a.nbands;
                    const int* xs0 = srct + 2 * a.nbands + 2 * kMaxWorld;
                    const int* cs = xs0 + kMaxWorld + kMaxL;  // [nsrc + 1] chunk prefix
                    const int* rq = cs + kMaxWorld + 1;       // [nsrc] rows per source
#pragma unroll
                    for (int k = 0; k < kX4; ++k) {
                        const int c = max(min(bx + k * bd, nx4 - 1), 0);
                        int q = 0;
                        while (q + 1 < nsrc && c >= cs[q + 1]) ++q;
                        const int off = 4 * (c - cs[q]), st = min(off, rq[q] - 4);
                        xsh[k] = off - st;
                        const int pos = xs0[q] + st;  // stage position of the loaded float4
                        xv[k] = *reinterpret_cast<const f4*>(a.xrecv + xb[q] + pos);
                        xm[k] = *reinterpret_cast<const u4*>(a.xmap + pos);
                    }
                }
                if (pass == 0) {
                    const int mm = min(tid, mcnt - 1);
                    zi = a.z[m0 + mm];
                    wv = a.w[m0 + mm];
                }
            }
            NET_STAMP(11, __builtin_amdgcn_s_memtime());
            if (pass == 0 && !(a.abl & 4096)) {
                // zero padding while the loads are in flight (diagnostics: abl &
                // 4096 skips it -- wrong results).  The weight regions (W_l, b_l,
                // W_l^T and their slacks: the carve's first, up to X_0) are zeroed
                // whole with float4 stores, and after a barrier the x scatter
                // writes the sampled values over them; then u rows past the chunk,
                // u columns >= D up to the 16-multiple and the other slacks
                if (first) {
                    f4* z4 = reinterpret_cast<f4*>(sm);
                    const int nz4 = g.lx(0) >> 2;
                    constexpr int kZU = Geo::kFixed ? 8 : 1;
#pragma unroll kZU
                    for (int i = tid; i < nz4; i += bd) z4[i] = f4{0.f, 0.f, 0.f, 0.f};
                }
                const int cend = min((D + 15) & ~15, ldx0);
                for (int m = r16; m < mcnt; m += nr16)
                    if (D + c16 < cend) X0[m * ldx0 + D + c16] = 0.f;
                for (int i = tid; i < (Mp - mcnt) * ldx0; i += bd) X0[mcnt * ldx0 + i] = 0.f;
                if constexpr (Geo::kFixed) {
                    // every slack's offset a constant: one store per slack, wave k % nwaves
#pragma unroll
                    for (int k = 0; k < Geo::nslack(); ++k)
                        if (Geo::slack(k) >= Geo::lx(0) && k % (int)(bd >> 6) == wave_id())
                            sm[Geo::slack(k) + (tid & 63)] = 0.f;
                } else {
                    for (int k = wave_id(); k < g.nslack(); k += bd >> 6)  // wave-uniform slot
                        if (g.slack(k) >= g.lx(0)) sm[g.slack(k) + (tid & 63)] = 0.f;
                }
                if (first) __syncthreads();  // the zeroed weights before the x scatter
            }
            if (a.abl & 1) continue;
#pragma unroll
            for (int k = 0; k < kU4; ++k) {
                const int c = bu + k * bd;
                if (c < nu4) {
                    const int idx = 4 * c;
                    const int m = (int)(((float)idx + 0.5f) * rdu);  // exact for idx < 2^21
                    *reinterpret_cast<f4*>(X0 + m * ldx0 + idx - m * D) = uv[k];
                }
            }
            auto put = [&](float v, uint32_t mp) __attribute__((always_inline)) {
                sm[mp & 0xFFFFu] = v;
                if ((mp >> 16) != 0xFFFFu) sm[mp >> 16] = v;
            };
#pragma unroll
            for (int k = 0; k < kX4; ++k)
                if (bx + k * bd < nx4) {
                    if (MSRC && xsh[k]) {
                        // a source's last chunk: the float4 was loaded d = xsh
                        // elements early; its components d .. 3 are the chunk's
                        const int d = xsh[k];
                        put(xv[k][3], xm[k][3]);
                        if (d <= 2) put(xv[k][2], xm[k][2]);
                        if (d <= 1) put(xv[k][1], xm[k][1]);
                    } else {
                        put(xv[k][0], xm[k][0]);
                        put(xv[k][1], xm[k][1]);
                        put(xv[k][2], xm[k][2]);
                        put(xv[k][3], xm[k][3]);
                    }
                }
            if (pass == 0 && tid < nxt) put(xt, xmt);
            if (pass == 0 && tid < mcnt) {
                zw[tid] = __int_as_float(zi);
                zw[Mp + tid] = wv;
            }
        }
        for (int m = bd + tid; m < mcnt && !(a.abl & 1); m += bd) {  // chunks past one block
            zw[m] = __int_as_float(a.z[m0 + m]);
            zw[Mp + m] = a.w[m0 + m];
        }
    } else {
        // u chunk as a flat run of nu floats (one load path for every D: two
        // paths -- float4 rows and scalars -- are tail-merged by the compiler
        // into split loads serialised on s_waitcnt vmcnt, seen in the ISA)
        constexpr int kU = 16, kX = 12;
        const int nu = mcnt * D;
        const float rdu = 1.f / (float)D;
        const float* usrc = a.u + (int64_t)m0 * D;
        const int nx = FAM == PSVI_FAMILY_FULLCOV ? a.stage_len : 0;
        const int bd = nthr;
        for (int pass = 0; pass * kU * bd < nu || pass * kX * bd < nx || pass == 0; ++pass) {  // uniform
            const int bu = pass * kU * bd + tid, bx = pass * kX * bd + tid;
            float uv[kU];
            float xv[kX];
            uint32_t xm[kX];
            int zi = 0;
            float wv = 0.f;
            if (!(a.abl & 1)) {
#pragma unroll
                for (int k = 0; k < kU; ++k) uv[k] = usrc[max(min(bu + k * bd, nu - 1), 0)];
                if constexpr (FAM == PSVI_FAMILY_FULLCOV) {
                    if constexpr (!MSRC) {
                        const float* xr = a.xrecv + (int64_t)s * a.src_stride[0];
#pragma unroll
                        for (int k = 0; k < kX; ++k) {
                            const int r = max(min(bx + k * bd, nx - 1), 0);
                            xv[k] = xr[r];
                            xm[k] = a.xmap[r];
                        }
                    } else {
                        // stage position r -> x_recv through the source table in LDS (a
                        // per-lane pick among the kernel arguments makes the compiler
                        // copy the whole argument block to scratch)
                        const int64_t* xb = reinterpret_cast<const int64_t*>(srct) + a.nbands;
                        const int* xs0 = srct + 2 * a.nbands + 2 * kMaxWorld;
#pragma unroll
                        for (int k = 0; k < kX; ++k) {
                            const int r = max(min(bx + k * bd, nx - 1), 0);
                            int q = 0;
                            while (q + 1 < nsrc && r >= xs0[q + 1]) ++q;
                            xv[k] = a.xrecv[xb[q] + r];
                            xm[k] = a.xmap[r];
                        }
                    }
                }
                if (pass == 0) {
                    const int mm = min(tid, mcnt - 1);
                    zi = a.z[m0 + mm];
                    wv = a.w[m0 + mm];
                }
            }
            if (pass == 0) {
                // zero padding while the loads are in flight (disjoint from every
                // loaded element): W columns >= din (16 lanes a row) and rows >=
                // dout, u columns >= D up to the 16-multiple, u rows past the
                // chunk, the slacks before the stage
                for (int l = 0; l < L; ++l) {  // (the scalar path is never looped)
                    const int din = g.din(l), dout = g.dout(l), ldw = g.ldw(l);
                    const int rows = (dout + 15) & ~15;
                    if (l > 0) {  // W^T columns dout .. the 16-multiple (K padding of the propagation)
                        float* WT = sm + g.lwt(l);
                        for (int i = r16; i < din; i += nr16)
                            if (dout + c16 < rows) WT[i * g.ldwt(l) + dout + c16] = 0.f;
                    }
                    float* W = sm + g.lw(l);
                    for (int j = r16; j < dout; j += nr16)
                        for (int c = din + c16; c < ldw; c += 16) W[j * ldw + c] = 0.f;
                    for (int i = tid; i < (rows - dout) * ldw; i += bd) W[dout * ldw + i] = 0.f;
                }
                const int cend = min((D + 15) & ~15, ldx0);
                for (int m = r16; m < mcnt; m += nr16)
                    if (D + c16 < cend) X0[m * ldx0 + D + c16] = 0.f;
                for (int i = tid; i < (Mp - mcnt) * ldx0; i += bd) X0[mcnt * ldx0 + i] = 0.f;
                if constexpr (Geo::kFixed) {
                    // every slack's offset a constant: one store per slack, wave k % nwaves
#pragma unroll
                    for (int k = 0; k < Geo::nslack(); ++k)
                        if (k % (int)(bd >> 6) == wave_id()) sm[Geo::slack(k) + (tid & 63)] = 0.f;
                } else {
                    for (int k = wave_id(); k < g.nslack(); k += bd >> 6)  // wave-uniform slot
                        sm[g.slack(k) + (tid & 63)] = 0.f;
                }
            }
            if (a.abl & 1) continue;
#pragma unroll
            for (int k = 0; k < kU; ++k) {
                const int idx = bu + k * bd;
                if (idx < nu) {
                    const int m = (int)(((float)idx + 0.5f) * rdu);  // exact for idx < 2^21
                    X0[m * ldx0 + idx - m * D] = uv[k];
                }
            }
            if constexpr (FAM == PSVI_FAMILY_FULLCOV) {
#pragma unroll
                for (int k = 0; k < kX; ++k)
                    if (bx + k * bd < nx) {
                        sm[xm[k] & 0xFFFFu] = xv[k];
                        if ((xm[k] >> 16) != 0xFFFFu) sm[xm[k] >> 16] = xv[k];
                    }
            }
            if (pass == 0 && tid < mcnt) {
                zw[tid] = __int_as_float(zi);
                zw[Mp + tid] = wv;
            }
        }
        for (int m = bd + tid; m < mcnt && !(a.abl & 1); m += bd) {  // chunks past one block
            zw[m] = __int_as_float(a.z[m0 + m]);
            zw[Mp + m] = a.w[m0 + m];
        }
    }
    if (FAM != PSVI_FAMILY_FULLCOV && !(a.abl & 1)) {  // (never looped: MLOOP is full-cov only)
        // Normal.rsample: loc + eps * softplus(rho), elementwise into place
        constexpr int kB = 16;
        for (int l = 0; l < L; ++l) {
            const int din = g.din(l), dout = g.dout(l), nw = din * dout, n = nw + dout;
            float* W = sm + g.lw(l);
            float* WT = sm + g.lwt(l);
            float* Bv = sm + g.lb(l);
            const int ldw = g.ldw(l), ldwt = g.ldwt(l);
            const bool wt = l >= wt_lo;
            const float* mu = a.params + a.poff[l];
            const float* rho = mu + n;
            const float* eW = a.eps + a.eoff[l] + (int64_t)sg * nw;
            const float* eB = a.eps + a.eoff[l] + (int64_t)a.S_total * nw + (int64_t)sg * dout;
            const float rdin = 1.f / (float)din;
            for (int base = tid; base < n; base += kB * nthr) {
                float vm[kB], vr[kB], ve[kB];
#pragma unroll
                for (int k = 0; k < kB; ++k) {
                    const int idx = min(base + k * nthr, n - 1);
                    vm[k] = mu[idx];
                    vr[k] = rho[idx];
                    ve[k] = idx < nw ? eW[idx] : eB[idx - nw];
                }
#pragma unroll
                for (int k = 0; k < kB; ++k) {
                    const int idx = base + k * nthr;
                    if (idx >= n) break;
                    const float val = vm[k] + ve[k] * softplus_f(vr[k]);
                    if (idx < nw) {
                        // exact for idx < 2^21: (idx + 0.5) / din is >= 0.5/din from an integer
                        const int j = (int)(((float)idx + 0.5f) * rdin), i = idx - j * din;
                        W[j * ldw + i] = val;
                        if (wt) WT[i * ldwt + j] = val;
                    } else {
                        Bv[idx - nw] = val;
                    }
                }
            }
        }
    }
    NET_STAMP(5, __builtin_amdgcn_s_memtime());
    if (FAM == PSVI_FAMILY_FULLCOV && MSRC && first) {
        // every band's g_send offset for this sample (section 3's fc_addr)
        int64_t* boff = reinterpret_cast<int64_t*>(srct);
        for (int i = tid; i < a.nbands; i += nthr) {
            const NetBand bd = a.bands[i];
            boff[i] = bd.base + (int64_t)s * bd.stride;
        }
    }
    if (a.stamps && (tid & 63) == 0) stl[16 + wave_id()] = wstart;
    __syncthreads();  // the LDS stores
    NET_STAMP(1, __builtin_amdgcn_s_memtime());
    if (a.stamps && tid == 0) {
        unsigned long long mx = 0;
        for (int q = 0; q < (nthr >> 6); ++q) mx = max(mx, stl[16 + q]);
        stl[15] = mx;
    }

    // ---- 2. the row chain.  A layer's output rows depend only on the same
    // rows of its input, and so do the loss head and the gradient propagation
    // G_{l-1} = (G_l W_l) * 1[X_l > 0]: wave w carries the chunk's 16-row
    // tiles w, w + nwaves, ... through the whole forward (every column tile of
    // a layer), the loss head and the backward propagation without a
    // workgroup barrier -- it re-reads only LDS rows it wrote itself, after an
    // lgkmcnt drain.  Rows past the chunk and columns past dout (up to the
    // 16-multiple within the stride) are written zero.  The weight gradients,
    // which sum over every row, follow ONE barrier (section 3).
    // The inner objective's loss head (C <= 16: one column tile, a row's
    // logits on the 16 lanes of a DPP row) runs in the head GEMM's epilogue:
    // log-softmax over the lanes, weighted NLL, dlogits w_m (softmax - onehot)
    // stored in place of the logits.
    const int C = g.dout(L - 1);
    const bool fuse_head = a.outer == 0 && C <= 16 && !(a.abl & 4);
    const bool bwd = !(a.abl & 8) && a.outer != 1;
    // outer backward: input gradient of the pseudopoint rows (d loss / d u)
    const bool dx0 = bwd && a.outer == 2 && a.du_part != nullptr && own_lo == 0;
    // outer backward: d loss / d pseudo_s and d loss / d data_s scale the rows
    const float cp = a.outer == 2 ? a.rowcoef[2 * s] : 1.f;
    const float cd = a.outer == 2 ? a.rowcoef[2 * s + 1] : 1.f;
    const int nwv = nthr >> 6, lane = tid & 63;
    auto drain = []() __attribute__((always_inline)) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
    // G_l: dlogits for l = L - 1, else the l-th gradient buffer (stride of X_{l+1})
    auto gbuf = [&](int l) __attribute__((always_inline)) {
        return l == L - 1 ? sm + g.ldl() : sm + g.lg(l);
    };
    auto gld = [&](int l) __attribute__((always_inline)) { return l == L - 1 ? g.lddl() : g.ldx(l + 1); };
    for (int pt = wave_id(); 16 * pt < Mp; pt += nwv) {  // wave-uniform
        const int r0 = 16 * pt;
        // diagnostics (abl & 64): the first tile's forward twice (its stamps record the second)
        for (int rep = 0; rep < (((a.abl & 64) && pt == wave_id()) ? 2 : 1); ++rep)
#pragma unroll kUL
        for (int l = 0; l < L; ++l) {
            if (a.abl & 2) break;
            const int din = g.din(l), dout = g.dout(l);
            const bool head = l == L - 1;
            const float* X = sm + g.lx(l) + r0 * g.ldx(l);
            float* Xn = (head ? sm + g.ldl() : sm + g.lx(l + 1)) + r0 * (head ? g.lddl() : g.ldx(l + 1));
            const float* Bv = sm + g.lb(l);
            const int ldn = head ? g.lddl() : g.ldx(l + 1), jend = min((dout + 15) & ~15, ldn);
            if (head && fuse_head) {
                // the row's logits sit on lanes j < C of its 16: the reductions
                // span the smallest power of two >= C (the fixed geometry: C = 2,
                // one lane exchange) -- a row of 16 otherwise
                constexpr int kHeadLanes = Geo::kHeadLanes;
                auto epi = [&](int m, int j, floatx4 v, int rot) {  // j = i16: every lane of the row takes part
                    const bool jl = j < C;
                    const float b = Bv[min(j, C - 1)];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = m + ((r + rot) & 3), rg = r0 + row;
                        const float y = v[r] + b;
                        const float mx = lanes_max<kHeadLanes>(jl ? y : -INFINITY);
                        const float lse = mx + logf(lanes_sum<kHeadLanes>(jl ? expf(y - mx) : 0.f));
                        const int zr = __float_as_int(zw[rg]);
                        const float wr = zw[Mp + rg];
                        const bool ok = rg < mcnt;
                        const float dl = (ok && jl) ? wr * (expf(y - lse) - (j == zr ? 1.f : 0.f)) : 0.f;
                        if (j < jend) Xn[row * ldn + j] = dl;
                        if (ok && j == zr) part += wr * (lse - y);
                    }
                };
                row_gemm<true, true>(dout, din, X, g.ldx(l), sm + g.lw(l), g.ldw(l), epi);
            } else {
                auto epi = [&](int m, int j, floatx4 v, int rot) {
                    if (j < jend) {
                        const bool jl = j < dout;
                        const float b = Bv[min(j, dout - 1)];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float y = v[r] + b;
                            const int row = m + ((r + rot) & 3);
                            Xn[row * ldn + j] = (jl && r0 + row < mcnt) ? (head ? y : fmaxf(y, 0.f)) : 0.f;
                        }
                    }
                };
                row_gemm<true, true>(dout, din, X, g.ldx(l), sm + g.lw(l), g.ldw(l), epi);
            }
            drain();
            if (pt == 0 && l < 3) NET_STAMP(6 + l, __builtin_amdgcn_s_memtime());
        }
        // ---- loss head on VALU (C > 16, the outer objective): lanes 0..15
        // take the tile's rows, logits -> weighted NLL, dlogits in place
        if (!fuse_head && !(a.abl & 4) && lane < 16 && r0 + lane < mcnt) {
            const int m = r0 + lane;
            const int ldl = g.lddl();
            float* row = sm + g.ldl() + m * ldl;
            const int zm = __float_as_int(zw[m]);
            const float wm = zw[Mp + m] * (m0 + m < a.n_pseudo ? cp : cd);
            float mx = -INFINITY, lz = 0.f;
            for (int c = 0; c < C; ++c) {
                mx = fmaxf(mx, row[c]);
                if (c == zm) lz = row[c];
            }
            float se = 0.f;
            for (int c = 0; c < C; ++c) se += expf(row[c] - mx);
            const float lse = mx + logf(se);
            if (a.outer == 1) {
                const int mg = m0 + m;
                a.nll_rows[(size_t)s * a.M + mg] = lse - lz;
                if (a.prob_rows && mg >= a.n_pseudo) {
                    float* pr = a.prob_rows + ((size_t)s * (a.M - a.n_pseudo) + mg - a.n_pseudo) * C;
                    for (int c = 0; c < C; ++c) pr[c] = expf(row[c] - lse);
                }
            } else {
                part += wm * (lse - lz);
                for (int c = 0; c < C; ++c) row[c] = wm * (expf(row[c] - lse) - (c == zm ? 1.f : 0.f));
            }
        }
        drain();
        if (pt == 0) NET_STAMP(9, __builtin_amdgcn_s_memtime());
        if (!bwd) continue;
        // ---- backward propagation down to the lowest owned layer
#pragma unroll kUL
        for (int l = L - 1; l > 0; --l) {
            if (l <= own_lo) continue;  // (uniform: the role)
            const int din = g.din(l), dout = g.dout(l);
            const float* G = gbuf(l) + r0 * gld(l);
            const int ldx = g.ldx(l);
            const float* X = sm + g.lx(l) + r0 * ldx;
            float* Gn = gbuf(l - 1) + r0 * ldx;  // G_{l-1}: the stride of X_l
            const int iend = min((din + 15) & ~15, ldx);
            auto epi = [&](int m, int i, floatx4 v, int rot) {
                if (i < iend) {
                    const bool il = i < din;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = m + ((r + rot) & 3);
                        Gn[row * ldx + i] = (il && X[row * ldx + i] > 0.f) ? v[r] : 0.f;
                    }
                }
            };
            if constexpr (FAM == PSVI_FAMILY_FULLCOV)
                row_gemm<true, true>(din, dout, G, gld(l), sm + g.lwt(l), g.ldwt(l), epi);
            else  // mean-field: K = dout is small (the classifier), W read down k
                row_gemm<true, false>(din, dout, G, gld(l), sm + g.lw(l), g.ldw(l), epi);
            drain();
        }
        if (pt == 0) NET_STAMP(10, __builtin_amdgcn_s_memtime());
        if (dx0) {
            // du[s][m][i] = sum_j G_0[m][j] W_0[j][i] for the tile's pseudopoint rows
            const int din = g.din(0), dout = g.dout(0);
            auto epi = [&](int m, int i, floatx4 v, int rot) {
                if (i < din) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int mm = r0 + m + ((r + rot) & 3), mg = m0 + mm;
                        if (mm < mcnt && mg < a.n_pseudo)
                            a.du_part[((size_t)s * a.n_pseudo + mg) * din + i] = v[r];
                    }
                }
            };
            row_gemm<true, false>(din, dout, gbuf(0) + r0 * gld(0), gld(0), sm + g.lw(0), g.ldw(0), epi);
        }
    }
    __syncthreads();  // every tile's rows of X_l and G_l
    NET_STAMP(2, __builtin_amdgcn_s_memtime());

    // ---- 3. weight gradients of the owned layers, dW_l = G_l^T X_l and the
    // biases' column sums (sums over every row of the chunk), all layers' tiles
    // in one round-robin over the waves
    float sink = 0.f;
    // gradient element o of layer l: W rows j*din + i, then the biases
    auto emit = [&](int l, int o, float v) {
        if (a.abl & 16) { sink += v; return; }
        if constexpr (FAM == PSVI_FAMILY_MEANFIELD) {
            a.mf_slots[((size_t)s * gridDim.z + blockIdx.z) * a.slot_ld + a.woff[l] + o] = v;
        } else {
            // one writer per element (per chunk slot when the pseudopoints are
            // chunked; net_slot_sum_kernel adds the slots in chunk order)
            float* dst = (a.gslot ? a.gslot + (int64_t)blockIdx.z * a.gsz : a.gsend) +
                         fc_addr(a, nsrc, srct, l, o, s);
            if (first || kCarry) *dst = v;
            else *dst += v;  // a looped chunk: this lane wrote the element before
        }
    };
    // outer backward: the sampled-KL path, d nkl_s / d x_s = -x_s / s0^2,
    // added once per sample (pseudopoint chunk 0)
    const float ckv = (a.outer == 2 && blockIdx.z == 0 && first) ? a.ck[s] * a.inv_s0sq : 0.f;
    if (bwd) {
        int first = 0;
#pragma unroll kUL
        for (int l = L - 1; l >= 0; --l) {
            if (l >= own_hi || l < own_lo) continue;  // (uniform: the role)
            // dW_l[j][i] = sum_m G_l[m][j] X_l[m][i]: both operands k(=m)-strided
            const int din = g.din(l), dout = g.dout(l);
            const float* Wl = sm + g.lw(l);
            const int ldw = g.ldw(l);
            auto epi = [&](int j0, int i, floatx4 v, int rot) {
                if (i < din) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int j = j0 + ((r + rot) & 3);
                        if (j < dout) {
                            float gv = v[r];
                            if (a.outer == 2) gv -= ckv * Wl[j * ldw + i];
                            emit(l, j * din + i, gv);
                        }
                    }
                }
            };
            if constexpr (kCarry) {
                const int cm = nloop == 1 ? 0 : ch == 0 ? 1 : ch + 1 < nloop ? 3 : 2;
                mfma_gemm_carry<kWcUnits>(dout, din, Mp, first, gbuf(l), gld(l), sm + g.lx(l),
                                          g.ldx(l), epi, wc[l], cm, nthr >> 6);
            } else {
                mfma_gemm<false, false>(dout, din, Mp, first, gbuf(l), gld(l), sm + g.lx(l),
                                        g.ldx(l), epi, nthr >> 6);
            }
            first += gemm_units(dout, din);
        }
        // bias gradients: column sums of G_l over the chunk.  A wave takes
        // columns 16 q .. 16 q + 15 of one layer: lane (k4, i16) reads the
        // float4 of columns 16 q + 4 k4 .. + 3 in rows i16, i16 + 16, ... (the
        // GEMM's conflict-free ds_read_b128 pattern), then DPP row sums over i16.
        const int i16 = lane & 15, k4 = lane >> 4;
        int qb = 0;
#pragma unroll kUL
        for (int l = L - 1; l >= 0; --l) {
            if (l >= own_hi || l < own_lo) continue;  // (uniform: the role)
            const int din = g.din(l), dout = g.dout(l);
            const float* G = gbuf(l);
            const int ldg = gld(l);
            const int nq = (dout + 15) >> 4;
            for (int q = ((wave_id() - first - qb) % nwv + nwv) % nwv; q < nq; q += nwv) {  // wave-uniform
                const int j0 = 16 * q + 4 * k4;
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                for (int m = i16; m < mcnt; m += 16) {
                    const float4 g4 = *reinterpret_cast<const float4*>(G + m * ldg + j0);
                    acc.x += g4.x; acc.y += g4.y; acc.z += g4.z; acc.w += g4.w;
                }
                const float s0 = row16_sum(acc.x), s1 = row16_sum(acc.y), s2 = row16_sum(acc.z),
                            s3 = row16_sum(acc.w);
                // lanes i16 = 0..3 of the row emit one column each, in parallel
                if (i16 < 4 && j0 + i16 < dout) {
                    const int j = j0 + i16;
                    float b = i16 == 0 ? s0 : i16 == 1 ? s1 : i16 == 2 ? s2 : s3;
                    if (a.outer == 2) b -= ckv * sm[g.lb(l) + j];
                    if constexpr (kCarry) {
                        // (a wave holds at most one column tile of a layer: nq <= waves)
                        if (nloop > 1 && ch == 0) {
                            bc[l] = b;
                        } else if (ch + 1 < nloop) {
                            bc[l] += b;
                        } else {
                            emit(l, dout * din + j, nloop > 1 ? bc[l] + b : b);
                        }
                    } else {
                        emit(l, dout * din + j, b);
                    }
                }
                if constexpr (kCarry) break;  // one column tile per wave (fixed shapes)
            }
            qb += nq;
        }
    }
    asm volatile("" ::"v"(sink));
    }
    if constexpr (MLOOP) {
        if (++ch < nloop) {
            __syncthreads();  // the next chunk overwrites X_l, G_l, z / w
            goto chunk_top;
        }
    }
    NET_STAMP(3, __builtin_amdgcn_s_memtime());
    if (role == 0 && a.outer == 0) {  // the chunk's weighted NLL (role 1 computed the same)
        const float tot = block_sum(part, sm + g.lred());
        if (tid == 0) atomicAdd(a.nll_out, (double)tot);
    }
    if (a.rn_out) {
        // the next step's normals (psvi_randn's stream), split over the grid's
        // workgroups.  Last, so that no s_waitcnt of the phases above waits for
        // these stores to retire.
        const int64_t nqa = (a.rn_n + 3) / 4;
        const int64_t qlo = nqa * a.rn_part / a.rn_nparts, nq = nqa * (a.rn_part + 1) / a.rn_nparts;
        const int nblk = gridDim.x * gridDim.y * gridDim.z;
        const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int64_t per = (nq - qlo + nblk - 1) / nblk, q1 = min(nq, qlo + (b + 1) * per);
        if (a.rn_planes) {
            const EpsPlanes P = *a.rn_P;
            for (int64_t q = qlo + b * per + tid; q < q1; q += nthr)
                randn_quad_planes(a.rn_out, a.rn_n, a.rn_seed, a.rn_off, q, P, a.rn_planes);
        } else {
            for (int64_t q = qlo + b * per + tid; q < q1; q += nthr)
                randn_quad<true>(a.rn_out, a.rn_n, a.rn_seed, a.rn_off, q);
        }
    }
    NET_STAMP(12, __builtin_amdgcn_s_memtime());
    NET_STAMP(14, __builtin_amdgcn_s_memrealtime());
    if (a.stamps && threadIdx.x < 16)  // wave 0 wrote them: in order, no barrier needed
        a.stamps[(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 16 + threadIdx.x] =
            stl[threadIdx.x];
}

static inline int rup(int x, int m) { return (x + m - 1) / m * m; }

// LDS floats for a chunk of `mc` pseudopoints (layout and padding contract
// in the header comment); fills the carve into `a` when given.  The full-cov
// x stage bookkeeping (source blocks) is added here; the carve itself is
// net_carve's, the same function the fixed-geometry kernels evaluate at
// compile time.
static size_t net_lds_floats(const psvi_plan& p, int mc, NetArgs* a) {
    NetDims d{};
    d.L = p.L;
    for (int l = 0; l < p.L; ++l) {
        d.din[l] = p.lay[l].din;
        d.dout[l] = p.lay[l].dout;
    }
    const int nbands = (p.family == PSVI_FAMILY_FULLCOV && p.world > 1) ? p.band_base[p.L] : 0;
    const NetCarve c = net_carve(d, mc, nbands);
    if (a) {
        for (int l = 0; l < kMaxL; ++l) {
            a->lw[l] = c.lw[l]; a->ldw[l] = c.ldw[l]; a->lb[l] = c.lb[l];
            a->lx[l] = c.lx[l]; a->ldx[l] = c.ldx[l]; a->lwt[l] = c.lwt[l];
            a->ldwt[l] = c.ldwt[l]; a->lg[l] = c.lg[l];
        }
        for (int k = 0; k < kNetSlack; ++k) a->slack[k] = c.slack[k];
        a->ldl = c.ldl; a->lddl = c.lddl; a->lred = c.lred; a->lsrc = c.lsrc;
        a->lzw = c.lzw; a->lstamp = c.lstamp; a->Mp = c.Mp;
        a->nslack = c.nslack; a->nslack_early = c.nslack_early; a->lds_f4 = c.lds_f4;
        if (p.family == PSVI_FAMILY_FULLCOV) {  // the x row's source blocks (no LDS)
            int st = 0;
            for (int q = 0; q < p.world; ++q) {
                a->stage_off[q] = st;
                st += p.rows_tot[q];
            }
            a->stage_off[p.world] = st;
            a->stage_len = st;
        }
    }
    return (size_t)c.lds_f4 * 4;
}

// g_send = the pseudopoint chunks' dW slots added in chunk order (run-to-run
// bitwise reproducible; every element of every slot has one writer)
__global__ __launch_bounds__(256) void net_slot_sum_kernel(const float* __restrict__ slots,
                                                           int nslot, int64_t n,
                                                           float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float t = slots[i];
    for (int z = 1; z < nslot; ++z) t += slots[z * n + i];
    out[i] = t;
}

int g_net_threads = 0;        // psvi_debug_set(PSVI_DBG_NET_THREADS, n): 0 = by chunk size
int g_net_split_below = 256;  // split when a rank has fewer samples than CUs (psvi_debug_set(PSVI_DBG_NET_SPLIT_BELOW, n))
int g_net_wg_target = 256;    // workgroups a split rank aims for (psvi_debug_set(PSVI_DBG_NET_WG_TARGET, n))

size_t net_plan_geometry(psvi_plan& p) {
    // One workgroup per sample and all M pseudopoints when the samples alone
    // fill the chip.  Otherwise two role workgroups per sample (disjoint
    // gradient outputs), and pseudopoint chunks only if that still leaves
    // CUs idle or the buffers exceed the LDS (partial dW into per-chunk slots,
    // summed in chunk order).  LDS <= 160 KiB per workgroup.
    const int S_local = std::max(1, p.s_cnt[p.rank]);
    const int M = p.d.M;
    const bool split = S_local < g_net_split_below;
    p.net_roles = (split && p.L > 1) ? 2 : 1;
    int mchunks = 1;
    if (split)
        while (S_local * p.net_roles * mchunks < g_net_wg_target && (M + mchunks) / (mchunks + 1) >= 16)
            ++mchunks;
    // chunks forced by the LDS alone (the samples already fill the chip) are
    // looped inside the workgroups of a full-cov plan (NetArgs::mloop)
    const bool fill_one = mchunks == 1;
    for (;;) {
        const int mc = (M + mchunks - 1) / mchunks;
        const size_t bytes = net_lds_floats(p, mc, nullptr) * 4;
        if (bytes <= 160 * 1024 || mc == 1) {
            p.mchunks = (M + mc - 1) / mc;
            p.mc = mc;
            p.net_lds = bytes;
            p.net_threads = g_net_threads ? g_net_threads : (rup(mc, 16) >= 48 ? 512 : 256);
            p.net_mloop = p.family == PSVI_FAMILY_FULLCOV && fill_one && p.mchunks > 1;
            return bytes;
        }
        ++mchunks;
    }
}

// The full-cov x map: for every position of a sample's x row as the network
// kernel loads it (source blocks back to back, each in its x-shard column
// order: runs of rows), the LDS float offset of W_l[j][i] (row r = j din + i)
// or b_l[r - din dout], and of W_l^T[i][j] for l >= 1 (0xFFFF: none) -- so
// the load phase places each element with one lookup.  The world > 1 band
// table: per 64-row band, g_send's base offset for sample 0 (the owner's
// block + the band's column - its first row) and the owner's row stride.
void net_xmap(const psvi_plan& p, std::vector<uint32_t>& xmap, std::vector<NetBand>& bands) {
    NetArgs a{};
    net_lds_floats(p, p.mc, &a);
    xmap.clear();
    bands.clear();
    const int S_local = p.s_cnt[p.rank];
    int64_t base = 0;
    std::vector<int64_t> src_base(p.world);
    for (int q = 0; q < p.world; ++q) {
        src_base[q] = base;
        base += (int64_t)S_local * p.rows_tot[q];
        for (const ShardRun& run : p.runs[q]) {
            const int l = run.layer, din = p.lay[l].din, nw = din * p.lay[l].dout;
            for (int r = run.lo; r < run.hi; ++r) {
                uint32_t w, wt = 0xFFFFu;
                if (r < nw) {
                    const int j = r / din, i = r - j * din;
                    w = (uint32_t)(a.lw[l] + j * a.ldw[l] + i);
                    if (l > 0) wt = (uint32_t)(a.lwt[l] + i * a.ldwt[l] + j);
                } else {
                    w = (uint32_t)(a.lb[l] + r - nw);
                }
                xmap.push_back(w | wt << 16);
            }
        }
    }
    if (p.world > 1)
        for (int l = 0; l < p.L; ++l)
            for (int b = 0; 64 * b < p.lay[l].n; ++b) {
                const int gb = p.band_base[l] + b, q = p.band_owner[gb];
                bands.push_back(NetBand{src_base[q] + p.band_coloff[gb], p.rows_tot[q], 0});
            }
}

int g_net_ablation = 0;  // psvi_debug_set(PSVI_DBG_NET_ABLATION, mask)
int g_net_mloop_off = 0;  // psvi_debug_set(PSVI_DBG_NET_MLOOP_OFF, 1): a workgroup per pseudopoint chunk + slots (A/B)
int g_net_scalar_loads = 0;  // psvi_debug_set(PSVI_DBG_NET_SCALAR_LOADS, 1): the scalar load path (A/B)
int g_net_geo_off = 0;  // psvi_debug_set(PSVI_DBG_NET_GEO_OFF, 1): the run-time geometry for fn2 too (A/B)
unsigned long long* g_net_stamps = nullptr;  // psvi_debug_set_ptr(PSVI_DBG_NET_STAMPS, buf)

void net_set_lds_limit() {
    // gfx950: up to 160 KiB of LDS per workgroup
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_MEANFIELD, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, false, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, true, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, false, true, false, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, true, true, false, 2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, false, true, true, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)net_kernel<PSVI_FAMILY_FULLCOV, true, true, true, 2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

// The fixed fn2 geometry (NetGeo<1 / 2>) applies: the 64 -> 40 -> 40 -> 2
// full-cov stack with 100-row pseudopoint chunks (Mp = 112), float4 loads;
// the run-time carve then equals the compile-time one (the same net_carve)
static bool net_fn2_geo(const psvi_plan& p) {
    if (g_net_geo_off || p.family != PSVI_FAMILY_FULLCOV || p.L != kFn2Dims.L) return false;
    for (int l = 0; l < p.L; ++l)
        if (p.lay[l].din != kFn2Dims.din[l] || p.lay[l].dout != kFn2Dims.dout[l]) return false;
    return net_rup(p.mc, 16) == kFn2Mp && p.net_threads == 512;
}

// float4 loads of the full-cov x row: u rows of D % 4 == 0 floats, and every
// source block empty or at least one float4 wide (a block's last chunk is
// loaded at its rows - 4)
static bool net_vec_ok(const psvi_plan& p) {
    if (p.lay[0].din % 4 || g_net_scalar_loads) return false;
    for (int q = 0; q < p.world; ++q)
        if (p.rows_tot[q] > 0 && p.rows_tot[q] < 4) return false;
    return true;
}

hipError_t launch_net(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                      const float* params, const float* eps, float* mf_slots,
                      const float* xrecv, float* gsend, double* nll_out, hipStream_t st,
                      float* rn_out, int64_t rn_n, uint64_t rn_seed, uint64_t rn_off,
                      const NetOuter* outer, uint16_t* rn_planes, int s_begin, int s_count,
                      int rn_part, int rn_nparts) {
    NetArgs a{};
    const int S_loc = p.s_cnt[p.rank];
    if (s_count < 0) s_count = S_loc - s_begin;
    if (s_begin < 0 || s_count < 0 || s_begin + s_count > S_loc || rn_nparts < 1 || rn_part < 0 ||
        rn_part >= rn_nparts)
        return hipErrorInvalidValue;
    a.s_begin = s_begin;
    a.rn_part = rn_part;
    a.rn_nparts = rn_nparts;
    if (outer) {
        a.outer = outer->mode;
        a.n_pseudo = outer->n_pseudo;
        a.nll_rows = outer->nll_rows;
        a.rowcoef = outer->rowcoef;
        a.ck = outer->ck;
        a.du_part = outer->du_part;
        a.prob_rows = outer->prob_rows;
    }
    a.inv_s0sq = 1.f / (p.d.prior_sd * p.d.prior_sd);
    a.rn_out = rn_out;  // 16-byte aligned (workspace buffers)
    a.rn_n = rn_n;
    a.rn_seed = rn_seed;
    a.rn_off = rn_off;
    a.rn_P = p.d_eps_planes;
    a.rn_planes = rn_planes && p.d_eps_planes ? rn_planes : nullptr;
    if (rn_planes && !p.d_eps_planes) return hipErrorInvalidValue;
    a.L = p.L;
    a.M = p.d.M;
    a.mc = p.mc;
    a.S_total = p.d.S;
    a.s_goff = p.s_off[p.rank];
    a.gslot = p.family == PSVI_FAMILY_FULLCOV && p.mchunks > 1 ? p.d_net_slots : nullptr;
    a.gsz = (int64_t)p.s_cnt[p.rank] * p.n_tot;
    a.nroles = p.net_roles;
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
    a.params = params; a.eps = eps; a.mf_slots = mf_slots; a.slot_ld = p.n_tot;
    a.xrecv = xrecv; a.gsend = gsend;
    if (p.family == PSVI_FAMILY_FULLCOV) {
        const int S_local = p.s_cnt[p.rank];
        a.nsrc = p.world;
        int64_t base = 0;
        for (int q = 0; q < p.world; ++q) {
            a.src_base[q] = base;
            a.src_stride[q] = p.rows_tot[q];
            base += (int64_t)S_local * p.rows_tot[q];
        }
        for (int l = 0; l < p.L; ++l) {
            a.xcol0[l] = p.xcol_l[0][l];
            a.bbase[l] = p.band_base[l];
        }
        int c0 = 0;
        for (int q = 0; q < p.world; ++q) {
            a.src_chunk0[q] = c0;
            c0 += (p.rows_tot[q] + 3) / 4;
        }
        a.src_chunk0[p.world] = c0;
        a.xmap = p.d_net_xmap;
        a.bands = p.d_net_bands;
        a.nbands = p.world > 1 ? p.band_base[p.L] : 0;
        if (!a.xmap || (p.world > 1 && !a.bands)) return hipErrorInvalidValue;
    }
    // the inner objective of a full-cov plan whose pseudopoints exceed the LDS
    // loops its chunks inside each workgroup (one x load, no slots, no slot sum)
    const bool loop = p.net_mloop && a.outer == 0 && !g_net_mloop_off &&
                      p.family == PSVI_FAMILY_FULLCOV && net_vec_ok(p);
    a.mloop = loop ? p.mchunks : 1;
    if (loop) a.gslot = nullptr;
    // the outer forward pass has no backward: one role
    dim3 grid(s_count, a.outer == 1 ? 1 : p.net_roles, loop ? 1 : p.mchunks),
        block(p.net_threads);
    // a launch without samples still owes its part of the next step's draw
    // (every rank passes the same global eps to its update): the draw on its
    // own (the whole of it when this is its only part)
    if (s_count == 0) {
        if (!rn_out || rn_n <= 0 || rn_part > 0) return hipSuccess;
        return launch_randn(rn_out, rn_n, rn_seed, rn_off, st, nullptr, 0,
                            rn_planes ? &p.eps_planes : nullptr, rn_planes);
    }
    // per-chunk slots are summed over all the rank's samples: whole launches only
    if (a.gslot && a.outer != 1 && (s_begin != 0 || s_count != S_loc)) return hipErrorInvalidValue;
    const bool fn2 = net_vec_ok(p) && net_fn2_geo(p);
    if (fn2 && p.world > 1 && a.nbands != kFn2Bands) return hipErrorInvalidValue;
    if (p.family == PSVI_FAMILY_MEANFIELD)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_MEANFIELD, false>), grid, block, p.net_lds, st, a);
    else if (fn2 && loop && p.world > 1)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, true, true, true, 2>), grid, block, p.net_lds, st, a);
    else if (fn2 && loop)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, false, true, true, 1>), grid, block, p.net_lds, st, a);
    else if (fn2 && p.world > 1)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, true, true, false, 2>), grid, block, p.net_lds, st, a);
    else if (fn2)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, false, true, false, 1>), grid, block, p.net_lds, st, a);
    else if (loop && p.world > 1)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, true, true, true>), grid, block, p.net_lds, st, a);
    else if (loop)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, false, true, true>), grid, block, p.net_lds, st, a);
    else if (p.world > 1 && net_vec_ok(p))
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, true, true>), grid, block, p.net_lds, st, a);
    else if (p.world > 1)
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, true>), grid, block, p.net_lds, st, a);
    else if (net_vec_ok(p))
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, false, true>), grid, block, p.net_lds, st, a);
    else
        hipLaunchKernelGGL((net_kernel<PSVI_FAMILY_FULLCOV, false>), grid, block, p.net_lds, st, a);
    if (a.gslot && a.outer != 1) {
        hipLaunchKernelGGL(net_slot_sum_kernel, dim3((unsigned)((a.gsz + 255) / 256)), dim3(256), 0,
                           st, (const float*)a.gslot, p.mchunks, a.gsz, gsend);
    }
    return hipGetLastError();
}

}  // namespace psvi
