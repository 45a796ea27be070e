// capi.cpp -- extern "C" boundary of libpsvi_hip.so (declared in include/psvi_hip.h).
//
// Plans hold the immutable geometry of one (family, layer sizes, S, M, world,
// rank) configuration: sample shards, nnz-balanced row shards of every
// full-cov layer, and the device work lists of the packed-triangular kernels.
// Steps are pure stream-ordered kernel launches + hipMemsetAsync (graph
// capturable: no allocation, no synchronisation).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "psvi_diag.h"
#include "psvi_internal.hpp"

namespace psvi {
size_t net_plan_geometry(psvi_plan& p);  // kernels_net.hip
void net_set_lds_limit();                // kernels_net.hip
extern int g_net_ablation;               // kernels_net.hip
extern int g_net_scalar_loads;           // kernels_net.hip
extern unsigned long long* g_net_stamps; // kernels_net.hip
extern int g_upd_ablation;               // kernels_mvn.hip
extern int g_stream_off;                 // kernels_mvn.hip
extern int g_stream_bf_off;              // kernels_mvn.hip
extern unsigned long long* g_bf_stamps;  // kernels_mvn.hip
extern int g_ks_off;                     // kernels_mvn.hip
extern int g_fs_off;                     // kernels_mvn.hip
extern int g_fwd_pair_bf;                  // kernels_mvn.hip
extern int g_stream_fold_off;              // kernels_mvn.hip
extern int g_fs_bf_off;                  // kernels_mvn.hip
extern int g_ks_bf_off;                  // kernels_mvn.hip
static int g_ks_wgs = 0;                 // psvi_debug_set(PSVI_DBG_KSTREAM_WGS): plan creation
extern int g_lenet_abl;                  // kernels_lenet.hip
extern int g_net_split_below;            // kernels_net.hip
extern int g_net_threads;                // kernels_net.hip
extern int g_net_wg_target;              // kernels_net.hip
extern int g_net_mloop_off;              // kernels_net.hip
extern int g_net_geo_off;                // kernels_net.hip
extern int g_fwd_ablation;               // kernels_mvn.hip
extern unsigned long long* g_fwd_stamps; // kernels_mvn.hip
extern unsigned long long* g_upd_stamps; // kernels_mvn.hip
extern unsigned long long* g_rop_stamps; // kernels_rop.hip
extern int g_rop_valu;                     // kernels_rop.hip
}  // namespace psvi

using namespace psvi;

namespace {

thread_local std::string g_err;
int g_stream_wgs = 0;       // psvi_debug_set(PSVI_DBG_STREAM_WGS, n): streaming-update workgroups (0 = 256)
int g_stream_rr = 0;        // psvi_debug_set(PSVI_DBG_STREAM_RR, 1): runs dealt round-robin over XCDs (A/B)
int g_stream_cost = -1;     // psvi_debug_set(PSVI_DBG_STREAM_COST, first% + 1000 diag%): tile cost weights (tuning)
int g_upd_chunk_tiles = 0;  // psvi_debug_set(PSVI_DBG_UPD_CHUNK, n): c-blocks per update chunk (0 = auto)

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* where) {
    g_err = std::string(where) + ": " + hipGetErrorString(e);
    return (int)e;
}

#define HIP_TRY(expr)                                      \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
    } while (0)

constexpr int kFwdKChunk = 256;  // columns of L per forward work item
constexpr int64_t kLenetRowFloats = 2 * 1176 + 400 * 2 + 120 * 2 + 84 * 2 + 10;  // per (s, m): P1, routed d P1, ...

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Row shards.  World > 1 full-cov: whole 64-row bands, so that every rank's
// update and sample work is whole 64 x 64 tiles of L (a band split between
// two ranks would be computed by both).  Band b of a layer holds b + 1 tiles
// (its strict-lower triangle); the bands of all layers are dealt largest
// first to the least-loaded rank (ties: the lower rank), which balances the
// tile counts to within one small band (C4 at 8 ranks: 151..153 of 1,215
// tiles; a contiguous nnz split would make a rank compute up to 216 tiles
// because its partial edge bands count whole).  A rank's rows are the union
// of its bands -- runs of consecutive bands -- and its x-shard columns run
// layer-major in row order.  World 1 (and the replicated mean-field / LeNet
// rows): one run per layer.
void assign_rows(psvi_plan& p) {
    for (int q = 0; q < p.world; ++q) {
        p.rows_tot[q] = 0;
        p.runs[q].clear();
    }
    p.band_owner.clear();
    p.band_coloff.clear();
    int nbt = 0;
    for (int l = 0; l < p.L; ++l) {
        p.band_base[l] = nbt;
        nbt += (p.lay[l].n - 1) / 64 + 1;
    }
    p.band_base[p.L] = nbt;
    const bool banded = p.family == PSVI_FAMILY_FULLCOV && p.world > 1;
    std::vector<int> owner(nbt, 0);
    if (banded) {
        std::vector<int> order(nbt);
        std::vector<double> cost(nbt);
        for (int l = 0; l < p.L; ++l)
            for (int b = 0; b < p.band_base[l + 1] - p.band_base[l]; ++b)
                cost[p.band_base[l] + b] = b + 1.0;
        for (int i = 0; i < nbt; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
        std::vector<double> load(p.world, 0.0);
        for (int i : order) {
            const int q = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            owner[i] = q;
            load[q] += cost[i];
        }
    }
    p.band_coloff.assign(nbt, 0);
    for (int q = 0; q < p.world; ++q)
        for (int l = 0; l < p.L; ++l) {
            const int n = p.lay[l].n;
            p.xcol_l[q][l] = p.rows_tot[q];
            for (int b = 0; 64 * b < n; ++b) {
                const int gb = p.band_base[l] + b;
                if (banded && owner[gb] != q) continue;
                const int r0 = 64 * b, r1 = std::min(n, r0 + 64);
                std::vector<ShardRun>& rv = p.runs[q];
                if (!rv.empty() && rv.back().layer == l && rv.back().hi == r0)
                    rv.back().hi = r1;
                else
                    rv.push_back(ShardRun{l, r0, r1, p.rows_tot[q]});
                p.band_coloff[gb] = p.rows_tot[q] - r0;
                p.rows_tot[q] += r1 - r0;
            }
        }
    p.band_owner = owner;
}

template <class T>
int upload(const std::vector<T>& v, T** dst) {
    *dst = nullptr;
    if (v.empty()) return 0;
    HIP_TRY(hipMalloc((void**)dst, sizeof(T) * v.size()));
    HIP_TRY(hipMemcpy(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    return 0;
}

int check_desc(const psvi_net_desc* d) {
    if (!d) return fail(PSVI_EINVAL, "null descriptor");
    if (d->n_layers < 1 || d->n_layers > PSVI_MAX_LAYERS)
        return fail(PSVI_EINVAL, "n_layers out of range [1, 8]");
    for (int l = 0; l <= d->n_layers; ++l)
        if (d->dims[l] < 1) return fail(PSVI_EINVAL, "layer dims must be >= 1");
    if (d->S < 1) return fail(PSVI_EINVAL, "S must be >= 1");
    if (d->M < 1) return fail(PSVI_EINVAL, "M must be >= 1");
    if (!(d->prior_sd > 0.f)) return fail(PSVI_EINVAL, "prior_sd must be > 0");
    return 0;
}

// Workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8), each with
// its own L2.  Keep every band's chunks on one XCD (its G slice and the eps
// blocks it shares with neighbouring bands then stay in that L2): bands go
// greedily, largest first, to the least-loaded XCD; each XCD's chunks run
// largest first; the per-XCD queues are interleaved at stride 8 and padded
// with empty chunks (k0 == k1, no work).
static std::vector<UpdChunk> xcd_order(const std::vector<UpdChunk>& in) {
    constexpr int kXcd = 8;
    auto work = [](const UpdChunk& c) { return (c.k1 - c.k0) + c.diag; };
    std::vector<std::vector<UpdChunk>> band;  // chunks of one (layer, r0)
    for (const UpdChunk& c : in) {
        if (band.empty() || band.back()[0].layer != c.layer || band.back()[0].r0 != c.r0)
            band.emplace_back();
        band.back().push_back(c);
    }
    std::vector<int> bw(band.size());
    for (size_t i = 0; i < band.size(); ++i)
        for (const UpdChunk& c : band[i]) bw[i] += work(c);
    std::vector<size_t> idx(band.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return bw[a] > bw[b]; });
    std::vector<std::vector<UpdChunk>> q(kXcd);
    std::vector<long> load(kXcd, 0);
    for (size_t i : idx) {
        const int x = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        load[x] += bw[i];
        q[x].insert(q[x].end(), band[i].begin(), band[i].end());
    }
    size_t len = 0;
    for (auto& v : q) {
        std::stable_sort(v.begin(), v.end(),
                         [&](const UpdChunk& a, const UpdChunk& b) { return work(a) > work(b); });
        len = std::max(len, v.size());
    }
    std::vector<UpdChunk> out;
    out.reserve(len * kXcd);
    const UpdChunk empty{0, 0, 0, 0, 0, 0, 0, 0, -1};
    for (size_t j = 0; j < len; ++j)
        for (int x = 0; x < kXcd; ++x) out.push_back(j < q[x].size() ? q[x][j] : empty);
    return out;
}

// K-split streaming update tables (S > 128): the rank's tiles band-major
// (the diagonal tile last in its band), units (tile, 128-sample pass) cut
// into equal-cost contiguous runs -- a tile's last unit also carries its
// Adam epilogue (about half a pass) -- one run per workgroup, two workgroups
// per CU.  XCD-aware placement as the stream kernel: workgroup w runs on XCD
// w % 8, so XCD x takes a contiguous eighth of the run list (its bands' G
// slices and eps column blocks stay in that XCD's L2).
void build_kstream(psvi_plan& p) {
    const int r = p.rank, np = (p.d.S + kKsPass - 1) / kKsPass;
    std::vector<KsTile>& tiles = p.h_ks_tiles;
    tiles.clear();
    for (const ShardRun& run : p.runs[r])
        for (int b = run.lo / 64; 64 * b < run.hi; ++b)
            for (int k = 0; k <= b; ++k)
                tiles.push_back(KsTile{run.layer, 64 * b, k, k == b, 64 * b,
                                       std::min(64 * b + 64, p.lay[run.layer].n), run.col - run.lo, -1});
    const int T = (int)tiles.size();
    p.h_ks_segs.clear();
    p.h_ks_off.clear();
    p.n_kwg = p.n_ks_slots = p.n_ks_cnt = 0;
    if (T == 0) return;
    const int64_t U = (int64_t)T * np;
    int nwg = (int)std::min<int64_t>(U, g_ks_wgs > 0 ? g_ks_wgs : 512);
    if (nwg >= 8) nwg -= nwg % 8;
    // unit cost: 1 per pass, + 0.5 on a tile's last pass (its epilogue)
    std::vector<double> cum(U + 1, 0.0);
    for (int64_t u = 0; u < U; ++u) cum[u + 1] = cum[u] + 1.0 + (u % np == np - 1 ? 0.5 : 0.0);
    std::vector<int64_t> cut(nwg + 1, 0);
    cut[nwg] = U;
    for (int w = 1; w < nwg; ++w) {
        const double target = cum[U] * w / nwg;
        int64_t t = (int64_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        cut[w] = std::max(cut[w - 1] + 1, std::min(t, U - (nwg - w)));
    }
    // contributors per tile
    std::vector<int> ncon(T, 0);
    for (int w = 0; w < nwg; ++w)
        for (int64_t u = cut[w]; u < cut[w + 1];) {
            const int t = (int)(u / np);
            ++ncon[t];
            u = std::min<int64_t>(cut[w + 1], (int64_t)(t + 1) * np);
        }
    std::vector<int> slot0(T, -1), seen(T, 0);
    for (int t = 0; t < T; ++t)
        if (ncon[t] > 1) {
            slot0[t] = p.n_ks_slots;
            p.n_ks_slots += ncon[t];
            tiles[t].cnt = p.n_ks_cnt++;
        }
    std::vector<std::vector<KsSeg>> per(nwg);
    for (int w = 0; w < nwg; ++w)
        for (int64_t u = cut[w]; u < cut[w + 1];) {
            const int t = (int)(u / np);
            const int64_t ue = std::min<int64_t>(cut[w + 1], (int64_t)(t + 1) * np);
            per[w].push_back(KsSeg{t, (int)(u - (int64_t)t * np), (int)(ue - (int64_t)t * np),
                                   slot0[t], ncon[t], seen[t]++});
            u = ue;
        }
    // XCD placement: workgroup w -> run (w % 8) * (nwg / 8) + w / 8
    std::vector<int> run_of(nwg);
    for (int w = 0; w < nwg; ++w)
        run_of[w] = (nwg % 8 == 0) ? (w % 8) * (nwg / 8) + w / 8 : w;
    p.h_ks_off.push_back(0);
    for (int w = 0; w < nwg; ++w) {
        const auto& v = per[run_of[w]];
        p.h_ks_segs.insert(p.h_ks_segs.end(), v.begin(), v.end());
        p.h_ks_off.push_back((int)p.h_ks_segs.size());
    }
    p.n_kwg = nwg;
}

// Segmented sample tables (S > 128): units (row block of 64, 128-sample pass,
// 64-column block of L) ordered row block-major, then pass, then column block
// (a run accumulates x over consecutive column blocks of one (row block,
// pass)); equal-count contiguous runs, one per workgroup, two workgroups per
// CU; a run's piece of one (row block, pass) is a segment writing its own
// slot, and the reduce adds a (row block, pass)'s slots in segment order.
// XCD placement as the K-split update: workgroup w -> run (w % 8) (nwg / 8) + w / 8.
// One table for nwg_max workgroups (into segs / off / rbs and the counts).
static void build_fseg_table(const psvi_plan& p, int nwg_max, std::vector<FsSeg>& segs,
                             std::vector<int>& off, std::vector<FwdRowBlock>& rbs, int& n_wg,
                             int& n_slots, int& n_rb) {
    const int r = p.rank, np = (p.d.S + kKsPass - 1) / kKsPass;
    struct Blk {
        int layer, r0, r1, xcol, nkb;
    };
    std::vector<Blk> blks;
    for (const ShardRun& run : p.runs[r]) {
        const int n = p.lay[run.layer].n;
        for (int r0 = run.lo; r0 < run.hi; r0 += kFwdRows) {
            const int r1 = std::min(r0 + kFwdRows, run.hi);
            const int kmax = std::max(0, std::min(r1 - 1, n - 2));
            blks.push_back(Blk{run.layer, r0, r1, run.col + (r0 - run.lo), (kmax + 63) / 64});
        }
    }
    segs.clear();
    off.clear();
    rbs.clear();
    n_wg = n_slots = n_rb = 0;
    const int B = (int)blks.size();
    std::vector<int64_t> ub(B + 1, 0);
    for (int b = 0; b < B; ++b) ub[b + 1] = ub[b] + (int64_t)blks[b].nkb * np;
    const int64_t U = ub[B];
    if (U == 0) return;
    int nwg = (int)std::min<int64_t>(U, nwg_max);
    if (nwg >= 8) nwg -= nwg % 8;
    std::vector<int64_t> cut(nwg + 1);
    for (int w = 0; w <= nwg; ++w) cut[w] = U * w / nwg;
    // segments per workgroup; group g = b * np + pass
    struct Piece {
        int b, pass, kb0, kb1;
    };
    std::vector<std::vector<Piece>> per(nwg);
    std::vector<int> nseg((size_t)B * np, 0);
    for (int w = 0; w < nwg; ++w) {
        int b = (int)(std::upper_bound(ub.begin(), ub.end(), cut[w]) - ub.begin()) - 1;
        for (int64_t u = cut[w]; u < cut[w + 1];) {
            while (u >= ub[b + 1]) ++b;
            const int nkb = blks[b].nkb;
            const int pass = (int)((u - ub[b]) / nkb), kb = (int)((u - ub[b]) % nkb);
            const int64_t ue = std::min<int64_t>(cut[w + 1], ub[b] + (int64_t)(pass + 1) * nkb);
            per[w].push_back(Piece{b, pass, kb, kb + (int)(ue - u)});
            ++nseg[(size_t)b * np + pass];
            u = ue;
        }
    }
    std::vector<int> slot0((size_t)B * np), seen((size_t)B * np, 0);
    for (int b = 0; b < B; ++b)
        for (int q = 0; q < np; ++q) {
            const size_t g = (size_t)b * np + q;
            slot0[g] = n_slots;
            n_slots += nseg[g];
            rbs.push_back(FwdRowBlock{nseg[g] > 0 ? slot0[g] : 0, nseg[g], blks[b].r1 - blks[b].r0,
                                            blks[b].xcol, blks[b].layer, blks[b].r0, kKsPass * q});
        }
    off.push_back(0);
    for (int w = 0; w < nwg; ++w) {
        const int run = (nwg % 8 == 0) ? (w % 8) * (nwg / 8) + w / 8 : w;
        for (const Piece& pc : per[run]) {
            const Blk& bk = blks[pc.b];
            const size_t g = (size_t)pc.b * np + pc.pass;
            segs.push_back(FsSeg{bk.layer, bk.r0, bk.r1, pc.pass, 64 * pc.kb0, 64 * pc.kb1,
                                 slot0[g] + seen[g]++, 0});
        }
        off.push_back((int)segs.size());
    }
    n_wg = nwg;
    n_rb = (int)rbs.size();
}

// The sample's table over 512 workgroups (two per CU), and the HVP pair's over
// 256 (one eight-wave workgroup per CU: runs twice as long, fewer slots).
void build_fseg(psvi_plan& p) {
    build_fseg_table(p, 512, p.h_fs_segs, p.h_fs_off, p.h_fs_rb, p.n_fswg, p.n_fs_slots, p.n_fs_rb);
    build_fseg_table(p, 256, p.h_fp_segs, p.h_fp_off, p.h_fp_rb, p.n_fpwg, p.n_fp_slots, p.n_fp_rb);
}

// make_lenet (neural_net.py:334-359): five mean-field-style layers, the first
// two convolutions ("din" = in_channels * 25), the last one a single shared
// sample.  Samples are sharded like the mean-field family.
int build_lenet_plan(psvi_plan& p) {
    static const int din[5] = {25, 150, 400, 120, 84}, dout[5] = {6, 16, 120, 84, 10};
    const int S = p.d.S;
    p.d.n_layers = 5;
    p.d.dims[0] = 784;
    for (int l = 0; l < 5; ++l) p.d.dims[l + 1] = dout[l];
    p.L = 5;
    int64_t po = 0, eo = 0;
    int wo = 0;
    for (int l = 0; l < 5; ++l) {
        LayerInfo& li = p.lay[l];
        li.din = din[l];
        li.dout = dout[l];
        li.n = din[l] * dout[l] + dout[l];
        li.nc = 0;
        li.poff = po;
        li.eoff = eo;
        li.woff = wo;
        po += 2 * (int64_t)li.n;
        eo += (l < 4 ? (int64_t)S : 1) * li.n;
        wo += li.n;
    }
    p.P = po;
    p.Peps = eo;
    p.n_tot = wo;
    for (int q = 0; q < p.world; ++q) {
        const int base = S / p.world, rem = S % p.world;
        p.s_cnt[q] = base + (q < rem ? 1 : 0);
        p.s_off[q] = q * base + std::min(q, rem);
        p.rows_tot[q] = 0;
    }
    p.acc_count = 2 * (int64_t)p.n_tot;
    p.ws_bytes = align256(sizeof(float) * (size_t)p.acc_count);
    const int64_t kMaxOff = (int64_t(1) << 31) - 4096;
    if (p.Peps > kMaxOff || (int64_t)p.s_cnt[p.rank] * p.d.M * kLenetRowFloats > kMaxOff * 4)
        return fail(PSVI_EUNSUP, "LeNet scratch beyond the supported size");
    return 0;
}

int build_plan(psvi_plan& p) {
    if (p.family == PSVI_FAMILY_LENET) return build_lenet_plan(p);
    const psvi_net_desc& d = p.d;
    p.L = d.n_layers;
    int64_t po = 0, eo = 0;
    int wo = 0;
    for (int l = 0; l < p.L; ++l) {
        LayerInfo& li = p.lay[l];
        li.din = d.dims[l];
        li.dout = d.dims[l + 1];
        li.n = li.din * li.dout + li.dout;
        li.nc = (int64_t)(li.n - 1) * (li.n - 2) / 2;
        li.poff = po;
        li.eoff = eo;
        li.woff = wo;
        po += p.family == PSVI_FAMILY_MEANFIELD ? 2 * (int64_t)li.n : 2 * (int64_t)li.n + li.nc;
        eo += (int64_t)d.S * li.n;
        wo += li.n;
    }
    p.P = po;
    p.Peps = eo;
    int64_t tb = 0;
    for (int l = 0; l < p.L; ++l) {
        LayerInfo& li = p.lay[l];
        li.nb = p.family == PSVI_FAMILY_FULLCOV ? (li.n - 1) / 64 + 1 : 0;
        li.tbase = tb;
        tb += (int64_t)li.nb * (li.nb + 1) / 2;
    }
    p.tiles_total = tb;
    p.n_tot = wo;
    // sample shards
    for (int q = 0; q < p.world; ++q) {
        const int base = d.S / p.world, rem = d.S % p.world;
        p.s_cnt[q] = base + (q < rem ? 1 : 0);
        p.s_off[q] = q * base + std::min(q, rem);
    }
    // row shards
    assign_rows(p);
    p.acc_count = 2 * (int64_t)p.n_tot;
    net_plan_geometry(p);
    if (p.net_lds > 160 * 1024)
        return fail(PSVI_EUNSUP, "layer too wide for the per-sample LDS network kernel");
    // the kernels address parameters, eps and the x / g shards with 32-bit offsets
    const int64_t kMaxOff = (int64_t(1) << 31) - 4096;
    int rows_max = 0;
    for (int q = 0; q < p.world; ++q) rows_max = std::max(rows_max, p.rows_tot[q]);
    if (p.P > kMaxOff || p.Peps > kMaxOff || (int64_t)d.S * rows_max > kMaxOff ||
        (int64_t)d.S * p.n_tot > kMaxOff)
        return fail(PSVI_EUNSUP, "buffers beyond 2^31 floats are not supported");

    const int S = d.S, r = p.rank;
    if (p.family == PSVI_FAMILY_FULLCOV) {
        std::vector<FwdItem> fwd;
        std::vector<UpdChunk> upd;
        std::vector<FwdRowBlock> frb, ufrb;
        int nslots = 0;
        // c-blocks per update chunk: about one chunk per workgroup slot
        // (256 CUs x 3 resident update workgroups), at least one
        int tiles = 0;
        for (const ShardRun& run : p.runs[r])
            for (int b = run.lo / 64; 64 * b < run.hi; ++b) tiles += b + 1;
        const int ch = g_upd_chunk_tiles > 0 ? g_upd_chunk_tiles : std::max(1, (tiles + 511) / 512);
        for (const ShardRun& run : p.runs[r]) {
            const int l = run.layer, n = p.lay[l].n, lo = run.lo, hi = run.hi;
            const int xc = run.col;
            for (int r0 = lo; r0 < hi; r0 += kFwdRows) {
                const int r1 = std::min(r0 + kFwdRows, hi);
                const int kmax = std::max(0, std::min(r1 - 1, n - 2));
                const int nit = std::max(1, (kmax + kFwdKChunk - 1) / kFwdKChunk);
                // even split, multiples of 64 columns (the kernel's LDS stage)
                const int steps = (kmax + 63) / 64;
                const int slot0 = (int)fwd.size();
                for (int i = 0; i < nit; ++i) {
                    const int k0 = std::min(kmax, 64 * (int)((int64_t)steps * i / nit));
                    const int k1 = std::min(kmax, 64 * (int)((int64_t)steps * (i + 1) / nit));
                    if (i > 0 && k0 >= k1) continue;
                    fwd.push_back(FwdItem{l, r0, r1, k0, k1, xc + (r0 - lo), (int)fwd.size()});
                }
                frb.push_back(FwdRowBlock{slot0, (int)fwd.size() - slot0, r1 - r0, xc + (r0 - lo), l, r0});
            }
            // bands of 64 absolute rows; c-blocks 0..b, the last one diagonal.
            // Each band is also a row block of the fused next-step sample: its
            // chunks' partial slots are consecutive.
            for (int b = lo / 64; 64 * b < hi; ++b) {
                const int slot0 = nslots;
                for (int k0 = 0; k0 <= b; k0 += ch) {
                    const int k1 = std::min(b + 1, k0 + ch);
                    upd.push_back(UpdChunk{l, 64 * b, k0, k1, lo, hi, xc - lo, k1 == b + 1, nslots++});
                }
                const int r0 = std::max(64 * b, lo), r1 = std::min(64 * b + 64, hi);
                ufrb.push_back(FwdRowBlock{slot0, nslots - slot0, r1 - r0, xc + (r0 - lo), l, r0});
            }
        }
        // longest forward items first
        std::stable_sort(fwd.begin(), fwd.end(), [](const FwdItem& a, const FwdItem& b) {
            return (a.k1 - a.k0) > (b.k1 - b.k0);
        });
        p.h_fwd = fwd;
        p.h_frb = frb;
        p.n_frb = (int)frb.size();
        p.h_upd = xcd_order(upd);
        // fusion needs band-aligned row blocks (rank row ranges start at 0) and
        // one LDS pass of samples
        p.fuse_sample = p.world == 1 && S <= 128;
        p.h_ufrb = ufrb;
        p.n_ufrb = (int)ufrb.size();
        p.n_uslots = nslots;
        // streaming fused update: the tile list (layer-major, band-major, the
        // diagonal tile last in its band) cut into equal contiguous runs, one
        // per workgroup (one workgroup per CU)
        if (p.fuse_sample && S % 32 == 0 && p.world == 1) {
            std::vector<uint32_t> tmap;
            std::vector<int> tband;  // band id per tile
            int nband = 0;
            for (int l = 0; l < p.L; ++l)
                for (int b = 0; b < p.lay[l].nb; ++b, ++nband)
                    for (int k = 0; k <= b; ++k) {
                        tmap.push_back((uint32_t)l << 28 | (uint32_t)b << 14 | (uint32_t)k);
                        tband.push_back(nband);
                    }
            const int T = (int)tmap.size();
            const int nwg = std::max(1, std::min(g_stream_wgs > 0 ? g_stream_wgs : 256, T));
            // equal-cost runs: a band's diagonal (last) tile also updates the
            // band's mean / sd, flushes its slot, drains and takes the band's
            // ticket (and, for the last arriver, the combine after the walk); a
            // band's first tile follows a G reload and split.  Weights 1.5 and
            // 1.0 of a plain tile: the fastest of a sweep at C3
            // (tools/stream_cost_sweep.py: 55.7 - 56.3 us per step against 58.4
            // at the round-5 weights 0.35 / 0.4, which predate the in-kernel
            // combine); workgroup stamps (tools/bf_stamps.py) show the slowest
            // workgroups are the ones with band boundaries
            std::vector<double> cum(T + 1, 0.0);
            for (int t = 0; t < T; ++t) {
                const uint32_t k = tmap[t] & 0x3fff, b = (tmap[t] >> 14) & 0x3fff;
                const double wd = g_stream_cost >= 0 ? (g_stream_cost / 1000) * 0.01 : 1.5;
                const double wf = g_stream_cost >= 0 ? (g_stream_cost % 1000) * 0.01 : 1.0;
                cum[t + 1] = cum[t] + 1.0 + (k == b ? wd : 0.0) + (k == 0 ? wf : 0.0);
            }
            std::vector<int> cut(nwg + 1, 0);
            cut[nwg] = T;
            for (int w = 1; w < nwg; ++w) {
                const double target = cum[T] * w / nwg;
                int t = (int)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
                cut[w] = std::max(cut[w - 1] + 1, std::min(t, T - (nwg - w)));
            }
            std::vector<std::vector<int>> band_slots(nband);
            int ns = 0;
            for (int w = 0; w < nwg; ++w) {
                const int t0 = cut[w], t1 = cut[w + 1];
                p.h_str.push_back(StreamRange{t0, t1, ns, t0 < T ? tmap[t0] : 0u});
                int ends = 0;
                for (int t = t0; t < t1; ++t)
                    if (t == t0 || tband[t] != tband[t - 1]) {
                        band_slots[tband[t]].push_back(ns++);
                        ++ends;
                    }
                p.str_max_ends = std::max(p.str_max_ends, ends);
            }
            int bid = 0;
            for (int l = 0; l < p.L; ++l)
                for (int b = 0; b < p.lay[l].nb; ++b, ++bid) {
                    const int r0 = 64 * b, R = std::min(64, p.lay[l].n - r0);
                    const auto& sl = band_slots[bid];
                    p.h_sfrb.push_back(FwdRowBlock{sl.front(), (int)sl.size(), R,
                                                   p.xcol_l[r][l] + r0, l, r0});
                }
            // XCD-aware placement: workgroup w runs on XCD w % 8 (round-robin
            // dispatch), so XCD x takes the contiguous eighth [x per, (x + 1) per)
            // of the run list -- its bands' G slices and the eps / eps' columns
            // up to its last band stay in that XCD's L2 instead of every XCD
            // touching every band of both layers
            if (nwg % 8 == 0 && !g_stream_rr) {
                const int per = nwg / 8;
                std::vector<StreamRange> xr(nwg);
                for (int w = 0; w < nwg; ++w) xr[w] = p.h_str[(w % 8) * per + w / 8];
                p.h_str.swap(xr);
            }
            p.n_str = (int)p.h_str.size();
            p.n_sfrb = (int)p.h_sfrb.size();
            p.n_sslots = ns;
        }
        p.upd_tiles = tiles;
        // the K-split tables at every S: the Adam update at S > 128, the
        // gradient mode (the HVP's reparameterised backward) at any S
        build_kstream(p);
        // the segmented sample at every S (x_0 of a loop, the HVP's tangent
        // sample, the sharded step): equal runs over 512 workgroups
        build_fseg(p);
        p.n_fwd = (int)fwd.size();
        p.n_upd = (int)p.h_upd.size();
        const size_t xs = sizeof(float) * (size_t)S * p.rows_tot[r];
        p.ws_bytes = align256(xs) * 2 + 256;
    } else {
        p.ws_bytes = align256(sizeof(float) * (size_t)p.acc_count);
    }
    return 0;
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Diagnostics (PSVI_DBG_LOOP_TIMING): HIP events around the network and the
// update launches of every `g_loop_every`-th full-cov inner-loop step.
int g_loop_every = 0;
std::vector<hipEvent_t> g_loop_ev[2];  // [net, update] x (start, end) pairs

void loop_events_clear() {
    for (auto& v : g_loop_ev) {
        for (hipEvent_t e : v) (void)hipEventDestroy(e);
        v.clear();
    }
}

// records the next start or end event of phase k on the stream
hipError_t loop_event(int k, hipStream_t st) {
    hipEvent_t e;
    const hipError_t rc = hipEventCreate(&e);
    if (rc != hipSuccess) return rc;
    g_loop_ev[k].push_back(e);
    return hipEventRecord(e, st);
}

}  // namespace

extern "C" {

const char* psvi_last_error(void) { return g_err.c_str(); }
const char* psvi_version(void) { return "psvi_hip 0.1.0 (gfx950)"; }

int psvi_debug_set(int32_t key, int32_t value) {
    switch (key) {
        case PSVI_DBG_LOOP_TIMING: loop_events_clear(); g_loop_every = value; return 0;
        case PSVI_DBG_NET_ABLATION: g_net_ablation = value; return 0;
        case PSVI_DBG_UPD_ABLATION: g_upd_ablation = value; return 0;
        case PSVI_DBG_NET_SPLIT_BELOW: g_net_split_below = value; return 0;
        case PSVI_DBG_NET_WG_TARGET:
            if (value < 1) return fail(PSVI_EINVAL, "workgroup target must be >= 1");
            g_net_wg_target = value;
            return 0;
        case PSVI_DBG_FWD_ABLATION: g_fwd_ablation = value; return 0;
        case PSVI_DBG_UPD_CHUNK: g_upd_chunk_tiles = value; return 0;
        case PSVI_DBG_UPD_STREAM_OFF: g_stream_off = value; return 0;
        case PSVI_DBG_STREAM_BF_OFF: g_stream_bf_off = value; return 0;
        case PSVI_DBG_KSTREAM_OFF: g_ks_off = value; return 0;
        case PSVI_DBG_KSTREAM_WGS: g_ks_wgs = value; return 0;
        case PSVI_DBG_FWD_SEG_OFF: g_fs_off = value; return 0;
        case PSVI_DBG_FWD_SEG_BF_OFF: g_fs_bf_off = value; return 0;
        case PSVI_DBG_FWD_PAIR_BF: g_fwd_pair_bf = value; return 0;
        case PSVI_DBG_STREAM_FOLD_OFF: g_stream_fold_off = value; return 0;
        case PSVI_DBG_KSTREAM_BF_OFF: g_ks_bf_off = value; return 0;
        case PSVI_DBG_ROP_VALU: g_rop_valu = value; return 0;
        case PSVI_DBG_NET_SCALAR_LOADS: g_net_scalar_loads = value; return 0;
        case PSVI_DBG_NET_MLOOP_OFF: g_net_mloop_off = value; return 0;
        case PSVI_DBG_NET_GEO_OFF: g_net_geo_off = value; return 0;
        case PSVI_DBG_STREAM_WGS: g_stream_wgs = value; return 0;
        case PSVI_DBG_STREAM_COST: g_stream_cost = value; return 0;
        case PSVI_DBG_STREAM_RR: g_stream_rr = value; return 0;
        case PSVI_DBG_LENET_ABLATION: g_lenet_abl = value; return 0;
        case PSVI_DBG_NET_THREADS:
            if (value != 0 && value != 256 && value != 512) return fail(PSVI_EINVAL, "256 or 512");
            g_net_threads = value;
            return 0;
        default: return fail(PSVI_EINVAL, "unknown debug key");
    }
}

int psvi_debug_loop_timing(double* out) {
    if (!out) return fail(PSVI_EINVAL, "null out");
    for (int k = 0; k < 2; ++k) {
        double sum = 0.0;
        const auto& v = g_loop_ev[k];
        for (size_t i = 0; i + 1 < v.size(); i += 2) {
            float ms = 0.f;
            HIP_TRY(hipEventSynchronize(v[i + 1]));
            HIP_TRY(hipEventElapsedTime(&ms, v[i], v[i + 1]));
            sum += ms;
        }
        const size_t n = v.size() / 2;
        out[k] = n ? 1e3 * sum / (double)n : 0.0;
        if (k == 0) out[2] = (double)n;
    }
    loop_events_clear();
    return 0;
}

int psvi_debug_set_ptr(int32_t key, void* ptr) {
    switch (key) {
        case PSVI_DBG_NET_STAMPS: g_net_stamps = (unsigned long long*)ptr; return 0;
        case PSVI_DBG_UPD_STAMPS: g_upd_stamps = (unsigned long long*)ptr; return 0;
        case PSVI_DBG_BF_STAMPS: g_bf_stamps = (unsigned long long*)ptr; return 0;
        case PSVI_DBG_ROP_STAMPS: g_rop_stamps = (unsigned long long*)ptr; return 0;
        case PSVI_DBG_FWD_STAMPS: g_fwd_stamps = (unsigned long long*)ptr; return 0;
        default: return fail(PSVI_EINVAL, "unknown debug key");
    }
}

int psvi_plan_create(int32_t family, const psvi_net_desc* d, int32_t world, int32_t rank,
                     psvi_plan** out) {
    if (!out) return fail(PSVI_EINVAL, "null out");
    *out = nullptr;
    if (family != PSVI_FAMILY_MEANFIELD && family != PSVI_FAMILY_FULLCOV &&
        family != PSVI_FAMILY_LENET)
        return fail(PSVI_EINVAL, "unknown family");
    psvi_net_desc dl;
    if (family == PSVI_FAMILY_LENET && d) {  // fixed architecture: dims ignored
        dl = *d;
        dl.n_layers = 5;
        const int dims[6] = {784, 6, 16, 120, 84, 10};
        for (int l = 0; l < 6; ++l) dl.dims[l] = dims[l];
        d = &dl;
    }
    if (int rc = check_desc(d)) return rc;
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world)
        return fail(PSVI_EINVAL, "world/rank out of range (world <= 8)");
    int ndev = 0;
    const bool have_dev = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
    if (have_dev) {
        static std::once_flag once;
        std::call_once(once, net_set_lds_limit);
    }
    psvi_plan* p = new psvi_plan();
    p->family = family;
    p->d = *d;
    p->world = world;
    p->rank = rank;
    int rc = build_plan(*p);
    if (!rc && family == PSVI_FAMILY_FULLCOV && world == 1 && p->fuse_sample && p->tiles_total > 0 &&
        p->n_str > 0 && p->d.S == 128) {
        // the streaming update's bf16 planes of every draw (EpsPlanes): rows
        // padded to 64-column multiples, layers back to back
        psvi::EpsPlanes& E = p->eps_planes;
        E.L = p->L;
        int64_t po = 0, eo = 0;
        for (int l = 0; l < p->L; ++l) {
            const int n = p->lay[l].n;
            E.eoff[l] = eo;
            E.n[l] = n;
            E.npad[l] = (n + 63) / 64 * 64;
            E.poff[l] = po;
            eo += (int64_t)p->d.S * n;
            po += (int64_t)p->d.S * E.npad[l];
        }
        E.eoff[p->L] = eo;
        E.pl = (po + 63) / 64 * 64;
        p->bf_stream = eo == p->Peps;
    }
    if (!rc && have_dev) {
        // the only device allocations of the library: immutable work lists
        if (!(rc = upload(p->h_fwd, &p->d_fwd)) && !(rc = upload(p->h_frb, &p->d_frb)))
            rc = upload(p->h_upd, &p->d_upd);
        if (!rc && p->n_fwd > 0) {
            // split-K scratch of the sample phase (plan-owned, reused every step)
            const size_t bytes = sizeof(float) * (size_t)p->n_fwd * p->d.S * kFwdRows;
            if (hipMalloc((void**)&p->d_fwd_part, bytes) != hipSuccess)
                rc = fail(PSVI_EUNSUP, "cannot allocate the sample-phase scratch");
        }
        if (!rc && p->fuse_sample && p->n_uslots > 0) {
            const size_t bytes = sizeof(float) * (size_t)p->n_uslots * p->d.S * 64;
            if ((rc = upload(p->h_ufrb, &p->d_ufrb)) == 0 &&
                hipMalloc((void**)&p->d_upd_part, bytes) != hipSuccess)
                rc = fail(PSVI_EUNSUP, "cannot allocate the fused-sample scratch");
        }
        if (!rc && p->n_str > 0) {
            const size_t bytes = sizeof(float) * (size_t)p->n_sslots * p->d.S * 64;
            if (!(rc = upload(p->h_str, &p->d_str)) && !(rc = upload(p->h_sfrb, &p->d_sfrb)) &&
                (hipMalloc((void**)&p->d_str_part, bytes) != hipSuccess ||
                 hipMalloc((void**)&p->d_str_cnt, sizeof(int) * (size_t)std::max(1, p->n_sfrb)) != hipSuccess ||
                 hipMemset(p->d_str_cnt, 0, sizeof(int) * (size_t)std::max(1, p->n_sfrb)) != hipSuccess ||
                 hipMalloc((void**)&p->d_str_bms, sizeof(float) * 128 * (size_t)std::max(1, p->n_sfrb)) != hipSuccess))
                rc = fail(PSVI_EUNSUP, "cannot allocate the streaming-update scratch");
        }
        if (!rc && p->n_kwg > 0) {
            if (!(rc = upload(p->h_ks_tiles, &p->d_ks_tiles)) &&
                !(rc = upload(p->h_ks_segs, &p->d_ks_segs)))
                rc = upload(p->h_ks_off, &p->d_ks_off);
            const size_t sb = sizeof(float) * (size_t)std::max(1, p->n_ks_slots) * kKsSlotFloats;
            if (!rc && (hipMalloc((void**)&p->d_ks_slots, sb) != hipSuccess ||
                        hipMalloc((void**)&p->d_ks_cnt, sizeof(int) * std::max(1, p->n_ks_cnt)) !=
                            hipSuccess ||
                        hipMemset(p->d_ks_cnt, 0, sizeof(int) * std::max(1, p->n_ks_cnt)) !=
                            hipSuccess))
                rc = fail(PSVI_EUNSUP, "cannot allocate the K-split update's slots");
        }
        if (!rc && p->n_fswg > 0) {
            if (!(rc = upload(p->h_fs_segs, &p->d_fs_segs)) && !(rc = upload(p->h_fs_off, &p->d_fs_off)))
                rc = upload(p->h_fs_rb, &p->d_fs_rb);
            if (!rc && !(rc = upload(p->h_fp_segs, &p->d_fp_segs)) && !(rc = upload(p->h_fp_off, &p->d_fp_off)))
                rc = upload(p->h_fp_rb, &p->d_fp_rb);
            // (the slots serve both tables)
            const size_t sb = sizeof(float) * (size_t)std::max({1, p->n_fs_slots, p->n_fp_slots}) * kKsPass *
                              kFwdRows;
            if (!rc && hipMalloc((void**)&p->d_fs_part, sb) != hipSuccess)
                rc = fail(PSVI_EUNSUP, "cannot allocate the segmented sample's slots");
        }
        if (!rc && family == PSVI_FAMILY_FULLCOV) {
            std::vector<uint32_t> xmap;
            std::vector<NetBand> bands;
            net_xmap(*p, xmap, bands);
            if (!(rc = upload(xmap, &p->d_net_xmap)))
                rc = upload(bands, &p->d_net_bands);
        }
        if (!rc && family == PSVI_FAMILY_FULLCOV && p->mchunks > 1) {
            const size_t bytes = sizeof(float) * (size_t)p->mchunks *
                                 std::max(1, p->s_cnt[p->rank]) * p->n_tot;
            if (hipMalloc((void**)&p->d_net_slots, bytes) != hipSuccess)
                rc = fail(PSVI_EUNSUP, "cannot allocate the network's pseudopoint-chunk slots");
        }
        if (!rc && family == PSVI_FAMILY_MEANFIELD) {
            const size_t bytes = sizeof(float) * (size_t)std::max(1, p->s_cnt[p->rank]) *
                                 p->mchunks * p->n_tot;
            if (hipMalloc((void**)&p->d_mf_slots, bytes) != hipSuccess)
                rc = fail(PSVI_EUNSUP, "cannot allocate the mean-field gradient slots");
        }
        if (!rc && p->family == PSVI_FAMILY_FULLCOV && p->fuse_sample && p->tiles_total > 0 &&
            (hipStreamCreateWithFlags(&p->aux_st, hipStreamNonBlocking) != hipSuccess ||
             hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming) != hipSuccess ||
             hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming) != hipSuccess))
            rc = fail(PSVI_EUNSUP, "cannot create the inner loop's conversion stream");
        if (!rc && p->bf_stream) {
            std::vector<psvi::EpsPlanes> one(1, p->eps_planes);
            rc = upload(one, &p->d_eps_planes);
        }
        if (!rc && family == PSVI_FAMILY_LENET) {
            const size_t bytes = lenet_ws(*p, nullptr).bytes;
            if (hipMalloc(&p->d_lenet_ws, bytes) != hipSuccess)
                rc = fail(PSVI_EUNSUP, "cannot allocate the LeNet activation scratch");
        }
        p->on_device = rc == 0;
    }
    if (rc) {
        psvi_plan_destroy(p);
        return rc;
    }
    *out = p;
    return 0;
}

int psvi_plan_destroy(psvi_plan* p) {
    if (!p) return 0;
    if (p->d_fwd) (void)hipFree(p->d_fwd);
    if (p->d_frb) (void)hipFree(p->d_frb);
    if (p->d_fwd_part) (void)hipFree(p->d_fwd_part);
    if (p->d_ufrb) (void)hipFree(p->d_ufrb);
    if (p->d_str) (void)hipFree(p->d_str);
    if (p->d_sfrb) (void)hipFree(p->d_sfrb);
    if (p->d_str_part) (void)hipFree(p->d_str_part);
    if (p->d_str_cnt) (void)hipFree(p->d_str_cnt);
    if (p->d_str_bms) (void)hipFree(p->d_str_bms);
    if (p->d_upd_part) (void)hipFree(p->d_upd_part);
    if (p->d_upd) (void)hipFree(p->d_upd);
    if (p->d_lenet_ws) (void)hipFree(p->d_lenet_ws);
    if (p->d_mf_slots) (void)hipFree(p->d_mf_slots);
    if (p->d_net_slots) (void)hipFree(p->d_net_slots);
    if (p->d_net_xmap) (void)hipFree(p->d_net_xmap);
    if (p->d_ks_tiles) (void)hipFree(p->d_ks_tiles);
    if (p->d_ks_segs) (void)hipFree(p->d_ks_segs);
    if (p->d_ks_off) (void)hipFree(p->d_ks_off);
    if (p->d_ks_slots) (void)hipFree(p->d_ks_slots);
    if (p->d_ks_cnt) (void)hipFree(p->d_ks_cnt);
    if (p->d_fs_segs) (void)hipFree(p->d_fs_segs);
    if (p->d_fs_off) (void)hipFree(p->d_fs_off);
    if (p->d_fs_rb) (void)hipFree(p->d_fs_rb);
    if (p->d_fp_segs) (void)hipFree(p->d_fp_segs);
    if (p->d_fp_off) (void)hipFree(p->d_fp_off);
    if (p->d_fp_rb) (void)hipFree(p->d_fp_rb);
    if (p->d_fs_part) (void)hipFree(p->d_fs_part);
    if (p->d_net_bands) (void)hipFree(p->d_net_bands);
    if (p->d_eps_planes) (void)hipFree(p->d_eps_planes);
    if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
    if (p->ev_join) (void)hipEventDestroy(p->ev_join);
    if (p->aux_st) (void)hipStreamDestroy(p->aux_st);
    delete p;
    return 0;
}

static size_t loop_ws_bytes(const psvi_plan* p);
static size_t tiled_floats(const psvi_plan* p);

// psvi_outer_elbo_grad workspace: the step workspace (x / g or acc), then the
// per-row NLL [S][M], row coefficients [S][2], ck [S], sum ck, per-sample
// stats [S][2] doubles, and the per-sample input gradients [S][M][D]
struct OuterWs {
    float *nll, *rowcoef, *ck, *sck, *du;
    double* stats;
    size_t bytes;
};
static OuterWs outer_ws(const psvi_plan* p, void* ws);

// psvi_hvp workspace: the step workspace (x), x_dot [S][n_tot], G and G_dot
// [splits][S][n_tot], d_u parts [S][M][D], NLL_dot [S][M]
struct HvpWs {
    float *xd, *G, *Gd, *du, *nlld;
    float* part2;  // full-cov: split-K slots of the tangent sample (pair launch)
    size_t bytes;
};
static HvpWs hvp_ws(const psvi_plan* p, void* ws) {
    const size_t S = p->d.S, M = p->d.M, D = p->lay[0].din, nt = p->n_tot;
    char* b = (char*)ws;
    HvpWs o{};
    if (p->family == PSVI_FAMILY_LENET) {  // tangent scratch of launch_lenet_hvp
        o.bytes = lenet_tan_ws(*p, nullptr).bytes;
        return o;
    }
    size_t off = align256(p->ws_bytes);
    auto take = [&](size_t bytes) {
        char* r = b ? b + off : nullptr;
        off += align256(bytes);
        return r;
    };
    o.xd = (float*)take(sizeof(float) * S * nt);
    const size_t ns = rop_splits(*p);  // the R-op's row-block slots (summed into slot 0)
    o.G = (float*)take(sizeof(float) * ns * S * nt);
    o.Gd = (float*)take(sizeof(float) * ns * S * nt);
    o.du = (float*)take(sizeof(float) * S * M * D);
    o.nlld = (float*)take(sizeof(float) * S * M);
    if (p->family == PSVI_FAMILY_FULLCOV)
        o.part2 = (float*)take(sizeof(float) *
                               std::max({(size_t)p->n_fwd * S, (size_t)p->n_fp_slots * kKsPass,
                                         (size_t)p->n_fs_slots * kKsPass}) *
                               kFwdRows);  // item-grid or either segment table's slots
    o.bytes = off;
    return o;
}

static OuterWs outer_ws(const psvi_plan* p, void* ws);

// psvi_evaluate workspace: the outer workspace, then the data rows' softmax
// [S][M][C] (bounded by M rows) and the sample weights [S]
static size_t eval_prob_off(const psvi_plan* p);
static size_t eval_ws_bytes(const psvi_plan* p) {
    const size_t S = p->d.S, M = p->d.M, C = p->lay[p->L - 1].dout;
    return eval_prob_off(p) + align256(sizeof(float) * S * M * C) + align256(sizeof(float) * S);
}

static OuterWs outer_ws(const psvi_plan* p, void* ws) {
    const size_t S = p->d.S, M = p->d.M, D = plan_in_dim(*p);
    char* b = (char*)ws;
    OuterWs o{};
    size_t off = align256(p->ws_bytes);
    auto take = [&](size_t bytes) {
        char* r = b ? b + off : nullptr;
        off += align256(bytes);
        return r;
    };
    o.nll = (float*)take(sizeof(float) * S * M);
    o.rowcoef = (float*)take(sizeof(float) * 2 * S);
    o.ck = (float*)take(sizeof(float) * S);
    o.sck = (float*)take(sizeof(float));
    o.stats = (double*)take(sizeof(double) * 2 * S);
    o.du = (float*)take(sizeof(float) * S * M * D);
    o.bytes = off;
    return o;
}

int psvi_plan_query(const psvi_plan* p, int32_t key, int64_t* value) {
    if (!p || !value) return fail(PSVI_EINVAL, "null argument");
    const int r = p->rank;
    switch (key) {
        case PSVI_Q_PARAM_COUNT: *value = p->P; break;
        case PSVI_Q_EPS_COUNT: *value = p->Peps; break;
        case PSVI_Q_WS_BYTES: *value = (int64_t)p->ws_bytes; break;
        case PSVI_Q_S_LOCAL: *value = p->s_cnt[r]; break;
        case PSVI_Q_S_OFFSET: *value = p->s_off[r]; break;
        case PSVI_Q_ACC_COUNT: *value = p->acc_count; break;
        case PSVI_Q_ROWS_LOCAL: *value = p->rows_tot[r]; break;
        case PSVI_Q_XSHARD_COUNT: *value = (int64_t)p->d.S * p->rows_tot[r]; break;
        case PSVI_Q_LOOP_WS_BYTES: *value = (int64_t)loop_ws_bytes(p); break;
        case PSVI_Q_TILED_FLOATS: *value = (int64_t)tiled_floats(p); break;
        case PSVI_Q_XRECV_COUNT: *value = (int64_t)p->s_cnt[r] * p->n_tot; break;
        case PSVI_Q_OUTER_WS_BYTES: *value = (int64_t)outer_ws(p, nullptr).bytes; break;
        case PSVI_Q_HVP_WS_BYTES: *value = (int64_t)hvp_ws(p, nullptr).bytes; break;
        case PSVI_Q_EVAL_WS_BYTES: *value = (int64_t)eval_ws_bytes(p); break;
        case PSVI_Q_NET_PART_OK:
            *value = p->family == PSVI_FAMILY_FULLCOV && !(p->mchunks > 1 && !p->net_mloop);
            break;
        default: return fail(PSVI_EINVAL, "unknown query key");
    }
    return 0;
}

int psvi_plan_shard_info(const psvi_plan* p, int32_t r, int64_t* out) {
    if (!p || !out) return fail(PSVI_EINVAL, "null argument");
    if (r < 0 || r >= p->world) return fail(PSVI_EINVAL, "rank out of range");
    out[0] = p->s_off[r];
    out[1] = p->s_cnt[r];
    out[2] = p->rows_tot[r];
    for (int l = 0; l < PSVI_MAX_LAYERS; ++l) {
        int cnt = 0, nrun = 0, lo = 0;
        for (const ShardRun& run : p->runs[r])
            if (run.layer == l) {
                if (nrun++ == 0) lo = run.lo;
                cnt += run.hi - run.lo;
            }
        // the first row when the rank's rows of layer l are one run (or none),
        // -1 when they are several (psvi_plan_shard_runs lists them)
        out[3 + l] = nrun <= 1 ? lo : -1;
        out[3 + PSVI_MAX_LAYERS + l] = cnt;
    }
    return 0;
}

int psvi_plan_shard_runs(const psvi_plan* p, int32_t r, int64_t* out, int32_t cap,
                         int32_t* count) {
    if (!p || !count) return fail(PSVI_EINVAL, "null argument");
    if (r < 0 || r >= p->world) return fail(PSVI_EINVAL, "rank out of range");
    const int n = (int)p->runs[r].size();
    *count = n;
    if (!out) return 0;
    if (cap < n) return fail(PSVI_ENOSPC, "run buffer too small");
    for (int i = 0; i < n; ++i) {
        const ShardRun& run = p->runs[r][i];
        out[4 * i] = run.layer;
        out[4 * i + 1] = run.lo;
        out[4 * i + 2] = run.hi - run.lo;
        out[4 * i + 3] = run.col;
    }
    return 0;
}

// Every entry point that runs on a plan, except the loop that takes it up,
// drops the resident state of a PSVI_LOOP_KEEP call: it may have written the
// workspace, the parameters or the Adam state the state stands for.
static void drop_resident(const psvi_plan* p) {
    if (p) p->resident.valid = false;
}

static int check_step(const psvi_plan* p, const void* u, const void* z, const void* w,
                      const void* eps, size_t ws_bytes, const void* ws) {
    if (!p) return fail(PSVI_EINVAL, "null plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (p->world != 1) return fail(PSVI_ESTATE, "fused step needs world == 1 (use phases)");
    if (!u || !z || !w || !eps) return fail(PSVI_EINVAL, "null input pointer");
    if (!ws || ws_bytes < p->ws_bytes) return fail(PSVI_ENOSPC, "workspace too small");
    return 0;
}

static int step_impl(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                     const float* eps, float* params, float* m, float* v,
                     const psvi_adam_hp* hp, double* elbo_out, float* grad_out,
                     int include_kl, void* ws, hipStream_t st) {
    HIP_TRY(hipMemsetAsync(elbo_out, 0, sizeof(double), st));
    char* wsb = (char*)ws;
    if (p->family == PSVI_FAMILY_LENET) {
        float* acc = (float*)wsb;
        HIP_TRY(launch_lenet(*p, u, z, w, params, eps, acc, elbo_out, p->d_lenet_ws, st));
        HIP_TRY(launch_mf_update(*p, acc, params, m, v, hp, elbo_out, grad_out, include_kl, st));
    } else if (p->family == PSVI_FAMILY_MEANFIELD) {
        // per-(sample, chunk) gradient slots, summed in a fixed order by the update
        HIP_TRY(launch_net(*p, u, z, w, params, eps, p->d_mf_slots, nullptr, nullptr, elbo_out,
                           st));
        HIP_TRY(launch_mf_update(*p, nullptr, params, m, v, hp, elbo_out, grad_out, include_kl,
                                 st, eps));
    } else {
        const size_t xs = sizeof(float) * (size_t)p->d.S * p->rows_tot[0];
        float* x = (float*)wsb;
        float* g = (float*)(wsb + align256(xs));
        HIP_TRY(launch_mvn_fwd(*p, eps, params, x, st));
        HIP_TRY(launch_net(*p, u, z, w, nullptr, nullptr, nullptr, x, g, elbo_out, st));
        HIP_TRY(launch_mvn_update(*p, eps, g, params, m, v, hp, elbo_out, grad_out, include_kl,
                                  nullptr, nullptr, st));
    }
    return 0;
}

int psvi_inner_step(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                    const float* eps, float* params, float* adam_m, float* adam_v,
                    const psvi_adam_hp* hp, double* elbo_out, void* ws, size_t ws_bytes,
                    void* stream) {
    drop_resident(p);
    if (int rc = check_step(p, u, z, w, eps, ws_bytes, ws)) return rc;
    if (!params || !adam_m || !adam_v || !hp || !elbo_out)
        return fail(PSVI_EINVAL, "null state pointer");
    if (hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (hp->kind < 0 || hp->kind > 2) return fail(PSVI_EINVAL, "unknown adam kind");
    return step_impl(p, u, z, w, eps, params, adam_m, adam_v, hp, elbo_out, nullptr, 1, ws,
                     as_stream(stream));
}

int psvi_elbo_grad(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                   const float* eps, const float* params, int32_t include_kl, double* elbo_out,
                   float* grad_out, void* ws, size_t ws_bytes, void* stream) {
    drop_resident(p);
    if (int rc = check_step(p, u, z, w, eps, ws_bytes, ws)) return rc;
    if (!params || !elbo_out || !grad_out) return fail(PSVI_EINVAL, "null pointer");
    return step_impl(p, u, z, w, eps, const_cast<float*>(params), nullptr, nullptr, nullptr,
                     elbo_out, grad_out, include_kl ? 1 : 0, ws, as_stream(stream));
}

int psvi_mf_phase_accumulate(const psvi_plan* p, const float* u, const int32_t* z,
                             const float* w, const float* eps, const float* params, float* acc,
                             double* nll_out, void* stream) {
    drop_resident(p);
    if (!p || p->family == PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a mean-field plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (!u || !z || !w || !eps || !params || !acc || !nll_out)
        return fail(PSVI_EINVAL, "null pointer");
    hipStream_t st = as_stream(stream);
    if (p->family == PSVI_FAMILY_LENET) {
        HIP_TRY(launch_lenet(*p, u, z, w, params, eps, acc, nll_out, p->d_lenet_ws, st));
        return 0;
    }
    HIP_TRY(launch_net(*p, u, z, w, params, eps, p->d_mf_slots, nullptr, nullptr, nll_out, st));
    HIP_TRY(launch_mf_slot_acc(*p, eps, acc, st));
    return 0;
}

int psvi_mf_phase_update(const psvi_plan* p, const float* acc, float* params, float* adam_m,
                         float* adam_v, const psvi_adam_hp* hp, double* kl_out,
                         float* grad_out, int32_t include_kl, void* stream) {
    drop_resident(p);
    if (!p || p->family == PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a mean-field plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (!acc || !params) return fail(PSVI_EINVAL, "null pointer");
    if (!grad_out && (!adam_m || !adam_v || !hp)) return fail(PSVI_EINVAL, "null adam state");
    if (!grad_out && hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (!grad_out && (hp->kind < 0 || hp->kind > 2)) return fail(PSVI_EINVAL, "unknown adam kind");
    HIP_TRY(launch_mf_update(*p, acc, params, adam_m, adam_v, hp, kl_out, grad_out,
                             include_kl ? 1 : 0, as_stream(stream)));
    return 0;
}

int psvi_mvn_phase_sample(const psvi_plan* p, const float* eps, const float* params,
                          float* x_shard, void* stream) {
    drop_resident(p);
    if (!p || p->family != PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a full-cov plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    // a rank that owns no rows (fewer bands than ranks) has an empty x shard
    if (!eps || !params || (!x_shard && p->rows_tot[p->rank] > 0))
        return fail(PSVI_EINVAL, "null pointer");
    HIP_TRY(launch_mvn_fwd(*p, eps, params, x_shard, as_stream(stream)));
    return 0;
}

int psvi_mvn_phase_net(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                       const float* x_recv, float* g_send, double* nll_out, void* stream) {
    drop_resident(p);
    if (!p || p->family != PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a full-cov plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    // a rank without samples (S < world) has empty x / g blocks
    const bool none = p->s_cnt[p->rank] == 0;
    if (!u || !z || !w || (!none && (!x_recv || !g_send)) || !nll_out)
        return fail(PSVI_EINVAL, "null pointer");
    hipStream_t st = as_stream(stream);
    HIP_TRY(launch_net(*p, u, z, w, nullptr, nullptr, nullptr, x_recv, g_send, nll_out, st));
    return 0;
}

int psvi_mvn_phase_net_draw(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                            const float* x_recv, float* g_send, double* nll_out, float* eps_out,
                            int64_t n, uint64_t seed, uint64_t offset, void* stream) {
    drop_resident(p);
    if (!p || p->family != PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a full-cov plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    const bool none = p->s_cnt[p->rank] == 0;  // S < world: empty x / g blocks
    if (!u || !z || !w || (!none && (!x_recv || !g_send)) || !nll_out || !eps_out || n < 0)
        return fail(PSVI_EINVAL, "null pointer or bad count");
    if (offset % 4) return fail(PSVI_EINVAL, "randn offset must be a multiple of 4");
    if (reinterpret_cast<uintptr_t>(eps_out) % 16)
        return fail(PSVI_EINVAL, "eps_out must be 16-byte aligned");
    hipStream_t st = as_stream(stream);
    HIP_TRY(launch_net(*p, u, z, w, nullptr, nullptr, nullptr, x_recv, g_send, nll_out, st, eps_out, n,
                       seed, offset));
    return 0;
}

int psvi_mvn_phase_net_part(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                            const float* x_recv, float* g_send, double* nll_out, int32_t s_begin,
                            int32_t s_count, float* eps_out, int64_t n, uint64_t seed,
                            uint64_t offset, int32_t part, int32_t nparts, void* stream) {
    drop_resident(p);
    if (!p || p->family != PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a full-cov plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    const int S_loc = p->s_cnt[p->rank];
    if (s_begin < 0 || s_count < 0 || s_begin + s_count > S_loc)
        return fail(PSVI_EINVAL, "sample range outside the rank's samples");
    if (nparts < 1 || part < 0 || part >= nparts) return fail(PSVI_EINVAL, "bad draw part");
    if (!u || !z || !w || (s_count > 0 && (!x_recv || !g_send)) || !nll_out || n < 0 ||
        (n > 0 && !eps_out))
        return fail(PSVI_EINVAL, "null pointer or bad count");
    if (offset % 4) return fail(PSVI_EINVAL, "randn offset must be a multiple of 4");
    if (eps_out && reinterpret_cast<uintptr_t>(eps_out) % 16)
        return fail(PSVI_EINVAL, "eps_out must be 16-byte aligned");
    if (p->mchunks > 1 && !p->net_mloop && (s_begin != 0 || s_count != S_loc))
        return fail(PSVI_EUNSUP, "per-chunk gradient slots: whole sample launches only");
    hipStream_t st = as_stream(stream);
    HIP_TRY(launch_net(*p, u, z, w, nullptr, nullptr, nullptr, x_recv, g_send, nll_out, st,
                       n > 0 ? eps_out : nullptr, n, seed, offset, nullptr, nullptr, s_begin, s_count,
                       part, nparts));
    return 0;
}

int psvi_mvn_phase_update(const psvi_plan* p, const float* eps, const float* g_shard,
                          float* params, float* adam_m, float* adam_v, const psvi_adam_hp* hp,
                          double* kl_out, float* grad_out, int32_t include_kl, void* stream) {
    drop_resident(p);
    if (!p || p->family != PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a full-cov plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (!eps || (!g_shard && p->rows_tot[p->rank] > 0) || !params)
        return fail(PSVI_EINVAL, "null pointer");
    if (!grad_out && (!adam_m || !adam_v || !hp)) return fail(PSVI_EINVAL, "null adam state");
    if (!grad_out && hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (!grad_out && (hp->kind < 0 || hp->kind > 2)) return fail(PSVI_EINVAL, "unknown adam kind");
    HIP_TRY(launch_mvn_update(*p, eps, g_shard, params, adam_m, adam_v, hp, kl_out, grad_out,
                              include_kl ? 1 : 0, nullptr, nullptr, as_stream(stream)));
    return 0;
}

int psvi_mvn_phase_update_sample(const psvi_plan* p, const float* eps, const float* g_shard,
                                 float* params, float* adam_m, float* adam_v,
                                 const psvi_adam_hp* hp, double* kl_out, int32_t include_kl,
                                 const float* eps_next, float* x_next, void* stream) {
    drop_resident(p);
    if (!p || p->family != PSVI_FAMILY_FULLCOV) return fail(PSVI_ESTATE, "not a full-cov plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    const bool rows = p->rows_tot[p->rank] > 0;  // no rows: empty G and x shards
    if (!eps || !params || !eps_next || (rows && (!g_shard || !x_next)))
        return fail(PSVI_EINVAL, "null pointer");
    if (!adam_m || !adam_v || !hp) return fail(PSVI_EINVAL, "null adam state");
    if (hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (hp->kind < 0 || hp->kind > 2) return fail(PSVI_EINVAL, "unknown adam kind");
    HIP_TRY(launch_mvn_update(*p, eps, g_shard, params, adam_m, adam_v, hp, kl_out, nullptr,
                              include_kl ? 1 : 0, eps_next, x_next, as_stream(stream)));
    return 0;
}

static int64_t eps_stride(const psvi_plan* p) { return (p->Peps + 3) / 4 * 4; }

// tiled corr/m/v state: full-cov, world 1, one LDS pass of samples.  The
// write-through (sc1) stores of the stream kernel and the chunked kernel's
// tiled epilogue address all three arrays through ONE buffer descriptor
// (num_records 0x7fffffff, m / v at 32-bit byte offsets), so the whole state
// must stay below 2^31 bytes; larger plans keep corr / m / v packed (the
// chunked kernel with plain stores) instead of overflowing those offsets.
static bool tiled_ok(const psvi_plan* p) {
    return p->family == PSVI_FAMILY_FULLCOV && p->fuse_sample && p->tiles_total > 0 &&
           3 * p->tiles_total * 4096 * (int64_t)sizeof(float) < 0x7fffffff - 16;
}
static size_t tiled_floats(const psvi_plan* p) {
    return tiled_ok(p) ? 3 * (size_t)p->tiles_total * 4096 : 0;
}

// psvi_inner_loop workspace: the step workspace (x, g, a 256-byte tail), two
// eps buffers each followed by 64 floats of zeros (the streaming update's
// loads past a layer's last column block land there, unclamped), the tiled
// state
static size_t loop_ebuf_bytes(const psvi_plan* p) {
    return align256(sizeof(float) * ((size_t)eps_stride(p) + 64));
}
// the bf16 planes of one draw (three planes of EpsPlanes::pl elements)
static size_t loop_pbuf_bytes(const psvi_plan* p) {
    return p->bf_stream ? align256(3 * sizeof(uint16_t) * (size_t)p->eps_planes.pl) : 0;
}
static size_t loop_ws_bytes(const psvi_plan* p) {
    return align256(p->ws_bytes) + 2 * loop_ebuf_bytes(p) + align256(sizeof(float) * tiled_floats(p)) +
           2 * loop_pbuf_bytes(p);
}

int psvi_mvn_tiled_convert(const psvi_plan* p, float* params, float* adam_m, float* adam_v,
                           float* tstate, int32_t to_tiled, void* stream) {
    drop_resident(p);
    if (!p || !tiled_ok(p)) return fail(PSVI_EUNSUP, "plan has no tiled state (full-cov, world 1, S <= 128)");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (!params || !adam_m || !adam_v || !tstate) return fail(PSVI_EINVAL, "null pointer");
    HIP_TRY(launch_mvn_tile_convert(*p, params, adam_m, adam_v, tstate, to_tiled != 0,
                                    as_stream(stream)));
    return 0;
}

int psvi_mvn_phase_update_tiled(const psvi_plan* p, const float* eps, const float* g_shard,
                                float* params, float* adam_m, float* adam_v, float* tstate,
                                const psvi_adam_hp* hp, double* kl_out, int32_t include_kl,
                                const float* eps_next, float* x_next, void* stream) {
    drop_resident(p);
    if (!p || !tiled_ok(p)) return fail(PSVI_EUNSUP, "plan has no tiled state (full-cov, world 1, S <= 128)");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (!eps || !g_shard || !params || !adam_m || !adam_v || !tstate || !hp)
        return fail(PSVI_EINVAL, "null pointer");
    if (!eps_next != !x_next) return fail(PSVI_EINVAL, "eps_next and x_next go together");
    if (hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (hp->kind < 0 || hp->kind > 2) return fail(PSVI_EINVAL, "unknown adam kind");
    HIP_TRY(launch_mvn_update(*p, eps, g_shard, params, adam_m, adam_v, hp, kl_out, nullptr,
                              include_kl ? 1 : 0, eps_next, x_next, as_stream(stream), tstate));
    return 0;
}

int psvi_inner_loop(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                    const float* eps, uint64_t seed, uint64_t offset, int32_t T, float* params,
                    float* adam_m, float* adam_v, const psvi_adam_hp* hp, double* elbo_out,
                    void* ws, size_t ws_bytes, void* stream) {
    return psvi_inner_loop_ex(p, u, z, w, eps, seed, offset, T, params, adam_m, adam_v, hp,
                              elbo_out, ws, ws_bytes, 0, stream);
}

int psvi_inner_loop_ex(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                       const float* eps, uint64_t seed, uint64_t offset, int32_t T, float* params,
                       float* adam_m, float* adam_v, const psvi_adam_hp* hp, double* elbo_out,
                       void* ws, size_t ws_bytes, int32_t flags, void* stream) {
    if (!p) return fail(PSVI_EINVAL, "null plan");
    if (flags & ~(PSVI_LOOP_KEEP | PSVI_LOOP_RESUME)) return fail(PSVI_EINVAL, "unknown loop flags");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (p->world != 1) return fail(PSVI_ESTATE, "inner loop needs world == 1 (use phases)");
    if (!u || !z || !w || !params || !adam_m || !adam_v || !hp || !elbo_out)
        return fail(PSVI_EINVAL, "null pointer");
    if (T < 0) return fail(PSVI_EINVAL, "T must be >= 0");
    if (hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (hp->kind < 0 || hp->kind > 2) return fail(PSVI_EINVAL, "unknown adam kind");
    if (!eps && offset % 4) return fail(PSVI_EINVAL, "randn offset must be a multiple of 4");
    if (!ws || ws_bytes < loop_ws_bytes(p)) return fail(PSVI_ENOSPC, "workspace too small");
    hipStream_t st = as_stream(stream);
    char* wsb = (char*)ws;
    const int64_t es = eps_stride(p);
    float* ebuf[2] = {(float*)(wsb + align256(p->ws_bytes)),
                      (float*)(wsb + align256(p->ws_bytes) + loop_ebuf_bytes(p))};
    // eps of step t: the caller's [T][EPS_COUNT] array, or Philox (seed, offset + t * stride)
    auto eps_t = [&](int t) -> const float* {
        if (eps) return eps + (size_t)t * p->Peps;
        float* b = ebuf[t & 1];
        return launch_randn(b, p->Peps, seed, offset + (uint64_t)t * es, st) == hipSuccess ? b
                                                                                         : nullptr;
    };
    // eps of step 0 with the ELBO accumulators cleared: Philox mode folds the
    // clear into the draw's launch
    auto first_eps = [&]() -> const float* {
        if (eps) {
            return hipMemsetAsync(elbo_out, 0, sizeof(double) * (size_t)T, st) == hipSuccess
                       ? eps
                       : nullptr;
        }
        return launch_randn(ebuf[0], p->Peps, seed, offset, st, elbo_out, T) == hipSuccess
                   ? ebuf[0]
                   : nullptr;
    };
    psvi_adam_hp h = *hp;
    if (p->family == PSVI_FAMILY_MEANFIELD) {
        // two launches per step: the network kernel (which also draws the next
        // step's eps in Philox mode) and the slot-reducing update; the ELBO
        // accumulators are cleared once for the whole loop
        if (T == 0) return 0;
        const float* e = first_eps();
        if (!e) return fail(PSVI_EUNSUP, "randn launch failed");
        for (int t = 0; t < T; ++t) {
            h.step = hp->step + t;
            const bool draw = !eps && t + 1 < T;
            float* en_buf = draw ? ebuf[(t + 1) & 1] : nullptr;
            HIP_TRY(launch_net(*p, u, z, w, params, e, p->d_mf_slots, nullptr, nullptr,
                               elbo_out + t, st, en_buf, draw ? p->Peps : 0, seed,
                               offset + (uint64_t)(t + 1) * es));
            HIP_TRY(launch_mf_update(*p, nullptr, params, adam_m, adam_v, &h, elbo_out + t,
                                     nullptr, 1, st, e));
            e = t + 1 < T ? (eps ? eps + (size_t)(t + 1) * p->Peps : en_buf) : nullptr;
        }
        return 0;
    }
    if (p->family != PSVI_FAMILY_FULLCOV) {
        for (int t = 0; t < T; ++t) {
            const float* e = eps_t(t);
            if (!e) return fail(PSVI_EUNSUP, "randn launch failed");
            h.step = hp->step + t;
            if (int rc = step_impl(p, u, z, w, e, params, adam_m, adam_v, &h, elbo_out + t,
                                   nullptr, 1, ws, st))
                return rc;
        }
        return 0;
    }
    // full-cov: sample x_0, then per step net + update, the update also sampling
    // the next step's x from the updated parameters (fused where the plan allows)
    const size_t xs = sizeof(float) * (size_t)p->d.S * p->rows_tot[0];
    float* x = (float*)wsb;
    float* g = (float*)(wsb + align256(xs));
    // corr / m / v live in the tiled layout for the whole loop when the plan allows
    float* ts = tiled_ok(p) ? (float*)(wsb + align256(p->ws_bytes) + 2 * loop_ebuf_bytes(p))
                            : nullptr;
    // Philox mode: eps, eps' and G are the loop's own buffers -- their 64-float
    // pads are zeroed with the tiled conversion and the streaming update reads
    // them unclamped
    const bool padded = ts && !eps;
    // Philox mode on a bf-stream plan: every draw also as bf16 planes, one
    // plane buffer per eps buffer (their row pads zeroed here, never drawn)
    uint16_t* pbuf[2] = {nullptr, nullptr};
    if (padded && p->bf_stream) {
        char* pb = wsb + align256(p->ws_bytes) + 2 * loop_ebuf_bytes(p) +
                   align256(sizeof(float) * tiled_floats(p));
        pbuf[0] = (uint16_t*)pb;
        pbuf[1] = (uint16_t*)(pb + loop_pbuf_bytes(p));
    }
    float* pads[3] = {padded ? ebuf[0] + p->Peps : nullptr, padded ? ebuf[1] + p->Peps : nullptr,
                      padded ? g + (size_t)p->d.S * p->rows_tot[0] : nullptr};
    if (T == 0) return 0;
    // resident state of the last KEEP call (dropped by every call; taken up by
    // a RESUME call that continues it)
    const psvi_plan::Resident res = p->resident;
    p->resident.valid = false;
    const bool keep = (flags & PSVI_LOOP_KEEP) && padded;
    const bool resume = (flags & PSVI_LOOP_RESUME) && padded && res.valid && res.ws == ws &&
                        res.params == params && res.m == adam_m && res.v == adam_v &&
                        res.seed == seed && res.offset == offset;
    // eps buffer of step t (a resumed loop's step 0 is where the last one left it)
    const int eb0 = resume ? res.ebuf : 0;
    auto bi = [&](int t) { return (t + eb0) & 1; };
    bool join = false;
    const float* e;
    if (resume) {
        // the tiled state, step 0's eps (+ planes) and x are in ws already; the
        // ELBO accumulators cleared by the draw kernel's zero-fill with no draw
        // (a library kernel: hipMemsetAsync's first use in a process loads the
        // runtime's own fill kernels inside the caller's timed region)
        HIP_TRY(launch_randn(ebuf[1 - bi(0)], 0, 0, 0, st, elbo_out, T));
        e = ebuf[bi(0)];
    } else {
        // packed -> tiled state on the plan's conversion stream, behind x_0 and the
        // first network step (joined before the first update)
        if (ts && p->aux_st) {
            HIP_TRY(hipEventRecord(p->ev_fork, st));
            HIP_TRY(hipStreamWaitEvent(p->aux_st, p->ev_fork, 0));
            HIP_TRY(launch_mvn_tile_convert(*p, params, adam_m, adam_v, ts, true, p->aux_st, pads));
            HIP_TRY(hipEventRecord(p->ev_join, p->aux_st));
            join = true;
        } else if (ts) {
            HIP_TRY(launch_mvn_tile_convert(*p, params, adam_m, adam_v, ts, true, st, pads));
        }
        if (pbuf[0]) {
            HIP_TRY(hipMemsetAsync(pbuf[0], 0, 2 * loop_pbuf_bytes(p), st));
            HIP_TRY(launch_randn(ebuf[0], p->Peps, seed, offset, st, elbo_out, T, &p->eps_planes, pbuf[0]));
            e = ebuf[0];
        } else {
            e = first_eps();
        }
        if (!e) return fail(PSVI_EUNSUP, "randn launch failed");
        HIP_TRY(launch_mvn_fwd(*p, e, params, x, st));
    }
    for (int t = 0; t < T; ++t) {
        h.step = hp->step + t;
        // Philox mode: the network kernel also draws the next step's eps (KEEP:
        // the last step too, for the next call)
        const bool last = t + 1 == T;
        const bool draw = !eps && (!last || keep);
        float* en_buf = draw ? ebuf[bi(t + 1)] : nullptr;
        uint16_t* en_pl = draw ? pbuf[bi(t + 1)] : nullptr;
        const bool tm = g_loop_every > 0 && t % g_loop_every == 0;
        if (tm) HIP_TRY(loop_event(0, st));
        HIP_TRY(launch_net(*p, u, z, w, nullptr, nullptr, nullptr, x, g, elbo_out + t,
                           st, en_buf, draw ? p->Peps : 0, seed, offset + (uint64_t)(t + 1) * es,
                           nullptr, en_pl));
        if (tm) HIP_TRY(loop_event(0, st));
        const float* en = !last ? (eps ? eps + (size_t)(t + 1) * p->Peps : en_buf) : (keep ? en_buf : nullptr);
        if (tm) HIP_TRY(loop_event(1, st));
        if (join) {
            HIP_TRY(hipStreamWaitEvent(st, p->ev_join, 0));
            join = false;
        }
        // the last step (no next sample) writes corr / m / v back to the packed
        // arrays; KEEP: it samples as every step, then the tiled state is copied out
        HIP_TRY(launch_mvn_update(*p, e, g, params, adam_m, adam_v, &h, elbo_out + t, nullptr, 1,
                                  en, en ? x : nullptr, st, ts, ts && !en, nullptr, padded,
                                  pbuf[bi(t)], en ? en_pl : nullptr));
        if (tm) HIP_TRY(loop_event(1, st));
        e = en;
    }
    if (keep) {
        HIP_TRY(launch_mvn_tile_convert(*p, params, adam_m, adam_v, ts, false, st, nullptr));
        p->resident = psvi_plan::Resident{true, ws, params, adam_m, adam_v, seed,
                                          offset + (uint64_t)T * es, bi(T)};
    }
    return 0;
}

// ext_coef == nullptr: the whole objective (stats, forward, combine, backward).
// Otherwise [rowcoef (S x 2) | ck (S) | sck (1)] replace the combine: the
// backward of a caller-formed softmax over samples (sample-sharded outer).
static int outer_impl(const psvi_plan* p, int32_t n_pseudo, const float* x_all,
                      const int32_t* z_all, const float* w_all, const float* eps,
                      const float* params, double* loss_out, float* grad_params,
                      float* grad_u, float* grad_w, double* sample_out,
                      const float* ext_coef, void* ws, size_t ws_bytes, void* stream,
                      int ablated = 0) {
    drop_resident(p);
    if (!p) return fail(PSVI_EINVAL, "null plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (p->world != 1) return fail(PSVI_ESTATE, "the outer objective needs world == 1");
    if (p->d.S < 1) return fail(PSVI_EINVAL, "S must be >= 1");
    if (p->d.S > 2048) return fail(PSVI_EUNSUP, "the outer objective supports S <= 2048");
    if (n_pseudo < 0 || n_pseudo > p->d.M) return fail(PSVI_EINVAL, "n_pseudo out of [0, M]");
    if (!x_all || !z_all || !w_all || !eps || !params || (!loss_out && !ext_coef))
        return fail(PSVI_EINVAL, "null pointer");
    if (grad_u && !grad_params)
        return fail(PSVI_EINVAL, "grad_u needs grad_params (one backward pass gives both)");
    const OuterWs o = outer_ws(p, ws);
    if (!ws || ws_bytes < o.bytes) return fail(PSVI_ENOSPC, "workspace too small");
    hipStream_t st = as_stream(stream);
    char* wsb = (char*)ws;
    float* x = nullptr;
    float* g = nullptr;
    float* acc = nullptr;
    if (p->family == PSVI_FAMILY_FULLCOV) {
        const size_t xs = sizeof(float) * (size_t)p->d.S * p->rows_tot[0];
        x = (float*)wsb;
        g = (float*)(wsb + align256(xs));
        HIP_TRY(launch_mvn_fwd(*p, eps, params, x, st));
    } else {
        acc = (float*)wsb;
    }
    if (!ext_coef) HIP_TRY(launch_outer_stats(*p, params, eps, x, o.stats, st));
    // 1. forward: every row's NLL
    NetOuter fw{1, n_pseudo, o.nll, nullptr, nullptr, nullptr};
    if (p->family == PSVI_FAMILY_LENET)
        HIP_TRY(launch_lenet(*p, x_all, z_all, w_all, params, eps, nullptr, nullptr,
                             p->d_lenet_ws, st, &fw));
    else
        HIP_TRY(launch_net(*p, x_all, z_all, w_all, params, eps, nullptr, x, nullptr, nullptr,
                           st, nullptr, 0, 0, 0, &fw));
    if (!ext_coef) {
        // 2. per-sample terms, softmax over samples, loss, backward coefficients
        HIP_TRY(launch_outer_combine(*p, n_pseudo, params, w_all, o.nll, o.stats, loss_out,
                                     o.rowcoef, o.ck, o.sck, grad_w, sample_out, ablated, st));
    } else {
        const size_t S = p->d.S;
        HIP_TRY(hipMemcpyAsync(o.rowcoef, ext_coef, sizeof(float) * 2 * S,
                               hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(o.ck, ext_coef + 2 * S, sizeof(float) * S,
                               hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(o.sck, ext_coef + 3 * S, sizeof(float), hipMemcpyDeviceToDevice,
                               st));
        if (grad_w) HIP_TRY(launch_outer_gradw(*p, n_pseudo, o.nll, o.rowcoef, grad_w, st));
    }
    if (!grad_params) return 0;
    // 3. backward through the network with the row coefficients (+ sampled-KL path)
    NetOuter bw{2, n_pseudo, nullptr, o.rowcoef, o.ck, grad_u ? o.du : nullptr};
    if (p->family == PSVI_FAMILY_FULLCOV) {
        HIP_TRY(launch_net(*p, x_all, z_all, w_all, nullptr, nullptr, nullptr, x, g, nullptr, st,
                           nullptr, 0, 0, 0, &bw));
        // 4. reparameterised backward (no KL term: the sampled KL came in through G)
        HIP_TRY(launch_mvn_update(*p, eps, g, const_cast<float*>(params), nullptr, nullptr,
                                  nullptr, nullptr, grad_params, 0, nullptr, nullptr, st));
    } else if (p->family == PSVI_FAMILY_LENET) {
        HIP_TRY(launch_lenet(*p, x_all, z_all, w_all, params, eps, acc, nullptr, p->d_lenet_ws,
                             st, &bw));
        HIP_TRY(launch_mf_update(*p, acc, const_cast<float*>(params), nullptr, nullptr, nullptr,
                                 nullptr, grad_params, 0, st));
    } else {
        HIP_TRY(launch_net(*p, x_all, z_all, w_all, params, eps, p->d_mf_slots, nullptr, nullptr,
                           nullptr, st, nullptr, 0, 0, 0, &bw));
        HIP_TRY(launch_mf_update(*p, nullptr, const_cast<float*>(params), nullptr, nullptr,
                                 nullptr, nullptr, grad_params, 0, st, eps));
    }
    // 5. explicit log-det term on the scales; d loss / d u
    HIP_TRY(launch_outer_finish(*p, n_pseudo, params, o.sck, grad_params, o.du, grad_u, st));
    return 0;
}

static size_t eval_prob_off(const psvi_plan* p) { return outer_ws(p, nullptr).bytes; }

int psvi_outer_elbo_grad(const psvi_plan* p, int32_t n_pseudo, const float* x_all,
                         const int32_t* z_all, const float* w_all, const float* eps,
                         const float* params, double* loss_out, float* grad_params,
                         float* grad_u, float* grad_w, double* sample_out, void* ws,
                         size_t ws_bytes, void* stream) {
    return outer_impl(p, n_pseudo, x_all, z_all, w_all, eps, params, loss_out, grad_params,
                      grad_u, grad_w, sample_out, nullptr, ws, ws_bytes, stream);
}

int psvi_outer_ablated_elbo_grad(const psvi_plan* p, const float* x_all,
                                 const int32_t* z_all, const float* w_all, const float* eps,
                                 const float* params, double* loss_out, float* grad_params,
                                 double* sample_out, void* ws, size_t ws_bytes, void* stream) {
    if (p && p->family == PSVI_FAMILY_FULLCOV)
        return fail(PSVI_EUNSUP, "PSVI_Ablated's sampled KL sums VILinear layers only; a "
                                 "full-covariance model has none (the reference fails there)");
    return outer_impl(p, 0, x_all, z_all, w_all, eps, params, loss_out, grad_params, nullptr,
                      nullptr, sample_out, nullptr, ws, ws_bytes, stream, 1);
}

int psvi_outer_elbo_grad_coef(const psvi_plan* p, int32_t n_pseudo, const float* x_all,
                              const int32_t* z_all, const float* w_all, const float* eps,
                              const float* params, const float* coef, float* grad_params,
                              float* grad_u, float* grad_w, void* ws, size_t ws_bytes,
                              void* stream) {
    if (!coef) return fail(PSVI_EINVAL, "null coefficients");
    return outer_impl(p, n_pseudo, x_all, z_all, w_all, eps, params, nullptr, grad_params,
                      grad_u, grad_w, nullptr, coef, ws, ws_bytes, stream);
}

int psvi_evaluate(const psvi_plan* p, int32_t n_pseudo, const float* x_all, const int32_t* z_all,
                  const float* w_all, const float* eps, const float* params, int32_t correction,
                  float* probs_out, double* stats_out, void* ws, size_t ws_bytes, void* stream) {
    drop_resident(p);
    if (!p) return fail(PSVI_EINVAL, "null plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (p->world != 1) return fail(PSVI_ESTATE, "evaluate needs world == 1");
    if (p->d.S < 2) return fail(PSVI_EINVAL, "evaluate needs S > 1 (psvi_classes.py:1036)");
    if (p->d.S > 2048) return fail(PSVI_EUNSUP, "evaluate supports S <= 2048");
    if (n_pseudo < 0 || n_pseudo > p->d.M) return fail(PSVI_EINVAL, "n_pseudo out of [0, M]");
    if (!x_all || !z_all || !w_all || !eps || !params || !stats_out)
        return fail(PSVI_EINVAL, "null pointer");
    if (!ws || ws_bytes < eval_ws_bytes(p)) return fail(PSVI_ENOSPC, "workspace too small");
    hipStream_t st = as_stream(stream);
    const OuterWs o = outer_ws(p, ws);
    char* wsb = (char*)ws;
    float* prob = (float*)(wsb + eval_prob_off(p));
    float* W = (float*)(wsb + eval_prob_off(p) +
                        align256(sizeof(float) * (size_t)p->d.S * p->d.M * p->lay[p->L - 1].dout));
    float* x = nullptr;
    if (p->family == PSVI_FAMILY_FULLCOV) {
        x = (float*)wsb;
        HIP_TRY(launch_mvn_fwd(*p, eps, params, x, st));
    }
    HIP_TRY(launch_outer_stats(*p, params, eps, x, o.stats, st));
    NetOuter fw{1, n_pseudo, o.nll, nullptr, nullptr, nullptr, prob};
    if (p->family == PSVI_FAMILY_LENET)
        HIP_TRY(launch_lenet(*p, x_all, z_all, w_all, params, eps, nullptr, nullptr,
                             p->d_lenet_ws, st, &fw));
    else
        HIP_TRY(launch_net(*p, x_all, z_all, w_all, params, eps, nullptr, x, nullptr, nullptr,
                           st, nullptr, 0, 0, 0, &fw));
    HIP_TRY(launch_eval(*p, n_pseudo, params, w_all, z_all, o.nll, o.stats, prob,
                        correction ? 1 : 0, W, probs_out, stats_out, st));
    return 0;
}

int psvi_hvp_partial(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
                     const float* eps, const float* params, const float* vec,
                     int32_t include_kl, float* hv_out, float* du_out, float* dw_out, void* ws,
                     size_t ws_bytes, void* stream) {
    drop_resident(p);
    if (!p) return fail(PSVI_EINVAL, "null plan");
    if (!p->on_device) return fail(PSVI_ESTATE, "plan was created without a HIP device");
    if (p->world != 1) return fail(PSVI_ESTATE, "psvi_hvp needs world == 1");
    if (!u || !z || !w || !eps || !params || !vec || !hv_out)
        return fail(PSVI_EINVAL, "null pointer");
    if (p->family == PSVI_FAMILY_LENET) {
        if (!ws || ws_bytes < lenet_tan_ws(*p, nullptr).bytes)
            return fail(PSVI_ENOSPC, "workspace too small");
        HIP_TRY(launch_lenet_hvp(*p, u, z, w, eps, params, vec, hv_out, du_out, dw_out, ws,
                                 as_stream(stream), include_kl != 0));
        return 0;
    }
    if (rop_rows(*p) == 0)
        return fail(PSVI_EUNSUP, "model too wide for the per-sample R-op kernel's LDS");
    const HvpWs o = hvp_ws(p, ws);
    if (!ws || ws_bytes < o.bytes) return fail(PSVI_ENOSPC, "workspace too small");
    hipStream_t st = as_stream(stream);
    float* x = nullptr;
    if (p->family == PSVI_FAMILY_FULLCOV) {
        x = (float*)ws;
        // x = mean + L eps; x_dot = v_mean + (sigmoid(sd) v_sd) eps + v_corr eps
        HIP_TRY(launch_mvn_fwd_pair(*p, eps, params, x, vec, o.xd, o.part2, st));
    }
    // two row-block slots per sample: added by their consumers (the K-split
    // gradient mode at staging, the assembly at its loads) rather than by a
    // slot-sum launch, when the K-split gradient mode runs
    const bool two = rop_splits(*p) == 2 &&
                     (p->family != PSVI_FAMILY_FULLCOV || mvn_grad_takes_slots(*p));
    const int64_t slot2 = two ? (int64_t)p->d.S * p->n_tot : 0;
    HIP_TRY(launch_net_rop(*p, u, z, w, x, o.xd, params, vec, eps, o.G, o.Gd,
                           du_out ? o.du : nullptr, dw_out ? o.nlld : nullptr, st, !two));
    if (p->family == PSVI_FAMILY_FULLCOV)  // J^T G_dot (mean, sd, corr; + the corr KL block)
        HIP_TRY(launch_mvn_update(*p, eps, o.Gd, const_cast<float*>(params), nullptr, nullptr,
                                  nullptr, nullptr, hv_out, 0, nullptr, nullptr, st, nullptr,
                                  false, include_kl ? vec : nullptr, false, nullptr, nullptr,
                                  two ? o.Gd + slot2 : nullptr));
    HIP_TRY(launch_hvp_assemble(*p, params, vec, eps, o.G, o.Gd, o.du, o.nlld, hv_out, du_out,
                                dw_out, st, include_kl != 0, slot2));
    return 0;
}

int psvi_hvp(const psvi_plan* p, const float* u, const int32_t* z, const float* w,
             const float* eps, const float* params, const float* vec, float* hv_out,
             float* du_out, float* dw_out, void* ws, size_t ws_bytes, void* stream) {
    return psvi_hvp_partial(p, u, z, w, eps, params, vec, 1, hv_out, du_out, dw_out, ws,
                            ws_bytes, stream);
}

int psvi_adam_adjoint(int64_t n, const float* lt, float* lm, float* lv, const float* adam_m,
                      const float* adam_v, const float* grad, float* lg_out,
                      const psvi_adam_hp* hp, void* stream) {
    if (n < 0 || !lt || !lm || !lv || !adam_m || !adam_v || !grad || !lg_out || !hp)
        return fail(PSVI_EINVAL, "bad adam adjoint arguments");
    if (hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (hp->kind != PSVI_ADAM_HIGHER && hp->kind != PSVI_ADAM_HYPERGRAD)
        return fail(PSVI_EUNSUP, "adam adjoint: higher / hypergrad variants only");
    HIP_TRY(launch_adam_adjoint(n, lt, lm, lv, adam_m, adam_v, grad, lg_out, hp,
                                as_stream(stream)));
    return 0;
}

int psvi_nonfinite(const void* data, int64_t n, int32_t dtype, int32_t* flag, void* stream) {
    if (!data || !flag || n < 0 || (dtype != 0 && dtype != 1))
        return fail(PSVI_EINVAL, "bad nonfinite arguments");
    HIP_TRY(launch_nonfinite(data, n, dtype, flag, as_stream(stream)));
    return 0;
}

int psvi_randn(float* out, int64_t n, uint64_t seed, uint64_t offset, void* stream) {
    if (!out || n < 0) return fail(PSVI_EINVAL, "bad randn arguments");
    if (offset % 4) return fail(PSVI_EINVAL, "randn offset must be a multiple of 4");
    HIP_TRY(launch_randn(out, n, seed, offset, as_stream(stream)));
    return 0;
}

int psvi_adam_update(int64_t n, float* params, const float* grad, float* adam_m, float* adam_v,
                     const psvi_adam_hp* hp, void* stream) {
    if (n < 0 || !params || !grad || !adam_m || !adam_v || !hp)
        return fail(PSVI_EINVAL, "bad adam arguments");
    if (hp->step < 1) return fail(PSVI_EINVAL, "adam step must be >= 1");
    if (hp->kind < 0 || hp->kind > 2) return fail(PSVI_EINVAL, "unknown adam kind");
    HIP_TRY(launch_adam(n, params, grad, adam_m, adam_v, hp, as_stream(stream)));
    return 0;
}

size_t psvi_cg_ws_bytes(void) { return cg_ws_bytes(); }

int psvi_cg_scale(int64_t n, const float* hv, double lr, float* out, void* stream) {
    if (n < 0 || !hv || !out) return fail(PSVI_EINVAL, "bad cg_scale arguments");
    HIP_TRY(launch_cg_scale(n, hv, lr, out, as_stream(stream)));
    return 0;
}

int psvi_cg_pap(int64_t n, const float* hv1, const float* hv2, double lr, const double* p,
                double* state, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || !hv1 || !hv2 || !p || !state || !ws) return fail(PSVI_EINVAL, "bad cg_pap arguments");
    if (ws_bytes < cg_ws_bytes()) return fail(PSVI_EINVAL, "cg workspace too small");
    HIP_TRY(launch_cg_pap(n, hv1, hv2, lr, p, state, ws, as_stream(stream)));
    return 0;
}

int psvi_cg_residual(int64_t n, const float* hv1, const float* hv2, double lr, double* r,
                     double* state, double tol, void* ws, size_t ws_bytes, void* stream) {
    if (n < 0 || !hv1 || !hv2 || !r || !state || !ws)
        return fail(PSVI_EINVAL, "bad cg_residual arguments");
    if (ws_bytes < cg_ws_bytes()) return fail(PSVI_EINVAL, "cg workspace too small");
    HIP_TRY(launch_cg_residual(n, hv1, hv2, lr, r, state, tol, ws, as_stream(stream)));
    return 0;
}

int psvi_cg_update(int64_t n, double* x, double* p, float* p32, const double* r,
                   const double* state, void* stream) {
    if (n < 0 || !x || !p || !p32 || !r || !state) return fail(PSVI_EINVAL, "bad cg_update arguments");
    HIP_TRY(launch_cg_update(n, x, p, p32, r, state, as_stream(stream)));
    return 0;
}

}  // extern "C"
