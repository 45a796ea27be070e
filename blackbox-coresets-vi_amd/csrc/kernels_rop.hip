// kernels_rop.hip -- Hessian-vector products of the inner ELBO (psvi_hvp) for
// hypergrad's CG_normaleq (the `hyper` trainer's implicit hypergradient).
//
// Reference (/root/reference):
//   PSVI.hyper_step            psvi/inference/psvi_classes.py:602-687
//   CG_normaleq / jvp / grd    psvi/hypergrad/hypergradients.py:199-244, 300-311
//   GradientDescent fp_map     psvi/hypergrad/diff_optimizers.py:51-60, 157-159
// The reference differentiates autograd's gradient graph a second time; here
// the product is forward-over-reverse (Pearlmutter's R-op) at fixed eps:
//   tangent sample    x_dot_s = J_s vec  (full-cov: v_mean + Lv eps_s with
//                     Lv = diag(sigmoid(sd) v_sd) + lower(v_corr); mean-field:
//                     v_mu + sigmoid(rho) v_rho eps_s)
//   tangent forward   a_dot = h_dot W^T + h W_dot^T + b_dot, h_dot = 1[a>0] a_dot
//   head              delta = w_m (p - onehot), delta_dot = w_m p (a_dot - p.a_dot),
//                     NLL_dot = (p - onehot).a_dot
//   R-backward        dW_dot = delta_dot^T h + delta^T h_dot,
//                     delta_dot' = (delta_dot W + delta W_dot) 1[a>0]
// (net_rop_kernel: one workgroup per sample, rows in chunks, VALU), then the
// reparameterised backward of G_dot (the update kernel's gradient mode for
// full-cov), the softplus curvature sum_s (G_s . eps_s) sigmoid'(sd) v_sd and
// the KL Hessian (hvp_param_kernel).  The mixed products the hypergradient
// needs come out of the same pass: d/du (vec . grad) = sum_s delta_dot_0 W +
// delta_0 W_dot, d/dw_m (vec . grad) = sum_s NLL_dot_sm.
#include <algorithm>

#include "mfma_tiles.hpp"
#include "psvi_internal.hpp"

namespace psvi {

struct RopArgs {
    int L, M, S, n_tot, family, rc, maxd;
    int nsplit;  // workgroups per sample (row blocks), each storing its G / G_dot partial
                 // into its own slot [split][S][n_tot]; slot_sum_kernel adds them in order
    int single;  // 1: the workgroup's rows are one chunk -- weight gradients go straight
                 // to its slot (no LDS accumulators)
    int din[kMaxL], dout[kMaxL], woff[kMaxL];
    int64_t poff[kMaxL], eoff[kMaxL];
    int lx, lxd, lg, lgd, lh[kMaxL + 1], lhd[kMaxL + 1], ld0, ld1, ldd0, ldd1;  // LDS carve
    // W_l / W_dot_l in LDS: rows of an odd stride ldw[l] (a lane per output row
    // then hits its own bank), layer l at xo[l] of the X / XD regions, b after W
    int ldw[kMaxL], xo[kMaxL];
    // MFMA form (net_rop_mfma_kernel): X_l (l = 0..L) at mxo[l], rows of
    // ldxm[l] floats = [h | h_dot] halves of kx[l] = rup16(width) (X_0: the u
    // rows alone; X_L: logits and their tangents); W2_l at mwo[l], rup16(dout)
    // rows of ldwm[l] = [W | W_dot] halves of kx[l]; b_l | b_dot_l at mbo[l]
    // (halves of kx[l + 1])
    int mxo[kMaxL + 1], ldxm[kMaxL + 1], kx[kMaxL + 1], mwo[kMaxL], ldwm[kMaxL], mbo[kMaxL], lstamp;
    int jw[kMaxL], jbl[kMaxL], jb, ju;  // load jobs: layer l's W2 rows from jw[l], bias rows from jb + jbl[l], u rows from ju
    const float* u;
    const int32_t* z;
    const float* w;
    const float* x;    // full-cov: x_s   [S][n_tot]
    const float* xd;   // full-cov: x_dot [S][n_tot]
    const float* params;
    const float* vec;
    const float* eps;
    float* G;          // [S][n_tot]
    float* Gd;         // [S][n_tot]
    float* du;         // [S][M][D]
    float* nlld;       // [S][M]
    unsigned long long* stamps;  // diagnostics: 16 phase-clock sums per workgroup (nullptr)
};

unsigned long long* g_rop_stamps = nullptr;  // psvi_debug_set_ptr(PSVI_DBG_ROP_STAMPS, buf)

// layers at most this wide (the loss head) run the 16-lane K-split forms:
// the 2 x 2 register blocks leave all but a few threads idle there
constexpr int kRopNarrow = 8;

__global__ __launch_bounds__(512) void net_rop_kernel(RopArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const int L = a.L, D = a.din[0], C = a.dout[L - 1];
    float* X = sm + a.lx;
    float* XD = sm + a.lxd;
    float* GA = sm + a.lg;
    float* GDA = sm + a.lgd;
    // diagnostics (thread 0): shader clocks summed per phase -- 0 weights,
    // 1 inputs, 2-4 forward layers, 5 head, 6-8 backward layers (top first),
    // 9 the slot stores; slot 15 = chunks
    unsigned long long tph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tlast = 0;
    int nchunk = 0;
    auto ph = [&](int q) __attribute__((always_inline)) {
        if (a.stamps && tid == 0) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            if (q >= 0) tph[q] += tt - tlast;
            tlast = tt;
        }
    };
    ph(-1);
    // sampled weights and their tangents, in the per-sample weight layout
    // (layer l at woff_l: W row-major [dout][din], then b)
    for (int l = 0; l < L && a.family == PSVI_FAMILY_FULLCOV; ++l) {
        // full-cov: the layer's x / x_dot loads all in flight (clamped indices,
        // kB per thread), then the scatter; a load-use per element serialised
        // the phase on the memory latency
        constexpr int kB = 8;
        const int din = a.din[l], dout = a.dout[l], n = din * dout + dout, nw = din * dout;
        const float rdin = 1.f / (float)din;
        const float* xr = a.x + (int64_t)s * a.n_tot + a.woff[l];
        const float* xdr = a.xd + (int64_t)s * a.n_tot + a.woff[l];
        for (int base = tid; base < n; base += kB * nt) {
            float xv[kB], xdv[kB];
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                const int i = min(base + k * nt, n - 1);
                xv[k] = xr[i];
                xdv[k] = xdr[i];
            }
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                const int i = base + k * nt;
                if (i >= n) break;
                // exact for i < 2^21: (i + 0.5) / din is >= 0.5 / din from an integer
                const int j = (int)(((float)i + 0.5f) * rdin);
                const int dst = a.xo[l] + (i < nw ? j * a.ldw[l] + (i - j * din)
                                                  : dout * a.ldw[l] + (i - nw));
                X[dst] = xv[k];
                XD[dst] = xdv[k];
                if (!a.single) {
                    GA[a.woff[l] + i] = 0.f;
                    GDA[a.woff[l] + i] = 0.f;
                }
            }
        }
    }
    for (int l = 0; l < L && a.family != PSVI_FAMILY_FULLCOV; ++l) {
        const int din = a.din[l], dout = a.dout[l], n = din * dout + dout, nw = din * dout;
        for (int i = tid; i < n; i += nt) {
            const int o = a.woff[l] + i;
            float xv, xdv;
            {
                const float e = i < nw ? a.eps[a.eoff[l] + (int64_t)s * nw + i]
                                       : a.eps[a.eoff[l] + (int64_t)a.S * nw + (int64_t)s * dout + i - nw];
                const int64_t pm = a.poff[l] + i, pr = pm + n;
                const float rho = a.params[pr];
                xv = a.params[pm] + softplus_f(rho) * e;
                xdv = a.vec[pm] + sigmoid_f(rho) * a.vec[pr] * e;
            }
            const int dst = a.xo[l] + (i < nw ? (i / din) * a.ldw[l] + i % din
                                              : dout * a.ldw[l] + (i - nw));
            X[dst] = xv;
            XD[dst] = xdv;
            if (!a.single) {
                GA[o] = 0.f;
                GDA[o] = 0.f;
            }
        }
    }
    __syncthreads();
    ph(0);
    const int rows_per = (a.M + a.nsplit - 1) / a.nsplit;
    const int m_lo = blockIdx.y * rows_per, m_hi = min(a.M, m_lo + rows_per);
    for (int m0 = m_lo; m0 < m_hi; m0 += a.rc) {
        const int rc = min(a.rc, m_hi - m0);
        // inputs: h_0 = u rows, h_dot_0 = 0 (the loads of a pass all in flight)
        {
            constexpr int kB = 8;
            const float* ur = a.u + (int64_t)m0 * D;
            const int nu = rc * D;
            for (int base = tid; base < nu; base += kB * nt) {
                float uv[kB];
#pragma unroll
                for (int k = 0; k < kB; ++k) uv[k] = ur[min(base + k * nt, nu - 1)];
#pragma unroll
                for (int k = 0; k < kB; ++k) {
                    const int i = base + k * nt;
                    if (i >= nu) break;
                    sm[a.lh[0] + i] = uv[k];
                    sm[a.lhd[0] + i] = 0.f;
                }
            }
        }
        __syncthreads();
        ph(1);
        ++nchunk;
        // forward + tangent forward: 2 rows x 2 outputs per thread (8 LDS
        // reads per 12 FMAs; clamped duplicates at odd edges, stored once)
        for (int l = 0; l < L; ++l) {
            const int din = a.din[l], dout = a.dout[l], ldw = a.ldw[l];
            const float* W = X + a.xo[l];
            const float* Wd = XD + a.xo[l];
            const float* b = W + dout * ldw;
            const float* bd = Wd + dout * ldw;
            const float* H = sm + a.lh[l];
            const float* HD = sm + a.lhd[l];
            float* Hn = sm + a.lh[l + 1];
            float* HDn = sm + a.lhd[l + 1];
            if (dout <= kRopNarrow) {
                // narrow layer (the head): a 16-lane row per (row m, output o),
                // lane j summing inputs i = j, j + 16, ..; DPP row sums
                const int np = rc * dout, nrow = nt >> 4, lr = tid & 15;
                const int trips = (np + nrow - 1) / nrow;
                for (int t = 0; t < trips; ++t) {  // uniform: every lane of every row active
                    const int pr = t * nrow + (tid >> 4);
                    const bool valid = pr < np;
                    const int m = valid ? pr / dout : 0, o = valid ? pr - m * dout : 0;
                    float acc = 0.f, accd = 0.f;
                    for (int i = lr; i < din; i += 16) {
                        const float hv = H[m * din + i], hdv = HD[m * din + i];
                        const float wv = W[o * ldw + i], wdv = Wd[o * ldw + i];
                        acc = fmaf(hv, wv, acc);
                        accd = fmaf(hdv, wv, fmaf(hv, wdv, accd));
                    }
                    acc = row16_sum(acc) + b[o];
                    accd = row16_sum(accd) + bd[o];
                    if (valid && lr == 0) {
                        const int qq = m * dout + o;
                        const bool on = l == L - 1 || acc > 0.f;
                        Hn[qq] = l == L - 1 ? acc : (on ? acc : 0.f);
                        HDn[qq] = on ? accd : 0.f;
                    }
                }
                __syncthreads();
                ph(2 + min(l, 2));
                continue;
            }
            const int nbo = (dout + 1) >> 1, nb = ((rc + 1) >> 1) * nbo;
            for (int q = tid; q < nb; q += nt) {
                const int bm = q / nbo, bo = q - bm * nbo;
                const int ma = 2 * bm, o0 = 2 * bo;
                const int mb = min(ma + 1, rc - 1), o1 = min(o0 + 1, dout - 1);
                float acc[2][2], accd[2][2];
                acc[0][0] = acc[1][0] = b[o0];
                acc[0][1] = acc[1][1] = b[o1];
                accd[0][0] = accd[1][0] = bd[o0];
                accd[0][1] = accd[1][1] = bd[o1];
                const float* h0 = H + ma * din;
                const float* h1 = H + mb * din;
                const float* hd0 = HD + ma * din;
                const float* hd1 = HD + mb * din;
                const float* w0 = W + o0 * ldw;
                const float* w1 = W + o1 * ldw;
                const float* wd0 = Wd + o0 * ldw;
                const float* wd1 = Wd + o1 * ldw;
                if ((din & 3) == 0) {
                    // h / h_dot rows as float4 (rows 16-byte aligned when din % 4 == 0)
                    for (int i = 0; i < din; i += 4) {
                        const float4 ha = *reinterpret_cast<const float4*>(h0 + i);
                        const float4 hb = *reinterpret_cast<const float4*>(h1 + i);
                        const float4 hda = *reinterpret_cast<const float4*>(hd0 + i);
                        const float4 hdb = *reinterpret_cast<const float4*>(hd1 + i);
                        const float hv4[2][4] = {{ha.x, ha.y, ha.z, ha.w}, {hb.x, hb.y, hb.z, hb.w}};
                        const float hdv4[2][4] = {{hda.x, hda.y, hda.z, hda.w},
                                                  {hdb.x, hdb.y, hdb.z, hdb.w}};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float wv[2] = {w0[i + j], w1[i + j]}, wdv[2] = {wd0[i + j], wd1[i + j]};
#pragma unroll
                            for (int r = 0; r < 2; ++r)
#pragma unroll
                                for (int c = 0; c < 2; ++c) {
                                    acc[r][c] = fmaf(hv4[r][j], wv[c], acc[r][c]);
                                    accd[r][c] = fmaf(hdv4[r][j], wv[c], fmaf(hv4[r][j], wdv[c], accd[r][c]));
                                }
                        }
                    }
                } else {
#pragma unroll 4
                    for (int i = 0; i < din; ++i) {
                        const float hv[2] = {h0[i], h1[i]}, hdv[2] = {hd0[i], hd1[i]};
                        const float wv[2] = {w0[i], w1[i]}, wdv[2] = {wd0[i], wd1[i]};
#pragma unroll
                        for (int r = 0; r < 2; ++r)
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                acc[r][c] = fmaf(hv[r], wv[c], acc[r][c]);
                                accd[r][c] = fmaf(hdv[r], wv[c], fmaf(hv[r], wdv[c], accd[r][c]));
                            }
                    }
                }
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        if ((r && mb == ma) || (c && o1 == o0)) continue;
                        const int qq = (r ? mb : ma) * dout + (c ? o1 : o0);
                        const float av = acc[r][c], ad = accd[r][c];
                        if (l < L - 1) {
                            Hn[qq] = av > 0.f ? av : 0.f;
                            HDn[qq] = av > 0.f ? ad : 0.f;
                        } else {
                            Hn[qq] = av;
                            HDn[qq] = ad;
                        }
                    }
            }
            __syncthreads();
            ph(2 + min(l, 2));
        }
        // head: delta = w (p - onehot), delta_dot = w p (a_dot - p.a_dot)
        float* Dl = sm + a.ld0;
        float* DDl = sm + a.ldd0;
        float* Dn = sm + a.ld1;
        float* DDn = sm + a.ldd1;
        for (int m = tid; m < rc; m += nt) {
            const float* lg = sm + a.lh[L] + m * C;
            const float* ld = sm + a.lhd[L] + m * C;
            const int zm = a.z[m0 + m];
            const float wm = a.w[m0 + m];
            float mx = -INFINITY;
            for (int c = 0; c < C; ++c) mx = fmaxf(mx, lg[c]);
            float se = 0.f;
            for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
            const float lse = mx + logf(se);
            float pad = 0.f, nd = 0.f;
            for (int c = 0; c < C; ++c) pad += expf(lg[c] - lse) * ld[c];
            for (int c = 0; c < C; ++c) {
                const float p = expf(lg[c] - lse);
                const float pmo = p - (c == zm ? 1.f : 0.f);
                nd = fmaf(pmo, ld[c], nd);
                Dl[m * a.maxd + c] = wm * pmo;
                DDl[m * a.maxd + c] = wm * p * (ld[c] - pad);
            }
            if (a.nlld) a.nlld[(int64_t)s * a.M + m0 + m] = nd;
        }
        __syncthreads();
        ph(5);
        // R-backward: weight gradients 2 outputs x 2 inputs per thread, the
        // propagation 2 rows x 2 inputs (as the forward)
        for (int l = L - 1; l >= 0; --l) {
            const int din = a.din[l], dout = a.dout[l], nw = din * dout, ldw = a.ldw[l];
            const float* W = X + a.xo[l];
            const float* Wd = XD + a.xo[l];
            const float* H = sm + a.lh[l];
            const float* HD = sm + a.lhd[l];
            // one chunk: straight into this row block's slot; else the LDS
            // accumulators (added over chunks, stored at the end)
            const int64_t gslot = ((int64_t)blockIdx.y * a.S + s) * a.n_tot + a.woff[l];
            float* GW = a.single ? a.G + gslot : GA + a.woff[l];
            float* GDW = a.single ? a.Gd + gslot : GDA + a.woff[l];
            auto put = [&](float* P, int i, float v) __attribute__((always_inline)) {
                if (a.single) P[i] = v;
                else P[i] += v;
            };
            const int md = a.maxd;
            const int nbi = (din + 1) >> 1, nbw = ((dout + 1) >> 1) * nbi;
            if (dout <= kRopNarrow) {
                // narrow layer: a 16-lane row per weight (then per bias), lane j
                // summing rows m = j, j + 16, ..; DPP row sums
                const int ne = nw + dout, nrow = nt >> 4, lr = tid & 15;
                const int trips = (ne + nrow - 1) / nrow;
                for (int t = 0; t < trips; ++t) {  // uniform
                    const int e = t * nrow + (tid >> 4);
                    const bool valid = e < ne;
                    float g = 0.f, gd = 0.f;
                    if (e < nw) {  // row-uniform
                        const int o = e / din, i = e - o * din;
                        for (int m = lr; m < rc; m += 16) {
                            const float dl = Dl[m * md + o], ddl = DDl[m * md + o];
                            const float hv = H[m * din + i], hdv = HD[m * din + i];
                            g = fmaf(dl, hv, g);
                            gd = fmaf(ddl, hv, fmaf(dl, hdv, gd));
                        }
                    } else {
                        const int o = valid ? e - nw : 0;
                        for (int m = lr; m < rc; m += 16) {
                            g += Dl[m * md + o];
                            gd += DDl[m * md + o];
                        }
                    }
                    g = row16_sum(g);
                    gd = row16_sum(gd);
                    if (valid && lr == 0) {
                        put(GW, e, g);
                        put(GDW, e, gd);
                    }
                }
            }
            // wide layers with din % 4 == 0: 2 outputs x 4 inputs per thread, h
            // and h_dot rows read as float4 (6 LDS reads per 24 FMAs instead of
            // 8 per 12); the rest keep the 2 x 2 blocks
            const bool wide4 = dout > kRopNarrow && (din & 3) == 0;
            if (wide4) {
                const int nbi4 = din >> 2, nbw4 = ((dout + 1) >> 1) * nbi4;
                for (int q = tid; q < nbw4 + dout; q += nt) {
                    if (q < nbw4) {
                        const int bo = q / nbi4, bi = q - bo * nbi4;
                        const int o0 = 2 * bo, o1 = min(o0 + 1, dout - 1), i0 = 4 * bi;
                        float g[2][4], gd[2][4];
#pragma unroll
                        for (int r = 0; r < 2; ++r)
#pragma unroll
                            for (int c = 0; c < 4; ++c) g[r][c] = gd[r][c] = 0.f;
#pragma unroll 2
                        for (int m = 0; m < rc; ++m) {
                            const float dl[2] = {Dl[m * md + o0], Dl[m * md + o1]};
                            const float ddl[2] = {DDl[m * md + o0], DDl[m * md + o1]};
                            const float4 h4 = *reinterpret_cast<const float4*>(H + m * din + i0);
                            const float4 hd4 = *reinterpret_cast<const float4*>(HD + m * din + i0);
                            const float hv[4] = {h4.x, h4.y, h4.z, h4.w};
                            const float hdv[4] = {hd4.x, hd4.y, hd4.z, hd4.w};
#pragma unroll
                            for (int r = 0; r < 2; ++r)
#pragma unroll
                                for (int c = 0; c < 4; ++c) {
                                    g[r][c] = fmaf(dl[r], hv[c], g[r][c]);
                                    gd[r][c] = fmaf(ddl[r], hv[c], fmaf(dl[r], hdv[c], gd[r][c]));
                                }
                        }
#pragma unroll
                        for (int r = 0; r < 2; ++r) {
                            if (r && o1 == o0) continue;
#pragma unroll
                            for (int c = 0; c < 4; ++c) {
                                const int qq = (r ? o1 : o0) * din + i0 + c;
                                put(GW, qq, g[r][c]);
                                put(GDW, qq, gd[r][c]);
                            }
                        }
                    } else {
                        const int o = q - nbw4;
                        float g = 0.f, gd = 0.f;
                        for (int m = 0; m < rc; ++m) {
                            g += Dl[m * md + o];
                            gd += DDl[m * md + o];
                        }
                        put(GW, nw + o, g);
                        put(GDW, nw + o, gd);
                    }
                }
            }
            for (int q = tid; q < (dout <= kRopNarrow || wide4 ? 0 : nbw + dout); q += nt) {
                if (q < nbw) {
                    const int bo = q / nbi, bi = q - bo * nbi;
                    const int o0 = 2 * bo, i0 = 2 * bi;
                    const int o1 = min(o0 + 1, dout - 1), i1 = min(i0 + 1, din - 1);
                    float g[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, gd[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll 4
                    for (int m = 0; m < rc; ++m) {
                        const float dl[2] = {Dl[m * md + o0], Dl[m * md + o1]};
                        const float ddl[2] = {DDl[m * md + o0], DDl[m * md + o1]};
                        const float hv[2] = {H[m * din + i0], H[m * din + i1]};
                        const float hdv[2] = {HD[m * din + i0], HD[m * din + i1]};
#pragma unroll
                        for (int r = 0; r < 2; ++r)
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                g[r][c] = fmaf(dl[r], hv[c], g[r][c]);
                                gd[r][c] = fmaf(ddl[r], hv[c], fmaf(dl[r], hdv[c], gd[r][c]));
                            }
                    }
#pragma unroll
                    for (int r = 0; r < 2; ++r)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            if ((r && o1 == o0) || (c && i1 == i0)) continue;
                            const int qq = (r ? o1 : o0) * din + (c ? i1 : i0);
                            put(GW, qq, g[r][c]);
                            put(GDW, qq, gd[r][c]);
                        }
                } else {
                    const int o = q - nbw;
                    float g = 0.f, gd = 0.f;
                    for (int m = 0; m < rc; ++m) {
                        g += Dl[m * md + o];
                        gd += DDl[m * md + o];
                    }
                    put(GW, nw + o, g);
                    put(GDW, nw + o, gd);
                }
            }
            if (l > 0 || a.du) {
                // delta' = (delta W) 1[h > 0]   (h = relu(a_{l-1}); none at the input)
                const int nbp = ((rc + 1) >> 1) * nbi;
                for (int q = tid; q < nbp; q += nt) {
                    const int bm = q / nbi, bi = q - bm * nbi;
                    const int ma = 2 * bm, i0 = 2 * bi;
                    const int mb = min(ma + 1, rc - 1), i1 = min(i0 + 1, din - 1);
                    float t[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, td[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll 4
                    for (int o = 0; o < dout; ++o) {
                        const float dl[2] = {Dl[ma * md + o], Dl[mb * md + o]};
                        const float ddl[2] = {DDl[ma * md + o], DDl[mb * md + o]};
                        const float wv[2] = {W[o * ldw + i0], W[o * ldw + i1]};
                        const float wdv[2] = {Wd[o * ldw + i0], Wd[o * ldw + i1]};
#pragma unroll
                        for (int r = 0; r < 2; ++r)
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                t[r][c] = fmaf(dl[r], wv[c], t[r][c]);
                                td[r][c] = fmaf(ddl[r], wv[c], fmaf(dl[r], wdv[c], td[r][c]));
                            }
                    }
#pragma unroll
                    for (int r = 0; r < 2; ++r)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            if ((r && mb == ma) || (c && i1 == i0)) continue;
                            const int m = r ? mb : ma, i = c ? i1 : i0;
                            if (l > 0) {
                                const bool on = H[m * din + i] > 0.f;
                                Dn[m * md + i] = on ? t[r][c] : 0.f;
                                DDn[m * md + i] = on ? td[r][c] : 0.f;
                            } else {
                                a.du[((int64_t)s * a.M + m0 + m) * D + i] = td[r][c];
                            }
                        }
                }
            }
            __syncthreads();
            ph(6 + min(L - 1 - l, 2));
            float* t0 = Dl; Dl = Dn; Dn = t0;
            float* t1 = DDl; DDl = DDn; DDn = t1;
        }
    }
    // this row block's partial into its own slot (no atomics, no zeroing)
    const int64_t slot = ((int64_t)blockIdx.y * a.S + s) * a.n_tot;
    for (int o = tid; o < (a.single ? 0 : a.n_tot); o += nt) {
        a.G[slot + o] = GA[o];
        a.Gd[slot + o] = GDA[o];
    }
    ph(9);
    if (a.stamps && tid == 0) {
        unsigned long long* o = a.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16;
        for (int q = 0; q < 10; ++q) o[q] = tph[q];
        o[15] = nchunk;
    }
}

// ------------------------------------------------------------ MFMA R-op
// The R-op's GEMMs come in pairs -- a product and its tangent -- over the same
// operands and their tangent halves:
//   X[p][q] = sum_k A(p,k) B(q,k)
//   Y[p][q] = sum_k A(p,k) B'(q,k) + A'(p,k) B(q,k)
// with A' = A + oa, B' = B + ob (each row holds [value | tangent]).  TA / TB
// false: that tangent operand is zero (the u rows); WX false: X is not formed.
// Operands as the network kernel's tiles (mfma_tiles.hpp): k-contiguous as one
// float4 per lane and k-group, k-strided as four rows in the kbase / kstep
// order; v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation).
template <bool ACONT, bool BCONT, int NQ, bool TA, bool TB, bool WX>
struct RopFrag {
    using T = TileOps<ACONT, BCONT, NQ>;
    static constexpr bool PERM = T::PERM;
    floatx4 a, at, b[NQ], bt[NQ];
    __device__ __forceinline__ static floatx4 ld(const float* p, int ldx, bool cont) {
        return __builtin_bit_cast(floatx4, T::ld(p, ldx, cont));
    }
    __device__ __forceinline__ void load(const float* pa, int lda, int oa, const float* pb, int ldb,
                                         int ob) {
        a = ld(pa, lda, ACONT);
        if (TA) at = ld(pa + oa, lda, ACONT);
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            const float* q = pb + 16 * c * (BCONT ? ldb : 1);
            b[c] = ld(q, ldb, BCONT);
            if (TB) bt[c] = ld(q + ob, ldb, BCONT);
        }
    }
    __device__ __forceinline__ void mma(floatx4 (&x)[NQ], floatx4 (&y)[NQ]) const {
#pragma unroll
        for (int c = 0; c < NQ; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (WX) x[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[c][j], x[c], 0, 0, 0);
                if (TB) y[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], bt[c][j], y[c], 0, 0, 0);
                if (TA) y[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(at[j], b[c][j], y[c], 0, 0, 0);
            }
    }
};

// Units of one 16-row tile x NQ column tiles dealt round-robin to the waves
// (from wave `first`); per unit the k-groups run two deep (the next group's
// LDS reads issued before the current group's MFMAs).  The epilogue gets
// (first row of the lane's four, column, X and Y of the four rows, rotation):
// odd lane-groups hand their rows over rotated by two, as the network kernel's
// epilogues (row (r + rot) & 3 of the four is value r).
template <bool ACONT, bool BCONT, int NQ, bool TA, bool TB, bool WX, class Epi>
__device__ __forceinline__ void rop_steps(int nu, int tqu, int nk, int u0, int nwv, const float* A,
                                          int lda, int oa, const float* B, int ldb, int ob, Epi epi) {
    using F = RopFrag<ACONT, BCONT, NQ, TA, TB, WX>;
    constexpr bool PERM = F::PERM;
    const int lane = threadIdx.x & 63, i16 = lane & 15, k4 = lane >> 4;
    const int da = ACONT ? 16 : 16 * lda, db = BCONT ? 16 : 16 * ldb;
    const int rot = (k4 & 1) << 1, r0 = kbase<PERM>(k4);
    for (int u = u0; u < nu; u += nwv) {  // wave-uniform
        const int pt = u / tqu, p0 = pt << 4, q0 = ((u - pt * tqu) * NQ) << 4;
        const float* pa = ACONT ? A + (p0 + i16) * lda + 4 * k4 : A + r0 * lda + p0 + i16;
        const float* pb = BCONT ? B + (q0 + i16) * ldb + 4 * k4 : B + r0 * ldb + q0 + i16;
        floatx4 x[NQ], y[NQ];
#pragma unroll
        for (int c = 0; c < NQ; ++c) x[c] = y[c] = floatx4{0.f, 0.f, 0.f, 0.f};
        // two k-groups per trip with fixed registers (the next group's LDS
        // reads in flight across the current group's MFMAs), then the tail
        F f0, f1;
        f0.load(pa, lda, oa, pb, ldb, ob);
        int kg = 0;
        for (; kg + 2 < nk; kg += 2) {
            pa += da;
            pb += db;
            f1.load(pa, lda, oa, pb, ldb, ob);
            f0.mma(x, y);
            pa += da;
            pb += db;
            f0.load(pa, lda, oa, pb, ldb, ob);
            f1.mma(x, y);
        }
        if (kg + 1 < nk) {
            pa += da;
            pb += db;
            f1.load(pa, lda, oa, pb, ldb, ob);
            f0.mma(x, y);
            f1.mma(x, y);
        } else {
            f0.mma(x, y);
        }
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            const floatx4 vx = x[c], vy = y[c];
            epi(p0 + 4 * k4, q0 + 16 * c + i16, rot ? floatx4{vx[2], vx[3], vx[0], vx[1]} : vx,
                rot ? floatx4{vy[2], vy[3], vy[0], vy[1]} : vy, rot);
        }
    }
}

// P x Q outputs, contraction over K16 / 16 k-groups of 16 (operand rows or
// columns past the true length are zero in LDS), single 16 x 16 tiles dealt
// round-robin to the waves (rows of up to three column tiles per unit were
// measured slower in round 5: 256 VGPRs).
template <bool ACONT, bool BCONT, bool TA, bool TB, bool WX, class Epi>
__device__ __forceinline__ void rop_gemm(int P, int Q, int K16, int first, const float* A,
                                         int lda, int oa, const float* B, int ldb, int ob, Epi epi) {
    const int nwv = blockDim.x >> 6, wid = wave_id();
    const int tp = (P + 15) >> 4, tq = (Q + 15) >> 4, nk = K16 >> 4;
    const int u0 = ((wid - first) % nwv + nwv) % nwv;
    rop_steps<ACONT, BCONT, 1, TA, TB, WX>(tp * tq, tq, nk, u0, nwv, A, lda, oa, B, ldb, ob, epi);
}

// The R-op on the matrix cores: one workgroup per (sample, row block), its
// rows in one pass (launch_net_rop takes this form when the carve fits the LDS).
// Per layer l, forward: [a | a_dot] = X_l [W | W_dot]^T pairs (X = h W^T,
// Y = h W_dot^T + h_dot W^T) + [b | b_dot], the ReLU and its mask in the
// epilogue into X_{l+1}; the head in place on X_L (delta | delta_dot); per
// layer backward: the weight gradients [G | G_dot] = D^T [h | h_dot] pairs
// (a contraction over the rows, both operands k-strided) straight into the
// row block's slot, then the propagation D W / D W_dot + D_dot W masked by
// 1[h > 0] in place over X_l (after a barrier: the weight gradients read it),
// or at the input the d/du tangent rows.  Every region's padding (columns to
// kx, W rows to rup16(dout)) is written zero; rows past the block's are never
// written: their over-reads feed only output rows that are not stored, and the
// contraction over rows masks them.
__device__ __forceinline__ void lds_dma4(rsrc_t r, float* lds, uint32_t voff) {
    // one dword per lane into LDS at the wave-uniform base `lds` + 4 lane
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}

template <bool FC>
__global__ __launch_bounds__(512) void net_rop_mfma_kernel(RopArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const int L = a.L, D = a.din[0], C = a.dout[L - 1];
    const int rows_per = (a.M + a.nsplit - 1) / a.nsplit;
    const int m0 = blockIdx.y * rows_per, rc = max(0, min(a.M, m0 + rows_per) - m0);
    // diagnostics (thread 0): phase clocks summed into LDS past the carve
    // (a register array indexed at run time would live in scratch)
    unsigned long long* tph = reinterpret_cast<unsigned long long*>(sm + a.lstamp);
    unsigned long long tlast = 0;
    auto ph = [&](int q) __attribute__((always_inline)) {
        if (a.stamps && tid == 0) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            if (q >= 0) tph[q] += tt - tlast;
            tlast = tt;
        }
    };
    if (a.stamps && tid == 0)
        for (int q = 0; q < 10; ++q) tph[q] = 0;
    ph(-1);
    // ---- the load phase as wave jobs (a job: one row of up to 64 columns,
    // lane = column; no per-element index arithmetic, coalesced loads, the
    // padding columns written by the same instruction): W2_l rows (value and
    // tangent halves), then the [b | b_dot] rows, then the u rows into X_0
    // (tangent half zero).  Full-cov: buffer loads straight into LDS, every
    // job's loads in flight at once (a lane past the row's data reads the
    // buffer's out-of-range 0).  Mean-field: the sampled values are formed in
    // registers, a few jobs' loads in flight.
    {
        const int lane = tid & 63, wid = wave_id(), nwv = nt >> 6;
        const int nch0 = (a.kx[0] + 63) >> 6;
        const int njobs = a.ju + rc * nch0;
        // job j -> kind (0 W2 row, 1 bias row, 2 u row), layer, row, first column (uniform)
        auto decode = [&](int j, int& kind, int& l, int& row, int& c0) __attribute__((always_inline)) {
            l = 0;
            if (j < a.jb) {
                kind = 0;
                while (l + 1 < L && j >= a.jw[l + 1]) ++l;
                const int r = j - a.jw[l], nch = (a.kx[l] + 63) >> 6;
                row = nch == 1 ? r : r / nch;
                c0 = (r - row * nch) << 6;
            } else if (j < a.ju) {
                kind = 1;
                while (l + 1 < L && j >= a.jb + a.jbl[l + 1]) ++l;
                row = 0;
                c0 = (j - a.jb - a.jbl[l]) << 6;
            } else {
                kind = 2;
                const int r = j - a.ju;
                row = nch0 == 1 ? r : r / nch0;
                c0 = (r - row * nch0) << 6;
            }
        };
        if constexpr (FC) {
            // per layer (its dimensions read once), the layer's rows dealt to
            // the waves; the DMAs are fire-and-forget, so the deal's imbalance
            // costs issue slots only
            const rsrc_t rx = make_rsrc(a.x + (int64_t)s * a.n_tot, 4 * (int64_t)a.n_tot);
            const rsrc_t rxd = make_rsrc(a.xd + (int64_t)s * a.n_tot, 4 * (int64_t)a.n_tot);
            const rsrc_t ru = make_rsrc(a.u + (int64_t)m0 * D, 4 * (int64_t)rc * D);
            for (int l = 0; l < L; ++l) {  // uniform
                const int din = a.din[l], dout = a.dout[l], kxl = a.kx[l], kq = a.kx[l + 1];
                const int ldw = a.ldwm[l], nch = (kxl + 63) >> 6, woff = a.woff[l];
                float* const W2 = sm + a.mwo[l];
                for (int r = wid; r < kq * nch; r += nwv) {  // wave-uniform
                    const int row = nch == 1 ? r : r / nch, c0 = (r - row * nch) << 6, c = c0 + lane;
                    float* d = W2 + row * ldw + c0;
                    if (c < kxl) {
                        const uint32_t vo = row < dout && c < din ? 4u * (uint32_t)(woff + row * din + c) : kOOB;
                        lds_dma4(rx, d, vo);
                        lds_dma4(rxd, d + kxl, vo);
                    }
                }
                float* const bb = sm + a.mbo[l];
                for (int c0 = 64 * ((wid + l) % nwv); c0 < kq; c0 += 64 * nwv) {  // wave-uniform
                    const int c = c0 + lane;
                    if (c < kq) {
                        const uint32_t vo = c < dout ? 4u * (uint32_t)(woff + din * dout + c) : kOOB;
                        lds_dma4(rx, bb + c0, vo);
                        lds_dma4(rxd, bb + kq + c0, vo);
                    }
                }
            }
            {
                const int kx0 = a.kx[0], ld0 = a.ldxm[0];
                for (int r = wid; r < rc * nch0; r += nwv) {  // wave-uniform
                    const int row = nch0 == 1 ? r : r / nch0, c0 = (r - row * nch0) << 6, c = c0 + lane;
                    float* d = sm + a.mxo[0] + row * ld0 + c0;
                    if (c < kx0) {
                        lds_dma4(ru, d, c < D ? 4u * (uint32_t)(row * D + c) : kOOB);
                    }
                }
            }
            // rows rc .. rup16(rc) of every activation region (contiguous) and
            // the u rows' tangent half: zero, by plain stores (disjoint from the DMAs)
            {
                const int nz = ((rc + 15) & ~15) - rc;
                for (int l = 0; l <= L; ++l) {
                    float4* z4 = reinterpret_cast<float4*>(sm + a.mxo[l] + rc * a.ldxm[l]);
                    for (int i = tid; i < (nz * a.ldxm[l]) >> 2; i += nt) z4[i] = float4{0.f, 0.f, 0.f, 0.f};
                }
                const int kx0 = a.kx[0], q4 = kx0 >> 2;
                for (int i = tid; i < rc * q4; i += nt) {
                    const int row = i / q4;
                    reinterpret_cast<float4*>(sm + a.mxo[0] + row * a.ldxm[0] + kx0)[i - row * q4] =
                        float4{0.f, 0.f, 0.f, 0.f};
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (D < a.kx[0]) {
                // layer 0's ones column, over this wave's own DMA'd rows
                const int ld0 = a.ldxm[0];
                for (int r = wid; r < rc * nch0; r += nwv) {  // wave-uniform
                    const int row = nch0 == 1 ? r : r / nch0, c0 = (r - row * nch0) << 6;
                    if (c0 + lane == D) sm[a.mxo[0] + row * ld0 + D] = 1.f;
                }
            }
        } else {
            auto fetch_w = [&](int l, int i, float& xv, float& xdv) __attribute__((always_inline)) {
                // element i of layer l's sampled weights (W row-major, then b) and its tangent
                const int dout = a.dout[l], nw = a.din[l] * dout, n = nw + dout;
                const float e = i < nw ? a.eps[a.eoff[l] + (int64_t)s * nw + i]
                                       : a.eps[a.eoff[l] + (int64_t)a.S * nw + (int64_t)s * dout + i - nw];
                const int64_t pm = a.poff[l] + i, pr = pm + n;
                const float rho = a.params[pr];
                xv = a.params[pm] + softplus_f(rho) * e;
                xdv = a.vec[pm] + sigmoid_f(rho) * a.vec[pr] * e;
            };
            {
                const int nz = ((rc + 15) & ~15) - rc;
                for (int l = 0; l <= L; ++l)
                    for (int i = tid; i < nz * a.ldxm[l]; i += nt) sm[a.mxo[l] + rc * a.ldxm[l] + i] = 0.f;
            }
            for (int j = wid; j < njobs; j += nwv) {  // wave-uniform
                int kind, l, row, c0;
                decode(j, kind, l, row, c0);
                const int c = c0 + lane;
                float v0 = 0.f, v1 = 0.f;
                if (kind == 0) {
                    if (row < a.dout[l] && c < a.din[l]) fetch_w(l, row * a.din[l] + c, v0, v1);
                    if (c < a.kx[l]) {
                        float* w2 = sm + a.mwo[l] + row * a.ldwm[l] + c;
                        w2[0] = v0;
                        w2[a.kx[l]] = v1;
                    }
                } else if (kind == 1) {
                    if (c < a.dout[l]) fetch_w(l, a.din[l] * a.dout[l] + c, v0, v1);
                    if (c < a.kx[l + 1]) {
                        sm[a.mbo[l] + c] = v0;
                        sm[a.mbo[l] + a.kx[l + 1] + c] = v1;
                    }
                } else {
                    v0 = c == D ? 1.f : 0.f;  // the ones column
                    if (c < D) v0 = a.u[(int64_t)(m0 + row) * D + c];
                    if (c < a.kx[0]) {
                        float* x0 = sm + a.mxo[0] + row * a.ldxm[0] + c;
                        x0[0] = v0;
                        x0[a.kx[0]] = 0.f;
                    }
                }
            }
        }
    }
    __syncthreads();
    ph(0);
    // ---- forward + tangent forward, a workgroup barrier per layer.  A layer
    // whose input width is not a 16-multiple gets a column of ones at din in h
    // (W's padding column there is zero), so the weight-gradient GEMM yields
    // the bias gradient as its column din.  (A row chain -- each wave carrying
    // its 16-row tiles through every layer with no barrier -- leaves half the
    // waves idle at C3's 50-row blocks and measured slower.)
    for (int l = 0; l < L; ++l) {
        const int dout = a.dout[l], kxl = a.kx[l], kq = a.kx[l + 1], ldn = a.ldxm[l + 1];
        const float* bl = sm + a.mbo[l];
        float* Xn = sm + a.mxo[l + 1];
        const bool last = l == L - 1;
        auto epi = [&](int pr, int q, floatx4 vx, floatx4 vy, int rot) __attribute__((always_inline)) {
            const float b = bl[q], bd = bl[kq + q];  // zero past dout, as the W2 rows
            const bool one = !last && q == dout;     // the next layer's ones column
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = pr + ((r + rot) & 3);
                if (m < rc) {
                    const float av = vx[r] + b, ad = vy[r] + bd;
                    const bool on = last || av > 0.f;
                    Xn[m * ldn + q] = one ? 1.f : on ? av : 0.f;
                    Xn[m * ldn + kq + q] = on ? ad : 0.f;
                }
            }
        };
        rop_gemm<true, true, true, true, true>(rc, dout, kxl, 0, sm + a.mxo[l], a.ldxm[l], kxl,
                                                     sm + a.mwo[l], a.ldwm[l], kxl, epi);
        __syncthreads();
        ph(2 + min(l, 2));
    }
    // ---- head, in place on X_L: delta = w (p - onehot), delta_dot = w p (a_dot - p.a_dot)
    for (int m = tid; m < rc; m += nt) {
        float* lg = sm + a.mxo[L] + m * a.ldxm[L];
        float* ld = lg + a.kx[L];
        const int zm = a.z[m0 + m];
        const float wm = a.w[m0 + m];
        float mx = -INFINITY;
        for (int c = 0; c < C; ++c) mx = fmaxf(mx, lg[c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += expf(lg[c] - mx);
        const float lse = mx + logf(se);
        float pad = 0.f, nd = 0.f;
        for (int c = 0; c < C; ++c) pad += expf(lg[c] - lse) * ld[c];
        for (int c = 0; c < C; ++c) {
            const float p = expf(lg[c] - lse), ldc = ld[c];
            const float pmo = p - (c == zm ? 1.f : 0.f);
            nd = fmaf(pmo, ldc, nd);
            lg[c] = wm * pmo;
            ld[c] = wm * p * (ldc - pad);
        }
        if (a.nlld) a.nlld[(int64_t)s * a.M + m0 + m] = nd;
    }
    __syncthreads();
    ph(5);
    // ---- R-backward
    for (int l = L - 1; l >= 0; --l) {
        const int din = a.din[l], dout = a.dout[l], nw = din * dout, kxl = a.kx[l], kq = a.kx[l + 1];
        const float* Dl = sm + a.mxo[l + 1];  // [delta | delta_dot] rows
        const int ldd = a.ldxm[l + 1], ldx = a.ldxm[l];
        float* Xl = sm + a.mxo[l];
        const float* W2 = sm + a.mwo[l];
        const int64_t gslot = ((int64_t)blockIdx.y * a.S + s) * a.n_tot + a.woff[l];
        float* GW = a.G + gslot;
        float* GDW = a.Gd + gslot;
        // weight gradients: G[o][i] = sum_m delta[m][o] h[m][i],
        // G_dot[o][i] = sum_m delta[m][o] h_dot[m][i] + delta_dot[m][o] h[m][i]
        // (the ones column: column din is the bias gradient)
        const bool ones = din < kxl;
        auto wepi = [&](int pr, int q, floatx4 vx, floatx4 vy, int rot) __attribute__((always_inline)) {
            if (q > din || (q == din && !ones)) return;
            const int e0 = q < din ? q : nw, es = q < din ? din : 1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = pr + ((r + rot) & 3);
                if (o < dout) {
                    GW[o * es + e0] = vx[r];
                    GDW[o * es + e0] = vy[r];
                }
            }
        };
        const int K16 = (rc + 15) & ~15;
        rop_gemm<false, false, true, true, true>(dout, din + (ones ? 1 : 0), K16, 0, Dl, ldd, kq, Xl,
                                                       ldx, kxl, wepi);
        ph(1);
        // bias gradients without a ones column: column sums of delta / delta_dot, a wave per column
        if (!ones) {
            const int lane = tid & 63, nwv = nt >> 6;
            for (int o = wave_id(); o < dout; o += nwv) {  // wave-uniform
                float g = 0.f, gd = 0.f;
                for (int m = lane; m < rc; m += 64) {
                    g += Dl[m * ldd + o];
                    gd += Dl[m * ldd + kq + o];
                }
                g = wave_sum(g);
                gd = wave_sum(gd);
                if (lane == 0) {
                    GW[nw + o] = g;
                    GDW[nw + o] = gd;
                }
            }
        }
        ph(9);
        if (l > 0) {
            __syncthreads();  // the weight gradients have read X_l
            // delta' = (delta W) 1[h > 0], delta_dot' = (delta W_dot + delta_dot W) 1[h > 0]
            auto pepi = [&](int pr, int q, floatx4 vx, floatx4 vy, int rot) __attribute__((always_inline)) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = pr + ((r + rot) & 3);
                    if (m < rc) {
                        float* xr = Xl + m * ldx;
                        const bool on = xr[q] > 0.f;  // zero in the padding columns
                        xr[q] = on ? vx[r] : 0.f;
                        xr[kxl + q] = on ? vy[r] : 0.f;
                    }
                }
            };
            rop_gemm<true, false, true, true, true>(rc, din, kq, 0, Dl, ldd, kq, W2, a.ldwm[l], kxl, pepi);
            __syncthreads();
        } else if (a.du) {
            // d/du of (vec . grad): the input rows' delta_dot (no mask at the input)
            auto uepi = [&](int pr, int q, floatx4 vx, floatx4 vy, int rot) __attribute__((always_inline)) {
                if (q >= D) return;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = pr + ((r + rot) & 3);
                    if (m < rc) a.du[((int64_t)s * a.M + m0 + m) * D + q] = vy[r];
                }
            };
            rop_gemm<true, false, true, true, true>(rc, din, kq, 0, Dl, ldd, kq, W2, a.ldwm[0], kxl, uepi);
        }
        ph(6 + min(L - 1 - l, 2));
    }
    if (a.stamps && tid == 0) {
        unsigned long long* o = a.stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16;
        for (int q = 0; q < 10; ++q) o[q] = tph[q];
        o[15] = 1;
    }
}

// G += the other row blocks' slots, G_dot likewise, in slot order (slot 0
// holds the sum afterwards)
__global__ __launch_bounds__(256) void slot_sum_kernel(float* __restrict__ G, float* __restrict__ Gd,
                                                       int64_t n, int nsplit) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float g = G[i], gd = Gd[i];
    for (int k = 1; k < nsplit; ++k) {
        g += G[k * n + i];
        gd += Gd[k * n + i];
    }
    G[i] = g;
    Gd[i] = gd;
}

// Hv assembly.  The sums over the S samples run in parallel: a workgroup
// takes 64 consecutive elements (one per lane) and its sixteen waves a
// sixteenth of the samples each, in order; the partials are added in wave order
// (run-to-run bitwise reproducible).  Per parameter element e of layer l:
//   ge = sum_s G_s eps_s,  gd = sum_s G_dot_s,  gde = sum_s G_dot_s eps_s,
// then the softplus curvature ge sigmoid'(sd) v_sd and the KL Hessian (the
// corr block of full-cov is added by the update kernel's gradient mode, which
// also wrote sum G_dot, diag(G_dot^T E) sigmoid(sd) for full-cov).
constexpr int kAsmWaves = 16;  // 1024 threads: a C3 grid is 68 workgroups, so depth per CU matters
__device__ __forceinline__ void sample_quarter(int S, int wv, int& s0, int& s1) {
    const int q = (S + kAsmWaves - 1) / kAsmWaves;
    s0 = min(S, wv * q);
    s1 = min(S, s0 + q);
}

template <bool SLOTS, bool FC>
__device__ __forceinline__ void hvp_param_body(const RopArgs& a, float* hv, float inv_s0sq, float klw,
                                               int64_t slot2, int bx) {
    // SLOTS: G / G_dot still in the R-op's two row-block slots (slot 1 at
    // + slot2), added here as slot_sum_kernel would: slot 0 + slot 1.  FC:
    // full-cov needs sum_s G eps alone (the update kernel's gradient mode did G_dot)
    auto gl = [&](const float* P, int64_t i) __attribute__((always_inline)) {
        return SLOTS ? P[i] + P[slot2 + i] : P[i];
    };
    __shared__ float part[kAsmWaves][3][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int e = bx * 64 + lane;
    const bool live = e < a.n_tot;
    const int ec = live ? e : a.n_tot - 1;
    int l = 0;
    while (l + 1 < a.L && ec >= a.woff[l + 1]) ++l;
    const int n = a.din[l] * a.dout[l] + a.dout[l], k = ec - a.woff[l], nw = n - a.dout[l];
    // eps of sample s at ebase + s * es (mean-field weights and biases are
    // stored in separate [S][.] blocks)
    int64_t ebase;
    int es;
    if (a.family == PSVI_FAMILY_FULLCOV) {
        ebase = a.eoff[l] + k;
        es = n;
    } else if (k < nw) {
        ebase = a.eoff[l] + k;
        es = nw;
    } else {
        ebase = a.eoff[l] + (int64_t)a.S * nw + (k - nw);
        es = a.dout[l];
    }
    int s0, s1;
    sample_quarter(a.S, wv, s0, s1);
    float ge = 0.f, gd = 0.f, gde = 0.f;
    int s = s0;
    for (; s + 4 <= s1; s += 4) {  // four samples' loads in flight
        float g4[4], d4[4], e4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            g4[j] = gl(a.G, (int64_t)(s + j) * a.n_tot + ec);
            d4[j] = FC ? 0.f : gl(a.Gd, (int64_t)(s + j) * a.n_tot + ec);
            e4[j] = a.eps[ebase + (int64_t)(s + j) * es];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ge = fmaf(g4[j], e4[j], ge);
            gd += d4[j];
            gde = fmaf(d4[j], e4[j], gde);
        }
    }
    for (; s < s1; ++s) {
        const float g = gl(a.G, (int64_t)s * a.n_tot + ec), dv = FC ? 0.f : gl(a.Gd, (int64_t)s * a.n_tot + ec);
        const float ev = a.eps[ebase + (int64_t)s * es];
        ge = fmaf(g, ev, ge);
        gd += dv;
        gde = fmaf(dv, ev, gde);
    }
    part[wv][0][lane] = ge;
    part[wv][1][lane] = gd;
    part[wv][2][lane] = gde;
    __syncthreads();
    if (wv != 0 || !live) return;
    ge = gd = gde = 0.f;
#pragma unroll
    for (int w = 0; w < kAsmWaves; ++w) {
        ge += part[w][0][lane];
        gd += part[w][1][lane];
        gde += part[w][2][lane];
    }
    const float kls = klw * inv_s0sq;  // klw = 0: a sample shard's partial product without KL
    const int64_t pm = a.poff[l] + k, ps = pm + n;
    const float r = a.params[ps], sp = softplus_f(r), sg = sigmoid_f(r);
    const float vsd = a.vec[ps];
    const float kl2 = klw * ((1.f / (sp * sp) + inv_s0sq) * sg * sg + (sp * inv_s0sq - 1.f / sp) * sg * (1.f - sg));
    const float curv = ge * sg * (1.f - sg) * vsd + kl2 * vsd;
    if (a.family == PSVI_FAMILY_FULLCOV) {
        hv[pm] += a.vec[pm] * kls;
        hv[ps] += curv;
    } else {
        hv[pm] = gd + a.vec[pm] * kls;
        hv[ps] = gde * sg + curv;
    }
}

// dst[j] = sum_s src[s * stride + j], j < n: lanes over j, waves over sample
// quarters, partials in wave order (d_u = sum_s du_dot_s, d_w = sum_s NLL_dot_s)
__device__ __forceinline__ void sample_sum_body(const float* __restrict__ src, int64_t stride, int S,
                                                int64_t n, float* __restrict__ dst, int bx) {
    __shared__ float part[kAsmWaves][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)bx * 64 + lane, jc = j < n ? j : n - 1;
    int s0, s1;
    sample_quarter(S, wv, s0, s1);
    float t = 0.f;
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = src[(int64_t)(s + q) * stride + jc];
#pragma unroll
        for (int q = 0; q < 4; ++q) t += v[q];
    }
    for (; s < s1; ++s) t += src[(int64_t)s * stride + jc];
    part[wv][lane] = t;
    __syncthreads();
    if (wv != 0 || j >= n) return;
    t = 0.f;
#pragma unroll
    for (int w = 0; w < kAsmWaves; ++w) t += part[w][lane];
    dst[j] = t;
}

// The assembly and both mixed-product sums in one launch: workgroups
// [0, nbp) the parameter elements, then nbu of d_u, then the d_w ones (a
// workgroup-uniform branch; three launches before)
template <bool SLOTS, bool FC>
__global__ __launch_bounds__(1024) void hvp_assemble_kernel(RopArgs a, float* hv, float inv_s0sq, float klw,
                                                           int64_t slot2, int nbp, const float* du,
                                                           int64_t ndu, float* d_u, int nbu,
                                                           const float* nlld, float* d_w) {
    const int b = blockIdx.x;
    if (b < nbp)
        hvp_param_body<SLOTS, FC>(a, hv, inv_s0sq, klw, slot2, b);
    else if (b < nbp + nbu)
        sample_sum_body(du, ndu, a.S, ndu, d_u, b - nbp);
    else
        sample_sum_body(nlld, a.M, a.S, a.M, d_w, b - nbp - nbu);
}

static int rup4(int x) { return (x + 3) & ~3; }

// LDS carve for rows in chunks of rc; returns floats
static size_t rop_carve(const psvi_plan& p, int rc, RopArgs* a, bool with_g = true) {
    size_t off = 0;
    auto take = [&](size_t nfl) {
        const size_t o = off;
        off += (nfl + 3) & ~size_t(3);
        return (int)o;
    };
    int maxd = 0;
    for (int l = 0; l < p.L; ++l) maxd = std::max(maxd, std::max(p.lay[l].din, p.lay[l].dout));
    maxd = rup4(maxd) | 1;  // odd row stride of the delta buffers
    int xo[kMaxL], ldw[kMaxL], xtot = 0;
    for (int l = 0; l < p.L; ++l) {
        ldw[l] = p.lay[l].din | 1;
        xo[l] = xtot;
        xtot += p.lay[l].dout * ldw[l] + p.lay[l].dout;
    }
    const int lx = take(xtot), lxd = take(xtot);
    const int lg = with_g ? take(p.n_tot) : 0, lgd = with_g ? take(p.n_tot) : 0;
    int lh[kMaxL + 1], lhd[kMaxL + 1];
    for (int l = 0; l <= p.L; ++l) {
        const int d = l < p.L ? p.lay[l].din : p.lay[p.L - 1].dout;
        lh[l] = take((size_t)rc * d);
        lhd[l] = take((size_t)rc * d);
    }
    const int ld0 = take((size_t)rc * maxd), ld1 = take((size_t)rc * maxd);
    const int ldd0 = take((size_t)rc * maxd), ldd1 = take((size_t)rc * maxd);
    if (a) {
        a->lx = lx; a->lxd = lxd; a->lg = lg; a->lgd = lgd;
        for (int l = 0; l < p.L; ++l) { a->xo[l] = xo[l]; a->ldw[l] = ldw[l]; }
        for (int l = 0; l <= p.L; ++l) { a->lh[l] = lh[l]; a->lhd[l] = lhd[l]; }
        a->ld0 = ld0; a->ld1 = ld1; a->ldd0 = ldd0; a->ldd1 = ldd1;
        a->maxd = maxd;
        a->rc = rc;
    }
    return off;
}

// LDS carve of the MFMA form for a row block of `rows`; returns floats.  The
// activation regions come first, so a 16-row tile's over-read past a region's
// rows stays inside the allocation (tail slack when the weights after the last
// one are shorter than that).
static size_t rop_mfma_carve(const psvi_plan& p, int rows, RopArgs* a) {
    const int L = p.L;
    int kx[kMaxL + 1], mxo[kMaxL + 1], ldxm[kMaxL + 1], mwo[kMaxL], ldwm[kMaxL], mbo[kMaxL];
    for (int l = 0; l < L; ++l) kx[l] = (p.lay[l].din + 15) & ~15;
    kx[L] = (p.lay[L - 1].dout + 15) & ~15;
    size_t off = 0;
    for (int l = 0; l <= L; ++l) {
        ldxm[l] = 2 * kx[l] + 8;  // == 8 (mod 16); X_0's tangent half is zero
        mxo[l] = (int)off;
        off += (size_t)rows * ldxm[l];
    }
    const size_t x_end = off;
    for (int l = 0; l < L; ++l) {
        ldwm[l] = 2 * kx[l] + 8;
        mwo[l] = (int)off;
        off += (size_t)kx[l + 1] * ldwm[l];
    }
    for (int l = 0; l < L; ++l) {
        mbo[l] = (int)off;
        off += 2 * (size_t)kx[l + 1];
    }
    const size_t over = (size_t)(((rows + 15) & ~15) - rows) * ldxm[L];
    if (off - x_end < over) off = x_end + over;
    off = (off + 3) & ~size_t(3);
    const int lstamp = (int)off;
    off += 20;  // 10 uint64 phase clocks (diagnostics)
    if (a) {
        int j = 0;
        for (int l = 0; l < L; ++l) {
            a->jw[l] = j;
            j += kx[l + 1] * ((kx[l] + 63) >> 6);
        }
        a->jb = j;
        for (int l = 0; l < L; ++l) {
            a->jbl[l] = j - a->jb;
            j += (kx[l + 1] + 63) >> 6;
        }
        a->ju = j;
        a->lstamp = lstamp;
        for (int l = 0; l <= L; ++l) { a->kx[l] = kx[l]; a->mxo[l] = mxo[l]; a->ldxm[l] = ldxm[l]; }
        for (int l = 0; l < L; ++l) { a->mwo[l] = mwo[l]; a->ldwm[l] = ldwm[l]; a->mbo[l] = mbo[l]; }
    }
    return off;
}

constexpr size_t kRopLds = 160 * 1024;
// psvi_debug_set(PSVI_DBG_ROP_VALU, 1): the VALU R-op kernel (the form for
// row blocks past the LDS) on every shape (A/B)
int g_rop_valu = 0;

// rows per chunk that fit the LDS (0: the model's weights alone do not fit)
int rop_rows(const psvi_plan& p) {
    for (int rc = 64; rc >= 1; rc >>= 1)
        if (rop_carve(p, rc, nullptr) * 4 <= kRopLds) return rc;
    return 0;
}

// two workgroups per sample while the samples alone leave CUs idle
int rop_splits(const psvi_plan& p) { return (p.d.S < 256 && p.d.M > 1) ? 2 : 1; }

static void rop_fill(const psvi_plan& p, RopArgs& a) {
    a.L = p.L;
    a.M = p.d.M;
    a.S = p.d.S;
    a.n_tot = p.n_tot;
    a.family = p.family;
    for (int l = 0; l < p.L; ++l) {
        a.din[l] = p.lay[l].din;
        a.dout[l] = p.lay[l].dout;
        a.woff[l] = p.lay[l].woff;
        a.poff[l] = p.lay[l].poff;
        a.eoff[l] = p.lay[l].eoff;
    }
}

hipError_t launch_net_rop(const psvi_plan& p, const float* u, const int32_t* z, const float* w,
                          const float* x, const float* xd, const float* params, const float* vec,
                          const float* eps, float* G, float* Gd, float* du, float* nlld,
                          hipStream_t st, bool sum_slots) {
    static bool once = [] {
        (void)hipFuncSetAttribute((const void*)net_rop_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRopLds);
        for (const void* f : {(const void*)net_rop_mfma_kernel<false>,
                              (const void*)net_rop_mfma_kernel<true>})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRopLds);
        return true;
    }();
    (void)once;
    RopArgs a{};
    rop_fill(p, a);
    a.nsplit = rop_splits(p);
    {
        // the matrix-core form when a row block fits the LDS in one pass
        // rows padded to a 16-multiple: the rows past a block's own are zero
        // (the contraction over rows runs to the 16-multiple)
        const int rows = (((p.d.M + a.nsplit - 1) / a.nsplit) + 15) & ~15;
        const size_t lds = rop_mfma_carve(p, rows, &a) * 4;
        if (g_rop_valu != 1 && lds <= kRopLds) {
            a.u = u; a.z = z; a.w = w; a.x = x; a.xd = xd;
            a.params = params; a.vec = vec; a.eps = eps;
            a.G = G; a.Gd = Gd; a.du = du; a.nlld = nlld;
            a.stamps = g_rop_stamps;
            a.single = 1;
            const dim3 grid(p.d.S, a.nsplit), block(512);
            const bool fc = p.family == PSVI_FAMILY_FULLCOV;
            if (fc)
                hipLaunchKernelGGL((net_rop_mfma_kernel<true>), grid, block, lds, st, a);
            else
                hipLaunchKernelGGL((net_rop_mfma_kernel<false>), grid, block, lds, st, a);
            if (a.nsplit > 1 && sum_slots) {
                const int64_t n = (int64_t)p.d.S * p.n_tot;
                hipLaunchKernelGGL(slot_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                                   G, Gd, n, a.nsplit);
            }
            return hipGetLastError();
        }
    }
    // a workgroup's rows in one chunk when they fit without the LDS gradient
    // accumulators (C3: 50 rows, 146 KB): every phase then runs once per
    // workgroup instead of once per chunk
    const int rows_per = (p.d.M + a.nsplit - 1) / a.nsplit;
    const bool single = rop_carve(p, rows_per, nullptr, false) * 4 <= kRopLds;
    const int rc = single ? rows_per : rop_rows(p);
    if (rc == 0) return hipErrorInvalidValue;
    const size_t lds = rop_carve(p, rc, &a, !single) * 4;
    a.single = single ? 1 : 0;
    a.u = u; a.z = z; a.w = w; a.x = x; a.xd = xd;
    a.params = params; a.vec = vec; a.eps = eps;
    a.G = G; a.Gd = Gd; a.du = du; a.nlld = nlld;
    a.stamps = g_rop_stamps;
    hipLaunchKernelGGL(net_rop_kernel, dim3(p.d.S, a.nsplit), dim3(512), lds, st, a);
    if (a.nsplit > 1 && sum_slots) {
        const int64_t n = (int64_t)p.d.S * p.n_tot;
        hipLaunchKernelGGL(slot_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, G,
                           Gd, n, a.nsplit);
    }
    return hipGetLastError();
}

hipError_t launch_hvp_assemble(const psvi_plan& p, const float* params, const float* vec,
                               const float* eps, const float* G, const float* Gd, const float* du,
                               const float* nlld, float* hv, float* d_u, float* d_w,
                               hipStream_t st, bool include_kl, int64_t slot2) {
    RopArgs a{};
    rop_fill(p, a);
    a.params = params; a.vec = vec; a.eps = eps;
    a.G = const_cast<float*>(G);
    a.Gd = const_cast<float*>(Gd);
    const float s0 = p.d.prior_sd;
    const int nbp = (int)((p.n_tot + 63) / 64), M = p.d.M, D = p.lay[0].din;
    const int64_t ndu = (int64_t)M * D;
    const int nbu = d_u ? (int)((ndu + 63) / 64) : 0, nbw = d_w ? (M + 63) / 64 : 0;
    const dim3 pg((unsigned)(nbp + nbu + nbw)), pb(64 * kAsmWaves);
    const float is2 = 1.f / (s0 * s0), klw = include_kl ? 1.f : 0.f;
    const bool fc = p.family == PSVI_FAMILY_FULLCOV;
    if (slot2 && fc)
        hipLaunchKernelGGL((hvp_assemble_kernel<true, true>), pg, pb, 0, st, a, hv, is2, klw, slot2, nbp, du, ndu, d_u, nbu, nlld, d_w);
    else if (slot2)
        hipLaunchKernelGGL((hvp_assemble_kernel<true, false>), pg, pb, 0, st, a, hv, is2, klw, slot2, nbp, du, ndu, d_u, nbu, nlld, d_w);
    else if (fc)
        hipLaunchKernelGGL((hvp_assemble_kernel<false, true>), pg, pb, 0, st, a, hv, is2, klw, slot2, nbp, du, ndu, d_u, nbu, nlld, d_w);
    else
        hipLaunchKernelGGL((hvp_assemble_kernel<false, false>), pg, pb, 0, st, a, hv, is2, klw, slot2, nbp, du, ndu, d_u, nbu, nlld, d_w);
    return hipGetLastError();
}

}  // namespace psvi
