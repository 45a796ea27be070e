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
// takes 64 consecutive elements (one per lane) and its four waves a quarter
// of the samples each, in order; the four partials are added in wave order
// (run-to-run bitwise reproducible).  Per parameter element e of layer l:
//   ge = sum_s G_s eps_s,  gd = sum_s G_dot_s,  gde = sum_s G_dot_s eps_s,
// then the softplus curvature ge sigmoid'(sd) v_sd and the KL Hessian (the
// corr block of full-cov is added by the update kernel's gradient mode, which
// also wrote sum G_dot, diag(G_dot^T E) sigmoid(sd) for full-cov).
constexpr int kAsmWaves = 4;
__device__ __forceinline__ void sample_quarter(int S, int wv, int& s0, int& s1) {
    const int q = (S + kAsmWaves - 1) / kAsmWaves;
    s0 = min(S, wv * q);
    s1 = min(S, s0 + q);
}

__global__ __launch_bounds__(256) void hvp_param_kernel(RopArgs a, float* hv, float inv_s0sq,
                                                        float klw) {
    __shared__ float part[kAsmWaves][3][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + lane;
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
            g4[j] = a.G[(int64_t)(s + j) * a.n_tot + ec];
            d4[j] = a.Gd[(int64_t)(s + j) * a.n_tot + ec];
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
        const float g = a.G[(int64_t)s * a.n_tot + ec], dv = a.Gd[(int64_t)s * a.n_tot + ec];
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
__global__ __launch_bounds__(256) void sample_sum_kernel(const float* __restrict__ src,
                                                         int64_t stride, int S, int64_t n,
                                                         float* __restrict__ dst) {
    __shared__ float part[kAsmWaves][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t j = (int64_t)blockIdx.x * 64 + lane, jc = j < n ? j : n - 1;
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

constexpr size_t kRopLds = 160 * 1024;

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
                          hipStream_t st) {
    static bool once = [] {
        (void)hipFuncSetAttribute((const void*)net_rop_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kRopLds);
        return true;
    }();
    (void)once;
    RopArgs a{};
    rop_fill(p, a);
    a.nsplit = rop_splits(p);
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
    if (a.nsplit > 1) {
        const int64_t n = (int64_t)p.d.S * p.n_tot;
        hipLaunchKernelGGL(slot_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, G,
                           Gd, n, a.nsplit);
    }
    return hipGetLastError();
}

hipError_t launch_hvp_assemble(const psvi_plan& p, const float* params, const float* vec,
                               const float* eps, const float* G, const float* Gd, const float* du,
                               const float* nlld, float* hv, float* d_u, float* d_w,
                               hipStream_t st, bool include_kl) {
    RopArgs a{};
    rop_fill(p, a);
    a.params = params; a.vec = vec; a.eps = eps;
    a.G = const_cast<float*>(G);
    a.Gd = const_cast<float*>(Gd);
    const float s0 = p.d.prior_sd;
    hipLaunchKernelGGL(hvp_param_kernel, dim3((unsigned)((p.n_tot + 63) / 64)), dim3(256), 0, st,
                       a, hv, 1.f / (s0 * s0), include_kl ? 1.f : 0.f);
    const int S = p.d.S, M = p.d.M, D = p.lay[0].din;
    if (d_u) {
        const int64_t n = (int64_t)M * D;
        hipLaunchKernelGGL(sample_sum_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, du,
                           n, S, n, d_u);
    }
    if (d_w)
        hipLaunchKernelGGL(sample_sum_kernel, dim3((unsigned)((M + 63) / 64)), dim3(256), 0, st,
                           nlld, (int64_t)M, S, (int64_t)M, d_w);
    return hipGetLastError();
}

}  // namespace psvi
