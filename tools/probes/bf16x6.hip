// Probe: fp32-faithful GEMM tiles on the bf16 matrix cores (three bf16 pieces
// per operand, six products) against v_mfma_f32_32x32x2_f32, for the two
// products of the streaming update's tile (kernels_mvn.hip mvn_stream_kernel):
//   dLT[c][r] = sum_s E[s][c] G[s][r]          (K = S = 128)
//   Y[s][r]   = sum_c E2[s][c] L[r][c]         (K = 64 columns; L = dLT, the
//                                                accumulator as the B operand)
// One workgroup of 4 waves (2 x 2 quadrants of 32 x 32), operands in LDS.
// Prints max error / sum |a b| against float64 for both paths and the
// shader clocks of each product (s_memtime), averaged over REPS repetitions.
//   hipcc --offload-arch=gfx950 -O3 bf16x6.hip -o bf16x6 && ./bf16x6
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef short bf8v __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int S = 128, NC = 64, REPS = 16;

__device__ __forceinline__ unsigned short bfbits(__bf16 x) { return __builtin_bit_cast(unsigned short, x); }
__device__ __forceinline__ float bf2f(unsigned short b) { return __uint_as_float((unsigned)b << 16); }

// a = a0 + a1 + a2, each bf16 (round to nearest even); exact for normal fp32
__device__ __forceinline__ void split3(float a, unsigned short& a0, unsigned short& a1, unsigned short& a2) {
    a0 = bfbits((__bf16)a);
    const float r1 = a - bf2f(a0);
    a1 = bfbits((__bf16)r1);
    const float r2 = r1 - bf2f(a1);
    a2 = bfbits((__bf16)r2);
}

__device__ __forceinline__ f16v mfma_bf(bf8v a, bf8v b, f16v c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// the six products, small terms first
__device__ __forceinline__ f16v mfma6(const bf8v (&a)[3], const bf8v (&b)[3], f16v c) {
    c = mfma_bf(a[2], b[0], c);
    c = mfma_bf(a[1], b[1], c);
    c = mfma_bf(a[0], b[2], c);
    c = mfma_bf(a[1], b[0], c);
    c = mfma_bf(a[0], b[1], c);
    c = mfma_bf(a[0], b[0], c);
    return c;
}

template <bool BF>
__global__ __launch_bounds__(256) void probe(const float* E, const float* G, const float* E2, float* dlt_f32,
                                             float* dlt_bf, float* y_f32, float* y_bf,
                                             unsigned long long* clk) {
    // fp32 images [s][64] for the f32 path (BF false); bf16 planes [3][c][s]
    // (E, G) and [3][s][c] (E2) for the bf16 path (BF true)
    constexpr int NF = BF ? 1 : S * NC, NP = BF ? 1 : 0;
    __shared__ float Ef[NF], Gf[NF], E2f[NF];
    __shared__ unsigned short Ep[3][BF ? NC : 1][S], Gp[3][BF ? NC : 1][S], E2p[3][BF ? S : 1][NC];
    (void)NP;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
    const int h = lane >> 5, l32 = lane & 31;
    for (int i = tid; i < S * NC; i += 256) {
        const int s = i / NC, c = i % NC;
        if constexpr (!BF) {
            Ef[i] = E[i];
            Gf[i] = G[i];
            E2f[i] = E2[i];
            continue;
        }
        unsigned short a0, a1, a2;
        split3(E[i], a0, a1, a2);
        Ep[0][c][s] = a0; Ep[1][c][s] = a1; Ep[2][c][s] = a2;
        split3(G[i], a0, a1, a2);
        Gp[0][c][s] = a0; Gp[1][c][s] = a1; Gp[2][c][s] = a2;
        split3(E2[i], a0, a1, a2);
        E2p[0][s][c] = a0; E2p[1][s][c] = a1; E2p[2][s][c] = a2;
    }
    __syncthreads();
    const int cq = 32 * wc + l32, rq = 32 * wr + l32;
    unsigned long long t0, t1, t2, t3, t4;
    f16v accf, accb, yf[4], yb[4];
    for (int rep = 0; rep < REPS; ++rep) {
        __syncthreads();
        t0 = __builtin_amdgcn_s_memtime();
        if constexpr (!BF) {
        // ---- f32: dLT quadrant, 64 MFMAs of K = 2
        for (int q = 0; q < 16; ++q) accf[q] = 0.f;
#pragma unroll
        for (int t = 0; t < S / 2; ++t)
            accf = __builtin_amdgcn_mfma_f32_32x32x2f32(Ef[(2 * t + h) * NC + cq], Gf[(2 * t + h) * NC + rq],
                                                        accf, 0, 0, 0);
        // keep the result live before the clock
        asm volatile("" ::"v"(accf[0]));
        }
        t1 = __builtin_amdgcn_s_memtime();
        if constexpr (BF) {
        // ---- bf16 x 6: 8 K-steps of 16 samples
        for (int q = 0; q < 16; ++q) accb[q] = 0.f;
#pragma unroll
        for (int t = 0; t < S / 16; ++t) {
            bf8v a[3], b[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                a[p] = *reinterpret_cast<const bf8v*>(&Ep[p][cq][16 * t + 8 * h]);
                b[p] = *reinterpret_cast<const bf8v*>(&Gp[p][rq][16 * t + 8 * h]);
            }
            accb = mfma6(a, b, accb);
        }
        asm volatile("" ::"v"(accb[0]));
        }
        t2 = __builtin_amdgcn_s_memtime();
        if constexpr (!BF) {
        // ---- Y = E2 L^T over this wave's 32 columns, 4 sample blocks: f32
        // (the accumulator as B: lane's L value for column c = 8g + 4h + e)
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            for (int q = 0; q < 16; ++q) yf[sb][q] = 0.f;
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int c = 32 * wc + 8 * g + 4 * h + e;
                    yf[sb] = __builtin_amdgcn_mfma_f32_32x32x2f32(E2f[(32 * sb + l32) * NC + c], accf[4 * g + e],
                                                                  yf[sb], 0, 0, 0);
                }
        }
        asm volatile("" ::"v"(yf[0][0]), "v"(yf[3][0]));
        }
        t3 = __builtin_amdgcn_s_memtime();
        if constexpr (BF) {
        // ---- bf16 x 6: split the accumulator (rows c of lane's column r)
        bf8v lb[2][3];
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                unsigned short a0, a1, a2;
                split3(accb[8 * st + j], a0, a1, a2);
                lb[st][0][j] = (short)a0;
                lb[st][1][j] = (short)a1;
                lb[st][2][j] = (short)a2;
            }
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            for (int q = 0; q < 16; ++q) yb[sb][q] = 0.f;
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                // element j of lane half h is row 16 st + 8 (j >> 2) + 4 h + (j & 3)
                bf8v a[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    const unsigned short* row = &E2p[p][32 * sb + l32][32 * wc + 16 * st + 4 * h];
                    typedef short s4 __attribute__((ext_vector_type(4)));
                    const s4 lo = *reinterpret_cast<const s4*>(row);
                    const s4 hi = *reinterpret_cast<const s4*>(row + 8);
                    a[p] = bf8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
                yb[sb] = mfma6(a, lb[st], yb[sb]);
            }
        }
        asm volatile("" ::"v"(yb[0][0]), "v"(yb[3][0]));
        }
        t4 = __builtin_amdgcn_s_memtime();
        if (tid == 0 && rep > 0) {
            clk[0] += t1 - t0;
            clk[1] += t2 - t1;
            clk[2] += t3 - t2;
            clk[3] += t4 - t3;
        }
    }
    // outputs: dLT[c][r], Y[s][r]
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
        if (!BF) dlt_f32[(32 * wc + row) * NC + rq] = accf[q];
        else dlt_bf[(32 * wc + row) * NC + rq] = accb[q];
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            // the two column halves add (wc = 0 / 1 each own 32 columns of the K)
            if (!BF) atomicAdd(&y_f32[(32 * sb + row) * NC + rq], yf[sb][q]);
            else atomicAdd(&y_bf[(32 * sb + row) * NC + rq], yb[sb][q]);
        }
    }
}

int main() {
    std::vector<float> E(S * NC), G(S * NC), E2(S * NC);
    srand(7);
    auto rn = []() {
        double u1 = (rand() + 1.0) / (RAND_MAX + 2.0), u2 = (rand() + 1.0) / (RAND_MAX + 2.0);
        return (float)(sqrt(-2 * log(u1)) * cos(6.283185307179586 * u2));
    };
    for (int i = 0; i < S * NC; ++i) {
        E[i] = rn();
        G[i] = 1e-3f * rn() * (float)exp(3.0 * rn());  // wide dynamic range
        E2[i] = rn();
    }
    float *dE, *dG, *dE2, *o[4];
    unsigned long long* dclk;
    hipMalloc(&dE, 4 * S * NC);
    hipMalloc(&dG, 4 * S * NC);
    hipMalloc(&dE2, 4 * S * NC);
    for (int i = 0; i < 4; ++i) {
        hipMalloc(&o[i], 4 * S * NC);
        hipMemset(o[i], 0, 4 * S * NC);
    }
    hipMalloc(&dclk, 8 * 4);
    hipMemset(dclk, 0, 32);
    hipMemcpy(dE, E.data(), 4 * S * NC, hipMemcpyHostToDevice);
    hipMemcpy(dG, G.data(), 4 * S * NC, hipMemcpyHostToDevice);
    hipMemcpy(dE2, E2.data(), 4 * S * NC, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe<false>, dim3(1), dim3(256), 0, 0, dE, dG, dE2, o[0], o[1], o[2], o[3], dclk);
    hipLaunchKernelGGL(probe<true>, dim3(1), dim3(256), 0, 0, dE, dG, dE2, o[0], o[1], o[2], o[3], dclk);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    std::vector<float> r[4];
    for (int i = 0; i < 4; ++i) {
        r[i].resize(S * NC);
        hipMemcpy(r[i].data(), o[i], 4 * S * NC, hipMemcpyDeviceToHost);
    }
    unsigned long long clk[4];
    hipMemcpy(clk, dclk, 32, hipMemcpyDeviceToHost);
    // float64 references, errors relative to sum |a b| per element
    double ed_f = 0, ed_b = 0, ey_f = 0, ey_b = 0;
    std::vector<double> L(NC * NC);
    for (int c = 0; c < NC; ++c)
        for (int rr = 0; rr < NC; ++rr) {
            double s = 0, sa = 0;
            for (int k = 0; k < S; ++k) {
                s += (double)E[k * NC + c] * G[k * NC + rr];
                sa += fabs((double)E[k * NC + c] * G[k * NC + rr]);
            }
            L[c * NC + rr] = s;
            ed_f = fmax(ed_f, fabs(r[0][c * NC + rr] - s) / sa);
            ed_b = fmax(ed_b, fabs(r[1][c * NC + rr] - s) / sa);
        }
    // Y from the kernel's own dLT (f32 path uses its f32 dLT, bf path its bf dLT)
    for (int s = 0; s < S; ++s)
        for (int rr = 0; rr < NC; ++rr) {
            double yf = 0, yb = 0, sa = 0;
            for (int c = 0; c < NC; ++c) {
                yf += (double)E2[s * NC + c] * r[0][c * NC + rr];
                yb += (double)E2[s * NC + c] * r[1][c * NC + rr];
                sa += fabs((double)E2[s * NC + c] * r[1][c * NC + rr]);
            }
            ey_f = fmax(ey_f, fabs(r[2][s * NC + rr] - yf) / sa);
            ey_b = fmax(ey_b, fabs(r[3][s * NC + rr] - yb) / sa);
        }
    printf("dLT  max err / sum|ab|: f32 %.3e  bf16x6 %.3e\n", ed_f, ed_b);
    printf("Y    max err / sum|ab|: f32 %.3e  bf16x6 %.3e\n", ey_f, ey_b);
    const double n = REPS - 1;
    printf("clocks per product (one wave): dLT f32 %.0f  bf16x6 %.0f | Y f32 %.0f  bf16x6 %.0f\n",
           clk[0] / n, clk[1] / n, clk[2] / n, clk[3] / n);
    return 0;
}
