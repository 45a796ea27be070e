// Probe: v_mfma_f32_16x16x4_f32 throughput inside one 512-thread workgroup per
// CU (the network kernel's shape): (0) register-only chains, 3 accumulators;
// (1) the forward GEMM of C3 layer 0 (112 x 48 x 64, units of one 16-row tile
// x 3 column tiles) with float4 LDS operand reads; (2) = (1) plus the
// epilogue's LDS stores; (3) = (1) with 16x16 tiles dealt singly (NQ = 1).
// Prints device time per launch and median shader-clock ticks per workgroup.
#include <hip/hip_runtime.h>
#include "../../blackbox-coresets-vi_amd/csrc/kernels_net.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void probe(float* out, unsigned long long* ticks, int reps) {
    __shared__ __attribute__((aligned(16))) float A[112 * 68 + 64];
    __shared__ __attribute__((aligned(16))) float B[48 * 68 + 64];
    __shared__ __attribute__((aligned(16))) float C[112 * 52 + 64];
    const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, k4 = lane >> 4;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < 112 * 68; i += 512) A[i] = (float)(i % 7) * 0.01f;
    for (int i = tid; i < 48 * 68; i += 512) B[i] = (float)(i % 5) * 0.01f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    floatx4 acc[3];
    for (int c = 0; c < 3; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    float sink = 0.f;
    for (int r = 0; r < reps; ++r) {
        if (MODE == 0) {
            // 2 units per SIMD x 48 MFMAs: the forward layer's MFMA count on the busiest SIMD
            if (wid < 7) {
                float a = A[lane], b = B[lane];
#pragma unroll 4
                for (int k = 0; k < 16; ++k)
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
            }
        } else if (MODE == 1 || MODE == 2) {
            if (wid < 7) {
                const int p = wid * 16 + i16;
                float4 a0 = *reinterpret_cast<const float4*>(A + p * 68 + 4 * k4), a1;
                float4 b0[3], b1[3];
#pragma unroll
                for (int c = 0; c < 3; ++c) b0[c] = *reinterpret_cast<const float4*>(B + (16 * c + i16) * 68 + 4 * k4);
                for (int kb = 0; kb < 64; kb += 32) {
                    a1 = *reinterpret_cast<const float4*>(A + p * 68 + kb + 16 + 4 * k4);
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        b1[c] = *reinterpret_cast<const float4*>(B + (16 * c + i16) * 68 + kb + 16 + 4 * k4);
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0[c].x, acc[c], 0, 0, 0);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0[c].y, acc[c], 0, 0, 0);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0[c].z, acc[c], 0, 0, 0);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0[c].w, acc[c], 0, 0, 0);
                    }
                    const int kn = kb + 32 < 64 ? kb + 32 : kb;
                    a0 = *reinterpret_cast<const float4*>(A + p * 68 + kn + 4 * k4);
#pragma unroll
                    for (int c = 0; c < 3; ++c)
                        b0[c] = *reinterpret_cast<const float4*>(B + (16 * c + i16) * 68 + kn + 4 * k4);
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1[c].x, acc[c], 0, 0, 0);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1[c].y, acc[c], 0, 0, 0);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1[c].z, acc[c], 0, 0, 0);
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1[c].w, acc[c], 0, 0, 0);
                    }
                }
                if (MODE == 2) {
#pragma unroll
                    for (int c = 0; c < 3; ++c)
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            C[(wid * 16 + 4 * k4 + q) * 52 + 16 * c + i16] = fmaxf(acc[c][q], 0.f);
                    for (int c = 0; c < 3; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
                }
            }
        } else if (MODE == 4 || MODE == 5) {
            // the network kernel's own GEMM driver (MODE 5: without its epilogue stores)
            auto epi = [&](int m, int j, floatx4 v, int) {
                if (MODE == 4 && j < 48) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) C[(m + q) * 52 + j] = fmaxf(v[q] + B[j], 0.f);
                } else {
                    sink += v[0];
                }
            };
            psvi::mfma_gemm<true, true>(112, 40, 64, 0, A, 68, B, 68, epi);
        } else {
            // 21 single tiles round-robin over 8 waves
            for (int u = wid; u < 21; u += 8) {
                const int p = (u / 3) * 16 + i16, q = (u % 3) * 16 + i16;
                floatx4 t = floatx4{0.f, 0.f, 0.f, 0.f};
                float4 a0 = *reinterpret_cast<const float4*>(A + p * 68 + 4 * k4), a1;
                float4 b0 = *reinterpret_cast<const float4*>(B + q * 68 + 4 * k4), b1;
                for (int kb = 0; kb < 64; kb += 32) {
                    a1 = *reinterpret_cast<const float4*>(A + p * 68 + kb + 16 + 4 * k4);
                    b1 = *reinterpret_cast<const float4*>(B + q * 68 + kb + 16 + 4 * k4);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, t, 0, 0, 0);
                    const int kn = kb + 32 < 64 ? kb + 32 : kb;
                    a0 = *reinterpret_cast<const float4*>(A + p * 68 + kn + 4 * k4);
                    b0 = *reinterpret_cast<const float4*>(B + q * 68 + kn + 4 * k4);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, t, 0, 0, 0);
                }
                acc[0] += t;
            }
        }
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < 3; ++c) sink += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    if (sink == 1234.5f) out[tid] = sink;
    if (tid == 0) ticks[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* nm, float* o, unsigned long long* tk, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, o, tk, reps);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(512), 0, 0, o, tk, reps);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> h(256);
    hipMemcpy(h.data(), tk, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    printf("%-44s %8.2f us/launch  %8.0f ticks/rep (median WG)\n", nm, ms * 100, (double)h[128] / reps);
}

int main() {
    float* o;
    unsigned long long* tk;
    hipMalloc(&o, 4096);
    hipMalloc(&tk, 256 * 8);
    const int reps = 100;
    run<0>("register chains, 96 MFMA per busiest SIMD", o, tk, reps);
    run<1>("fwd0 GEMM, NQ=3, float4 LDS reads", o, tk, reps);
    run<2>("fwd0 GEMM, NQ=3, + LDS epilogue", o, tk, reps);
    run<3>("fwd0 GEMM, 21 single tiles", o, tk, reps);
    run<4>("kernels_net.hip mfma_gemm (+ epilogue)", o, tk, reps);
    run<5>("kernels_net.hip mfma_gemm (no stores)", o, tk, reps);
    printf("ideal: 96 MFMA x 32 cycles = 3072 cycles per rep on the busiest SIMD\n");
    return 0;
}
