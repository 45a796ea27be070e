// Probe: per-CU vector-memory rate of dword vs dwordx4 buffer loads (aligned
// and 4-byte-misaligned) from an L2-resident 4 MiB buffer; 512 workgroups of
// 256 threads, each thread issues NL loads then sums them.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
template <int W, int MIS>
__global__ __launch_bounds__(256) void rate(const float* src, float* out, int nfl, int reps) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nfl * 4, 0x00020000);
    float acc = 0.f;
    const uint32_t base = (blockIdx.x * 64 * 1024 + threadIdx.x * 4 * W) % (nfl * 4 - 65536 * 4);
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t off = base + (k * 256 * W * 4) + MIS * 4 + r * 16384 * 4;
            if (W == 1) {
                acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off % (nfl * 4), 0, 0));
            } else {
                v4i v = __builtin_amdgcn_raw_buffer_load_b128(rs, off % (nfl * 4 - 64), 0, 0);
                acc += __builtin_bit_cast(float, v[0]) + __builtin_bit_cast(float, v[1]) +
                       __builtin_bit_cast(float, v[2]) + __builtin_bit_cast(float, v[3]);
            }
        }
    }
    if (acc == 123.f) out[threadIdx.x] = acc;
}
template <int W, int MIS>
void run(const char* nm, const float* d, float* o, int nfl) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int reps = 16, grid = 512;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rate<W, MIS>), dim3(grid), dim3(256), 0, 0, d, o, nfl, reps);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((rate<W, MIS>), dim3(grid), dim3(256), 0, 0, d, o, nfl, reps);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)grid * 256 * reps * 16 * 4 * W;
    const double insts = (double)grid * 4 * reps * 16;
    printf("%-28s %8.2f us  %8.1f GB/s  %6.2f ns per wave-instr per CU\n", nm, ms * 100,
           bytes / (ms / 10 * 1e-3) / 1e9, (ms / 10 * 1e6) / (insts / 256));
}
int main() {
    const int nfl = 1 << 20;
    float *d, *o;
    (void)hipMalloc(&d, nfl * 4); (void)hipMalloc(&o, 4096);
    (void)hipMemset(d, 0, nfl * 4);
    run<1, 0>("dword", d, o, nfl);
    run<4, 0>("dwordx4 aligned", d, o, nfl);
    run<4, 1>("dwordx4 +4B", d, o, nfl);
    run<4, 2>("dwordx4 +8B", d, o, nfl);
    return 0;
}
