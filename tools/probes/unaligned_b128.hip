// Probe: raw buffer b128 loads at 4-byte (not 16-byte) aligned offsets, and
// global float4 loads through a 4-byte aligned pointer, on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void probe(const float* src, float* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, n * 4, 0x00020000);
    // lane i loads 4 floats starting at element i (offset 4*i bytes)
    v4i v = __builtin_amdgcn_raw_buffer_load_b128(rs, i * 4, 0, 0);
    const float4* p4 = reinterpret_cast<const float4*>(src + (i % (n - 4)));
    float4 w = *p4;
    out[8 * i + 0] = __builtin_bit_cast(float, v[0]);
    out[8 * i + 1] = __builtin_bit_cast(float, v[1]);
    out[8 * i + 2] = __builtin_bit_cast(float, v[2]);
    out[8 * i + 3] = __builtin_bit_cast(float, v[3]);
    out[8 * i + 4] = w.x; out[8 * i + 5] = w.y; out[8 * i + 6] = w.z; out[8 * i + 7] = w.w;
}
int main() {
    const int n = 4096, T = 1024;
    std::vector<float> h(n);
    for (int i = 0; i < n; ++i) h[i] = (float)i;
    float *d, *o;
    hipMalloc(&d, n * 4); hipMalloc(&o, T * 8 * 4);
    hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(T / 256), dim3(256), 0, 0, d, o, n);
    std::vector<float> r(T * 8);
    hipMemcpy(r.data(), o, T * 8 * 4, hipMemcpyDeviceToHost);
    int bad_b = 0, bad_g = 0;
    for (int i = 0; i < T; ++i)
        for (int k = 0; k < 4; ++k) {
            if (r[8 * i + k] != (float)(i + k)) ++bad_b;
            if (r[8 * i + 4 + k] != (float)(i % (n - 4) + k)) ++bad_g;
        }
    printf("unaligned b128 buffer loads: %d bad of %d; float4 global: %d bad\n", bad_b, 4 * T, bad_g);
    printf("sample lane 1: %g %g %g %g | lane 3 float4: %g %g %g %g\n", r[8], r[9], r[10], r[11],
           r[28], r[29], r[30], r[31]);
    return (bad_b || bad_g) ? 1 : 0;
}
