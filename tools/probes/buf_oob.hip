// Probe: does a raw buffer load of 16 bytes that straddles num_records return
// the in-range dwords and zeros for the rest (per-dword range check)?
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* base, int nrec_floats, f32x4* out) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0,
                                                                  nrec_floats * 4, 0x00020000);
    const int t = threadIdx.x;  // start float offsets 0..15
    out[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, t * 4, 0, 0));
}

int main() {
    float h[32];
    for (int i = 0; i < 32; ++i) h[i] = 100.f + i;
    float* d;
    f32x4* o;
    hipMalloc(&d, sizeof h);
    hipMalloc(&o, 16 * sizeof(f32x4));
    hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(16), 0, 0, d, 10, o);
    f32x4 r[16];
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    for (int t = 6; t < 12; ++t)
        printf("start %2d: %g %g %g %g\n", t, r[t][0], r[t][1], r[t][2], r[t][3]);
    return 0;
}
