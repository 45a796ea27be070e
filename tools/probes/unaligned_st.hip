// Probe: global float4 stores at 4-byte (not 16-byte) aligned addresses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void st(float* dst, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;   // lane i writes [4i+1, 4i+5)
    if (4 * i + 5 <= n) {
        float4 v = make_float4(4 * i + 1, 4 * i + 2, 4 * i + 3, 4 * i + 4);
        *reinterpret_cast<float4*>(dst + 4 * i + 1) = v;
    }
}
int main() {
    const int n = 4096;
    float* d;
    (void)hipMalloc(&d, n * 4);
    (void)hipMemset(d, 0, n * 4);
    hipLaunchKernelGGL(st, dim3(n / 4 / 256), dim3(256), 0, 0, d, n);
    std::vector<float> h(n);
    (void)hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int k = 1; k < n - 3; ++k) bad += h[k] != (float)k;
    printf("unaligned float4 stores: %d bad of %d\n", bad, n - 4);
    return bad ? 1 : 0;
}
