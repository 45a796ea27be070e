// kernels_cg.hip -- the vector work of one conjugate-gradient iteration of
// hyper_step's CG_normaleq (psvi/hypergrad/CG_torch.py:9-45 over
// hypergradients.py:199-244's normal-equation operator), fused: three passes
// over the float64 vectors per iteration instead of the dozen ATen passes
// (and their fp32 <-> fp64 promotions) of the torch formulation.
//
// The operator A(p) = vmj - J vmj with vmj = lr H_A p and J y = y - lr H_B y
// (H_A at the fixed draw of w_mapped, H_B at a fresh draw per call) reads,
// per element, the two fp32 Hessian-vector products hv1 = H_A p and hv2 =
// H_B float(vmj):
//   vmj_i = lr * hv1_i (float64),  Ap_i = vmj_i - (vmj_i - lr * hv2_i).
// One iteration (state: rTr, then pAp, rnrn, the done flag, the step lengths):
//   cg_scale:    vmj32 = float(lr hv1)                 (H_B's input)
//   cg_pap:      pAp = sum_i p_i Ap_i                   (grid sum)
//   cg_residual: alpha = rTr / pAp; r <- r - alpha Ap; rnrn = sum r_i^2;
//                done |= sqrt(rnrn) < tol; the last block sets alpha_eff =
//                done ? 0 : alpha, beta = rnrn / rTr and, unless done, rTr =
//                rnrn
//   cg_update:   x <- x + alpha_eff p; unless done, p <- r + beta p; p32 =
//                float(p) (H_A's next input)
// Where the reference breaks (||r_new|| < tol), x keeps the previous iterate
// (alpha_eff = 0, selected, never multiplied by a non-finite alpha) and p
// freezes; r is then never read into x again, so it is updated in place.
// The grid sums are deterministic: each workgroup's fp64 partial goes to its
// slot with an sc1 store; after the storing wave's vmcnt drain one lane adds
// to the pass's counter (agent scope); the workgroup whose add returns the
// last count reads the slots with sc1 loads (MI355X_MICROARCH.md hand-off
// table, first row) and adds them in a fixed order, writes the scalars and
// resets the counter.
#include "psvi_internal.hpp"

namespace psvi {

constexpr int kCgThreads = 256;
constexpr int kCgBlocks = 1024;  // grid of the reductions (4 per CU)
// state (float64): [0] rTr, [1] pAp, [2] rnrn, [3] done (0 / 1), [4] alpha_eff,
// [5] beta, [6] alpha
enum { kRtr = 0, kPap = 1, kRnrn = 2, kDone = 3, kAeff = 4, kBeta = 5, kAlpha = 6 };

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// block sum in wave order (fixed: run-to-run bitwise), valid in thread 0
__device__ __forceinline__ double block_sum_d(double v, double* red) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kCgThreads / 64; ++i) t += red[i];
    return t;
}

// The grid sum's hand-off: thread 0 holds this block's partial.  Every thread
// calls it; returns true in thread 0 of the last-arriving block, with the
// total in *tot.  The last block reads the slots with all its threads (four
// loads per thread in flight, then the block sum in wave order: a fixed order,
// whichever block arrives last).
__device__ __forceinline__ bool grid_sum(double part, double* slots, unsigned* cnt, double* tot, double* red) {
    __shared__ unsigned last;
    if (threadIdx.x == 0) {
        __hip_atomic_store(slots + blockIdx.x, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return false;  // uniform
    static_assert(kCgBlocks <= 4 * kCgThreads, "four slots per thread");
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const unsigned b = threadIdx.x + i * kCgThreads;
        v[i] = b < gridDim.x ? __hip_atomic_load(slots + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    }
    const double t = block_sum_d((v[0] + v[1]) + (v[2] + v[3]), red);
    if (threadIdx.x == 0) {
        *tot = t;
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return threadIdx.x == 0;
}

__device__ __forceinline__ double cg_ap(float h1, float h2, double lr) {
    const double vmj = lr * (double)h1;
    return vmj - (vmj - lr * (double)h2);
}

__global__ __launch_bounds__(kCgThreads) void cg_scale_kernel(int64_t n, const float* __restrict__ hv,
                                                              double lr, float* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kCgThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kCgThreads)
        out[i] = (float)(lr * (double)hv[i]);
}

__global__ __launch_bounds__(kCgThreads) void cg_pap_kernel(int64_t n, const float* __restrict__ hv1,
                                                            const float* __restrict__ hv2, double lr,
                                                            const double* __restrict__ p,
                                                            double* state, double* slots,
                                                            unsigned* cnt) {
    __shared__ double red[kCgThreads / 64];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kCgThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kCgThreads)
        acc += p[i] * cg_ap(hv1[i], hv2[i], lr);
    const double part = block_sum_d(acc, red);
    double tot;
    __syncthreads();  // red reused by the grid sum
    if (grid_sum(part, slots, cnt, &tot, red)) state[kPap] = tot;
}

__global__ __launch_bounds__(kCgThreads) void cg_residual_kernel(int64_t n, const float* __restrict__ hv1,
                                                                 const float* __restrict__ hv2,
                                                                 double lr, double* __restrict__ r,
                                                                 double* state, double tol,
                                                                 double* slots, unsigned* cnt) {
    __shared__ double red[kCgThreads / 64];
    const double rtr = state[kRtr], alpha = rtr / state[kPap];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kCgThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kCgThreads) {
        const double rn = r[i] - alpha * cg_ap(hv1[i], hv2[i], lr);
        r[i] = rn;
        acc += rn * rn;
    }
    const double part = block_sum_d(acc, red);
    double rnrn;
    __syncthreads();  // red reused by the grid sum
    if (grid_sum(part, slots, cnt, &rnrn, red)) {
        // every block has read rTr and pAp: the scalars of the next pass
        const bool done = state[kDone] != 0.0 || sqrt(rnrn) < tol;
        state[kRnrn] = rnrn;
        state[kAlpha] = alpha;
        state[kAeff] = done ? 0.0 : alpha;
        state[kBeta] = rnrn / rtr;
        state[kDone] = done ? 1.0 : 0.0;
        if (!done) state[kRtr] = rnrn;
    }
}

__global__ __launch_bounds__(kCgThreads) void cg_update_kernel(int64_t n, double* __restrict__ x,
                                                               double* __restrict__ p,
                                                               float* __restrict__ p32,
                                                               const double* __restrict__ r,
                                                               const double* state) {
    const double aeff = state[kAeff], beta = state[kBeta];
    const bool done = state[kDone] != 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kCgThreads + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kCgThreads) {
        const double pi = p[i];
        x[i] += aeff * pi;
        if (!done) {
            const double pn = r[i] + beta * pi;
            p[i] = pn;
            p32[i] = (float)pn;
        }
    }
}

static int cg_blocks(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(kCgBlocks, (n + kCgThreads - 1) / kCgThreads));
}

size_t cg_ws_bytes() { return (size_t)kCgBlocks * sizeof(double) + 64; }

hipError_t launch_cg_scale(int64_t n, const float* hv, double lr, float* out, hipStream_t st) {
    hipLaunchKernelGGL(cg_scale_kernel, dim3(cg_blocks(n)), dim3(kCgThreads), 0, st, n, hv, lr, out);
    return hipGetLastError();
}

// ws: kCgBlocks partial slots, then the counter (zeroed by the caller once;
// every reduction leaves it at 0)
hipError_t launch_cg_pap(int64_t n, const float* hv1, const float* hv2, double lr, const double* p,
                         double* state, void* ws, hipStream_t st) {
    double* slots = static_cast<double*>(ws);
    unsigned* cnt = reinterpret_cast<unsigned*>(slots + kCgBlocks);
    hipLaunchKernelGGL(cg_pap_kernel, dim3(cg_blocks(n)), dim3(kCgThreads), 0, st, n, hv1, hv2, lr, p,
                       state, slots, cnt);
    return hipGetLastError();
}

hipError_t launch_cg_residual(int64_t n, const float* hv1, const float* hv2, double lr, double* r,
                              double* state, double tol, void* ws, hipStream_t st) {
    double* slots = static_cast<double*>(ws);
    unsigned* cnt = reinterpret_cast<unsigned*>(slots + kCgBlocks);
    hipLaunchKernelGGL(cg_residual_kernel, dim3(cg_blocks(n)), dim3(kCgThreads), 0, st, n, hv1, hv2,
                       lr, r, state, tol, slots, cnt);
    return hipGetLastError();
}

hipError_t launch_cg_update(int64_t n, double* x, double* p, float* p32, const double* r,
                            const double* state, hipStream_t st) {
    hipLaunchKernelGGL(cg_update_kernel, dim3(cg_blocks(n)), dim3(kCgThreads), 0, st, n, x, p, p32, r,
                       state);
    return hipGetLastError();
}

}  // namespace psvi
