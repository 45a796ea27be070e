// mfma_tiles.hpp -- the v_mfma_f32_16x16x4_f32 operand helpers shared by the
// network kernel (kernels_net.hip) and the R-op kernel (kernels_rop.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace psvi {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- MFMA tile
// C[p][q] = sum_k A(p,k) B(q,k) for a 16-row tile and NQ 16-column tiles,
// k in groups of 16.
//   ACONT: A(p,k) = A[p*lda + k] (one float4 per lane and k-group), else
//          A(p,k) = A[k*lda + p] (four floats); BCONT likewise for B(q,k).
// Lane l = 16 k4 + i16 feeds row / column i16 and, to MFMA j of a k-group,
// k = kb + 4 k4 + j (the same k permutation on both operands), and holds
// D[p0 + 4 k4 + r][q0 + 16c + i16], r = 0..3 (v_mfma_f32_16x16x4_f32 layout):
// the epilogue gets (first row, column, the four rows' values).
// k order of a 16-wide k-group.  Lane-group k4 feeds MFMA j of the group
// with k = kperm(k4, j).  A k-contiguous operand reads one float4 per lane,
// so k = 4 k4 + j.  When both operands are k-strided the order is free, and
// k = (j & 1) + 4 (j >> 1) + 2 (k4 & 1) + 8 (k4 >> 1) puts the two
// lane-groups of a 32-lane half two rows apart: with row strides == 8 (mod 16)
// floats that is 16 banks, so their ds_read_b32 are conflict-free (4 k4 rows
// apart would be 0 banks mod 32: 2-way).
template <bool PERM>
__device__ __forceinline__ int kbase(int k4) { return PERM ? 2 * (k4 & 1) + 8 * (k4 >> 1) : 4 * k4; }
template <bool PERM>
__device__ __forceinline__ int kstep(int j) { return PERM ? (j & 1) + 4 * (j >> 1) : j; }

template <bool ACONT, bool BCONT, int NQ>
struct TileOps {
    static constexpr bool PERM = !ACONT && !BCONT;
    float4 a;
    float4 b[NQ];
    // k-contiguous: one float4 at p; k-strided: the rows kstep(0..3) below p
    __device__ __forceinline__ static float4 ld(const float* p, int ldx, bool cont) {
        if (cont) return *reinterpret_cast<const float4*>(p);
        return make_float4(p[kstep<PERM>(0) * ldx], p[kstep<PERM>(1) * ldx], p[kstep<PERM>(2) * ldx],
                           p[kstep<PERM>(3) * ldx]);
    }
    // pa / pb: this lane's first operand element of the k-group; column tile c
    // of B sits 16 c rows (BCONT) or 16 c columns further
    __device__ __forceinline__ void load(const float* pa, int lda, const float* pb, int ldb) {
        a = ld(pa, lda, ACONT);
#pragma unroll
        for (int c = 0; c < NQ; ++c) b[c] = ld(pb + 16 * c * (BCONT ? ldb : 1), ldb, BCONT);
    }
    // A's k >= K read as 0 (the last k-group of a row GEMM whose K is not a
    // 16-multiple: a k-contiguous A row runs past its end into the next row,
    // which another wave of the row chain may not have written yet -- LDS
    // left by an earlier kernel, possibly NaN, against zero weights)
    __device__ __forceinline__ void mask_a(int kb, int K) {
        const int k0 = kb + 4 * (int)((threadIdx.x & 63) >> 4);
        a.x = k0 < K ? a.x : 0.f;
        a.y = k0 + 1 < K ? a.y : 0.f;
        a.z = k0 + 2 < K ? a.z : 0.f;
        a.w = k0 + 3 < K ? a.w : 0.f;
    }
    __device__ __forceinline__ void mma(floatx4 (&acc)[NQ]) const {
#pragma unroll
        for (int c = 0; c < NQ; ++c) {
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[c].x, acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[c].y, acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[c].z, acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[c].w, acc[c], 0, 0, 0);
        }
    }
};

}  // namespace psvi
