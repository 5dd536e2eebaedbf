// Register-resident GVP building blocks shared by the K5g message kernels (gmp_gvp.hip) and the
// node feed-forward kernels (gmp_gvp_ff.hip): one wave per 16-row chunk, lane l holding row
// i = l & 15 and feature group g = l >> 4 (features 16p + 4g + q, the v_mfma_f32_16x16x4_f32 B
// operand and C/D order, so chained Linears stay in registers); the xyz components of a vector
// channel sit in the same lane.
#pragma once

#include "gmp_common.h"

namespace gmp {
namespace gvpk {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// y[tile t] += sum_k W[16t + i][k] x[k]  over K = 16 * TI features (x in slot layout)
template <int TO, int TI>
__device__ __forceinline__ void gemm_wx(const float* __restrict__ sW, int ldw, const f32x4 (&x)[TI],
                                        f32x4 (&y)[TO], int i, int g) {
#pragma unroll
  for (int p = 0; p < TI; ++p) {
    f32x4 a[TO];
#pragma unroll
    for (int t = 0; t < TO; ++t) a[t] = *reinterpret_cast<const f32x4*>(sW + (16 * t + i) * ldw + 16 * p + 4 * g);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < TO; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][c], x[p][c], y[t], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// y[tile t] += sum_o W[o][16t + i] gin[o]   (W is (16 * TIN) x ldw, output 16 * TO features)
template <int TO, int TIN>
__device__ __forceinline__ void gemm_wtx(const float* __restrict__ sW, int ldw,
                                         const f32x4 (&gin)[TIN], f32x4 (&y)[TO], int i, int g) {
#pragma unroll
  for (int p = 0; p < TIN; ++p) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float* wrow = sW + (16 * p + 4 * g + c) * ldw + i;
      float a[TO];
#pragma unroll
      for (int t = 0; t < TO; ++t) a[t] = wrow[16 * t];
#pragma unroll
      for (int t = 0; t < TO; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], gin[p][c], y[t], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int T>
__device__ __forceinline__ void zero(f32x4 (&x)[T]) {
#pragma unroll
  for (int p = 0; p < T; ++p) x[p] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// scalar row (D features) of a row-major tensor: this lane's slots
template <int T>
__device__ __forceinline__ void ld_row(f32x4 (&x)[T], const float* __restrict__ row, int g) {
#pragma unroll
  for (int p = 0; p < T; ++p) x[p] = *reinterpret_cast<const f32x4*>(row + 16 * p + 4 * g);
}
template <int T>
__device__ __forceinline__ void st_row(float* __restrict__ row, const f32x4 (&x)[T], int g) {
#pragma unroll
  for (int p = 0; p < T; ++p) *reinterpret_cast<f32x4*>(row + 16 * p + 4 * g) = x[p];
}
template <int T>
__device__ __forceinline__ void add_row(f32x4 (&x)[T], const float* __restrict__ row, int g) {
#pragma unroll
  for (int p = 0; p < T; ++p) x[p] += *reinterpret_cast<const f32x4*>(row + 16 * p + 4 * g);
}
// LDS vector slots
template <int T>
__device__ __forceinline__ void ld_vec(f32x4 (&x)[T], const float* v, int g) {
#pragma unroll
  for (int p = 0; p < T; ++p) x[p] = *reinterpret_cast<const f32x4*>(v + 16 * p + 4 * g);
}

// vector row in the reference's (channel, xyz) layout, C = 16 * T channels:
// v[x][p][q] = row[(16p + 4g + q) * 3 + x]
template <int T>
__device__ __forceinline__ void ld_vrow(f32x4 (&v)[3][T], const float* __restrict__ row, int g) {
#pragma unroll
  for (int p = 0; p < T; ++p) {
    const f32x4* r4 = reinterpret_cast<const f32x4*>(row + (16 * p + 4 * g) * 3);
    const f32x4 a = r4[0], b = r4[1], c = r4[2];  // 12 floats: (q, x) q-major
    v[0][p] = f32x4{a[0], a[3], b[2], c[1]};
    v[1][p] = f32x4{a[1], b[0], b[3], c[2]};
    v[2][p] = f32x4{a[2], b[1], c[0], c[3]};
  }
}
template <int T>
__device__ __forceinline__ void st_vrow(float* __restrict__ row, const f32x4 (&v)[3][T], int g) {
#pragma unroll
  for (int p = 0; p < T; ++p) {
    f32x4* r4 = reinterpret_cast<f32x4*>(row + (16 * p + 4 * g) * 3);
    r4[0] = f32x4{v[0][p][0], v[1][p][0], v[2][p][0], v[0][p][1]};
    r4[1] = f32x4{v[1][p][1], v[2][p][1], v[0][p][2], v[1][p][2]};
    r4[2] = f32x4{v[2][p][2], v[0][p][3], v[1][p][3], v[2][p][3]};
  }
}

// norm over xyz with the reference's clamp (gvp_layer.py:66-73): sqrt(max(sum x^2, 1e-8))
template <int T>
__device__ __forceinline__ void vnorm(const f32x4 (&vh)[3][T], f32x4 (&vn)[T], f32x4 (&sq)[T]) {
#pragma unroll
  for (int p = 0; p < T; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float s2 = vh[0][p][q] * vh[0][p][q] + vh[1][p][q] * vh[1][p][q] + vh[2][p][q] * vh[2][p][q];
      sq[p][q] = s2;
      vn[p][q] = sqrtf(fmaxf(s2, 1e-8f));
    }
}

}  // namespace gvpk
}  // namespace gmp
