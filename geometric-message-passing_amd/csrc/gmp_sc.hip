// K8: MACE symmetric contraction (models/mace_modules/symmetric_contraction.py:88-188,
// element_dependent=False) for node features x (B, C, 9) = C channels of 0e+1o+2e (reshape_irreps,
// irreps_tools.py:63-79), all three output irreps (0e, 1o, 2e; M = 1 + 3 + 5 = 9 rows) at once.
//
// With the per-channel coefficient tensors A_nu[c] = sum_k U_nu[..., k] W_nu[k, c] (prepared by
// the host), the reference's nested contraction ((A3 x + A2) x + A1) x is the polynomial
//   out[b, c, m] = sum_ijk A3[c, m, ijk] x_i x_j x_k + sum_ij A2[c, m, ij] x_i x_j
//                + sum_i A1[c, m, i] x_i          (x = x[b, c, :])
// written directly in the mul_ir output layout [0e: c | 1o: C + 3c + m' | 2e: 4C + 5c + m''].
// One thread per (node, channel) with the channel's A (819 x 9 floats, monomial-major) in LDS.
// Backward: dx by the product rule (same loop), dA = sum_b g[b,c,m] (monomial of x[b,c])
// reduced over node groups into per-group partials (summed in fixed order by the caller).
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kM = 9;                 // output rows (0e, 1o x3, 2e x5)
constexpr int kQ1 = 9, kQ2 = 81, kQ3 = 729;
constexpr int kQ = kQ1 + kQ2 + kQ3;   // monomials up to degree 3
constexpr int kSC = 256;

// LDS coefficient layout: a[q * 9 + m], q over [deg1 (9) | deg2 (81) | deg3 (729)]
__device__ __forceinline__ void load_coeffs(int c, int corr, const float* __restrict__ A1,
                                            const float* __restrict__ A2,
                                            const float* __restrict__ A3, float* a) {
  // A_nu global layout (C, 9, 9^nu): transpose to monomial-major in LDS
  for (int e = threadIdx.x; e < kM * kQ1; e += blockDim.x) {
    const int m = e / kQ1, q = e - m * kQ1;
    a[q * kM + m] = A1[((int64_t)c * kM + m) * kQ1 + q];
  }
  if (corr >= 2)
    for (int e = threadIdx.x; e < kM * kQ2; e += blockDim.x) {
      const int m = e / kQ2, q = e - m * kQ2;
      a[(kQ1 + q) * kM + m] = A2[((int64_t)c * kM + m) * kQ2 + q];
    }
  if (corr >= 3)
    for (int e = threadIdx.x; e < kM * kQ3; e += blockDim.x) {
      const int m = e / kQ3, q = e - m * kQ3;
      a[(kQ1 + kQ2 + q) * kM + m] = A3[((int64_t)c * kM + m) * kQ3 + q];
    }
}

__device__ __forceinline__ int out_col(int C, int c, int m) {
  return m == 0 ? c : (m < 4 ? C + 3 * c + (m - 1) : 4 * C + 5 * c + (m - 4));
}

template <int CORR>
__global__ __launch_bounds__(kSC) void sc_fwd_kernel(int64_t B, int C, const float* __restrict__ x,
                                                     const float* __restrict__ A1,
                                                     const float* __restrict__ A2,
                                                     const float* __restrict__ A3,
                                                     float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float a[];
  const int c = blockIdx.y;
  load_coeffs(c, CORR, A1, A2, A3, a);
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * kSC + threadIdx.x;
  if (b >= B) return;
  float xv[9];
  const float* xr = x + (b * C + c) * 9;
#pragma unroll
  for (int i = 0; i < 9; ++i) xv[i] = xr[i];
  float acc[kM];
#pragma unroll
  for (int m = 0; m < kM; ++m) acc[m] = 0.f;
  if (CORR >= 3) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const float xij = xv[i] * xv[j];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const float z = xij * xv[k];
          const float* ar = a + (kQ1 + kQ2 + (i * 9 + j) * 9 + k) * kM;
#pragma unroll
          for (int m = 0; m < kM; ++m) acc[m] += ar[m] * z;
        }
      }
  }
  if (CORR >= 2) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const float z = xv[i] * xv[j];
        const float* ar = a + (kQ1 + i * 9 + j) * kM;
#pragma unroll
        for (int m = 0; m < kM; ++m) acc[m] += ar[m] * z;
      }
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float* ar = a + i * kM;
#pragma unroll
    for (int m = 0; m < kM; ++m) acc[m] += ar[m] * xv[i];
  }
  float* orow = out + b * (int64_t)(9 * C);
#pragma unroll
  for (int m = 0; m < kM; ++m) orow[out_col(C, c, m)] = acc[m];
}

template <int CORR>
__global__ __launch_bounds__(kSC) void sc_bwd_x_kernel(int64_t B, int C,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ A1,
                                                       const float* __restrict__ A2,
                                                       const float* __restrict__ A3,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) float a[];
  const int c = blockIdx.y;
  load_coeffs(c, CORR, A1, A2, A3, a);
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * kSC + threadIdx.x;
  if (b >= B) return;
  float xv[9], g[kM], d[9];
  const float* xr = x + (b * C + c) * 9;
  const float* gr = gout + b * (int64_t)(9 * C);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    xv[i] = xr[i];
    d[i] = 0.f;
  }
#pragma unroll
  for (int m = 0; m < kM; ++m) g[m] = gr[out_col(C, c, m)];
  if (CORR >= 3) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const float xij = xv[i] * xv[j];
        float sk = 0.f;  // sum_k gA[ijk] x_k  (-> d_i x_j and d_j x_i terms)
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const float* ar = a + (kQ1 + kQ2 + (i * 9 + j) * 9 + k) * kM;
          float gA = 0.f;
#pragma unroll
          for (int m = 0; m < kM; ++m) gA += ar[m] * g[m];
          d[k] += gA * xij;
          sk += gA * xv[k];
        }
        d[i] += sk * xv[j];
        d[j] += sk * xv[i];
      }
  }
  if (CORR >= 2) {
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const float* ar = a + (kQ1 + i * 9 + j) * kM;
        float gA = 0.f;
#pragma unroll
        for (int m = 0; m < kM; ++m) gA += ar[m] * g[m];
        d[i] += gA * xv[j];
        d[j] += gA * xv[i];
      }
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float* ar = a + i * kM;
    float gA = 0.f;
#pragma unroll
    for (int m = 0; m < kM; ++m) gA += ar[m] * g[m];
    d[i] += gA;
  }
  float* dr = dx + (b * C + c) * 9;
#pragma unroll
  for (int i = 0; i < 9; ++i) dr[i] = d[i];
}

// dA partials: part[grp, c, m, q] = sum_{b in group grp} g[b, c, m] * mono_q(x[b, c])
// (q over deg1 | deg2 | deg3 as in the LDS layout; entries with q beyond the correlation are 0)
constexpr int kNodeBatch = 8;

template <int CORR>
__global__ __launch_bounds__(kSC) void sc_bwd_a_kernel(int64_t B, int C, int64_t nodes_per_group,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ part) {
  constexpr int NQ = CORR == 1 ? kQ1 : (CORR == 2 ? kQ1 + kQ2 : kQ);
  constexpr int NE = NQ * kM;                            // entries (q, m), m fastest
  constexpr int PER = (NE + kSC - 1) / kSC;
  __shared__ float zq[kNodeBatch][NQ];
  __shared__ float gm[kNodeBatch][kM];
  const int c = blockIdx.y;
  const int64_t grp = blockIdx.x;
  const int64_t b0 = grp * nodes_per_group;
  const int64_t b1 = (b0 + nodes_per_group < B) ? b0 + nodes_per_group : B;
  float acc[PER];
#pragma unroll
  for (int t = 0; t < PER; ++t) acc[t] = 0.f;
  for (int64_t bb = b0; bb < b1; bb += kNodeBatch) {
    const int nb = (int)((b1 - bb) < kNodeBatch ? (b1 - bb) : kNodeBatch);
    __syncthreads();
    for (int e = threadIdx.x; e < kNodeBatch * NQ; e += kSC) {
      const int n = e / NQ, q = e - n * NQ;
      float z = 0.f;
      if (n < nb) {
        const float* xr = x + ((bb + n) * C + c) * 9;
        if (q < kQ1) {
          z = xr[q];
        } else if (q < kQ1 + kQ2) {
          const int r = q - kQ1;
          z = xr[r / 9] * xr[r % 9];
        } else {
          const int r = q - kQ1 - kQ2;
          z = xr[r / 81] * xr[(r / 9) % 9] * xr[r % 9];
        }
      }
      zq[n][q] = z;
    }
    for (int e = threadIdx.x; e < kNodeBatch * kM; e += kSC) {
      const int n = e / kM, m = e - n * kM;
      gm[n][m] = (n < nb) ? gout[(bb + n) * (int64_t)(9 * C) + out_col(C, c, m)] : 0.f;
    }
    __syncthreads();
    for (int n = 0; n < kNodeBatch; ++n) {
#pragma unroll
      for (int t = 0; t < PER; ++t) {
        const int e = threadIdx.x + kSC * t;
        if (e < NE) acc[t] += zq[n][e / kM] * gm[n][e % kM];
      }
    }
  }
  float* pr = part + (grp * C + c) * (int64_t)(kM * kQ);
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int e = threadIdx.x + kSC * t;
    if (e < NE) {
      const int q = e / kM, m = e - q * kM;
      pr[m * kQ + q] = acc[t];
    }
  }
}

size_t coeff_smem(int corr) {
  const int nq = corr == 1 ? kQ1 : (corr == 2 ? kQ1 + kQ2 : kQ);
  return (size_t)nq * kM * sizeof(float);
}

template <class K>
int set_smem(K k, size_t bytes) {
  return hip_check(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)bytes));
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_sc_groups(int64_t n_nodes) {
  // node groups of the dA reduction: enough workgroups (x C channels) to fill the device
  int64_t g = ceil_div(n_nodes, 512);
  if (g > 64) g = 64;
  return (int)(g < 1 ? 1 : g);
}

int gmp_symmetric_contraction_fwd_f32(int64_t n_nodes, int channels, int correlation,
                                      const float* x, const float* A1, const float* A2,
                                      const float* A3, float* out, void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && channels > 0 && channels <= 65535);
  GMP_CHECK_ARG(correlation >= 1 && correlation <= 3);
  GMP_CHECK_ARG(x && A1 && out && (correlation < 2 || A2) && (correlation < 3 || A3));
  if (n_nodes == 0) return GMP_OK;
  const dim3 grid((unsigned)ceil_div(n_nodes, kSC), (unsigned)channels);
  const size_t smem = coeff_smem(correlation);
  hipStream_t s = as_stream(stream);
  int rc;
#define GMP_SC_FWD(CR)                                                                        \
  {                                                                                           \
    auto k = sc_fwd_kernel<CR>;                                                               \
    if ((rc = set_smem(k, smem))) return rc;                                                  \
    k<<<grid, kSC, smem, s>>>(n_nodes, channels, x, A1, A2, A3, out);                         \
  }
  if (correlation == 3) GMP_SC_FWD(3) else if (correlation == 2) GMP_SC_FWD(2) else GMP_SC_FWD(1)
#undef GMP_SC_FWD
  return launch_status();
}

int gmp_symmetric_contraction_bwd_f32(int64_t n_nodes, int channels, int correlation,
                                      const float* x, const float* A1, const float* A2,
                                      const float* A3, const float* gout, float* dx,
                                      float* dA_partials, void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && channels > 0 && channels <= 65535);
  GMP_CHECK_ARG(correlation >= 1 && correlation <= 3);
  GMP_CHECK_ARG(x && A1 && gout && (correlation < 2 || A2) && (correlation < 3 || A3));
  if (n_nodes == 0) return GMP_OK;
  hipStream_t s = as_stream(stream);
  int rc;
  if (dx) {
    const dim3 grid((unsigned)ceil_div(n_nodes, kSC), (unsigned)channels);
    const size_t smem = coeff_smem(correlation);
#define GMP_SC_BWDX(CR)                                                                       \
  {                                                                                           \
    auto k = sc_bwd_x_kernel<CR>;                                                             \
    if ((rc = set_smem(k, smem))) return rc;                                                  \
    k<<<grid, kSC, smem, s>>>(n_nodes, channels, x, A1, A2, A3, gout, dx);                    \
  }
    if (correlation == 3) GMP_SC_BWDX(3) else if (correlation == 2) GMP_SC_BWDX(2) else GMP_SC_BWDX(1)
#undef GMP_SC_BWDX
    if ((rc = launch_status())) return rc;
  }
  if (dA_partials) {
    const int G = gmp_sc_groups(n_nodes);
    const int64_t per = ceil_div(n_nodes, G);
    const dim3 grid((unsigned)G, (unsigned)channels);
    if (correlation == 3)
      sc_bwd_a_kernel<3><<<grid, kSC, 0, s>>>(n_nodes, channels, per, x, gout, dA_partials);
    else if (correlation == 2)
      sc_bwd_a_kernel<2><<<grid, kSC, 0, s>>>(n_nodes, channels, per, x, gout, dA_partials);
    else
      sc_bwd_a_kernel<1><<<grid, kSC, 0, s>>>(n_nodes, channels, per, x, gout, dA_partials);
    if ((rc = launch_status())) return rc;
  }
  return GMP_OK;
}

}  // extern "C"
