// K8: MACE symmetric contraction (models/mace_modules/symmetric_contraction.py:88-188,
// element_dependent=False) for node features x (B, C, 9) = C channels of 0e+1o+2e (reshape_irreps,
// irreps_tools.py:63-79), all three output irreps (0e, 1o, 2e; M = 1 + 3 + 5 = 9 rows) at once.
//
// With the per-channel coefficient tensors A_nu[c] = sum_k U_nu[..., k] W_nu[k, c] (prepared by
// the host), the reference's nested contraction ((A3 x + A2) x + A1) x is the polynomial
//   out[b, c, m] = sum_ijk A3[c, m, ijk] x_i x_j x_k + sum_ij A2[c, m, ij] x_i x_j
//                + sum_i A1[c, m, i] x_i          (x = x[b, c, :])
// written directly in the mul_ir output layout [0e: c | 1o: C + 3c + m' | 2e: 4C + 5c + m''].
// evaluated over the symmetric monomial basis below (the caller passes the folded coefficients).
// One thread per (node, channel) with the channel's coefficients (219 x 9 floats, monomial-major)
// in LDS.  Backward: dx by the product rule (same loop), dA~ = sum_b g[b,c,m] (monomial of
// x[b,c]) reduced over node groups into per-group partials (summed in fixed order by the caller).
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kM = 9;                 // output rows (0e, 1o x3, 2e x5)
// Symmetric monomial basis: x_i x_j x_k is symmetric in its indices, so the host folds every
// permutation's coefficient into the sorted one (A~_nu[c, m, q] = sum over the distinct
// permutations of q of A_nu[c, m, .]; exact algebra, fp32 re-association only) and the
// contraction runs over 9 + 45 + 165 = 219 monomials instead of 9 + 81 + 729 = 819 (3.7x
// fewer multiply-adds in all three kernels).  Order: deg1 i | deg2 i <= j | deg3 i <= j <= k,
// lexicographic.
constexpr int kQ1 = 9, kQ2 = 45, kQ3 = 165;
constexpr int kQ = kQ1 + kQ2 + kQ3;   // 219
constexpr int kSC = 256;

template <int CORR>
constexpr int nq() { return CORR == 1 ? kQ1 : (CORR == 2 ? kQ1 + kQ2 : kQ); }

// LDS coefficient layout: a[q * 9 + m] (monomial-major: one q's 9 rows are contiguous and every
// lane of the block reads the same address -> broadcast reads)
template <int CORR>
__device__ __forceinline__ void load_coeffs(int c, const float* __restrict__ A1,
                                            const float* __restrict__ A2,
                                            const float* __restrict__ A3, float* a) {
  for (int e = threadIdx.x; e < kM * kQ1; e += blockDim.x) {
    const int m = e / kQ1, q = e - m * kQ1;
    a[q * kM + m] = A1[((int64_t)c * kM + m) * kQ1 + q];
  }
  if (CORR >= 2)
    for (int e = threadIdx.x; e < kM * kQ2; e += blockDim.x) {
      const int m = e / kQ2, q = e - m * kQ2;
      a[(kQ1 + q) * kM + m] = A2[((int64_t)c * kM + m) * kQ2 + q];
    }
  if (CORR >= 3)
    for (int e = threadIdx.x; e < kM * kQ3; e += blockDim.x) {
      const int m = e / kQ3, q = e - m * kQ3;
      a[(kQ1 + kQ2 + q) * kM + m] = A3[((int64_t)c * kM + m) * kQ3 + q];
    }
}

__device__ __forceinline__ int out_col(int C, int c, int m) {
  return m == 0 ? c : (m < 4 ? C + 3 * c + (m - 1) : 4 * C + 5 * c + (m - 4));
}

// visit every monomial q (in basis order) with its factors: f(q, z, i, j, k, deg)
template <int CORR, class F>
__device__ __forceinline__ void for_monomials(const float (&xv)[9], F&& f) {
#pragma unroll
  for (int i = 0; i < 9; ++i) f(i, xv[i], i, 0, 0, 1);
  if (CORR >= 2) {
    int q = kQ1;
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = i; j < 9; ++j) {
        f(q, xv[i] * xv[j], i, j, 0, 2);
        ++q;
      }
  }
  if (CORR >= 3) {
    int q = kQ1 + kQ2;
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
      for (int j = i; j < 9; ++j) {
        const float xij = xv[i] * xv[j];
#pragma unroll
        for (int k = j; k < 9; ++k) {
          f(q, xij * xv[k], i, j, k, 3);
          ++q;
        }
      }
  }
}

template <int CORR>
__global__ __launch_bounds__(kSC) void sc_fwd_kernel(int64_t B, int C, const float* __restrict__ x,
                                                     const float* __restrict__ A1,
                                                     const float* __restrict__ A2,
                                                     const float* __restrict__ A3,
                                                     float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float a[kQ * kM];
  const int c = blockIdx.y;
  load_coeffs<CORR>(c, A1, A2, A3, a);
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
  for_monomials<CORR>(xv, [&](int q, float z, int, int, int, int) {
    const float* ar = a + q * kM;
#pragma unroll
    for (int m = 0; m < kM; ++m) acc[m] += ar[m] * z;
  });
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
  __shared__ __attribute__((aligned(16))) float a[kQ * kM];
  const int c = blockIdx.y;
  load_coeffs<CORR>(c, A1, A2, A3, a);
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
  // d/dx_t of (gA_q * x_i x_j x_k) = gA_q * (x_j x_k [t = i] + x_i x_k [t = j] + x_i x_j [t = k])
  // (repeated indices add up to the power rule)
  for_monomials<CORR>(xv, [&](int q, float, int i, int j, int k, int deg) {
    const float* ar = a + q * kM;
    float gA = 0.f;
#pragma unroll
    for (int m = 0; m < kM; ++m) gA += ar[m] * g[m];
    if (deg == 1) {
      d[i] += gA;
    } else if (deg == 2) {
      d[i] += gA * xv[j];
      d[j] += gA * xv[i];
    } else {
      d[i] += gA * (xv[j] * xv[k]);
      d[j] += gA * (xv[i] * xv[k]);
      d[k] += gA * (xv[i] * xv[j]);
    }
  });
  float* dr = dx + (b * C + c) * 9;
#pragma unroll
  for (int i = 0; i < 9; ++i) dr[i] = d[i];
}

// dA~ partials: part[grp, c, m, q] = sum_{b in group grp} g[b, c, m] * mono_q(x[b, c]).
// One thread per monomial q (its factor indices fixed) and all 9 rows m; nodes staged through
// LDS in batches, their x and g rows read as broadcasts.
constexpr int kNodeBatch = 32;

template <int CORR>
__global__ __launch_bounds__(kSC) void sc_bwd_a_kernel(int64_t B, int C, int64_t nodes_per_group,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ part) {
  constexpr int NQ = nq<CORR>();
  __shared__ float xs[kNodeBatch][9];
  __shared__ float gs[kNodeBatch][kM];
  const int c = blockIdx.y;
  const int64_t grp = blockIdx.x;
  const int64_t b0 = grp * nodes_per_group;
  const int64_t b1 = (b0 + nodes_per_group < B) ? b0 + nodes_per_group : B;
  // this thread's monomial (q < NQ): factor indices (i, j, k) and degree
  const int q = threadIdx.x;
  int fi = 0, fj = 0, fk = 0, deg = 0;
  if (q < kQ1) {
    fi = q; deg = 1;
  } else if (q < kQ1 + kQ2) {
    int r = q - kQ1, i = 0;
    while (r >= 9 - i) { r -= 9 - i; ++i; }
    fi = i; fj = i + r; deg = 2;
  } else if (q < kQ) {
    int r = q - kQ1 - kQ2, i = 0;
    while (r >= (9 - i) * (10 - i) / 2) { r -= (9 - i) * (10 - i) / 2; ++i; }
    int j = i;
    while (r >= 9 - j) { r -= 9 - j; ++j; }
    fi = i; fj = j; fk = j + r; deg = 3;
  }
  float acc[kM];
#pragma unroll
  for (int m = 0; m < kM; ++m) acc[m] = 0.f;
  for (int64_t bb = b0; bb < b1; bb += kNodeBatch) {
    const int nb = (int)((b1 - bb) < kNodeBatch ? (b1 - bb) : kNodeBatch);
    __syncthreads();
    for (int e = threadIdx.x; e < kNodeBatch * 9; e += kSC) {
      const int n = e / 9, t = e - n * 9;
      xs[n][t] = (n < nb) ? x[((bb + n) * C + c) * 9 + t] : 0.f;
      gs[n][t] = (n < nb) ? gout[(bb + n) * (int64_t)(9 * C) + out_col(C, c, t)] : 0.f;
    }
    __syncthreads();
    if (q < NQ) {
      for (int n = 0; n < nb; ++n) {
        float z = xs[n][fi];
        if (deg >= 2) z *= xs[n][fj];
        if (deg >= 3) z *= xs[n][fk];
#pragma unroll
        for (int m = 0; m < kM; ++m) acc[m] += gs[n][m] * z;
      }
    }
  }
  if (q < NQ) {
    float* pr = part + (grp * C + c) * (int64_t)(kM * NQ);
#pragma unroll
    for (int m = 0; m < kM; ++m) pr[m * NQ + q] = acc[m];
  }
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
  hipStream_t s = as_stream(stream);
#define GMP_SC_FWD(CR) \
  sc_fwd_kernel<CR><<<grid, kSC, 0, s>>>(n_nodes, channels, x, A1, A2, A3, out);
  if (correlation == 3) { GMP_SC_FWD(3) } else if (correlation == 2) { GMP_SC_FWD(2) } else { GMP_SC_FWD(1) }
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
#define GMP_SC_BWDX(CR) \
  sc_bwd_x_kernel<CR><<<grid, kSC, 0, s>>>(n_nodes, channels, x, A1, A2, A3, gout, dx);
    if (correlation == 3) { GMP_SC_BWDX(3) } else if (correlation == 2) { GMP_SC_BWDX(2) } else { GMP_SC_BWDX(1) }
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
