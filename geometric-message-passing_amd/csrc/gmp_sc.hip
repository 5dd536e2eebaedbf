// K8: MACE symmetric contraction (models/mace_modules/symmetric_contraction.py:88-188,
// element_dependent=False) for node features x (B, C, D) = C channels of 0e+1o(+2e(+3o)) --
// D = (L+1)^2 for max_ell L = 1, 2, 3 (reshape_irreps, irreps_tools.py:63-79) -- all L+1 output
// irreps (M = D rows) at once.
//
// With the per-channel coefficient tensors A_nu[c] = sum_k U_nu[..., k] W_nu[k, c] (prepared by
// the host), the reference's nested contraction (((A4 x + A3) x + A2) x + A1) x is the polynomial
//   out[b, c, m] = sum_{nu <= corr} sum_{i1..inu} A_nu[c, m, i1..inu] x_i1 ... x_inu
// (x = x[b, c, :]) written directly in the mul_ir output layout [0e: c | 1o: C + 3c + m' |
// 2e: 4C + 5c + m'' | 3o: 9C + 7c + m'''], evaluated over the symmetric monomial basis below
// (the caller passes the folded coefficients).  One thread per (node, channel), grid-stride over
// nodes, with the channel's coefficients (NQ x D floats, monomial-major) in LDS.  Backward: dx by
// the product rule (same loop), dA~ = sum_b g[b,c,m] (monomial of x[b,c]) reduced over node groups
// into per-group partials (summed in fixed order by the caller).
#include "gmp_common.h"

namespace gmp {
namespace {

// Symmetric monomial basis: x_i x_j x_k is symmetric in its indices, so the host folds every
// permutation's coefficient into the sorted one (A~_nu[c, m, q] = sum over the distinct
// permutations of q of A_nu[c, m, .]; exact algebra, fp32 re-association only) and the
// contraction runs over C(D + nu - 1, nu) monomials of degree nu instead of D^nu (D = 9, nu = 3:
// 165 instead of 729).  Order: deg1 i | deg2 i <= j | deg3 i <= j <= k | deg4 i <= j <= k <= l,
// lexicographic within a degree.
__host__ __device__ constexpr int nq_deg(int D, int deg) {
  return deg == 1 ? D
       : deg == 2 ? D * (D + 1) / 2
       : deg == 3 ? D * (D + 1) * (D + 2) / 6
                  : D * (D + 1) * (D + 2) * (D + 3) / 24;
}
__host__ __device__ constexpr int nq_total(int D, int corr) {
  return (corr >= 1 ? nq_deg(D, 1) : 0) + (corr >= 2 ? nq_deg(D, 2) : 0) +
         (corr >= 3 ? nq_deg(D, 3) : 0) + (corr >= 4 ? nq_deg(D, 4) : 0);
}
constexpr int kSC = 256;
constexpr int kNodeBlocks = 16;  // node blocks per channel (grid-stride: coefficients load once)

// compiled (D, corr): D in {4, 9, 16}; corr <= 4 for D <= 9, <= 3 for D = 16 (the D = 16, nu = 4
// table, 4844 x 16 floats, exceeds LDS)
__host__ __device__ constexpr bool sc_supported(int D, int corr) {
  return corr >= 1 && ((D == 4 || D == 9) ? corr <= 4 : (D == 16 ? corr <= 3 : false));
}

// LDS coefficient layout: a[q * D + m] (monomial-major: one q's D rows are contiguous and every
// lane of the block reads the same address -> broadcast reads)
template <int D, int CORR>
__device__ __forceinline__ void load_coeffs(int c, const float* __restrict__ A1,
                                            const float* __restrict__ A2,
                                            const float* __restrict__ A3,
                                            const float* __restrict__ A4, float* a) {
  const float* As[4] = {A1, A2, A3, A4};
  int q0 = 0;
#pragma unroll
  for (int nu = 1; nu <= CORR; ++nu) {
    const int nqd = nq_deg(D, nu);
    const float* An = As[nu - 1];
    for (int e = threadIdx.x; e < D * nqd; e += blockDim.x) {
      const int m = e / nqd, q = e - m * nqd;
      a[(q0 + q) * D + m] = An[((int64_t)c * D + m) * nqd + q];
    }
    q0 += nqd;
  }
}

// output column of row m (irrep block l = floor(sqrt(m)), component m - l^2) of channel c
__device__ __forceinline__ int out_col(int C, int c, int m) {
  const int l = m >= 9 ? 3 : (m >= 4 ? 2 : (m >= 1 ? 1 : 0));
  return l * l * C + (2 * l + 1) * c + (m - l * l);
}

// The monomial walk: rolled loops over the basis in order, this thread's x (and dx) in a private
// LDS row.  (r04: a fully unrolled walk with x and dx in registers measured slower at the C4
// shape -- 1.75 / 3.80 ms against 1.05 / 3.03 ms forward / backward at 50k nodes x 128
// channels, scripts/mb_sc.py: 256 VGPRs and 404 B of scratch per lane in its backward -- and
// compiled for minutes at D = 16.)
template <int D, int CORR, class F>
__device__ __forceinline__ void for_monomials(const float* xv, F&& f) {
  int q = 0;
#pragma unroll 1
  for (int i = 0; i < D; ++i) f(q++, xv[i], i, 0, 0, 0, 1);
  if constexpr (CORR >= 2) {
#pragma unroll 1
    for (int i = 0; i < D; ++i)
#pragma unroll 1
      for (int j = i; j < D; ++j) f(q++, xv[i] * xv[j], i, j, 0, 0, 2);
  }
  if constexpr (CORR >= 3) {
#pragma unroll 1
    for (int i = 0; i < D; ++i)
#pragma unroll 1
      for (int j = i; j < D; ++j) {
        const float xij = xv[i] * xv[j];
#pragma unroll 1
        for (int k = j; k < D; ++k) f(q++, xij * xv[k], i, j, k, 0, 3);
      }
  }
  if constexpr (CORR >= 4) {
#pragma unroll 1
    for (int i = 0; i < D; ++i)
#pragma unroll 1
      for (int j = i; j < D; ++j) {
        const float xij = xv[i] * xv[j];
#pragma unroll 1
        for (int k = j; k < D; ++k) {
          const float xijk = xij * xv[k];
#pragma unroll 1
          for (int l = k; l < D; ++l) f(q++, xijk * xv[l], i, j, k, l, 4);
        }
      }
  }
}

template <int D, int CORR>
__global__ __launch_bounds__(kSC) void sc_fwd_kernel(int64_t B, int C,
                                                        const float* __restrict__ x,
                                                        const float* __restrict__ A1,
                                                        const float* __restrict__ A2,
                                                        const float* __restrict__ A3,
                                                        const float* __restrict__ A4,
                                                        float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float a[];
  float* xt = a + nq_total(D, CORR) * D + threadIdx.x * (D + 1);  // this thread's x row
  const int c = blockIdx.y;
  load_coeffs<D, CORR>(c, A1, A2, A3, A4, a);
  __syncthreads();
  for (int64_t b = (int64_t)blockIdx.x * kSC + threadIdx.x; b < B; b += (int64_t)gridDim.x * kSC) {
    const float* xr = x + (b * C + c) * D;
    for (int i = 0; i < D; ++i) xt[i] = xr[i];
    float acc[D];
#pragma unroll
    for (int m = 0; m < D; ++m) acc[m] = 0.f;
    for_monomials<D, CORR>(xt, [&](int q, float z, int, int, int, int, int) {
      const float* ar = a + q * D;
#pragma unroll
      for (int m = 0; m < D; ++m) acc[m] += ar[m] * z;
    });
    float* orow = out + b * (int64_t)(D * C);
#pragma unroll
    for (int m = 0; m < D; ++m) orow[out_col(C, c, m)] = acc[m];
  }
}

template <int D, int CORR>
__global__ __launch_bounds__(kSC) void sc_bwd_x_kernel(int64_t B, int C,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ A1,
                                                          const float* __restrict__ A2,
                                                          const float* __restrict__ A3,
                                                          const float* __restrict__ A4,
                                                          const float* __restrict__ gout,
                                                          float* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) float a[];
  float* xt = a + nq_total(D, CORR) * D + threadIdx.x * (2 * D + 1);  // x row | dx row
  float* dt = xt + D;
  const int c = blockIdx.y;
  load_coeffs<D, CORR>(c, A1, A2, A3, A4, a);
  __syncthreads();
  for (int64_t b = (int64_t)blockIdx.x * kSC + threadIdx.x; b < B; b += (int64_t)gridDim.x * kSC) {
    float g[D];
    const float* xr = x + (b * C + c) * D;
    const float* gr = gout + b * (int64_t)(D * C);
    for (int i = 0; i < D; ++i) {
      xt[i] = xr[i];
      dt[i] = 0.f;
    }
#pragma unroll
    for (int m = 0; m < D; ++m) g[m] = gr[out_col(C, c, m)];
    for_monomials<D, CORR>(xt, [&](int q, float, int i, int j, int k, int l, int deg) {
      const float* ar = a + q * D;
      float gA = 0.f;
#pragma unroll
      for (int m = 0; m < D; ++m) gA += ar[m] * g[m];
      if (deg == 1) {
        dt[i] += gA;
      } else if (deg == 2) {
        dt[i] += gA * xt[j];
        dt[j] += gA * xt[i];
      } else if (deg == 3) {
        dt[i] += gA * (xt[j] * xt[k]);
        dt[j] += gA * (xt[i] * xt[k]);
        dt[k] += gA * (xt[i] * xt[j]);
      } else {
        const float xij = xt[i] * xt[j], xkl = xt[k] * xt[l];
        dt[i] += gA * (xt[j] * xkl);
        dt[j] += gA * (xt[i] * xkl);
        dt[k] += gA * (xij * xt[l]);
        dt[l] += gA * (xij * xt[k]);
      }
    });
    float* dr = dx + (b * C + c) * D;
    for (int i = 0; i < D; ++i) dr[i] = dt[i];
  }
}

// factor indices of monomial q of degree deg (q counted within its degree, lexicographic)
__device__ __forceinline__ void decode_monomial(int D, int deg, int r, int (&f)[4]) {
  int lo = 0;
  for (int t = 0; t < deg; ++t) {
    // number of sorted (deg - t - 1)-tuples over [v, D) for each candidate first index v
    const int rest = deg - t - 1;
    int v = lo;
    while (true) {
      const int n = D - v;  // values available from v on
      int cnt = 1;          // C(n - 1 + rest, rest): sorted tuples starting with v
      for (int s = 1; s <= rest; ++s) cnt = cnt * (n - 1 + s) / s;
      if (r < cnt) break;
      r -= cnt;
      ++v;
    }
    f[t] = v;
    lo = v;
  }
}

// dA~ partials: part[grp, c, m, q] = sum_{b in group grp} g[b, c, m] * mono_q(x[b, c]).
// Thread t owns monomials t, t + kSC, ... (QPT of them) and all D rows m; nodes staged through
// LDS in batches, their x and g rows read as broadcasts.
constexpr int kNodeBatch = 32;

template <int D, int CORR>
__global__ __launch_bounds__(kSC) void sc_bwd_a_kernel(int64_t B, int C, int64_t nodes_per_group,
                                                       const float* __restrict__ x,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ part) {
  constexpr int NQ = nq_total(D, CORR);
  constexpr int QPT = (NQ + kSC - 1) / kSC;
  __shared__ float xs[kNodeBatch][D];
  __shared__ float gs[kNodeBatch][D];
  const int c = blockIdx.y;
  const int64_t grp = blockIdx.x;
  const int64_t b0 = grp * nodes_per_group;
  const int64_t b1 = (b0 + nodes_per_group < B) ? b0 + nodes_per_group : B;
  int fac[QPT][4], deg[QPT];
#pragma unroll
  for (int u = 0; u < QPT; ++u) {
    const int q = threadIdx.x + u * kSC;
    fac[u][0] = fac[u][1] = fac[u][2] = fac[u][3] = 0;
    deg[u] = 0;
    int r = q;
    for (int dg = 1; dg <= CORR && q < NQ; ++dg) {
      if (r < nq_deg(D, dg)) {
        deg[u] = dg;
        decode_monomial(D, dg, r, fac[u]);
        break;
      }
      r -= nq_deg(D, dg);
    }
  }
  float acc[QPT][D];
#pragma unroll
  for (int u = 0; u < QPT; ++u)
#pragma unroll
    for (int m = 0; m < D; ++m) acc[u][m] = 0.f;
  for (int64_t bb = b0; bb < b1; bb += kNodeBatch) {
    const int nb = (int)((b1 - bb) < kNodeBatch ? (b1 - bb) : kNodeBatch);
    __syncthreads();
    for (int e = threadIdx.x; e < kNodeBatch * D; e += kSC) {
      const int n = e / D, t = e - n * D;
      xs[n][t] = (n < nb) ? x[((bb + n) * C + c) * D + t] : 0.f;
      gs[n][t] = (n < nb) ? gout[(bb + n) * (int64_t)(D * C) + out_col(C, c, t)] : 0.f;
    }
    __syncthreads();
    for (int n = 0; n < nb; ++n) {
#pragma unroll
      for (int u = 0; u < QPT; ++u) {
        if (deg[u] == 0) continue;
        float z = xs[n][fac[u][0]];
        if (deg[u] >= 2) z *= xs[n][fac[u][1]];
        if (deg[u] >= 3) z *= xs[n][fac[u][2]];
        if (deg[u] >= 4) z *= xs[n][fac[u][3]];
#pragma unroll
        for (int m = 0; m < D; ++m) acc[u][m] += gs[n][m] * z;
      }
    }
  }
  float* pr = part + (grp * C + c) * (int64_t)(D * NQ);
#pragma unroll
  for (int u = 0; u < QPT; ++u) {
    const int q = threadIdx.x + u * kSC;
    if (q >= NQ) continue;
#pragma unroll
    for (int m = 0; m < D; ++m) pr[m * NQ + q] = acc[u][m];
  }
}

template <int D, int CORR>
int sc_launch(int64_t n_nodes, int channels, const float* x, const float* A1, const float* A2,
              const float* A3, const float* A4, float* out, const float* gout, float* dx,
              float* dA_partials, hipStream_t s) {
  constexpr int NQ = nq_total(D, CORR);
  const int smem_f = (NQ * D + kSC * (D + 1)) * 4;
  const int smem_b = (NQ * D + kSC * (2 * D + 1)) * 4;
  const dim3 grid((unsigned)std::min<int64_t>(ceil_div(n_nodes, kSC), kNodeBlocks),
                  (unsigned)channels);
  int rc;
  auto fwd_k = sc_fwd_kernel<D, CORR>;
  auto bwd_k = sc_bwd_x_kernel<D, CORR>;
  if (out) {
    if ((rc = hip_check(hipFuncSetAttribute((const void*)fwd_k,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, smem_f))))
      return rc;
    fwd_k<<<grid, kSC, smem_f, s>>>(n_nodes, channels, x, A1, A2, A3, A4, out);
    if ((rc = launch_status())) return rc;
  }
  if (dx) {
    if ((rc = hip_check(hipFuncSetAttribute((const void*)bwd_k,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, smem_b))))
      return rc;
    bwd_k<<<grid, kSC, smem_b, s>>>(n_nodes, channels, x, A1, A2, A3, A4, gout, dx);
    if ((rc = launch_status())) return rc;
  }
  if (dA_partials) {
    const int G = gmp_sc_groups(n_nodes);
    const int64_t per = ceil_div(n_nodes, (int64_t)G);
    sc_bwd_a_kernel<D, CORR><<<dim3((unsigned)G, (unsigned)channels), kSC, 0, s>>>(
        n_nodes, channels, per, x, gout, dA_partials);
    if ((rc = launch_status())) return rc;
  }
  return GMP_OK;
}

int sc_dispatch(int64_t n_nodes, int channels, int dim, int corr, const float* x,
                const float* A1, const float* A2, const float* A3, const float* A4, float* out,
                const float* gout, float* dx, float* dA_partials, hipStream_t s) {
#define LAUNCH_SC(DD, CR)                                                                     \
  if (dim == DD && corr == CR)                                                             \
    return sc_launch<DD, CR>(n_nodes, channels, x, A1, A2, A3, A4, out, gout, dx, dA_partials, s);
  LAUNCH_SC(9, 1) LAUNCH_SC(9, 2) LAUNCH_SC(9, 3) LAUNCH_SC(9, 4)
  LAUNCH_SC(4, 1) LAUNCH_SC(4, 2) LAUNCH_SC(4, 3) LAUNCH_SC(4, 4)
  LAUNCH_SC(16, 1) LAUNCH_SC(16, 2) LAUNCH_SC(16, 3)
#undef LAUNCH_SC
  return GMP_ERR_UNSUPPORTED;
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

int gmp_sc_monomials(int dim, int correlation) {
  return sc_supported(dim, correlation) ? nq_total(dim, correlation) : -1;
}

int gmp_symmetric_contraction_fwd_f32(int64_t n_nodes, int channels, int dim, int correlation,
                                      const float* x, const float* A1, const float* A2,
                                      const float* A3, const float* A4, float* out,
                                      void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && channels > 0 && channels <= 65535);
  if (!sc_supported(dim, correlation)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(x && A1 && out && (correlation < 2 || A2) && (correlation < 3 || A3) &&
                (correlation < 4 || A4));
  if (n_nodes == 0) return GMP_OK;
  return sc_dispatch(n_nodes, channels, dim, correlation, x, A1, A2, A3, A4, out, nullptr,
                     nullptr, nullptr, as_stream(stream));
}

int gmp_symmetric_contraction_bwd_f32(int64_t n_nodes, int channels, int dim, int correlation,
                                      const float* x, const float* A1, const float* A2,
                                      const float* A3, const float* A4, const float* gout,
                                      float* dx, float* dA_partials, void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && channels > 0 && channels <= 65535);
  if (!sc_supported(dim, correlation)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(x && A1 && gout && (correlation < 2 || A2) && (correlation < 3 || A3) &&
                (correlation < 4 || A4));
  if (n_nodes == 0) return GMP_OK;
  return sc_dispatch(n_nodes, channels, dim, correlation, x, A1, A2, A3, A4, nullptr, gout, dx,
                     dA_partials, as_stream(stream));
}

}  // extern "C"
