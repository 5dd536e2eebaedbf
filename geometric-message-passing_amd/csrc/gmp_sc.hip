// K8: MACE symmetric contraction (models/mace_modules/symmetric_contraction.py:20-188,
// element_dependent=False) for node features x (B, C, D) = C channels of ANY irreps list
// (reshape_irreps, irreps_tools.py:63-79: 0e+1o+2e, both parities, repeated l, max_ell up to 5 or
// more; D <= 63 components per channel) and any output irreps list of C channels each (M <= 255
// rows), correlation 1..4.
//
// With the per-channel coefficient tensors A_nu[c] = sum_k U_nu[..., k] W_nu[k, c] (built by the
// host, differentiably), the reference's nested contraction (((A4 x + A3) x + A2) x + A1) x is the
// polynomial
//   out[b, c, m] = sum_{nu <= corr} sum_{i1..inu} A_nu[c, m, i1..inu] x_i1 ... x_inu,
// x = x[b, c, :].  The monomials are symmetric in their indices, so the host folds every
// permutation's coefficient into the sorted index tuple, and the couplings that reach row m are
// sparse: real Clebsch-Gordan selection rules (parity, |l1 - l2| <= l <= l1 + l2, the m-selection
// of the real basis) and the antisymmetric couplings that vanish on symmetric monomials leave ~10 %
// of the (row, monomial) pairs non-zero (C4's 0e+1o+2e at correlation 3: 247 of 1,971;
// 0e+1o+2e+3o at correlation 4: 8,652 of 77,504).  The host keeps that pattern -- the TERM LIST,
// identical for every channel because the weights are dense -- and the kernels walk it:
//   term t = (row m_t, factors f0..f3 of its monomial; a factor index D addresses a constant 1.0
//   slot, so degree < 4 monomials need no branch), coefficient coef[c, t].
// Plan (int32, built once per module): [row_ptr (M + 1) | out_base (M) | out_stride (M) |
// terms (T)], terms of row m at row_ptr[m] .. row_ptr[m+1] - 1, sorted by monomial; term word =
// f0 | f1 << 6 | f2 << 12 | f3 << 18 | m << 24.  Output column of (row m, channel c):
// out_base[m] + out_stride[m] c (the mul_ir layout of the output irreps: block offset + (2l+1) c +
// component).
//
// Mapping: a workgroup owns a tile of CT channels (lane = channel fastest, 256 / CT nodes per
// pass, grid-stride over nodes); the coefficients are term-major (coef (T, C): a tile reads CT
// consecutive floats per term, from L1 / L2), term words are wave-uniform (scalar loads), each
// thread's x row (and dx row) sits in a private LDS row with an odd stride.  Lanes of one node
// read / write its CT channels' x, g and out entries -- runs of CT * (2l+1) floats per output
// block instead of one scattered float per lane.  dcoef[t, c] = sum_b g[b, c, m_t] mono_t(x[b, c])
// runs over (term, channel) pairs of a channel tile with the node group's x / g rows staged
// through LDS, reduced over node groups into per-group partials (summed in fixed order by the
// caller).  Deterministic: fixed orders throughout, no atomics.
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kSC = 256;
constexpr int kMaxDim = 63;     // factor fields are 6 bits; index D is the 1.0 slot
constexpr int kMaxRows = 255;   // row field is 8 bits
constexpr int kMaxCT = 16;      // channels per workgroup tile of the forward / dx kernels
constexpr int kQPT = 16;        // dcoef kernel: (term, channel) pairs per thread
constexpr int kPairs = kSC * kQPT;
constexpr int kStageLds = 16384; // floats of staged node rows in the dcoef kernel

struct Plan {
  const int* row_ptr;
  const int* out_base;
  const int* out_stride;
  const unsigned* terms;
};
__device__ __forceinline__ Plan plan_of(const int* p, int M) {
  return Plan{p, p + M + 1, p + 2 * M + 1, reinterpret_cast<const unsigned*>(p + 3 * M + 1)};
}

__host__ __device__ constexpr int row_stride(int D) { return (D + 1) | 1; }

__device__ __forceinline__ float mono(const float* xt, unsigned f) {
  return (xt[f & 63u] * xt[(f >> 6) & 63u]) * (xt[(f >> 12) & 63u] * xt[(f >> 18) & 63u]);
}

__device__ __forceinline__ void load_row(float* xt, const float* __restrict__ xr, int D) {
  for (int i = 0; i < D; ++i) xt[i] = xr[i];
  xt[D] = 1.f;
}

__global__ __launch_bounds__(kSC) void sc_fwd_kernel(int64_t B, int C, int D, int M, int T, int CT,
                                                        const int* __restrict__ plan,
                                                        const float* __restrict__ coef,
                                                        const float* __restrict__ x,
                                                        float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xt = sm + threadIdx.x * row_stride(D);
  const int cl = threadIdx.x % CT, npb = kSC / CT, c = blockIdx.y * CT + cl;
  if (threadIdx.x >= npb * CT || c >= C) return;  // (no barrier in this kernel)
  const Plan P = plan_of(plan, M);
  const float* cf = coef + c;  // coef[t, c] at cf[t C]: CT consecutive floats per term
  for (int64_t b = (int64_t)blockIdx.x * npb + threadIdx.x / CT; b < B;
       b += (int64_t)gridDim.x * npb) {
    load_row(xt, x + (b * C + c) * D, D);
    float* orow = out + b * (int64_t)M * C;
    int t = P.row_ptr[0];
    for (int m = 0; m < M; ++m) {
      const int t1 = P.row_ptr[m + 1];
      float acc = 0.f;
      for (; t < t1; ++t) acc = fmaf(cf[(int64_t)t * C], mono(xt, P.terms[t]), acc);
      orow[P.out_base[m] + P.out_stride[m] * c] = acc;
    }
  }
}

__global__ __launch_bounds__(kSC) void sc_bwd_x_kernel(int64_t B, int C, int D, int M, int T,
                                                          int CT, const int* __restrict__ plan,
                                                          const float* __restrict__ coef,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ gout,
                                                          float* __restrict__ dx) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int RS = row_stride(D);
  float* xt = sm + threadIdx.x * RS;
  float* dt = sm + kSC * RS + threadIdx.x * RS;
  const int cl = threadIdx.x % CT, npb = kSC / CT, c = blockIdx.y * CT + cl;
  if (threadIdx.x >= npb * CT || c >= C) return;  // (no barrier in this kernel)
  const Plan P = plan_of(plan, M);
  const float* cf = coef + c;
  for (int64_t b = (int64_t)blockIdx.x * npb + threadIdx.x / CT; b < B;
       b += (int64_t)gridDim.x * npb) {
    load_row(xt, x + (b * C + c) * D, D);
    for (int i = 0; i <= D; ++i) dt[i] = 0.f;
    const float* grow = gout + b * (int64_t)M * C;
    int t = P.row_ptr[0];
    for (int m = 0; m < M; ++m) {
      const int t1 = P.row_ptr[m + 1];
      const float gm = grow[P.out_base[m] + P.out_stride[m] * c];
      for (; t < t1; ++t) {
        // d/dx of x_f0 x_f1 x_f2 x_f3: one product-rule term per factor (a repeated factor gets
        // each of its terms; the 1.0 slot D collects the padding factors' terms, unused)
        const unsigned f = P.terms[t];
        const unsigned i0 = f & 63u, i1 = (f >> 6) & 63u, i2 = (f >> 12) & 63u, i3 = (f >> 18) & 63u;
        const float a = xt[i0], bb = xt[i1], cc = xt[i2], d = xt[i3];
        const float w = gm * cf[(int64_t)t * C], ab = a * bb, cd = cc * d;
        dt[i0] = fmaf(w, bb * cd, dt[i0]);
        dt[i1] = fmaf(w, a * cd, dt[i1]);
        dt[i2] = fmaf(w, ab * d, dt[i2]);
        dt[i3] = fmaf(w, ab * cc, dt[i3]);
      }
    }
    float* dr = dx + (b * C + c) * D;
    for (int i = 0; i < D; ++i) dr[i] = dt[i];
  }
}

// dcoef partials: part[grp, t, c] = sum_{b in group grp} g[b, c, m_t] mono_t(x[b, c]).  A
// workgroup owns a node group (blockIdx.x), a channel tile of CT channels (blockIdx.y) and a
// range of <= kPairs / CT terms (blockIdx.z); thread pair p = tid + 256 u is (term t0 + p / CT,
// channel p % CT).  The group's nodes are staged through LDS NB at a time: x rows (+ the 1.0
// slot) and g rows of the tile's channels.
__global__ __launch_bounds__(kSC) void sc_bwd_coef_kernel(int64_t B, int C, int D, int M, int T,
                                                             int CT, int NB,
                                                             int64_t nodes_per_group,
                                                             const int* __restrict__ plan,
                                                             const float* __restrict__ x,
                                                             const float* __restrict__ gout,
                                                             float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xsb = sm;                          // [NB][CT][D + 1]
  float* gsb = sm + NB * CT * (D + 1);      // [NB][CT][M]
  const int c0 = blockIdx.y * CT;
  const int64_t grp = blockIdx.x;
  const int tpb = kPairs / CT;              // terms per workgroup
  const int t0 = blockIdx.z * tpb;
  const int nt = min(tpb, T - t0);
  const Plan P = plan_of(plan, M);
  const int64_t b0 = grp * nodes_per_group;
  const int64_t b1 = (b0 + nodes_per_group < B) ? b0 + nodes_per_group : B;
  const int rounds = (nt * CT + kSC - 1) / kSC;  // uniform, <= kQPT
  unsigned f[kQPT];
  int xo[kQPT], go[kQPT];
  float acc[kQPT];
#pragma unroll
  for (int u = 0; u < kQPT; ++u) {
    const int p = threadIdx.x + u * kSC, tl = p / CT, j = p - tl * CT;
    const bool ok = u < rounds && tl < nt && c0 + j < C;
    f[u] = ok ? P.terms[t0 + tl] : 0xffffffffu;
    xo[u] = j * (D + 1);
    go[u] = ok ? j * M + (int)(f[u] >> 24) : 0;
    acc[u] = 0.f;
  }
  for (int64_t bb = b0; bb < b1; bb += NB) {
    const int nb = (int)((b1 - bb) < NB ? (b1 - bb) : NB);
    __syncthreads();
    for (int e = threadIdx.x; e < NB * CT * (D + 1); e += kSC) {
      const int i = e % (D + 1), r = e / (D + 1), j = r % CT, n = r / CT;
      xsb[e] = (n < nb && i < D && c0 + j < C) ? x[((bb + n) * C + c0 + j) * D + i] : 1.f;
    }
    for (int e = threadIdx.x; e < NB * CT * M; e += kSC) {
      const int j = e % CT, r = e / CT, m = r % M, n = r / M;
      gsb[(n * CT + j) * M + m] =
          (n < nb && c0 + j < C)
              ? gout[(bb + n) * (int64_t)M * C + P.out_base[m] + P.out_stride[m] * (c0 + j)]
              : 0.f;
    }
    __syncthreads();
    for (int n = 0; n < nb; ++n) {
      const float* xr = xsb + n * CT * (D + 1);
      const float* gr = gsb + n * CT * M;
#pragma unroll
      for (int u = 0; u < kQPT; ++u) {
        if (u < rounds && f[u] != 0xffffffffu)
          acc[u] = fmaf(gr[go[u]], mono(xr + xo[u], f[u]), acc[u]);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < kQPT; ++u) {
    const int p = threadIdx.x + u * kSC, tl = p / CT, j = p - tl * CT;
    if (u < rounds && tl < nt && c0 + j < C) part[(grp * T + t0 + tl) * C + c0 + j] = acc[u];
  }
}

unsigned node_blocks(int64_t B, int C, int CT) {
  // enough workgroups for the chip (~8 per CU over the channel tiles), each sweeping nodes
  const int64_t tiles = ceil_div((int64_t)C, (int64_t)CT);
  int64_t want = ceil_div((int64_t)8 * device_cu_count(), tiles);
  if (want < 1) want = 1;
  const int64_t most = ceil_div(B, (int64_t)(kSC / CT));
  return (unsigned)(want < most ? want : most);
}

template <class K>
int allow_smem(K k, size_t bytes) {
  return hip_check(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)bytes));
}

bool shape_ok(int channels, int dim, int rows, int n_terms) {
  return channels > 0 && channels <= 65535 && dim >= 1 && dim <= kMaxDim && rows >= 1 &&
         rows <= kMaxRows && n_terms >= 0;
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_sc_groups(int64_t n_nodes) {
  // node groups of the dcoef reduction: ~256 nodes each, at most 128
  int64_t g = ceil_div(n_nodes, 256);
  if (g > 128) g = 128;
  return (int)(g < 1 ? 1 : g);
}

int gmp_symmetric_contraction_fwd_f32(int64_t n_nodes, int channels, int dim, int rows,
                                      int n_terms, const int32_t* plan, const float* coef,
                                      const float* x, float* out, void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && shape_ok(channels, dim, rows, n_terms));
  if (n_nodes == 0) return GMP_OK;  // (an empty batch's x / out may be NULL)
  GMP_CHECK_ARG(plan && x && out && (n_terms == 0 || coef));
  const int CT = channels < kMaxCT ? channels : kMaxCT;
  const size_t smem = (size_t)kSC * row_stride(dim) * sizeof(float);
  int rc;
  if ((rc = allow_smem(sc_fwd_kernel, smem))) return rc;
  sc_fwd_kernel<<<dim3(node_blocks(n_nodes, channels, CT), (unsigned)ceil_div(channels, CT)), kSC,
                  smem, as_stream(stream)>>>(n_nodes, channels, dim, rows, n_terms, CT, plan, coef,
                                             x, out);
  return launch_status();
}

int gmp_symmetric_contraction_bwd_f32(int64_t n_nodes, int channels, int dim, int rows,
                                      int n_terms, const int32_t* plan, const float* coef,
                                      const float* x, const float* gout, float* dx,
                                      float* dcoef_partials, void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && shape_ok(channels, dim, rows, n_terms));
  hipStream_t s = as_stream(stream);
  if (n_nodes == 0) {
    // an empty node batch (x / gout / dx may be NULL): the single partial group is all zeros
    if (dcoef_partials && n_terms > 0)
      return hip_check(
          hipMemsetAsync(dcoef_partials, 0, (size_t)n_terms * channels * sizeof(float), s));
    return GMP_OK;
  }
  GMP_CHECK_ARG(plan && x && gout && (n_terms == 0 || coef || !dx));
  int rc;
  if (dx) {
    const int CT = channels < kMaxCT ? channels : kMaxCT;
    const size_t smem = (size_t)2 * kSC * row_stride(dim) * sizeof(float);
    if ((rc = allow_smem(sc_bwd_x_kernel, smem))) return rc;
    sc_bwd_x_kernel<<<dim3(node_blocks(n_nodes, channels, CT), (unsigned)ceil_div(channels, CT)),
                      kSC, smem, s>>>(n_nodes, channels, dim, rows, n_terms, CT, plan, coef, x,
                                      gout, dx);
    if ((rc = launch_status())) return rc;
  }
  if (dcoef_partials && n_terms > 0) {
    const int G = gmp_sc_groups(n_nodes);
    const int64_t per = ceil_div(n_nodes, (int64_t)G);
    int CT = kPairs / n_terms;  // channels per tile: all of a tile's pairs in one workgroup
    if (CT > kMaxCT) CT = kMaxCT;
    if (CT > channels) CT = channels;
    if (CT < 1) CT = 1;
    const int tpb = kPairs / CT;
    int NB = kStageLds / (CT * (dim + 1 + rows));
    if (NB > 32) NB = 32;
    if (NB < 1) NB = 1;
    const size_t smem = (size_t)NB * CT * (dim + 1 + rows) * sizeof(float);
    if ((rc = allow_smem(sc_bwd_coef_kernel, smem))) return rc;
    sc_bwd_coef_kernel<<<dim3((unsigned)G, (unsigned)ceil_div(channels, CT),
                              (unsigned)ceil_div(n_terms, tpb)),
                         kSC, smem, s>>>(n_nodes, channels, dim, rows, n_terms, CT, NB, per, plan,
                                         x, gout, dcoef_partials);
    if ((rc = launch_status())) return rc;
  }
  return GMP_OK;
}

}  // extern "C"
