// K7: e3nn FullyConnectedTensorProduct(in1, sh, out, shared_weights=False) with per-edge weights
// + scatter-sum to the receiver (models/layers/tfn_layer.py:82-87), forward and backward.
//
//   out[n, o, w, k] = sum_{e: ei0[e] = n} sum_{p -> o} sum_u W_e[p, u, w] z_e[p, u, k]
//   z_e[p, u, k]    = alpha_p sum_{i,j} C_p[i, j, k] x[ei1[e], b1(p), u, i] Y_e[b2(p), j]
//
// Edges are processed in receiver (ei0)-sorted order; a workgroup owns a node-aligned range of
// a chunk of edges, so each receiver row is summed in one workgroup in a fixed order (no
// atomics; a receiver split across two chunks is read-modify-written by consecutive launches on
// the same stream).  The per-edge weights W_e (E_chunk x weight_numel, from the radial MLP,
// models/layers/tfn_layer.py:73-77) are produced chunk by chunk by the caller, so the kernels
// stream them once (HBM-bound: 4 * weight_numel bytes per edge per pass).
//
// Register layout: thread t = output channel w; each thread keeps its (2l_o+1) accumulators of
// every output block in registers.  The output-block structure is a template parameter
// (MACE: 0e,1o,2e ; TFN gated: 0e,0e,1o,2e) so all register indices are compile-time.
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kTP = 128;          // threads per workgroup (max channel multiplicity)
constexpr int kMaxPaths = 16;
constexpr int kMaxIn = 1152;      // max in1 row dim
constexpr int kMaxZ = 5120;       // max sum_p mul1 * (2lo+1)

struct Path {
  int l1, l2, lo, mul1, mul_out, x_off, y_off, io, out_off, z_off, cg_off, pad;
  long long w_off;
  float alpha, pad2;
};

struct Desc {
  int n_paths, in_dim, out_dim, sh_dim;
  long long weight_numel;
  int z_size, n_blocks;
  int blk_off[4], blk_mul[4], blk_l[4];
};

template <int L>
struct Dim {
  static constexpr int v = 2 * L + 1;
};

// Node-aligned partition of the chunk [c0, c1) of receiver-sorted edges over G workgroups.
__device__ __forceinline__ int64_t lower_bound64(const int64_t* __restrict__ a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int64_t chunk_node_begin(const int64_t* __restrict__ rowptr,
                                                    int64_t n_nodes, int64_t c0, int64_t c1,
                                                    int64_t b, int64_t G) {
  if (b <= 0) {  // node containing edge c0
    int64_t n = lower_bound64(rowptr, n_nodes + 1, c0 + 1) - 1;
    return n < 0 ? 0 : n;
  }
  if (b >= G) return lower_bound64(rowptr, n_nodes + 1, c1);
  return lower_bound64(rowptr, n_nodes + 1, c0 + (c1 - c0) * b / G);
}

// z for one edge: zs[z_off + u*(2lo+1) + k] = alpha sum_ij C x Y  (threads over (p, u) pairs)
__device__ void compute_z(const Path* sp, int n_paths, const float* sCG, const float* sx,
                          const float* sy, float* zs) {
  for (int p = 0; p < n_paths; ++p) {
    const Path P = sp[p];
    const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
    const float* C = sCG + P.cg_off;
    for (int u = threadIdx.x; u < P.mul1; u += blockDim.x) {
      const float* xu = sx + P.x_off + u * d1;
      for (int k = 0; k < d3; ++k) {
        float s = 0.f;
        for (int i = 0; i < d1; ++i) {
          float t = 0.f;
          for (int j = 0; j < d2; ++j) t += C[(i * d2 + j) * d3 + k] * sy[P.y_off + j];
          s += xu[i] * t;
        }
        zs[P.z_off + u * d3 + k] = P.alpha * s;
      }
    }
  }
}

template <int D>
__device__ __forceinline__ void tp_path_accumulate(const float* __restrict__ wrow, const float* zs,
                                                   int mul1, int mul_out, int z_off, int t,
                                                   float (&acc)[D]) {
  if (t >= mul_out) return;
  int u = 0;
  for (; u + 4 <= mul1; u += 4) {
    float wv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) wv[q] = wrow[(int64_t)(u + q) * mul_out + t];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < D; ++k) acc[k] += wv[q] * zs[z_off + (u + q) * D + k];
  }
  for (; u < mul1; ++u) {
    const float wv = wrow[(int64_t)u * mul_out + t];
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] += wv * zs[z_off + u * D + k];
  }
}

template <int NB, int L0, int L1, int L2, int L3>
struct Acc {
  float a0[Dim<L0>::v], a1[Dim<L1>::v], a2[Dim<L2>::v], a3[Dim<L3>::v];
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < Dim<L0>::v; ++k) a0[k] = 0.f;
#pragma unroll
    for (int k = 0; k < Dim<L1>::v; ++k) a1[k] = 0.f;
#pragma unroll
    for (int k = 0; k < Dim<L2>::v; ++k) a2[k] = 0.f;
#pragma unroll
    for (int k = 0; k < Dim<L3>::v; ++k) a3[k] = 0.f;
  }
};

template <int NB, int L0, int L1, int L2, int L3, int LB>
__device__ __forceinline__ float* acc_block(Acc<NB, L0, L1, L2, L3>& A);

// -------------------------------------------------------------------------------- forward
template <int NB, int L0, int L1, int L2, int L3>
__global__ __launch_bounds__(kTP) void tp_fwd_kernel(
    Desc desc, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh, const float* __restrict__ W,
    const int64_t* __restrict__ rowptr, const int64_t* __restrict__ src_sorted,
    const int64_t* __restrict__ perm, int64_t n_nodes, int64_t c0, int64_t c1,
    float* __restrict__ out) {
  __shared__ Path sp[kMaxPaths];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sCG = smem;                 // cg_len
  float* sx = sCG + cg_len;          // in_dim
  float* sy = sx + desc.in_dim;      // 16
  float* zs = sy + 16;               // z_size
  const int t = threadIdx.x;
  for (int i = t; i < desc.n_paths; i += blockDim.x) sp[i] = paths[i];
  for (int i = t; i < cg_len; i += blockDim.x) sCG[i] = cg[i];
  __syncthreads();

  const int64_t G = gridDim.x;
  const int64_t nb = chunk_node_begin(rowptr, n_nodes, c0, c1, blockIdx.x, G);
  const int64_t ne = chunk_node_begin(rowptr, n_nodes, c0, c1, blockIdx.x + 1, G);
  for (int64_t n = nb; n < ne; ++n) {
    int64_t e0 = rowptr[n], e1 = rowptr[n + 1];
    e0 = e0 < c0 ? c0 : e0;
    e1 = e1 > c1 ? c1 : e1;
    if (e0 >= e1) continue;
    Acc<NB, L0, L1, L2, L3> A;
    A.zero();
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t s = src_sorted[e];      // node gathered from (ei1)
      const int64_t eo = perm[e];           // original edge id (for sh)
      for (int i = t; i < desc.in_dim; i += blockDim.x) sx[i] = x[s * desc.in_dim + i];
      if (t < desc.sh_dim) sy[t] = sh[eo * desc.sh_dim + t];
      __syncthreads();
      compute_z(sp, desc.n_paths, sCG, sx, sy, zs);
      __syncthreads();
      const float* We = W + (e - c0) * desc.weight_numel;
      for (int p = 0; p < desc.n_paths; ++p) {
        const Path P = sp[p];
        const float* wrow = We + P.w_off;
        switch (P.io) {
          case 0: tp_path_accumulate<Dim<L0>::v>(wrow, zs, P.mul1, P.mul_out, P.z_off, t, A.a0); break;
          case 1: if (NB > 1) tp_path_accumulate<Dim<L1>::v>(wrow, zs, P.mul1, P.mul_out, P.z_off, t, A.a1); break;
          case 2: if (NB > 2) tp_path_accumulate<Dim<L2>::v>(wrow, zs, P.mul1, P.mul_out, P.z_off, t, A.a2); break;
          default: if (NB > 3) tp_path_accumulate<Dim<L3>::v>(wrow, zs, P.mul1, P.mul_out, P.z_off, t, A.a3); break;
        }
      }
      __syncthreads();  // before the next edge overwrites sx / zs
    }
    float* orow = out + n * desc.out_dim;
#define GMP_TP_STORE(B, ARR, L)                                                   \
    if (NB > B && t < desc.blk_mul[B]) {                                          \
      float* o = orow + desc.blk_off[B] + t * Dim<L>::v;                          \
      _Pragma("unroll") for (int k = 0; k < Dim<L>::v; ++k) o[k] += A.ARR[k];     \
    }
    GMP_TP_STORE(0, a0, L0)
    GMP_TP_STORE(1, a1, L1)
    GMP_TP_STORE(2, a2, L2)
    GMP_TP_STORE(3, a3, L3)
#undef GMP_TP_STORE
  }
}

// -------------------------------------------------------------------------------- backward
// Per edge (grad of the receiver row g = dL/dout[n], same for all edges of n):
//   dW_e[p,u,w] = sum_k z[p,u,k] g[o(p),w,k]
//   dz[p,u,k]   = sum_w W_e[p,u,w] g[o(p),w,k]
//   dx_e[b1,u,i] = sum_{p on b1} alpha_p sum_{j,k} C[i,j,k] Y[j] dz[p,u,k]
//   dY_e[j]      = sum_p alpha_p sum_{u,i,k} C[i,j,k] x[u,i] dz[p,u,k]
constexpr int kRows = 16;  // u rows per W tile (kTP / 8 threads per row)

template <int D>
__device__ __forceinline__ void tp_bwd_path(const float* __restrict__ Wp, float* __restrict__ dWp,
                                            const float* zs, const float* sg, float* dzs,
                                            float* sWt, int mul1, int mul_out, int z_off,
                                            int g_off, int t) {
  // thread t's gradient row of this output block
  float gt[D];
#pragma unroll
  for (int k = 0; k < D; ++k) gt[k] = (t < mul_out) ? sg[g_off + t * D + k] : 0.f;
  const int row = t >> 3, part = t & 7;
  const int cols = (mul_out + 7) / 8;
  for (int u0 = 0; u0 < mul1; u0 += kRows) {
    const int nrows = (mul1 - u0 < kRows) ? mul1 - u0 : kRows;
    // coalesced W tile load (nrows x mul_out) into LDS; dW for the same tile
    for (int r = 0; r < nrows; ++r) {
      if (t < mul_out) {
        const int u = u0 + r;
        sWt[r * 129 + t] = Wp[(int64_t)u * mul_out + t];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < D; ++k) s += zs[z_off + u * D + k] * gt[k];
        dWp[(int64_t)u * mul_out + t] = s;
      }
    }
    __syncthreads();
    // dz: 8 threads per row, each a contiguous slice of the channels, shuffle-reduced
    float dz[D];
#pragma unroll
    for (int k = 0; k < D; ++k) dz[k] = 0.f;
    if (row < nrows) {
      for (int c = part * cols; c < (part + 1) * cols && c < mul_out; ++c) {
        const float wv = sWt[row * 129 + c];
#pragma unroll
        for (int k = 0; k < D; ++k) dz[k] += wv * sg[g_off + c * D + k];
      }
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1)
#pragma unroll
      for (int k = 0; k < D; ++k) dz[k] += __shfl_xor(dz[k], m);
    if (row < nrows && part == 0) {
#pragma unroll
      for (int k = 0; k < D; ++k) dzs[z_off + (u0 + row) * D + k] = dz[k];
    }
    __syncthreads();
  }
}

template <int NB, int L0, int L1, int L2, int L3>
__global__ __launch_bounds__(kTP) void tp_bwd_kernel(
    Desc desc, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh, const float* __restrict__ W,
    const int64_t* __restrict__ rowptr, const int64_t* __restrict__ src_sorted,
    const int64_t* __restrict__ perm, int64_t n_nodes, int64_t c0, int64_t c1,
    const float* __restrict__ gout, float* __restrict__ dW, float* __restrict__ dx_edge,
    float* __restrict__ dY_edge) {
  __shared__ Path sp[kMaxPaths];
  __shared__ float sred[kTP / 64][16];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sCG = smem;
  float* sx = sCG + cg_len;
  float* sy = sx + desc.in_dim;
  float* zs = sy + 16;
  float* dzs = zs + desc.z_size;
  float* sg = dzs + desc.z_size;            // out_dim
  float* sWt = sg + desc.out_dim;           // kRows x 129
  const int t = threadIdx.x;
  for (int i = t; i < desc.n_paths; i += blockDim.x) sp[i] = paths[i];
  for (int i = t; i < cg_len; i += blockDim.x) sCG[i] = cg[i];
  __syncthreads();

  const int64_t G = gridDim.x;
  const int64_t nb = chunk_node_begin(rowptr, n_nodes, c0, c1, blockIdx.x, G);
  const int64_t ne = chunk_node_begin(rowptr, n_nodes, c0, c1, blockIdx.x + 1, G);
  for (int64_t n = nb; n < ne; ++n) {
    int64_t e0 = rowptr[n], e1 = rowptr[n + 1];
    e0 = e0 < c0 ? c0 : e0;
    e1 = e1 > c1 ? c1 : e1;
    if (e0 >= e1) continue;
    for (int i = t; i < desc.out_dim; i += blockDim.x) sg[i] = gout[n * desc.out_dim + i];
    for (int64_t e = e0; e < e1; ++e) {
      const int64_t s = src_sorted[e];
      const int64_t eo = perm[e];
      for (int i = t; i < desc.in_dim; i += blockDim.x) sx[i] = x[s * desc.in_dim + i];
      if (t < desc.sh_dim) sy[t] = sh[eo * desc.sh_dim + t];
      __syncthreads();
      compute_z(sp, desc.n_paths, sCG, sx, sy, zs);
      __syncthreads();
      const float* We = W + (e - c0) * desc.weight_numel;
      float* dWe = dW + (e - c0) * desc.weight_numel;
      for (int p = 0; p < desc.n_paths; ++p) {
        const Path P = sp[p];
        const int g_off = desc.blk_off[P.io];
        switch (P.lo) {
          case 0: tp_bwd_path<1>(We + P.w_off, dWe + P.w_off, zs, sg, dzs, sWt, P.mul1, P.mul_out, P.z_off, g_off, t); break;
          case 1: tp_bwd_path<3>(We + P.w_off, dWe + P.w_off, zs, sg, dzs, sWt, P.mul1, P.mul_out, P.z_off, g_off, t); break;
          default: tp_bwd_path<5>(We + P.w_off, dWe + P.w_off, zs, sg, dzs, sWt, P.mul1, P.mul_out, P.z_off, g_off, t); break;
        }
      }
      // dx_e (threads over in-row entries) and dY_e partials (threads over (p, u))
      float* dxe = dx_edge + e * desc.in_dim;
      for (int i = t; i < desc.in_dim; i += blockDim.x) dxe[i] = 0.f;
      __syncthreads();
      float dyp[9];
#pragma unroll
      for (int j = 0; j < 9; ++j) dyp[j] = 0.f;
      for (int p = 0; p < desc.n_paths; ++p) {
        const Path P = sp[p];
        const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
        const float* C = sCG + P.cg_off;
        for (int u = t; u < P.mul1; u += blockDim.x) {
          const float* dz = dzs + P.z_off + u * d3;
          const float* xu = sx + P.x_off + u * d1;
          for (int i = 0; i < d1; ++i) {
            float acc = 0.f;
#pragma unroll
            for (int jj = 0; jj < 9; ++jj) {  // compile-time register index for dyp
              const int j = jj - P.y_off;
              if (j < 0 || j >= d2) continue;
              float cz = 0.f;
              for (int k = 0; k < d3; ++k) cz += C[(i * d2 + j) * d3 + k] * dz[k];
              acc += cz * sy[jj];
              dyp[jj] += P.alpha * cz * xu[i];
            }
            // a thread owns row u of block b1 for every path on that block: no race
            dxe[P.x_off + u * d1 + i] += P.alpha * acc;
          }
        }
      }
      // block reduction of dY partials
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        float v = dyp[j];
        for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
        dyp[j] = v;
      }
      if ((t & 63) == 0) {
#pragma unroll
        for (int j = 0; j < 9; ++j) sred[t >> 6][j] = dyp[j];
      }
      __syncthreads();
      if (t < desc.sh_dim) {
        float v = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) v += sred[w][t];
        dY_edge[e * desc.sh_dim + t] = v;
      }
      __syncthreads();
    }
  }
}

bool desc_ok(const Desc& d, int layout) {
  if (d.n_paths <= 0 || d.n_paths > kMaxPaths || d.in_dim <= 0 || d.in_dim > kMaxIn ||
      d.z_size <= 0 || d.z_size > kMaxZ || d.sh_dim != 9 || d.weight_numel <= 0)
    return false;
  if (d.n_blocks != (layout == 0 ? 3 : 4)) return false;
  int dim = 0;
  for (int b = 0; b < d.n_blocks; ++b) {
    if (d.blk_mul[b] <= 0 || d.blk_mul[b] > kTP || d.blk_off[b] != dim) return false;
    dim += d.blk_mul[b] * (2 * d.blk_l[b] + 1);
  }
  return dim == d.out_dim;
}

size_t fwd_smem(const Desc& d, int cg_len) {
  return (size_t)(cg_len + d.in_dim + 16 + d.z_size) * sizeof(float);
}
size_t bwd_smem(const Desc& d, int cg_len) {
  return (size_t)(cg_len + d.in_dim + 16 + 2 * d.z_size + d.out_dim + kRows * 129) * sizeof(float);
}

int64_t grid_for_chunk(int64_t edges) {
  int64_t g = ceil_div(edges, 8);  // ~8 edges (a few receivers) per workgroup
  const int64_t cap = (int64_t)device_cu_count() * 8;
  if (g > cap) g = cap;
  return g < 1 ? 1 : g;
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

/* layout codes: 0 = out blocks (0e, 1o, 2e) [MACE]; 1 = (0e, 0e, 1o, 2e) [TFN gated] */
int gmp_tp_conv_fwd_f32(int layout, const void* desc_host, const void* paths_dev,
                        const float* cg_dev, int cg_len, const float* x, const float* sh,
                        const float* W, const int64_t* rowptr, const int64_t* src_sorted,
                        const int64_t* perm, int64_t n_nodes, int64_t c0, int64_t c1, float* out,
                        void* stream) {
  GMP_CHECK_ARG(desc_host && paths_dev && cg_dev && x && sh && W && rowptr && src_sorted && perm && out);
  const Desc d = *reinterpret_cast<const Desc*>(desc_host);
  GMP_CHECK_ARG(desc_ok(d, layout) && cg_len > 0 && cg_len <= 4096);
  GMP_CHECK_ARG(c0 >= 0 && c1 >= c0);
  if (c1 == c0) return GMP_OK;
  hipStream_t s = as_stream(stream);
  const size_t smem = fwd_smem(d, cg_len);
  GMP_CHECK_ARG(smem <= 160 * 1024);
  const unsigned G = (unsigned)grid_for_chunk(c1 - c0);
  int rc;
  if (layout == 0) {
    auto k = tp_fwd_kernel<3, 0, 1, 2, 0>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kTP, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, rowptr, src_sorted, perm, n_nodes, c0, c1, out);
  } else if (layout == 1) {
    auto k = tp_fwd_kernel<4, 0, 0, 1, 2>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kTP, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, rowptr, src_sorted, perm, n_nodes, c0, c1, out);
  } else {
    return GMP_ERR_UNSUPPORTED;
  }
  return launch_status();
}

int gmp_tp_conv_bwd_f32(int layout, const void* desc_host, const void* paths_dev,
                        const float* cg_dev, int cg_len, const float* x, const float* sh,
                        const float* W, const int64_t* rowptr, const int64_t* src_sorted,
                        const int64_t* perm, int64_t n_nodes, int64_t c0, int64_t c1,
                        const float* gout, float* dW, float* dx_edge, float* dY_edge,
                        void* stream) {
  GMP_CHECK_ARG(desc_host && paths_dev && cg_dev && x && sh && W && rowptr && src_sorted && perm);
  GMP_CHECK_ARG(gout && dW && dx_edge && dY_edge);
  const Desc d = *reinterpret_cast<const Desc*>(desc_host);
  GMP_CHECK_ARG(desc_ok(d, layout) && cg_len > 0 && cg_len <= 4096);
  GMP_CHECK_ARG(c0 >= 0 && c1 >= c0 && d.sh_dim <= 9);
  if (c1 == c0) return GMP_OK;
  hipStream_t s = as_stream(stream);
  const size_t smem = bwd_smem(d, cg_len);
  GMP_CHECK_ARG(smem <= 160 * 1024);
  const unsigned G = (unsigned)grid_for_chunk(c1 - c0);
  int rc;
  if (layout == 0) {
    auto k = tp_bwd_kernel<3, 0, 1, 2, 0>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kTP, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, rowptr, src_sorted, perm, n_nodes, c0, c1, gout, dW, dx_edge, dY_edge);
  } else if (layout == 1) {
    auto k = tp_bwd_kernel<4, 0, 0, 1, 2>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kTP, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, rowptr, src_sorted, perm, n_nodes, c0, c1, gout, dW, dx_edge, dY_edge);
  } else {
    return GMP_ERR_UNSUPPORTED;
  }
  return launch_status();
}

}  // extern "C"
