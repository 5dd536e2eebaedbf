// K7: e3nn FullyConnectedTensorProduct(in1, sh, out, shared_weights=False) with per-edge weights,
// the message half of models/layers/tfn_layer.py:82-87, forward and backward.
//
//   msg[e, o, w, k] = sum_{p -> o} sum_u W_e[p, u, w] z_e[p, u, k]
//   z_e[p, u, k]    = alpha_p sum_i x[ei1[e], b1(p), u, i] t_e[p, i, k],
//   t_e[p, i, k]    = sum_j C_p[i, j, k] Y_e[b2(p), j]
//
// The per-edge weight rows W_e (weight_numel floats: 721 kB per edge for MACE-128) are produced
// chunk by chunk by the radial MLP (library GEMM) and streamed exactly once here, so both
// kernels are HBM-bound on that stream (forward: read W; backward: read W, write dW).
//
// Work decomposition: one wave per workgroup, each wave owns a contiguous range of
// receiver-sorted edge positions of the chunk (no receiver alignment: messages are written per
// edge and summed per receiver afterwards by the deterministic segmented reduce, so the result is
// independent of chunking and grid size).  Per edge and path, z_p (mul1 x (2lo+1)) is built in
// LDS, then the weight rows are streamed with 16-byte loads: lanes split a row's mul_out outputs
// (4 per lane) and rows are interleaved across lane groups; the output-block accumulators stay in
// registers (block structure = template parameters: MACE 0e,1o,2e; TFN gated 0e,0e,1o,2e).
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kMaxPaths = 48;   // TFN / MACE at l <= 3: 27 paths; both parities, gated: 33
constexpr int kMaxBlocks = 8;   // output irreps blocks (TFN gated both parities l <= 2: 7)
constexpr int kMaxSh = 16;      // SH components (l <= 3) of the node-form z kernels
constexpr int kMaxCg = 4096;    // CG floats of a descriptor (TFN l <= 3: 1,959)
constexpr int kMaxIn = 1152;     // max in1 row dim
constexpr int kMaxMul = 128;     // max mul1 / mul_out of a path
constexpr int kMaxOut = 2048;    // max out row dim

struct Path {
  int l1, l2, lo, mul1, mul_out, x_off, y_off, io, out_off, z_off, cg_off, pad;
  long long w_off;
  float alpha, pad2;
};

struct Desc {
  int n_paths, in_dim, out_dim, sh_dim;
  long long weight_numel;
  int z_size, n_blocks;
  int blk_off[kMaxBlocks], blk_mul[kMaxBlocks], blk_l[kMaxBlocks];
};

typedef float v4f __attribute__((ext_vector_type(4)));

template <int L>
struct Dim {
  static constexpr int v = 2 * L + 1;
};

__device__ __forceinline__ int pow2_ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// LDS layout of one wave (floats)
struct Smem {
  float* cg;   // cg_len
  float* x;    // in_dim (sender row)
  float* y;    // 16 (SH row)
  float* t;    // 32 (t_p[i, k] of the current path)
  float* z;    // kMaxMul * 5 (z_p, in place dz_p in the backward)
  float* g;    // out_dim (backward: receiver gradient row)
  float* dx;   // in_dim (backward: dx row accumulator)
};

__device__ __forceinline__ Smem carve(float* base, int cg_len, int in_dim, int out_dim) {
  Smem s;
  s.cg = base;
  s.x = s.cg + ((cg_len + 3) & ~3);
  s.y = s.x + ((in_dim + 3) & ~3);
  s.t = s.y + 16;
  s.z = s.t + 32;
  s.g = s.z + kMaxMul * 5;
  s.dx = s.g + ((out_dim + 3) & ~3);
  return s;
}

// stage the sender row and the SH row of edge (sorted position) e
__device__ __forceinline__ void stage_edge(const Desc& d, const float* __restrict__ x,
                                           const float* __restrict__ sh, int64_t src, int64_t eo,
                                           Smem& s, int lane) {
  const float* xr = x + src * d.in_dim;
  if ((d.in_dim & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(xr);
    float4* s4 = reinterpret_cast<float4*>(s.x);
    for (int i = lane; i < (d.in_dim >> 2); i += kWave) s4[i] = x4[i];
  } else {
    for (int i = lane; i < d.in_dim; i += kWave) s.x[i] = xr[i];
  }
  if (lane < d.sh_dim) s.y[lane] = sh[eo * d.sh_dim + lane];
}

// t_p[i, k] = sum_j C[i, j, k] Y[y_off + j], then z_p[u, k] = alpha sum_i x[x_off + u d1 + i] t[i, k]
__device__ __forceinline__ void build_z(const Path& P, Smem& s, int lane) {
  const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
  if (lane < d1 * d3) {
    const int i = lane / d3, k = lane - i * d3;
    const float* C = s.cg + P.cg_off;
    float a = 0.f;
    for (int j = 0; j < d2; ++j) a += C[(i * d2 + j) * d3 + k] * s.y[P.y_off + j];
    s.t[lane] = a;
  }
  __syncthreads();
  for (int u = lane; u < P.mul1; u += kWave) {
    const float* xu = s.x + P.x_off + u * d1;
    for (int k = 0; k < d3; ++k) {
      float a = 0.f;
      for (int i = 0; i < d1; ++i) a += xu[i] * s.t[i * d3 + k];
      s.z[u * d3 + k] = P.alpha * a;
    }
  }
  __syncthreads();
}

// -------------------------------------------------------------------------------- forward
// lanes: Lr = pow2 >= mul_out/4 lanes per row (one float4 of outputs each), R = 64/Lr rows per
// load instruction; acc[q][k] = partial msg[w = 4c + q, k] over the rows of lane group r.
template <int D>
__device__ __forceinline__ void fwd_path(const float* __restrict__ Wp, const float* zs, int m1,
                                         int mo, int lane, float (&acc)[4][D]) {
  const int f4 = mo >> 2;
  const int Lr = pow2_ceil(f4), R = kWave / Lr;
  const int r = lane / Lr, c = lane - r * Lr;
  if (c >= f4) return;
  const v4f* __restrict__ base = reinterpret_cast<const v4f*>(Wp) + c;
  constexpr int U = 8;
  int u = r;
  for (; u + (U - 1) * R < m1; u += U * R) {
    v4f w[U];
#pragma unroll
    for (int q = 0; q < U; ++q) w[q] = __builtin_nontemporal_load(base + (int64_t)(u + q * R) * f4);
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const float* zu = zs + (u + q * R) * D;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const float zk = zu[k];
        acc[0][k] += w[q].x * zk;
        acc[1][k] += w[q].y * zk;
        acc[2][k] += w[q].z * zk;
        acc[3][k] += w[q].w * zk;
      }
    }
  }
  for (; u < m1; u += R) {
    const v4f w = __builtin_nontemporal_load(base + (int64_t)u * f4);
    const float* zu = zs + u * D;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const float zk = zu[k];
      acc[0][k] += w.x * zk;
      acc[1][k] += w.y * zk;
      acc[2][k] += w.z * zk;
      acc[3][k] += w.w * zk;
    }
  }
}

template <int D>
__device__ __forceinline__ void zero_acc(float (&a)[4][D]) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < D; ++k) a[q][k] = 0.f;
}

// reduce the row groups and write block b of the message row: msg[blk_off + w*D + k]
template <int D>
__device__ __forceinline__ void fwd_store(float (&acc)[4][D], int mo, float* __restrict__ row,
                                          int lane) {
  const int f4 = mo >> 2;
  const int Lr = pow2_ceil(f4);
  for (int s = Lr; s < kWave; s <<= 1)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < D; ++k) acc[q][k] += __shfl_xor(acc[q][k], s);
  if (lane < f4) {
    float* o = row + 4 * lane * D;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < D; ++k) o[q * D + k] = acc[q][k];
  }
}

template <int NB, int L0, int L1, int L2, int L3>
__global__ __launch_bounds__(kWave) void tp_fwd_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh, const float* __restrict__ W,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t c0,
    int64_t c1, float* __restrict__ msg) {
  __shared__ Path sp[kMaxPaths];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Smem s = carve(smem, cg_len, d.in_dim, d.out_dim);
  const int lane = threadIdx.x;
  for (int i = lane; i < d.n_paths; i += kWave) sp[i] = paths[i];
  for (int i = lane; i < cg_len; i += kWave) s.cg[i] = cg[i];
  __syncthreads();
  const int64_t n = c1 - c0, G = gridDim.x, b = blockIdx.x;
  const int64_t e_begin = c0 + n * b / G, e_end = c0 + n * (b + 1) / G;
  for (int64_t e = e_begin; e < e_end; ++e) {
    stage_edge(d, x, sh, src_sorted[e], perm[e], s, lane);
    __syncthreads();
    float a0[4][Dim<L0>::v], a1[4][Dim<L1>::v], a2[4][Dim<L2>::v], a3[4][Dim<L3>::v];
    zero_acc(a0);
    zero_acc(a1);
    zero_acc(a2);
    zero_acc(a3);
    const float* We = W + (e - c0) * d.weight_numel;
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = sp[p];
      build_z(P, s, lane);
      const float* Wp = We + P.w_off;
      switch (P.io) {
        case 0: fwd_path(Wp, s.z, P.mul1, P.mul_out, lane, a0); break;
        case 1: if (NB > 1) fwd_path(Wp, s.z, P.mul1, P.mul_out, lane, a1); break;
        case 2: if (NB > 2) fwd_path(Wp, s.z, P.mul1, P.mul_out, lane, a2); break;
        default: if (NB > 3) fwd_path(Wp, s.z, P.mul1, P.mul_out, lane, a3); break;
      }
      __syncthreads();  // z is rebuilt for the next path
    }
    float* row = msg + e * d.out_dim;
    fwd_store(a0, d.blk_mul[0], row + d.blk_off[0], lane);
    if (NB > 1) fwd_store(a1, d.blk_mul[1], row + d.blk_off[1], lane);
    if (NB > 2) fwd_store(a2, d.blk_mul[2], row + d.blk_off[2], lane);
    if (NB > 3) fwd_store(a3, d.blk_mul[3], row + d.blk_off[3], lane);
  }
}

// -------------------------------------------------------------------------------- backward
// Per edge, with g = dL/dout[receiver] (the receiver row of the output gradient):
//   dW_e[p,u,w] = sum_k z[p,u,k] g[o(p),w,k]
//   dz[p,u,k]   = sum_w W_e[p,u,w] g[o(p),w,k]
//   dx_e[b1,u,i] = sum_{p on b1} alpha_p sum_k dz[p,u,k] t_p[i,k]
//   dY_e[j]      = sum_p alpha_p sum_{u,i,k} C[i,j,k] x[u,i] dz[p,u,k]
// Row streaming: Lr = min(8, pow2 >= mul_out/4) lanes per row, each lane nq = f4/Lr float4
// columns (interleaved so that a load instruction covers whole 128-byte row segments); dz over a
// row is a log2(Lr)-step shuffle reduction, written in place over z in LDS.
template <int D>
__device__ __forceinline__ void bwd_path(const float* __restrict__ Wp, float* __restrict__ dWp,
                                         float* zs, const float* gb, int m1, int mo, int lane) {
  const int f4 = mo >> 2;
  const int Lr = pow2_ceil(f4) < 8 ? pow2_ceil(f4) : 8;
  const int nq = (f4 + Lr - 1) / Lr;   // <= 4 (mo <= 128)
  const int R = kWave / Lr;
  const int r = lane / Lr, c = lane - r * Lr;
  float g[4][4][D];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int q = c + Lr * t;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < D; ++k) g[t][j][k] = (t < nq && q < f4) ? gb[(4 * q + j) * D + k] : 0.f;
  }
  const v4f* __restrict__ W4 = reinterpret_cast<const v4f*>(Wp);
  v4f* __restrict__ dW4 = reinterpret_cast<v4f*>(dWp);
  const int iters = (m1 + R - 1) / R;
  for (int it = 0; it < iters; ++it) {
    const int u = it * R + r;
    const bool valid = u < m1;
    float z[D];
#pragma unroll
    for (int k = 0; k < D; ++k) z[k] = valid ? zs[u * D + k] : 0.f;
    v4f w[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int q = c + Lr * t;
      w[t] = (valid && t < nq && q < f4) ? __builtin_nontemporal_load(W4 + (int64_t)u * f4 + q)
                                         : v4f{0.f, 0.f, 0.f, 0.f};
    }
    float dz[D];
#pragma unroll
    for (int k = 0; k < D; ++k) dz[k] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int q = c + Lr * t;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < D; ++k) a += z[k] * g[t][j][k];
        o[j] = a;
      }
      if (valid && t < nq && q < f4)
        __builtin_nontemporal_store(v4f{o[0], o[1], o[2], o[3]}, dW4 + (int64_t)u * f4 + q);
#pragma unroll
      for (int k = 0; k < D; ++k)
        dz[k] += w[t].x * g[t][0][k] + w[t].y * g[t][1][k] + w[t].z * g[t][2][k] + w[t].w * g[t][3][k];
    }
    for (int s2 = 1; s2 < Lr; s2 <<= 1)
#pragma unroll
      for (int k = 0; k < D; ++k) dz[k] += __shfl_xor(dz[k], s2);
    if (valid && c == 0) {
#pragma unroll
      for (int k = 0; k < D; ++k) zs[u * D + k] = dz[k];  // in place: row u read above by this group
    }
  }
}

// dx / dY contributions of one path from dz_p (in s.z)
__device__ __forceinline__ void bwd_inputs(const Path& P, Smem& s, int lane, float (&dyp)[9]) {
  const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
  const float* C = s.cg + P.cg_off;
  for (int u = lane; u < P.mul1; u += kWave) {  // lane owns u (same for every path): no race
    const float* dz = s.z + u * d3;
    const float* xu = s.x + P.x_off + u * d1;
    float* dxu = s.dx + P.x_off + u * d1;
    for (int i = 0; i < d1; ++i) {
      float a = 0.f;
      for (int k = 0; k < d3; ++k) a += dz[k] * s.t[i * d3 + k];
      dxu[i] += P.alpha * a;
#pragma unroll
      for (int jj = 0; jj < 9; ++jj) {  // compile-time register index for dyp
        const int j = jj - P.y_off;
        if (j < 0 || j >= d2) continue;
        float cz = 0.f;
        for (int k = 0; k < d3; ++k) cz += C[(i * d2 + j) * d3 + k] * dz[k];
        dyp[jj] += P.alpha * cz * xu[i];
      }
    }
  }
}

template <int NB, int L0, int L1, int L2, int L3>
__global__ __launch_bounds__(kWave) void tp_bwd_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh, const float* __restrict__ W,
    const int64_t* __restrict__ recv_sorted, const int64_t* __restrict__ src_sorted,
    const int64_t* __restrict__ perm, int64_t c0, int64_t c1, const float* __restrict__ gout,
    float* __restrict__ dW, float* __restrict__ dx_edge, float* __restrict__ dY_edge) {
  __shared__ Path sp[kMaxPaths];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Smem s = carve(smem, cg_len, d.in_dim, d.out_dim);
  const int lane = threadIdx.x;
  for (int i = lane; i < d.n_paths; i += kWave) sp[i] = paths[i];
  for (int i = lane; i < cg_len; i += kWave) s.cg[i] = cg[i];
  __syncthreads();
  const int64_t n = c1 - c0, G = gridDim.x, b = blockIdx.x;
  const int64_t e_begin = c0 + n * b / G, e_end = c0 + n * (b + 1) / G;
  int64_t cur = -1;
  for (int64_t e = e_begin; e < e_end; ++e) {
    const int64_t rcv = recv_sorted[e];
    if (rcv != cur) {  // receiver gradient row (shared by the receiver's consecutive edges)
      for (int i = lane; i < d.out_dim; i += kWave) s.g[i] = gout[rcv * d.out_dim + i];
      cur = rcv;
    }
    stage_edge(d, x, sh, src_sorted[e], perm[e], s, lane);
    for (int i = lane; i < d.in_dim; i += kWave) s.dx[i] = 0.f;
    __syncthreads();
    float dyp[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) dyp[j] = 0.f;
    const float* We = W + (e - c0) * d.weight_numel;
    float* dWe = dW + (e - c0) * d.weight_numel;
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = sp[p];
      build_z(P, s, lane);
      const float* gb = s.g + d.blk_off[P.io];
      switch (P.lo) {
        case 0: bwd_path<1>(We + P.w_off, dWe + P.w_off, s.z, gb, P.mul1, P.mul_out, lane); break;
        case 1: bwd_path<3>(We + P.w_off, dWe + P.w_off, s.z, gb, P.mul1, P.mul_out, lane); break;
        default: bwd_path<5>(We + P.w_off, dWe + P.w_off, s.z, gb, P.mul1, P.mul_out, lane); break;
      }
      __syncthreads();
      bwd_inputs(P, s, lane, dyp);
      __syncthreads();  // z / t are rebuilt for the next path
    }
    float* dxr = dx_edge + e * d.in_dim;
    for (int i = lane; i < d.in_dim; i += kWave) dxr[i] = s.dx[i];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      float v = dyp[j];
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
      dyp[j] = v;
    }
    if (lane < d.sh_dim) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < 9; ++j) v = (lane == j) ? dyp[j] : v;
      dY_edge[e * d.sh_dim + lane] = v;
    }
    __syncthreads();
  }
}

// -------------------------------------------------------------------------------- node form
// Receiver-factorised form (the radial MLP's second Linear commutes with the receiver sum):
//   msg_n[w, k] = sum_{e -> n} sum_u (sum_j a_e[j] W2[(u,w), j]) z_e[u, k]
//              = sum_{u, j} W2[(u,w), j] S_n[k, u, j],   S_n[k, u, j] = sum_{e -> n} z_e[u, k] a_e[j]
// The host forms S with batched GEMMs over degree-padded receivers and contracts it with W2 in
// one GEMM per path; these kernels produce z (per edge, per path, layout [p][e][k][u], alpha
// folded in) and map dz back to dx_e / dY_e.  zbuf path p region: rows (n_e + 1) x (d3 * mul1)
// starting at z_off_p * (n_e + 1); row n_e (padding) is left untouched (the host zeroes it).
__global__ __launch_bounds__(kWave) void tp_edge_z_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t e0,
    int64_t e1, float* __restrict__ zbuf) {
  __shared__ Path sp[kMaxPaths];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Smem s = carve(smem, cg_len, d.in_dim, d.out_dim);
  const int lane = threadIdx.x;
  for (int i = lane; i < d.n_paths; i += kWave) sp[i] = paths[i];
  for (int i = lane; i < cg_len; i += kWave) s.cg[i] = cg[i];
  __syncthreads();
  const int64_t ne = e1 - e0, G = gridDim.x, b = blockIdx.x;
  const int64_t eb = e0 + ne * b / G, ee = e0 + ne * (b + 1) / G;
  for (int64_t e = eb; e < ee; ++e) {
    stage_edge(d, x, sh, src_sorted[e], perm[e], s, lane);
    __syncthreads();
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = sp[p];
      const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
      if (lane < d1 * d3) {
        const int i = lane / d3, k = lane - i * d3;
        const float* C = s.cg + P.cg_off;
        float a = 0.f;
        for (int j = 0; j < d2; ++j) a += C[(i * d2 + j) * d3 + k] * s.y[P.y_off + j];
        s.t[lane] = a;
      }
      __syncthreads();
      float* zr = zbuf + (int64_t)P.z_off * (ne + 1) + (e - e0) * (int64_t)(d3 * P.mul1);
      for (int u = lane; u < P.mul1; u += kWave) {
        const float* xu = s.x + P.x_off + u * d1;
        for (int k = 0; k < d3; ++k) {
          float a = 0.f;
          for (int i = 0; i < d1; ++i) a += xu[i] * s.t[i * d3 + k];
          zr[k * P.mul1 + u] = P.alpha * a;
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(kWave) void tp_edge_z_bwd_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t e0,
    int64_t e1, const float* __restrict__ dzbuf, float* __restrict__ dx_edge,
    float* __restrict__ dY_edge) {
  __shared__ Path sp[kMaxPaths];
  extern __shared__ __attribute__((aligned(16))) float smem[];
  Smem s = carve(smem, cg_len, d.in_dim, d.out_dim);
  const int lane = threadIdx.x;
  for (int i = lane; i < d.n_paths; i += kWave) sp[i] = paths[i];
  for (int i = lane; i < cg_len; i += kWave) s.cg[i] = cg[i];
  __syncthreads();
  const int64_t ne = e1 - e0, G = gridDim.x, b = blockIdx.x;
  const int64_t eb = e0 + ne * b / G, ee = e0 + ne * (b + 1) / G;
  for (int64_t e = eb; e < ee; ++e) {
    stage_edge(d, x, sh, src_sorted[e], perm[e], s, lane);
    for (int i = lane; i < d.in_dim; i += kWave) s.dx[i] = 0.f;
    __syncthreads();
    float dyp[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) dyp[j] = 0.f;
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = sp[p];
      const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
      const float* C = s.cg + P.cg_off;
      if (lane < d1 * d3) {
        const int i = lane / d3, k = lane - i * d3;
        float a = 0.f;
        for (int j = 0; j < d2; ++j) a += C[(i * d2 + j) * d3 + k] * s.y[P.y_off + j];
        s.t[lane] = a;
      }
      __syncthreads();
      const float* dzr = dzbuf + (int64_t)P.z_off * (ne + 1) + (e - e0) * (int64_t)(d3 * P.mul1);
      for (int u = lane; u < P.mul1; u += kWave) {  // lane owns u for every path: no race on dx
        float dz[5];
        for (int k = 0; k < d3; ++k) dz[k] = dzr[k * P.mul1 + u];
        const float* xu = s.x + P.x_off + u * d1;
        float* dxu = s.dx + P.x_off + u * d1;
        for (int i = 0; i < d1; ++i) {
          float a = 0.f;
          for (int k = 0; k < d3; ++k) a += dz[k] * s.t[i * d3 + k];
          dxu[i] += P.alpha * a;
#pragma unroll
          for (int jj = 0; jj < 9; ++jj) {
            const int j = jj - P.y_off;
            if (j < 0 || j >= d2) continue;
            float cz = 0.f;
            for (int k = 0; k < d3; ++k) cz += C[(i * d2 + j) * d3 + k] * dz[k];
            dyp[jj] += P.alpha * cz * xu[i];
          }
        }
      }
      __syncthreads();
    }
    float* dxr = dx_edge + (e - e0) * d.in_dim;
    for (int i = lane; i < d.in_dim; i += kWave) dxr[i] = s.dx[i];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      float v = dyp[j];
      for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
      dyp[j] = v;
    }
    if (lane < d.sh_dim) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < 9; ++j) v = (lane == j) ? dyp[j] : v;
      dY_edge[(e - e0) * d.sh_dim + lane] = v;
    }
    __syncthreads();
  }
}

bool desc_ok(const Desc& d, int layout) {
  if (d.n_paths <= 0 || d.n_paths > kMaxPaths || d.in_dim <= 0 || d.in_dim > kMaxIn ||
      d.out_dim <= 0 || d.out_dim > kMaxOut || d.sh_dim != 9 || d.weight_numel <= 0 ||
      (d.weight_numel & 3) != 0)
    return false;
  if (d.n_blocks != (layout == 0 ? 3 : 4)) return false;
  int dim = 0;
  for (int b = 0; b < d.n_blocks; ++b) {
    const int m = d.blk_mul[b];
    if (m <= 0 || m > kMaxMul || (m & 3) != 0 || d.blk_off[b] != dim) return false;
    dim += m * (2 * d.blk_l[b] + 1);
  }
  return dim == d.out_dim;
}

// node-form z / dz kernels: any output block structure (the path GEMMs scatter the outputs),
// l <= 3 everywhere (paths are checked by the host plan), SH rows of (lmax + 1)^2 floats
// (x rows are read straight from global memory: no LDS bound on in_dim)
bool desc_ok_z(const Desc& d) {
  return d.n_paths > 0 && d.n_paths <= kMaxPaths && d.in_dim > 0 && d.in_dim <= (1 << 16) &&
         (d.sh_dim == 1 || d.sh_dim == 4 || d.sh_dim == 9 || d.sh_dim == kMaxSh ||
          d.sh_dim == 25 || d.sh_dim == 36) &&
         d.z_size > 0 && d.n_blocks > 0 && d.n_blocks <= kMaxBlocks;
}

size_t smem_bytes(const Desc& d, int cg_len, bool bwd) {
  size_t f = (size_t)((cg_len + 3) & ~3) + ((d.in_dim + 3) & ~3) + 16 + 32 + kMaxMul * 5;
  if (bwd) f += (size_t)((d.out_dim + 3) & ~3) + d.in_dim;
  return f * sizeof(float);
}

// -------------------------------------------------------------------------------- z, v2
// Per-edge z / dz kernels of the node form without LDS staging or barriers: one wave per edge
// (grid-stride), lane owns channels u = lane, lane + 64 (mul1 <= 128), the CG contraction with
// the edge's SH is unrolled per (l1, l2, lo) at compile time (coefficients are wave-uniform:
// scalar loads), the per-edge backward accumulates dx in registers per input block (one block
// per l1) and dY as per-lane partials reduced once per edge.  HBM-bound on the z / dz rows.
__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

template <int L1, int L2, int LO>
__device__ __forceinline__ void t_table(const float* __restrict__ C, const float (&Y)[kMaxSh],
                                        float (&T)[2 * L1 + 1][2 * LO + 1]) {
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1, D3 = 2 * LO + 1, YO = L2 * L2;
#pragma unroll
  for (int i = 0; i < D1; ++i)
#pragma unroll
    for (int k = 0; k < D3; ++k) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < D2; ++j) a += C[(i * D2 + j) * D3 + k] * Y[YO + j];
      T[i][k] = a;
    }
  __builtin_amdgcn_sched_barrier(0);  // consume the coefficients as they arrive
}

template <int L1, int L2, int LO>
__device__ __forceinline__ void z_path(const Path& P, const float* __restrict__ C,
                                       const float (&Y)[kMaxSh], const float* __restrict__ xrow,
                                       float* __restrict__ zr, int lane) {
  constexpr int D1 = 2 * L1 + 1, D3 = 2 * LO + 1;
  float T[D1][D3];
  t_table<L1, L2, LO>(C, Y, T);
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int u = lane + 64 * uu;
    if (u < P.mul1) {
      float xu[D1];
#pragma unroll
      for (int i = 0; i < D1; ++i) xu[i] = xrow[P.x_off + u * D1 + i];
#pragma unroll
      for (int k = 0; k < D3; ++k) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < D1; ++i) a += xu[i] * T[i][k];
        zr[k * P.mul1 + u] = P.alpha * a;
      }
    }
  }
}

// The sender row's entries for the lane's channels (u = lane, lane + 64) of the l = 0, 1, 2 input
// blocks, loaded once per edge before any z store (r06): with the loads inside z_path, every
// path's loads queued behind the previous path's z stores (vmcnt retires in issue order), one
// exposed round trip per path and edge.
struct XPre {
  float x0[2], x1[2][3], x2[2][5];
};
template <int L1>
__device__ __forceinline__ float xpre(const XPre& x, int uu, int i) {
  if constexpr (L1 == 0) return x.x0[uu];
  else if constexpr (L1 == 1) return x.x1[uu][i];
  else return x.x2[uu][i];
}
template <int L1, int L2, int LO>
__device__ __forceinline__ void z_path_pre(const Path& P, const float* __restrict__ C,
                                           const float (&Y)[kMaxSh], const XPre& xp,
                                           float* __restrict__ zr, int lane) {
  constexpr int D1 = 2 * L1 + 1, D3 = 2 * LO + 1;
  float T[D1][D3];
  t_table<L1, L2, LO>(C, Y, T);
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int u = lane + 64 * uu;
    if (u < P.mul1) {
#pragma unroll
      for (int k = 0; k < D3; ++k) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < D1; ++i) a += xpre<L1>(xp, uu, i) * T[i][k];
        zr[k * P.mul1 + u] = P.alpha * a;
      }
    }
  }
}

struct DxAcc {
  float d0[2], d1[2][3], d2[2][5], d3[2][7];
};

template <int L1, int L2, int LO>
__device__ __forceinline__ void z_bwd_path(const Path& P, const float* __restrict__ C,
                                           const float (&Y)[kMaxSh],
                                           const float* __restrict__ xrow,
                                           const float* __restrict__ dzr, DxAcc& dx,
                                           float (&dyp)[kMaxSh], int lane) {
  constexpr int D1 = 2 * L1 + 1, D2 = 2 * L2 + 1, D3 = 2 * LO + 1, YO = L2 * L2;
  float T[D1][D3];
  t_table<L1, L2, LO>(C, Y, T);
  float M[D3][D1];  // sum over this lane's channels of dz[k] x[i]
#pragma unroll
  for (int k = 0; k < D3; ++k)
#pragma unroll
    for (int i = 0; i < D1; ++i) M[k][i] = 0.f;
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int u = lane + 64 * uu;
    if (u < P.mul1) {
      float xu[D1], dz[D3];
#pragma unroll
      for (int i = 0; i < D1; ++i) xu[i] = xrow[P.x_off + u * D1 + i];
#pragma unroll
      for (int k = 0; k < D3; ++k) dz[k] = P.alpha * dzr[k * P.mul1 + u];
#pragma unroll
      for (int i = 0; i < D1; ++i) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < D3; ++k) a += T[i][k] * dz[k];
        if constexpr (L1 == 0) dx.d0[uu] += a;
        else if constexpr (L1 == 1) dx.d1[uu][i] += a;
        else if constexpr (L1 == 2) dx.d2[uu][i] += a;
        else dx.d3[uu][i] += a;
      }
#pragma unroll
      for (int k = 0; k < D3; ++k)
#pragma unroll
        for (int i = 0; i < D1; ++i) M[k][i] += dz[k] * xu[i];
    }
  }
  // dY_j += sum_{i,k} C[i, j, k] M[k][i]  (per-lane partial; reduced once per edge)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < D2; ++j) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < D1; ++i)
#pragma unroll
      for (int k = 0; k < D3; ++k) a += C[(i * D2 + j) * D3 + k] * M[k][i];
    dyp[YO + j] += a;
  }
}

// (l1, l2, lo) with l <= 3 and |l1 - l2| <= lo <= l1 + l2 (every triangle, any parities): the
// l <= 2 paths (LAUNCH_Z_PATHS2) and those with an l = 3 (LAUNCH_Z_PATHS3)
#define LAUNCH_Z_PATHS3(X)                                                                        \
  X(0, 3, 3) X(1, 2, 3) X(1, 3, 2) X(1, 3, 3) X(2, 1, 3) X(2, 2, 3) X(2, 3, 1) X(2, 3, 2)      \
  X(2, 3, 3) X(3, 0, 3) X(3, 1, 2) X(3, 1, 3) X(3, 2, 1) X(3, 2, 2) X(3, 2, 3) X(3, 3, 0)      \
  X(3, 3, 1) X(3, 3, 2) X(3, 3, 3)

// the l <= 2 subset (LM = 2 kernels: the l = 3 cases compiled out, so their registers are too --
// MACE-128 / TFN max_ell = 2: 59 instead of 91 VGPRs for z, 5 -> 8 waves per SIMD)
#define LAUNCH_Z_PATHS2(X)                                                                        \
  X(0, 0, 0) X(0, 1, 1) X(0, 2, 2) X(1, 0, 1) X(1, 1, 0) X(1, 1, 1) X(1, 1, 2) X(1, 2, 1)      \
  X(1, 2, 2) X(2, 0, 2) X(2, 1, 1) X(2, 1, 2) X(2, 2, 0) X(2, 2, 1) X(2, 2, 2)

// SH row of the edge: sh_dim = (lmax + 1)^2 in {1, 4, 9, 16} components (zeros past sh_dim)
__device__ __forceinline__ void load_y(const float* __restrict__ sh, int64_t eo, int sh_dim,
                                       float (&Y)[kMaxSh]) {
#pragma unroll
  for (int j = 0; j < kMaxSh; ++j) Y[j] = j < sh_dim ? sh[eo * sh_dim + j] : 0.f;
}

// LM: the largest l of any path (host-supplied; an LM = 2 kernel skips l = 3 paths)
template <int LM>
__global__ __launch_bounds__(256) void tp_edge_z2_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t e0,
    int64_t e1, float* __restrict__ zbuf) {
  __shared__ float sC[kMaxCg];  // CG table (wave-uniform reads: LDS broadcast)
  for (int c = threadIdx.x; c < cg_len; c += blockDim.x) sC[c] = cg[c];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t ne = e1 - e0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  // one input block per l1 <= 2 (wave-uniform, from the path table): the sender row is
  // preloaded per edge (XPre); otherwise (l = 3, or a repeated l) each path loads its own
  int xo[3] = {-1, -1, -1}, xm[3] = {0, 0, 0};
  bool pre = LM == 2;
  for (int p = 0; p < d.n_paths; ++p) {
    const Path P = paths[p];
    if (P.l1 > 2 || (xo[P.l1] >= 0 && xo[P.l1] != P.x_off)) pre = false;
    else {
      xo[P.l1] = P.x_off;
      xm[P.l1] = P.mul1;
    }
  }
  if (pre) {
    for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < ne; k += nw) {
      const int64_t e = e0 + __builtin_amdgcn_readfirstlane((int)k);
      const int64_t src = src_sorted[e], eo = perm[e];
      float Y[kMaxSh];
      load_y(sh, eo, d.sh_dim, Y);
      const float* xrow = x + src * d.in_dim;
      XPre xp;
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int u = lane + 64 * uu;
        xp.x0[uu] = u < xm[0] ? xrow[xo[0] + u] : 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) xp.x1[uu][i] = u < xm[1] ? xrow[xo[1] + 3 * u + i] : 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i) xp.x2[uu][i] = u < xm[2] ? xrow[xo[2] + 5 * u + i] : 0.f;
      }
      for (int p = 0; p < d.n_paths; ++p) {
        const Path P = paths[p];
        const float* C = sC + P.cg_off;
        float* zr = zbuf + (int64_t)P.z_off * (ne + 1) + k * (int64_t)((2 * P.lo + 1) * P.mul1);
        switch (P.l1 * 16 + P.l2 * 4 + P.lo) {
#define LAUNCH_ZP_CASE(A, B, O) \
  case A * 16 + B * 4 + O: z_path_pre<A, B, O>(P, C, Y, xp, zr, lane); break;
          LAUNCH_Z_PATHS2(LAUNCH_ZP_CASE)
#undef LAUNCH_ZP_CASE
          default: break;
        }
      }
    }
    return;
  }
  for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < ne; k += nw) {
    const int64_t e = e0 + __builtin_amdgcn_readfirstlane((int)k);
    const int64_t src = src_sorted[e], eo = perm[e];
    float Y[kMaxSh];
    load_y(sh, eo, d.sh_dim, Y);
    const float* xrow = x + src * d.in_dim;
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = paths[p];
      const float* C = sC + P.cg_off;
      float* zr = zbuf + (int64_t)P.z_off * (ne + 1) + k * (int64_t)((2 * P.lo + 1) * P.mul1);
      switch (P.l1 * 16 + P.l2 * 4 + P.lo) {
#define LAUNCH_Z_CASE(A, B, O) \
  case A * 16 + B * 4 + O: z_path<A, B, O>(P, C, Y, xrow, zr, lane); break;
        LAUNCH_Z_PATHS2(LAUNCH_Z_CASE)
#undef LAUNCH_Z_CASE
#define LAUNCH_Z_CASE3(A, B, O)                                                 \
  case A * 16 + B * 4 + O:                                                   \
    if constexpr (LM == 3) z_path<A, B, O>(P, C, Y, xrow, zr, lane);         \
    break;
        LAUNCH_Z_PATHS3(LAUNCH_Z_CASE3)
#undef LAUNCH_Z_CASE3
        default: break;
      }
    }
  }
}

template <int LM>
__global__ __launch_bounds__(256) void tp_edge_z2_bwd_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t e0,
    int64_t e1, const float* __restrict__ dzbuf, float* __restrict__ dx_edge,
    float* __restrict__ dY_edge) {
  __shared__ float sC[kMaxCg];  // CG table (wave-uniform reads: LDS broadcast)
  for (int c = threadIdx.x; c < cg_len; c += blockDim.x) sC[c] = cg[c];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t ne = e1 - e0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  // input blocks (one per l1, as the path table lays them out; wave-uniform): the dx row is
  // written block by block, entries of the row no path reads are written as zero.  Input irreps
  // with a repeated l (both parities: 0e + 0o, ..) take the grouped form: per input block (its
  // first path, sblk) the paths reading it accumulate in registers, then the block is stored.
  __shared__ int sblk[kMaxPaths + 1];  // [count, first path of each distinct input block ..]
  int xoff[4] = {-1, -1, -1, -1}, xmul[4] = {0, 0, 0, 0};
  bool grouped = false;
  for (int p = 0; p < d.n_paths; ++p) {
    const Path P = paths[p];
    grouped |= xoff[P.l1] >= 0 && xoff[P.l1] != P.x_off;
    xoff[P.l1] = P.x_off;
    xmul[P.l1] = P.mul1;
  }
  if (grouped && threadIdx.x == 0) {
    int nb = 0;
    for (int p = 0; p < d.n_paths; ++p) {
      bool first = true;
      for (int q = 0; q < p; ++q) first &= paths[q].x_off != paths[p].x_off;
      if (first) sblk[1 + nb++] = p;
    }
    sblk[0] = nb;
  }
  __syncthreads();
  auto zero_dx = [&](DxAcc& dx) {
#pragma unroll
    for (int uu = 0; uu < 2; ++uu) {
      dx.d0[uu] = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i) dx.d1[uu][i] = 0.f;
#pragma unroll
      for (int i = 0; i < 5; ++i) dx.d2[uu][i] = 0.f;
#pragma unroll
      for (int i = 0; i < 7; ++i) dx.d3[uu][i] = 0.f;
    }
  };
  for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < ne; k += nw) {
    const int64_t e = e0 + __builtin_amdgcn_readfirstlane((int)k);
    const int64_t src = src_sorted[e], eo = perm[e];
    float Y[kMaxSh], dyp[kMaxSh];
    load_y(sh, eo, d.sh_dim, Y);
#pragma unroll
    for (int j = 0; j < kMaxSh; ++j) dyp[j] = 0.f;
    DxAcc dx;
    zero_dx(dx);
    const float* xrow = x + src * d.in_dim;
    float* dxr = dx_edge + k * d.in_dim;
    auto run_path = [&](const Path& P) {
      const float* C = sC + P.cg_off;
      const float* dzr =
          dzbuf + (int64_t)P.z_off * (ne + 1) + k * (int64_t)((2 * P.lo + 1) * P.mul1);
      switch (P.l1 * 16 + P.l2 * 4 + P.lo) {
#define LAUNCH_ZB_CASE(A, B, O) \
  case A * 16 + B * 4 + O: z_bwd_path<A, B, O>(P, C, Y, xrow, dzr, dx, dyp, lane); break;
        LAUNCH_Z_PATHS2(LAUNCH_ZB_CASE)
#undef LAUNCH_ZB_CASE
#define LAUNCH_ZB_CASE3(A, B, O)                                                          \
  case A * 16 + B * 4 + O:                                                             \
    if constexpr (LM == 3) z_bwd_path<A, B, O>(P, C, Y, xrow, dzr, dx, dyp, lane);     \
    break;
        LAUNCH_Z_PATHS3(LAUNCH_ZB_CASE3)
#undef LAUNCH_ZB_CASE3
        default: break;
      }
    };
    // this lane's channels of input block (offset, mul, l) from the l-slot of dx
    auto store_block = [&](int off, int mul, int l) {
#pragma unroll
      for (int uu = 0; uu < 2; ++uu) {
        const int u = lane + 64 * uu;
        if (u >= mul) continue;
        if (l == 0) {
          dxr[off + u] = dx.d0[uu];
        } else if (l == 1) {
#pragma unroll
          for (int i = 0; i < 3; ++i) dxr[off + 3 * u + i] = dx.d1[uu][i];
        } else if (l == 2) {
#pragma unroll
          for (int i = 0; i < 5; ++i) dxr[off + 5 * u + i] = dx.d2[uu][i];
        } else {
#pragma unroll
          for (int i = 0; i < 7; ++i) dxr[off + 7 * u + i] = dx.d3[uu][i];
        }
      }
    };
    int covered = 0;
    if (!grouped) {
      for (int p = 0; p < d.n_paths; ++p) run_path(paths[p]);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (xoff[b] >= 0) store_block(xoff[b], xmul[b], b);
      covered = xmul[0] + 3 * xmul[1] + 5 * xmul[2] + 7 * xmul[3];
    } else {
      const int nb = sblk[0];
      for (int b = 0; b < nb; ++b) {
        const Path Pb = paths[sblk[1 + b]];
        zero_dx(dx);
        for (int p = sblk[1 + b]; p < d.n_paths; ++p) {
          const Path P = paths[p];
          if (P.x_off == Pb.x_off) run_path(P);
        }
        store_block(Pb.x_off, Pb.mul1, Pb.l1);
        covered += Pb.mul1 * (2 * Pb.l1 + 1);
      }
    }
    if (covered != d.in_dim) {
      for (int c = lane; c < d.in_dim; c += 64) {  // rows read by no path: zero
        bool in = false;
        for (int p = 0; p < d.n_paths; ++p) {
          const Path P = paths[p];
          in |= c >= P.x_off && c < P.x_off + P.mul1 * (2 * P.l1 + 1);
        }
        if (!in) dxr[c] = 0.f;
      }
    }
    float dyv = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxSh; ++j) {
      if (j < d.sh_dim) {  // wave-uniform
        const float v = wave_sum64(dyp[j]);
        dyv = (lane == j) ? v : dyv;
      }
    }
    if (lane < d.sh_dim) dY_edge[k * d.sh_dim + lane] = dyv;
  }
}

// ---------------------------------------------------------------------- z, runtime l <= 5
// Plans with an l of 4 or 5 (TFN / MACE max_ell = 5, experiments/rotsym.ipynb) take these
// kernels: the same per-edge arithmetic with runtime (l1, l2, lo) loops.  One wave per edge; the
// edge's SH row (36 floats) and each path's T = C . Y table (<= 11 x 11) go through a per-wave
// LDS slice (computed once by the wave's lanes, read as broadcasts), the CG table through LDS /
// global as the fixed-l kernels.  Not tuned (widening configs at one layer).
constexpr int kMaxShG = 36, kMaxTG = 121;
constexpr int kMaxCgG = 8192;  // CG floats of a descriptor (generic kernels)

__device__ __forceinline__ void gen_t_table(const float* C, const float* sY, int d1, int d2,
                                            int d3, int yo, float* sT, int lane) {
  for (int t = lane; t < d1 * d3; t += 64) {
    const int i = t / d3, k = t - i * d3;
    float a = 0.f;
    for (int j = 0; j < d2; ++j) a += C[(i * d2 + j) * d3 + k] * sY[yo + j];
    sT[t] = a;
  }
}

__global__ __launch_bounds__(256) void tp_edge_z_gen_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t e0,
    int64_t e1, float* __restrict__ zbuf) {
  __shared__ float sC[kMaxCgG];
  __shared__ float sYT[4][kMaxShG + kMaxTG];
  for (int c = threadIdx.x; c < cg_len; c += blockDim.x) sC[c] = cg[c];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sY = sYT[wv];
  float* sT = sYT[wv] + kMaxShG;
  const int64_t ne = e1 - e0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t k = (int64_t)blockIdx.x * 4 + wv; k < ne; k += nw) {
    const int64_t e = e0 + __builtin_amdgcn_readfirstlane((int)k);
    const int64_t src = src_sorted[e], eo = perm[e];
    if (lane < d.sh_dim) sY[lane] = sh[eo * d.sh_dim + lane];
    const float* xrow = x + src * d.in_dim;
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = paths[p];
      const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1;
      __builtin_amdgcn_wave_barrier();  // the slice's previous readers are this wave's lanes
      gen_t_table(sC + P.cg_off, sY, d1, d2, d3, P.l2 * P.l2, sT, lane);
      __builtin_amdgcn_wave_barrier();
      float* zr = zbuf + (int64_t)P.z_off * (ne + 1) + k * (int64_t)(d3 * P.mul1);
      for (int u = lane; u < P.mul1; u += 64) {
        const float* xu = xrow + P.x_off + u * d1;
        for (int kk = 0; kk < d3; ++kk) {
          float a = 0.f;
          for (int i = 0; i < d1; ++i) a += xu[i] * sT[i * d3 + kk];
          zr[kk * P.mul1 + u] = P.alpha * a;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ __launch_bounds__(256) void tp_edge_z_gen_bwd_kernel(
    Desc d, const Path* __restrict__ paths, const float* __restrict__ cg, int cg_len,
    const float* __restrict__ x, const float* __restrict__ sh,
    const int64_t* __restrict__ src_sorted, const int64_t* __restrict__ perm, int64_t e0,
    int64_t e1, const float* __restrict__ dzbuf, float* __restrict__ dx_edge,
    float* __restrict__ dY_edge) {
  __shared__ float sC[kMaxCgG];
  __shared__ float sYT[4][kMaxShG + kMaxTG];
  __shared__ float sdY[4][kMaxShG];
  for (int c = threadIdx.x; c < cg_len; c += blockDim.x) sC[c] = cg[c];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* sY = sYT[wv];
  float* sT = sYT[wv] + kMaxShG;
  const int64_t ne = e1 - e0;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t k = (int64_t)blockIdx.x * 4 + wv; k < ne; k += nw) {
    const int64_t e = e0 + __builtin_amdgcn_readfirstlane((int)k);
    const int64_t src = src_sorted[e], eo = perm[e];
    __builtin_amdgcn_wave_barrier();
    if (lane < d.sh_dim) {
      sY[lane] = sh[eo * d.sh_dim + lane];
      sdY[wv][lane] = 0.f;
    }
    const float* xrow = x + src * d.in_dim;
    float* dxr = dx_edge + k * d.in_dim;
    // the dx row: zero (each entry by the lane that will accumulate it: u = lane + 64 t),
    // entries no path reads included, then one read-modify-write pass per path
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = paths[p];
      const int d1 = 2 * P.l1 + 1;
      for (int u = lane; u < P.mul1; u += 64)
        for (int i = 0; i < d1; ++i) dxr[P.x_off + u * d1 + i] = 0.f;
    }
    for (int c = lane; c < d.in_dim; c += 64) {
      bool in = false;
      for (int p = 0; p < d.n_paths; ++p) {
        const Path P = paths[p];
        in |= c >= P.x_off && c < P.x_off + P.mul1 * (2 * P.l1 + 1);
      }
      if (!in) dxr[c] = 0.f;
    }
    for (int p = 0; p < d.n_paths; ++p) {
      const Path P = paths[p];
      const int d1 = 2 * P.l1 + 1, d2 = 2 * P.l2 + 1, d3 = 2 * P.lo + 1, yo = P.l2 * P.l2;
      __builtin_amdgcn_wave_barrier();
      gen_t_table(sC + P.cg_off, sY, d1, d2, d3, yo, sT, lane);
      __builtin_amdgcn_wave_barrier();
      const float* C = sC + P.cg_off;
      const float* dzr = dzbuf + (int64_t)P.z_off * (ne + 1) + k * (int64_t)(d3 * P.mul1);
      // per lane: dx[u, i] += alpha sum_k T[i, k] dz[u, k]; dY_j partials
      // sum_{u, i, k} C[i, j, k] x[u, i] alpha dz[u, k]
      float dyp[11];
      for (int j = 0; j < 11; ++j) dyp[j] = 0.f;
      for (int u = lane; u < P.mul1; u += 64) {
        const float* xu = xrow + P.x_off + u * d1;
        float dz[11];
#pragma unroll
        for (int kk = 0; kk < 11; ++kk) dz[kk] = kk < d3 ? P.alpha * dzr[kk * P.mul1 + u] : 0.f;
        for (int i = 0; i < d1; ++i) {
          float a = 0.f;
#pragma unroll
          for (int kk = 0; kk < 11; ++kk)
            if (kk < d3) a += sT[i * d3 + kk] * dz[kk];
          dxr[P.x_off + u * d1 + i] += a;
          const float xi = xu[i];
#pragma unroll
          for (int j = 0; j < 11; ++j) {
            if (j < d2) {
              float c = 0.f;
#pragma unroll
              for (int kk = 0; kk < 11; ++kk)
                if (kk < d3) c += C[(i * d2 + j) * d3 + kk] * dz[kk];
              dyp[j] += xi * c;
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 11; ++j) {
        if (j < d2) {  // wave-uniform
          const float v = wave_sum64(dyp[j]);
          if (lane == 0) sdY[wv][yo + j] += v;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < d.sh_dim) dY_edge[k * d.sh_dim + lane] = sdY[wv][lane];
  }
}

// The l <= 2 instantiation (z 59 vs 91 VGPRs, 8 vs 5 waves per SIMD) measured within noise of
// the l <= 3 one on the MACE / TFN steps (r03); kept as the tighter-register form.
int64_t z2_blocks(int64_t edges) {
  const int64_t cap = (int64_t)device_cu_count() * 8;  // 32 resident waves per CU
  int64_t g = (edges + 3) / 4;
  g = g < cap ? g : cap;
  return g < 1 ? 1 : g;
}

int64_t grid_for_chunk(int64_t edges) {
  const int64_t cap = (int64_t)device_cu_count() * 8;  // ~8 resident waves per CU
  int64_t g = edges < cap ? edges : cap;
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
                        const float* W, const int64_t* src_sorted, const int64_t* perm,
                        int64_t c0, int64_t c1, float* msg, void* stream) {
  GMP_CHECK_ARG(desc_host && paths_dev && cg_dev && x && sh && W && src_sorted && perm && msg);
  const Desc d = *reinterpret_cast<const Desc*>(desc_host);
  GMP_CHECK_ARG(desc_ok(d, layout) && cg_len > 0 && cg_len <= 4096);
  GMP_CHECK_ARG(c0 >= 0 && c1 >= c0);
  if (c1 == c0) return GMP_OK;
  hipStream_t s = as_stream(stream);
  const size_t smem = smem_bytes(d, cg_len, false);
  GMP_CHECK_ARG(smem <= 64 * 1024);
  const unsigned G = (unsigned)grid_for_chunk(c1 - c0);
  int rc;
  if (layout == 0) {
    auto k = tp_fwd_kernel<3, 0, 1, 2, 0>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kWave, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, src_sorted, perm, c0, c1, msg);
  } else {
    auto k = tp_fwd_kernel<4, 0, 0, 1, 2>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kWave, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, src_sorted, perm, c0, c1, msg);
  }
  return launch_status();
}

int gmp_tp_conv_bwd_f32(int layout, const void* desc_host, const void* paths_dev,
                        const float* cg_dev, int cg_len, const float* x, const float* sh,
                        const float* W, const int64_t* recv_sorted, const int64_t* src_sorted,
                        const int64_t* perm, int64_t c0, int64_t c1, const float* gout,
                        float* dW, float* dx_edge, float* dY_edge, void* stream) {
  GMP_CHECK_ARG(desc_host && paths_dev && cg_dev && x && sh && W && recv_sorted && src_sorted &&
                perm);
  GMP_CHECK_ARG(gout && dW && dx_edge && dY_edge);
  const Desc d = *reinterpret_cast<const Desc*>(desc_host);
  GMP_CHECK_ARG(desc_ok(d, layout) && cg_len > 0 && cg_len <= 4096);
  GMP_CHECK_ARG(c0 >= 0 && c1 >= c0);
  if (c1 == c0) return GMP_OK;
  hipStream_t s = as_stream(stream);
  const size_t smem = smem_bytes(d, cg_len, true);
  GMP_CHECK_ARG(smem <= 64 * 1024);
  const unsigned G = (unsigned)grid_for_chunk(c1 - c0);
  int rc;
  if (layout == 0) {
    auto k = tp_bwd_kernel<3, 0, 1, 2, 0>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kWave, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, recv_sorted, src_sorted, perm, c0, c1, gout, dW, dx_edge, dY_edge);
  } else {
    auto k = tp_bwd_kernel<4, 0, 0, 1, 2>;
    if ((rc = set_smem(k, smem))) return rc;
    k<<<G, kWave, smem, s>>>(d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, W, recv_sorted, src_sorted, perm, c0, c1, gout, dW, dx_edge, dY_edge);
  }
  return launch_status();
}

int gmp_tp_edge_z_lmax_f32(const void* desc_host, int l_max, const void* paths_dev,
                           const float* cg_dev, int cg_len, const float* x, const float* sh,
                           const int64_t* src_sorted, const int64_t* perm, int64_t e0, int64_t e1,
                           float* zbuf, void* stream) {
  GMP_CHECK_ARG(desc_host && paths_dev && cg_dev && x && sh && src_sorted && perm && zbuf);
  const Desc d = *reinterpret_cast<const Desc*>(desc_host);
  GMP_CHECK_ARG(desc_ok_z(d) && cg_len > 0 && cg_len <= (l_max > 3 ? kMaxCgG : kMaxCg));
  GMP_CHECK_ARG(e0 >= 0 && e1 >= e0 && l_max >= 0 && l_max <= 5);
  if (e1 == e0) return GMP_OK;
  const unsigned grid = (unsigned)z2_blocks(e1 - e0);
  if (l_max > 3 || d.sh_dim > kMaxSh)
    tp_edge_z_gen_kernel<<<grid, 256, 0, as_stream(stream)>>>(
        d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm, e0, e1, zbuf);
  else if (l_max <= 2 && d.sh_dim <= 9)
    tp_edge_z2_kernel<2><<<grid, 256, 0, as_stream(stream)>>>(
        d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm, e0, e1, zbuf);
  else
    tp_edge_z2_kernel<3><<<grid, 256, 0, as_stream(stream)>>>(
        d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm, e0, e1, zbuf);
  return launch_status();
}

int gmp_tp_edge_z_f32(const void* desc_host, const void* paths_dev, const float* cg_dev,
                      int cg_len, const float* x, const float* sh, const int64_t* src_sorted,
                      const int64_t* perm, int64_t e0, int64_t e1, float* zbuf, void* stream) {
  return gmp_tp_edge_z_lmax_f32(desc_host, 3, paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm,
                                e0, e1, zbuf, stream);
}

int gmp_tp_edge_z_bwd_lmax_f32(const void* desc_host, int l_max, const void* paths_dev,
                               const float* cg_dev, int cg_len, const float* x, const float* sh,
                               const int64_t* src_sorted, const int64_t* perm, int64_t e0,
                               int64_t e1, const float* dzbuf, float* dx_edge, float* dY_edge,
                               void* stream) {
  GMP_CHECK_ARG(desc_host && paths_dev && cg_dev && x && sh && src_sorted && perm && dzbuf &&
                dx_edge && dY_edge);
  const Desc d = *reinterpret_cast<const Desc*>(desc_host);
  GMP_CHECK_ARG(desc_ok_z(d) && cg_len > 0 && cg_len <= (l_max > 3 ? kMaxCgG : kMaxCg));
  GMP_CHECK_ARG(e0 >= 0 && e1 >= e0 && l_max >= 0 && l_max <= 5);
  if (e1 == e0) return GMP_OK;
  const unsigned grid = (unsigned)z2_blocks(e1 - e0);
  if (l_max > 3 || d.sh_dim > kMaxSh)
    tp_edge_z_gen_bwd_kernel<<<grid, 256, 0, as_stream(stream)>>>(
        d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm, e0, e1, dzbuf,
        dx_edge, dY_edge);
  else if (l_max <= 2 && d.sh_dim <= 9)
    tp_edge_z2_bwd_kernel<2><<<grid, 256, 0, as_stream(stream)>>>(
        d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm, e0, e1, dzbuf,
        dx_edge, dY_edge);
  else
    tp_edge_z2_bwd_kernel<3><<<grid, 256, 0, as_stream(stream)>>>(
        d, (const Path*)paths_dev, cg_dev, cg_len, x, sh, src_sorted, perm, e0, e1, dzbuf,
        dx_edge, dY_edge);
  return launch_status();
}

int gmp_tp_edge_z_bwd_f32(const void* desc_host, const void* paths_dev, const float* cg_dev,
                          int cg_len, const float* x, const float* sh, const int64_t* src_sorted,
                          const int64_t* perm, int64_t e0, int64_t e1, const float* dzbuf,
                          float* dx_edge, float* dY_edge, void* stream) {
  return gmp_tp_edge_z_bwd_lmax_f32(desc_host, 3, paths_dev, cg_dev, cg_len, x, sh, src_sorted,
                                    perm, e0, e1, dzbuf, dx_edge, dY_edge, stream);
}

}  // extern "C"
