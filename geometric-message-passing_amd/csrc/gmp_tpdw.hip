// K7f: the dW2p weight gradient of the receiver-factorised tensor-product convolution with the S
// intermediate built in the kernel instead of read from HBM (tfn_layer.py:73-87 regrouped, see
// gmp_tp.hip "node form"):
//
//   dW2p[(u, j), w] = sum_(n, k) S[(n, k), (u, j)] G[(n, k), w],
//   S[(n, k), (u, j)] = sum_{e -> n} Z[e, k mul1 + u] A[e, j]
//
// The unfused backward writes S (N (2lo+1) x mul1 H floats: 32.8 GB for a MACE-128 lo = 2 path
// at 1M edges) with gmp_tp_node_outer_f32 and streams it back through the split-plane outer sum;
// here each workgroup owns a 256-row block of dW2p -- a block of 16 channels u x 16 radial
// features j -- and, per 32-deep k stage of (receiver, k) rows, builds that block's S rows from
// the receivers' z and a rows (f32 MFMA 16x16x4 with the edge index as the k dimension: the
// arithmetic of the S kernel), splits them into the three bf16 planes of the dW MFMA's A image
// in LDS and accumulates the stage on the bf16 MFMA (six plane products, f32 accumulation: the
// K7g arithmetic, gmp_tpgemm.hip).  S never reaches HBM; z, a and G are read from L2 by the
// 16 x 16 blocks that share them.
//
// Stages hold whole receivers: RS = 32 / (2lo+1) receivers, rows r = rho (2lo+1) + k, the
// remaining rows zero.  Workgroup grid: row blocks x n_split receiver ranges, dealt so that the
// workgroups of one receiver range share an XCD (their z / a rows share its L2); each writes a
// partial slab, summed in range order by gmp_wgrad's ordered column sum (deterministic).
#include "gmp_common.h"

namespace gmp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kDT = 512;             // threads (8 waves)
constexpr int kDR = 256;             // dW rows per workgroup (16 u x 16 j)
constexpr int kAPl = kDR * 64;       // bytes of one A plane image (256 rows x 32 bf16)
constexpr int kEChunk = 32;          // edges per S-build register batch (8 MFMA k steps)

__device__ __forceinline__ void split3s(float x, unsigned short& h, unsigned short& m,
                                        unsigned short& l) {
  const bf16x2 bh = __builtin_convertvector(f32x2{x, 0.f}, bf16x2);
  const f32x2 r1 = f32x2{x, 0.f} - __builtin_convertvector(bh, f32x2);
  const bf16x2 bm = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(bm, f32x2);
  const bf16x2 bl = __builtin_convertvector(r2, bf16x2);
  h = (unsigned short)(__builtin_bit_cast(unsigned, bh) & 0xffffu);
  m = (unsigned short)(__builtin_bit_cast(unsigned, bm) & 0xffffu);
  l = (unsigned short)(__builtin_bit_cast(unsigned, bl) & 0xffffu);
}

// [row][32 k] bf16 image with 64-byte rows, 16-byte chunk q at q ^ ((row >> 1) & 3) (as K7g):
// byte offset of element (row, k)
__device__ __forceinline__ int eoffk(int row, int k) {
  return row * 64 + 16 * ((k >> 3) ^ ((row >> 1) & 3)) + 2 * (k & 7);
}
__device__ __forceinline__ int xoffc(int row, int chunk) {
  return row * 64 + 16 * (chunk ^ ((row >> 1) & 3));
}
__device__ __forceinline__ bf16x8 asb(u32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// NB = mul_out (64 or 128): waves WM x WN over the 256 x NB block, wave tile (256 / WM) x
// (NB / WN) = RT x CT MFMA tiles
template <int NB>
struct DwCfg {
  static constexpr int WN = NB == 128 ? 2 : 1;
  static constexpr int WM = 8 / WN;
  static constexpr int RT = kDR / WM / 16;  // 4 (NB 128) or 2 (NB 64)
  static constexpr int CT = NB / WN / 16;   // 4
  static constexpr int BPl = NB * 64;       // bytes of one B plane image
  static constexpr int STG = 3 * kAPl + 3 * BPl;
};

template <int NB>
__global__ __launch_bounds__(kDT, 1) void tp_node_dw_kernel(
    int n_recv, int d3, int mul1, int H, const int64_t* __restrict__ eoff,
    const float* __restrict__ Z, const float* __restrict__ A, const float* __restrict__ G,
    float* __restrict__ part, int tiles_j, int n_tiles, int n_split, int stages_per_split) {
  using C = DwCfg<NB>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smd[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int w = d3 * mul1;
  const int RS = 32 / d3, RR = RS * d3;  // receivers per stage, live rows per stage

  // XCD-contiguous logical id (blocks b, b + 8, ... share an XCD): the n_tiles workgroups of a
  // receiver range are consecutive, so they run on one XCD and share its L2
  const int64_t nwg = (int64_t)n_tiles * n_split;
  int64_t L;
  {
    const int64_t b = blockIdx.x, x = b & 7, q = nwg >> 3, r = nwg & 7;
    L = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int sp = (int)(L / n_tiles), tile = (int)(L - (int64_t)sp * n_tiles);
  const int u0 = 16 * (tile / tiles_j), j0 = 16 * (tile % tiles_j);
  const int n_stages = (n_recv + RS - 1) / RS;
  const int st0 = sp * stages_per_split;
  const int st1 = min(st0 + stages_per_split, n_stages);

  const int wm = wv / C::WN, wn = wv % C::WN;
  f32x4 acc[C::RT][C::CT];
#pragma unroll
  for (int r = 0; r < C::RT; ++r)
#pragma unroll
    for (int c = 0; c < C::CT; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- producers of one stage's images (A: S rows of this block, B: G rows), software-
  // pipelined: the stage's edge ranges (meta) are loaded two stages ahead, its z / a / G values
  // one stage ahead into registers (issued before the previous stage's MFMAs), and the S MFMAs,
  // splits and LDS writes run after them.  Wave wv owns stage rows r = 4 wv .. 4 wv + 3 (one
  // MFMA chain over the receiver's edges each): lane (li, g) feeds A = Z[e][k mul1 + u0 + li]
  // and B = A[e][j0 + li] for e = 4 s + g, and holds D[u = 4 g + q][j = li].
  constexpr int kQ = kEChunk / 4;
  int m_e0[4], m_e1[4];           // edge range per item (e1 == e0: empty or dead row)
  float zv[4][kQ], av[4][kQ];     // the first kEChunk edges of each item
  float gv[8];                    // this thread's G values: rows 8 kg .. 8 kg + 7, column w'

  auto load_meta = [&](int st, int (&e0)[4], int (&e1)[4]) {
    const int na = st * RS;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int r = 4 * wv + it, rho = r / d3, n = na + rho;
      e0[it] = e1[it] = 0;
      if (st < st1 && r < RR && n < n_recv) {
        e0[it] = (int)eoff[n];
        e1[it] = (int)eoff[n + 1];
      }
    }
  };
  auto load_vals = [&](int st) {
    const int na = st * RS;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int r = 4 * wv + it, k = r - (r / d3) * d3;
      const float* zc = Z + (int64_t)k * mul1 + u0 + li;
      const float* ac = A + j0 + li;
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        const int e = m_e0[it] + 4 * q + g;
        const bool ok = e < m_e1[it];
        zv[it][q] = ok ? zc[(int64_t)e * w] : 0.f;
        av[it][q] = ok ? ac[(int64_t)e * H] : 0.f;
      }
    }
    {
      const int wc = tid % NB, kg = tid / NB;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = 8 * kg + i;
        const bool ok = tid < 4 * NB && st < st1 && r < RR && na + r / d3 < n_recv;
        gv[i] = ok ? G[((int64_t)na * d3 + r) * NB + wc] : 0.f;
      }
    }
  };
  auto build = [&](int buf) {
    unsigned char* aimg = smd + buf * C::STG;
    unsigned char* bimg = aimg + 3 * kAPl;
    // four independent MFMA chains (one per item), interleaved over the k steps
    f32x4 sacc[4];
    int nqm = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      sacc[it] = f32x4{0.f, 0.f, 0.f, 0.f};
      nqm = max(nqm, (min(m_e1[it] - m_e0[it], kEChunk) + 3) >> 2);
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q)
      if (q < nqm)
#pragma unroll
        for (int it = 0; it < 4; ++it)
          sacc[it] = __builtin_amdgcn_mfma_f32_16x16x4f32(zv[it][q], av[it][q], sacc[it], 0, 0, 0);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      if (m_e1[it] - m_e0[it] > kEChunk) {  // rare: in-degree > kEChunk, the rest directly
        const int r = 4 * wv + it, k = r - (r / d3) * d3;
        const float* zc = Z + (int64_t)k * mul1 + u0 + li;
        const float* ac = A + j0 + li;
        for (int eb = m_e0[it] + kEChunk; eb < m_e1[it]; eb += 4) {
          const int e = eb + g;
          const bool ok = e < m_e1[it];
          const float z1 = ok ? zc[(int64_t)e * w] : 0.f;
          const float a1 = ok ? ac[(int64_t)e * H] : 0.f;
          sacc[it] = __builtin_amdgcn_mfma_f32_16x16x4f32(z1, a1, sacc[it], 0, 0, 0);
        }
      }
    }
    // lane: S[u = 4g + q][j = li] of the wave's four columns r = 4 wv .. 4 wv + 3 -> per row
    // (u, j) and plane one 8-byte write of four consecutive k (columns r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      unsigned short h[4], m[4], l[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) split3s(sacc[it][q], h[it], m[it], l[it]);
      const int off = eoffk((4 * g + q) * 16 + li, 4 * wv);
      *reinterpret_cast<u32x2*>(aimg + off) =
          u32x2{h[0] | ((unsigned)h[1] << 16), h[2] | ((unsigned)h[3] << 16)};
      *reinterpret_cast<u32x2*>(aimg + kAPl + off) =
          u32x2{m[0] | ((unsigned)m[1] << 16), m[2] | ((unsigned)m[3] << 16)};
      *reinterpret_cast<u32x2*>(aimg + 2 * kAPl + off) =
          u32x2{l[0] | ((unsigned)l[1] << 16), l[2] | ((unsigned)l[3] << 16)};
    }
    // G: thread -> B image row w' = tid % NB, k chunk kg = tid / NB (8 rows r of the stage):
    // three 16-byte writes
    if (tid < 4 * NB) {
      const int wc = tid % NB, kg = tid / NB;
      unsigned ph[4], pm[4], pl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        unsigned short h0, m0, l0, h1, m1, l1;
        split3s(gv[2 * i], h0, m0, l0);
        split3s(gv[2 * i + 1], h1, m1, l1);
        ph[i] = h0 | ((unsigned)h1 << 16);
        pm[i] = m0 | ((unsigned)m1 << 16);
        pl[i] = l0 | ((unsigned)l1 << 16);
      }
      const int off = xoffc(wc, kg);
      *reinterpret_cast<u32x4*>(bimg + off) = u32x4{ph[0], ph[1], ph[2], ph[3]};
      *reinterpret_cast<u32x4*>(bimg + C::BPl + off) = u32x4{pm[0], pm[1], pm[2], pm[3]};
      *reinterpret_cast<u32x4*>(bimg + 2 * C::BPl + off) = u32x4{pl[0], pl[1], pl[2], pl[3]};
    }
  };

  // ---- consumer: acc += A^T-image x B-image over one 32-deep stage (x3 products)
  auto consume = [&](int buf) {
    const unsigned char* aimg = smd + buf * C::STG;
    const unsigned char* bimg = aimg + 3 * kAPl;
    u32x4 b[C::CT][3];
#pragma unroll
    for (int c = 0; c < C::CT; ++c) {
      const int off = xoffc((NB / C::WN) * wn + 16 * c + li, g);
#pragma unroll
      for (int p = 0; p < 3; ++p) b[c][p] = *reinterpret_cast<const u32x4*>(bimg + p * C::BPl + off);
    }
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt) {
      u32x4 a[3];
      const int off = xoffc((kDR / C::WM) * wm + 16 * rt + li, g);
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const u32x4*>(aimg + p * kAPl + off);
#pragma unroll
      for (int c = 0; c < C::CT; ++c) {
        f32x4 t = acc[rt][c];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[2]), asb(b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[1]), asb(b[c][1]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[0]), asb(b[c][2]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[1]), asb(b[c][0]), t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[0]), asb(b[c][1]), t, 0, 0, 0);
        acc[rt][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(asb(a[0]), asb(b[c][0]), t, 0, 0, 0);
      }
    }
  };

  if (st0 < st1) {
    int n_e0[4], n_e1[4];  // meta of the stage after the one in registers
    load_meta(st0, m_e0, m_e1);
    load_vals(st0);
    load_meta(st0 + 1, n_e0, n_e1);
    build(0);
    __syncthreads();
    for (int st = st0; st < st1; ++st) {
      const int buf = (st - st0) & 1;
      const bool more = st + 1 < st1;
      if (more) {
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          m_e0[it] = n_e0[it];
          m_e1[it] = n_e1[it];
        }
        load_vals(st + 1);                  // lands while the MFMAs below run
        load_meta(st + 2, n_e0, n_e1);
      }
      consume(buf);
      if (more) build(buf ^ 1);  // the buffer consumed one stage ago
      __syncthreads();
    }
  }

  // partial slab sp: rows (u0 + u) H + j0 + j, NB columns (row-major); C/D map of 16x16x32:
  // col = lane & 15, row = 4 (lane >> 4) + q
  float* out = part + (int64_t)sp * ((int64_t)mul1 * H * NB);
#pragma unroll
  for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
    for (int c = 0; c < C::CT; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = (kDR / C::WM) * wm + 16 * rt + 4 * g + q;  // u * 16 + j
        const int64_t grow = (int64_t)(u0 + (row >> 4)) * H + j0 + (row & 15);
        out[grow * NB + (NB / C::WN) * wn + 16 * c + li] = acc[rt][c][q];
      }
}

// ordered sum of the n_split slabs: dW[x] = sum_sp part[sp][x] (slab order; deterministic)
constexpr int kSumU = 16;
__global__ __launch_bounds__(256) void tp_dw_sum_kernel(const float* __restrict__ part,
                                                        int n_split, int64_t X,
                                                        float* __restrict__ dW) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= X) return;
  float s = 0.f;
  for (int s0 = 0; s0 < n_split; s0 += kSumU) {
    float v[kSumU];
#pragma unroll
    for (int u = 0; u < kSumU; ++u) v[u] = s0 + u < n_split ? part[(int64_t)(s0 + u) * X + x] : 0.f;
#pragma unroll
    for (int u = 0; u < kSumU; ++u)
      if (s0 + u < n_split) s += v[u];
  }
  dW[x] = s;
}

int dw_split(int64_t n_tiles, int64_t n_stages) {
  // ~2 workgroups per CU over the launch, a multiple of 8 ranges (one per XCD round), each
  // range >= 16 stages
  int64_t s = ceil_div(2 * (int64_t)device_cu_count(), n_tiles);
  s = ceil_div(s, 8) * 8;
  const int64_t cap = ceil_div(n_stages, 16);
  if (s > cap) s = cap;
  return (int)(s < 1 ? 1 : s);
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

size_t gmp_tp_node_dw_workspace_size(int64_t n_recv, int64_t d3, int64_t mul1, int64_t H,
                                     int64_t mul_out) {
  if (d3 <= 0 || d3 > 32 || mul1 <= 0 || H <= 0 || mul_out <= 0) return 0;
  const int64_t n_tiles = (mul1 / 16) * (H / 16);
  const int64_t n_stages = ceil_div(n_recv, 32 / d3);
  if (n_tiles <= 0) return 0;
  return (size_t)dw_split(n_tiles, n_stages) * (size_t)(mul1 * H * mul_out) * sizeof(float);
}

int gmp_tp_node_dw_f32(int64_t n_recv, int64_t d3, int64_t mul1, int64_t H, int64_t mul_out,
                       const int64_t* eoff, const float* Z, const float* A, const float* G,
                       float* dW, void* workspace, size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(n_recv >= 0 && d3 >= 1 && d3 <= 32 && mul1 > 0 && H > 0);
  GMP_CHECK_ARG(mul1 % 16 == 0 && H % 16 == 0 && mul1 * d3 <= (1 << 20));
  if (!(mul_out == 64 || mul_out == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(dW);
  hipStream_t s = as_stream(stream);
  const int64_t X = mul1 * H * mul_out;
  if (n_recv == 0) return hip_check(hipMemsetAsync(dW, 0, X * sizeof(float), s));
  GMP_CHECK_ARG(eoff && Z && A && G && workspace);
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(G) % 16 == 0);
  if (workspace_bytes < gmp_tp_node_dw_workspace_size(n_recv, d3, mul1, H, mul_out))
    return GMP_ERR_WORKSPACE;
  const int64_t tiles_j = H / 16, n_tiles = (mul1 / 16) * tiles_j;
  const int64_t RS = 32 / d3, n_stages = ceil_div(n_recv, RS);
  const int n_split = dw_split(n_tiles, n_stages);
  const int64_t sps = ceil_div(n_stages, n_split);
  GMP_CHECK_ARG(n_stages < (1LL << 31) && n_tiles * n_split < (1LL << 31));
  float* part = static_cast<float*>(workspace);
  int rc = 0;
#define GMP_DW(NB)                                                                           \
  {                                                                                          \
    auto k = tp_node_dw_kernel<NB>;                                                          \
    const int smem = 2 * DwCfg<NB>::STG;                                                     \
    if ((rc = hip_check(hipFuncSetAttribute((const void*)k,                                  \
                                            hipFuncAttributeMaxDynamicSharedMemorySize, smem)))) \
      return rc;                                                                             \
    k<<<(unsigned)(n_tiles * n_split), kDT, smem, s>>>(                                      \
        (int)n_recv, (int)d3, (int)mul1, (int)H, eoff, Z, A, G, part, (int)tiles_j,          \
        (int)n_tiles, n_split, (int)sps);                                                    \
  }
  if (mul_out == 128) GMP_DW(128) else GMP_DW(64)
#undef GMP_DW
  rc = launch_status();
  if (rc) return rc;
  tp_dw_sum_kernel<<<(unsigned)ceil_div(X, 256), 256, 0, s>>>(part, n_split, X, dW);
  return launch_status();
}

}  // extern "C"
