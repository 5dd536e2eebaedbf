// K15: EGNN node update + next-layer node projections in one launch (gfx950).  Reference:
// models/layers/egnn_layer.py:82-86 (update), models/egnn.py:75-76 (residual), :28-29 (the first
// message Linear whose node half AB this kernel also produces).  Design notes: DESIGN.md "K15".
#include "gmp_egnn_common.h"

namespace gmp {
namespace {

// ================================================================================== K15 node update
// EGNN node update of one layer + the next layer's node projections, in one launch
// (egnn_layer.py:82-86 update, egnn.py:75-76 residual, and the AB = [h W1a^T | h W1b^T] split of
// the next layer's first message Linear, egnn_layer.py:28-29):
//   u  = W0 [h | m_aggr] + b0;  x1 = act(LN1(u));  x2 = act(LN2(W3 x1 + b3))
//   h' = h + x2 (residual) or x2;   AB' = [h' W1a'^T | h' W1b'^T]   (optional)
// A workgroup (8 waves) owns kNodeRT * 8 tiles of 16 node rows; the three weight matrices pass
// through LDS one after the other as 2-plane fp16 images (the K4 arithmetic: 22-bit operands,
// f32 accumulation); the row tiles stay in registers between the phases (lane layout as K4:
// row = lane & 15, features 16 p + 4 g + c).  The images are built once per forward for every
// layer (egnn_node_image_kernel: one workgroup per 16-row tile of a matrix, each tile with its
// own power-of-two scale, so no cross-workgroup max) and copied into LDS with 16-byte loads: the
// r05 first form converted the f32 weights in every workgroup (max pass, column means, plane
// pass: ~60 of its ~90 us).  GEMM inputs: [h | m] and h' take a per-row power-of-two scale (max
// over the row), act(LN1) the static LayerNorm bound (relu: folded into the affine's vectors).
// SAVE (training): x_hat1, x_hat2 ((2, N, d)) and their 1/std ((2, N)) for the LayerNorm
// backwards.  Replaces ~8 launches per layer (split Linear x2, LN+act x2, Linear, residual add,
// weight concatenation, AB GEMM) and their (N, d) round trips.
constexpr int kNodeWaves = 8;
constexpr int kNodeRT = 2;  // row tiles per wave: 256 rows per workgroup
enum NodeVec { NV0_B0 = 0, NV0_G1, NV0_BE1, NV0_B3, NV0_G2, NV0_BE2, NV0_G1S, NV0_BE1S, NVN };

// one layer's weight image (bytes): [W0 hi | W0 lo] (d rows, 2d + 16 halfs), [W3 hi | W3 lo]
// (d rows, d + 16), [Wab hi | Wab lo] (2d rows = W1a' then W1b', d + 16), then the per-tile
// exponents (int): W0 d / 16, W3 d / 16, Wab 2d / 16
template <int D>
struct NImg {
  static constexpr int LDH0 = 2 * D + 16, LDH = D + 16;
  static constexpr int W0H = D * LDH0, W3H = D * LDH, WAH = 2 * D * LDH;  // halfs per plane
  static constexpr size_t off_w0 = 0;
  static constexpr size_t off_w3 = off_w0 + (size_t)2 * W0H * 2;
  static constexpr size_t off_wa = off_w3 + (size_t)2 * W3H * 2;
  static constexpr size_t off_exp = off_wa + (size_t)2 * WAH * 2;
  static constexpr int T0 = D / 16, T3 = D / 16, TA = 2 * D / 16;
  static constexpr size_t bytes = off_exp + 256;
  static constexpr int PLANES = W0H > WAH ? W0H : WAH;  // LDS image area: 2 x PLANES halfs
  static constexpr size_t smem_bytes() {
    return (size_t)(NVN * D + 64) * 4 + (size_t)2 * PLANES * 2;
  }
};

struct NodeImgArgs {  // up to 8 layers per image launch
  gmp_egnn_node_params p[8];
  int n;
};

// one workgroup (256 threads) per 16-row tile of a layer's W0, W3 or Wab: the tile's max |w|
// -> its exponent s (max |w| 2^s < 2^15), then the hi / lo fp16 planes of w 2^s in hf_pos
// column order (the layout gemm_img reads)
template <int D>
__global__ __launch_bounds__(256) void egnn_node_image_kernel(NodeImgArgs A,
                                                              unsigned char* __restrict__ img) {
  using I = NImg<D>;
  constexpr int TL = I::T0 + I::T3 + I::TA;
  __shared__ unsigned smx;
  const int layer = blockIdx.x / TL, tt = blockIdx.x - layer * TL;
  const gmp_egnn_node_params& P = A.p[layer];
  int mat, t;
  if (tt < I::T0) { mat = 0; t = tt; }
  else if (tt < I::T0 + I::T3) { mat = 1; t = tt - I::T0; }
  else { mat = 2; t = tt - I::T0 - I::T3; }
  if (mat == 2 && P.W1n == nullptr) return;  // (block-uniform)
  const int K = mat == 0 ? 2 * D : D, ldh = mat == 0 ? I::LDH0 : I::LDH;
  const int plane = mat == 0 ? I::W0H : (mat == 1 ? I::W3H : I::WAH);
  unsigned char* base = img + (size_t)layer * I::bytes;
  _Float16* hW = reinterpret_cast<_Float16*>(base + (mat == 0 ? I::off_w0 : (mat == 1 ? I::off_w3 : I::off_wa)));
  auto src = [&](int o, int k) -> float {
    if (mat == 0) return P.W0[(int64_t)o * 2 * D + k];
    if (mat == 1) return P.W3[(int64_t)o * D + k];
    return P.W1n[(int64_t)(o % D) * P.ld1 + (o / D) * D + k];
  };
  constexpr int kMaxPer = 16;  // 16 rows x <= 2d columns over 256 threads: <= 16 per thread
  const int n = 16 * K;
  float w[kMaxPer];
  float mx = 0.f;
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const int e = threadIdx.x + u * 256;
    w[u] = e < n ? src(16 * t + e / K, e % K) : 0.f;
    mx = fmaxf(mx, fabsf(w[u]));
  }
  if (threadIdx.x == 0) smx = 0u;
  __syncthreads();
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(&smx, __float_as_uint(mx));
  __syncthreads();
  const int s = scale_exp(__uint_as_float(smx));
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const int e = threadIdx.x + u * 256;
    if (e < n) {
      const int o = 16 * t + e / K, k = e % K;
      const float v = ldexpf(w[u], s);
      const _Float16 hi = (_Float16)v;
      _Float16* dst = hW + o * ldh + hf_pos(k);
      dst[0] = hi;
      dst[plane] = (_Float16)(v - (float)hi);
    }
  }
  if (threadIdx.x == 0) {
    int* ex = reinterpret_cast<int*>(base + I::off_exp);
    ex[mat == 0 ? t : (mat == 1 ? I::T0 + t : I::T0 + I::T3 + t)] = s;
  }
}

// copy `bytes` (a multiple of 16) of image into LDS with 16-byte loads, kU in flight per thread
__device__ __forceinline__ void copy_image(void* dst, const void* src, int bytes) {
  constexpr int kU = 9;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  const int n = bytes / 16;
  for (int i0 = threadIdx.x; i0 < n; i0 += kU * blockDim.x) {
    uint4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * blockDim.x;
      if (i < n) v[u] = s[i];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * blockDim.x;
      if (i < n) d[i] = v[u];
    }
  }
}

// y[TO tiles] += W x over K = 16 KT features (the image: rows 16 t + i, ldh halfs, lo plane at
// +plane); x scaled by fx first unless XS.  gemm_h2s generalised to K != d and TO != d / 16,
// with the A operand (the two W planes) of step q + 1 read from LDS while step q's three MFMAs
// run (two register buffers): at two waves per SIMD the r05 first form waited out each LDS read
// (817 waits for 960 MFMAs per wave).
template <int KT, int TO, bool XS>
__device__ __forceinline__ void gemm_img(const _Float16* __restrict__ hW, int ldh, int plane,
                                         float fx, const f32x4 (&x)[KT], f32x4 (&y)[TO], int i,
                                         int g) {
  constexpr int NB = KT / 2, NQ = NB * TO, PD = 2;  // prefetch distance (PD + 1 buffers)
  const _Float16* base = hW + i * ldh + 8 * g;
  h16x8 ah[PD + 1], al[PD + 1];
#pragma unroll
  for (int q = 0; q < PD && q < NQ; ++q) {
    const _Float16* row = base + 16 * (q % TO) * ldh + 32 * (q / TO);
    ah[q] = *reinterpret_cast<const h16x8*>(row);
    al[q] = *reinterpret_cast<const h16x8*>(row + plane);
  }
  h16x8 bh, bl;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int p = q / TO, t = q % TO;
    if (t == 0) {
      if constexpr (XS) split8(x[2 * p], x[2 * p + 1], bh, bl);
      else split8(x[2 * p] * fx, x[2 * p + 1] * fx, bh, bl);
    }
    if (q + PD < NQ) {
      const int qn = q + PD;
      const _Float16* row = base + 16 * (qn % TO) * ldh + 32 * (qn / TO);
      ah[qn % (PD + 1)] = *reinterpret_cast<const h16x8*>(row);
      al[qn % (PD + 1)] = *reinterpret_cast<const h16x8*>(row + plane);
    }
    const int b = q % (PD + 1);
    f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[b], bh, y[t], 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], bl, acc, 0, 0, 0);
    y[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], bh, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// per-row power-of-two input exponent from the row's max |x| (the row's 4 lane groups)
template <int KT>
__device__ __forceinline__ int row_exp(const f32x4 (&x)[KT]) {
  float mx = 0.f;
#pragma unroll
  for (int p = 0; p < KT; ++p)
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(x[p][0]), fabsf(x[p][1])), fmaxf(fabsf(x[p][2]), fabsf(x[p][3]))));
  return scale_exp(max_groups(mx));
}

// accumulators of output tile t start at bias * 2^(sx + s_t) (s_t: the image tile's exponent);
// after the products they are brought back to scale 1
template <int TO>
__device__ __forceinline__ void tiles_init(f32x4 (&y)[TO], const float* sV, int vb, int D,
                                           const int* sexp, int sx, int g) {
#pragma unroll
  for (int t = 0; t < TO; ++t) {
    const f32x4 b = vb >= 0 ? *reinterpret_cast<const f32x4*>(sV + vb * D + 16 * t + 4 * g)
                            : f32x4{0.f, 0.f, 0.f, 0.f};
    y[t] = b * ldexpf(1.f, sx + sexp[t]);
  }
}
template <int TO>
__device__ __forceinline__ void tiles_unscale(f32x4 (&y)[TO], const int* sexp, int sx) {
#pragma unroll
  for (int t = 0; t < TO; ++t) y[t] *= ldexpf(1.f, -(sx + sexp[t]));
}

template <int D, int ACT, bool RESID, bool AB, bool SAVE>
__global__ __launch_bounds__(kNodeWaves * 64, 2) void egnn_node_fwd_kernel(
    int64_t n_nodes, const float* __restrict__ h, const float* __restrict__ m_aggr,
    gmp_egnn_node_params P, const unsigned char* __restrict__ img, float eps,
    float* __restrict__ h_out, float* __restrict__ ab_out, float* __restrict__ xsave,
    float* __restrict__ rsave) {
  using I = NImg<D>;
  constexpr int T = D / 16;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sV = smem;                                           // NVN vectors
  int* sexp = reinterpret_cast<int*>(smem + NVN * D);         // tile exponents (<= 32)
  float* sscal = smem + NVN * D + 48;                         // scalars
  _Float16* hW = reinterpret_cast<_Float16*>(smem + NVN * D + 64);
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * (kNodeWaves * kNodeRT * 16);
  auto row_of = [&](int rt) { return row0 + (int64_t)(rt * kNodeWaves + wid) * 16 + i; };
  const int* gexp = reinterpret_cast<const int*>(img + I::off_exp);

  // ---- phase 1: x1 = act(LN1(W0 [h | m] + b0))
  copy_image(hW, img + I::off_w0, 2 * I::W0H * 2);
  if (threadIdx.x < I::T0 + I::T3 + I::TA) sexp[threadIdx.x] = gexp[threadIdx.x];
  if (threadIdx.x >= 64 && threadIdx.x < 128) {  // the LN1 bound (one wave): |act(LN1)| <= B
    unsigned gw = 0u, gb = 0u;
    for (int k = threadIdx.x - 64; k < D; k += 64) {
      gw = max(gw, __float_as_uint(fabsf(P.ln1_w[k])));
      gb = max(gb, __float_as_uint(fabsf(P.ln1_b[k])));
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      gw = max(gw, (unsigned)__shfl_xor((int)gw, off, 64));
      gb = max(gb, (unsigned)__shfl_xor((int)gb, off, 64));
    }
    if (threadIdx.x == 64) sscal[0] = sqrtf((float)D) * __uint_as_float(gw) + __uint_as_float(gb);
  }
  for (int k = threadIdx.x; k < D; k += blockDim.x) {
    sV[NV0_B0 * D + k] = P.b0[k];
    sV[NV0_G1 * D + k] = P.ln1_w[k];
    sV[NV0_BE1 * D + k] = P.ln1_b[k];
    sV[NV0_B3 * D + k] = P.b3[k];
    sV[NV0_G2 * D + k] = P.ln2_w[k];
    sV[NV0_BE2 * D + k] = P.ln2_b[k];
  }
  __syncthreads();
  constexpr bool XS = ACT == GMP_ACT_RELU;
  const int ex3 = scale_exp(sscal[0]);  // static input exponent of the W3 product
  for (int k = threadIdx.x; k < D; k += blockDim.x) {
    sV[NV0_G1S * D + k] = ldexpf(P.ln1_w[k], XS ? ex3 : 0);
    sV[NV0_BE1S * D + k] = ldexpf(P.ln1_b[k], XS ? ex3 : 0);
  }
  // (the vectors above are read after the next barrier)

  f32x4 keep[kNodeRT][T];  // x1 (phase 1 -> 2), h' (phase 2 -> 3)
#pragma unroll
  for (int rt = 0; rt < kNodeRT; ++rt) {
    const int64_t r = row_of(rt);
    const int64_t rc = r < n_nodes ? r : n_nodes - 1;
    f32x4 x[2 * T];
    load_row<D>(*reinterpret_cast<f32x4(*)[T]>(&x[0]), h + rc * D, g);
    load_row<D>(*reinterpret_cast<f32x4(*)[T]>(&x[T]), m_aggr + rc * D, g);
    const int sx = row_exp<2 * T>(x);
    f32x4 y[T];
    tiles_init<T>(y, sV, NV0_B0, D, sexp, sx, g);
    gemm_img<2 * T, T, false>(hW, I::LDH0, I::W0H, ldexpf(1.f, sx), x, y, i, g);
    tiles_unscale<T>(y, sexp, sx);
    const float r1 = ln_normalize<D, true>(y, eps);
    if (SAVE && r < n_nodes) {
      store_row<D>(xsave + r * D, y, g);
      if (g == 0) rsave[r] = r1;
    }
#pragma unroll
    for (int p = 0; p < T; ++p) keep[rt][p] = y[p];
  }
  __syncthreads();  // every wave is done with the W0 image

  // ---- phase 2: x2 = act(LN2(W3 x1 + b3)); h' = h + x2
  copy_image(hW, img + I::off_w3, 2 * I::W3H * 2);
  __syncthreads();
  const int* e3 = sexp + I::T0;
#pragma unroll
  for (int rt = 0; rt < kNodeRT; ++rt) {
    const int64_t r = row_of(rt);
    const int64_t rc = r < n_nodes ? r : n_nodes - 1;
    affine_act<D, ACT>(keep[rt], sV, NV0_G1S, NV0_BE1S, g);  // (relu: scaled by 2^ex3)
    f32x4 y[T];
    tiles_init<T>(y, sV, NV0_B3, D, e3, ex3, g);
    gemm_img<T, T, XS>(hW, I::LDH, I::W3H, ldexpf(1.f, ex3), keep[rt], y, i, g);
    tiles_unscale<T>(y, e3, ex3);
    const float r2 = ln_normalize<D, true>(y, eps);
    if (SAVE && r < n_nodes) {
      store_row<D>(xsave + ((size_t)n_nodes + r) * D, y, g);
      if (g == 0) rsave[n_nodes + r] = r2;
    }
    affine_act<D, ACT>(y, sV, NV0_G2, NV0_BE2, g);
    if constexpr (RESID) {
      f32x4 hh[T];
      load_row<D>(hh, h + rc * D, g);
#pragma unroll
      for (int p = 0; p < T; ++p) y[p] += hh[p];
    }
    if (r < n_nodes) store_row<D>(h_out + r * D, y, g);
#pragma unroll
    for (int p = 0; p < T; ++p) keep[rt][p] = y[p];
  }
  if constexpr (!AB) return;
  __syncthreads();

  // ---- phase 3: AB' = [h' W1a'^T | h' W1b'^T]
  copy_image(hW, img + I::off_wa, 2 * I::WAH * 2);
  __syncthreads();
  const int* ea = sexp + I::T0 + I::T3;
#pragma unroll
  for (int rt = 0; rt < kNodeRT; ++rt) {
    const int64_t r = row_of(rt);
    const int sx = row_exp<T>(keep[rt]);
    const float fx = ldexpf(1.f, sx);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 y[T];
      tiles_init<T>(y, sV, -1, D, ea + half * T, sx, g);
      gemm_img<T, T, false>(hW + half * D * I::LDH, I::LDH, I::WAH, fx, keep[rt], y, i, g);
      tiles_unscale<T>(y, ea + half * T, sx);
      if (r < n_nodes) store_row<D>(ab_out + r * 2 * D + half * D, y, g);
    }
  }
}

template <int D, int ACT, bool RESID, bool AB, bool SAVE>
int launch_node(int64_t N, const float* h, const float* m, const gmp_egnn_node_params& P,
                const unsigned char* img, float eps, float* h_out, float* ab_out, float* xsave,
                float* rsave, hipStream_t s) {
  auto k = egnn_node_fwd_kernel<D, ACT, RESID, AB, SAVE>;
  const size_t smem = NImg<D>::smem_bytes();
  int rc = prep_kernel(k, smem);
  if (rc) return rc;
  const int64_t rows = (int64_t)kNodeWaves * kNodeRT * 16;
  k<<<(unsigned)ceil_div(N, rows), kNodeWaves * 64, smem, s>>>(N, h, m, P, img, eps, h_out,
                                                                ab_out, xsave, rsave);
  return launch_status();
}

// ================================================================================== K15b backward
// The node update's backward in one launch (r06): from the upstream gradient g of h_out and the
// forward's saved x_hat1, x_hat2 / 1/std,
//   dz2 = g act'(x_hat2 w2 + b2), dpre2 = LN2'(dz2 w2);  dx1 = W3^T dpre2;
//   dz1 = dx1 act'(x_hat1 w1 + b1), dpre1 = LN1'(dz1 w1);
//   dh = W0[:, :d]^T dpre1 (+ g: residual), dm = W0[:, d:]^T dpre1,
// and the LayerNorm affine gradients [dw1 | db1 | dw2 | db2] = sum_rows [dz1 x1 | dz1 | dz2 x2 |
// dz2] as one partial row per workgroup (fixed order).  dpre1, dpre2 are written for the
// caller's weight sums (dW0 = dpre1^T [h | m], dW3 = dpre2^T act(LN1)).  Exact f32 MFMA; one
// 16-row tile per wave, 8 waves per workgroup; W3 then W0 pass through the same LDS region (two
// phases, the row tile's dpre1 and g carried in registers between them).  Replaces two
// LayerNorm-backward kernels with their partial-sum finishes, three library GEMMs and the
// residual add per layer (r05 trace: ~190 us of the ~9 ms EGNN step per layer).
constexpr int kNbWaves = 8;
template <int D>
__device__ __forceinline__ float slot(const f32x4 (&x)[D / 16], int s) { return x[s >> 2][s & 3]; }
template <int D>
struct NbCfg {
  static constexpr int LD3 = D + 4, LD0 = 2 * D + 4;
  static constexpr int W_FLOATS = D * LD0;                // the larger of W3 / W0 in LDS
  static constexpr int VEC = W_FLOATS;                    // ln1w, ln1b, ln2w, ln2b (4 D)
  static constexpr size_t smem_bytes() { return (size_t)(W_FLOATS + 4 * D) * sizeof(float); }
};

// y[slot(k)] += sum_o W[o][k0 + k] gin[slot(o)] with W row stride ldw
template <int D>
__device__ __forceinline__ void gemm_wtx_ld(const float* __restrict__ sW, int ldw,
                                            const f32x4 (&gin)[D / 16], f32x4 (&y)[D / 16], int i,
                                            int g) {
  constexpr int T = D / 16;
#pragma unroll
  for (int p = 0; p < T; ++p) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float* wrow = sW + (16 * p + 4 * g + c) * ldw + i;
      float a[T];
#pragma unroll
      for (int t = 0; t < T; ++t) a[t] = wrow[16 * t];
#pragma unroll
      for (int t = 0; t < T; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], gin[p][c], y[t], 0, 0, 0);
      gemm_fence();
    }
  }
}

// rows x cols floats of a row-major global matrix (row stride sld) into LDS (row stride ld),
// float4 loads issued together per thread
template <int ROWS, int COLS>
__device__ __forceinline__ void nb_copy(float* dst, int ld, const float* __restrict__ src,
                                        int64_t sld) {
  constexpr int N4 = ROWS * COLS / 4, PER = (N4 + kNbWaves * 64 - 1) / (kNbWaves * 64);
  f32x4 r[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int x = threadIdx.x + k * kNbWaves * 64;
    const int row = x / (COLS / 4), c4 = x - row * (COLS / 4);
    if (x < N4) r[k] = *reinterpret_cast<const f32x4*>(src + row * sld + 4 * c4);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int x = threadIdx.x + k * kNbWaves * 64;
    const int row = x / (COLS / 4), c4 = x - row * (COLS / 4);
    if (x < N4) *reinterpret_cast<f32x4*>(dst + row * ld + 4 * c4) = r[k];
  }
}

template <int D, int ACT, bool RES>
__global__ __launch_bounds__(kNbWaves * 64) void egnn_node_bwd_kernel(
    int64_t N, const float* __restrict__ gout, const float* __restrict__ xsave,
    const float* __restrict__ rsave, const float* __restrict__ W0, const float* __restrict__ W3,
    const float* __restrict__ ln1w, const float* __restrict__ ln1b,
    const float* __restrict__ ln2w, const float* __restrict__ ln2b, float* __restrict__ dh,
    float* __restrict__ dm, float* __restrict__ dpre1_out, float* __restrict__ dpre2_out,
    float* __restrict__ partials) {
  using C = NbCfg<D>;
  constexpr int T = D / 16, K = VecAcc<D>::K;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sV = smem + C::VEC;  // [ln1w | ln1b | ln2w | ln2b]
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const int wid = threadIdx.x >> 6;
  nb_copy<D, D>(smem, C::LD3, W3, D);
  for (int x = threadIdx.x; x < D; x += blockDim.x) {
    sV[x] = ln1w[x];
    sV[D + x] = ln1b[x];
    sV[2 * D + x] = ln2w[x];
    sV[3 * D + x] = ln2b[x];
  }
  const int64_t r0 = (int64_t)blockIdx.x * (kNbWaves * 16) + wid * 16;
  const bool valid = r0 + i < N;
  const int64_t n = valid ? r0 + i : N - 1;
  const float vf = valid ? 1.f : 0.f;
  const size_t ND = (size_t)N * D;
  f32x4 gr[T], xh[T], a[T];
  load_row<D>(gr, gout + n * D, g);
  load_row<D>(xh, xsave + ND + n * D, g);  // x_hat2
  const float rs2 = rsave[N + n], rs1 = rsave[n];
  float vacc[4][K];
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int k = 0; k < K; ++k) vacc[v][k] = 0.f;
  __syncthreads();
  // ---- LN2 + act backward: dz2 -> dpre2 (a)
#pragma unroll
  for (int p = 0; p < T; ++p) {
    const f32x4 w = vec4<D>(sV, 2, p, g), b = vec4<D>(sV, 3, p, g);
#pragma unroll
    for (int q = 0; q < 4; ++q) a[p][q] = vf * gr[p][q] * act_df<ACT>(xh[p][q] * w[q] + b[q]);
  }
  accumulate_vec<D>([&](int s) { return slot<D>(a, s) * slot<D>(xh, s); }, vacc[2], i);
  accumulate_vec<D>([&](int s) { return slot<D>(a, s); }, vacc[3], i);
#pragma unroll
  for (int p = 0; p < T; ++p) a[p] *= vec4<D>(sV, 2, p, g);
  ln_backward<D>(a, xh, rs2);
  if (valid) store_row<D>(dpre2_out + n * D, a, g);
  // ---- dx1 = W3^T dpre2 (xh <- dx1), then LN1 + act backward: dpre1 (a)
  load_row<D>(xh, xsave + n * D, g);  // x_hat1 (in flight during the product)
  f32x4 dx[T];
#pragma unroll
  for (int p = 0; p < T; ++p) dx[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  gemm_wtx_ld<D>(smem, C::LD3, a, dx, i, g);
#pragma unroll
  for (int p = 0; p < T; ++p) {
    const f32x4 w = vec4<D>(sV, 0, p, g), b = vec4<D>(sV, 1, p, g);
#pragma unroll
    for (int q = 0; q < 4; ++q) a[p][q] = vf * dx[p][q] * act_df<ACT>(xh[p][q] * w[q] + b[q]);
  }
  accumulate_vec<D>([&](int s) { return slot<D>(a, s) * slot<D>(xh, s); }, vacc[0], i);
  accumulate_vec<D>([&](int s) { return slot<D>(a, s); }, vacc[1], i);
#pragma unroll
  for (int p = 0; p < T; ++p) a[p] *= vec4<D>(sV, 0, p, g);
  ln_backward<D>(a, xh, rs1);
  if (valid) store_row<D>(dpre1_out + n * D, a, g);
  // ---- phase B: W0 replaces W3 in LDS; dh = W0[:, :d]^T dpre1 (+ g), dm = W0[:, d:]^T dpre1
  __syncthreads();
  nb_copy<D, 2 * D>(smem, C::LD0, W0, 2 * D);
  __syncthreads();
  if (!RES) {
#pragma unroll
    for (int p = 0; p < T; ++p) gr[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  gemm_wtx_ld<D>(smem, C::LD0, a, gr, i, g);
  if (valid) store_row<D>(dh + n * D, gr, g);
#pragma unroll
  for (int p = 0; p < T; ++p) gr[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  gemm_wtx_ld<D>(smem + D, C::LD0, a, gr, i, g);
  if (valid) store_row<D>(dm + n * D, gr, g);
  // ---- workgroup partial row of [dw1 | db1 | dw2 | db2] (waves in order: deterministic)
  __syncthreads();  // every wave is done with W0: reuse that LDS
  float* red = smem;  // [wave][4 D]
  if (acc_owner<D>(i)) {
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int k = 0; k < K; ++k) red[wid * 4 * D + v * D + featq(acc_slot<D>(i, k), g)] = vacc[v][k];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 4 * D; t += blockDim.x) {
    float sacc = 0.f;
    for (int w = 0; w < kNbWaves; ++w) sacc += red[w * 4 * D + t];
    partials[(int64_t)blockIdx.x * 4 * D + t] = sacc;
  }
}

template <int D, int ACT, bool RES>
int launch_node_bwd(int64_t N, const float* g, const float* xs, const float* rs, const float* W0,
                    const float* W3, const float* l1w, const float* l1b, const float* l2w,
                    const float* l2b, float* dh, float* dm, float* dp1, float* dp2, float* part,
                    hipStream_t s) {
  auto k = egnn_node_bwd_kernel<D, ACT, RES>;
  const size_t smem = NbCfg<D>::smem_bytes();
  int rc = prep_kernel_once((const void*)k, smem);
  if (rc) return rc;
  k<<<(unsigned)ceil_div(N, kNbWaves * 16), kNbWaves * 64, smem, s>>>(
      N, g, xs, rs, W0, W3, l1w, l1b, l2w, l2b, dh, dm, dp1, dp2, part);
  return launch_status();
}

size_t image_bytes(int64_t d) {
  return d == 128 ? NImg<128>::bytes : d == 64 ? NImg<64>::bytes : d == 32 ? NImg<32>::bytes : 0;
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

size_t gmp_egnn_node_image_bytes(int64_t d) { return image_bytes(d); }

int gmp_egnn_node_image_f32(int64_t d, int64_t n_layers, const gmp_egnn_node_params* params,
                            void* images, void* stream) {
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(n_layers >= 0 && (n_layers == 0 || (params && images)));
  GMP_CHECK_ARG(reinterpret_cast<uintptr_t>(images) % 16 == 0);
  for (int64_t l = 0; l < n_layers; ++l) {
    const gmp_egnn_node_params& P = params[l];
    GMP_CHECK_ARG(P.W0 && P.W3 && (P.W1n == nullptr || P.ld1 >= 2 * d));
  }
  hipStream_t s = as_stream(stream);
  for (int64_t l0 = 0; l0 < n_layers; l0 += 8) {
    NodeImgArgs A;
    A.n = (int)(n_layers - l0 < 8 ? n_layers - l0 : 8);
    for (int j = 0; j < 8; ++j) A.p[j] = params[l0 + (j < A.n ? j : 0)];
    unsigned char* out = reinterpret_cast<unsigned char*>(images) + (size_t)l0 * image_bytes(d);
    const int tl = (int)(d / 16 + d / 16 + 2 * d / 16);
    const unsigned grid = (unsigned)(A.n * tl);
    if (d == 128) egnn_node_image_kernel<128><<<grid, 256, 0, s>>>(A, out);
    else if (d == 64) egnn_node_image_kernel<64><<<grid, 256, 0, s>>>(A, out);
    else egnn_node_image_kernel<32><<<grid, 256, 0, s>>>(A, out);
    const int rc = launch_status();
    if (rc) return rc;
  }
  return GMP_OK;
}

int gmp_egnn_node_fwd_f32(int64_t n_nodes, int64_t d, const float* h, const float* m_aggr,
                          const gmp_egnn_node_params* params, const void* image, int act,
                          int residual, float ln_eps, float* h_out, float* ab_out,
                          float* save_xhat, float* save_rstd, void* stream) {
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(n_nodes >= 0 && (act == 0 || act == 1) && params && h_out && image);
  const gmp_egnn_node_params& P = *params;
  GMP_CHECK_ARG(P.b0 && P.ln1_w && P.ln1_b && P.b3 && P.ln2_w && P.ln2_b);
  GMP_CHECK_ARG((save_xhat == nullptr) == (save_rstd == nullptr));
  if (n_nodes == 0) return GMP_OK;
  GMP_CHECK_ARG(h && m_aggr && aligned16(h) && aligned16(m_aggr) && aligned16(h_out));
  GMP_CHECK_ARG(aligned16(image));
  GMP_CHECK_ARG(ab_out == nullptr || aligned16(ab_out));
  GMP_CHECK_ARG(save_xhat == nullptr || aligned16(save_xhat));
  if (egnn_f32()) return GMP_ERR_UNSUPPORTED;  // (the exact-f32 A/B mode: the caller's ops)
  hipStream_t s = as_stream(stream);
  const unsigned char* img = reinterpret_cast<const unsigned char*>(image);
  int rc = GMP_OK;
  const bool ab = ab_out != nullptr, sv = save_xhat != nullptr, res = residual != 0;
#define LAUNCH_NODE4(DD, AA, RR, BB, SS)                                                       \
  rc = launch_node<DD, AA, RR, BB, SS>(n_nodes, h, m_aggr, P, img, ln_eps, h_out, ab_out, \
                                       save_xhat, save_rstd, s)
#define LAUNCH_NODE3(DD, AA)                                                               \
  if (res) { if (ab) { if (sv) LAUNCH_NODE4(DD, AA, true, true, true);                   \
                       else LAUNCH_NODE4(DD, AA, true, true, false); }                   \
             else { if (sv) LAUNCH_NODE4(DD, AA, true, false, true);                     \
                    else LAUNCH_NODE4(DD, AA, true, false, false); } }                   \
  else { if (ab) { if (sv) LAUNCH_NODE4(DD, AA, false, true, true);                      \
                   else LAUNCH_NODE4(DD, AA, false, true, false); }                      \
         else { if (sv) LAUNCH_NODE4(DD, AA, false, false, true);                        \
                else LAUNCH_NODE4(DD, AA, false, false, false); } }
#define LAUNCH_NODE2(DD) if (act == 0) { LAUNCH_NODE3(DD, 0) } else { LAUNCH_NODE3(DD, 1) }
  if (d == 128) { LAUNCH_NODE2(128) } else if (d == 64) { LAUNCH_NODE2(64) } else { LAUNCH_NODE2(32) }
#undef LAUNCH_NODE2
#undef LAUNCH_NODE3
#undef LAUNCH_NODE4
  return rc;
}

int64_t gmp_egnn_node_bwd_partial_rows(int64_t n_nodes) {
  return n_nodes > 0 ? ceil_div(n_nodes, kNbWaves * 16) : 0;
}

int gmp_egnn_node_bwd_f32(int64_t n_nodes, int64_t d, int act, int residual, const float* grad_h,
                          const float* save_xhat, const float* save_rstd, const float* W0,
                          const float* W3, const float* ln1_w, const float* ln1_b,
                          const float* ln2_w, const float* ln2_b, float* dh, float* dm,
                          float* dpre1, float* dpre2, float* partials, void* stream) {
  if (!(d == 32 || d == 64 || d == 128)) return GMP_ERR_UNSUPPORTED;
  GMP_CHECK_ARG(n_nodes >= 0 && (act == 0 || act == 1));
  if (n_nodes == 0) return GMP_OK;
  GMP_CHECK_ARG(grad_h && save_xhat && save_rstd && W0 && W3 && ln1_w && ln1_b && ln2_w &&
                ln2_b && dh && dm && dpre1 && dpre2 && partials);
  GMP_CHECK_ARG(aligned16(grad_h) && aligned16(save_xhat) && aligned16(W0) && aligned16(W3) &&
                aligned16(dh) && aligned16(dm) && aligned16(dpre1) && aligned16(dpre2));
  hipStream_t s = as_stream(stream);
  int rc;
#define LNB(DD, AA, RR)                                                                        \
  rc = launch_node_bwd<DD, AA, RR>(n_nodes, grad_h, save_xhat, save_rstd, W0, W3, ln1_w, ln1_b, \
                                   ln2_w, ln2_b, dh, dm, dpre1, dpre2, partials, s)
#define LNB2(DD)                                                             \
  if (act == 0) { if (residual) LNB(DD, 0, true); else LNB(DD, 0, false); } \
  else { if (residual) LNB(DD, 1, true); else LNB(DD, 1, false); }
  if (d == 128) { LNB2(128) } else if (d == 64) { LNB2(64) } else { LNB2(32) }
#undef LNB2
#undef LNB
  return rc;
}

}  // extern "C"
