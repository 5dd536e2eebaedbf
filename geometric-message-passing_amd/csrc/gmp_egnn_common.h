// Device helpers shared by the EGNN kernels (K4 gmp_egnn.hip, K15 gmp_egnn_node.hip): the lane
// layout, the 2-plane fp16 (HF) product machinery, LayerNorm / activation pieces, segmented sums.
// See gmp_egnn.hip for the design notes.
#pragma once
#include <stdlib.h>

#include "gmp_common.h"

namespace gmp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// One workgroup per CU (W2 + W3 in LDS).  Forward: 12 waves (<= 168 VGPRs -> 3 per SIMD; the HF
// form fits since r05's static scales and fma_mix splits, 8 waves before); backward: 8 waves
// (<= 256 VGPRs -> 2 per SIMD).
constexpr int kFwdWaves = 12;
template <bool HF>
constexpr int fwd_waves() { return kFwdWaves; }
constexpr int kBwdWaves = 8;

template <int D>
struct Cfg {
  static constexpr int T = D / 16;   // f32x4 groups per lane = 16-feature MFMA tiles
  static constexpr int N = D / 4;    // feature slots per lane
  static constexpr int LDW = D + 4;  // LDS row stride of W (floats)
};

// feature held by lane group g in slot s = 4p + c
__device__ __forceinline__ constexpr int featq(int s, int g) { return 16 * (s >> 2) + 4 * g + (s & 3); }

// LDS vectors.  The first NVB are the parameters as given; the HF path adds pre-scaled copies
// (DESIGN.md "K4 r05"): V_B2S / V_B3S = the centred biases times 2^(ex + sw) (the products'
// accumulator scale), V_LN1WS / V_LN1BS = the first LayerNorm's affine times 2^ex2 (relu is
// positively homogeneous, so act(x w 2^ex + b 2^ex) = 2^ex act(x w + b) exactly; y1 feeds only
// the W2 product).  (The message m = act(LN2) is aggregated as well, so it stays unscaled.)
enum VecId {
  V_W1D = 0, V_B1, V_LN1W, V_LN1B, V_B2, V_LN2W, V_LN2B, V_B3, V_LN3W, V_LN3B, V_W4, NVB,
  V_B2S = NVB, V_B3S, V_LN1WS, V_LN1BS, NV
};

template <int D>
constexpr int carry_stride() { return D / 4 + 4; }

// HF path: W as hi / lo fp16 planes of W 2^sw, columns in the MFMA k order (see gemm_h2), row
// stride d + 16 halfs (below)
template <int D>
struct HCfg {
  // row stride d + 16 halfs (288 B at d = 128; 16-byte units = 2 mod 16): the four 16-lane
  // groups of a ds_read_b128 A read hit 64 distinct banks and the transposed 8-byte reads of the
  // x_hat3 recompute are 2-way (the floor for 8-byte pieces of 16-byte-aligned rows).  r03 / r04
  // used d + 8 (272 B): 2-way / 4-way, 0.34 / 0.51 of the forward / backward LDS cycles in bank
  // conflicts (SQ counters, r04).
  static constexpr int LDH = D + 16;
  static constexpr int PLANE = D * LDH;  // halfs
  static constexpr int MAT = 2 * PLANE;  // halfs per matrix (= floats for two matrices)
};

// LDS, f32 path: W2 | W3 (rows of d + 4 floats) | NV vectors + 12 | per-wave carries
// [wave][g][d/4 + 4].  HF path: NV vectors + 12 scalars (scale exponents, max scratch) |
// carries | W2 planes | W3 planes — the vectors first, so their reads fold into the 16-bit
// ds_read offset of one base register instead of holding one address register each.
template <int D, int NW, bool HF>
constexpr size_t smem_vec_off() { return HF ? 0 : (size_t)2 * D * Cfg<D>::LDW; }
template <int D, int NW, bool HF>
constexpr size_t smem_carry_off() { return smem_vec_off<D, NW, HF>() + NV * D + 12; }
template <int D, int NW, bool HF>
constexpr size_t smem_mats_off() {
  return HF ? smem_carry_off<D, NW, HF>() + (size_t)NW * 4 * carry_stride<D>() : 0;
}
template <int D, int NW, bool HF>
constexpr size_t smem_total() {
  return (HF ? smem_mats_off<D, NW, HF>() + HCfg<D>::MAT
             : smem_carry_off<D, NW, HF>() + (size_t)NW * 4 * carry_stride<D>()) * sizeof(float);
}

template <int ACT>
__device__ __forceinline__ float act_f(float z) {
  if (ACT == GMP_ACT_RELU) return z > 0.f ? z : 0.f;
  const float sg = 1.f / (1.f + __expf(-z));
  return z * sg;
}
template <int ACT>
__device__ __forceinline__ float act_df(float z) {
  if (ACT == GMP_ACT_RELU) return z > 0.f ? 1.f : 0.f;
  const float sg = 1.f / (1.f + __expf(-z));
  return sg * (1.f + z * (1.f - sg));
}

// ---------------------------------------------------------------------------------- LDS setup
// TRANSPOSE (backward): W2^T / W3^T, so the transposed products read 16-byte rows too
template <int D, bool TRANSPOSE = false>
__device__ void load_params_to_lds(float* smem, const gmp_egnn_params& P) {
  constexpr int LDW = Cfg<D>::LDW;
  float* sW2 = smem;
  float* sW3 = smem + D * LDW;
  float* sV = smem + 2 * D * LDW;
  for (int i = threadIdx.x; i < D * D / 4; i += blockDim.x) {
    const int o = (4 * i) / D, k = (4 * i) % D;
    const float4 a = reinterpret_cast<const float4*>(P.W2)[i];
    const float4 b = reinterpret_cast<const float4*>(P.W3)[i];
    if (TRANSPOSE) {
      sW2[(k + 0) * LDW + o] = a.x; sW2[(k + 1) * LDW + o] = a.y;
      sW2[(k + 2) * LDW + o] = a.z; sW2[(k + 3) * LDW + o] = a.w;
      sW3[(k + 0) * LDW + o] = b.x; sW3[(k + 1) * LDW + o] = b.y;
      sW3[(k + 2) * LDW + o] = b.z; sW3[(k + 3) * LDW + o] = b.w;
    } else {
      *reinterpret_cast<float4*>(sW2 + o * LDW + k) = a;
      *reinterpret_cast<float4*>(sW3 + o * LDW + k) = b;
    }
  }
  const float* vsrc[NVB] = {P.w1d, P.b1, P.ln1_w, P.ln1_b, P.b2, P.ln2_w,
                            P.ln2_b, P.b3, P.ln3_w, P.ln3_b, P.w4};
  for (int i = threadIdx.x; i < NVB * D; i += blockDim.x) sV[i] = vsrc[i / D][i % D];
}

// exponent s with max|v| 2^s < 2^15 (fp16 range with headroom), clamped to [-60, 60]
__device__ __forceinline__ int scale_exp(float mx) {
  if (!(mx > 0.f) || !(mx < 3.0e38f)) return 0;
  int e;
  (void)frexpf(mx, &e);  // mx < 2^e
  const int s = 15 - e;
  return s < -60 ? -60 : (s > 60 ? 60 : s);
}

// HF: hi / lo planes of W2 and W3 (or their transposes) scaled by 2^sw (one exponent per matrix
// from a block-wide max |W|, kept as floats after the vectors).  Natural column k = 16 tt + 4 g
// + q goes to position 32 (tt >> 1) + 8 g + 4 (tt & 1) + q: the 8 halfs a lane feeds one
// 16x16x32 MFMA (k = 8 g + j of block p) are then the slots x[2p][0..3], x[2p + 1][0..3] it
// already holds.
__device__ __forceinline__ int hf_pos(int k) {
  const int tt = k >> 4, gg = (k >> 2) & 3, q = k & 3;
  return 32 * (tt >> 1) + 8 * gg + 4 * (tt & 1) + q;
}
// the effective static input exponent of a forward product: sx clamped so that sx + sw stays in
// [-100, 100] (the accumulator scale 2^(sx + sw) and its inverse are normal floats)
__device__ __forceinline__ int clamp_in_exp(int sx, int sw) {
  return sx < -100 - sw ? -100 - sw : (sx > 100 - sw ? 100 - sw : sx);
}

// CMASK bit m: centre matrix m (0: W2, 1: W3) and its bias over the output dimension,
// W_c[o][k] = W[o][k] - mean_o W[o][k], b_c = b - mean(b).  The centred product's outputs then
// have zero mean, LN(W_c x + b_c) = LN(W x + b) exactly in real arithmetic, and the LayerNorm
// after it needs no mean pass (ln_rms).  The backward needs no change: LayerNorm's input gradient
// has zero mean, so W_c^T dpre = W^T dpre and dW = dpre x^T are the original ones.
// `scratch` (2 d + 2 floats: the column and bias means) is the carry area, unused until the loop.
template <int D, bool TRANSPOSE, int CMASK, int ACT>
__device__ void load_params_hf(float* sV, _Float16* hW, float* scratch, const gmp_egnn_params& P) {
  using H = HCfg<D>;
  // scalars after the vectors: [0] [1] exponents of W2 / W3, [2] [3] the static (clamped) input
  // exponents ex2 / ex3 of the forward products (below), [4..9] max scratch
  unsigned* mxw = reinterpret_cast<unsigned*>(sV + NV * D + 4);
  if (threadIdx.x < 6) mxw[threadIdx.x] = 0u;
  __syncthreads();
  if (threadIdx.x < 2 * D) {  // column (mat, k): mean over the output rows and max |W| (fixed order)
    const int mat = threadIdx.x / D, k = threadIdx.x - mat * D;
    const float* W = mat ? P.W3 : P.W2;
    float s = 0.f, m = 0.f;
#pragma unroll 8
    for (int o = 0; o < D; ++o) {
      const float w = W[o * D + k];
      s += w;
      m = fmaxf(m, fabsf(w));
    }
    const float mean = ((CMASK >> mat) & 1) ? s * (1.f / D) : 0.f;
    scratch[threadIdx.x] = mean;
    atomicMax(&mxw[mat], __float_as_uint(m + fabsf(mean)));  // >= max |W_c| (a bound suffices)
  } else if (threadIdx.x < 2 * D + 64) {  // bias means (one wave, fixed-order butterfly)
    const int l = threadIdx.x - 2 * D;
    float a = 0.f, b = 0.f;
    for (int k = l; k < D; k += 64) {
      a += P.b2[k];
      b += P.b3[k];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      a += __shfl_xor(a, off, 64);
      b += __shfl_xor(b, off, 64);
    }
    if (l == 0) {
      scratch[2 * D] = (CMASK & 1) ? a * (1.f / D) : 0.f;
      scratch[2 * D + 1] = (CMASK & 2) ? b * (1.f / D) : 0.f;
    }
  }
  // forward inputs of W2 / W3 are act(x_hat * w + b) of a LayerNorm over d features:
  // |x_hat| <= sqrt(d - 1), |act(z)| <= |z| (relu, silu) => |input| <= sqrt(d) max|w| + max|b|
  if (threadIdx.x >= 2 * D + 64 && threadIdx.x < 2 * D + 128) {
    unsigned a = 0u, b = 0u, c = 0u, e = 0u;
    for (int k = threadIdx.x - 2 * D - 64; k < D; k += 64) {
      a = max(a, __float_as_uint(fabsf(P.ln1_w[k])));
      b = max(b, __float_as_uint(fabsf(P.ln1_b[k])));
      c = max(c, __float_as_uint(fabsf(P.ln2_w[k])));
      e = max(e, __float_as_uint(fabsf(P.ln2_b[k])));
    }
    atomicMax(&mxw[2], a);
    atomicMax(&mxw[3], b);
    atomicMax(&mxw[4], c);
    atomicMax(&mxw[5], e);
  }
  __syncthreads();
  const int s2 = scale_exp(__uint_as_float(mxw[0])), s3 = scale_exp(__uint_as_float(mxw[1]));
  const float rd = sqrtf((float)D);
  const int ex2 = clamp_in_exp(scale_exp(rd * __uint_as_float(mxw[2]) + __uint_as_float(mxw[3])), s2);
  const int ex3 = clamp_in_exp(scale_exp(rd * __uint_as_float(mxw[4]) + __uint_as_float(mxw[5])), s3);
  __syncthreads();  // (the scratch words are overwritten below)
#pragma unroll 8
  for (int i = threadIdx.x; i < 2 * D * D; i += blockDim.x) {
    const int mat = i / (D * D), e = i - mat * D * D;
    const int o = e / D, k = e - o * D;  // W[o][k]
    const float w = ldexpf((mat ? P.W3 : P.W2)[e] - scratch[mat * D + k], mat ? s3 : s2);
    const int r = TRANSPOSE ? k : o, c = TRANSPOSE ? o : k;
    const _Float16 hi = (_Float16)w;
    _Float16* dst = hW + mat * H::MAT + r * H::LDH + hf_pos(c);
    dst[0] = hi;
    dst[H::PLANE] = (_Float16)(w - (float)hi);
  }
  const float* vsrc[NVB] = {P.w1d, P.b1, P.ln1_w, P.ln1_b, P.b2, P.ln2_w,
                            P.ln2_b, P.b3, P.ln3_w, P.ln3_b, P.w4};
  for (int i = threadIdx.x; i < NVB * D; i += blockDim.x) sV[i] = vsrc[i / D][i % D];
  // pre-scaled copies: accumulator biases at 2^(ex + sw); relu inputs at 2^ex (silu is not
  // homogeneous: its inputs are scaled in the operand split instead)
  for (int k = threadIdx.x; k < D; k += blockDim.x) {
    sV[V_B2S * D + k] = ldexpf(P.b2[k] - scratch[2 * D], ex2 + s2);
    sV[V_B3S * D + k] = ldexpf(P.b3[k] - scratch[2 * D + 1], ex3 + s3);
    const int e1 = ACT == GMP_ACT_RELU ? ex2 : 0;
    sV[V_LN1WS * D + k] = ldexpf(P.ln1_w[k], e1);
    sV[V_LN1BS * D + k] = ldexpf(P.ln1_b[k], e1);
  }
  if (threadIdx.x == 0) {
    sV[NV * D + 0] = (float)s2;
    sV[NV * D + 1] = (float)s3;
    sV[NV * D + 2] = (float)ex2;
    sV[NV * D + 3] = (float)ex3;
  }
}

// this lane's 4 consecutive slots (4p..4p+3) of LDS vector v
template <int D>
__device__ __forceinline__ f32x4 vec4(const float* sV, int v, int p, int g) {
  return *reinterpret_cast<const f32x4*>(sV + v * D + 16 * p + 4 * g);
}

template <int D>
__device__ __forceinline__ void load_vec(f32x4 (&x)[D / 16], const float* sV, int v, int g) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p) x[p] = vec4<D>(sV, v, p, g);
}

// row of a (rows, d) global tensor: this lane's slots
template <int D>
__device__ __forceinline__ void load_row(f32x4 (&x)[D / 16], const float* __restrict__ row, int g) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p) x[p] = *reinterpret_cast<const f32x4*>(row + 16 * p + 4 * g);
}
template <int D>
__device__ __forceinline__ void store_row(float* __restrict__ row, const f32x4 (&x)[D / 16], int g) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p) *reinterpret_cast<f32x4*>(row + 16 * p + 4 * g) = x[p];
}
// streaming store (per-edge tensors consumed by later kernels: keep them out of L2)
template <int D>
__device__ __forceinline__ void stream_row(float* __restrict__ row, const f32x4 (&x)[D / 16], int g) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p)
    __builtin_nontemporal_store(x[p], reinterpret_cast<f32x4*>(row + 16 * p + 4 * g));
}

// ---------------------------------------------------------------------------------- windows
// Predicated stores without branches: a buffer descriptor over the rows one 16-edge chunk can
// touch (wave-uniform base row r0, n rows), and per-lane byte offsets that are pushed out of
// the window (kOob) for lanes that must not store — the range check drops those.  With no
// store under a divergent branch the compiler's wait before the next chunk's prefetched ids
// is a counted vmcnt, not a drain of this chunk's stores.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kOob = 0x40000000u;  // > any window (<= 16 rows of <= 512 B)
constexpr int kAuxNT = 2;               // nt: streaming per-edge rows, keep them out of L2

__device__ __forceinline__ rsrc_t rows_window(const float* base, int r0, int n, int ld) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base) + (size_t)(unsigned)r0 * ld, 0,
                                           n * ld * 4, 0x00020000);
}
template <int D, int AUX>
__device__ __forceinline__ void store_row_w(rsrc_t w, unsigned off, const f32x4 (&x)[D / 16], int g) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, x[p]),
                                           w, off + (16 * p + 4 * g) * 4, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void store3_w(rsrc_t w, unsigned off, float a, float b, float c) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a), w, off, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(b), w, off + 4, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(c), w, off + 8, 0, AUX);
}

// ---------------------------------------------------------------------------------- MFMA GEMMs
// gemm_fence() bounds how far the scheduler may hoist LDS operand reads (register pressure).
__device__ __forceinline__ void gemm_fence() { __builtin_amdgcn_sched_barrier(0); }
// y[slot(o)] += sum_k W[o][k] x[slot(k)]   (W row-major [o][k] in LDS; lane i = edge = l & 15)
// SPLIT > 1: the output tiles in SPLIT groups, so only T/SPLIT A rows are live at a time
// (register pressure in the backward)
template <int D, int SPLIT = 1>
__device__ __forceinline__ void gemm_wx(const float* __restrict__ sW, const f32x4 (&x)[D / 16],
                                        f32x4 (&y)[D / 16], int i, int g) {
  constexpr int T = Cfg<D>::T, LDW = Cfg<D>::LDW;
  constexpr int TS = (T % SPLIT == 0) ? T / SPLIT : T;
#pragma unroll
  for (int p = 0; p < T; ++p) {  // contraction block: features 16p + 4g' + c
#pragma unroll
    for (int t0 = 0; t0 < T; t0 += TS) {
      f32x4 a[TS];
#pragma unroll
      for (int t = 0; t < TS; ++t)
        a[t] = *reinterpret_cast<const f32x4*>(sW + (16 * (t0 + t) + i) * LDW + 16 * p + 4 * g);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < TS; ++t)
          y[t0 + t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][c], x[p][c], y[t0 + t], 0, 0, 0);
      gemm_fence();
    }
  }
}

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kTilesPerFence = 2;  // HF products: output tiles between scheduling fences

// 2-plane fp16 split of 8 (already scaled) floats a[0..3], b[0..3]: hi = RNE fp16 of v, lo = RNE
// fp16 of v - hi (exact in f32, so one rounding: bitwise (_Float16)(v - (float)hi)).  hi by
// v_cvt_pk_f16_f32 (two values per instruction); lo by v_fma_mix{lo,hi}_f16 v * 1.0 - hi, which
// reads the fp16 hi straight from the packed pair — 3 instructions per pair where the compiler's
// form (two cvt_f32_f16, a packed subtract, a second cvt_pk) takes 5.  The trailing s_nop 1 is the
// VALU-write -> MFMA-operand wait the compiler does not insert after an asm statement
// (cdna_hip_programming.md §5.7 item 2).
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, h16x8& bh, h16x8& bl) {
  const h16x2 p0 = {(_Float16)a[0], (_Float16)a[1]}, p1 = {(_Float16)a[2], (_Float16)a[3]};
  const h16x2 p2 = {(_Float16)b[0], (_Float16)b[1]}, p3 = {(_Float16)b[2], (_Float16)b[3]};
  const unsigned u0 = __builtin_bit_cast(unsigned, p0), u1 = __builtin_bit_cast(unsigned, p1);
  const unsigned u2 = __builtin_bit_cast(unsigned, p2), u3 = __builtin_bit_cast(unsigned, p3);
  unsigned l0, l1, l2, l3;
  // (1.0 from a register: an inline constant's interpretation in a mixed-precision operand slot
  // is not something to rely on)
  const float one = 1.0f;
  asm("v_fma_mixlo_f16 %0, %4, %16, -%12 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %5, %16, -%12 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %1, %6, %16, -%13 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %7, %16, -%13 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %2, %8, %16, -%14 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %2, %9, %16, -%14 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %3, %10, %16, -%15 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %3, %11, %16, -%15 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "s_nop 1"
      : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]),
        "v"(u0), "v"(u1), "v"(u2), "v"(u3), "s"(one));
  bh = __builtin_bit_cast(h16x8, (u32x4){u0, u1, u2, u3});
  bl = __builtin_bit_cast(h16x8, (u32x4){l0, l1, l2, l3});
}

__device__ __forceinline__ float max_groups(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// HF: y[slot(o)] += sum_k W[o][k] x[slot(k)] on the f16 MFMA.  x of this lane's edge is scaled
// by 2^sx (max |x| 2^sx < 2^15, from the 4 lane groups of the edge), W sits in LDS as planes of
// W 2^sw; y is brought to scale 2^(sx + sw), accumulated with lo*hi + hi*lo + hi*hi per k block
// (22-bit operands; the dropped lo*lo term is ~2^-22 relative) and scaled back.  Power-of-two
// scalings are exact, so the f32 accumulation rounds as on unscaled values.
// DYN: the x exponent from this edge's max |x| (backward: gradients have no a-priori bound);
// otherwise sx_static (forward: bounded LayerNorm-activation inputs, load_params_hf) — the
// per-edge reduction ahead of the products costs live registers the forward does not have.
template <int D, bool DYN>
__device__ __forceinline__ void gemm_h2(const _Float16* __restrict__ hW, int sw, int sx_static,
                                        const f32x4 (&x)[D / 16], f32x4 (&y)[D / 16], int i,
                                        int g) {
  using H = HCfg<D>;
  constexpr int T = D / 16, PB = D / 32;
  int sx = sx_static;
  if constexpr (DYN) {
    float mx = 0.f;
#pragma unroll
    for (int p = 0; p < T; ++p)
#pragma unroll
      for (int c = 0; c < 4; ++c) mx = fmaxf(mx, fabsf(x[p][c]));
    sx = scale_exp(max_groups(mx));
  }
  sx = clamp_in_exp(sx, sw);
  const float fx = ldexpf(1.f, sx), up = ldexpf(1.f, sx + sw), down = ldexpf(1.f, -(sx + sw));
#pragma unroll
  for (int t = 0; t < T; ++t) y[t] *= up;
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    h16x8 bh, bl;
    split8(x[2 * p] * fx, x[2 * p + 1] * fx, bh, bl);
#pragma unroll
    for (int t = 0; t < T; ++t) {
      // compiler-level fence: keeps the A reads from being hoisted ahead of the operand split
      // (and out of registers' reach) as a block
      if (t % kTilesPerFence == 0) asm volatile("" ::: "memory");
      const _Float16* row = hW + (16 * t + i) * H::LDH + 32 * p + 8 * g;
      const h16x8 ah = *reinterpret_cast<const h16x8*>(row);
      const h16x8 al = *reinterpret_cast<const h16x8*>(row + H::PLANE);
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, y[t], 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
      y[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
      if (t % kTilesPerFence == kTilesPerFence - 1) gemm_fence();  // bounds hoisted reads
    }
  }
#pragma unroll
  for (int t = 0; t < T; ++t) y[t] *= down;
}

// HF forward product with static scales (r05): y (the accumulators, initialised with the bias
// pre-scaled to 2^(ex + sw): V_B2S / V_B3S) += W_c x at scale 2^(ex + sw), and it STAYS at that
// scale: the LayerNorm that follows folds 2^-(ex + sw) into its 1/std (ln_rms), so there is no
// scale-up / scale-down pass over the accumulators.  XS: x already carries 2^ex (relu: the
// affine's pre-scaled vectors); otherwise (silu) it is scaled here.  Planes, operands and MFMA
// order are gemm_h2's: bitwise the r04 products.
constexpr int kOperandPrefetch = 1;  // LDS A-operand prefetch distance (k blocks) of gemm_h2s
template <int D, bool XS>
__device__ __forceinline__ void gemm_h2s(const _Float16* __restrict__ hW, int ex,
                                         const f32x4 (&x)[D / 16], f32x4 (&y)[D / 16], int i,
                                         int g) {
  using H = HCfg<D>;
  constexpr int T = D / 16, PB = D / 32, NQ = PB * T, PD = kOperandPrefetch;
  const float fx = ldexpf(1.f, ex);
  // the A operand (W planes) of step q + PD is read from LDS while step q's MFMAs run
  const _Float16* base = hW + i * H::LDH + 8 * g;
  h16x8 ah[PD + 1], al[PD + 1];
#pragma unroll
  for (int q = 0; q < PD; ++q) {
    const _Float16* row = base + 16 * (q % T) * H::LDH + 32 * (q / T);
    ah[q] = *reinterpret_cast<const h16x8*>(row);
    al[q] = *reinterpret_cast<const h16x8*>(row + H::PLANE);
  }
  h16x8 bh, bl;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int p = q / T, t = q % T;
    if (t == 0) {
      if constexpr (XS) split8(x[2 * p], x[2 * p + 1], bh, bl);
      else split8(x[2 * p] * fx, x[2 * p + 1] * fx, bh, bl);
    }
    if (q + PD < NQ) {
      const int qn = q + PD;
      const _Float16* row = base + 16 * (qn % T) * H::LDH + 32 * (qn / T);
      ah[qn % (PD + 1)] = *reinterpret_cast<const h16x8*>(row);
      al[qn % (PD + 1)] = *reinterpret_cast<const h16x8*>(row + H::PLANE);
    }
    const int b = q % (PD + 1);
    f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[b], bh, y[t], 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], bl, acc, 0, 0, 0);
    y[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], bh, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// HF, the FORWARD product y[slot(o)] += sum_k W[o][k] x[slot(k)] read from the TRANSPOSED planes
// (rows k, columns hf_pos(o): the backward's LDS image) with ds_read_b64_tr_b16.  Per 16-lane
// group g and k block p, two transposed reads per plane (lane 4q + c of the group supplies row
// 32p + 4g + q resp. 32p + 16 + 4g + q, physical columns hf_pos(16t + 4c .. 4c + 3), which are
// contiguous) deliver to lane i the 8 halfs W[16t + i][32p + 16h + 4g + q] of the A fragment
// that gemm_h2 reads as one row.  Same planes, scales and MFMA order: bitwise the forward's
// product (the backward recomputes x_hat3 instead of reading it, gmp_egnn_set_save_xhat3).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ h16x4 lds_tr16(const _Float16* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(h16x4, v);
}

template <int D, bool XS>
__device__ __forceinline__ void gemm_h2s_tr(const _Float16* __restrict__ hWt, int ex,
                                            const f32x4 (&x)[D / 16], f32x4 (&y)[D / 16],
                                            int lane, int g) {
  using H = HCfg<D>;
  constexpr int T = D / 16, PB = D / 32;
  const float fx = ldexpf(1.f, ex);
  const int q = (lane & 15) >> 2, c = lane & 3;
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    h16x8 bh, bl;
    if constexpr (XS) split8(x[2 * p], x[2 * p + 1], bh, bl);
    else split8(x[2 * p] * fx, x[2 * p + 1] * fx, bh, bl);
    const _Float16* rowk = hWt + (32 * p + 4 * g + q) * H::LDH + 8 * c;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if (t % kTilesPerFence == 0) asm volatile("" ::: "memory");
      const _Float16* a0 = rowk + 32 * (t >> 1) + 4 * (t & 1);
      const _Float16* a1 = a0 + 16 * H::LDH;
      const h16x4 h0 = lds_tr16(a0), h1 = lds_tr16(a1);
      const h16x4 l0 = lds_tr16(a0 + H::PLANE), l1 = lds_tr16(a1 + H::PLANE);
      const h16x8 ah = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      const h16x8 al = {l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, y[t], 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
      y[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
      if (t % kTilesPerFence == kTilesPerFence - 1) gemm_fence();
    }
  }
}

// y[slot(k)] += sum_o W[o][k] gin[slot(o)]   (transposed product for the backward)
template <int D>
__device__ __forceinline__ void gemm_wtx(const float* __restrict__ sW, const f32x4 (&gin)[D / 16],
                                         f32x4 (&y)[D / 16], int i, int g) {
  constexpr int T = Cfg<D>::T, LDW = Cfg<D>::LDW;
#pragma unroll
  for (int p = 0; p < T; ++p) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float* wrow = sW + (16 * p + 4 * g + c) * LDW + i;
      float a[T];
#pragma unroll
      for (int t = 0; t < T; ++t) a[t] = wrow[16 * t];
#pragma unroll
      for (int t = 0; t < T; ++t) y[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], gin[p][c], y[t], 0, 0, 0);
      gemm_fence();
    }
  }
}

// ---------------------------------------------------------------------------------- cross-lane
// All in-wave exchanges are VALU (DPP, permlane swaps), never ds_bpermute: the LDS pipe stays
// free for the W operand reads.
// DPP within a 16-lane row; lanes without a source get 0
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  // bound_ctrl: lanes without a source read 0, so no "old" operand has to be materialised
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// the partner of lane i (within its 16-lane row) at reduce-scatter level M: i^8 (row_ror:8),
// i^7 (row_half_mirror: flips bit 2 like i^4), i^2, i^1 (quad_perm)
template <int M>
__device__ __forceinline__ float rs_partner(float v) {
  if constexpr (M == 8) return dpp<0x128>(v);
  else if constexpr (M == 4) return dpp<0x141>(v);
  else if constexpr (M == 2) return dpp<0x4E>(v);
  else return dpp<0xB1>(v);
}
// sum over the 4 lane groups of an edge (lanes l, l^16, l^32, l^48): permlane16/32 swaps of
// v with itself return {v, partner} in some order, so r[0] + r[1] = v + partner
__device__ __forceinline__ float sum_groups(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// ---------------------------------------------------------------------------------- LayerNorm

// in place: x <- (x - mean) * rstd  (x_hat); returns rstd.  Two-pass statistics.
template <int D, bool RSQ = false>
__device__ __forceinline__ float ln_normalize(f32x4 (&x)[D / 16], float eps) {
  constexpr int T = D / 16;
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < T; ++p) s += (x[p][0] + x[p][1]) + (x[p][2] + x[p][3]);
  const float mean = sum_groups(s) * (1.f / D);
  float v = 0.f;
#pragma unroll
  for (int p = 0; p < T; ++p) {
    x[p] -= mean;
    v += x[p][0] * x[p][0] + x[p][1] * x[p][1] + x[p][2] * x[p][2] + x[p][3] * x[p][3];
  }
  const float var = sum_groups(v) * (1.f / D) + eps;
  const float rstd = RSQ ? __builtin_amdgcn_rsqf(var) : 1.f / sqrtf(var);  // (RSQ: the HF path)
#pragma unroll
  for (int p = 0; p < T; ++p) x[p] *= rstd;
  return rstd;
}

// x <- (x - mean(x)) * rstd with the forward's own rstd (ln_normalize's first pass): x_hat from
// the recomputed pre-LayerNorm row, bitwise the forward's
template <int D>
__device__ __forceinline__ void ln_recenter(f32x4 (&x)[D / 16], float rstd) {
  constexpr int T = D / 16;
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < T; ++p) s += (x[p][0] + x[p][1]) + (x[p][2] + x[p][3]);
  const float mean = sum_groups(s) * (1.f / D);
#pragma unroll
  for (int p = 0; p < T; ++p) {
    x[p] -= mean;
    x[p] *= rstd;
  }
}

// HF path (r05): the LayerNorm of a centred product's output y_s = 2^k y (zero mean by
// construction, load_params_hf): x_hat = y rstd, rstd = 1 / sqrt(mean(y^2) + eps), with the
// scale 2^-k folded into the multiplier (x_hat = y_s (rstd 2^-k): the same rounding as y rstd).
// No mean pass, no scale-down pass.  rstd by v_rsq_f32.  Returns rstd (saved for the backward).
template <int D>
__device__ __forceinline__ float ln_rms(f32x4 (&x)[D / 16], float eps, int k) {
  constexpr int T = D / 16;
  float v = 0.f;
#pragma unroll
  for (int p = 0; p < T; ++p) v += x[p][0] * x[p][0] + x[p][1] * x[p][1] + x[p][2] * x[p][2] + x[p][3] * x[p][3];
  const float rstd = __builtin_amdgcn_rsqf(ldexpf(sum_groups(v), -2 * k) * (1.f / D) + eps);
  const float r = ldexpf(rstd, -k);
#pragma unroll
  for (int p = 0; p < T; ++p) x[p] *= r;
  return rstd;
}

// dpre = rstd * (gr - mean(gr) - xhat * mean(gr * xhat)), gr = dL/dxhat ; in place on gr
template <int D>
__device__ __forceinline__ void ln_backward(f32x4 (&gr)[D / 16], const f32x4 (&xhat)[D / 16],
                                            float rstd) {
  constexpr int T = D / 16;
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int p = 0; p < T; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      a += gr[p][c];
      b += gr[p][c] * xhat[p][c];
    }
  a = sum_groups(a) * (1.f / D);
  b = sum_groups(b) * (1.f / D);
#pragma unroll
  for (int p = 0; p < T; ++p) gr[p] = rstd * (gr[p] - a - xhat[p] * b);
}

// x <- act(x * w + b) with LDS vectors w, b
template <int D, int ACT>
__device__ __forceinline__ void affine_act(f32x4 (&x)[D / 16], const float* sV, int vw, int vb, int g) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p) {
    const f32x4 w = vec4<D>(sV, vw, p, g), b = vec4<D>(sV, vb, p, g);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[p][c] = act_f<ACT>(x[p][c] * w[c] + b[c]);
  }
}

// ---------------------------------------------------------------------------------- segments
// inclusive segmented scan over the 16 edge lanes of each group; `head` = first lane of this
// lane's segment inside the chunk.
template <int OFF, int T>
__device__ __forceinline__ void seg_scan_level(f32x4 (&x)[T], int i, int head) {
  const bool take = (i - OFF) >= head;
#pragma unroll
  for (int p = 0; p < T; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float u = dpp<0x110 + OFF>(x[p][c]);  // row_shr:OFF = lane i - OFF
      if (take) x[p][c] += u;
    }
}
template <int T>
__device__ __forceinline__ void seg_scan(f32x4 (&x)[T], int i, int head) {
  seg_scan_level<1>(x, i, head);
  seg_scan_level<2>(x, i, head);
  seg_scan_level<4>(x, i, head);
  seg_scan_level<8>(x, i, head);
}

// Reduce-scatter over the 16 edge lanes (levels M = 8, 4, 2, 1; partners rs_partner<M>).
template <int N, int M, int N0>
struct RS {
  __device__ __forceinline__ static void run(float (&x)[N0], int i) {
    if constexpr (M == 0) {
      return;
    } else if constexpr (N >= 2) {
      constexpr int H = N / 2;
      const bool up = (i & M) != 0;
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const float lo = x[k], hi = x[k + H];
        x[k] = (up ? hi : lo) + rs_partner<M>(up ? lo : hi);
      }
      RS<H, M / 2, N0>::run(x, i);
    } else {
      x[0] += rs_partner<M>(x[0]);
      RS<1, M / 2, N0>::run(x, i);
    }
  }
};

template <int D>
struct VecAcc {
  static constexpr int N = D / 4;
  static constexpr int K = (N >= 16) ? N / 16 : 1;  // accumulated values per lane per vector
};
// slot of accumulator k of lane i, and whether lane i owns it (counted once)
template <int D>
__device__ __forceinline__ int acc_slot(int i, int k) {
  constexpr int N = D / 4;
  if constexpr (N >= 16) return (N / 16) * i + k;
  else return i / (16 / N);
}
template <int D>
__device__ __forceinline__ bool acc_owner(int i) {
  constexpr int N = D / 4;
  if constexpr (N >= 16) return true;
  else return (i % (16 / N)) == 0;
}

// acc += reduce-scatter over the 16 edge lanes of f(slot); the first level is formed on the fly
// so only N/2 temporaries are live.
template <int D, class F>
__device__ __forceinline__ void accumulate_vec(F f, float (&acc)[VecAcc<D>::K], int i) {
  constexpr int N = D / 4, H = N / 2;
  float t[H];
  const bool up = (i & 8) != 0;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float lo = f(k), hi = f(k + H);
    t[k] = (up ? hi : lo) + rs_partner<8>(up ? lo : hi);
  }
  RS<H, 4, H>::run(t, i);
#pragma unroll
  for (int k = 0; k < VecAcc<D>::K; ++k) acc[k] += t[k];
}

// Node-aligned, edge-balanced wave partition: wave w owns nodes [nb(w), nb(w+1)).
__device__ __forceinline__ int64_t node_begin(const int64_t* __restrict__ rowptr, int64_t n_nodes,
                                              int64_t n_edges, int64_t w, int64_t n_waves) {
  if (w >= n_waves) return n_nodes;
  if (w <= 0) return 0;
  const int64_t target = (n_edges * w) / n_waves;
  int64_t lo = 0, hi = n_nodes;  // first n in [0, n_nodes] with rowptr[n] >= target
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// carry of the open segment: lane 15 of each group stores, lane 0 of the next chunk adds.
template <int D>
__device__ __forceinline__ void carry_store(float* cbuf, const f32x4 (&x)[D / 16], const float (&p3)[3]) {
#pragma unroll
  for (int p = 0; p < D / 16; ++p) *reinterpret_cast<f32x4*>(cbuf + 4 * p) = x[p];
  cbuf[D / 4 + 0] = p3[0];
  cbuf[D / 4 + 1] = p3[1];
  cbuf[D / 4 + 2] = p3[2];
}
// every lane reads its group's carry (one broadcast read) and adds take * carry: no select, no
// divergent load.  The carry buffer is zeroed before the loop (carry_clear), so it always holds
// finite values.  Lanes past the wave's range keep their (finite, clamped-edge) values: they
// lie after every valid lane of the chunk, so no valid lane's scan reads them, and they never
// store.
template <int D>
__device__ __forceinline__ void carry_apply(const float* cbuf, f32x4 (&x)[D / 16], float (&p3)[3],
                                            bool take) {
  const float tf = take ? 1.f : 0.f;
#pragma unroll
  for (int p = 0; p < D / 16; ++p) {
    const f32x4 c = *reinterpret_cast<const f32x4*>(cbuf + 4 * p);
#pragma unroll
    for (int q = 0; q < 4; ++q) x[p][q] = __builtin_fmaf(c[q], tf, x[p][q]);
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) p3[c] = __builtin_fmaf(cbuf[D / 4 + c], tf, p3[c]);
}
// zero this wave's four group carries (before the loop)
template <int D>
__device__ __forceinline__ void carry_clear(float* wave_cbuf, int lane) {
  for (int k = lane; k < 4 * carry_stride<D>(); k += 64) wave_cbuf[k] = 0.f;
}

struct EdgeCtx {
  int e, ec, i, j, seg0, seg1;  // 32-bit (n_nodes, n_edges < 2^31 checked at the C ABI)
  bool valid;
  float rx, ry, rz, dist;
  float pjx, pjy, pjz;
};

// Receiver / sender of edge e, prefetched one 16-edge chunk ahead so that the gathers that
// depend on them (rowptr, pos, node rows) are issued together at the start of the next chunk:
// one exposed memory round trip per chunk instead of a chain of three.  Lanes past the wave's
// range read the last edge of the graph range (every load stays in bounds and branch-free;
// results of those lanes are masked by EdgeCtx::valid).
struct EdgeIJ {
  int i, j;
};
__device__ __forceinline__ int clamp_edge(int e, int e_hi) {
  e = e < e_hi ? e : e_hi - 1;
  return e > 0 ? e : 0;
}
__device__ __forceinline__ EdgeIJ load_ij(int base, int lane_e, int e_hi,
                                          const int64_t* __restrict__ recv,
                                          const int64_t* __restrict__ send) {
  const int ec = clamp_edge(base + lane_e, e_hi);
  // low dwords of the int64 indices (values < 2^31)
  EdgeIJ r;
  r.i = reinterpret_cast<const int*>(recv)[2 * ec];
  r.j = reinterpret_cast<const int*>(send)[2 * ec];
  return r;
}

__device__ __forceinline__ EdgeCtx edge_ctx(EdgeIJ ij, int base, int lane_e, int e_hi,
                                            int n_nodes, const int64_t* __restrict__ rowptr,
                                            const float* __restrict__ pos) {
  EdgeCtx c;
  c.e = base + lane_e;
  c.ec = clamp_edge(c.e, e_hi);
  c.valid = c.e < e_hi;
  c.i = ((unsigned)ij.i < (unsigned)n_nodes) ? ij.i : 0;
  c.j = ((unsigned)ij.j < (unsigned)n_nodes) ? ij.j : c.i;  // out-of-range sender (flagged by
                                                            // the CSR build): stay in bounds
  const int* rp = reinterpret_cast<const int*>(rowptr);
  c.seg0 = rp[2 * c.i];
  c.seg1 = rp[2 * c.i + 2];
  c.rx = pos[3 * c.i + 0];  // pos_i (pos_j subtracted by edge_geom, after the issue burst)
  c.ry = pos[3 * c.i + 1];
  c.rz = pos[3 * c.i + 2];
  c.dist = 0.f;
  c.pjx = pos[3 * c.j + 0];
  c.pjy = pos[3 * c.j + 1];
  c.pjz = pos[3 * c.j + 2];
  return c;
}
// rel = pos_i - pos_j (egnn_layer.py:64), dist = |rel|: called once the chunk's loads are issued.
// FAST (the HF path, forward and backward alike): v_sqrt_f32 (~1 ulp) instead of the correctly
// rounded sequence.
template <bool FAST = false>
__device__ __forceinline__ void edge_geom(EdgeCtx& c) {
  c.rx -= c.pjx;
  c.ry -= c.pjy;
  c.rz -= c.pjz;
  const float q = c.rx * c.rx + c.ry * c.ry + c.rz * c.rz;
  c.dist = FAST ? __builtin_amdgcn_sqrtf(q) : sqrtf(q);
}

// first pre-activation AB[i,:d] + AB[j,d:] + w1d*dist + b1.  All 2*d/4 row loads are issued
// back to back (one round trip) before any is consumed; the scheduler would otherwise batch
// them four at a time with a full wait between batches.
template <int D, bool FAST, class Ctx>
__device__ __forceinline__ void load_pre1(f32x4 (&x)[D / 16], const float* arow, const float* brow,
                                          const float* sV, Ctx& c, int g) {
  f32x4 b[D / 16];
#pragma unroll
  for (int p = 0; p < D / 16; ++p) {
    x[p] = *reinterpret_cast<const f32x4*>(arow + 16 * p + 4 * g);
    b[p] = *reinterpret_cast<const f32x4*>(brow + 16 * p + 4 * g);
  }
  __builtin_amdgcn_sched_barrier(0);
  edge_geom<FAST>(c);
  const float dist = c.dist;
#pragma unroll
  for (int p = 0; p < D / 16; ++p)
    x[p] = (x[p] + b[p]) + (vec4<D>(sV, V_W1D, p, g) * dist + vec4<D>(sV, V_B1, p, g));
}

// row r of a (rows, ld) fp32 tensor (64-bit offset)
__device__ __forceinline__ const float* rowp(const float* base, int r, int ld) {
  return base + (size_t)(unsigned)r * (size_t)ld;
}
__device__ __forceinline__ float* rowp(float* base, int r, int ld) {
  return base + (size_t)(unsigned)r * (size_t)ld;
}

// wave-uniform range of this wave (scalar registers)
struct WaveRange {
  int e_lo, e_hi, n_lo, n_hi;  // edges [e_lo, e_hi) = the in-edges of receivers [n_lo, n_hi)
};
__device__ __forceinline__ WaveRange wave_range(const int64_t* __restrict__ rowptr, int64_t n_nodes,
                                                int64_t n_edges, int64_t n_waves, int wid,
                                                int nwb) {
  const int64_t wave = (int64_t)blockIdx.x * nwb + wid;
  const int64_t nb = node_begin(rowptr, n_nodes, n_edges, wave, n_waves);
  const int64_t ne = node_begin(rowptr, n_nodes, n_edges, wave + 1, n_waves);
  WaveRange r;
  r.e_lo = (nb < ne) ? (int)rowptr[nb] : 0;
  r.e_hi = (nb < ne) ? (int)rowptr[ne] : 0;
  r.e_lo = __builtin_amdgcn_readfirstlane(r.e_lo);
  r.e_hi = __builtin_amdgcn_readfirstlane(r.e_hi);
  r.n_lo = __builtin_amdgcn_readfirstlane((int)nb);
  r.n_hi = __builtin_amdgcn_readfirstlane((int)ne);
  return r;
}

// The receiver rows of the wave's zero in-degree nodes: zeros.  The edge loop writes a row at
// each segment end only, so these are the rows it never writes; covering them here replaces
// two full memsets of the outputs per launch (r04: ~11 us of fill kernels + their boundaries
// per layer).  The waves' node ranges partition [0, n_nodes).
template <int D>
__device__ __forceinline__ void zero_isolated(const WaveRange& wr, const int64_t* __restrict__ rowptr,
                                              float* __restrict__ rows, float* __restrict__ rows3,
                                              int lane) {
  const int* rp = reinterpret_cast<const int*>(rowptr);  // low dwords (values < 2^31)
  for (int n = wr.n_lo + lane; n < wr.n_hi; n += 64) {
    if (rp[2 * n] == rp[2 * n + 2]) {
      float4* r = reinterpret_cast<float4*>(rows + (size_t)n * D);
#pragma unroll
      for (int k = 0; k < D / 4; ++k) r[k] = float4{0.f, 0.f, 0.f, 0.f};
      rows3[3 * (size_t)n] = 0.f;
      rows3[3 * (size_t)n + 1] = 0.f;
      rows3[3 * (size_t)n + 2] = 0.f;
    }
  }
}


// 1: the f32-MFMA (exact fmaf chain) products instead of the HF path (gmp_egnn_set_f32_mfma)
bool egnn_f32();

// the dynamic-LDS attribute, set once per (device, kernel): a hipFuncSetAttribute before every
// launch showed as ~10 us gaps in front of the K4 / K15 launches (r05 trace)
int prep_kernel_once(const void* k, size_t smem);
template <class K>
inline int prep_kernel(K k, size_t smem) {
  return prep_kernel_once((const void*)k, smem);
}

inline bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace gmp
