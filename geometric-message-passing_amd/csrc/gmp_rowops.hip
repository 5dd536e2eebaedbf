// K12: fused LayerNorm + activation over rows (node-level MLPs on the path: the EGNN update
// mlp_upd = Linear -> LayerNorm -> act -> Linear -> LayerNorm -> act, egnn_layer.py:37-39 and
// :82-86; GVP's scalar LayerNorm, gvp_layer.py:221-243, with act = identity).
//   forward : xhat = (x - mean) * rstd, rstd = 1/sqrt(var + eps) (biased var, two-pass),
//             y = act(xhat * gamma + beta); xhat and rstd are saved for the backward
//   backward: dz = gy * act'(xhat*gamma + beta); dgamma = sum dz*xhat, dbeta = sum dz;
//             dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dz * gamma
// One wave per row (lane f handles features f, f + 64, ...); row reductions on DPP + permlane
// swaps.  gamma/beta gradients: per-workgroup partial rows (registers across a grid-stride
// loop), summed in workgroup order by the caller-visible second kernel — deterministic.
#include "gmp_common.h"

namespace gmp {
namespace {

constexpr int kRowT = 256;        // 4 waves = 4 rows in flight per workgroup
constexpr int kMaxF = 8;          // features per lane (d <= 512)
constexpr int kRowBlocks = 256;   // backward grid (partials rows; ~50 rows per wave at 50k)

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over all 64 lanes, result in every lane
__device__ __forceinline__ float wave_sum(float v) {
  v += dppf<0x128>(v);  // row_ror:8
  v += dppf<0x124>(v);  // row_ror:4
  v += dppf<0x122>(v);  // row_ror:2
  v += dppf<0x121>(v);  // row_ror:1
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  v = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  // lanes summed in different orders: make the result wave-uniform
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// act: 0 relu, 1 silu, 2 identity
template <int ACT>
__device__ __forceinline__ float act_fwd(float z) {
  if (ACT == 0) return z > 0.f ? z : 0.f;
  if (ACT == 1) return z * (1.f / (1.f + __expf(-z)));
  return z;
}
template <int ACT>
__device__ __forceinline__ float act_grad(float z) {
  if (ACT == 0) return z > 0.f ? 1.f : 0.f;
  if (ACT == 1) {
    const float sg = 1.f / (1.f + __expf(-z));
    return sg * (1.f + z * (1.f - sg));
  }
  return 1.f;
}

template <int ACT>
__global__ __launch_bounds__(kRowT) void ln_act_fwd_kernel(
    int64_t rows, int d, const float* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ y, float* __restrict__ xhat,
    float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (kRowT / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * d;
  float v[kMaxF];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxF; ++k) {
    const int f = lane + 64 * k;
    v[k] = f < d ? xr[f] : 0.f;
    s += v[k];
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxF; ++k) {
    const int f = lane + 64 * k;
    v[k] = f < d ? v[k] - mean : 0.f;
    q += v[k] * v[k];
  }
  const float rstd = 1.f / sqrtf(wave_sum(q) / (float)d + eps);
#pragma unroll
  for (int k = 0; k < kMaxF; ++k) {
    const int f = lane + 64 * k;
    if (f < d) {
      const float xh = v[k] * rstd;
      xhat[r * d + f] = xh;
      y[r * d + f] = act_fwd<ACT>(xh * gamma[f] + beta[f]);
    }
  }
  if (lane == 0) rstd_out[r] = rstd;
}

// narrow rows (D = 8, 16, 32): 64 / D rows per wave instruction, row sums by xor butterflies
// inside the D-lane group (same two-pass statistics as above)
template <int D>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int m = D / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

template <int ACT, int D>
__global__ __launch_bounds__(kRowT) void ln_act_fwd_small_kernel(
    int64_t rows, const float* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ y, float* __restrict__ xhat,
    float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63, f = lane % D;
  const int64_t r = ((int64_t)blockIdx.x * (kRowT / 64) + (threadIdx.x >> 6)) * (64 / D) + lane / D;
  const int64_t rc = r < rows ? r : rows - 1;
  const float v0 = x[rc * D + f];
  const float mean = group_sum<D>(v0) * (1.f / D);
  const float v = v0 - mean;
  const float rstd = 1.f / sqrtf(group_sum<D>(v * v) / (float)D + eps);
  if (r >= rows) return;
  const float xh = v * rstd;
  xhat[r * D + f] = xh;
  y[r * D + f] = act_fwd<ACT>(xh * gamma[f] + beta[f]);
  if (f == 0) rstd_out[r] = rstd;
}

template <int ACT>
__global__ __launch_bounds__(kRowT) void ln_act_bwd_kernel(
    int64_t rows, int d, const float* __restrict__ gy, const float* __restrict__ xhat,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ gx, float* __restrict__ partials) {
  __shared__ float red[kRowT / 64][2 * 512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float dg[kMaxF], db[kMaxF];
#pragma unroll
  for (int k = 0; k < kMaxF; ++k) dg[k] = db[k] = 0.f;
  // kRB consecutive rows per wave and step: their loads are issued together (the one-row loop
  // was latency-bound: ~1 TB/s); the gamma / beta sums still add rows in increasing order
  constexpr int kRB = 2;
  const int64_t stride = (int64_t)gridDim.x * (kRowT / 64) * kRB;
  for (int64_t r0 = ((int64_t)blockIdx.x * (kRowT / 64) + wv) * kRB; r0 < rows; r0 += stride) {
    float rs[kRB], xh[kRB][kMaxF], gv[kRB][kMaxF];
#pragma unroll
    for (int j = 0; j < kRB; ++j) {
      const int64_t r = r0 + j;
      const bool ok = r < rows;
      rs[j] = ok ? rstd_in[r] : 0.f;
#pragma unroll
      for (int k = 0; k < kMaxF; ++k) {
        const int f = lane + 64 * k;
        xh[j][k] = (ok && f < d) ? xhat[r * d + f] : 0.f;
        gv[j][k] = (ok && f < d) ? gy[r * d + f] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < kRB; ++j) {
      const int64_t r = r0 + j;
      if (r >= rows) break;  // wave-uniform
      float g[kMaxF];
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < kMaxF; ++k) {
        const int f = lane + 64 * k;
        g[k] = 0.f;
        if (f < d) {
          const float gm = gamma[f];
          const float dz = gv[j][k] * act_grad<ACT>(xh[j][k] * gm + beta[f]);
          dg[k] += dz * xh[j][k];
          db[k] += dz;
          g[k] = dz * gm;
        }
        a += g[k];
        b += g[k] * xh[j][k];
      }
      a = wave_sum(a) / (float)d;
      b = wave_sum(b) / (float)d;
#pragma unroll
      for (int k = 0; k < kMaxF; ++k) {
        const int f = lane + 64 * k;
        if (f < d) gx[r * d + f] = rs[j] * (g[k] - a - xh[j][k] * b);
      }
    }
  }
  // workgroup partial: waves in order
#pragma unroll
  for (int k = 0; k < kMaxF; ++k) {
    const int f = lane + 64 * k;
    if (f < d) {
      red[wv][f] = dg[k];
      red[wv][512 + f] = db[k];
    }
  }
  __syncthreads();
  for (int f = threadIdx.x; f < 2 * d; f += kRowT) {
    const int off = f < d ? f : 512 + (f - d);
    float s = 0.f;
    for (int w = 0; w < kRowT / 64; ++w) s += red[w][off];
    partials[(int64_t)blockIdx.x * 2 * d + f] = s;
  }
}

// r04 form for d = 64 F (F = 1, 2, 4): lane l holds the F consecutive features F l .. F l + F - 1
// of a row (one 4F-byte load per lane and tensor), each wave takes kRB4 rows per iteration (their
// loads issued together) over a short grid-stride loop; the grid is sized to give every SIMD
// several waves (r03's 256-workgroup grid ran one wave per SIMD through ~25 dependent rounds:
// 70 us for 50k x 128).  [dgamma | dbeta]: one partial row per workgroup (sum_rows_kernel).
constexpr int kRB4 = 4;
template <int ACT, int F>
__global__ __launch_bounds__(kRowT) void ln_act_bwd_vec_kernel(
    int64_t rows, const float* __restrict__ gy, const float* __restrict__ xhat,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ gx, float* __restrict__ partials) {
  constexpr int D = 64 * F;
  typedef float fv __attribute__((ext_vector_type(F)));
  __shared__ float red[kRowT / 64][2 * D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const fv gm = *reinterpret_cast<const fv*>(gamma + F * lane);
  const fv bt = *reinterpret_cast<const fv*>(beta + F * lane);
  fv dg = {}, db = {};
  const int64_t stride = (int64_t)gridDim.x * (kRowT / 64) * kRB4;
  for (int64_t r0 = ((int64_t)blockIdx.x * (kRowT / 64) + wv) * kRB4; r0 < rows; r0 += stride) {
    float rs[kRB4];
    fv xh[kRB4], gv[kRB4];
#pragma unroll
    for (int j = 0; j < kRB4; ++j) {
      const int64_t r = r0 + j < rows ? r0 + j : rows - 1;  // clamped: loads stay in bounds
      rs[j] = rstd_in[r];
      xh[j] = *reinterpret_cast<const fv*>(xhat + r * D + F * lane);
      gv[j] = *reinterpret_cast<const fv*>(gy + r * D + F * lane);
    }
#pragma unroll
    for (int j = 0; j < kRB4; ++j) {
      const int64_t r = r0 + j;
      if (r >= rows) break;  // wave-uniform
      fv g;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < F; ++k) {
        const float dz = gv[j][k] * act_grad<ACT>(xh[j][k] * gm[k] + bt[k]);
        dg[k] += dz * xh[j][k];
        db[k] += dz;
        g[k] = dz * gm[k];
        a += g[k];
        b += g[k] * xh[j][k];
      }
      a = wave_sum(a) * (1.f / D);
      b = wave_sum(b) * (1.f / D);
      fv o;
#pragma unroll
      for (int k = 0; k < F; ++k) o[k] = rs[j] * (g[k] - a - xh[j][k] * b);
      *reinterpret_cast<fv*>(gx + r * D + F * lane) = o;
    }
  }
#pragma unroll
  for (int k = 0; k < F; ++k) {
    red[wv][F * lane + k] = dg[k];
    red[wv][D + F * lane + k] = db[k];
  }
  __syncthreads();
  for (int f = threadIdx.x; f < 2 * D; f += kRowT) {
    float sacc = 0.f;
#pragma unroll
    for (int w = 0; w < kRowT / 64; ++w) sacc += red[w][f];
    partials[(int64_t)blockIdx.x * 2 * D + f] = sacc;
  }
}

// r04 form for narrow rows, D = 8, 16, 32 (GVP's edge-scalar LayerNorm: 1M rows of 32): a wave
// instruction covers R = 64 / D rows (lane l: row l / D, feature l % D), kRB4 such row groups per
// iteration with their loads issued together; row sums by xor butterflies inside the D-lane
// group (every lane of a group gets the same sum).  The generic kernel ran one row per wave
// instruction with 64 - D idle lanes and ~500 dependent iterations per wave (0.65 ms for 1M x 32).
// [dgamma | dbeta]: per-lane sums over the lane's rows, then the (wave, row slot) partials of
// each feature added in fixed order -> one partial row per workgroup (sum_rows_kernel).
template <int ACT, int D>
__global__ __launch_bounds__(kRowT) void ln_act_bwd_small_kernel(
    int64_t rows, const float* __restrict__ gy, const float* __restrict__ xhat,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ gx, float* __restrict__ partials) {
  constexpr int R = 64 / D;
  __shared__ float red[kRowT / 64 * R][2 * D];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int f = lane % D, rsub = lane / D;
  const float gm = gamma[f], bt = beta[f];
  float dg = 0.f, db = 0.f;
  const int64_t stride = (int64_t)gridDim.x * (kRowT / 64) * R * kRB4;
  for (int64_t r0 = ((int64_t)blockIdx.x * (kRowT / 64) + wv) * R * kRB4; r0 < rows;
       r0 += stride) {
    float rs[kRB4], xh[kRB4], gv[kRB4];
#pragma unroll
    for (int j = 0; j < kRB4; ++j) {
      int64_t r = r0 + j * R + rsub;
      r = r < rows ? r : rows - 1;  // clamped: loads stay in bounds
      rs[j] = rstd_in[r];
      xh[j] = xhat[r * D + f];
      gv[j] = gy[r * D + f];
    }
#pragma unroll
    for (int j = 0; j < kRB4; ++j) {
      const int64_t r = r0 + j * R + rsub;
      const float dz = gv[j] * act_grad<ACT>(xh[j] * gm + bt);
      const float g = dz * gm;
      const float a = group_sum<D>(g) * (1.f / D);
      const float b = group_sum<D>(g * xh[j]) * (1.f / D);
      if (r < rows) {
        dg += dz * xh[j];
        db += dz;
        gx[r * D + f] = rs[j] * (g - a - xh[j] * b);
      }
    }
  }
  red[wv * R + rsub][f] = dg;
  red[wv * R + rsub][D + f] = db;
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * D; c += kRowT) {
    float sacc = 0.f;
#pragma unroll
    for (int w = 0; w < kRowT / 64 * R; ++w) sacc += red[w][c];
    partials[(int64_t)blockIdx.x * 2 * D + c] = sacc;
  }
}

// vec-kernel grid: ~16 rows per wave (four iterations of kRB4), at most 1024 workgroups
int vec_blocks(int64_t rows) {
  const int64_t b = ceil_div(rows, (kRowT / 64) * kRB4 * 4);
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

// out[f] = sum over the partial rows (f < 2d: [dgamma | dbeta]) in a fixed order: thread
// (column c, row group q) sums rows q, q + kSG, ... ; the kSG group sums are then added in
// group order.  Deterministic.
constexpr int kSC = 16, kSG = 16;  // columns x row groups per block (256 threads: fits beside
                                   // the side stream's kernels); each thread's rows load in
                                   // one burst for <= 256 rows
__global__ __launch_bounds__(kSC * kSG) void sum_rows_kernel(const float* __restrict__ partials,
                                                             int nrows, int width,
                                                             float* __restrict__ out) {
  __shared__ float part[kSG][kSC];
  const int c = threadIdx.x % kSC, q = threadIdx.x / kSC;
  const int f = blockIdx.x * kSC + c;
  // rows q, q + kSG, ... added in that order; their loads are issued kU at a time (one memory
  // round trip per kU rows instead of one per row: the loop was latency-bound)
  constexpr int kU = 16;
  float s = 0.f;
  if (f < width) {
    for (int r0 = q; r0 < nrows; r0 += kU * kSG) {
      float v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int r = r0 + u * kSG;
        v[u] = r < nrows ? partials[(int64_t)r * width + f] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (r0 + u * kSG < nrows) s += v[u];
    }
  }
  part[q][c] = s;
  __syncthreads();
  if (q == 0 && f < width) {
    float t = 0.f;
    for (int g = 0; g < kSG; ++g) t += part[g][c];
    out[f] = t;
  }
}

// generic backward grid: at most kRowBlocks workgroups (one partial row each)
int bwd_blocks(int64_t rows) {
  const int64_t b = ceil_div(rows, kRowT / 64);
  return (int)(b < kRowBlocks ? (b < 1 ? 1 : b) : kRowBlocks);
}

// GVP vector LayerNorm (gvp_layer.py:232-243 with the clamp of _norm_no_nan, :66-73): rows of C
// channels x 3 (xyz), out = v / sqrt(mean_c max(|v_c|^2, 1e-8)).  A G-lane group per row (G =
// the power of two >= C, lane = channel, its 3 floats contiguous with the neighbours': coalesced
// 12-byte pieces), 64 / G rows per wave; the mean by xor butterflies inside the group (the same
// sum in every lane of it).  Backward recomputes the norm from v:
//   dv_c = g_c / vn - (sum_c' g_c'.v_c') v_c [|v_c|^2 >= eps] / (C vn^3)
// (clamp passes the gradient where the input reaches the bound, as torch's clamp_min does).
template <int G>
__device__ __forceinline__ float gsum(float v) {
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

template <int G, bool BWD>
__global__ __launch_bounds__(kRowT) void vec_norm_kernel(int64_t rows, int C,
                                                         const float* __restrict__ v,
                                                         const float* __restrict__ gout,
                                                         float* __restrict__ out) {
  const int lane = threadIdx.x & 63, c = lane % G;
  const int64_t r = ((int64_t)blockIdx.x * (kRowT / 64) + (threadIdx.x >> 6)) * (64 / G) + lane / G;
  const bool ok = r < rows && c < C;
  const int64_t o = (r < rows ? r : rows - 1) * 3 * (int64_t)C + 3 * (c < C ? c : 0);
  float x = 0.f, y = 0.f, z = 0.f;
  if (ok) {
    x = v[o];
    y = v[o + 1];
    z = v[o + 2];
  }
  const float q = x * x + y * y + z * z;
  const float s2 = ok ? fmaxf(q, 1e-8f) : 0.f;
  const float m = gsum<G>(s2) / (float)C;
  const float vn = sqrtf(m), inv = 1.f / vn;
  if constexpr (!BWD) {
    if (ok) {
      out[o] = x / vn;
      out[o + 1] = y / vn;
      out[o + 2] = z / vn;
    }
  } else {
    float gx = 0.f, gy = 0.f, gz = 0.f;
    if (ok) {
      gx = gout[o];
      gy = gout[o + 1];
      gz = gout[o + 2];
    }
    const float dot = gsum<G>(gx * x + gy * y + gz * z);
    const float k = (q >= 1e-8f) ? dot * inv * inv * inv / (float)C : 0.f;
    if (ok) {
      out[o] = gx / vn - k * x;
      out[o + 1] = gy / vn - k * y;
      out[o + 2] = gz / vn - k * z;
    }
  }
}

template <bool BWD>
int vec_norm_launch(int64_t rows, int64_t C, const float* v, const float* g, float* out,
                    hipStream_t s) {
  const int G = C <= 1 ? 1 : C <= 2 ? 2 : C <= 4 ? 4 : C <= 8 ? 8 : C <= 16 ? 16 : C <= 32 ? 32 : 64;
  const unsigned grid = (unsigned)ceil_div(rows, (int64_t)(kRowT / 64) * (64 / G));
#define LAUNCH_VN(GG) \
  vec_norm_kernel<GG, BWD><<<grid, kRowT, 0, s>>>(rows, (int)C, v, g, out)
  switch (G) {
    case 1: LAUNCH_VN(1); break;
    case 2: LAUNCH_VN(2); break;
    case 4: LAUNCH_VN(4); break;
    case 8: LAUNCH_VN(8); break;
    case 16: LAUNCH_VN(16); break;
    case 32: LAUNCH_VN(32); break;
    default: LAUNCH_VN(64); break;
  }
#undef LAUNCH_VN
  return launch_status();
}

// _norm_no_nan over the xyz axis of (rows, 3, h) rows (gvp_layer.py:66-73 as GVP.forward applies
// it to vh, :101-170): out (rows, h) = sqrt(max(sum_x vh[x, c]^2, 1e-8)); backward
// dvh[x, c] = g[c] vh[x, c] / out[c] where the sum reaches the bound (torch's clamp_min mask).
// One thread per (row, c): the three strided loads coalesce across c.
template <bool BWD>
__global__ __launch_bounds__(kRowT) void xyz_norm_kernel(int64_t n, int h,
                                                         const float* __restrict__ vh,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * kRowT + threadIdx.x;
  if (t >= n) return;
  const int64_t r = t / h, c = t - r * h, o = r * 3 * (int64_t)h + c;
  const float x = vh[o], y = vh[o + h], z = vh[o + 2 * h];
  const float q = x * x + y * y + z * z;
  const float nv = sqrtf(fmaxf(q, 1e-8f));
  if constexpr (!BWD) {
    out[t] = nv;
  } else {
    const float k = q >= 1e-8f ? g[t] / nv : 0.f;
    out[o] = k * x;
    out[o + h] = k * y;
    out[o + 2 * h] = k * z;
  }
}

bool small_form(int64_t d) { return d == 8 || d == 16 || d == 32; }

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_ln_act_fwd_f32(int64_t rows, int64_t d, const float* x, const float* gamma,
                       const float* beta, float eps, int act, float* y, float* xhat_save,
                       float* rstd_save, void* stream) {
  GMP_CHECK_ARG(rows >= 0 && d > 0 && d <= 64 * kMaxF && act >= 0 && act <= 2);
  if (rows == 0) return GMP_OK;
  GMP_CHECK_ARG(x && gamma && beta && y && xhat_save && rstd_save);
  hipStream_t s = as_stream(stream);
  if (small_form(d)) {
    const unsigned gs = (unsigned)ceil_div(rows, (kRowT / 64) * (64 / d));
#define LAUNCH_LNF(A, D) \
  ln_act_fwd_small_kernel<A, D><<<gs, kRowT, 0, s>>>(rows, x, gamma, beta, eps, y, xhat_save, rstd_save)
#define LAUNCH_LNF_D(A) \
  if (d == 8) LAUNCH_LNF(A, 8); else if (d == 16) LAUNCH_LNF(A, 16); else LAUNCH_LNF(A, 32)
    if (act == 0) { LAUNCH_LNF_D(0); } else if (act == 1) { LAUNCH_LNF_D(1); } else { LAUNCH_LNF_D(2); }
#undef LAUNCH_LNF_D
#undef LAUNCH_LNF
    return launch_status();
  }
  const unsigned grid = (unsigned)ceil_div(rows, kRowT / 64);
  if (act == 0)
    ln_act_fwd_kernel<0><<<grid, kRowT, 0, s>>>(rows, (int)d, x, gamma, beta, eps, y, xhat_save,
                                                rstd_save);
  else if (act == 1)
    ln_act_fwd_kernel<1><<<grid, kRowT, 0, s>>>(rows, (int)d, x, gamma, beta, eps, y, xhat_save,
                                                rstd_save);
  else
    ln_act_fwd_kernel<2><<<grid, kRowT, 0, s>>>(rows, (int)d, x, gamma, beta, eps, y, xhat_save,
                                                rstd_save);
  return launch_status();
}

bool vec_form(int64_t d) { return d == 64 || d == 128 || d == 256; }

// The backward's partial rows: the narrow / vectorised kernels (with grad_gamma_beta) write
// vec_blocks(rows) rows, the generic kernel (every other case, and grad_gamma_beta == NULL: the
// caller-reduces form) bwd_blocks(rows).  The workspace covers whichever runs (the
// r04 size was the vectorised count alone, which the generic fallback overran below ~16k rows).
size_t gmp_ln_act_bwd_workspace_size(int64_t rows, int64_t d) {
  const int64_t v = vec_blocks(rows), b = bwd_blocks(rows);
  return (size_t)(v > b ? v : b) * 2 * (size_t)d * sizeof(float);
}

int gmp_ln_act_bwd_f32(int64_t rows, int64_t d, const float* grad_y, const float* xhat,
                       const float* rstd, const float* gamma, const float* beta, int act,
                       float* grad_x, float* grad_gamma_beta, void* workspace,
                       size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(rows >= 0 && d > 0 && d <= 64 * kMaxF && act >= 0 && act <= 2);
  GMP_CHECK_ARG(grad_gamma_beta || workspace);
  hipStream_t s = as_stream(stream);
  const int G = bwd_blocks(rows);
  float* part = reinterpret_cast<float*>(workspace);
  if (rows == 0) {
    if (grad_gamma_beta)
      return hip_check(hipMemsetAsync(grad_gamma_beta, 0, 2 * d * sizeof(float), s));
    return hip_check(hipMemsetAsync(part, 0, (size_t)G * 2 * d * sizeof(float), s));
  }
  GMP_CHECK_ARG(grad_y && xhat && rstd && gamma && beta && grad_x && workspace);
  if (workspace_bytes < gmp_ln_act_bwd_workspace_size(rows, d)) return GMP_ERR_WORKSPACE;
  const uintptr_t al = reinterpret_cast<uintptr_t>(grad_y) | reinterpret_cast<uintptr_t>(xhat) |
                       reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) |
                       reinterpret_cast<uintptr_t>(grad_x);
  int rows_written = G;  // partial rows for sum_rows_kernel
  if (small_form(d) && grad_gamma_beta) {
    rows_written = vec_blocks(rows);
#define LAUNCH_LNS(A, D)                                                                 \
  ln_act_bwd_small_kernel<A, D><<<rows_written, kRowT, 0, s>>>(rows, grad_y, xhat, rstd, gamma, \
                                                               beta, grad_x, part)
#define LAUNCH_LNS_D(A) \
  if (d == 8) LAUNCH_LNS(A, 8); else if (d == 16) LAUNCH_LNS(A, 16); else LAUNCH_LNS(A, 32)
    if (act == 0) { LAUNCH_LNS_D(0); } else if (act == 1) { LAUNCH_LNS_D(1); } else { LAUNCH_LNS_D(2); }
#undef LAUNCH_LNS_D
#undef LAUNCH_LNS
  } else if (vec_form(d) && grad_gamma_beta && al % (d / 16) == 0) {
    rows_written = vec_blocks(rows);
#define LAUNCH_LNV(A, F)                                                                \
  ln_act_bwd_vec_kernel<A, F><<<rows_written, kRowT, 0, s>>>(rows, grad_y, xhat, rstd, gamma, \
                                                             beta, grad_x, part)
#define LAUNCH_LNV_F(A) \
  if (d == 64) LAUNCH_LNV(A, 1); else if (d == 128) LAUNCH_LNV(A, 2); else LAUNCH_LNV(A, 4)
    if (act == 0) { LAUNCH_LNV_F(0); } else if (act == 1) { LAUNCH_LNV_F(1); } else { LAUNCH_LNV_F(2); }
#undef LAUNCH_LNV_F
#undef LAUNCH_LNV
  } else if (act == 0) {
    ln_act_bwd_kernel<0><<<G, kRowT, 0, s>>>(rows, (int)d, grad_y, xhat, rstd, gamma, beta,
                                             grad_x, part);
  } else if (act == 1) {
    ln_act_bwd_kernel<1><<<G, kRowT, 0, s>>>(rows, (int)d, grad_y, xhat, rstd, gamma, beta,
                                             grad_x, part);
  } else {
    ln_act_bwd_kernel<2><<<G, kRowT, 0, s>>>(rows, (int)d, grad_y, xhat, rstd, gamma, beta,
                                             grad_x, part);
  }
  const int rc = launch_status();
  if (rc || !grad_gamma_beta) return rc;  // NULL: the caller reduces the G partial rows
  sum_rows_kernel<<<(unsigned)ceil_div(2 * d, kSC), kSC * kSG, 0, s>>>(part, rows_written,
                                                                       (int)(2 * d),
                                                                       grad_gamma_beta);
  return launch_status();
}

int gmp_vec_norm_fwd_f32(int64_t rows, int64_t channels, const float* v, float* out,
                         void* stream) {
  GMP_CHECK_ARG(rows >= 0 && channels >= 1 && channels <= 64);
  if (rows == 0) return GMP_OK;
  GMP_CHECK_ARG(v && out);
  return vec_norm_launch<false>(rows, channels, v, nullptr, out, as_stream(stream));
}

int gmp_vec_norm_bwd_f32(int64_t rows, int64_t channels, const float* v, const float* grad_out,
                         float* grad_v, void* stream) {
  GMP_CHECK_ARG(rows >= 0 && channels >= 1 && channels <= 64);
  if (rows == 0) return GMP_OK;
  GMP_CHECK_ARG(v && grad_out && grad_v);
  return vec_norm_launch<true>(rows, channels, v, grad_out, grad_v, as_stream(stream));
}

int gmp_xyz_norm_fwd_f32(int64_t rows, int64_t h, const float* vh, float* out, void* stream) {
  GMP_CHECK_ARG(rows >= 0 && h >= 1);
  if (rows == 0) return GMP_OK;
  GMP_CHECK_ARG(vh && out);
  const int64_t n = rows * h;
  xyz_norm_kernel<false><<<(unsigned)ceil_div(n, (int64_t)kRowT), kRowT, 0, as_stream(stream)>>>(
      n, (int)h, vh, nullptr, out);
  return launch_status();
}

int gmp_xyz_norm_bwd_f32(int64_t rows, int64_t h, const float* vh, const float* grad_out,
                         float* grad_vh, void* stream) {
  GMP_CHECK_ARG(rows >= 0 && h >= 1);
  if (rows == 0) return GMP_OK;
  GMP_CHECK_ARG(vh && grad_out && grad_vh);
  const int64_t n = rows * h;
  xyz_norm_kernel<true><<<(unsigned)ceil_div(n, (int64_t)kRowT), kRowT, 0, as_stream(stream)>>>(
      n, (int)h, vh, grad_out, grad_vh);
  return launch_status();
}

int64_t gmp_ln_act_bwd_partial_rows(int64_t rows) { return bwd_blocks(rows); }

int gmp_sum_rows_f32(const float* partials, int64_t nrows, int64_t width, float* out,
                     void* stream) {
  GMP_CHECK_ARG(nrows >= 0 && width >= 0 && width <= INT32_MAX && nrows <= INT32_MAX);
  if (width == 0) return GMP_OK;
  GMP_CHECK_ARG(out && (nrows == 0 || partials));
  hipStream_t s = as_stream(stream);
  if (nrows == 0) return hip_check(hipMemsetAsync(out, 0, width * sizeof(float), s));
  sum_rows_kernel<<<(unsigned)ceil_div(width, kSC), kSC * kSG, 0, s>>>(partials, (int)nrows,
                                                                       (int)width, out);
  return launch_status();
}

}  // extern "C"
