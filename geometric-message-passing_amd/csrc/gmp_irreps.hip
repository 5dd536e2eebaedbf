// K16: per-node irreps epilogues of the TP convolution (models/layers/tfn_layer.py:89-92):
// e3nn nn.Gate(scalars [silu], gates [sigmoid], gated) and e3nn nn.BatchNorm(irreps) (training:
// batch statistics + running-stat update; eval: running statistics), forward and backward.
// HBM-bound row-major (B, C) passes; reductions are fixed-order partial sums (deterministic),
// accumulated in fp64 (the statistics of 50k-row batches feed a mean-centred output).
//
// Gate (e3nn 0.5 nn.Gate over tfn_layer.py:45-63): y = [c_act silu(x_s), x_v * c_gate
// sigmoid(x_g)] with the normalize2mom constants c_act, c_gate baked in by the caller.
// Column maps are built once per module on the host:
//   out_map (c_out, 2) int32: {source column, gate column or -1 (scalar)}
//   in_map  (c_in, 4)  int32: {kind, a, b, d}; kind 0 scalar (a = out col); 1 gate (a = first
//     out col of its gated channel, b = first in col of that channel, d = 2l+1); 2 gated
//     (a = out col, b = gate col).
//
// BatchNorm (e3nn 0.5 nn.BatchNorm, reduce 'mean', normalization 'component', affine): per
// channel u of an irrep block (mul x (2l+1) columns): scalars (0e) are centred by the batch
// mean over (B, 2l+1); every channel is scaled by w_u (mean over (B, 2l+1) of f^2 + eps)^-1/2;
// scalars get + bias.  running_mean / running_var <- (1 - m) old + m batch value.
//   col_chan (C) int32: channel of column c;  chan_info (nf, 2) int32: {2l+1, scalar index
//   (into running_mean / bias) or -1}.
#include "gmp_common.h"

namespace gmp {
namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void gate_fwd_kernel(int64_t B, int c_in, int c_out, const int2* __restrict__ omap,
                                float c_act, float c_gate, const float* __restrict__ x,
                                float* __restrict__ y) {
  const int64_t n = B * c_out;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / c_out;
    const int j = (int)(i - b * c_out);
    const int2 m = omap[j];
    const float* xr = x + b * c_in;
    const float v = xr[m.x];
    y[i] = m.y < 0 ? c_act * (v * sigm(v)) : v * (c_gate * sigm(xr[m.y]));
  }
}

__global__ void gate_bwd_kernel(int64_t B, int c_in, int c_out, const int4* __restrict__ imap,
                                float c_act, float c_gate, const float* __restrict__ x,
                                const float* __restrict__ gy, float* __restrict__ gx) {
  const int64_t n = B * c_in;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / c_in;
    const int c = (int)(i - b * c_in);
    const int4 m = imap[c];
    const float* xr = x + b * c_in;
    const float* gr = gy + b * c_out;
    float r;
    if (m.x == 0) {  // d/dx c silu(x) = c s (1 + x (1 - s))
      const float v = xr[c], s = sigm(v);
      r = gr[m.y] * c_act * (s * (1.f + v * (1.f - s)));
    } else if (m.x == 1) {  // gate: c s (1 - s) sum_k g[o + k] x_v[k]
      const float s = sigm(xr[c]);
      float acc = 0.f;
      for (int k = 0; k < m.w; ++k) acc += gr[m.y + k] * xr[m.z + k];
      r = acc * (c_gate * (s * (1.f - s)));
    } else {  // gated: g c sigmoid(x_gate)
      r = gr[m.y] * (c_gate * sigm(xr[m.z]));
    }
    gx[i] = r;
  }
}

// ---------------------------------------------------------------------------- BatchNorm
constexpr int kBnCols = 64;    // columns per block (lane = column: coalesced row segments)
constexpr int kBnRows = 256;   // minimum rows per partial
constexpr int kBnMaxRb = 32;   // at most this many row-block partials per column

inline int64_t bn_rows_per_block(int64_t B) {
  const int64_t r = ceil_div(B, kBnMaxRb);
  return r > kBnRows ? r : kBnRows;
}

enum BnMode { kSum = 0, kSqDev = 1, kGrad = 2 };

// part0[rb][c] = sum over the row block of (x - shift[chan]) (kSum: shift 0) or its square
// (kSqDev); kGrad: part0 = sum gy, part1 = sum gy (x - shift).  4 waves split the rows
// (stride 4), combined in wave order through LDS.
template <int MODE>
__global__ void __launch_bounds__(256) bn_partials_kernel(
    int64_t B, int C, int64_t rpb, const int* __restrict__ col_chan,
    const float* __restrict__ shift, const float* __restrict__ x, const float* __restrict__ gy,
    double* __restrict__ part0, double* __restrict__ part1) {
  __shared__ double red[2][4][kBnCols];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * kBnCols + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rpb;
  const int64_t r1 = r0 + rpb < B ? r0 + rpb : B;
  double a0 = 0.0, a1 = 0.0;
  if (c < C) {
    const float sh = MODE == kSum ? 0.f : shift[col_chan[c]];
    for (int64_t r = r0 + wv; r < r1; r += 4) {
      const double v = (double)(x[r * C + c] - sh);
      if (MODE == kSum) {
        a0 += v;
      } else if (MODE == kSqDev) {
        a0 += v * v;
      } else {
        const double g = (double)gy[r * C + c];
        a0 += g;
        a1 += g * v;
      }
    }
  }
  red[0][wv][lane] = a0;
  red[1][wv][lane] = a1;
  __syncthreads();
  if (wv == 0 && c < C) {
    const double s0 = ((red[0][0][lane] + red[0][1][lane]) + red[0][2][lane]) + red[0][3][lane];
    part0[(int64_t)blockIdx.y * C + c] = s0;
    if (MODE == kGrad) {
      const double s1 = ((red[1][0][lane] + red[1][1][lane]) + red[1][2][lane]) + red[1][3][lane];
      part1[(int64_t)blockIdx.y * C + c] = s1;
    }
  }
}

// per channel: the sum over its columns (first column chan_col[u], d columns) and row blocks,
// in a fixed order
__device__ __forceinline__ double chan_total(const double* __restrict__ part, int nrb, int C,
                                             int c0, int d) {
  double s = 0.0;
  for (int k = 0; k < d; ++k) {
    double t = 0.0;
    for (int rb = 0; rb < nrb; ++rb) t += part[(int64_t)rb * C + c0 + k];
    s += t;
  }
  return s;
}

// STAGE 0 (training, after kSum): shift[u] = batch mean (scalars) / 0, running_mean update.
// STAGE 1 (training, after kSqDev): invstd[u] = (norm + eps)^-1/2, running_var update.
// STAGE 2 (eval): shift / invstd from the running statistics.
template <int STAGE>
__global__ void bn_finalize_kernel(int nf, int C, int nrb, int64_t B,
                                   const int* __restrict__ chan_col,
                                   const int2* __restrict__ chan_info,
                                   const double* __restrict__ part, float momentum, float eps,
                                   float* __restrict__ running_mean,
                                   float* __restrict__ running_var, float* __restrict__ shift,
                                   float* __restrict__ invstd) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nf) return;
  const int2 info = chan_info[u];
  const int d = info.x, si = info.y;
  const double cnt = (double)B * (double)d;
  if (STAGE == 0) {
    float m = 0.f;
    if (si >= 0) {
      m = (float)(chan_total(part, nrb, C, chan_col[u], d) / cnt);
      if (running_mean) running_mean[si] = (1.f - momentum) * running_mean[si] + momentum * m;
    }
    shift[u] = m;
  } else if (STAGE == 1) {
    const float nv = (float)(chan_total(part, nrb, C, chan_col[u], d) / cnt);
    if (running_var) running_var[u] = (1.f - momentum) * running_var[u] + momentum * nv;
    invstd[u] = 1.f / sqrtf(nv + eps);
  } else {
    shift[u] = si >= 0 ? running_mean[si] : 0.f;
    invstd[u] = 1.f / sqrtf(running_var[u] + eps);
  }
}

__global__ void bn_apply_kernel(int64_t B, int C, const int* __restrict__ col_chan,
                                const int2* __restrict__ chan_info,
                                const float* __restrict__ shift, const float* __restrict__ invstd,
                                const float* __restrict__ weight, const float* __restrict__ bias,
                                const float* __restrict__ x, float* __restrict__ y) {
  const int64_t n = B * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int u = col_chan[c];
    const int si = chan_info[u].y;
    const float s = invstd[u] * weight[u];
    float v = (x[i] - shift[u]) * s;
    if (si >= 0 && bias) v += bias[si];
    y[i] = v;
  }
}

// backward coefficients per channel: gbias = sum gy (scalars), gweight = sum gy xc invstd;
// dx = s (gy - mg) - xc k with s = w invstd, training: mg = mean gy (scalars; 0 otherwise),
// k = s mean(gy xc) invstd^2; eval: mg = k = 0.
__global__ void bn_bwd_finalize_kernel(int nf, int C, int nrb, int64_t B, int training,
                                       const int* __restrict__ chan_col,
                                       const int2* __restrict__ chan_info,
                                       const double* __restrict__ part0,
                                       const double* __restrict__ part1,
                                       const float* __restrict__ weight,
                                       const float* __restrict__ invstd,
                                       float* __restrict__ gweight, float* __restrict__ gbias,
                                       float* __restrict__ coef) {
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nf) return;
  const int2 info = chan_info[u];
  const int d = info.x, si = info.y;
  const double cnt = (double)B * (double)d;
  const double sg = chan_total(part0, nrb, C, chan_col[u], d);
  const double sgx = chan_total(part1, nrb, C, chan_col[u], d);
  const float is = invstd[u], s = weight[u] * is;
  if (gweight) gweight[u] = (float)(sgx * is);
  if (si >= 0 && gbias) gbias[si] = (float)sg;
  coef[3 * u] = s;
  coef[3 * u + 1] = training && si >= 0 ? (float)(sg / cnt) : 0.f;
  coef[3 * u + 2] = training ? (float)((double)s * (sgx / cnt) * ((double)is * is)) : 0.f;
}

__global__ void bn_bwd_apply_kernel(int64_t B, int C, const int* __restrict__ col_chan,
                                    const float* __restrict__ shift,
                                    const float* __restrict__ coef, const float* __restrict__ x,
                                    const float* __restrict__ gy, float* __restrict__ gx) {
  const int64_t n = B * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int u = col_chan[c];
    const float s = coef[3 * u], mg = coef[3 * u + 1], k = coef[3 * u + 2];
    gx[i] = s * (gy[i] - mg) - (x[i] - shift[u]) * k;
  }
}

int grid_elems(int64_t n) {
  int64_t g = ceil_div(n, 256);
  const int64_t cap = (int64_t)device_cu_count() * 16;
  return (int)(g > cap ? cap : (g < 1 ? 1 : g));
}

struct BnWs {
  float *part0, *part1, *coef;
  int* chan_col;
};

size_t bn_ws_floats(int64_t B, int C, int nf) {
  const int64_t nrb = ceil_div(B, bn_rows_per_block(B));
  return (size_t)(4 * nrb * C + 3 * (int64_t)nf + nf + 64);  // 2 fp64 partial planes
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_gate_fwd_f32(int64_t B, int c_in, int c_out, const int32_t* out_map, float c_act,
                     float c_gate, const float* x, float* y, void* stream) {
  GMP_CHECK_ARG(B >= 0 && c_in > 0 && c_out > 0);
  if (B == 0) return GMP_OK;
  GMP_CHECK_ARG(out_map && x && y);
  gate_fwd_kernel<<<grid_elems(B * c_out), 256, 0, as_stream(stream)>>>(
      B, c_in, c_out, reinterpret_cast<const int2*>(out_map), c_act, c_gate, x, y);
  return launch_status();
}

int gmp_gate_bwd_f32(int64_t B, int c_in, int c_out, const int32_t* in_map, float c_act,
                     float c_gate, const float* x, const float* grad_y, float* grad_x,
                     void* stream) {
  GMP_CHECK_ARG(B >= 0 && c_in > 0 && c_out > 0);
  if (B == 0) return GMP_OK;
  GMP_CHECK_ARG(in_map && x && grad_y && grad_x);
  gate_bwd_kernel<<<grid_elems(B * c_in), 256, 0, as_stream(stream)>>>(
      B, c_in, c_out, reinterpret_cast<const int4*>(in_map), c_act, c_gate, x, grad_y, grad_x);
  return launch_status();
}

size_t gmp_irreps_bn_workspace_size(int64_t B, int C, int nf) {
  return bn_ws_floats(B, C, nf) * sizeof(float);
}

int gmp_irreps_bn_fwd_f32(int64_t B, int C, int nf, const int32_t* col_chan,
                          const int32_t* chan_col, const int32_t* chan_info, const float* x,
                          const float* weight, const float* bias, float* running_mean,
                          float* running_var, int training, float momentum, float eps, float* y,
                          float* save_shift, float* save_invstd, void* workspace,
                          size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(B >= 0 && C > 0 && nf > 0);
  GMP_CHECK_ARG(col_chan && chan_col && chan_info && weight && save_shift && save_invstd);
  if (!training) GMP_CHECK_ARG(running_var);  // (running_mean: read for scalar channels only)
  if (training && B == 0) return GMP_OK;
  GMP_CHECK_ARG(B == 0 || (x && y));
  GMP_CHECK_ARG(workspace && workspace_bytes >= gmp_irreps_bn_workspace_size(B, C, nf));
  hipStream_t s = as_stream(stream);
  const int2* info = reinterpret_cast<const int2*>(chan_info);
  const int64_t rpb = bn_rows_per_block(B);
  const int nrb = (int)ceil_div(B, rpb);
  double* part = static_cast<double*>(workspace);
  const dim3 pg((unsigned)ceil_div(C, kBnCols), (unsigned)(nrb > 0 ? nrb : 1));
  const int fg = (int)ceil_div(nf, 256);
  if (training) {
    bn_partials_kernel<kSum><<<pg, 256, 0, s>>>(B, C, rpb, col_chan, nullptr, x, nullptr, part,
                                                nullptr);
    bn_finalize_kernel<0><<<fg, 256, 0, s>>>(nf, C, nrb, B, chan_col, info, part, momentum, eps,
                                             running_mean, running_var, save_shift, save_invstd);
    bn_partials_kernel<kSqDev><<<pg, 256, 0, s>>>(B, C, rpb, col_chan, save_shift, x, nullptr, part,
                                                  nullptr);
    bn_finalize_kernel<1><<<fg, 256, 0, s>>>(nf, C, nrb, B, chan_col, info, part, momentum, eps,
                                             running_mean, running_var, save_shift, save_invstd);
  } else {
    bn_finalize_kernel<2><<<fg, 256, 0, s>>>(nf, C, 0, B, chan_col, info, nullptr, momentum, eps,
                                             running_mean, running_var, save_shift, save_invstd);
  }
  if (B > 0)
    bn_apply_kernel<<<grid_elems(B * C), 256, 0, s>>>(B, C, col_chan, info, save_shift,
                                                      save_invstd, weight, bias, x, y);
  return launch_status();
}

int gmp_irreps_bn_bwd_f32(int64_t B, int C, int nf, const int32_t* col_chan,
                          const int32_t* chan_col, const int32_t* chan_info, const float* x,
                          const float* grad_y, const float* weight, const float* save_shift,
                          const float* save_invstd, int training, float* grad_x,
                          float* grad_weight, float* grad_bias, void* workspace,
                          size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(B >= 0 && C > 0 && nf > 0);
  GMP_CHECK_ARG(col_chan && chan_col && chan_info && weight && save_shift && save_invstd);
  GMP_CHECK_ARG(workspace && workspace_bytes >= gmp_irreps_bn_workspace_size(B, C, nf));
  GMP_CHECK_ARG(B == 0 || (x && grad_y && grad_x));
  hipStream_t s = as_stream(stream);
  const int2* info = reinterpret_cast<const int2*>(chan_info);
  const int64_t rpb = bn_rows_per_block(B);
  const int nrb = (int)ceil_div(B, rpb);
  double* p0 = static_cast<double*>(workspace);
  double* p1 = p0 + (int64_t)nrb * C;
  float* coef = reinterpret_cast<float*>(p1 + (int64_t)nrb * C);
  const dim3 pg((unsigned)ceil_div(C, kBnCols), (unsigned)(nrb > 0 ? nrb : 1));
  if (B > 0)
    bn_partials_kernel<kGrad><<<pg, 256, 0, s>>>(B, C, rpb, col_chan, save_shift, x, grad_y, p0, p1);
  bn_bwd_finalize_kernel<<<(int)ceil_div(nf, 256), 256, 0, s>>>(
      nf, C, nrb, B, training, chan_col, info, p0, p1, weight, save_invstd, grad_weight,
      grad_bias, coef);
  if (B > 0)
    bn_bwd_apply_kernel<<<grid_elems(B * C), 256, 0, s>>>(B, C, col_chan, save_shift, coef, x,
                                                          grad_y, grad_x);
  return launch_status();
}

}  // extern "C"
