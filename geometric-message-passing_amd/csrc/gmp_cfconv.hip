// K13: SchNet CFConv message + aggregation fused (PyG 2.3.1 CFConv, called at schnet.py:72):
//   message   msg[e] = x[src[e]] * W[e]            (CFConv.message: x_j * W)
//   aggregate out[i] = sum_{e : dst[e] = i} msg[e] (aggr "add", dim_size = N)
// The (E, F) message is never written: a wave owns one receiver segment of the stable CSR and
// streams its W rows (the only E-sized operand, read once) while the x rows come from L2 (the
// (N, F) node table is 25.6 MB at N = 50k, F = 128).  The same kernel run over the SENDER CSR
// with x := grad_out and the gather index := dst is the x-gradient of the forward; the
// W-gradient is the per-edge product grad_out[dst[e]] * x[src[e]] (gmp_cfconv_wgrad_f32).
// Per segment the rows are summed lane-strided in CSR order, then across the R row groups of
// the wave by xor shuffles — a fixed order: deterministic, no atomics.
// Gather indices outside [0, n_x) contribute zero and set *err (the CSR build flags the
// segment index the same way); the host checks the flags once per graph.
// Scaled forms (SchNet's W = filter(edge_attr) * C, schnet.py:72 over PyG CFConv.forward): a
// per-edge factor s[e] multiplies W[e] at load time (rounded as the reference's separate
// product), and the W-gradient is written as (g[dst] * x[src]) * s[e] — the gradient w.r.t.
// the filter output, so the (E, F) product W * C is never materialised.
#include "gmp_common.h"

namespace gmp {
namespace {

__device__ __forceinline__ int pow2_at_least(int64_t c) {
  int l = 1;
  while (l < c && l < 64) l <<= 1;
  return l;
}

__device__ __forceinline__ float4 fma4(float4 a, float4 b, float4 acc) {
  acc.x = fmaf(a.x, b.x, acc.x);
  acc.y = fmaf(a.y, b.y, acc.y);
  acc.z = fmaf(a.z, b.z, acc.z);
  acc.w = fmaf(a.w, b.w, acc.w);
  return acc;
}

__device__ __forceinline__ float4 scale4(float4 v, float s) {
  return make_float4(v.x * s, v.y * s, v.z * s, v.w * s);
}

template <bool SCALED>
__global__ __launch_bounds__(256) void cfconv_gather_mul_sum(
    const float4* __restrict__ x, int64_t n_x, const int64_t* __restrict__ xidx,
    const float4* __restrict__ w, const float* __restrict__ es, const int64_t* __restrict__ perm,
    const int64_t* __restrict__ rowptr, int64_t n_seg, int64_t cpr, float4* __restrict__ out,
    int32_t* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (seg >= n_seg) return;  // seg is wave-uniform: the whole wave leaves together
  const int64_t k0 = rowptr[seg], k1 = rowptr[seg + 1];
  const int lpr = pow2_at_least(cpr);
  const int R = 64 / lpr, sub = lane / lpr;
  for (int64_t cb = 0; cb < cpr; cb += 64) {
    const int64_t c = cb + lane % lpr;
    const bool active = c < cpr;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t k = k0 + sub;
    for (; k + R < k1; k += 2 * R) {  // two rows in flight per lane
      const int64_t e0 = perm[k], e1 = perm[k + R];
      const int64_t j0 = xidx[e0], j1 = xidx[e1];
      const bool ok0 = j0 >= 0 && j0 < n_x, ok1 = j1 >= 0 && j1 < n_x;
      if (active) {
        float4 w0 = w[e0 * cpr + c], w1 = w[e1 * cpr + c];
        if (SCALED) {
          w0 = scale4(w0, es[e0]);
          w1 = scale4(w1, es[e1]);
        }
        const float4 x0 = ok0 ? x[j0 * cpr + c] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 x1 = ok1 ? x[j1 * cpr + c] : make_float4(0.f, 0.f, 0.f, 0.f);
        acc = fma4(x0, w0, acc);
        acc = fma4(x1, w1, acc);
      }
      if (!(ok0 && ok1) && lane % lpr == 0) *err = 1;
    }
    if (k < k1) {
      const int64_t e0 = perm[k];
      const int64_t j0 = xidx[e0];
      const bool ok0 = j0 >= 0 && j0 < n_x;
      if (active && ok0) {
        float4 w0 = w[e0 * cpr + c];
        if (SCALED) w0 = scale4(w0, es[e0]);
        acc = fma4(x[j0 * cpr + c], w0, acc);
      }
      if (!ok0 && lane % lpr == 0) *err = 1;
    }
    for (int off = lpr; off < 64; off <<= 1) {
      acc.x += __shfl_xor(acc.x, off);
      acc.y += __shfl_xor(acc.y, off);
      acc.z += __shfl_xor(acc.z, off);
      acc.w += __shfl_xor(acc.w, off);
    }
    if (lane < lpr && active) out[seg * cpr + c] = acc;
  }
}

// dw[e] = g[gidx[e]] * x[xidx[e]] (* s[e]), one float4 per thread, grid-stride.
template <bool SCALED>
__global__ __launch_bounds__(256) void cfconv_wgrad(
    const float4* __restrict__ g, int64_t n_g, const int64_t* __restrict__ gidx,
    const float4* __restrict__ x, int64_t n_x, const int64_t* __restrict__ xidx,
    const float* __restrict__ es, int64_t n_items, int64_t cpr, float4* __restrict__ dw,
    int32_t* __restrict__ err) {
  const int64_t total = n_items * cpr;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t / cpr, c = t - e * cpr;
    const int64_t a = gidx[e], b = xidx[e];
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a >= 0 && a < n_g && b >= 0 && b < n_x) {
      const float4 p = g[a * cpr + c], q = x[b * cpr + c];
      r = make_float4(p.x * q.x, p.y * q.y, p.z * q.z, p.w * q.w);
      if (SCALED) r = scale4(r, es[e]);
    } else {
      *err = 1;
    }
    dw[t] = r;
  }
}

bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_cfconv_aggregate_scaled_f32(const float* x, int64_t n_x, const int64_t* xidx,
                                    const float* w, const float* escale, int64_t n_items,
                                    int64_t F, const int64_t* perm, const int64_t* rowptr,
                                    int64_t n_seg, float* out, int32_t* err, void* stream) {
  GMP_CHECK_ARG(n_x >= 0 && n_items >= 0 && F >= 0 && n_seg >= 0);
  if (n_seg == 0 || F == 0) return GMP_OK;
  GMP_CHECK_ARG(F % 4 == 0 && rowptr && out && err);
  GMP_CHECK_ARG(n_items == 0 || (x && xidx && w && perm));
  GMP_CHECK_ARG(aligned16(out) && (n_items == 0 || (aligned16(x) && aligned16(w))));
  const unsigned grid = (unsigned)ceil_div(n_seg, 4);
  if (escale)
    cfconv_gather_mul_sum<true><<<grid, 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(x), n_x, xidx, reinterpret_cast<const float4*>(w), escale,
        perm, rowptr, n_seg, F / 4, reinterpret_cast<float4*>(out), err);
  else
    cfconv_gather_mul_sum<false><<<grid, 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(x), n_x, xidx, reinterpret_cast<const float4*>(w), nullptr,
        perm, rowptr, n_seg, F / 4, reinterpret_cast<float4*>(out), err);
  return launch_status();
}

int gmp_cfconv_aggregate_f32(const float* x, int64_t n_x, const int64_t* xidx, const float* w,
                             int64_t n_items, int64_t F, const int64_t* perm,
                             const int64_t* rowptr, int64_t n_seg, float* out, int32_t* err,
                             void* stream) {
  return gmp_cfconv_aggregate_scaled_f32(x, n_x, xidx, w, nullptr, n_items, F, perm, rowptr,
                                         n_seg, out, err, stream);
}

int gmp_cfconv_wgrad_scaled_f32(const float* g, int64_t n_g, const int64_t* gidx, const float* x,
                                int64_t n_x, const int64_t* xidx, const float* escale,
                                int64_t n_items, int64_t F, float* dw, int32_t* err,
                                void* stream) {
  GMP_CHECK_ARG(n_g >= 0 && n_x >= 0 && n_items >= 0 && F >= 0);
  if (n_items == 0 || F == 0) return GMP_OK;
  GMP_CHECK_ARG(F % 4 == 0 && g && gidx && x && xidx && dw && err);
  GMP_CHECK_ARG(aligned16(g) && aligned16(x) && aligned16(dw));
  const int64_t total = n_items * (F / 4);
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(total, 256), 256 * 64);
  if (escale)
    cfconv_wgrad<true><<<grid, 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(g), n_g, gidx, reinterpret_cast<const float4*>(x), n_x,
        xidx, escale, n_items, F / 4, reinterpret_cast<float4*>(dw), err);
  else
    cfconv_wgrad<false><<<grid, 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4*>(g), n_g, gidx, reinterpret_cast<const float4*>(x), n_x,
        xidx, nullptr, n_items, F / 4, reinterpret_cast<float4*>(dw), err);
  return launch_status();
}

int gmp_cfconv_wgrad_f32(const float* g, int64_t n_g, const int64_t* gidx, const float* x,
                         int64_t n_x, const int64_t* xidx, int64_t n_items, int64_t F, float* dw,
                         int32_t* err, void* stream) {
  return gmp_cfconv_wgrad_scaled_f32(g, n_g, gidx, x, n_x, xidx, nullptr, n_items, F, dw, err,
                                     stream);
}

}  // extern "C"
