// Index-side kernels of libgmp: stable CSR build, row gather (K2), segmented reduce (K3) and
// its backward.  All HBM-bound; see DESIGN.md §Kernels for the per-unit byte counts.
#include <hipcub/hipcub.hpp>

#include <map>
#include <mutex>
#include <utility>

#include "gmp_common.h"

namespace gmp {

thread_local int g_last_hip_error = 0;

int device_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      cus = prop.multiProcessorCount;
    if (cus <= 0) cus = 256;
  }
  return cus;
}

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

int key_bits(int64_t n_seg) {
  int b = 1;
  while ((int64_t(1) << b) <= n_seg) ++b;  // keys in [0, n_seg] (n_seg = out-of-range sentinel)
  return b;
}

size_t cub_sort_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 32,
                                     (hipStream_t)0);
  return bytes;
}

__global__ void csr_prepare_keys(const int64_t* __restrict__ index, int64_t n, int64_t n_seg,
                                 uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                 int32_t* __restrict__ err_flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = index[i];
    bool ok = (k >= 0) && (k < n_seg);
    if (!ok && err_flag) *err_flag = 1;
    keys[i] = ok ? (uint32_t)k : (uint32_t)n_seg;
    vals[i] = (uint32_t)i;
  }
}

// rowptr[s] = first sorted position k with key[k] >= s (s = 0..n_seg).
__global__ void csr_finish(const uint32_t* __restrict__ keys_sorted,
                           const uint32_t* __restrict__ vals_sorted, int64_t n, int64_t n_seg,
                           const int64_t* __restrict__ payload, int64_t* __restrict__ perm,
                           int64_t* __restrict__ rowptr, int64_t* __restrict__ index_sorted,
                           int64_t* __restrict__ payload_out) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= n;
       k += (int64_t)gridDim.x * blockDim.x) {
    int64_t prev = (k == 0) ? -1 : (int64_t)keys_sorted[k - 1];
    int64_t cur = (k == n) ? n_seg : (int64_t)keys_sorted[k];
    for (int64_t s = prev + 1; s <= cur && s <= n_seg; ++s) rowptr[s] = k;
    if (k < n) {
      int64_t p = vals_sorted[k];
      if (perm) perm[k] = p;
      if (index_sorted) index_sorted[k] = (cur < n_seg) ? cur : -1;
      if (payload_out) payload_out[k] = payload[p];
    }
  }
}

template <int VEC>
__global__ void gather_rows_kernel(const float* __restrict__ src, int64_t n_rows, int64_t F,
                                   const int64_t* __restrict__ index, int64_t n_index,
                                   float* __restrict__ out, int32_t* __restrict__ err_flag) {
  const int64_t fv = F / VEC;
  const int64_t total = n_index * fv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t e = t / fv, c = t - e * fv;
    int64_t r = index[e];
    if constexpr (VEC == 4) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r >= 0 && r < n_rows) v = reinterpret_cast<const float4*>(src + r * F)[c];
      else if (err_flag) *err_flag = 1;
      reinterpret_cast<float4*>(out + e * F)[c] = v;
    } else {
      float v = 0.f;
      if (r >= 0 && r < n_rows) v = src[r * F + c];
      else if (err_flag) *err_flag = 1;
      out[e * F + c] = v;
    }
  }
}

// ------------------------------------------------------------------------------ K3 wave reduce
// A wave reduces rows [k_beg, k_end) of the (perm-indexed) item list.  Lanes are split into
// R = 64/LPR row slots x LPR column lanes (LPR = lanes per row, a power of two >= F/VEC, <= 64),
// so a 128-float row uses 32 lanes and two rows are read per step; rows are unrolled x4.
// Partials of the R row slots are combined in a fixed order (deterministic).
struct RedVal {
  float v;
  int64_t arg;
};

template <int REDUCE>
__device__ __forceinline__ void red_combine(float& acc, int64_t& arg, float x, int64_t xa) {
  if (REDUCE == GMP_REDUCE_MAX) {
    if (x > acc || (x == acc && xa < arg)) { acc = x; arg = xa; }
  } else {
    acc += x;
  }
}

template <int VEC, int REDUCE>
__device__ __forceinline__ void wave_reduce_rows(const float* __restrict__ src, int64_t F,
                                                 const int64_t* __restrict__ perm, int64_t k_beg,
                                                 int64_t k_end, int64_t n_items, int64_t c,
                                                 int lpr, float (&acc)[VEC], int64_t (&arg)[VEC]) {
  const int lane = threadIdx.x & 63;
  const int R = 64 / lpr, sub = lane / lpr;
#pragma unroll
  for (int v = 0; v < VEC; ++v) {
    acc[v] = (REDUCE == GMP_REDUCE_MAX) ? -INFINITY : 0.f;
    arg[v] = n_items;
  }
  const bool active = c < F / VEC;
  int64_t k = k_beg + sub;
  for (; k + 3 * R < k_end; k += 4 * R) {
    int64_t it[4];
    float x[4][VEC];
#pragma unroll
    for (int u = 0; u < 4; ++u) it[u] = perm ? perm[k + u * R] : (k + u * R);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* p = src + it[u] * F + c * VEC;
      if (!active) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) x[u][v] = 0.f;
      } else if constexpr (VEC == 4) {
        float4 q = *reinterpret_cast<const float4*>(p);
        x[u][0] = q.x; x[u][1] = q.y; x[u][2] = q.z; x[u][3] = q.w;
      } else if constexpr (VEC == 2) {
        float2 q = *reinterpret_cast<const float2*>(p);
        x[u][0] = q.x; x[u][1] = q.y;
      } else {
        x[u][0] = p[0];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < VEC; ++v) red_combine<REDUCE>(acc[v], arg[v], x[u][v], it[u]);
  }
  for (; k < k_end; k += R) {
    const int64_t i = perm ? perm[k] : k;
    if (active) {
      const float* p = src + i * F + c * VEC;
#pragma unroll
      for (int v = 0; v < VEC; ++v) red_combine<REDUCE>(acc[v], arg[v], p[v], i);
    }
  }
  // combine the R row slots (lanes differing in the bits above log2(lpr))
  for (int m = lpr; m < 64; m <<= 1) {
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const float ox = __shfl_xor(acc[v], m);
      const int64_t oa = __shfl_xor(arg[v], m);
      if (REDUCE == GMP_REDUCE_MAX) {
        // keep the larger value; ties -> first occurrence (smallest item index)
        if (ox > acc[v] || (ox == acc[v] && oa < arg[v])) { acc[v] = ox; arg[v] = oa; }
      } else {
        // fixed order: lower slot + upper slot
        const bool upper = (lane & m) != 0;
        acc[v] = upper ? ox + acc[v] : acc[v] + ox;
      }
    }
  }
}

__device__ __forceinline__ int lanes_per_row(int64_t cpr) {
  int l = 1;
  while (l < cpr && l < 64) l <<= 1;
  return l;
}

// One wave per segment.
template <int VEC, int REDUCE>
__global__ __launch_bounds__(256) void segment_reduce_wave(
    const float* __restrict__ src, int64_t n_items, int64_t F, const int64_t* __restrict__ perm,
    const int64_t* __restrict__ rowptr, int64_t n_seg, float* __restrict__ out,
    int64_t* __restrict__ argmax) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (seg >= n_seg) return;
  const int64_t k0 = rowptr[seg], k1 = rowptr[seg + 1];
  const int64_t cpr = F / VEC;
  const int lpr = lanes_per_row(cpr);
  for (int64_t cb = 0; cb < cpr; cb += 64) {
    const int64_t c = cb + lane % lpr;
    float acc[VEC];
    int64_t arg[VEC];
    wave_reduce_rows<VEC, REDUCE>(src, F, perm, k0, k1, n_items, c, lpr, acc, arg);
    const int64_t cnt = k1 - k0;
    if (lane < lpr && c < cpr) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float r = acc[v];
        if (REDUCE == GMP_REDUCE_MEAN) r = r / (float)(cnt > 0 ? cnt : 1);
        if (REDUCE == GMP_REDUCE_MAX && cnt == 0) r = 0.f;
        out[seg * F + c * VEC + v] = r;
        if (REDUCE == GMP_REDUCE_MAX && argmax) argmax[seg * F + c * VEC + v] = arg[v];
      }
    }
  }
}

// Long segments (sum / mean): block (seg, part) reduces a contiguous slice of the segment with
// its 4 waves; partial[seg][part][F] in a fixed order; finished by segment_split_finish.
template <int VEC, int REDUCE>
__global__ __launch_bounds__(256) void segment_reduce_split(
    const float* __restrict__ src, int64_t n_items, int64_t F, const int64_t* __restrict__ perm,
    const int64_t* __restrict__ rowptr, int64_t n_seg, int64_t S, float* __restrict__ partial) {
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t seg = blockIdx.x / S, part = blockIdx.x % S;
  const int64_t k0 = rowptr[seg], k1 = rowptr[seg + 1], len = k1 - k0;
  const int64_t pb = k0 + len * part / S, pe = k0 + len * (part + 1) / S;
  const int64_t wb = pb + (pe - pb) * w / 4, we = pb + (pe - pb) * (w + 1) / 4;
  const int64_t cpr = F / VEC;
  const int lpr = lanes_per_row(cpr);
  for (int64_t cb = 0; cb < cpr; cb += 64) {
    const int64_t c = cb + lane % lpr;
    float acc[VEC];
    int64_t arg[VEC];
    wave_reduce_rows<VEC, REDUCE>(src, F, perm, wb, we, n_items, c, lpr, acc, arg);
    if (lane < lpr) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) red[w][lane * VEC + v] = acc[v];
    }
    __syncthreads();
    if (w == 0 && lane < lpr && c < cpr) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const float t = ((red[0][lane * VEC + v] + red[1][lane * VEC + v]) + red[2][lane * VEC + v]) +
                        red[3][lane * VEC + v];
        partial[(seg * S + part) * F + c * VEC + v] = t;
      }
    }
    __syncthreads();
  }
}

template <int REDUCE>
__global__ void segment_split_finish(const float* __restrict__ partial, const int64_t* __restrict__ rowptr,
                                     int64_t n_seg, int64_t S, int64_t F, float* __restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n_seg * F;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t seg = t / F, f = t - seg * F;
    float s = 0.f;
    for (int64_t p = 0; p < S; ++p) s += partial[(seg * S + p) * F + f];
    if (REDUCE == GMP_REDUCE_MEAN) {
      const int64_t cnt = rowptr[seg + 1] - rowptr[seg];
      s = s / (float)(cnt > 0 ? cnt : 1);
    }
    out[t] = s;
  }
}

// Small feature dims (F < 16): one thread per (segment, feature).
template <int REDUCE>
__global__ void segment_reduce_thread(const float* __restrict__ src, int64_t n_items, int64_t F,
                                      const int64_t* __restrict__ perm,
                                      const int64_t* __restrict__ rowptr, int64_t n_seg,
                                      float* __restrict__ out, int64_t* __restrict__ argmax) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n_seg * F;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t seg = t / F, f = t - seg * F;
    int64_t k0 = rowptr[seg], k1 = rowptr[seg + 1];
    float acc = (REDUCE == GMP_REDUCE_MAX) ? -INFINITY : 0.f;
    int64_t arg = n_items;
    for (int64_t k = k0; k < k1; ++k) {
      int64_t i = perm ? perm[k] : k;
      float x = src[i * F + f];
      if (REDUCE == GMP_REDUCE_MAX) {
        if (x > acc) { acc = x; arg = i; }
      } else {
        acc += x;
      }
    }
    int64_t cnt = k1 - k0;
    if (REDUCE == GMP_REDUCE_MEAN) acc = acc / (float)(cnt > 0 ? cnt : 1);
    if (REDUCE == GMP_REDUCE_MAX && cnt == 0) acc = 0.f;
    out[t] = acc;
    if (REDUCE == GMP_REDUCE_MAX && argmax) argmax[t] = arg;
  }
}

template <int REDUCE>
__global__ void segment_reduce_bwd_kernel(const float* __restrict__ grad_out, int64_t n_seg,
                                          int64_t F, const int64_t* __restrict__ index,
                                          int64_t n_items, const int64_t* __restrict__ rowptr,
                                          const int64_t* __restrict__ argmax,
                                          float* __restrict__ grad_src) {
  const int64_t total = n_items * F;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t e = t / F, f = t - e * F;
    int64_t s = index[e];
    float g = 0.f;
    if (s >= 0 && s < n_seg) {
      g = grad_out[s * F + f];
      if (REDUCE == GMP_REDUCE_MEAN) {
        int64_t cnt = rowptr[s + 1] - rowptr[s];
        g = g / (float)(cnt > 0 ? cnt : 1);
      } else if (REDUCE == GMP_REDUCE_MAX) {
        g = (argmax[s * F + f] == e) ? g : 0.f;
      }
    }
    grad_src[t] = g;
  }
}

// SUM / MEAN with F % 4 == 0: one float4 per thread, 32-bit index arithmetic (n_items * F / 4
// < 2^31): the mean backward of a 1M-edge x 128 message is a row gather at HBM speed
template <int REDUCE>
__global__ void segment_reduce_bwd_vec4_kernel(const float4* __restrict__ grad_out, int n_seg,
                                               int F4, const int64_t* __restrict__ index,
                                               int total, const int64_t* __restrict__ rowptr,
                                               float4* __restrict__ grad_src) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int e = t / F4, f = t - e * F4;
    const int64_t sg = index[e];
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if (sg >= 0 && sg < n_seg) {
      g = grad_out[sg * F4 + f];
      if (REDUCE == GMP_REDUCE_MEAN) {
        const int64_t cnt = rowptr[sg + 1] - rowptr[sg];
        const float inv = 1.f / (float)(cnt > 0 ? cnt : 1);
        g.x *= inv; g.y *= inv; g.z *= inv; g.w *= inv;
      }
    }
    grad_src[t] = g;
  }
}

inline int grid_for(int64_t work, int threads) {
  int64_t g = ceil_div(work, threads);
  int64_t cap = (int64_t)device_cu_count() * 16;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_abi_version(void) { return GMP_ABI_VERSION; }

const char* gmp_error_string(int code) {
  switch (code) {
    case GMP_OK: return "ok";
    case GMP_ERR_ARG: return "invalid argument";
    case GMP_ERR_HIP: return "HIP runtime error";
    case GMP_ERR_UNSUPPORTED: return "unsupported shape for this kernel";
    case GMP_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown error";
  }
}

int gmp_last_hip_error(void) { return g_last_hip_error; }

size_t gmp_csr_workspace_size(int64_t n_items, int64_t n_seg) {
  (void)n_seg;
  if (n_items <= 0) return kAlign;
  size_t n = (size_t)n_items;
  return 4 * align_up(n * sizeof(uint32_t)) + align_up(cub_sort_bytes(n_items)) + kAlign;
}

int gmp_csr_build(const int64_t* index, int64_t n_items, int64_t n_seg, const int64_t* payload,
                  int64_t* perm, int64_t* rowptr, int64_t* index_sorted, int64_t* payload_out,
                  int32_t* err_flag, void* workspace, size_t workspace_bytes, void* stream) {
  GMP_CHECK_ARG(n_items >= 0 && n_seg >= 0 && rowptr != nullptr);
  GMP_CHECK_ARG(n_items < (int64_t(1) << 31) && n_seg < (int64_t(1) << 31) - 1);
  GMP_CHECK_ARG(n_items == 0 || index != nullptr);
  GMP_CHECK_ARG(payload_out == nullptr || payload != nullptr);
  hipStream_t s = as_stream(stream);
  if (n_items == 0) {
    int rc = hip_check(hipMemsetAsync(rowptr, 0, (n_seg + 1) * sizeof(int64_t), s));
    return rc;
  }
  if (workspace_bytes < gmp_csr_workspace_size(n_items, n_seg) || workspace == nullptr)
    return GMP_ERR_WORKSPACE;
  char* ws = reinterpret_cast<char*>(
      (reinterpret_cast<uintptr_t>(workspace) + kAlign - 1) / kAlign * kAlign);
  size_t nb = align_up((size_t)n_items * sizeof(uint32_t));
  uint32_t* keys_in = reinterpret_cast<uint32_t*>(ws);
  uint32_t* keys_out = reinterpret_cast<uint32_t*>(ws + nb);
  uint32_t* vals_in = reinterpret_cast<uint32_t*>(ws + 2 * nb);
  uint32_t* vals_out = reinterpret_cast<uint32_t*>(ws + 3 * nb);
  void* temp = ws + 4 * nb;
  size_t temp_bytes = cub_sort_bytes(n_items);

  csr_prepare_keys<<<grid_for(n_items, 256), 256, 0, s>>>(index, n_items, n_seg, keys_in, vals_in,
                                                          err_flag);
  int rc = launch_status();
  if (rc) return rc;
  rc = hip_check(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in,
                                                    vals_out, (int)n_items, 0, key_bits(n_seg), s));
  if (rc) return rc;
  csr_finish<<<grid_for(n_items + 1, 256), 256, 0, s>>>(keys_out, vals_out, n_items, n_seg,
                                                        payload, perm, rowptr, index_sorted,
                                                        payload_out);
  return launch_status();
}

int gmp_gather_rows_f32(const float* src, int64_t n_rows, int64_t F, const int64_t* index,
                        int64_t n_index, float* out, int32_t* err_flag, void* stream) {
  GMP_CHECK_ARG(n_rows >= 0 && F >= 0 && n_index >= 0);
  if (n_index == 0 || F == 0) return GMP_OK;
  GMP_CHECK_ARG(src && index && out);
  hipStream_t s = as_stream(stream);
  bool v4 = (F % 4 == 0) && (reinterpret_cast<uintptr_t>(src) % 16 == 0) &&
            (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  if (v4) {
    gather_rows_kernel<4><<<grid_for(n_index * F / 4, 256), 256, 0, s>>>(src, n_rows, F, index,
                                                                         n_index, out, err_flag);
  } else {
    gather_rows_kernel<1><<<grid_for(n_index * F, 256), 256, 0, s>>>(src, n_rows, F, index,
                                                                     n_index, out, err_flag);
  }
  return launch_status();
}

static int64_t split_parts(int64_t n_items, int64_t n_seg, int reduce) {
  if (reduce == GMP_REDUCE_MAX || n_seg <= 0) return 1;
  const int64_t avg = n_items / n_seg;
  int64_t S = avg < 2048 ? 1 : ceil_div(avg, 1024);
  // Few segments over many items (an embedding-table gradient: 50k nodes of one atom type
  // into a 100-row table; pools): one wave per segment would leave the chip idle and run the
  // longest segment serially, so spread the segments over up to 2048 workgroups (at most 64
  // parts each: segment_split_finish sums the parts serially per output element).
  if (n_seg < 2048 && n_items >= 16384)
    S = std::max<int64_t>(S, std::min<int64_t>(ceil_div(2048, n_seg), 64));
  return S > 4096 ? 4096 : S;
}

size_t gmp_segment_reduce_workspace_size(int64_t n_items, int64_t n_seg, int64_t F, int reduce) {
  const int64_t S = split_parts(n_items, n_seg, reduce);
  return S > 1 ? (size_t)(n_seg * S * F) * sizeof(float) : 0;
}

int gmp_segment_reduce_f32(const float* src, int64_t n_items, int64_t F, const int64_t* perm,
                           const int64_t* rowptr, int64_t n_seg, int reduce, float* out,
                           int64_t* argmax, void* workspace, size_t workspace_bytes,
                           void* stream) {
  GMP_CHECK_ARG(n_items >= 0 && F >= 0 && n_seg >= 0);
  GMP_CHECK_ARG(reduce == GMP_REDUCE_SUM || reduce == GMP_REDUCE_MEAN || reduce == GMP_REDUCE_MAX);
  if (n_seg == 0 || F == 0) return GMP_OK;
  GMP_CHECK_ARG(rowptr && out && (n_items == 0 || src));
  hipStream_t s = as_stream(stream);
  const bool a16 = (reinterpret_cast<uintptr_t>(src) % 16 == 0);
  const bool a8 = (reinterpret_cast<uintptr_t>(src) % 8 == 0);
  const int vec = (F % 4 == 0 && a16) ? 4 : (F % 2 == 0 && a8) ? 2 : 1;
  const int64_t S = split_parts(n_items, n_seg, reduce);
  if (S > 1 && workspace && workspace_bytes >= gmp_segment_reduce_workspace_size(n_items, n_seg, F, reduce)) {
    float* part = reinterpret_cast<float*>(workspace);
    const unsigned g = (unsigned)(n_seg * S);
#define LAUNCH_SPLIT(V, RED) segment_reduce_split<V, RED><<<g, 256, 0, s>>>(src, n_items, F, perm, rowptr, n_seg, S, part)
    if (reduce == GMP_REDUCE_SUM) {
      if (vec == 4) LAUNCH_SPLIT(4, GMP_REDUCE_SUM); else if (vec == 2) LAUNCH_SPLIT(2, GMP_REDUCE_SUM); else LAUNCH_SPLIT(1, GMP_REDUCE_SUM);
    } else {
      if (vec == 4) LAUNCH_SPLIT(4, GMP_REDUCE_MEAN); else if (vec == 2) LAUNCH_SPLIT(2, GMP_REDUCE_MEAN); else LAUNCH_SPLIT(1, GMP_REDUCE_MEAN);
    }
#undef LAUNCH_SPLIT
    int rc = launch_status();
    if (rc) return rc;
    if (reduce == GMP_REDUCE_SUM)
      segment_split_finish<GMP_REDUCE_SUM><<<grid_for(n_seg * F, 256), 256, 0, s>>>(part, rowptr, n_seg, S, F, out);
    else
      segment_split_finish<GMP_REDUCE_MEAN><<<grid_for(n_seg * F, 256), 256, 0, s>>>(part, rowptr, n_seg, S, F, out);
    return launch_status();
  }
#define LAUNCH_SEG_LAUNCH(VEC, RED)                                                            \
  segment_reduce_wave<VEC, RED><<<(unsigned)ceil_div(n_seg, 4), 256, 0, s>>>(              \
      src, n_items, F, perm, rowptr, n_seg, out, argmax)
#define LAUNCH_SEG_DISPATCH(RED)                                                               \
  do {                                                                                      \
    if (F < 4 && n_items < 64 * n_seg)                                                      \
      segment_reduce_thread<RED><<<grid_for(n_seg * F, 256), 256, 0, s>>>(                 \
          src, n_items, F, perm, rowptr, n_seg, out, argmax);                               \
    else if (vec == 4) LAUNCH_SEG_LAUNCH(4, RED);                                              \
    else if (vec == 2) LAUNCH_SEG_LAUNCH(2, RED);                                              \
    else LAUNCH_SEG_LAUNCH(1, RED);                                                            \
  } while (0)
  if (reduce == GMP_REDUCE_SUM) LAUNCH_SEG_DISPATCH(GMP_REDUCE_SUM);
  else if (reduce == GMP_REDUCE_MEAN) LAUNCH_SEG_DISPATCH(GMP_REDUCE_MEAN);
  else LAUNCH_SEG_DISPATCH(GMP_REDUCE_MAX);
#undef LAUNCH_SEG_DISPATCH
#undef LAUNCH_SEG_LAUNCH
  return launch_status();
}

int gmp_segment_reduce_bwd_f32(const float* grad_out, int64_t n_seg, int64_t F,
                               const int64_t* index, int64_t n_items, const int64_t* rowptr,
                               int reduce, const int64_t* argmax, float* grad_src, void* stream) {
  GMP_CHECK_ARG(n_items >= 0 && F >= 0 && n_seg >= 0);
  GMP_CHECK_ARG(reduce == GMP_REDUCE_SUM || reduce == GMP_REDUCE_MEAN || reduce == GMP_REDUCE_MAX);
  if (n_items == 0 || F == 0) return GMP_OK;
  GMP_CHECK_ARG(grad_out && index && grad_src);
  GMP_CHECK_ARG(reduce != GMP_REDUCE_MEAN || rowptr);
  GMP_CHECK_ARG(reduce != GMP_REDUCE_MAX || argmax);
  hipStream_t s = as_stream(stream);
  const bool vec4 = reduce != GMP_REDUCE_MAX && F % 4 == 0 && n_items * F / 4 < INT32_MAX &&
                    n_seg < INT32_MAX && reinterpret_cast<uintptr_t>(grad_out) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(grad_src) % 16 == 0;
  if (vec4) {
    const int total = (int)(n_items * F / 4);
    const int gv = grid_for(total, 256);
    auto go = reinterpret_cast<const float4*>(grad_out);
    auto gs = reinterpret_cast<float4*>(grad_src);
    if (reduce == GMP_REDUCE_SUM)
      segment_reduce_bwd_vec4_kernel<GMP_REDUCE_SUM><<<gv, 256, 0, s>>>(go, (int)n_seg, (int)(F / 4),
                                                                        index, total, rowptr, gs);
    else
      segment_reduce_bwd_vec4_kernel<GMP_REDUCE_MEAN><<<gv, 256, 0, s>>>(go, (int)n_seg, (int)(F / 4),
                                                                         index, total, rowptr, gs);
    return launch_status();
  }
  int g = grid_for(n_items * F, 256);
  if (reduce == GMP_REDUCE_SUM)
    segment_reduce_bwd_kernel<GMP_REDUCE_SUM><<<g, 256, 0, s>>>(grad_out, n_seg, F, index, n_items,
                                                                rowptr, argmax, grad_src);
  else if (reduce == GMP_REDUCE_MEAN)
    segment_reduce_bwd_kernel<GMP_REDUCE_MEAN><<<g, 256, 0, s>>>(grad_out, n_seg, F, index,
                                                                 n_items, rowptr, argmax, grad_src);
  else
    segment_reduce_bwd_kernel<GMP_REDUCE_MAX><<<g, 256, 0, s>>>(grad_out, n_seg, F, index, n_items,
                                                                rowptr, argmax, grad_src);
  return launch_status();
}

}  // extern "C"
