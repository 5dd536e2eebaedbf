// Shared helpers for the gfx950 kernels of libgmp (HIP, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gmp.h"

namespace gmp {

// last HIP error seen by any entry point (diagnostics only)
extern thread_local int g_last_hip_error;

inline int hip_check(hipError_t e) {
  if (e != hipSuccess) {
    g_last_hip_error = static_cast<int>(e);
    return GMP_ERR_HIP;
  }
  return GMP_OK;
}

inline int launch_status() { return hip_check(hipGetLastError()); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Number of CUs on the device the stream belongs to (cached per process; MI355X: 256).
int device_cu_count();

// A zeroed completion-ticket word for last-workgroup reductions on stream s (NULL if none can
// be provided, e.g. during a graph capture before first use).
unsigned* stream_ticket(hipStream_t s);

// A block of kTicketWords zeroed ticket words for two-level last-workgroup reductions on stream s
// (tree_finish below), NULL as stream_ticket.  Every user leaves the words it takes zeroed.
constexpr int kTicketWords = 128;
unsigned* stream_ticket_block(hipStream_t s);

// Deterministic two-level finish of a reduction whose G workgroups each published a partial row
// of `width` floats (part[g * width + x]): the last workgroup of each group of kTreeGroup (ticket
// tickets[1 + group]) adds its group's rows in workgroup order into grow[group]; the last group
// finisher (ticket tickets[0]) adds the group rows in group order into out.  Call after the
// workgroup's partial row is written, from every thread of the block (block-uniform).  Tickets are
// left zeroed.  G <= kTreeGroup * (kTicketWords - 1).
constexpr int kTreeGroup = 32;
__device__ inline void tree_finish(const float* part, float* grow, int G, int width, float* out,
                                   unsigned* tickets) {
  __shared__ unsigned s_last;
  const int grp = blockIdx.x / kTreeGroup, g0 = grp * kTreeGroup;
  const int gn = (G - g0) < kTreeGroup ? (G - g0) : kTreeGroup;
  const int ngrp = (G + kTreeGroup - 1) / kTreeGroup;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(&tickets[1 + grp], 1u);
    s_last = (t == (unsigned)gn - 1) ? 1u : 0u;
    if (s_last) atomicExch(&tickets[1 + grp], 0u);
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  for (int x = threadIdx.x; x < width; x += blockDim.x) {
    float acc = 0.f;
    for (int g = 0; g < gn; ++g) acc += part[(int64_t)(g0 + g) * width + x];
    if (ngrp == 1) out[x] = acc;
    else grow[(int64_t)grp * width + x] = acc;
  }
  if (ngrp == 1) return;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(&tickets[0], 1u);
    s_last = (t == (unsigned)ngrp - 1) ? 1u : 0u;
    if (s_last) atomicExch(&tickets[0], 0u);
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  for (int x = threadIdx.x; x < width; x += blockDim.x) {
    float acc = 0.f;
    for (int g = 0; g < ngrp; ++g) acc += grow[(int64_t)g * width + x];
    out[x] = acc;
  }
}

}  // namespace gmp

#define GMP_CHECK_ARG(cond) \
  do {                      \
    if (!(cond)) return GMP_ERR_ARG; \
  } while (0)
