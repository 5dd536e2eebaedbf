// K10: device side of graph batching (PyG Batch.from_data_list semantics as
// the reference's loaders produce it, experiments/utils/train_utils.py:28,132).  The host packs
// the per-graph arrays back to back into pinned staging buffers and copies them once; this kernel
// turns graph-local edge indices into batch-global ones and writes the `batch` vector:
//   edge e of graph g (edge_ptr[g] <= e < edge_ptr[g+1]):  out[:, e] = local[:, e] + node_ptr[g]
//   node a of graph g (node_ptr[g] <= a < node_ptr[g+1]):  batch[a] = g
// Graphs are found by binary search over the (B+1)-entry prefix arrays (empty graphs allowed).
// A local index outside [0, n_g) sets *err (same contract as the CSR build's range flag).
#include "gmp_common.h"

namespace gmp {
namespace {

// largest g in [0, B) with ptr[g] <= x (ptr non-decreasing, ptr[0] = 0, x < ptr[B])
__device__ __forceinline__ int64_t owner(const int64_t* __restrict__ ptr, int64_t B, int64_t x) {
  int64_t lo = 0, hi = B;  // invariant: ptr[lo] <= x < ptr[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (ptr[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ void collate_kernel(const int64_t* __restrict__ local, int64_t E,
                               const int64_t* __restrict__ node_ptr,
                               const int64_t* __restrict__ edge_ptr, int64_t B, int64_t N,
                               int64_t* __restrict__ out, int64_t* __restrict__ batch,
                               int* __restrict__ err) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < E + N; t += stride) {
    if (t < E) {
      const int64_t g = owner(edge_ptr, B, t);
      const int64_t off = node_ptr[g], n_g = node_ptr[g + 1] - off;
      const int64_t s = local[t], d = local[E + t];
      if (err && (s < 0 || s >= n_g || d < 0 || d >= n_g)) atomicOr(err, 1);
      out[t] = s + off;
      out[E + t] = d + off;
    } else {
      const int64_t a = t - E;
      batch[a] = owner(node_ptr, B, a);
    }
  }
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_batch_collate(const int64_t* edge_index_local, int64_t n_edges, const int64_t* node_ptr,
                      const int64_t* edge_ptr, int64_t n_graphs, int64_t n_nodes,
                      int64_t* edge_index_out, int64_t* batch_out, int* err, void* stream) {
  GMP_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_graphs >= 0);
  const int64_t work = n_edges + n_nodes;
  if (work == 0) return GMP_OK;
  GMP_CHECK_ARG(n_graphs > 0 && node_ptr && edge_ptr);
  GMP_CHECK_ARG(n_edges == 0 || (edge_index_local && edge_index_out));
  GMP_CHECK_ARG(n_nodes == 0 || batch_out);
  int64_t grid = ceil_div(work, 256);
  const int64_t cap = (int64_t)device_cu_count() * 16;
  if (grid > cap) grid = cap;
  collate_kernel<<<(int)grid, 256, 0, as_stream(stream)>>>(
      edge_index_local, n_edges, node_ptr, edge_ptr, n_graphs, n_nodes, edge_index_out,
      batch_out, err);
  return launch_status();
}

}  // extern "C"
