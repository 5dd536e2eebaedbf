// K9: radius graph on the device (the step before the path).  The reference
// takes a precomputed edge_index; the builder it constructs (PyG SchNet's RadiusInteractionGraph,
// models/schnet.py:47 -> torch_cluster.radius_graph(pos, r, batch, loop=False,
// max_num_neighbors)) is restated here with the selection rule of torch_cluster's GPU kernel:
// for target i, candidates are the nodes j of the same graph with dist2 < r*r taken in
// ascending j (i itself included), the first max_num_neighbors + 1 are kept, then the self
// pair is dropped.  max_num_neighbors <= 0 keeps every candidate.
//   dist2 = ((dx*dx + dy*dy) + dz*dz), dx = p_i - p_j   (fp32, round-to-nearest, no contraction)
// Cell-list binning (cell edge >= r, cells keyed by (graph, cell)): nodes are bucketed with the
// stable CSR build (gmp_csr_build); one thread per target scans its 27 neighbour cells twice
// (count, then fill with a bounded sorted insert), so edge_index comes out sorted by
// (target, source) — deterministic and bit-exact against the CPU restatement.
#include "gmp_common.h"

namespace gmp {
namespace {

struct Grid {
  float lo[3];
  float inv_cell;
  int n[3];
};

__device__ __forceinline__ int cell_coord(float p, float lo, float inv, int n) {
  int c = (int)floorf(__fmul_rn(__fsub_rn(p, lo), inv));
  return c < 0 ? 0 : (c >= n ? n - 1 : c);
}

__global__ void cell_kernel(const float* __restrict__ pos, const int64_t* __restrict__ batch,
                            int64_t N, Grid G, int64_t* __restrict__ cell) {
  for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < N;
       a += (int64_t)gridDim.x * blockDim.x) {
    const int cx = cell_coord(pos[3 * a + 0], G.lo[0], G.inv_cell, G.n[0]);
    const int cy = cell_coord(pos[3 * a + 1], G.lo[1], G.inv_cell, G.n[1]);
    const int cz = cell_coord(pos[3 * a + 2], G.lo[2], G.inv_cell, G.n[2]);
    const int64_t b = batch ? batch[a] : 0;
    cell[a] = ((b * G.n[2] + cz) * G.n[1] + cy) * G.n[0] + cx;
  }
}

__device__ __forceinline__ float dist2(const float* __restrict__ pos, int64_t i, int64_t j) {
  const float dx = __fsub_rn(pos[3 * i + 0], pos[3 * j + 0]);
  const float dy = __fsub_rn(pos[3 * i + 1], pos[3 * j + 1]);
  const float dz = __fsub_rn(pos[3 * i + 2], pos[3 * j + 2]);
  return __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
}

// MODE 0: counts[i] = number of sources kept for target i; MODE 1: write them at offs[i],
// ascending (bounded insert: the counts[i] smallest non-self candidates).
// bounded sorted insert of j into arr[0, filled) with capacity cap (keeps the cap smallest)
template <typename T>
__device__ __forceinline__ void bounded_insert(T* arr, int64_t& filled, int64_t cap, int64_t j) {
  if (filled == cap && !(j < (int64_t)arr[cap - 1])) return;
  int64_t b = (filled < cap ? filled++ : cap - 1) - 1;
  while (b >= 0 && (int64_t)arr[b] > j) {
    arr[b + 1] = arr[b];
    --b;
  }
  arr[b + 1] = (T)j;
}

constexpr int kRT = 256;   // threads per block
constexpr int kLB = 48;    // per-thread LDS sort buffer (sources of one target)
constexpr int kLS = kLB + 1;  // odd stride: lanes on distinct banks

template <int MODE>
__global__ __launch_bounds__(kRT) void radius_kernel(const float* __restrict__ pos, const int64_t* __restrict__ batch,
                              int64_t N, float r2, int64_t max_nb, Grid G,
                              const int64_t* __restrict__ cell, const int64_t* __restrict__ crow,
                              const int64_t* __restrict__ cperm, int64_t* __restrict__ counts,
                              const int64_t* __restrict__ offs, int64_t* __restrict__ src) {
  __shared__ int s_buf[MODE ? kRT * kLS : 1];
  const int64_t per_graph = (int64_t)G.n[0] * G.n[1] * G.n[2];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = cell[i];
    const int64_t gbase = (c / per_graph) * per_graph;
    const int64_t lc = c - gbase;
    const int cx = (int)(lc % G.n[0]), cy = (int)((lc / G.n[0]) % G.n[1]),
              cz = (int)(lc / ((int64_t)G.n[0] * G.n[1]));
    const int64_t b_i = batch ? batch[i] : 0;
    int64_t n_all = 0, n_lt = 0;  // MODE 0: candidates incl. self / those with j < i
    int64_t filled = 0;           // MODE 1
    const int64_t base = MODE ? offs[i] : 0;
    const int64_t cap = MODE ? offs[i + 1] - base : 0;
    int* lbuf = s_buf + (MODE ? threadIdx.x * kLS : 0);
    const bool in_lds = cap <= kLB;
    for (int z = cz - 1; z <= cz + 1; ++z) {
      if (z < 0 || z >= G.n[2]) continue;
      for (int y = cy - 1; y <= cy + 1; ++y) {
        if (y < 0 || y >= G.n[1]) continue;
        for (int x = cx - 1; x <= cx + 1; ++x) {
          if (x < 0 || x >= G.n[0]) continue;
          const int64_t cc = gbase + ((int64_t)z * G.n[1] + y) * G.n[0] + x;
          for (int64_t k = crow[cc]; k < crow[cc + 1]; ++k) {
            const int64_t j = cperm[k];
            if (batch && batch[j] != b_i) continue;  // cells are per graph; guards bad keys
            if (!(dist2(pos, i, j) < r2)) continue;
            if (!MODE) {
              ++n_all;
              n_lt += (j < i);
              continue;
            }
            if (j == i || cap == 0) continue;
            if (in_lds) bounded_insert(lbuf, filled, cap, j);
            else bounded_insert(src + base, filled, cap, j);
          }
        }
      }
    }
    if (MODE && in_lds) {
      for (int64_t a = 0; a < cap; ++a) src[base + a] = lbuf[a];
    }
    if (!MODE) {
      // torch_cluster keeps the first max_nb + 1 candidates (self included), then drops self
      const int64_t kept = max_nb > 0 && n_all > max_nb + 1 ? max_nb + 1 : n_all;
      const bool self_kept = max_nb <= 0 || n_lt < max_nb + 1;
      counts[i] = kept - (self_kept ? 1 : 0);
    }
  }
}

int grid1d(int64_t n) {
  int64_t g = ceil_div(n, 256);
  const int64_t cap = (int64_t)device_cu_count() * 16;
  return (int)(g > cap ? cap : (g < 1 ? 1 : g));
}

}  // namespace
}  // namespace gmp

using namespace gmp;

extern "C" {

int gmp_radius_cells_f32(const float* pos, const int64_t* batch, int64_t n_nodes,
                         const float* lo3, float inv_cell, const int* dims3, int64_t* cell_out,
                         void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && lo3 && dims3 && inv_cell > 0.f);
  if (n_nodes == 0) return GMP_OK;
  GMP_CHECK_ARG(pos && cell_out && dims3[0] > 0 && dims3[1] > 0 && dims3[2] > 0);
  Grid G{{lo3[0], lo3[1], lo3[2]}, inv_cell, {dims3[0], dims3[1], dims3[2]}};
  cell_kernel<<<grid1d(n_nodes), 256, 0, as_stream(stream)>>>(pos, batch, n_nodes, G, cell_out);
  return launch_status();
}

static int radius_launch(int mode, const float* pos, const int64_t* batch, int64_t n_nodes,
                         float r, int64_t max_nb, const float* lo3, float inv_cell,
                         const int* dims3, const int64_t* cell, const int64_t* cell_rowptr,
                         const int64_t* cell_perm, int64_t* counts, const int64_t* offsets,
                         int64_t* src_out, void* stream) {
  GMP_CHECK_ARG(n_nodes >= 0 && lo3 && dims3 && r > 0.f);
  if (n_nodes == 0) return GMP_OK;
  GMP_CHECK_ARG(n_nodes <= INT32_MAX);  // LDS sort buffer holds 32-bit node ids
  GMP_CHECK_ARG(pos && cell && cell_rowptr && cell_perm);
  GMP_CHECK_ARG(dims3[0] > 0 && dims3[1] > 0 && dims3[2] > 0);
  GMP_CHECK_ARG(inv_cell > 0.f && inv_cell <= 1.f / r);  // cell edge >= r: 27 cells suffice
  Grid G{{lo3[0], lo3[1], lo3[2]}, inv_cell, {dims3[0], dims3[1], dims3[2]}};
  const float r2 = r * r;
  if (mode == 0) {
    GMP_CHECK_ARG(counts);
    radius_kernel<0><<<grid1d(n_nodes), kRT, 0, as_stream(stream)>>>(
        pos, batch, n_nodes, r2, max_nb, G, cell, cell_rowptr, cell_perm, counts, nullptr,
        nullptr);
  } else {
    GMP_CHECK_ARG(offsets && src_out);
    radius_kernel<1><<<grid1d(n_nodes), kRT, 0, as_stream(stream)>>>(
        pos, batch, n_nodes, r2, max_nb, G, cell, cell_rowptr, cell_perm, nullptr, offsets,
        src_out);
  }
  return launch_status();
}

int gmp_radius_count_f32(const float* pos, const int64_t* batch, int64_t n_nodes, float r,
                         int64_t max_num_neighbors, const float* lo3, float inv_cell,
                         const int* dims3, const int64_t* cell, const int64_t* cell_rowptr,
                         const int64_t* cell_perm, int64_t* counts, void* stream) {
  return radius_launch(0, pos, batch, n_nodes, r, max_num_neighbors, lo3, inv_cell, dims3, cell,
                       cell_rowptr, cell_perm, counts, nullptr, nullptr, stream);
}

int gmp_radius_fill_f32(const float* pos, const int64_t* batch, int64_t n_nodes, float r,
                        int64_t max_num_neighbors, const float* lo3, float inv_cell,
                        const int* dims3, const int64_t* cell, const int64_t* cell_rowptr,
                        const int64_t* cell_perm, const int64_t* offsets, int64_t* src_out,
                        void* stream) {
  return radius_launch(1, pos, batch, n_nodes, r, max_num_neighbors, lo3, inv_cell, dims3, cell,
                       cell_rowptr, cell_perm, nullptr, offsets, src_out, stream);
}

}  // extern "C"
