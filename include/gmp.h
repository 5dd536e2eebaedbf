/*
 * gmp.h — C ABI of the MI355X (gfx950) geometric message-passing hot path.
 *
 * The reference (NW-JEFF/Geometric-Message-Passing) has no native code of its own: its hot path
 * runs through PyG `MessagePassing.propagate`, `torch_scatter.scatter` (C++/CUDA custom ops
 * `torch.ops.torch_scatter.scatter_sum/mean/max`) and e3nn modules.  Each
 * entry point below replaces one of those call sites; the replaced interface is cited per
 * function as reference file:line.
 *
 * Conventions (all functions):
 *   - plain device pointers, int64 sizes, fp32 features, int64 indices (the reference dtypes);
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); no function allocates,
 *     frees or synchronises; all work is enqueued on `stream` (graph-capture safe);
 *   - return GMP_OK (0) or a negative error code (gmp_error_string); argument checks are done
 *     on the host before anything is enqueued; device-side index range errors are reported
 *     through an optional int32 device flag (`err_flag`, set to 1; caller checks when it wants);
 *   - outputs are fully written (zero rows included) unless documented as accumulating.
 */
#ifndef GMP_H_
#define GMP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3 (r04): K8 symmetric contraction takes the per-channel dim and A4 (gmp_sc_monomials added);
 * the TP descriptor holds 8 output blocks (128 bytes), <= 48 paths.
 * 2 (r04): EGNN forward / backward take save_planes; gmp_egnn_set_xhat_mode and
 * gmp_egnn_edge_bwd_ab_f32 removed.  (r03 changed gmp_triplet_fill_f32 under version 1.)
 * 4 (r05): gmp_egnn_node_fwd_f32 / gmp_egnn_node_params added.
 * Version 5 (r05): the opt-in TP kernels K7s / K7f (gmp_tp_node_fwd_fused_f32,
 * gmp_tp_z_fused_layout_*, gmp_tp_node_dw_*), the row GEMM (gmp_split_x3_f32, gmp_gemm_x3_f32),
 * gmp_tp_gemm_set_rings, gmp_wgrad_set_grid_cap and the CU-masked stream entries removed; K8 takes
 * the sparse term plan (any irreps), gmp_sc_monomials removed.
 * Version 6 (r06): gmp_gvp_ff_{fwd,bwd}_f32 (K17, the GVPConvLayer node feed-forward) and
 * gmp_egnn_node_bwd_f32 / gmp_egnn_node_bwd_partial_rows (K15b) added. */
#define GMP_ABI_VERSION 6

enum {
  GMP_OK = 0,
  GMP_ERR_ARG = -1,         /* bad pointer / size / unsupported combination */
  GMP_ERR_HIP = -2,         /* a HIP runtime call failed (see gmp_last_hip_error) */
  GMP_ERR_UNSUPPORTED = -3, /* shape not supported by this fused kernel */
  GMP_ERR_WORKSPACE = -4    /* workspace too small */
};

enum { GMP_REDUCE_SUM = 0, GMP_REDUCE_MEAN = 1, GMP_REDUCE_MAX = 2 };
enum { GMP_ACT_RELU = 0, GMP_ACT_SILU = 1 };

int gmp_abi_version(void);
const char* gmp_error_string(int code);
int gmp_last_hip_error(void);

/* ------------------------------------------------------------------------------------------
 * Index preprocessing: stable CSR of an index array (receiver-sorted edge lists).
 * Replaces the implicit ordering work of torch_scatter's atomics (egnn_layer.py:77,79;
 * tfn_layer.py:87; PyG aggregate): we sort once per graph and reduce deterministically.
 *   perm[k]      = position of the k-th item in stable order of index (k = 0..n_items-1)
 *   rowptr[s]    = first k with index[perm[k]] >= s   (s = 0..n_seg), rowptr[n_seg] = n_items
 *   payload_out  = payload[perm] (optional, may be NULL)
 * Workspace: gmp_csr_workspace_size(n_items, n_seg) bytes.
 * ------------------------------------------------------------------------------------------ */
size_t gmp_csr_workspace_size(int64_t n_items, int64_t n_seg);
int gmp_csr_build(const int64_t* index, int64_t n_items, int64_t n_seg, const int64_t* payload,
                  int64_t* perm, int64_t* rowptr, int64_t* index_sorted, int64_t* payload_out,
                  int32_t* err_flag, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * K2 gather: out[e, :] = src[index[e], :]   (PyG `_collect` index_select of x_i / x_j,
 * torch_geometric MessagePassing.propagate; tfn_layer.py:85 `node_attr[dst]`).
 * Out-of-range index -> row of zeros and *err_flag = 1 (err_flag may be NULL).
 * ------------------------------------------------------------------------------------------ */
int gmp_gather_rows_f32(const float* src, int64_t n_rows, int64_t F, const int64_t* index,
                        int64_t n_index, float* out, int32_t* err_flag, void* stream);

/* ------------------------------------------------------------------------------------------
 * K3 segmented reduce over a CSR (torch_scatter.scatter(src, index, dim=0, dim_size, reduce)
 * with reduce in {sum/add, mean, max}; egnn_layer.py:77,79, tfn_layer.py:87, PyG aggregate,
 * global_add_pool / global_mean_pool).
 *   out[s, f] = reduce_{k in [rowptr[s], rowptr[s+1])} src[perm ? perm[k] : k, f]
 *   empty segments -> 0; mean divides by max(count, 1); max also writes argmax[s, f]
 *   (item index, n_items for empty segments; argmax may be NULL for sum/mean).
 * Summation order is fixed by the CSR (deterministic).  Long segments (average length >= 2048,
 * e.g. global pools) are split over workgroups when a workspace of
 * gmp_segment_reduce_workspace_size(...) bytes is given (NULL / too small = single-wave path).
 * ------------------------------------------------------------------------------------------ */
size_t gmp_segment_reduce_workspace_size(int64_t n_items, int64_t n_seg, int64_t F, int reduce);
int gmp_segment_reduce_f32(const float* src, int64_t n_items, int64_t F, const int64_t* perm,
                           const int64_t* rowptr, int64_t n_seg, int reduce, float* out,
                           int64_t* argmax, void* workspace, size_t workspace_bytes,
                           void* stream);

/* Backward of gmp_segment_reduce_f32 w.r.t. src (torch_scatter autograd):
 *   sum : grad_src[e] = grad_out[index[e]]
 *   mean: grad_src[e] = grad_out[index[e]] / max(count[index[e]], 1)   (count from rowptr)
 *   max : grad_src[e, f] = (argmax[index[e], f] == e) ? grad_out[index[e], f] : 0            */
int gmp_segment_reduce_bwd_f32(const float* grad_out, int64_t n_seg, int64_t F,
                               const int64_t* index, int64_t n_items, const int64_t* rowptr,
                               int reduce, const int64_t* argmax, float* grad_src, void* stream);

/* ------------------------------------------------------------------------------------------
 * K4 EGNN fused edge message + aggregation (egnn_layer.py:62-80 message/aggregate; the node
 * update :82-86 stays a node-level op).  Edges must be receiver-sorted (CSR from
 * gmp_csr_build on edge_index[1]).  The first message Linear(2d+1 -> d) is split as
 *   W1 [h_i | h_j | dist] = (h W1a^T)[i] + (h W1b^T)[j] + w1d * dist
 * so the node projections AB = [h W1a^T | h W1b^T] (N x 2d) are computed once per node by the
 * caller.  Per edge e = (j -> i), in registers:
 *   rel = pos[i]-pos[j]; dist = |rel|; y1 = act(LN1(AB[i,:d] + AB[j,d:] + w1d*dist + b1))
 *   m = act(LN2(W2 y1 + b2)); y3 = act(LN3(W3 m + b3)); s = w4.y3 + b4; shift = rel * s
 * and per receiver i (segmented, deterministic, no atomics):
 *   m_aggr[i] = sum_e m  (or mean if msg_mean), pos_aggr[i] = mean_e shift.
 * d in {32, 64, 128}.  LayerNorm eps = ln_eps.
 * ------------------------------------------------------------------------------------------ */
typedef struct gmp_egnn_params {
  const float* w1d;  /* (d)  column 2d of mlp_msg.0.weight   */
  const float* b1;   /* (d)  mlp_msg.0.bias                   */
  const float* ln1_w;
  const float* ln1_b;
  const float* W2;   /* (d,d) mlp_msg.3.weight, row-major [out][in] */
  const float* b2;
  const float* ln2_w;
  const float* ln2_b;
  const float* W3;   /* (d,d) mlp_pos.0.weight */
  const float* b3;
  const float* ln3_w;
  const float* ln3_b;
  const float* w4;   /* (d)  mlp_pos.3.weight */
  const float* b4;   /* (1)  mlp_pos.3.bias   */
} gmp_egnn_params;

/* save_xhat / save_rstd: both NULL (inference) or, for training, (save_planes, E, d) and (E, 3)
 * buffers that receive the LayerNorm outputs and their 1/std per edge (receiver-sorted rows) for
 * gmp_egnn_edge_bwd_f32: save_planes = 2 (default form) stores x_hat1, x_hat2 — the backward
 * recomputes x_hat3 from x_hat2 and the saved 1/std, bitwise the forward's value; 3 also stores
 * x_hat3.  The backward takes the same save_planes (the caller keeps it with the buffer). */
/* The two d x d products per edge chunk run by default on the f16 MFMA over 2-plane (hi + lo)
 * splits of the operands with power-of-two scaling (22-bit operands, f32 accumulation; relative
 * error ~2^-21 per product); gmp_egnn_set_f32_mfma(1) selects
 * the exact f32-MFMA fmaf chains.  Returns the previous setting. */
int gmp_egnn_set_f32_mfma(int on);
int gmp_egnn_edge_fwd_f32(int64_t n_nodes, int64_t n_edges, int64_t d, const float* AB,
                          const float* pos, const int64_t* rowptr, const int64_t* recv,
                          const int64_t* send, const gmp_egnn_params* params, int act,
                          int msg_mean, float ln_eps, float* m_aggr, float* pos_aggr,
                          float* save_xhat, int save_planes, float* save_rstd, void* stream);

/* K15 (r05): the EGNN node update of one layer and the next layer's node projections in one
 * launch — replaces egnn_layer.py:82-86 (update: mlp_upd(cat([h, m_aggr]))), egnn.py:75-76 (the
 * residual h + h_update) and the AB = [h W1a^T | h W1b^T] projection of the next layer's
 * mlp_msg.0 (egnn_layer.py:28-29; the node half of gmp_egnn_edge_fwd_f32's split Linear):
 *   x1 = act(LN1(W0 [h | m_aggr] + b0)); x2 = act(LN2(W3 x1 + b3));
 *   h_out = (residual ? h + x2 : x2);  ab_out = [h_out W1n[:, :d]^T | h_out W1n[:, d:2d]^T]
 * W0 = mlp_upd.0.weight (d, 2d) row-major; W3 = mlp_upd.3.weight (d, d); W1n = the next layer's
 * mlp_msg.0.weight (d, 2d + 1) with row stride ld1 (>= 2d), or NULL (that layer has no ab_out).
 * The three matrices enter as a weight IMAGE (2-plane fp16 tiles with per-16-row power-of-two
 * scales, the layout the kernel copies into LDS): gmp_egnn_node_image_f32 builds the images of
 * n_layers layers (params: a host array of n_layers structs) into `images`
 * (n_layers x gmp_egnn_node_image_bytes(d) bytes, 16-byte aligned) in one launch; rebuild after
 * every weight change.  gmp_egnn_node_fwd_f32 reads this layer's image and, from params, the
 * vectors b0, ln1_w, ln1_b, b3, ln2_w, ln2_b; ab_out non-NULL only if the image holds W1n.
 * save_xhat ((2, N, d): the two LayerNorm outputs) and save_rstd ((2, N): their 1/std) both NULL
 * (inference) or both set (training; the LayerNorm backwards read them).  Products as
 * gmp_egnn_edge_fwd_f32's HF path (2-plane fp16 splits, f32 accumulation); GMP_ERR_UNSUPPORTED
 * under gmp_egnn_set_f32_mfma(1) and for d outside {32, 64, 128}. */
typedef struct gmp_egnn_node_params {
  const float* W0;   /* (d, 2d) mlp_upd.0.weight */
  const float* b0;   /* (d) */
  const float* ln1_w;
  const float* ln1_b;
  const float* W3;   /* (d, d) mlp_upd.3.weight */
  const float* b3;
  const float* ln2_w;
  const float* ln2_b;
  const float* W1n;  /* next layer's mlp_msg.0.weight (d, 2d + 1), row stride ld1; or NULL */
  int64_t ld1;
} gmp_egnn_node_params;
size_t gmp_egnn_node_image_bytes(int64_t d);
int gmp_egnn_node_image_f32(int64_t d, int64_t n_layers, const gmp_egnn_node_params* params,
                            void* images, void* stream);
int gmp_egnn_node_fwd_f32(int64_t n_nodes, int64_t d, const float* h, const float* m_aggr,
                          const gmp_egnn_node_params* params, const void* image, int act,
                          int residual, float ln_eps, float* h_out, float* ab_out,
                          float* save_xhat, float* save_rstd, void* stream);

/* K15b (r06): backward of gmp_egnn_node_fwd_f32 (egnn_layer.py:82-86 update, egnn.py:75-76
 * residual) in one launch, from grad_h (N, d) of h_out and the forward's save_xhat (2, N, d),
 * save_rstd (2, N):  dz2 = grad_h act'(x_hat2 ln2_w + ln2_b), dpre2 = LN2'(dz2 ln2_w);
 * dz1 = (W3^T dpre2) act'(x_hat1 ln1_w + ln1_b), dpre1 = LN1'(dz1 ln1_w);
 * dh = W0[:, :d]^T dpre1 (+ grad_h when residual), dm = W0[:, d:]^T dpre1 (the m_aggr gradient);
 * dpre1, dpre2 (N, d) out for the weight sums (dW0 = dpre1^T [h | m], dW3 = dpre2^T
 * act(x_hat1 ln1_w + ln1_b)); partials (gmp_egnn_node_bwd_partial_rows(N), 4 d) per-workgroup rows
 * of [d ln1_w | d ln1_b | d ln2_w | d ln2_b], the caller sums them in row order.  W0 (d, 2d),
 * W3 (d, d) f32 row-major (not the forward's image); exact f32 products; d in {32, 64, 128}
 * (GMP_ERR_UNSUPPORTED otherwise), act 0 relu / 1 swish. */
int64_t gmp_egnn_node_bwd_partial_rows(int64_t n_nodes);
int gmp_egnn_node_bwd_f32(int64_t n_nodes, int64_t d, int act, int residual, const float* grad_h,
                          const float* save_xhat, const float* save_rstd, const float* W0,
                          const float* W3, const float* ln1_w, const float* ln1_b,
                          const float* ln2_w, const float* ln2_b, float* dh, float* dm,
                          float* dpre1, float* dpre2, float* partials, void* stream);
/* Backward of gmp_egnn_edge_fwd_f32 from its saved x_hat / rstd (no forward recompute).
 * Inputs g_m_aggr (N,d), g_pos_aggr (N,3), the forward's save_xhat (save_planes, E, d) and
 * save_rstd (E, 3).  Outputs:
 *   dA        (N,d)  receiver part of d(AB)[:, :d]   (segment-summed in-kernel)
 *   dpos_recv (N,3)  receiver part of d(pos)          (segment-summed in-kernel)
 *   per edge, in receiver-sorted order (row e):
 *     dpre1 (E,d)  grad of the first pre-activation   -> caller reduces by sender for
 *                  d(AB)[:, d:], and takes db1 = sum_e dpre1
 *     gdiff (E,3)  grad of rel                         -> caller: dpos[send] -= gdiff
 *     dpre2, dpre3 (E,d)                               -> caller: dW2 = dpre2^T y1,
 *                  dW3 = dpre3^T m, db2 = sum dpre2, db3 = sum dpre3, with y1 / m rebuilt
 *                  from x_hat1 / x_hat2 inside gmp_edge_outer_sum_act_f32
 *   vec_partials (n_blocks, 8*d+1): per-workgroup partial sums of
 *     [dln1_w, dln1_b, dln2_w, dln2_b, dln3_w, dln3_b, dw4, dw1d, db4]   (caller sums rows;
 *     n_blocks from gmp_egnn_edge_bwd_partials_rows). Deterministic. */
int64_t gmp_egnn_edge_bwd_partials_rows(int64_t n_edges, int64_t d);
int gmp_egnn_edge_bwd_f32(int64_t n_nodes, int64_t n_edges, int64_t d, const float* pos,
                          const int64_t* rowptr, const int64_t* recv, const int64_t* send,
                          const gmp_egnn_params* params, int act, int msg_mean,
                          const float* save_xhat, int save_planes, const float* save_rstd,
                          const float* g_m_aggr, const float* g_pos_aggr, float* dA,
                          float* dpos_recv, float* dpre1, float* gdiff, float* dpre2, float* dpre3,
                          float* vec_partials, void* stream);
/* As gmp_egnn_edge_bwd_f32, also folding max |dpre2| and max |dpre3| into amax[0], amax[1]
 * (float bit patterns, atomic max; caller zeroes): the A scales of the HF weight-gradient outer
 * sums (gmp_edge_outer_sum_act_hf_f32). */
int gmp_egnn_edge_bwd_amax_f32(int64_t n_nodes, int64_t n_edges, int64_t d, const float* pos,
                               const int64_t* rowptr, const int64_t* recv, const int64_t* send,
                               const gmp_egnn_params* params, int act, int msg_mean,
                               const float* save_xhat, int save_planes, const float* save_rstd,
                               const float* g_m_aggr, const float* g_pos_aggr, float* dA,
                               float* dpos_recv, float* dpre1, float* gdiff, float* dpre2,
                               float* dpre3, float* vec_partials, uint32_t* amax, void* stream);

/* ------------------------------------------------------------------------------------------
 * Edge-reduction GEMM for per-edge Linear weight gradients (egnn_layer.py:28-39 mlp_msg /
 * mlp_pos backward; replaces torch's dW = dpre^T x over E rows):
 *   C (d x d) = A^T B with A (K, d), B (K, d) row-major fp32, K = edges;
 *   colsum_A (d) = sum_k A[k, :] (the bias gradient; may be NULL).
 * Split-K over workgroups, partial slabs in `workspace` and an ordered second pass: bitwise
 * deterministic.  d in {32, 64, 128}.  Arithmetic (all outer-sum entry points below): f32
 * operands split exactly into three bf16 planes on the bf16 MFMA with f32 accumulation, the
 * six partial products of order <= 2^-16 summed (error vs fp64 <= 2^-26 of sum |a b|, within
 * 2x of the f32-MFMA kernels', below rocBLAS f32 GEMM's); gmp_wgrad_set_f32_mfma(1) selects the f32-MFMA
 * kernels instead, returns the previous setting.
 * ------------------------------------------------------------------------------------------ */
int gmp_wgrad_set_f32_mfma(int on);
size_t gmp_edge_outer_sum_workspace_size(int64_t K, int64_t d);
int gmp_edge_outer_sum_f32(int64_t K, int64_t d, const float* A, const float* B, float* C,
                           float* colsum_A, void* workspace, size_t workspace_bytes,
                           void* stream);
/* Same with the activation rebuilt from a saved LayerNorm output at load time:
 * C = A^T act(X * w + b) (+ colsum_A = colsum(A)), w, b per column (d), act 0 = relu, 1 = silu
 * (the EGNN y1 / m of egnn_layer.py:28-34 from x_hat1 / x_hat2).  Workspace as above. */
int gmp_edge_outer_sum_act_f32(int64_t K, int64_t d, const float* A, const float* X,
                               const float* w, const float* b, int act, float* C,
                               float* colsum_A, void* workspace, size_t workspace_bytes,
                               void* stream);
/* HF form of gmp_edge_outer_sum_act_f32 for LayerNorm rows X (|X| <= sqrt(d), the EGNN x_hat):
 * two scaled fp16 planes per operand, three MFMA products per stage (22-bit operands, f32
 * accumulation; ~2^-21 relative per product).  amax_A: device word holding max |A| as a float
 * bit pattern (gmp_egnn_edge_bwd_amax_f32 produces it for dpre2 / dpre3); B's scale comes from
 * sqrt(d) max|w| + max|b|.  Falls back to the split-plane x3 / f32-MFMA paths where those apply
 * (node-level K, gmp_wgrad_set_f32_mfma(1)). */
int gmp_edge_outer_sum_act_hf_f32(int64_t K, int64_t d, const float* A, const float* X,
                                  const float* w, const float* b, int act, const uint32_t* amax_A,
                                  float* C, float* colsum_A, void* workspace,
                                  size_t workspace_bytes, void* stream);

/* Rectangular variant (GVP message GVPs, gvp_layer.py:101-170 applied per edge at :319-324):
 * C (m x n) = A^T B, A (K, m), B (K, n) row-major, m, n multiples of 16, m <= 256,
 * (m/16)(n/16) <= 72; colsum_A (m) optional.  Same deterministic split-K reduction. */
size_t gmp_edge_outer_sum_rect_workspace_size(int64_t K, int64_t m, int64_t n);
/* gmp_edge_xyz_dot_f32 (r05): out[c] = sum_e sum_x A[e, 3c + x] v[e, x] for A (K, 3C) contiguous
 * 16-byte aligned, v (K, 3), C in {16, 48} (GMP_ERR_UNSUPPORTED otherwise): the xyz
 * contractions of the GVP first message's weight sums (sum dvpre . ev, sum dvh . ev,
 * gvp_layer.py:101-170 through the e_v column of W_h) in one pass over A; per-workgroup partial
 * rows in the workspace, added in a fixed order (deterministic). */
size_t gmp_edge_xyz_dot_workspace_size(int64_t K);
int gmp_edge_xyz_dot_f32(int64_t K, int64_t C, const float* A, const float* v, float* out,
                         void* workspace, size_t workspace_bytes, void* stream);
int gmp_edge_outer_sum_rect_f32(int64_t K, int64_t m, int64_t n, const float* A, const float* B,
                                float* C, float* colsum_A, void* workspace,
                                size_t workspace_bytes, void* stream);
/* General form (strided operands and output): C (m x n, row stride ldc) = A^T act(B),
 * A (K, m) with row stride lda, B (K, n) with row stride ldb (lda, ldb multiples of 4, A and B
 * 16-byte aligned), colsum_A (m) optional; act -1 = none, 0 = relu(B*w + b), 1 = silu(B*w + b)
 * (the activation prologue needs m == n in {32, 64, 128}).  Lets a Linear's weight gradient
 * be written straight into a column block of a wider parameter (egnn_layer.py:28 W1 =
 * [W1a | W1b | w1d]; :37 mlp_upd[0] over [h | m_aggr]) without concatenated copies.
 * Square 32/64/128 shapes use the square kernel, others the rectangular one. */
/* Two B operands as one: C (m x (n1 + n2)) = A^T [B1 | B2] for outer sums that share A (GVP:
 * dspre against [s | vn]), one pass over A; workspace gmp_edge_outer_sum_rect_workspace_size(K,
 * m, n1 + n2).  Split-plane path only: returns GMP_ERR_UNSUPPORTED where it does not apply
 * (narrow products, node-level K, f32-MFMA mode) — the caller then makes two calls. */
int gmp_edge_outer_sum_ex2_f32(int64_t K, int64_t m, int64_t n1, int64_t n2, const float* A,
                               int64_t lda, const float* B1, int64_t ldb1, const float* B2,
                               int64_t ldb2, float* C, int64_t ldc, float* colsum_A,
                               void* workspace, size_t workspace_bytes, void* stream);
size_t gmp_edge_outer_sum_ex_workspace_size(int64_t K, int64_t m, int64_t n);
int gmp_edge_outer_sum_ex_f32(int64_t K, int64_t m, int64_t n, const float* A, int64_t lda,
                              const float* B, int64_t ldb, int act, const float* w, const float* b,
                              float* C, int64_t ldc, float* colsum_A, void* workspace,
                              size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * K1 per-edge featurisation (models/mace.py:170-174, models/tfn.py:171-175,
 * models/mace_modules/radial.py:44-46,71-78, blocks.py:91-96; e3nn SphericalHarmonics(l<=2,
 * normalize=True, 'component')):
 *   vec = pos[ei0] - pos[ei1] (E,3); len = |vec| (E); sh (E,9); radial = bessel * cutoff (E,nb)
 * edge_index is (2, E) int64 (row 0 then row 1).  `bessel_weights` is a HOST array of nb floats
 * (the module buffer, copied into the kernel arguments).  Any output pointer may be NULL.
 * Backward: g_vec (E,3) from g_sh / g_radial (either may be NULL); the caller scatters g_vec to
 * pos[ei0] (+) and pos[ei1] (-).
 * ------------------------------------------------------------------------------------------ */
int gmp_edge_featurize_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                           int num_bessel, const float* bessel_weights, float prefactor,
                           float r_max, float p_cutoff, float* vec_out, float* len_out,
                           float* sh_out, float* radial_out, void* stream);
int gmp_edge_featurize_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                               int num_bessel, const float* bessel_weights, float prefactor,
                               float r_max, float p_cutoff, const float* g_sh,
                               const float* g_radial, float* g_vec, void* stream);
/* The same for SphericalHarmonics(lmax) with 0 <= lmax <= 3 (max_ell of models/tfn.py:51 /
 * mace.py:25): sh rows of (lmax + 1)^2 floats, the l = 3 block being e3nn's component-
 * normalised sh_3_m (the lmax = 2 entries above are these with lmax = 2). */
int gmp_edge_featurize_lmax_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                int lmax, int num_bessel, const float* bessel_weights,
                                float prefactor, float r_max, float p_cutoff, float* vec_out,
                                float* len_out, float* sh_out, float* radial_out, void* stream);
int gmp_edge_featurize_lmax_bwd_f32(const float* pos, const int64_t* edge_index,
                                    int64_t n_edges, int lmax, int num_bessel,
                                    const float* bessel_weights, float prefactor, float r_max,
                                    float p_cutoff, const float* g_sh, const float* g_radial,
                                    float* g_vec, void* stream);
/* GVP-GNN edge features (models/gvpgnn.py:106-112): len (E), radial (E,nb) as above and the unit
 * vectors nan_to_num(vec / len) (E,3; zero rows for zero-length edges).  Backward from g_radial /
 * g_unit (either may be NULL) to g_vec. */
int gmp_edge_featurize_gvp_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                               int num_bessel, const float* bessel_weights, float prefactor,
                               float r_max, float p_cutoff, float* len_out, float* radial_out,
                               float* unit_out, void* stream);
int gmp_edge_featurize_gvp_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                   int num_bessel, const float* bessel_weights, float prefactor,
                                   float r_max, float p_cutoff, const float* g_radial,
                                   const float* g_unit, float* g_vec, void* stream);
/* SchNet edge features (models/schnet.py:66-68; PyG 2.3.1 SchNet.forward, GaussianSmearing,
 * CFConv.forward): dist = |pos[row] - pos[col]| (E), rbf[e, k] = exp(coeff (dist - offsets[k])^2)
 * (E,G), cut = 0.5 (cos(dist pi / cutoff) + 1) (E).  `offsets` is the module's DEVICE buffer
 * (G <= 256).  Any output may be NULL.  Backward: g_vec (E,3) from g_dist / g_rbf / g_cut (any
 * may be NULL); the caller scatters g_vec to pos[row] (+) and pos[col] (-). */
int gmp_schnet_featurize_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                             int num_gaussians, const float* offsets, float coeff, float cutoff,
                             float* dist_out, float* rbf_out, float* cut_out, void* stream);
int gmp_schnet_featurize_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                 int num_gaussians, const float* offsets, float coeff,
                                 float cutoff, const float* g_dist, const float* g_rbf,
                                 const float* g_cut, float* g_vec, void* stream);

/* ------------------------------------------------------------------------------------------
 * K16 irreps epilogues of the TP convolution (models/layers/tfn_layer.py:89-92), row-major
 * (B, C) fp32 node features, all tables int32 on the DEVICE (built once per module):
 * Gate (e3nn nn.Gate, tfn_layer.py:45-63): y = [c_act silu(scalars), gated * c_gate
 *   sigmoid(gates)]; out_map (c_out, 2) = {source col, gate col or -1}; in_map (c_in, 4) =
 *   {kind 0 scalar / 1 gate / 2 gated, a, b, d} (gmp_irreps.hip header).
 * BatchNorm (e3nn nn.BatchNorm, component normalisation, affine): col_chan (C) channel of each
 *   column, chan_col (nf) first column of each channel, chan_info (nf, 2) = {2l+1, scalar index
 *   or -1}.  Training: batch statistics (fixed-order partial sums) and running-stat update in
 *   place (momentum); eval: running statistics.  save_shift / save_invstd (nf) feed the
 *   backward, which writes grad_x and grad_weight (nf) / grad_bias (number of scalar channels).
 * ------------------------------------------------------------------------------------------ */
int gmp_gate_fwd_f32(int64_t B, int c_in, int c_out, const int32_t* out_map, float c_act,
                     float c_gate, const float* x, float* y, void* stream);
int gmp_gate_bwd_f32(int64_t B, int c_in, int c_out, const int32_t* in_map, float c_act,
                     float c_gate, const float* x, const float* grad_y, float* grad_x,
                     void* stream);
size_t gmp_irreps_bn_workspace_size(int64_t B, int C, int nf);
int gmp_irreps_bn_fwd_f32(int64_t B, int C, int nf, const int32_t* col_chan,
                          const int32_t* chan_col, const int32_t* chan_info, const float* x,
                          const float* weight, const float* bias, float* running_mean,
                          float* running_var, int training, float momentum, float eps, float* y,
                          float* save_shift, float* save_invstd, void* workspace,
                          size_t workspace_bytes, void* stream);
int gmp_irreps_bn_bwd_f32(int64_t B, int C, int nf, const int32_t* col_chan,
                          const int32_t* chan_col, const int32_t* chan_info, const float* x,
                          const float* grad_y, const float* weight, const float* save_shift,
                          const float* save_invstd, int training, float* grad_x,
                          float* grad_weight, float* grad_bias, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * K7 tensor-product convolution messages (models/layers/tfn_layer.py:82-86): e3nn
 * FullyConnectedTensorProduct(in1, 1x0e+1x1o+1x2e, out, shared_weights=False) applied per edge
 * with per-edge weights W (chunk rows x weight_numel, produced by the radial MLP
 * tfn_layer.py:73-77).  The receiver sum of tfn_layer.py:87 (scatter(tp, ei[0], 'sum')) is the
 * segmented reduce above over the same receiver-sorted order.
 * Edges are addressed by their position k in the stable CSR of edge_index[0]:
 *   src_sorted[k] = ei1 of sorted edge k, perm[k] = original edge id, recv_sorted[k] = ei0.
 * x (N, in_dim) mul_ir; sh (E, 9) in ORIGINAL edge order; W row r = sorted edge c0 + r.
 * Forward writes msg rows c0..c1-1 (E x out_dim, sorted positions).
 * desc_host: host pointer to the descriptor {int n_paths, in_dim, out_dim, sh_dim;
 *   int64 weight_numel; int z_size, n_blocks; int blk_off[8], blk_mul[8], blk_l[8];}
 *   (128 bytes since ABI 3; <= 48 paths, <= 8 output blocks).  The per-edge-weight kernels below take l <= 2 (sh_dim 9, the
 *   two layouts); the node-form z / dz kernels (gmp_tp_edge_z*) take l <= 3 (sh_dim (lmax+1)^2
 *   <= 16, any block structure: max_ell = 3 models).
 * paths_dev: device array of 64-byte path records {int l1, l2, lo, mul1, mul_out, x_off, y_off,
 *   io, out_off, z_off, cg_off, pad; int64 w_off; float alpha, pad}; cg_dev: concatenated
 *   real CG tensors (cg_len floats).  layout: 0 = out blocks (0e,1o,2e), 1 = (0e,0e,1o,2e).
 *   Multiplicities <= 128 and multiples of 4.
 * Backward (per chunk): dW (chunk rows x weight_numel), dx_edge (E, in_dim) and dY_edge (E, 9)
 * at SORTED positions, given gout = dL/dout (N, out_dim) of the receiver sums.
 * ------------------------------------------------------------------------------------------ */
int gmp_tp_conv_fwd_f32(int layout, const void* desc_host, const void* paths_dev,
                        const float* cg_dev, int cg_len, const float* x, const float* sh,
                        const float* W, const int64_t* src_sorted, const int64_t* perm,
                        int64_t c0, int64_t c1, float* msg, void* stream);
int gmp_tp_conv_bwd_f32(int layout, const void* desc_host, const void* paths_dev,
                        const float* cg_dev, int cg_len, const float* x, const float* sh,
                        const float* W, const int64_t* recv_sorted, const int64_t* src_sorted,
                        const int64_t* perm, int64_t c0, int64_t c1, const float* gout,
                        float* dW, float* dx_edge, float* dY_edge, void* stream);

/* K7 receiver-factorised form helpers: per-edge z rows (alpha_p sum_ij C x Y) for the edges
 * [e0, e1) of a receiver chunk, in path-major layout: path p region starts at
 * z_off_p * (n_e + 1) floats (n_e = e1 - e0) and holds (n_e + 1) rows of (2lo+1) * mul1 floats,
 * k-major then u; row n_e is a padding row the kernels never write.  The backward maps dz (same
 * layout) to dx_edge (n_e, in_dim) and dY_edge (n_e, 9) for those edges (sorted positions).  */
int gmp_tp_edge_z_f32(const void* desc_host, const void* paths_dev, const float* cg_dev,
                      int cg_len, const float* x, const float* sh, const int64_t* src_sorted,
                      const int64_t* perm, int64_t e0, int64_t e1, float* zbuf, void* stream);
int gmp_tp_edge_z_bwd_f32(const void* desc_host, const void* paths_dev, const float* cg_dev,
                          int cg_len, const float* x, const float* sh, const int64_t* src_sorted,
                          const int64_t* perm, int64_t e0, int64_t e1, const float* dzbuf,
                          float* dx_edge, float* dY_edge, void* stream);
/* Same with l_max = the largest l of any path (input, SH or output irreps; 0..3): with
 * l_max <= 2 the kernels are the l <= 2 instantiation (fewer registers, more waves per SIMD).
 * The plain entries above are l_max = 3 (any path). */
int gmp_tp_edge_z_lmax_f32(const void* desc_host, int l_max, const void* paths_dev,
                           const float* cg_dev, int cg_len, const float* x, const float* sh,
                           const int64_t* src_sorted, const int64_t* perm, int64_t e0, int64_t e1,
                           float* zbuf, void* stream);
int gmp_tp_edge_z_bwd_lmax_f32(const void* desc_host, int l_max, const void* paths_dev,
                               const float* cg_dev, int cg_len, const float* x, const float* sh,
                               const int64_t* src_sorted, const int64_t* perm, int64_t e0,
                               int64_t e1, const float* dzbuf, float* dx_edge, float* dY_edge,
                               void* stream);

/* K7 receiver-factorised per-receiver kernels (tfn_layer.py:73-87 regrouped): for the
 * receivers n of a chunk with chunk-local edge offsets eoff[n]..eoff[n+1] (receiver-sorted),
 * Z (n_e, w) z rows of one path, A (n_e, H) radial hidden features (H % 16 == 0, <= 256):
 *   outer: S[n, r, j] = sum_e Z[e, r] A[e, j] (n_recv, w, H), Sb[n, r] = sum_e Z[e, r]
 *   apply: dZ[e, r] = sum_j T[n, r, j] A[e, j] + Tb[n, r];  dA[e, j] += sum_r Z[e, r] T[n, r, j]
 * (T = G [W2_p]^T, Tb = G b2_p^T from the path GEMMs; dA is accumulated, dZ overwritten). */
int gmp_tp_node_outer_f32(int64_t n_recv, int64_t w, int64_t H, const int64_t* eoff,
                          const float* Z, const float* A, float* S, float* Sb, void* stream);
int gmp_tp_node_apply_f32(int64_t n_recv, int64_t w, int64_t H, const int64_t* eoff,
                          const float* Z, const float* A, const float* T, const float* Tb,
                          float* dZ, float* dA, void* stream);
/* apply runs on the bf16 MFMA over exact three-plane splits where its shapes allow (2, the
 * default: the v3 kernel for H = 256 and w % 32 == 0, then the v2 kernel for w >= 512,
 * w % 32 == 0, H % 64 == 0, 16-byte aligned operands), else on the f32 MFMA; set_x3(1) skips the
 * v3 kernel, set_x3(0) forces the f32 one (tests cover every form).  Returns the previous
 * setting. */
int gmp_tp_apply_set_x3(int on);

/* K7g path GEMMs of the receiver-factorised TP convolution on the bf16 MFMA through exact
 * three-plane f32 splits (replaces the library f32 GEMMs out = S W2p + Sb b2p and
 * T = G W2p^T of tfn_layer.py:73-87 regrouped; f32-class accuracy, see gmp_tpgemm.hip).
 * split_w2: from one path's block of the second radial Linear, W2p (mul1 * mul_out rows (u, w)
 *   of H floats) and b2p (mul1 * mul_out), writes (each if not null) the forward B planes Bf
 *   (bf16 values B[p][w][u H + j] = W2[(u, w), j], B[p][w][mul1 H + u] = b2[u, w], stored in
 *   MFMA fragment order, below; mul_out % 16 == 0) and the backward B planes Bt (values
 *   B[p][u H + j][w] = W2[(u, w), j], an N = mul1 H by K = mul_out operand in the same fragment
 *   order; mul_out % 32 == 0).
 * gemm_x3: C (+)= [A1 | A2] B^T for A1 (M x K1, row stride lda1), A2 (M x K2, lda2; K2 may be 0),
 *   B = 3 bf16 planes of an N x (K1 + K2) operand in fragment order: value (p, n, k) at
 *   ((((k / 32) (N / 16) + n / 16) 3 + p) 64 + n % 16 + 16 ((k % 32) / 8)) 8 + k % 8 (each
 *   64-lane block is one v_mfma_f32_16x16x32 B operand; the kernel loads it straight into
 *   registers); ldb = K1 + K2 and bplane = N ldb are checked (the dense sizes); N % 16 == 0.
 *   Element (r, col) of C at (r / cgrp) cldg + (r % cgrp) cldr + col cldn (accumulate != 0:
 *   C += result).  K1, K2 multiples of 32; lda* multiples of 4; A, B 16-byte aligned.
 *   Deterministic (no atomics, fixed k order). */
int gmp_tp_split_w2_f32(int64_t mul1, int64_t mul_out, int64_t H, const float* W2p,
                        const float* b2p, void* Bf, void* Bt, void* stream);
int gmp_tp_gemm_x3_f32(int64_t M, int64_t N, int64_t K1, const float* A1, int64_t lda1,
                       int64_t K2, const float* A2, int64_t lda2, const void* Bp, int64_t ldb,
                       int64_t bplane, float* C, int64_t cgrp, int64_t cldg, int64_t cldr,
                       int64_t cldn, int accumulate, void* stream);
/* Short-K, wide-N form of gemm_x3 (the backward T = G W2p^T: K = mul_out <= 128, N = mul1 H):
 *   C (M x N, row stride ldc) = A B^T, A (M x K, lda) f32, B = 3 bf16 planes of the N x K
 *   operand in gemm_x3's fragment order (ldb = K, bplane = N K checked; N % 16 == 0);
 * K a multiple of 32, <= 128.  Each workgroup keeps its split A rows in LDS and sweeps a range
 * of column tiles with B loaded straight into registers; C is written with non-temporal
 * stores. */
int gmp_tp_gemm_x3_widen_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                             const void* Bp, int64_t ldb, int64_t bplane, float* C, int64_t ldc,
                             void* stream);
/* Wide edge/row reduction C (m_total x n, row stride ldc) = A^T B over K rows, A (K x m_total,
 * row stride lda), B (K x n, ldb), m_total a multiple of 128, n a multiple of 16 (<= 128): the
 * TP path GEMM dW2p = S^T G.  Split-plane bf16 MFMA (the K5 kernel with column blocks of 128),
 * deterministic split-K reduction through the workspace. */
size_t gmp_outer_sum_cols_workspace_size(int64_t K, int64_t m_total, int64_t n);
int gmp_outer_sum_cols_f32(int64_t K, int64_t m_total, int64_t n, const float* A, int64_t lda,
                           const float* B, int64_t ldb, float* C, int64_t ldc, void* workspace,
                           size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * K5g GVP-GNN message function (models/layers/gvp_layer.py:101-170 per edge via GVPConv.message
 * :319-324; configuration of models/gvpgnn.py: activations (relu, None), vector_gate, s = 128,
 * v = 16, edge (32, 1)).  Vector tensors in the reference's (channel, xyz) row layout.
 *   gmp_gvp_layer_*: one GVP (128, 16) -> (128, 16) on E rows; Ws (128 x 144) = ws.weight on
 *     [s | |vh|], Wsv (16 x 128), Wh, Wv (16 x 16); relu = scalar activation on/off.  Backward
 *     writes ds_in, dv_in and the per-edge weight-gradient factors dspre, spre (E,128),
 *     dgate, vn (E,16), vh, dvpre, dvh (E,48).
 *   gmp_gvp_msg0_*: the first message GVP on [s_j, e_s, s_i] / [v_j, e_v, v_i] (j = send,
 *     i = recv) from node projections P (N, 256) = [s W_a^T | s W_b^T] and Q (N, 288) =
 *     [v W_ha^T | v W_hb^T] (33 channels zero-padded to 48, (channel, xyz)), es (E, 32),
 *     ev (E, 3); We (128 x 32), Wn (128 x 48), Wv (16 x 48), wev (48) zero-padded.  Backward
 *     writes dspre, spre (E,128), dgate (E,16), vn (E,48), vh, dvh (E,144), dvpre (E,48),
 *     des (E,32), dev (E,3).
 * ------------------------------------------------------------------------------------------ */
int gmp_gvp_layer_fwd_f32(int64_t n_edges, int relu, const float* s_in, const float* v_in,
                          const float* Ws, const float* bs, const float* Wsv, const float* bsv,
                          const float* Wh, const float* Wv, float* s_out, float* v_out,
                          void* stream);
/* gmp_gvp_layer_bwd_f32: spre (the pre-activation scalar rows, only the dWsv weight sum reads
 * them) may be NULL -- the caller then forms dWsv = (sum_e dgate_e (x) [s_e | vn_e]) Ws^T +
 * (sum_e dgate_e) (x) bs without them (r04: 1 KB per edge of HBM traffic less); vh (read only
 * by dWv) may be NULL too -- dWv = (sum_(e,x) dvpre (x) v_in) Wh^T (r05: 0.4 KB per edge). */
int gmp_gvp_layer_bwd_f32(int64_t n_edges, int relu, const float* s_in, const float* v_in,
                          const float* Ws, const float* bs, const float* Wsv, const float* bsv,
                          const float* Wh, const float* Wv, const float* ds_out,
                          const float* dv_out, float* ds_in, float* dv_in, float* dspre,
                          float* spre, float* dgate, float* vn, float* vh, float* dvpre,
                          float* dvh, void* stream);
/* gmp_gvp_msg0_bwd_agg_f32: gmp_gvp_msg0_bwd_f32 walking the receiver-sorted edges (perm: original
 * edge of sorted position k, NULL if the edges are receiver-sorted; rowptr: the receiver CSR)
 * and also reducing over each receiver, in registers, the rows the receiver-side sums need:
 * dPb (n_nodes, 128) = S_i dspre, dQb (n_nodes, 144) = S_i dvh, sgate_recv (n_nodes, 16) =
 * S_i dgate, svpre_recv (n_nodes, 48) = S_i dvpre (receivers without edges: zero rows; tree
 * order inside a 16-edge chunk).  The per-edge outputs are bitwise gmp_gvp_msg0_bwd_f32's. */
int gmp_gvp_msg0_bwd_agg_f32(int64_t n_edges, int64_t n_nodes, const int64_t* send,
                             const int64_t* recv, const int64_t* perm, const int64_t* rowptr,
                             const float* P, const float* Q, const float* es, const float* ev,
                             const float* We, const float* Wn, const float* b, const float* Wv,
                             const float* Wsv, const float* bsv, const float* wev,
                             const float* ds_out, const float* dv_out, float* dspre, float* spre,
                             float* dgate, float* vn, float* vh, float* dvpre, float* dvh,
                             float* des, float* dev, float* dPb, float* dQb, float* sgate_recv,
                             float* svpre_recv, void* stream);
/* gmp_gvp_layer_fwd_agg_f32: the last message GVP of GVPConv fused with the receivers' sum /
 * mean (gvp_layer.py:319-324, aggr "add" / "mean" = reduce GMP_REDUCE_SUM / GMP_REDUCE_MEAN):
 * s_agg (n_nodes, 128), v_agg (n_nodes, 16, 3) directly, no per-edge output rows.  The receiver
 * CSR: rowptr (n_nodes + 1), skey (E) the receiver of sorted position k, perm (E) its original
 * edge (NULL: the edges are already receiver-sorted); s_in / v_in in original edge order.  Each
 * receiver's rows are summed in sorted order by an in-wave segmented scan (deterministic;
 * within fp32 rounding of K3's sequential sum); receivers without in-edges get zeros. */
int gmp_gvp_layer_fwd_agg_f32(int64_t n_edges, int64_t n_nodes, int reduce, const int64_t* perm,
                              const int64_t* skey, const int64_t* rowptr, const float* s_in,
                              const float* v_in, const float* Ws, const float* bs,
                              const float* Wsv, const float* bsv, const float* Wh,
                              const float* Wv, float* s_agg, float* v_agg, void* stream);
/* gmp_gvp_layer_bwd_agg_f32: the same backward for the last message GVP of GVPConv, whose
 * per-edge outputs feed the receivers' aggregation (gvp_layer.py:319-324, aggr "add" / "mean"
 * = reduce GMP_REDUCE_SUM / GMP_REDUCE_MEAN): ds_node (n_nodes, 128), dv_node (n_nodes, 16, 3)
 * are the aggregation's node gradients, gathered per edge at index[e] (the receiver; x 1 /
 * max(count, 1) for the mean with count = rowptr[n + 1] - rowptr[n] of the receiver CSR,
 * exactly K3's mean backward; an index outside [0, n_nodes) contributes zeros) -- the (E, 176)
 * per-edge gradient of gmp_segment_reduce_bwd_f32 is never materialised. */
int gmp_gvp_layer_bwd_agg_f32(int64_t n_edges, int64_t n_nodes, int reduce, const int64_t* index,
                              const int64_t* rowptr, int relu, const float* s_in,
                              const float* v_in, const float* Ws, const float* bs,
                              const float* Wsv, const float* bsv, const float* Wh,
                              const float* Wv, const float* ds_node, const float* dv_node,
                              float* ds_in, float* dv_in, float* dspre, float* spre,
                              float* dgate, float* vn, float* vh, float* dvpre, float* dvh,
                              void* stream);
/* gmp_gvp_edge_embed_{fwd,bwd}_f32 (K1e): the GVP-GNN edge embedding W_e (models/gvpgnn.py:73-77,
 * :116) = LayerNorm((R, 1)) then GVP((R, 1), (so, 1), activations (None, None), vector_gate,
 * h_dim 1) (gvp_layer.py:101-170, :221-243) over E edge rows: radial (E, R) row-major 16-byte
 * aligned, unit (E, 3); parameters ln_w, ln_b (R) [the LayerNorm's weight / bias, eps], wh (1)
 * [wh.weight], Ws (so, R + 1) [ws.weight], bs (so), wv (1) [wv.weight], wsv (so) [wsv.weight],
 * bsv (1).  Forward: es (E, so), ev (E, 3) [= (E, 1, 3)].  Backward: the parameters' gradients
 * from grad_es (E, so), grad_ev (E, 3) (radial / unit get none: positions without
 * requires_grad), packed in grad_params as [ln_w R | ln_b R | wh 1 | Ws so (R + 1) | bs so |
 * wv 1 | wsv so | bsv 1] (2R + 3 + so (R + 3) floats); per-workgroup partial rows in the
 * workspace, added in a fixed order (deterministic).  R = 8 and 1 <= so <= 32 are compiled
 * (GMP_ERR_UNSUPPORTED otherwise: the caller runs the module chain). */
int gmp_gvp_edge_embed_fwd_f32(int64_t n_edges, int64_t radial_dim, int64_t so,
                               const float* radial, const float* unit, const float* ln_w,
                               const float* ln_b, const float* wh, const float* Ws,
                               const float* bs, const float* wv, const float* wsv,
                               const float* bsv, float eps, float* es, float* ev, void* stream);
size_t gmp_gvp_edge_embed_bwd_workspace_size(int64_t n_edges);
int gmp_gvp_edge_embed_bwd_f32(int64_t n_edges, int64_t radial_dim, int64_t so,
                               const float* radial, const float* unit, const float* ln_w,
                               const float* ln_b, const float* wh, const float* Ws,
                               const float* bs, const float* wv, const float* wsv,
                               const float* bsv, float eps, const float* grad_es,
                               const float* grad_ev, float* grad_params, void* workspace,
                               size_t workspace_bytes, void* stream);
/* gmp_gvp_ff_{fwd,bwd}_f32 (K17, r06): the node feed-forward of GVPConvLayer
 * (models/layers/gvp_layer.py:361-366, :433-434 -- ff_func = GVP((128, 16), (512, 32)) with
 * activations (relu, None) then GVP((512, 32), (128, 16)) with (None, None), vector_gate, h_dim 32;
 * GVP.forward gvp_layer.py:140-170) over N node rows in one kernel per direction.  s (N, 128),
 * v (N, 16, 3) row-major, all row tensors 16-byte aligned; weights in the reference's nn.Linear
 * layout: Wh1 (32, 16), Ws1 (512, 160) [columns s | |vh1|], b1 (512), Wv1 (32, 32), Wsv1
 * (32, 512), bsv1 (32), Wh2 (32, 32), Ws2 (128, 544) [columns s1 | |vh2|], b2 (128), Wv2 (16, 32),
 * Wsv2 (16, 128), bsv2 (16); Ws1, Wsv1, Ws2 16-byte aligned.
 * Forward: s2 (N, 128), v2 (N, 16, 3), gate1 (N, 32) [the first GVP's gate pre-activation] and
 * the right operands of the weight sums, zero-padded: B1 = [s | vn1 | 0] (N, 192),
 * B2 = [s1 | vn2 | 0] (N, 576) [s1 = relu(p1), vn = |vh| clamped], B3 = [v | 0] (N, 64),
 * B4 = [v1 | 0] (N, 128) [v1 the first GVP's vector output, (channel, xyz)].
 * Backward (from gate1, B2, s2 = the second GVP's pre-activation, grad_s2, grad_v2): ds (N, 128),
 * dv (N, 16, 3) and the left operands A1 = [dp1 | dgate1 | 0] (N, 576), A2 = [dp2 | dgate2 | 0]
 * (N, 192), A3 = [dvh1 | du1] (N, 192), A4 = [dvh2 | du2 | 0] (N, 192) [dp the gradient at a
 * scalar Linear's output, du = grad_v * sigmoid(gate) at W_v vh, dvh at vh; (channel, xyz)].
 * With C_k = A_k^T B_k (sums over the N rows) and x~ the xyz diagonal of a (3a, 3b) block:
 *   dWs1 = C1[:512, :160], db1 = colsum(dp1), dWsv1 = C1[512:544, :160] Ws1^T + dbsv1 b1^T;
 *   dWs2 = C2[:128, :544], db2 = colsum(dp2), dWsv2 = C2[128:144, :544] Ws2^T + dbsv2 b2^T;
 *   dWh1 = C3[:96, :48]~, dWv1 = C3[96:, :48]~ Wh1^T; dWh2 = C4[:96, :96]~,
 *   dWv2 = C4[96:144, :96]~ Wh2^T.  Exact f32 products. */
int gmp_gvp_ff_fwd_f32(int64_t n_nodes, const float* s_in, const float* v_in, const float* Wh1,
                       const float* Ws1, const float* b1, const float* Wv1, const float* Wsv1,
                       const float* bsv1, const float* Wh2, const float* Ws2, const float* b2,
                       const float* Wv2, const float* Wsv2, const float* bsv2, float* s_out,
                       float* v_out, float* gate1_out, float* B1, float* B2, float* B3, float* B4,
                       void* stream);
int gmp_gvp_ff_bwd_f32(int64_t n_nodes, const float* v_in, const float* gate1, const float* B2,
                       const float* s2, const float* ds_out, const float* dv_out,
                       const float* Wh1, const float* Ws1, const float* b1, const float* Wv1,
                       const float* Wsv1, const float* bsv1, const float* Wh2, const float* Ws2,
                       const float* b2, const float* Wv2, const float* Wsv2, const float* bsv2,
                       float* ds_in, float* dv_in, float* A1, float* A2, float* A3, float* A4,
                       void* stream);
int gmp_gvp_msg0_fwd_f32(int64_t n_edges, const int64_t* send, const int64_t* recv,
                         const float* P, const float* Q, const float* es, const float* ev,
                         const float* We, const float* Wn, const float* b, const float* Wv,
                         const float* Wsv, const float* bsv, const float* wev, float* s_out,
                         float* v_out, void* stream);
/* gmp_gvp_msg0_bwd_f32: spre (E, 128) and vh (E, 144), read only by the dWsv / dWv weight sums,
 * may be NULL (r05): the caller then forms those sums from the node projections,
 *   dWsv = (dgate^T [es | vn]) [We | Wn]^T + (S_j dgate)^T Pa + (S_i dgate)^T Pb + (1^T dgate) b,
 *   dWv[o, h] = sum_(n,x) (S_j dvpre)[n, o, x] Qa[n, h, x] + (S_i dvpre) .. Qb + wev[h] u[o]
 * (S_j, S_i the sender / receiver segment sums, u[o] = sum_(e,x) dvpre[e, o, x] ev[e, x]):
 * 2.2 KB per edge of HBM traffic less per layer. */
int gmp_gvp_msg0_bwd_f32(int64_t n_edges, const int64_t* send, const int64_t* recv,
                         const float* P, const float* Q, const float* es, const float* ev,
                         const float* We, const float* Wn, const float* b, const float* Wv,
                         const float* Wsv, const float* bsv, const float* wev,
                         const float* ds_out, const float* dv_out, float* dspre, float* spre,
                         float* dgate, float* vn, float* vh, float* dvpre, float* dvh,
                         float* des, float* dev, void* stream);

/* ------------------------------------------------------------------------------------------
 * K9 radius graph.  Replaces torch_cluster.radius_graph(pos, r, batch,
 * loop=False, max_num_neighbors) as PyG SchNet's RadiusInteractionGraph builds it
 * (models/schnet.py:47; GPU-kernel selection rule): edge j -> i for j != i of the same graph with
 * ((dx*dx + dy*dy) + dz*dz) < r*r in fp32 (dx = p_i - p_j, no contraction); per target the first
 * max_num_neighbors + 1 candidates in ascending j (self included) are kept, then self is dropped
 * (max_num_neighbors <= 0: no cap).  batch may be NULL (one graph).  Cells have edge
 * 1/inv_cell >= r over the box [lo, lo + dims/inv_cell), keyed (graph, cell):
 *   cells: cell id per node -> the caller buckets nodes with gmp_csr_build over
 *          num_graphs*dims[0]*dims[1]*dims[2] segments (cell_rowptr, cell_perm);
 *   count: number of sources per target;  fill: the sources of target i at
 *          offsets[i]..offsets[i+1], ascending -> edge_index sorted by (target, source).
 * ------------------------------------------------------------------------------------------ */
int gmp_radius_cells_f32(const float* pos, const int64_t* batch, int64_t n_nodes,
                         const float* lo3, float inv_cell, const int* dims3, int64_t* cell_out,
                         void* stream);
int gmp_radius_count_f32(const float* pos, const int64_t* batch, int64_t n_nodes, float r,
                         int64_t max_num_neighbors, const float* lo3, float inv_cell,
                         const int* dims3, const int64_t* cell, const int64_t* cell_rowptr,
                         const int64_t* cell_perm, int64_t* counts, void* stream);
int gmp_radius_fill_f32(const float* pos, const int64_t* batch, int64_t n_nodes, float r,
                        int64_t max_num_neighbors, const float* lo3, float inv_cell,
                        const int* dims3, const int64_t* cell, const int64_t* cell_rowptr,
                        const int64_t* cell_perm, const int64_t* offsets, int64_t* src_out,
                        void* stream);

/* ------------------------------------------------------------------------------------------
 * K10 batch collation (PyG Batch.from_data_list as the reference's loaders
 * build it, experiments/utils/train_utils.py:28,132).  edge_index_local: (2, E) graph-local
 * indices of B graphs packed back to back; node_ptr / edge_ptr: (B+1) prefix sums of the
 * per-graph node / edge counts.  Writes edge_index_out = local + node_ptr[graph of edge] and
 * batch_out[a] = graph of node a.  A local index outside [0, n_g) sets *err to 1 (err may be
 * NULL).  Empty graphs are allowed.
 * ------------------------------------------------------------------------------------------ */
int gmp_batch_collate(const int64_t* edge_index_local, int64_t n_edges, const int64_t* node_ptr,
                      const int64_t* edge_ptr, int64_t n_graphs, int64_t n_nodes,
                      int64_t* edge_index_out, int64_t* batch_out, int* err, void* stream);

/* ------------------------------------------------------------------------------------------
 * K11 triplets + angles / torsions.  Replaces `xyz_to_dat`
 * (models/layers/spherenet_layer.py:496-564) and the triplet/angle block of the DimeNet forward
 * (models/dimenet.py:79-90, PyG DimeNet.triplets).  edge_index (2, E): e = (j -> i).
 * Adjacency by target, entries sorted by (target, source): adj_rowptr (N+1), adj_src (source
 * of each entry), adj_eid (edge id of each entry).
 *   count: counts[e] = in-degree(j) - #{in-edges of j with source i}; dist[e] = |p_i - p_j|
 *          (dist may be NULL);
 *   fill:  for t in [offsets[e], offsets[e+1]): idx_kj[t] = edge (k -> j) for the k != i in
 *          ascending order, idx_ji[t] = e; angle[t] (mode 0: SphereNet, vertex j; mode 1:
 *          DimeNet, vertex i; may be NULL); torsion[t] (mode 0 only, may be NULL).
 * Arithmetic reproduces the reference's torch CPU evaluation op by op (see gmp_triplet.hip).
 * ------------------------------------------------------------------------------------------ */
int gmp_triplet_count(const float* pos, const int64_t* edge_index, int64_t n_edges,
                      int64_t n_nodes, const int64_t* adj_rowptr, const int64_t* adj_src,
                      int64_t* counts, float* dist, void* stream);
int gmp_triplet_fill_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                         int64_t n_nodes, const int64_t* adj_rowptr, const int64_t* adj_src,
                         const int64_t* adj_eid, const int64_t* offsets, int64_t n_triplets,
                         int mode, int64_t* idx_kj, int64_t* idx_ji, float* angle,
                         float* torsion, int64_t* torsion_kn, void* stream);
/* Backward of dist (E) and angle (T) w.r.t. pos (DimeNet / SphereNet under autograd): writes
 * 3T + 2E rows of 3 floats (`rows`) and their node ids (`node`): vertex, u-end and v-end rows
 * of every triplet, then +/- rows of every edge's distance; d pos = the segmented sum of rows
 * by node (the caller's CSR; deterministic).  grad_dist / grad_angle may be NULL (zero). */
int gmp_triplet_geom_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                             const int64_t* idx_kj, const int64_t* idx_ji, int64_t n_triplets,
                             int mode, const float* grad_dist, const float* grad_angle,
                             float* rows, int64_t* node, void* stream);
/* Backward of the SphereNet torsion (spherenet_layer.py:535-559 under autograd) w.r.t. pos:
 * torsion_kn (T, from gmp_triplet_fill_f32; -1 = no candidate) is the scatter-min's winning
 * k_n, which alone receives the gradient (torch_scatter's arg routing).  Writes 4T rows of 3
 * floats and their node ids (i, j, k, k_n blocks of T); d pos = their segmented sum by node. */
int gmp_triplet_torsion_bwd_f32(const float* pos, const int64_t* edge_index, int64_t n_edges,
                                const int64_t* idx_kj, const int64_t* idx_ji,
                                const int64_t* torsion_kn, int64_t n_triplets,
                                const float* grad_torsion, float* rows, int64_t* node,
                                void* stream);

/* ------------------------------------------------------------------------------------------
 * K12 fused LayerNorm + activation over rows (node-level MLPs: EGNN mlp_upd,
 * egnn_layer.py:37-39 / :82-86; GVP scalar LayerNorm, gvp_layer.py:221-243 with act = 2).
 * x (rows, d), d <= 512; act 0 relu, 1 silu, 2 identity.  Forward writes y = act(LN(x)) and
 * saves xhat (rows, d) and rstd (rows) for the backward.  Backward: grad_x (rows, d) and
 * grad_gamma_beta (2d) = [dgamma | dbeta] (deterministic; workspace from
 * gmp_ln_act_bwd_workspace_size).  grad_gamma_beta may be NULL: the workspace then holds
 * gmp_ln_act_bwd_partial_rows(rows) partial rows of width 2d, to be reduced by the caller
 * (gmp_sum_rows_f32, e.g. later / on another stream: gamma and beta are leaves of the graph).
 * gmp_sum_rows_f32: out[c] = sum_r partials[r, c] in a fixed order (deterministic).
 * ------------------------------------------------------------------------------------------ */
int gmp_ln_act_fwd_f32(int64_t rows, int64_t d, const float* x, const float* gamma,
                       const float* beta, float eps, int act, float* y, float* xhat_save,
                       float* rstd_save, void* stream);
size_t gmp_ln_act_bwd_workspace_size(int64_t rows, int64_t d);
int gmp_ln_act_bwd_f32(int64_t rows, int64_t d, const float* grad_y, const float* xhat,
                       const float* rstd, const float* gamma, const float* beta, int act,
                       float* grad_x, float* grad_gamma_beta, void* workspace,
                       size_t workspace_bytes, void* stream);
int64_t gmp_ln_act_bwd_partial_rows(int64_t rows);
int gmp_sum_rows_f32(const float* partials, int64_t nrows, int64_t width, float* out,
                     void* stream);

/* ------------------------------------------------------------------------------------------
 * GVP vector LayerNorm (gvp_layer.py:232-243: v / sqrt(mean_c clamp(|v_c|^2, 1e-8)), the norm
 * of _norm_no_nan, :66-73).  v (rows, channels, 3) contiguous, 1 <= channels <= 64.  Forward
 * writes out = v / vn; backward recomputes vn from v and writes grad_v from grad_out (the clamp
 * passes the gradient where |v_c|^2 >= 1e-8, as torch's clamp_min).  No workspace.
 * ------------------------------------------------------------------------------------------ */
int gmp_vec_norm_fwd_f32(int64_t rows, int64_t channels, const float* v, float* out,
                         void* stream);
int gmp_vec_norm_bwd_f32(int64_t rows, int64_t channels, const float* v, const float* grad_out,
                         float* grad_v, void* stream);
/* _norm_no_nan over the xyz axis of vh (rows, 3, h) contiguous (GVP.forward's |vh|,
 * gvp_layer.py:66-73, :101-170): out (rows, h) = sqrt(max(sum_x vh^2, 1e-8)); backward
 * grad_vh (rows, 3, h) from grad_out (rows, h). */
int gmp_xyz_norm_fwd_f32(int64_t rows, int64_t h, const float* vh, float* out, void* stream);
int gmp_xyz_norm_bwd_f32(int64_t rows, int64_t h, const float* vh, const float* grad_out,
                         float* grad_vh, void* stream);

/* ------------------------------------------------------------------------------------------
 * K8 MACE symmetric contraction (models/mace_modules/symmetric_contraction.py:20-188 with
 * element_dependent=False; SymmetricContraction.forward :81-85 concatenates the per-output-irrep
 * Contraction.forward :150-185), all output irreps of C channels at once, any irreps: x (N, C, D)
 * = reshape_irreps of C x (irreps) (irreps_tools.py:63-79; D <= 63 components per channel, any
 * parities, repeated l), correlation 1..4 folded into one polynomial over symmetric monomials
 * and evaluated over the sparse TERM LIST of the module's coupling pattern:
 *   out[b, out_base[m] + out_stride[m] c] = sum_{t in row m} coef[t, c] prod_{r < 4} xx[f_r(t)]
 * with xx = [x[b, c, 0..D-1], 1.0] (factor index D = the constant 1: degree < 4 monomials).
 * plan (int32): [row_ptr (rows + 1) | out_base (rows) | out_stride (rows) | terms (n_terms)],
 *   term word f0 | f1 << 6 | f2 << 12 | f3 << 18 | m << 24 (m < rows <= 255), terms of row m at
 *   row_ptr[m] .. row_ptr[m+1] - 1 (summed in that order);
 * coef (n_terms, C), term-major: coef[t, c] = A~_nu[c, m_t, q_t], the folded coefficient
 *   A~_nu[c, m, q] = sum over the distinct permutations p of monomial q of
 *   sum_k U_nu[m, p, k] W_nu[k, c] (the host builds the plan once and coef per call,
 *   differentiably).  out (N, rows C).
 * Backward: dx (N, C, D) (may be NULL) and dcoef partials (gmp_sc_groups(N), n_terms, C) (may
 * be NULL; the caller sums the groups in order; N = 0 writes one all-zero group).
 * Deterministic.  (ABI 5: the plan form replaces
 * the dense per-degree A_nu arguments and gmp_sc_monomials.)
 * ------------------------------------------------------------------------------------------ */
int gmp_sc_groups(int64_t n_nodes);
int gmp_symmetric_contraction_fwd_f32(int64_t n_nodes, int channels, int dim, int rows,
                                      int n_terms, const int32_t* plan, const float* coef,
                                      const float* x, float* out, void* stream);
int gmp_symmetric_contraction_bwd_f32(int64_t n_nodes, int channels, int dim, int rows,
                                      int n_terms, const int32_t* plan, const float* coef,
                                      const float* x, const float* gout, float* dx,
                                      float* dcoef_partials, void* stream);

/* ------------------------------------------------------------------------------------------
 * K13 SchNet CFConv fused message + aggregation (PyG 2.3.1 CFConv.message `x_j * W` and
 * aggr "add", called at schnet.py:72; replaces the x_j gather, the (E, F) product and the
 * scatter-sum of a15):
 *   out[s, :] = sum_{k in [rowptr[s], rowptr[s+1])} x[xidx[perm[k]], :] * w[perm[k], :]
 * Forward: CSR over dst, xidx = src.  x-gradient: CSR over src, x = grad_out, xidx = dst.
 * F % 4 == 0, x / w / out 16-byte aligned.  Out-of-range xidx -> zero term, *err = 1.
 * gmp_cfconv_wgrad_f32: dw[e, :] = g[gidx[e], :] * x[xidx[e], :] (W-gradient, gidx = dst,
 * xidx = src); out-of-range -> zero row, *err = 1.  Deterministic (no atomics).
 * ------------------------------------------------------------------------------------------ */
int gmp_cfconv_aggregate_f32(const float* x, int64_t n_x, const int64_t* xidx, const float* w,
                             int64_t n_items, int64_t F, const int64_t* perm,
                             const int64_t* rowptr, int64_t n_seg, float* out, int32_t* err,
                             void* stream);
int gmp_cfconv_wgrad_f32(const float* g, int64_t n_g, const int64_t* gidx, const float* x,
                         int64_t n_x, const int64_t* xidx, int64_t n_items, int64_t F, float* dw,
                         int32_t* err, void* stream);
/* Scaled forms (SchNet W = filter(edge_attr) * C with the per-edge cosine cutoff C, never
 * materialised): the aggregate uses W[e] * escale[e] (rounded per element as the reference's
 * product); the W-gradient is written as (g[gidx[e]] * x[xidx[e]]) * escale[e], the gradient
 * w.r.t. filter(edge_attr).  escale may be NULL (= the unscaled entry points). */
int gmp_cfconv_aggregate_scaled_f32(const float* x, int64_t n_x, const int64_t* xidx,
                                    const float* w, const float* escale, int64_t n_items,
                                    int64_t F, const int64_t* perm, const int64_t* rowptr,
                                    int64_t n_seg, float* out, int32_t* err, void* stream);
int gmp_cfconv_wgrad_scaled_f32(const float* g, int64_t n_g, const int64_t* gidx, const float* x,
                                int64_t n_x, const int64_t* xidx, const float* escale,
                                int64_t n_items, int64_t F, float* dw, int32_t* err,
                                void* stream);

/* ------------------------------------------------------------------------------------------
 * K14 shifted softplus (PyG ShiftedSoftplus, the SchNet filter-network / interaction
 * activation, schnet.py:72): torch softplus semantics (beta 1, threshold 20) minus `shift`.
 *   fwd: y = (x > 20 ? x : log1p(exp(x))) - shift
 *   bwd: grad_x = x > 20 ? grad_y : grad_y * z / (z + 1), z = exp(x)
 * n % 4 == 0, 16-byte aligned pointers.
 * ------------------------------------------------------------------------------------------ */
int gmp_ssp_fwd_f32(const float* x, int64_t n, float shift, float* y, void* stream);
int gmp_ssp_bwd_f32(const float* x, const float* grad_y, int64_t n, float* grad_x,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GMP_H_ */
