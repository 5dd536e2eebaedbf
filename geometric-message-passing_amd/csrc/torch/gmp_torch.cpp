// PyTorch operator registration of the gmp C ABI (include/gmp.h): TORCH_LIBRARY(gmp, m).
//
// The reference's native boundary is torch_scatter's custom operators
// (`torch.ops.torch_scatter.scatter_sum/mean/max`, reached from `from torch_scatter import
// scatter` at models/layers/egnn_layer.py:4 and models/layers/tfn_layer.py:2).
// This file is the same kind of boundary for the MI355X kernels: one schema per C-ABI entry
// point, a CUDA(HIP)-key implementation that allocates outputs through the caching allocator,
// launches on the current stream OF THE INPUTS' DEVICE (device guard, as torch_scatter's
// CUDAGuard), checks dtype / device / contiguity / shape of every tensor argument and maps error
// codes to RuntimeError (TORCH_CHECK), and a Meta implementation (shapes only) so torch.compile /
// FakeTensor tracing treats every op as one opaque node.  No CPU fallback.
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/ATen.h>
#include <torch/library.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../../include/gmp.h"

namespace {

using at::Tensor;
using c10::optional;

// ------------------------------------------------------------------ device guard + checks
// Every CUDA implementation opens an OpGuard on its first tensor argument: the current device
// becomes that tensor's device (so the current stream is that device's stream), and every
// tensor checked afterwards must live on the same device.
thread_local int g_op_device = -1;

struct OpGuard {
  c10::hip::HIPGuardMasqueradingAsCUDA guard;
  int prev;
  static c10::Device dev_of(const Tensor& t, const char* op) {
    TORCH_CHECK(t.defined() && t.is_cuda(), "gmp.", op,
                ": inputs must be HIP device tensors (no CPU fallback)");
    return t.device();
  }
  OpGuard(const Tensor& t, const char* op) : guard(dev_of(t, op)), prev(g_op_device) {
    g_op_device = t.device().index();
  }
  ~OpGuard() { g_op_device = prev; }
};

void* cur_stream() {
  return reinterpret_cast<void*>(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

void check_rc(int rc, const char* name) {
  TORCH_CHECK(rc == GMP_OK, name, " failed: ", gmp_error_string(rc), " (code ", rc,
              ", hip error ", gmp_last_hip_error(), ")");
}

void on_device(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), "gmp: ", what, " must be a HIP device tensor (no CPU fallback)");
  TORCH_CHECK(g_op_device < 0 || t.device().index() == g_op_device, "gmp: ", what,
              " is on device ", t.device(), " but the op's inputs are on cuda:", g_op_device);
}
void need(const Tensor& t, at::ScalarType st, const char* what) {
  on_device(t, what);
  TORCH_CHECK(t.scalar_type() == st, "gmp: ", what, " has dtype ", t.scalar_type(), ", expected ",
              st);
  TORCH_CHECK(t.is_contiguous(), "gmp: ", what, " must be contiguous");
}
const Tensor& f32(const Tensor& t, const char* what) {
  need(t, at::kFloat, what);
  return t;
}
const Tensor& i64(const Tensor& t, const char* what) {
  need(t, at::kLong, what);
  return t;
}
const Tensor& i32(const Tensor& t, const char* what) {
  need(t, at::kInt, what);
  return t;
}
// shape check: t.sizes() == s
void shape(const Tensor& t, at::IntArrayRef s, const char* what) {
  TORCH_CHECK(t.sizes() == s, "gmp: ", what, " has shape ", t.sizes(), ", expected ", s);
}
void numel(const Tensor& t, int64_t n, const char* what) {
  TORCH_CHECK(t.numel() == n, "gmp: ", what, " has ", t.numel(), " elements, expected ", n);
}
void opt_f32(const optional<Tensor>& t, at::IntArrayRef s, const char* what) {
  if (t.has_value() && t->defined()) {
    f32(*t, what);
    shape(*t, s, what);
  }
}

float* fp(const Tensor& t) { return t.defined() && t.numel() ? t.data_ptr<float>() : nullptr; }
const float* cfp(const optional<Tensor>& t) {
  return t.has_value() && t->defined() && t->numel() ? t->data_ptr<float>() : nullptr;
}
int64_t* ip(const Tensor& t) { return t.defined() && t.numel() ? t.data_ptr<int64_t>() : nullptr; }
at::TensorOptions fopt(const Tensor& like) { return like.options().dtype(at::kFloat); }

int reduce_code(const std::string& r) {
  if (r == "sum" || r == "add") return GMP_REDUCE_SUM;
  if (r == "mean") return GMP_REDUCE_MEAN;
  if (r == "max") return GMP_REDUCE_MAX;
  TORCH_CHECK(false, "gmp: unsupported reduce '", r, "'");
}

// ------------------------------------------------------------------ index: CSR, gather, reduce
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> csr_build(const Tensor& index, int64_t n_seg,
                                                             const optional<Tensor>& payload) {
  OpGuard g(index, "csr_build");
  i64(index, "index");
  TORCH_CHECK(n_seg >= 0, "gmp.csr_build: n_seg >= 0");
  const int64_t n = index.numel();
  auto o = index.options();
  Tensor perm = at::empty({n}, o), rowptr = at::empty({n_seg + 1}, o), sorted = at::empty({n}, o);
  Tensor pl;
  if (payload.has_value()) {
    pl = i64(*payload, "payload");
    numel(pl, n, "payload");
  }
  Tensor pls = at::empty({pl.defined() ? n : 0}, o);
  Tensor err = at::zeros({1}, o.dtype(at::kInt));
  const size_t ws_b = gmp_csr_workspace_size(n, n_seg);
  Tensor ws = at::empty({(int64_t)ws_b}, o.dtype(at::kByte));
  check_rc(gmp_csr_build(ip(index), n, n_seg, pl.defined() ? ip(pl) : nullptr, ip(perm),
                         ip(rowptr), ip(sorted), pl.defined() ? ip(pls) : nullptr,
                         err.data_ptr<int32_t>(), ws.data_ptr(), ws_b, cur_stream()),
           "gmp_csr_build");
  return {perm, rowptr, sorted, pls, err};
}

Tensor gather_rows(const Tensor& src, const Tensor& index) {
  OpGuard g(src, "gather_rows");
  f32(src, "src");
  i64(index, "index");
  TORCH_CHECK(src.dim() == 2, "gmp.gather_rows: src must be 2-D");
  Tensor out = at::empty({index.numel(), src.size(1)}, src.options());
  check_rc(gmp_gather_rows_f32(fp(src), src.size(0), src.size(1), ip(index), index.numel(),
                               fp(out), nullptr, cur_stream()),
           "gmp_gather_rows_f32");
  return out;
}

std::tuple<Tensor, Tensor> segment_reduce(const Tensor& src, const optional<Tensor>& perm,
                                          const Tensor& rowptr, int64_t n_seg,
                                          const std::string& reduce) {
  OpGuard g(src, "segment_reduce");
  f32(src, "src");
  i64(rowptr, "rowptr");
  TORCH_CHECK(src.dim() == 2 && rowptr.numel() == n_seg + 1,
              "gmp.segment_reduce: src must be 2-D and rowptr hold n_seg + 1 offsets");
  const int red = reduce_code(reduce);
  const int64_t F = src.size(1);
  Tensor pm;
  if (perm.has_value()) {
    pm = i64(*perm, "perm");
    numel(pm, src.size(0), "perm");
  }
  Tensor out = at::empty({n_seg, F}, src.options());
  Tensor argmax = at::empty({red == GMP_REDUCE_MAX ? n_seg : 0, F}, rowptr.options());
  const size_t ws_b = gmp_segment_reduce_workspace_size(src.size(0), n_seg, F, red);
  Tensor ws = at::empty({(int64_t)ws_b}, src.options().dtype(at::kByte));
  check_rc(gmp_segment_reduce_f32(fp(src), src.size(0), F, pm.defined() ? ip(pm) : nullptr,
                                  ip(rowptr), n_seg, red, fp(out),
                                  red == GMP_REDUCE_MAX ? ip(argmax) : nullptr,
                                  ws_b ? ws.data_ptr() : nullptr, ws_b, cur_stream()),
           "gmp_segment_reduce_f32");
  return {out, argmax};
}

Tensor segment_reduce_bwd(const Tensor& grad_out, const Tensor& index, const Tensor& rowptr,
                          const std::string& reduce, const optional<Tensor>& argmax,
                          int64_t n_items) {
  OpGuard g(grad_out, "segment_reduce_bwd");
  f32(grad_out, "grad_out");
  i64(index, "index");
  i64(rowptr, "rowptr");
  TORCH_CHECK(grad_out.dim() == 2 && rowptr.numel() == grad_out.size(0) + 1 &&
                  index.numel() == n_items,
              "gmp.segment_reduce_bwd: grad_out (n_seg, F), rowptr (n_seg + 1), index (n_items)");
  const int red = reduce_code(reduce);
  Tensor am;
  if (argmax.has_value()) {
    am = i64(*argmax, "argmax");
    shape(am, grad_out.sizes(), "argmax");
  }
  TORCH_CHECK(red != GMP_REDUCE_MAX || am.defined(), "gmp.segment_reduce_bwd: max needs argmax");
  Tensor gs = at::empty({n_items, grad_out.size(1)}, grad_out.options());
  check_rc(gmp_segment_reduce_bwd_f32(fp(grad_out), grad_out.size(0), grad_out.size(1),
                                      ip(index), n_items, ip(rowptr), red,
                                      am.defined() ? ip(am) : nullptr, fp(gs), cur_stream()),
           "gmp_segment_reduce_bwd_f32");
  return gs;
}

// ------------------------------------------------------------------ EGNN fused edge kernels
gmp_egnn_params egnn_params(const std::vector<Tensor>& p, int64_t d) {
  TORCH_CHECK(p.size() == 14, "gmp.egnn: 14 parameter tensors expected");
  // w1d, b1, ln1_w, ln1_b, W2, b2, ln2_w, ln2_b, W3, b3, ln3_w, ln3_b, w4, b4
  static const int kind[14] = {1, 1, 1, 1, 2, 1, 1, 1, 2, 1, 1, 1, 1, 0};
  for (size_t k = 0; k < p.size(); ++k) {
    f32(p[k], "egnn parameter");
    const int64_t want = kind[k] == 2 ? d * d : (kind[k] == 1 ? d : 1);
    numel(p[k], want, "egnn parameter");
  }
  gmp_egnn_params P;
  P.w1d = fp(p[0]); P.b1 = fp(p[1]); P.ln1_w = fp(p[2]); P.ln1_b = fp(p[3]);
  P.W2 = fp(p[4]); P.b2 = fp(p[5]); P.ln2_w = fp(p[6]); P.ln2_b = fp(p[7]);
  P.W3 = fp(p[8]); P.b3 = fp(p[9]); P.ln3_w = fp(p[10]); P.ln3_b = fp(p[11]);
  P.w4 = fp(p[12]); P.b4 = fp(p[13]);
  return P;
}

// K15 weight images (gmp_egnn_node_image_f32) of L layers: W0s[l] (d, 2d), W3s[l] (d, d), W1ns[l] the
// next layer's mlp_msg.0.weight (d, >= 2d, unit column stride) or None.  -> uint8 (L, bytes).
Tensor egnn_node_image(const std::vector<Tensor>& W0s, const std::vector<Tensor>& W3s,
                       const std::vector<optional<Tensor>>& W1ns) {
  TORCH_CHECK(!W0s.empty() && W3s.size() == W0s.size() && W1ns.size() == W0s.size(),
              "gmp.egnn_node_image: one W0, W3 and W1n entry per layer");
  OpGuard g(W0s[0], "egnn_node_image");
  const int64_t L = (int64_t)W0s.size(), d = W0s[0].size(0);
  std::vector<gmp_egnn_node_params> P(L);
  for (int64_t l = 0; l < L; ++l) {
    f32(W0s[l], "W0");
    f32(W3s[l], "W3");
    TORCH_CHECK(W0s[l].dim() == 2 && W0s[l].size(0) == d && W0s[l].size(1) == 2 * d &&
                    W3s[l].dim() == 2 && W3s[l].size(0) == d && W3s[l].size(1) == d,
                "gmp.egnn_node_image: W0 (d, 2d), W3 (d, d)");
    P[l] = gmp_egnn_node_params{};
    P[l].W0 = fp(W0s[l]);
    P[l].W3 = fp(W3s[l]);
    const optional<Tensor>& w1 = W1ns[l];
    if (w1.has_value() && w1->defined()) {
      TORCH_CHECK(w1->scalar_type() == at::kFloat && w1->dim() == 2 && w1->size(0) == d &&
                      w1->size(1) >= 2 * d && w1->stride(1) == 1 && w1->stride(0) >= 2 * d &&
                      w1->device() == W0s[0].device(),
                  "gmp.egnn_node_image: W1n must be a (d, >= 2d) float32 matrix, unit column stride");
      P[l].W1n = w1->data_ptr<float>();
      P[l].ld1 = w1->stride(0);
    }
  }
  const size_t bytes = gmp_egnn_node_image_bytes(d);
  TORCH_CHECK(bytes > 0, "gmp.egnn_node_image: d must be 32, 64 or 128");
  Tensor img = at::empty({L, (int64_t)bytes}, W0s[0].options().dtype(at::kByte));
  check_rc(gmp_egnn_node_image_f32(d, L, P.data(), img.data_ptr(), cur_stream()),
           "gmp_egnn_node_image_f32");
  return img;
}

// K15 node update (gmp_egnn_node_fwd_f32): vecs = [b0, ln1_w, ln1_b, b3, ln2_w, ln2_b]; image =
// this layer's row of egnn_node_image; with_ab: the image holds the next layer's W1n.
// Returns (h_out (N, d), ab (N, 2d) or (0, 2d), xhat (2, N, d) or (0, N, d), rstd (2, N) or (0, N)).
std::tuple<Tensor, Tensor, Tensor, Tensor> egnn_node_fwd(
    const Tensor& h, const Tensor& m_aggr, const std::vector<Tensor>& vecs, const Tensor& image,
    bool with_ab, int64_t act, bool residual, double eps, bool train) {
  OpGuard g(h, "egnn_node_fwd");
  f32(h, "h");
  f32(m_aggr, "m_aggr");
  TORCH_CHECK(h.dim() == 2 && m_aggr.sizes() == h.sizes(), "gmp.egnn_node_fwd: h, m_aggr (N, d)");
  const int64_t N = h.size(0), d = h.size(1);
  TORCH_CHECK(vecs.size() == 6, "gmp.egnn_node_fwd: 6 parameter vectors expected");
  for (int k = 0; k < 6; ++k) {
    f32(vecs[k], "egnn_node parameter");
    numel(vecs[k], d, "egnn_node parameter");
  }
  TORCH_CHECK(image.scalar_type() == at::kByte && image.is_contiguous() &&
                  image.numel() == (int64_t)gmp_egnn_node_image_bytes(d) &&
                  image.device() == h.device(),
              "gmp.egnn_node_fwd: image must be one layer's row of egnn_node_image");
  gmp_egnn_node_params P{};
  P.b0 = fp(vecs[0]); P.ln1_w = fp(vecs[1]); P.ln1_b = fp(vecs[2]);
  P.b3 = fp(vecs[3]); P.ln2_w = fp(vecs[4]); P.ln2_b = fp(vecs[5]);
  Tensor ho = at::empty({N, d}, h.options());
  Tensor abo = at::empty({with_ab ? N : 0, 2 * d}, h.options());
  Tensor xh = at::empty({train ? 2 : 0, N, d}, h.options());
  Tensor rs = at::empty({train ? 2 : 0, N}, h.options());
  check_rc(gmp_egnn_node_fwd_f32(N, d, fp(h), fp(m_aggr), &P, image.data_ptr(), (int)act,
                                 residual ? 1 : 0, (float)eps, fp(ho),
                                 with_ab ? fp(abo) : nullptr, train ? fp(xh) : nullptr,
                                 train ? fp(rs) : nullptr, cur_stream()),
           "gmp_egnn_node_fwd_f32");
  return {ho, abo, xh, rs};
}

void egnn_graph_checks(const Tensor& pos, const Tensor& rowptr, const Tensor& recv,
                       const Tensor& send) {
  f32(pos, "pos");
  i64(rowptr, "rowptr");
  i64(recv, "recv");
  i64(send, "send");
  TORCH_CHECK(pos.dim() == 2 && pos.size(1) == 3, "gmp.egnn: pos must be (N, 3)");
  numel(rowptr, pos.size(0) + 1, "rowptr");
  numel(send, recv.numel(), "send");
}

std::tuple<Tensor, Tensor, Tensor, Tensor> egnn_edge_fwd(
    const Tensor& AB, const Tensor& pos, const Tensor& rowptr, const Tensor& recv,
    const Tensor& send, const std::vector<Tensor>& params, int64_t act, bool msg_mean, double eps,
    bool train, int64_t xhat_planes) {
  OpGuard g(AB, "egnn_edge_fwd");
  TORCH_CHECK(xhat_planes == 2 || xhat_planes == 3, "gmp.egnn_edge_fwd: xhat_planes is 2 or 3");
  f32(AB, "AB");
  egnn_graph_checks(pos, rowptr, recv, send);
  TORCH_CHECK(AB.dim() == 2 && AB.size(1) % 2 == 0 && AB.size(0) == pos.size(0),
              "gmp.egnn_edge_fwd: AB must be (N, 2d)");
  const int64_t N = pos.size(0), E = recv.numel(), d = AB.size(1) / 2;
  gmp_egnn_params P = egnn_params(params, d);
  Tensor m = at::empty({N, d}, fopt(AB)), pa = at::empty({N, 3}, fopt(AB));
  // training: the saved LayerNorm outputs, exactly the planes the forward writes (x_hat1, x_hat2
  // [, x_hat3]); the backward reads their count from xhat.size(0)
  Tensor xh = at::empty({train ? xhat_planes : 0, E, d}, fopt(AB));
  Tensor rs = at::empty({train ? E : 0, 3}, fopt(AB));
  check_rc(gmp_egnn_edge_fwd_f32(N, E, d, fp(AB), fp(pos), ip(rowptr), ip(recv), ip(send), &P,
                                 (int)act, msg_mean, (float)eps, fp(m), fp(pa),
                                 train ? fp(xh) : nullptr, (int)xhat_planes,
                                 train ? fp(rs) : nullptr, cur_stream()),
           "gmp_egnn_edge_fwd_f32");
  return {m, pa, xh, rs};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> egnn_edge_bwd(
    const Tensor& pos, const Tensor& rowptr, const Tensor& recv, const Tensor& send,
    const std::vector<Tensor>& params, int64_t act, bool msg_mean, const Tensor& xhat,
    const Tensor& rstd, const Tensor& g_m, const Tensor& g_p, const optional<Tensor>& amax) {
  OpGuard g(pos, "egnn_edge_bwd");
  egnn_graph_checks(pos, rowptr, recv, send);
  f32(xhat, "xhat");
  f32(rstd, "rstd");
  f32(g_m, "g_m_aggr");
  f32(g_p, "g_pos_aggr");
  // the forward's saved planes: (2, E, d) = x_hat1, x_hat2 (x_hat3 recomputed), or (3, E, d)
  TORCH_CHECK(xhat.dim() == 3 && (xhat.size(0) == 2 || xhat.size(0) == 3),
              "gmp.egnn_edge_bwd: xhat must be the forward's (2 or 3, E, d) planes");
  const int64_t N = pos.size(0), E = recv.numel(), d = xhat.size(2);
  shape(xhat, {xhat.size(0), E, d}, "xhat");
  shape(rstd, {E, 3}, "rstd");
  shape(g_m, {N, d}, "g_m_aggr");
  shape(g_p, {N, 3}, "g_pos_aggr");
  gmp_egnn_params P = egnn_params(params, d);
  if (amax.has_value()) {
    i32(*amax, "amax");
    TORCH_CHECK(amax->numel() >= 2, "gmp.egnn_edge_bwd: amax has 2 words");
  }
  auto o = fopt(pos);
  Tensor dA = at::empty({N, d}, o), dpr = at::empty({N, 3}, o), dp1 = at::empty({E, d}, o);
  Tensor gd = at::empty({E, 3}, o), dp2 = at::empty({E, d}, o), dp3 = at::empty({E, d}, o);
  Tensor part = at::empty({gmp_egnn_edge_bwd_partials_rows(E, d), 8 * d + 1}, o);
  check_rc(gmp_egnn_edge_bwd_amax_f32(
               N, E, d, fp(pos), ip(rowptr), ip(recv), ip(send), &P, (int)act, msg_mean,
               E > 0 ? fp(xhat) : nullptr, (int)xhat.size(0), fp(rstd), fp(g_m), fp(g_p), fp(dA),
               fp(dpr), fp(dp1), fp(gd), fp(dp2), fp(dp3), fp(part),
               amax.has_value() ? reinterpret_cast<uint32_t*>(amax->data_ptr<int32_t>())
                                : nullptr,
               cur_stream()),
           "gmp_egnn_edge_bwd_amax_f32");
  return {dA, dpr, dp1, gd, dp2, dp3, part};
}

// ------------------------------------------------------------------ SchNet CFConv, SSP
Tensor cfconv_aggregate(const Tensor& x, const Tensor& xidx, const Tensor& w, const Tensor& perm,
                        const Tensor& rowptr, int64_t n_seg, const optional<Tensor>& escale) {
  OpGuard g(x, "cfconv_aggregate");
  f32(x, "x");
  f32(w, "w");
  i64(xidx, "xidx");
  i64(perm, "perm");
  i64(rowptr, "rowptr");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == x.size(1),
              "gmp.cfconv_aggregate: x (N, F), w (E, F)");
  const int64_t E = w.size(0);
  numel(xidx, E, "xidx");
  numel(perm, E, "perm");
  numel(rowptr, n_seg + 1, "rowptr");
  opt_f32(escale, {E}, "escale");
  Tensor out = at::empty({n_seg, x.size(1)}, x.options());
  Tensor err = at::zeros({1}, x.options().dtype(at::kInt));
  check_rc(gmp_cfconv_aggregate_scaled_f32(fp(x), x.size(0), ip(xidx), fp(w), cfp(escale), E,
                                           x.size(1), ip(perm), ip(rowptr), n_seg, fp(out),
                                           err.data_ptr<int32_t>(), cur_stream()),
           "gmp_cfconv_aggregate_scaled_f32");
  return out;
}

Tensor cfconv_wgrad(const Tensor& gr, const Tensor& gidx, const Tensor& x, const Tensor& xidx,
                    const optional<Tensor>& escale) {
  OpGuard g(gr, "cfconv_wgrad");
  f32(gr, "g");
  f32(x, "x");
  i64(gidx, "gidx");
  i64(xidx, "xidx");
  TORCH_CHECK(gr.dim() == 2 && x.dim() == 2 && gr.size(1) == x.size(1),
              "gmp.cfconv_wgrad: g (N, F), x (N, F)");
  const int64_t E = gidx.numel();
  numel(xidx, E, "xidx");
  opt_f32(escale, {E}, "escale");
  Tensor dw = at::empty({E, x.size(1)}, x.options());
  Tensor err = at::zeros({1}, x.options().dtype(at::kInt));
  check_rc(gmp_cfconv_wgrad_scaled_f32(fp(gr), gr.size(0), ip(gidx), fp(x), x.size(0), ip(xidx),
                                       cfp(escale), E, x.size(1), fp(dw),
                                       err.data_ptr<int32_t>(), cur_stream()),
           "gmp_cfconv_wgrad_scaled_f32");
  return dw;
}

Tensor ssp_fwd(const Tensor& x, double shift) {
  OpGuard g(x, "ssp_fwd");
  f32(x, "x");
  Tensor y = at::empty_like(x);
  check_rc(gmp_ssp_fwd_f32(fp(x), x.numel(), (float)shift, fp(y), cur_stream()), "gmp_ssp_fwd_f32");
  return y;
}

Tensor ssp_bwd(const Tensor& x, const Tensor& gy) {
  OpGuard g(x, "ssp_bwd");
  f32(x, "x");
  f32(gy, "grad_y");
  shape(gy, x.sizes(), "grad_y");
  Tensor gx = at::empty_like(x);
  check_rc(gmp_ssp_bwd_f32(fp(x), fp(gy), x.numel(), fp(gx), cur_stream()), "gmp_ssp_bwd_f32");
  return gx;
}

// ------------------------------------------------------------------ LayerNorm + activation rows
std::tuple<Tensor, Tensor, Tensor> ln_act_fwd(const Tensor& x, const Tensor& gamma,
                                              const Tensor& beta, double eps, int64_t act) {
  OpGuard g(x, "ln_act_fwd");
  f32(x, "x");
  const int64_t d = x.size(-1), rows = x.numel() / d;
  f32(gamma, "gamma");
  f32(beta, "beta");
  numel(gamma, d, "gamma");
  numel(beta, d, "beta");
  Tensor y = at::empty_like(x), xh = at::empty_like(x), rs = at::empty({rows}, x.options());
  check_rc(gmp_ln_act_fwd_f32(rows, d, fp(x), fp(gamma), fp(beta), (float)eps, (int)act, fp(y),
                              fp(xh), fp(rs), cur_stream()),
           "gmp_ln_act_fwd_f32");
  return {y, xh, rs};
}

std::tuple<Tensor, Tensor> ln_act_bwd(const Tensor& gy, const Tensor& xhat, const Tensor& rstd,
                                      const Tensor& gamma, const Tensor& beta, int64_t act) {
  OpGuard g(gy, "ln_act_bwd");
  f32(gy, "grad_y");
  f32(xhat, "xhat");
  f32(rstd, "rstd");
  f32(gamma, "gamma");
  f32(beta, "beta");
  const int64_t d = xhat.size(-1), rows = xhat.numel() / d;
  shape(gy, xhat.sizes(), "grad_y");
  numel(rstd, rows, "rstd");
  numel(gamma, d, "gamma");
  numel(beta, d, "beta");
  Tensor gx = at::empty_like(xhat), gb = at::empty({2 * d}, xhat.options());
  const size_t ws_b = gmp_ln_act_bwd_workspace_size(rows, d);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, xhat.options().dtype(at::kByte));
  check_rc(gmp_ln_act_bwd_f32(rows, d, fp(gy), fp(xhat), fp(rstd), fp(gamma), fp(beta), (int)act,
                              fp(gx), fp(gb), ws.data_ptr(), ws_b, cur_stream()),
           "gmp_ln_act_bwd_f32");
  return {gx, gb};
}

// GVP vector LayerNorm rows (N, C, 3)
Tensor vec_norm_fwd(const Tensor& v) {
  OpGuard g(v, "vec_norm_fwd");
  f32(v, "v");
  TORCH_CHECK(v.dim() == 3 && v.size(2) == 3, "vec_norm_fwd: v must be (rows, channels, 3)");
  Tensor out = at::empty_like(v);
  check_rc(gmp_vec_norm_fwd_f32(v.size(0), v.size(1), fp(v), fp(out), cur_stream()),
           "gmp_vec_norm_fwd_f32");
  return out;
}

Tensor vec_norm_bwd(const Tensor& v, const Tensor& gout) {
  OpGuard g(v, "vec_norm_bwd");
  f32(v, "v");
  f32(gout, "grad_out");
  TORCH_CHECK(v.dim() == 3 && v.size(2) == 3, "vec_norm_bwd: v must be (rows, channels, 3)");
  shape(gout, v.sizes(), "grad_out");
  Tensor gv = at::empty_like(v);
  check_rc(gmp_vec_norm_bwd_f32(v.size(0), v.size(1), fp(v), fp(gout), fp(gv), cur_stream()),
           "gmp_vec_norm_bwd_f32");
  return gv;
}

// GVP |vh| over the xyz axis of (rows, 3, h)
Tensor xyz_norm_fwd(const Tensor& vh) {
  OpGuard g(vh, "xyz_norm_fwd");
  f32(vh, "vh");
  TORCH_CHECK(vh.dim() == 3 && vh.size(1) == 3, "xyz_norm_fwd: vh must be (rows, 3, h)");
  Tensor out = at::empty({vh.size(0), vh.size(2)}, vh.options());
  check_rc(gmp_xyz_norm_fwd_f32(vh.size(0), vh.size(2), fp(vh), fp(out), cur_stream()),
           "gmp_xyz_norm_fwd_f32");
  return out;
}

Tensor xyz_norm_bwd(const Tensor& vh, const Tensor& gout) {
  OpGuard g(vh, "xyz_norm_bwd");
  f32(vh, "vh");
  f32(gout, "grad_out");
  TORCH_CHECK(vh.dim() == 3 && vh.size(1) == 3, "xyz_norm_bwd: vh must be (rows, 3, h)");
  shape(gout, {vh.size(0), vh.size(2)}, "grad_out");
  Tensor gv = at::empty_like(vh);
  check_rc(gmp_xyz_norm_bwd_f32(vh.size(0), vh.size(2), fp(vh), fp(gout), fp(gv), cur_stream()),
           "gmp_xyz_norm_bwd_f32");
  return gv;
}

// ------------------------------------------------------------------ K1 featurisation
int64_t edge_checks(const Tensor& pos, const Tensor& edge_index) {
  f32(pos, "pos");
  i64(edge_index, "edge_index");
  TORCH_CHECK(pos.dim() == 2 && pos.size(1) == 3, "gmp: pos must be (N, 3)");
  TORCH_CHECK(edge_index.dim() == 2 && edge_index.size(0) == 2, "gmp: edge_index must be (2, E)");
  return edge_index.size(1);
}

std::tuple<Tensor, Tensor> edge_featurize(const Tensor& pos, const Tensor& edge_index,
                                          at::ArrayRef<double> bessel_w, double prefactor,
                                          double r_max, double p, int64_t lmax) {
  OpGuard g(pos, "edge_featurize");
  const int64_t E = edge_checks(pos, edge_index), nb = (int64_t)bessel_w.size();
  TORCH_CHECK(0 <= lmax && lmax <= 5, "gmp.edge_featurize: lmax in 0..5");
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor sh = at::empty({E, (lmax + 1) * (lmax + 1)}, pos.options());
  Tensor rad = at::empty({E, nb}, pos.options());
  check_rc(gmp_edge_featurize_lmax_f32(fp(pos), ip(edge_index), E, (int)lmax, (int)nb, w.data(),
                                       (float)prefactor, (float)r_max, (float)p, nullptr, nullptr,
                                       fp(sh), fp(rad), cur_stream()),
           "gmp_edge_featurize_lmax_f32");
  return {sh, rad};
}

Tensor edge_featurize_bwd(const Tensor& pos, const Tensor& edge_index,
                          at::ArrayRef<double> bessel_w, double prefactor, double r_max, double p,
                          const optional<Tensor>& g_sh, const optional<Tensor>& g_rad,
                          int64_t lmax) {
  OpGuard g(pos, "edge_featurize_bwd");
  const int64_t E = edge_checks(pos, edge_index), nb = (int64_t)bessel_w.size();
  TORCH_CHECK(0 <= lmax && lmax <= 5, "gmp.edge_featurize_bwd: lmax in 0..5");
  opt_f32(g_sh, {E, (lmax + 1) * (lmax + 1)}, "g_sh");
  opt_f32(g_rad, {E, nb}, "g_radial");
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor gv = at::empty({E, 3}, pos.options());
  check_rc(gmp_edge_featurize_lmax_bwd_f32(fp(pos), ip(edge_index), E, (int)lmax, (int)nb,
                                           w.data(), (float)prefactor, (float)r_max, (float)p,
                                           cfp(g_sh), cfp(g_rad), fp(gv), cur_stream()),
           "gmp_edge_featurize_lmax_bwd_f32");
  return gv;
}

std::tuple<Tensor, Tensor> edge_featurize_gvp(const Tensor& pos, const Tensor& edge_index,
                                              at::ArrayRef<double> bessel_w, double prefactor,
                                              double r_max, double p) {
  OpGuard g(pos, "edge_featurize_gvp");
  const int64_t E = edge_checks(pos, edge_index), nb = (int64_t)bessel_w.size();
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor rad = at::empty({E, nb}, pos.options()), unit = at::empty({E, 3}, pos.options());
  check_rc(gmp_edge_featurize_gvp_f32(fp(pos), ip(edge_index), E, (int)nb, w.data(),
                                      (float)prefactor, (float)r_max, (float)p, nullptr, fp(rad),
                                      fp(unit), cur_stream()),
           "gmp_edge_featurize_gvp_f32");
  return {rad, unit};
}

Tensor edge_featurize_gvp_bwd(const Tensor& pos, const Tensor& edge_index,
                              at::ArrayRef<double> bessel_w, double prefactor, double r_max,
                              double p, const optional<Tensor>& g_rad,
                              const optional<Tensor>& g_unit) {
  OpGuard g(pos, "edge_featurize_gvp_bwd");
  const int64_t E = edge_checks(pos, edge_index), nb = (int64_t)bessel_w.size();
  opt_f32(g_rad, {E, nb}, "g_radial");
  opt_f32(g_unit, {E, 3}, "g_unit");
  std::vector<float> w(bessel_w.begin(), bessel_w.end());
  Tensor gv = at::empty({E, 3}, pos.options());
  check_rc(gmp_edge_featurize_gvp_bwd_f32(fp(pos), ip(edge_index), E, (int)nb, w.data(),
                                          (float)prefactor, (float)r_max, (float)p, cfp(g_rad),
                                          cfp(g_unit), fp(gv), cur_stream()),
           "gmp_edge_featurize_gvp_bwd_f32");
  return gv;
}

std::tuple<Tensor, Tensor, Tensor> schnet_featurize(const Tensor& pos, const Tensor& edge_index,
                                                    const Tensor& offsets, double coeff,
                                                    double cutoff) {
  OpGuard g(pos, "schnet_featurize");
  const int64_t E = edge_checks(pos, edge_index);
  f32(offsets, "offsets");
  const int64_t G = offsets.numel();
  Tensor d = at::empty({E}, pos.options()), rbf = at::empty({E, G}, pos.options()),
         cut = at::empty({E}, pos.options());
  check_rc(gmp_schnet_featurize_f32(fp(pos), ip(edge_index), E, (int)G, fp(offsets),
                                    (float)coeff, (float)cutoff, fp(d), fp(rbf), fp(cut),
                                    cur_stream()),
           "gmp_schnet_featurize_f32");
  return {d, rbf, cut};
}

Tensor schnet_featurize_bwd(const Tensor& pos, const Tensor& edge_index, const Tensor& offsets,
                            double coeff, double cutoff, const optional<Tensor>& g_dist,
                            const optional<Tensor>& g_rbf, const optional<Tensor>& g_cut) {
  OpGuard g(pos, "schnet_featurize_bwd");
  const int64_t E = edge_checks(pos, edge_index);
  f32(offsets, "offsets");
  const int64_t G = offsets.numel();
  opt_f32(g_dist, {E}, "g_dist");
  opt_f32(g_rbf, {E, G}, "g_rbf");
  opt_f32(g_cut, {E}, "g_cut");
  Tensor gv = at::empty({E, 3}, pos.options());
  check_rc(gmp_schnet_featurize_bwd_f32(fp(pos), ip(edge_index), E, (int)G, fp(offsets),
                                        (float)coeff, (float)cutoff, cfp(g_dist), cfp(g_rbf),
                                        cfp(g_cut), fp(gv), cur_stream()),
           "gmp_schnet_featurize_bwd_f32");
  return gv;
}

// ------------------------------------------------------------------ K16 Gate / BatchNorm
Tensor gate_fwd(const Tensor& x, const Tensor& out_map, double c_act, double c_gate) {
  OpGuard g(x, "gate_fwd");
  f32(x, "x");
  i32(out_map, "out_map");
  TORCH_CHECK(x.dim() == 2 && out_map.dim() == 2 && out_map.size(1) == 2,
              "gmp.gate_fwd: x (B, c_in), out_map (c_out, 2)");
  const int64_t B = x.size(0), c_in = x.size(1), c_out = out_map.size(0);
  Tensor y = at::empty({B, c_out}, x.options());
  check_rc(gmp_gate_fwd_f32(B, (int)c_in, (int)c_out, out_map.data_ptr<int32_t>(), (float)c_act,
                            (float)c_gate, fp(x), fp(y), cur_stream()),
           "gmp_gate_fwd_f32");
  return y;
}

Tensor gate_bwd(const Tensor& x, const Tensor& grad_y, const Tensor& in_map, double c_act,
                double c_gate) {
  OpGuard g(x, "gate_bwd");
  f32(x, "x");
  f32(grad_y, "grad_y");
  i32(in_map, "in_map");
  TORCH_CHECK(x.dim() == 2 && grad_y.dim() == 2 && grad_y.size(0) == x.size(0),
              "gmp.gate_bwd: x (B, c_in), grad_y (B, c_out)");
  shape(in_map, {x.size(1), 4}, "in_map");
  const int64_t B = x.size(0), c_in = x.size(1), c_out = grad_y.size(1);
  Tensor gx = at::empty_like(x);
  check_rc(gmp_gate_bwd_f32(B, (int)c_in, (int)c_out, in_map.data_ptr<int32_t>(), (float)c_act,
                            (float)c_gate, fp(x), fp(grad_y), fp(gx), cur_stream()),
           "gmp_gate_bwd_f32");
  return gx;
}

void bn_table_checks(const Tensor& x, const Tensor& col_chan, const Tensor& chan_col,
                     const Tensor& chan_info, const Tensor& weight) {
  f32(x, "x");
  i32(col_chan, "col_chan");
  i32(chan_col, "chan_col");
  i32(chan_info, "chan_info");
  f32(weight, "weight");
  TORCH_CHECK(x.dim() == 2, "gmp.irreps_bn: x must be (B, C)");
  numel(col_chan, x.size(1), "col_chan");
  const int64_t nf = chan_col.numel();
  shape(chan_info, {nf, 2}, "chan_info");
  numel(weight, nf, "weight");
}

std::tuple<Tensor, Tensor, Tensor> irreps_bn_fwd(const Tensor& x, const Tensor& col_chan,
                                                 const Tensor& chan_col, const Tensor& chan_info,
                                                 const Tensor& weight,
                                                 const optional<Tensor>& bias,
                                                 Tensor running_mean, Tensor running_var,
                                                 bool training, double momentum, double eps) {
  OpGuard g(x, "irreps_bn_fwd");
  bn_table_checks(x, col_chan, chan_col, chan_info, weight);
  f32(running_mean, "running_mean");
  f32(running_var, "running_var");
  const int64_t B = x.size(0), C = x.size(1), nf = chan_col.size(0);
  numel(running_var, nf, "running_var");
  if (bias.has_value() && bias->defined() && bias->numel()) {
    f32(*bias, "bias");
    numel(*bias, running_mean.numel(), "bias");
  }
  Tensor y = at::empty_like(x), shift = at::empty({nf}, x.options()),
         invstd = at::empty({nf}, x.options());
  const size_t ws_b = gmp_irreps_bn_workspace_size(B, (int)C, (int)nf);
  Tensor ws = at::empty({(int64_t)ws_b}, x.options().dtype(at::kByte));
  check_rc(gmp_irreps_bn_fwd_f32(B, (int)C, (int)nf, col_chan.data_ptr<int32_t>(),
                                 chan_col.data_ptr<int32_t>(), chan_info.data_ptr<int32_t>(),
                                 fp(x), fp(weight), cfp(bias), fp(running_mean), fp(running_var),
                                 training ? 1 : 0, (float)momentum, (float)eps, fp(y), fp(shift),
                                 fp(invstd), ws.data_ptr(), ws_b, cur_stream()),
           "gmp_irreps_bn_fwd_f32");
  return {y, shift, invstd};
}

std::tuple<Tensor, Tensor, Tensor> irreps_bn_bwd(const Tensor& x, const Tensor& grad_y,
                                                 const Tensor& col_chan, const Tensor& chan_col,
                                                 const Tensor& chan_info, const Tensor& weight,
                                                 const Tensor& shift, const Tensor& invstd,
                                                 bool training, int64_t n_scalar) {
  OpGuard g(x, "irreps_bn_bwd");
  bn_table_checks(x, col_chan, chan_col, chan_info, weight);
  f32(grad_y, "grad_y");
  f32(shift, "shift");
  f32(invstd, "invstd");
  shape(grad_y, x.sizes(), "grad_y");
  const int64_t B = x.size(0), C = x.size(1), nf = chan_col.size(0);
  numel(shift, nf, "shift");
  numel(invstd, nf, "invstd");
  Tensor gx = at::empty_like(x), gw = at::empty({nf}, x.options()),
         gb = at::empty({n_scalar}, x.options());
  const size_t ws_b = gmp_irreps_bn_workspace_size(B, (int)C, (int)nf);
  Tensor ws = at::empty({(int64_t)ws_b}, x.options().dtype(at::kByte));
  check_rc(gmp_irreps_bn_bwd_f32(B, (int)C, (int)nf, col_chan.data_ptr<int32_t>(),
                                 chan_col.data_ptr<int32_t>(), chan_info.data_ptr<int32_t>(),
                                 fp(x), fp(grad_y), fp(weight), fp(shift), fp(invstd),
                                 training ? 1 : 0, fp(gx), fp(gw),
                                 n_scalar > 0 ? fp(gb) : nullptr, ws.data_ptr(), ws_b,
                                 cur_stream()),
           "gmp_irreps_bn_bwd_f32");
  return {gx, gw, gb};
}

// ------------------------------------------------------------------ K8 symmetric contraction
// plan: the int32 term plan of gmp_symmetric_contraction_fwd_f32 ([row_ptr | out_base |
// out_stride | terms], built and validated on the host by gmp_amd.equivariant); rows = M
int64_t sc_terms(const Tensor& x, const Tensor& plan, int64_t rows, const Tensor& coef) {
  f32(x, "x");
  TORCH_CHECK(x.dim() == 3, "gmp.symmetric_contraction: x must be (N, C, D)");
  TORCH_CHECK(x.size(2) >= 1 && x.size(2) <= 63, "gmp.symmetric_contraction: D must be 1..63");
  TORCH_CHECK(rows >= 1 && rows <= 255, "gmp.symmetric_contraction: rows must be 1..255");
  need(plan, at::kInt, "plan");
  TORCH_CHECK(plan.dim() == 1 && plan.numel() >= 3 * rows + 1,
              "gmp.symmetric_contraction: plan must hold 3 rows + 1 + n_terms int32");
  const int64_t T = plan.numel() - (3 * rows + 1);
  f32(coef, "coef");
  shape(coef, {T, x.size(1)}, "coef");
  return T;
}

Tensor symmetric_contraction_fwd(const Tensor& x, const Tensor& plan, int64_t rows,
                                 const Tensor& coef) {
  OpGuard g(x, "symmetric_contraction_fwd");
  const int64_t T = sc_terms(x, plan, rows, coef);
  const int64_t N = x.size(0), C = x.size(1), D = x.size(2);
  Tensor out = at::empty({N, rows * C}, x.options());
  check_rc(gmp_symmetric_contraction_fwd_f32(N, (int)C, (int)D, (int)rows, (int)T,
                                             plan.data_ptr<int32_t>(), fp(coef), fp(x), fp(out),
                                             cur_stream()),
           "gmp_symmetric_contraction_fwd_f32");
  return out;
}

std::tuple<Tensor, Tensor> symmetric_contraction_bwd(const Tensor& x, const Tensor& plan,
                                                     int64_t rows, const Tensor& coef,
                                                     const Tensor& gout) {
  OpGuard g(x, "symmetric_contraction_bwd");
  const int64_t T = sc_terms(x, plan, rows, coef);
  f32(gout, "gout");
  const int64_t N = x.size(0), C = x.size(1), D = x.size(2);
  shape(gout, {N, rows * C}, "gout");
  Tensor dx = at::empty_like(x);
  Tensor part = at::empty({gmp_sc_groups(N), T, C}, x.options());
  check_rc(gmp_symmetric_contraction_bwd_f32(N, (int)C, (int)D, (int)rows, (int)T,
                                             plan.data_ptr<int32_t>(), fp(coef), fp(x), fp(gout),
                                             fp(dx), fp(part), cur_stream()),
           "gmp_symmetric_contraction_bwd_f32");
  return {dx, part};
}

// ------------------------------------------------------------------ K7 per-edge z rows
// The host descriptor travels as int[] (n_paths, in_dim, out_dim, sh_dim, weight_numel, z_size,
// n_blocks, blk_off[8], blk_mul[8], blk_l[8] [, l_max]); the 64-byte path records as a device
// uint8 tensor.  l_max (the largest l of any path; default 3) picks the z kernels' instantiation.
struct TpDescHost {
  int n_paths, in_dim, out_dim, sh_dim;
  long long weight_numel;
  int z_size, n_blocks;
  int blk_off[8], blk_mul[8], blk_l[8];
};
static_assert(sizeof(TpDescHost) == 128, "descriptor layout (include/gmp.h)");

TpDescHost tp_desc(at::IntArrayRef d) {
  TORCH_CHECK(d.size() == 31 || d.size() == 32, "gmp.tp: descriptor has 31 (+ l_max) ints");
  TpDescHost h;
  h.n_paths = (int)d[0]; h.in_dim = (int)d[1]; h.out_dim = (int)d[2]; h.sh_dim = (int)d[3];
  h.weight_numel = d[4]; h.z_size = (int)d[5]; h.n_blocks = (int)d[6];
  for (int k = 0; k < 8; ++k) {
    h.blk_off[k] = (int)d[7 + k];
    h.blk_mul[k] = (int)d[15 + k];
    h.blk_l[k] = (int)d[23 + k];
  }
  return h;
}

// l_max the z / dz kernels are instantiated for: it must cover every input block's l and the SH
// order (sh_dim = (l_sh + 1)^2), else the l <= 2 instantiation would skip an l = 3 path and leave
// its z rows unwritten
int tp_lmax(at::IntArrayRef d) {
  const int l = d.size() == 32 ? (int)d[31] : 3;
  TORCH_CHECK(0 <= l && l <= 5, "gmp.tp: l_max in 0..5");
  const TpDescHost h = tp_desc(d);
  TORCH_CHECK(0 < h.n_blocks && h.n_blocks <= 8, "gmp.tp: 1..8 output blocks");
  for (int k = 0; k < h.n_blocks; ++k)
    TORCH_CHECK(h.blk_l[k] <= l, "gmp.tp: l_max ", l, " below output block l ", h.blk_l[k]);
  int l_sh = 0;
  while ((l_sh + 1) * (l_sh + 1) < h.sh_dim) ++l_sh;
  TORCH_CHECK((l_sh + 1) * (l_sh + 1) == h.sh_dim, "gmp.tp: sh_dim must be (l + 1)^2");
  TORCH_CHECK(l_sh <= l, "gmp.tp: l_max ", l, " below the spherical-harmonics order ", l_sh);
  return l;
}

void tp_edge_checks(const TpDescHost& h, const Tensor& paths, const Tensor& cg, const Tensor& x,
                    const Tensor& sh, const Tensor& src_sorted, const Tensor& perm, int64_t e0,
                    int64_t e1) {
  need(paths, at::kByte, "paths");
  numel(paths, 64 * (int64_t)h.n_paths, "paths");
  f32(cg, "cg");
  f32(x, "x");
  f32(sh, "sh");
  i64(src_sorted, "src_sorted");
  i64(perm, "perm");
  TORCH_CHECK(x.dim() == 2 && x.size(1) == h.in_dim, "gmp.tp_edge_z: x must be (N, in_dim)");
  const int64_t E = src_sorted.numel();
  shape(sh, {E, (int64_t)h.sh_dim}, "sh");
  numel(perm, E, "perm");
  TORCH_CHECK(0 <= e0 && e0 <= e1 && e1 <= E, "gmp.tp_edge_z: 0 <= e0 <= e1 <= E");
}

Tensor tp_edge_z(at::IntArrayRef desc, const Tensor& paths, const Tensor& cg, const Tensor& x,
                 const Tensor& sh, const Tensor& src_sorted, const Tensor& perm, int64_t e0,
                 int64_t e1) {
  OpGuard g(x, "tp_edge_z");
  const TpDescHost h = tp_desc(desc);
  tp_edge_checks(h, paths, cg, x, sh, src_sorted, perm, e0, e1);
  Tensor z = at::empty({(e1 - e0 + 1) * h.z_size}, x.options());
  check_rc(gmp_tp_edge_z_lmax_f32(&h, tp_lmax(desc), paths.data_ptr(), fp(cg), (int)cg.numel(),
                                  fp(x), fp(sh), ip(src_sorted), ip(perm), e0, e1, fp(z),
                                  cur_stream()),
           "gmp_tp_edge_z_lmax_f32");
  return z;
}

std::tuple<Tensor, Tensor> tp_edge_z_bwd(at::IntArrayRef desc, const Tensor& paths,
                                         const Tensor& cg, const Tensor& x, const Tensor& sh,
                                         const Tensor& src_sorted, const Tensor& perm, int64_t e0,
                                         int64_t e1, const Tensor& dz) {
  OpGuard g(x, "tp_edge_z_bwd");
  const TpDescHost h = tp_desc(desc);
  tp_edge_checks(h, paths, cg, x, sh, src_sorted, perm, e0, e1);
  f32(dz, "dz");
  numel(dz, (e1 - e0 + 1) * h.z_size, "dz");
  Tensor dx = at::empty({e1 - e0, (int64_t)h.in_dim}, x.options());
  Tensor dY = at::empty({e1 - e0, (int64_t)h.sh_dim}, x.options());
  check_rc(gmp_tp_edge_z_bwd_lmax_f32(&h, tp_lmax(desc), paths.data_ptr(), fp(cg),
                                      (int)cg.numel(), fp(x), fp(sh), ip(src_sorted), ip(perm),
                                      e0, e1, fp(dz), fp(dx), fp(dY), cur_stream()),
           "gmp_tp_edge_z_bwd_lmax_f32");
  return {dx, dY};
}

// per-edge-weight form (equivariant.TP_MODE = "edge", or radial hidden sizes outside the node form): the
// chunk [c0, c1) of receiver-sorted edges with its weights W (c1 - c0, weight_numel)
void tp_conv_fwd(int64_t layout, at::IntArrayRef desc, const Tensor& paths, const Tensor& cg,
                 const Tensor& x, const Tensor& sh, const Tensor& W, const Tensor& src_sorted,
                 const Tensor& perm, int64_t c0, int64_t c1, Tensor msg) {
  OpGuard g(x, "tp_conv_fwd");
  const TpDescHost h = tp_desc(desc);
  tp_edge_checks(h, paths, cg, x, sh, src_sorted, perm, c0, c1);
  f32(W, "W");
  f32(msg, "msg");
  shape(W, {c1 - c0, (int64_t)h.weight_numel}, "W");
  shape(msg, {src_sorted.numel(), (int64_t)h.out_dim}, "msg");
  check_rc(gmp_tp_conv_fwd_f32((int)layout, &h, paths.data_ptr(), fp(cg), (int)cg.numel(), fp(x),
                               fp(sh), fp(W), ip(src_sorted), ip(perm), c0, c1, fp(msg),
                               cur_stream()),
           "gmp_tp_conv_fwd_f32");
}

Tensor tp_conv_bwd(int64_t layout, at::IntArrayRef desc, const Tensor& paths, const Tensor& cg,
                   const Tensor& x, const Tensor& sh, const Tensor& W, const Tensor& recv_sorted,
                   const Tensor& src_sorted, const Tensor& perm, int64_t c0, int64_t c1,
                   const Tensor& gout, Tensor dx_edge, Tensor dY_edge) {
  OpGuard g(x, "tp_conv_bwd");
  const TpDescHost h = tp_desc(desc);
  tp_edge_checks(h, paths, cg, x, sh, src_sorted, perm, c0, c1);
  const int64_t E = src_sorted.numel();
  f32(W, "W");
  i64(recv_sorted, "recv_sorted");
  f32(gout, "gout");
  f32(dx_edge, "dx_edge");
  f32(dY_edge, "dY_edge");
  shape(W, {c1 - c0, (int64_t)h.weight_numel}, "W");
  numel(recv_sorted, E, "recv_sorted");
  TORCH_CHECK(gout.dim() == 2 && gout.size(1) == h.out_dim, "gmp.tp_conv_bwd: gout (N, out_dim)");
  shape(dx_edge, {E, (int64_t)h.in_dim}, "dx_edge");
  shape(dY_edge, {E, (int64_t)h.sh_dim}, "dY_edge");
  Tensor dW = at::empty_like(W);
  check_rc(gmp_tp_conv_bwd_f32((int)layout, &h, paths.data_ptr(), fp(cg), (int)cg.numel(), fp(x),
                               fp(sh), fp(W), ip(recv_sorted), ip(src_sorted), ip(perm), c0, c1,
                               fp(gout), fp(dW), fp(dx_edge), fp(dY_edge), cur_stream()),
           "gmp_tp_conv_bwd_f32");
  return dW;
}

// ------------------------------------------------------------------ K7 node form
void node_checks(const Tensor& eoff, const Tensor& Z, const Tensor& A, int64_t w) {
  i64(eoff, "eoff");
  f32(Z, "Z");
  f32(A, "A");
  TORCH_CHECK(eoff.numel() >= 1, "gmp.tp_node: eoff holds n_recv + 1 offsets");
  TORCH_CHECK(A.dim() == 2, "gmp.tp_node: A must be (n_e, H)");
  TORCH_CHECK(Z.dim() == 2 && Z.size(1) == w && Z.size(0) >= A.size(0),
              "gmp.tp_node: Z must be (>= n_e, w)");
}

std::tuple<Tensor, Tensor> tp_node_outer(const Tensor& eoff, const Tensor& Z, const Tensor& A,
                                         int64_t w) {
  OpGuard g(A, "tp_node_outer");
  node_checks(eoff, Z, A, w);
  const int64_t c = eoff.numel() - 1, H = A.size(1);
  Tensor S = at::empty({c, w, H}, A.options()), Sb = at::empty({c, w}, A.options());
  check_rc(gmp_tp_node_outer_f32(c, w, H, ip(eoff), fp(Z), fp(A), fp(S), fp(Sb), cur_stream()),
           "gmp_tp_node_outer_f32");
  return {S, Sb};
}

void tp_node_apply(const Tensor& eoff, const Tensor& Z, const Tensor& A, const Tensor& T,
                   const Tensor& Tb, Tensor dA, Tensor dZ) {
  OpGuard g(A, "tp_node_apply");
  const int64_t w = Z.size(1);
  node_checks(eoff, Z, A, w);
  const int64_t c = eoff.numel() - 1, H = A.size(1);
  f32(T, "T");
  f32(Tb, "Tb");
  f32(dA, "dA");
  f32(dZ, "dZ");
  numel(T, c * w * H, "T");
  numel(Tb, c * w, "Tb");
  shape(dA, A.sizes(), "dA");
  shape(dZ, Z.sizes(), "dZ");
  check_rc(gmp_tp_node_apply_f32(c, w, H, ip(eoff), fp(Z), fp(A), fp(T), fp(Tb), fp(dZ), fp(dA),
                                 cur_stream()),
           "gmp_tp_node_apply_f32");
}

Tensor tp_split_w2(const Tensor& W2, const Tensor& b2, int64_t off, int64_t mul1, int64_t mo,
                   bool fwd) {
  OpGuard g(W2, "tp_split_w2");
  f32(W2, "W2");
  f32(b2, "b2");
  TORCH_CHECK(W2.dim() == 2 && b2.numel() == W2.size(0), "gmp.tp_split_w2: W2 (wn, H), b2 (wn)");
  TORCH_CHECK(off >= 0 && mul1 > 0 && mo > 0 && off + mul1 * mo <= W2.size(0),
              "gmp.tp_split_w2: path block outside W2");
  const int64_t H = W2.size(1), K1 = mul1 * H;
  Tensor planes = at::empty({fwd ? 3 * mo * (K1 + mul1) : 3 * K1 * mo},
                            W2.options().dtype(at::kShort));
  check_rc(gmp_tp_split_w2_f32(mul1, mo, H, fp(W2) + off * H, fp(b2) + off,
                               fwd ? planes.data_ptr() : nullptr, fwd ? nullptr : planes.data_ptr(),
                               cur_stream()),
           "gmp_tp_split_w2_f32");
  return planes;
}

// C (+)= [A1 | A2] B^T with the grouped epilogue addressing of gmp_tp_gemm_x3_f32 (C mutated)
void tp_gemm_x3(const Tensor& A1, int64_t K1, const optional<Tensor>& A2, int64_t K2,
                const Tensor& Bp, int64_t ldb, int64_t N, Tensor C, int64_t c_offset,
                int64_t cgrp, int64_t cldg, int64_t cldr, int64_t cldn, bool accumulate) {
  OpGuard g(A1, "tp_gemm_x3");
  f32(A1, "A1");
  need(Bp, at::kShort, "B planes");
  f32(C, "C");
  TORCH_CHECK(A1.dim() == 2 && K1 <= A1.size(1), "gmp.tp_gemm_x3: A1 must be (M, >= K1)");
  const int64_t M = A1.size(0);
  if (A2.has_value() && A2->defined()) {
    f32(*A2, "A2");
    TORCH_CHECK(A2->dim() == 2 && A2->size(0) == M && K2 <= A2->size(1),
                "gmp.tp_gemm_x3: A2 must be (M, >= K2)");
  } else {
    TORCH_CHECK(K2 == 0, "gmp.tp_gemm_x3: K2 > 0 needs A2");
  }
  TORCH_CHECK(ldb == K1 + K2 && Bp.numel() >= 3 * N * ldb, "gmp.tp_gemm_x3: B planes hold 3 N ldb");
  TORCH_CHECK(cgrp > 0 && c_offset >= 0 && cldg >= 0 && cldr >= 0 && cldn >= 0,
              "gmp.tp_gemm_x3: epilogue addressing");
  if (M > 0 && N > 0) {
    const int64_t last = c_offset + ((M - 1) / cgrp) * cldg + std::min(cgrp - 1, M - 1) * cldr +
                         (N - 1) * cldn;
    TORCH_CHECK(last < C.numel(), "gmp.tp_gemm_x3: the output block reaches element ", last,
                " of C (", C.numel(), " elements)");
  }
  check_rc(gmp_tp_gemm_x3_f32(M, N, K1, fp(A1), A1.size(1), K2, cfp(A2),
                              A2.has_value() && A2->defined() ? A2->size(1) : 0, Bp.data_ptr(),
                              ldb, N * ldb, C.data_ptr<float>() + c_offset, cgrp, cldg, cldr, cldn,
                              accumulate, cur_stream()),
           "gmp_tp_gemm_x3_f32");
}

Tensor tp_gemm_x3_widen(const Tensor& A, const Tensor& Bp, int64_t N) {
  OpGuard g(A, "tp_gemm_x3_widen");
  f32(A, "A");
  need(Bp, at::kShort, "B planes");
  TORCH_CHECK(A.dim() == 2, "gmp.tp_gemm_x3_widen: A must be (M, K)");
  const int64_t M = A.size(0), K = A.size(1);
  TORCH_CHECK(Bp.numel() >= 3 * N * K, "gmp.tp_gemm_x3_widen: B planes hold 3 N K");
  Tensor C = at::empty({M, N}, A.options());
  check_rc(gmp_tp_gemm_x3_widen_f32(M, N, K, fp(A), K, Bp.data_ptr(), K, N * K, fp(C), N,
                                    cur_stream()),
           "gmp_tp_gemm_x3_widen_f32");
  return C;
}

Tensor outer_sum_cols(const Tensor& A, const Tensor& B) {
  OpGuard g(A, "outer_sum_cols");
  f32(A, "A");
  f32(B, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0),
              "gmp.outer_sum_cols: A (K, m), B (K, n)");
  const int64_t K = A.size(0), m = A.size(1), n = B.size(1);
  Tensor C = at::empty({m, n}, A.options());
  const size_t ws_b = gmp_outer_sum_cols_workspace_size(K, m, n);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  check_rc(gmp_outer_sum_cols_f32(K, m, n, fp(A), m, fp(B), n, fp(C), n, ws.data_ptr(), ws_b,
                                  cur_stream()),
           "gmp_outer_sum_cols_f32");
  return C;
}

// ------------------------------------------------------------------ edge outer sums (K5)
// out[c] = sum_(e,x) A[e, 3c + x] v[e, x]  (A (K, 3C), v (K, 3); C = 16 or 48)
Tensor edge_xyz_dot(const Tensor& A_, const Tensor& v_) {
  OpGuard g(A_, "edge_xyz_dot");
  f32(A_, "A");
  f32(v_, "v");
  TORCH_CHECK(A_.dim() == 2 && A_.size(1) % 3 == 0, "gmp.edge_xyz_dot: A must be (K, 3C)");
  const int64_t K = A_.size(0), C = A_.size(1) / 3;
  numel(v_, K * 3, "v");
  Tensor A = A_.contiguous(), v = v_.contiguous();
  Tensor out = at::empty({C}, A.options());
  const size_t ws_b = gmp_edge_xyz_dot_workspace_size(K);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  const int rc = gmp_edge_xyz_dot_f32(K, C, fp(A), fp(v), fp(out), ws.data_ptr(), ws_b,
                                      cur_stream());
  if (rc == GMP_ERR_UNSUPPORTED)
    return (A.view({K, C, 3}) * v.view({K, 1, 3})).sum(at::IntArrayRef{0, 2});
  check_rc(rc, "gmp_edge_xyz_dot_f32");
  return out;
}

std::tuple<Tensor, Tensor> edge_outer_sum(const Tensor& A, const Tensor& B) {
  OpGuard g(A, "edge_outer_sum");
  f32(A, "A");
  f32(B, "B");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0),
              "gmp.edge_outer_sum: A (K, m), B (K, n)");
  const int64_t K = A.size(0), m = A.size(1), n = B.size(1);
  Tensor C = at::empty({m, n}, A.options()), cs = at::empty({m}, A.options());
  const size_t ws_b = gmp_edge_outer_sum_ex_workspace_size(K, m, n);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  const int rc = gmp_edge_outer_sum_ex_f32(K, m, n, fp(A), m, fp(B), n, -1, nullptr, nullptr,
                                           fp(C), n, fp(cs), ws.data_ptr(), ws_b, cur_stream());
  if (rc == GMP_ERR_UNSUPPORTED) {  // outside the tile buckets: the library GEMM on the device
    at::mm_out(C, A.t(), B);
    at::sum_out(cs, A, {0});
  } else {
    check_rc(rc, "gmp_edge_outer_sum_ex_f32");
  }
  return {C, cs};
}

// operand view usable by the strided outer-sum kernels: (K, m) f32 on the op's device, unit
// column stride, row stride a multiple of 4 floats, 16-byte aligned base
bool rows_view_ok(const Tensor& t) {
  return t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 4 == 0 &&
         reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
}
Tensor rows_view(const Tensor& t, const char* what) {
  on_device(t, what);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.dim() == 2, "gmp: ", what, " must be 2-D f32");
  return rows_view_ok(t) ? t : t.contiguous();
}
void out_view(const Tensor& C, int64_t m, int64_t n, const char* what) {
  on_device(C, what);
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 2 && C.stride(1) == 1,
              "gmp: ", what, " must be a 2-D f32 view with unit column stride");
  shape(C, {m, n}, what);
}

// act(B * w + b) rows as the edge outer sums' prologue computes them (act 0 relu, 1 silu)
Tensor act_rows(const Tensor& B, int64_t act, const optional<Tensor>& w,
                const optional<Tensor>& b) {
  if (act < 0) return B;
  Tensor y = B * w->view({1, -1}) + b->view({1, -1});
  return act == 0 ? at::relu(y) : at::silu(y);
}

// C[:] = A^T act(B) (+ colsum[:] = colsum(A)) into strided views: the split-plane / f32-MFMA
// kernels, or the library GEMM on the device where the shape is outside their buckets.
void edge_outer_sum_ex(const Tensor& A_, const Tensor& B_, Tensor C,
                          const optional<Tensor>& colsum, int64_t act, const optional<Tensor>& w,
                          const optional<Tensor>& b) {
  OpGuard g(A_, "edge_outer_sum_ex");
  Tensor A = rows_view(A_, "A"), B = rows_view(B_, "B");
  TORCH_CHECK(A.size(0) == B.size(0), "gmp.edge_outer_sum_ex: A (K, m), B (K, n)");
  const int64_t K = A.size(0), m = A.size(1), n = B.size(1);
  out_view(C, m, n, "C");
  TORCH_CHECK(act >= -1 && act <= 1, "gmp.edge_outer_sum_ex: act -1, 0 or 1");
  if (act >= 0) {
    TORCH_CHECK(w.has_value() && b.has_value(), "gmp.edge_outer_sum_ex: act needs w, b");
    f32(*w, "w");
    f32(*b, "b");
    numel(*w, n, "w");
    numel(*b, n, "b");
  }
  if (colsum.has_value()) {
    f32(*colsum, "colsum");
    numel(*colsum, m, "colsum");
  }
  const size_t ws_b = gmp_edge_outer_sum_ex_workspace_size(K, m, n);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  const int rc = gmp_edge_outer_sum_ex_f32(
      K, m, n, fp(A), A.stride(0), fp(B), B.stride(0), (int)act, act >= 0 ? fp(*w) : nullptr,
      act >= 0 ? fp(*b) : nullptr, C.data_ptr<float>(), C.stride(0),
      colsum.has_value() ? fp(*colsum) : nullptr, ws.data_ptr(), ws_b, cur_stream());
  if (rc != GMP_ERR_UNSUPPORTED) {
    check_rc(rc, "gmp_edge_outer_sum_ex_f32");
    return;
  }
  C.copy_(at::mm(A.t(), act_rows(B, act, w, b)));
  if (colsum.has_value()) colsum->copy_(A.sum(0));
}

// C[:] = A^T [B1 | B2] (+ colsum) in one pass over A where the split-plane kernel applies, else
// as two edge_outer_sum_ex products
void edge_outer_sum_ex2(const Tensor& A_, const Tensor& B1_, const Tensor& B2_, Tensor C,
                           const optional<Tensor>& colsum) {
  OpGuard g(A_, "edge_outer_sum_ex2");
  Tensor A = rows_view(A_, "A"), B1 = rows_view(B1_, "B1"), B2 = rows_view(B2_, "B2");
  TORCH_CHECK(A.size(0) == B1.size(0) && A.size(0) == B2.size(0),
              "gmp.edge_outer_sum_ex2: A (K, m), B1 (K, n1), B2 (K, n2)");
  const int64_t K = A.size(0), m = A.size(1), n1 = B1.size(1), n2 = B2.size(1);
  out_view(C, m, n1 + n2, "C");
  if (colsum.has_value()) {
    f32(*colsum, "colsum");
    numel(*colsum, m, "colsum");
  }
  const size_t ws_b = gmp_edge_outer_sum_rect_workspace_size(K, m, n1 + n2);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  const int rc = gmp_edge_outer_sum_ex2_f32(K, m, n1, n2, fp(A), A.stride(0), fp(B1),
                                            B1.stride(0), fp(B2), B2.stride(0),
                                            C.data_ptr<float>(), C.stride(0),
                                            colsum.has_value() ? fp(*colsum) : nullptr,
                                            ws.data_ptr(), ws_b, cur_stream());
  if (rc != GMP_ERR_UNSUPPORTED) {
    check_rc(rc, "gmp_edge_outer_sum_ex2_f32");
    return;
  }
  edge_outer_sum_ex(A, B1, C.narrow(1, 0, n1), colsum, -1, c10::nullopt, c10::nullopt);
  edge_outer_sum_ex(A, B2, C.narrow(1, n1, n2), c10::nullopt, -1, c10::nullopt, c10::nullopt);
}

// (A^T act(X w + b), colsum(A)) for the EGNN y1 / m operands rebuilt from x_hat; with amax (the
// max |A| device word) the HF two-plane form
std::tuple<Tensor, Tensor> edge_outer_sum_act(const Tensor& A, const Tensor& X, const Tensor& w,
                                              const Tensor& b, int64_t act,
                                              const optional<Tensor>& amax) {
  OpGuard g(A, "edge_outer_sum_act");
  f32(A, "A");
  f32(X, "X");
  f32(w, "w");
  f32(b, "b");
  TORCH_CHECK(A.dim() == 2 && A.sizes() == X.sizes() && A.size(1) == w.numel() &&
                  b.numel() == w.numel(),
              "gmp.edge_outer_sum_act: A, X (K, d), w, b (d)");
  TORCH_CHECK(act == 0 || act == 1, "gmp.edge_outer_sum_act: act 0 (relu) or 1 (silu)");
  const int64_t K = A.size(0), d = A.size(1);
  Tensor C = at::empty({d, d}, A.options()), cs = at::empty({d}, A.options());
  const size_t ws_b = gmp_edge_outer_sum_workspace_size(K, d);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, A.options().dtype(at::kByte));
  int rc;
  if (amax.has_value()) {
    i32(*amax, "amax");
    rc = gmp_edge_outer_sum_act_hf_f32(
        K, d, fp(A), fp(X), fp(w), fp(b), (int)act,
        reinterpret_cast<const uint32_t*>(amax->data_ptr<int32_t>()), fp(C), fp(cs),
        ws.data_ptr(), ws_b, cur_stream());
  } else {
    rc = gmp_edge_outer_sum_act_f32(K, d, fp(A), fp(X), fp(w), fp(b), (int)act, fp(C), fp(cs),
                                    ws.data_ptr(), ws_b, cur_stream());
  }
  if (rc == GMP_ERR_UNSUPPORTED) {
    C.copy_(at::mm(A.t(), act_rows(X, act, w, b)));
    cs.copy_(A.sum(0));
  } else {
    check_rc(rc, amax.has_value() ? "gmp_edge_outer_sum_act_hf_f32" : "gmp_edge_outer_sum_act_f32");
  }
  return {C, cs};
}

// ------------------------------------------------------------------ K5g GVP message GVPs
void gvp_w_checks(const std::vector<Tensor>& W, const std::vector<std::vector<int64_t>>& shp) {
  TORCH_CHECK(W.size() == shp.size(), "gmp.gvp: ", shp.size(), " weight tensors expected");
  for (size_t k = 0; k < W.size(); ++k) {
    f32(W[k], "gvp weight");
    shape(W[k], shp[k], "gvp weight");
  }
}
// gvp_layer weights: Ws (128, 144), bs (128), Wsv (16, 128), bsv (16), Wh (16, 16), Wv (16, 16)
const std::vector<std::vector<int64_t>> kGvpLayerW = {{128, 144}, {128}, {16, 128}, {16},
                                                      {16, 16}, {16, 16}};
// gvp_msg0 weights: We (128, 32), Wn (128, 48), b (128), Wv (16, 48), Wsv (16, 128), bsv (16),
// wev (48)
const std::vector<std::vector<int64_t>> kGvpMsg0W = {{128, 32}, {128, 48}, {128}, {16, 48},
                                                     {16, 128}, {16}, {48}};

int64_t gvp_rows(const Tensor& s, const Tensor& v) {
  f32(s, "s");
  f32(v, "v");
  TORCH_CHECK(s.dim() == 2 && s.size(1) == 128, "gmp.gvp_layer: s must be (E, 128)");
  TORCH_CHECK(v.numel() == s.size(0) * 48, "gmp.gvp_layer: v must be (E, 16, 3)");
  return s.size(0);
}

std::tuple<Tensor, Tensor> gvp_layer_fwd(const Tensor& s, const Tensor& v,
                                         const std::vector<Tensor>& W, bool relu) {
  OpGuard g(s, "gvp_layer_fwd");
  const int64_t E = gvp_rows(s, v);
  gvp_w_checks(W, kGvpLayerW);
  Tensor so = at::empty_like(s), vo = at::empty_like(v);
  check_rc(gmp_gvp_layer_fwd_f32(E, relu ? 1 : 0, fp(s), fp(v), fp(W[0]), fp(W[1]), fp(W[2]),
                                 fp(W[3]), fp(W[4]), fp(W[5]), fp(so), fp(vo), cur_stream()),
           "gmp_gvp_layer_fwd_f32");
  return {so, vo};
}

std::vector<Tensor> gvp_layer_bwd(const Tensor& s, const Tensor& v, const std::vector<Tensor>& W,
                                  const Tensor& ds, const Tensor& dv, bool relu, bool want_factors) {
  OpGuard g(s, "gvp_layer_bwd");
  const int64_t E = gvp_rows(s, v);
  gvp_w_checks(W, kGvpLayerW);
  f32(ds, "ds");
  f32(dv, "dv");
  shape(ds, s.sizes(), "ds");
  shape(dv, v.sizes(), "dv");
  auto o = fopt(s);
  Tensor ds_in = at::empty_like(s), dv_in = at::empty_like(v);
  // spre, vh: only when the caller forms dWsv / dWv from them (want_factors; see gmp.h)
  const int64_t Ef = want_factors ? E : 0;
  Tensor dspre = at::empty({E, 128}, o), spre = at::empty({Ef, 128}, o);
  Tensor dgate = at::empty({E, 16}, o), vn = at::empty({E, 16}, o);
  Tensor vh = at::empty({Ef, 48}, o), dvpre = at::empty({E, 48}, o), dvh = at::empty({E, 48}, o);
  check_rc(gmp_gvp_layer_bwd_f32(E, relu ? 1 : 0, fp(s), fp(v), fp(W[0]), fp(W[1]), fp(W[2]),
                                 fp(W[3]), fp(W[4]), fp(W[5]), fp(ds), fp(dv), fp(ds_in),
                                 fp(dv_in), fp(dspre), want_factors ? fp(spre) : nullptr, fp(dgate),
                                 fp(vn), want_factors ? fp(vh) : nullptr, fp(dvpre), fp(dvh), cur_stream()),
           "gmp_gvp_layer_bwd_f32");
  return {ds_in, dv_in, dspre, spre, dgate, vn, vh, dvpre, dvh};
}

// K15b: the EGNN node update's backward; vecs = [ln1_w, ln1_b, ln2_w, ln2_b]; returns dh, dm,
// dpre1, dpre2 and gb = [d ln1_w | d ln1_b | d ln2_w | d ln2_b] (4 d; partial rows summed in order)
std::vector<Tensor> egnn_node_bwd(const Tensor& g, const Tensor& xhat, const Tensor& rstd,
                                  const Tensor& W0, const Tensor& W3,
                                  const std::vector<Tensor>& vecs, int64_t act, bool residual) {
  OpGuard og(g, "egnn_node_bwd");
  f32(g, "grad_h");
  TORCH_CHECK(g.dim() == 2, "gmp.egnn_node_bwd: grad_h (N, d)");
  const int64_t N = g.size(0), d = g.size(1);
  f32(xhat, "xhat");
  f32(rstd, "rstd");
  shape(xhat, {2, N, d}, "xhat");
  shape(rstd, {2, N}, "rstd");
  f32(W0, "W0");
  f32(W3, "W3");
  shape(W0, {d, 2 * d}, "W0");
  shape(W3, {d, d}, "W3");
  TORCH_CHECK(vecs.size() == 4, "gmp.egnn_node_bwd: 4 LayerNorm vectors expected");
  for (const auto& v : vecs) {
    f32(v, "LayerNorm vector");
    numel(v, d, "LayerNorm vector");
  }
  auto o = g.options();
  Tensor dh = at::empty({N, d}, o), dm = at::empty({N, d}, o);
  Tensor dp1 = at::empty({N, d}, o), dp2 = at::empty({N, d}, o);
  Tensor part = at::empty({gmp_egnn_node_bwd_partial_rows(N), 4 * d}, o);
  check_rc(gmp_egnn_node_bwd_f32(N, d, (int)act, residual ? 1 : 0, fp(g), fp(xhat), fp(rstd),
                                 fp(W0), fp(W3), fp(vecs[0]), fp(vecs[1]), fp(vecs[2]),
                                 fp(vecs[3]), fp(dh), fp(dm), fp(dp1), fp(dp2), fp(part),
                                 cur_stream()),
           "gmp_egnn_node_bwd_f32");
  Tensor gb = N > 0 ? part.sum(0) : at::zeros({4 * d}, o);
  return {dh, dm, dp1, dp2, gb};
}

// K17 node feed-forward: W = [Wh1, Ws1, b1, Wv1, Wsv1, bsv1, Wh2, Ws2, b2, Wv2, Wsv2, bsv2]
const std::vector<std::vector<int64_t>> kGvpFFW = {{32, 16}, {512, 160}, {512}, {32, 32},
                                                   {32, 512}, {32}, {32, 32}, {128, 544},
                                                   {128}, {16, 32}, {16, 128}, {16}};

// returns s2, v2, gate1, B1 (N, 192), B2 (N, 576), B3 (N, 64), B4 (N, 128) (gmp.h)
std::vector<Tensor> gvp_ff_fwd(const Tensor& s, const Tensor& v, const std::vector<Tensor>& W) {
  OpGuard g(s, "gvp_ff_fwd");
  const int64_t N = gvp_rows(s, v);
  gvp_w_checks(W, kGvpFFW);
  auto o = fopt(s);
  Tensor so = at::empty_like(s), vo = at::empty_like(v), gate1 = at::empty({N, 32}, o);
  Tensor B1 = at::empty({N, 192}, o), B2 = at::empty({N, 576}, o);
  Tensor B3 = at::empty({N, 64}, o), B4 = at::empty({N, 128}, o);
  check_rc(gmp_gvp_ff_fwd_f32(N, fp(s), fp(v), fp(W[0]), fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]),
                              fp(W[5]), fp(W[6]), fp(W[7]), fp(W[8]), fp(W[9]), fp(W[10]),
                              fp(W[11]), fp(so), fp(vo), fp(gate1), fp(B1), fp(B2), fp(B3), fp(B4),
                              cur_stream()),
           "gmp_gvp_ff_fwd_f32");
  return {so, vo, gate1, B1, B2, B3, B4};
}

// returns ds, dv, A1 (N, 576), A2 (N, 192), A3 (N, 192), A4 (N, 192) (gmp.h)
std::vector<Tensor> gvp_ff_bwd(const Tensor& v, const std::vector<Tensor>& W, const Tensor& gate1,
                               const Tensor& B2, const Tensor& s2, const Tensor& ds,
                               const Tensor& dv) {
  OpGuard g(v, "gvp_ff_bwd");
  const int64_t N = gvp_rows(s2, v);
  gvp_w_checks(W, kGvpFFW);
  for (const Tensor* t : {&gate1, &B2, &ds, &dv}) f32(*t, "gvp_ff saved / grad");
  shape(gate1, {N, 32}, "gate1");
  shape(B2, {N, 576}, "B2");
  shape(ds, s2.sizes(), "ds");
  shape(dv, v.sizes(), "dv");
  auto o = fopt(v);
  Tensor ds_in = at::empty_like(s2), dv_in = at::empty_like(v);
  Tensor A1 = at::empty({N, 576}, o), A2 = at::empty({N, 192}, o);
  Tensor A3 = at::empty({N, 192}, o), A4 = at::empty({N, 192}, o);
  check_rc(gmp_gvp_ff_bwd_f32(N, fp(v), fp(gate1), fp(B2), fp(s2), fp(ds), fp(dv), fp(W[0]),
                              fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]), fp(W[6]),
                              fp(W[7]), fp(W[8]), fp(W[9]), fp(W[10]), fp(W[11]), fp(ds_in),
                              fp(dv_in), fp(A1), fp(A2), fp(A3), fp(A4), cur_stream()),
           "gmp_gvp_ff_bwd_f32");
  return {ds_in, dv_in, A1, A2, A3, A4};
}

// the last message GVP fused with the receivers' sum / mean: (N, 128), (N, 16, 3) node rows
std::tuple<Tensor, Tensor> gvp_layer_fwd_agg(const Tensor& s, const Tensor& v,
                                             const std::vector<Tensor>& W,
                                             const optional<Tensor>& perm, const Tensor& skey,
                                             const Tensor& rowptr, int64_t n_nodes,
                                             const std::string& reduce) {
  OpGuard g(s, "gvp_layer_fwd_agg");
  const int64_t E = gvp_rows(s, v);
  gvp_w_checks(W, kGvpLayerW);
  i64(skey, "skey");
  i64(rowptr, "rowptr");
  shape(skey, {E}, "skey");
  shape(rowptr, {n_nodes + 1}, "rowptr");
  if (perm.has_value() && perm->defined()) {
    i64(*perm, "perm");
    shape(*perm, {E}, "perm");
  }
  const int red = reduce_code(reduce);
  TORCH_CHECK(red == GMP_REDUCE_SUM || red == GMP_REDUCE_MEAN,
              "gmp.gvp_layer_fwd_agg: reduce must be sum or mean");
  auto o = fopt(s);
  Tensor sa = at::empty({n_nodes, 128}, o), va = at::empty({n_nodes, 16, 3}, o);
  const bool hp = perm.has_value() && perm->defined();
  check_rc(gmp_gvp_layer_fwd_agg_f32(E, n_nodes, red, hp ? perm->data_ptr<int64_t>() : nullptr,
                                     skey.data_ptr<int64_t>(), rowptr.data_ptr<int64_t>(), fp(s),
                                     fp(v), fp(W[0]), fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]),
                                     fp(W[5]), fp(sa), fp(va), cur_stream()),
           "gmp_gvp_layer_fwd_agg_f32");
  return {sa, va};
}

// the last message GVP's backward with the receivers' sum / mean backward in its loads: ds, dv
// are the aggregation's node gradients (N, 128), (N, 16, 3); index the receiver per edge,
// rowptr its CSR row pointer (counts for the mean)
std::vector<Tensor> gvp_layer_bwd_agg(const Tensor& s, const Tensor& v,
                                      const std::vector<Tensor>& W, const Tensor& ds,
                                      const Tensor& dv, const Tensor& index,
                                      const Tensor& rowptr, const std::string& reduce, bool relu,
                                      bool want_factors) {
  OpGuard g(s, "gvp_layer_bwd_agg");
  const int64_t E = gvp_rows(s, v);
  gvp_w_checks(W, kGvpLayerW);
  f32(ds, "ds");
  f32(dv, "dv");
  const int64_t N = ds.size(0);
  shape(ds, {N, 128}, "ds");
  shape(dv, {N, 16, 3}, "dv");
  i64(index, "index");
  i64(rowptr, "rowptr");
  shape(index, {E}, "index");
  shape(rowptr, {N + 1}, "rowptr");
  const int red = reduce_code(reduce);
  TORCH_CHECK(red == GMP_REDUCE_SUM || red == GMP_REDUCE_MEAN,
              "gmp.gvp_layer_bwd_agg: reduce must be sum or mean");
  auto o = fopt(s);
  Tensor ds_in = at::empty_like(s), dv_in = at::empty_like(v);
  // spre, vh: only when the caller forms dWsv / dWv from them (want_factors; see gmp.h)
  const int64_t Ef = want_factors ? E : 0;
  Tensor dspre = at::empty({E, 128}, o), spre = at::empty({Ef, 128}, o);
  Tensor dgate = at::empty({E, 16}, o), vn = at::empty({E, 16}, o);
  Tensor vh = at::empty({Ef, 48}, o), dvpre = at::empty({E, 48}, o), dvh = at::empty({E, 48}, o);
  check_rc(gmp_gvp_layer_bwd_agg_f32(E, N, red, index.data_ptr<int64_t>(),
                                     rowptr.data_ptr<int64_t>(), relu ? 1 : 0, fp(s), fp(v),
                                     fp(W[0]), fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]),
                                     fp(ds), fp(dv), fp(ds_in), fp(dv_in), fp(dspre),
                                     want_factors ? fp(spre) : nullptr, fp(dgate), fp(vn),
                                     want_factors ? fp(vh) : nullptr,
                                     fp(dvpre), fp(dvh), cur_stream()),
           "gmp_gvp_layer_bwd_agg_f32");
  return {ds_in, dv_in, dspre, spre, dgate, vn, vh, dvpre, dvh};
}

// K1e: the GVP-GNN edge embedding (LayerNorm((R, 1)) + GVP((R, 1), (so, 1))) over edge rows.
// W = [ln_w (R), ln_b (R), wh (1, 1), Ws (so, R + 1), bs (so), wv (1, 1), wsv (1, so), bsv (1)]
int64_t gvp_embed_checks(const Tensor& radial, const Tensor& unit, const std::vector<Tensor>& W) {
  f32(radial, "radial");
  f32(unit, "unit");
  TORCH_CHECK(radial.dim() == 2, "gmp.gvp_edge_embed: radial must be (E, R)");
  const int64_t E = radial.size(0), R = radial.size(1);
  numel(unit, E * 3, "unit");
  TORCH_CHECK(W.size() == 8, "gmp.gvp_edge_embed: 8 parameter tensors");
  for (const auto& w : W) f32(w, "W");
  const int64_t so = W[3].size(0);
  TORCH_CHECK(W[3].dim() == 2 && W[3].size(1) == R + 1, "gmp.gvp_edge_embed: Ws (so, R + 1)");
  numel(W[0], R, "ln_w");
  numel(W[1], R, "ln_b");
  numel(W[2], 1, "wh");
  numel(W[4], so, "bs");
  numel(W[5], 1, "wv");
  numel(W[6], so, "wsv");
  numel(W[7], 1, "bsv");
  return E;
}

std::tuple<Tensor, Tensor> gvp_edge_embed_fwd(const Tensor& radial, const Tensor& unit,
                                              const std::vector<Tensor>& W, double eps) {
  OpGuard g(radial, "gvp_edge_embed_fwd");
  const int64_t E = gvp_embed_checks(radial, unit, W);
  const int64_t so = W[3].size(0);
  auto o = fopt(radial);
  Tensor es = at::empty({E, so}, o), ev = at::empty({E, 1, 3}, o);
  check_rc(gmp_gvp_edge_embed_fwd_f32(E, radial.size(1), so, fp(radial), fp(unit), fp(W[0]),
                                      fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]), fp(W[6]),
                                      fp(W[7]), (float)eps, fp(es), fp(ev), cur_stream()),
           "gmp_gvp_edge_embed_fwd_f32");
  return {es, ev};
}

Tensor gvp_edge_embed_bwd(const Tensor& radial, const Tensor& unit, const std::vector<Tensor>& W,
                          double eps, const Tensor& des, const Tensor& dev) {
  OpGuard g(radial, "gvp_edge_embed_bwd");
  const int64_t E = gvp_embed_checks(radial, unit, W);
  const int64_t R = radial.size(1), so = W[3].size(0);
  f32(des, "grad_es");
  f32(dev, "grad_ev");
  shape(des, {E, so}, "grad_es");
  numel(dev, E * 3, "grad_ev");
  auto o = fopt(radial);
  Tensor grad = at::empty({2 * R + 3 + so * (R + 3)}, o);
  const size_t ws_b = gmp_gvp_edge_embed_bwd_workspace_size(E);
  Tensor ws = at::empty({(int64_t)ws_b + 1}, o.dtype(at::kByte));
  check_rc(gmp_gvp_edge_embed_bwd_f32(E, R, so, fp(radial), fp(unit), fp(W[0]), fp(W[1]),
                                      fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]), fp(W[6]), fp(W[7]),
                                      (float)eps, fp(des), fp(dev), fp(grad), ws.data_ptr(), ws_b,
                                      cur_stream()),
           "gmp_gvp_edge_embed_bwd_f32");
  return grad;
}

int64_t gvp_msg0_checks(const Tensor& send, const Tensor& recv, const Tensor& P, const Tensor& Q,
                        const Tensor& es, const Tensor& ev, const std::vector<Tensor>& W) {
  i64(send, "send");
  i64(recv, "recv");
  f32(P, "P");
  f32(Q, "Q");
  f32(es, "es");
  f32(ev, "ev");
  const int64_t E = send.numel();
  numel(recv, E, "recv");
  TORCH_CHECK(P.dim() == 2 && P.size(1) == 256, "gmp.gvp_msg0: P must be (N, 256)");
  shape(Q, {P.size(0), 288}, "Q");
  shape(es, {E, 32}, "es");
  shape(ev, {E, 3}, "ev");
  gvp_w_checks(W, kGvpMsg0W);
  return E;
}

std::tuple<Tensor, Tensor> gvp_msg0_fwd(const Tensor& send, const Tensor& recv, const Tensor& P,
                                        const Tensor& Q, const Tensor& es, const Tensor& ev,
                                        const std::vector<Tensor>& W) {
  OpGuard g(P, "gvp_msg0_fwd");
  const int64_t E = gvp_msg0_checks(send, recv, P, Q, es, ev, W);
  auto o = fopt(P);
  Tensor so = at::empty({E, 128}, o), vo = at::empty({E, 16, 3}, o);
  check_rc(gmp_gvp_msg0_fwd_f32(E, ip(send), ip(recv), fp(P), fp(Q), fp(es), fp(ev), fp(W[0]),
                                fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]), fp(W[6]),
                                fp(so), fp(vo), cur_stream()),
           "gmp_gvp_msg0_fwd_f32");
  return {so, vo};
}

std::vector<Tensor> gvp_msg0_bwd(const Tensor& send, const Tensor& recv, const Tensor& P,
                                 const Tensor& Q, const Tensor& es, const Tensor& ev,
                                 const std::vector<Tensor>& W, const Tensor& ds,
                                 const Tensor& dv, bool want_factors) {
  OpGuard g(P, "gvp_msg0_bwd");
  const int64_t E = gvp_msg0_checks(send, recv, P, Q, es, ev, W);
  f32(ds, "ds");
  f32(dv, "dv");
  shape(ds, {E, 128}, "ds");
  numel(dv, E * 48, "dv");
  auto o = fopt(P);
  const int64_t Ef = want_factors ? E : 0;  // spre / vh rows (optional, see gmp.h)
  Tensor dspre = at::empty({E, 128}, o), spre = at::empty({Ef, 128}, o);
  Tensor dgate = at::empty({E, 16}, o), vn = at::empty({E, 48}, o);
  Tensor vh = at::empty({Ef, 144}, o), dvh = at::empty({E, 144}, o);
  Tensor dvpre = at::empty({E, 48}, o), des = at::empty({E, 32}, o), dev = at::empty({E, 3}, o);
  check_rc(gmp_gvp_msg0_bwd_f32(E, ip(send), ip(recv), fp(P), fp(Q), fp(es), fp(ev), fp(W[0]),
                                fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]), fp(W[6]),
                                fp(ds), fp(dv), fp(dspre), want_factors ? fp(spre) : nullptr,
                                fp(dgate), fp(vn), want_factors ? fp(vh) : nullptr, fp(dvpre),
                                fp(dvh), fp(des), fp(dev), cur_stream()),
           "gmp_gvp_msg0_bwd_f32");
  return {dspre, spre, dgate, vn, vh, dvpre, dvh, des, dev};
}

// gvp_msg0_bwd walking the receiver-sorted edges, with the receiver-side sums S_i dspre,
// S_i dvh, S_i dgate, S_i dvpre reduced in the kernel (appended to the outputs)
std::vector<Tensor> gvp_msg0_bwd_agg(const Tensor& send, const Tensor& recv, const Tensor& P,
                                     const Tensor& Q, const Tensor& es, const Tensor& ev,
                                     const std::vector<Tensor>& W, const Tensor& ds,
                                     const Tensor& dv, const optional<Tensor>& perm,
                                     const Tensor& rowptr, int64_t n_nodes, bool want_factors) {
  OpGuard g(P, "gvp_msg0_bwd_agg");
  const int64_t E = gvp_msg0_checks(send, recv, P, Q, es, ev, W);
  f32(ds, "ds");
  f32(dv, "dv");
  shape(ds, {E, 128}, "ds");
  numel(dv, E * 48, "dv");
  i64(rowptr, "rowptr");
  shape(rowptr, {n_nodes + 1}, "rowptr");
  const bool hp = perm.has_value() && perm->defined();
  if (hp) {
    i64(*perm, "perm");
    shape(*perm, {E}, "perm");
  }
  auto o = fopt(P);
  const int64_t Ef = want_factors ? E : 0;
  Tensor dspre = at::empty({E, 128}, o), spre = at::empty({Ef, 128}, o);
  Tensor dgate = at::empty({E, 16}, o), vn = at::empty({E, 48}, o);
  Tensor vh = at::empty({Ef, 144}, o), dvh = at::empty({E, 144}, o);
  Tensor dvpre = at::empty({E, 48}, o), des = at::empty({E, 32}, o), dev = at::empty({E, 3}, o);
  Tensor dPb = at::empty({n_nodes, 128}, o), dQb = at::empty({n_nodes, 144}, o);
  Tensor sgr = at::empty({n_nodes, 16}, o), svr = at::empty({n_nodes, 48}, o);
  check_rc(gmp_gvp_msg0_bwd_agg_f32(E, n_nodes, ip(send), ip(recv),
                                    hp ? perm->data_ptr<int64_t>() : nullptr,
                                    rowptr.data_ptr<int64_t>(), fp(P), fp(Q), fp(es), fp(ev),
                                    fp(W[0]), fp(W[1]), fp(W[2]), fp(W[3]), fp(W[4]), fp(W[5]),
                                    fp(W[6]), fp(ds), fp(dv), fp(dspre),
                                    want_factors ? fp(spre) : nullptr, fp(dgate), fp(vn),
                                    want_factors ? fp(vh) : nullptr, fp(dvpre), fp(dvh), fp(des),
                                    fp(dev), fp(dPb), fp(dQb), fp(sgr), fp(svr), cur_stream()),
           "gmp_gvp_msg0_bwd_agg_f32");
  return {dspre, spre, dgate, vn, vh, dvpre, dvh, des, dev, dPb, dQb, sgr, svr};
}

// ------------------------------------------------------------------ Meta (shape) kernels
namespace meta {
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> csr_build(const Tensor& index, int64_t n_seg,
                                                             const optional<Tensor>& payload) {
  auto o = index.options();
  const int64_t n = index.numel();
  return {at::empty({n}, o), at::empty({n_seg + 1}, o), at::empty({n}, o),
          at::empty({payload.has_value() ? n : 0}, o), at::empty({1}, o.dtype(at::kInt))};
}
Tensor gather_rows(const Tensor& src, const Tensor& index) {
  return at::empty({index.numel(), src.size(1)}, src.options());
}
std::tuple<Tensor, Tensor> segment_reduce(const Tensor& src, const optional<Tensor>&,
                                          const Tensor& rowptr, int64_t n_seg,
                                          const std::string& reduce) {
  const bool mx = reduce_code(reduce) == GMP_REDUCE_MAX;
  return {at::empty({n_seg, src.size(1)}, src.options()),
          at::empty({mx ? n_seg : 0, src.size(1)}, rowptr.options())};
}
Tensor segment_reduce_bwd(const Tensor& grad_out, const Tensor&, const Tensor&, const std::string&,
                          const optional<Tensor>&, int64_t n_items) {
  return at::empty({n_items, grad_out.size(1)}, grad_out.options());
}
std::tuple<Tensor, Tensor, Tensor, Tensor> egnn_edge_fwd(const Tensor& AB, const Tensor& pos,
                                                         const Tensor&, const Tensor& recv,
                                                         const Tensor&, const std::vector<Tensor>&,
                                                         int64_t, bool, double, bool train,
                                                         int64_t xhat_planes) {
  const int64_t N = pos.size(0), E = recv.numel(), d = AB.size(1) / 2;
  auto o = AB.options();
  return {at::empty({N, d}, o), at::empty({N, 3}, o),
          at::empty({train ? xhat_planes : 0, E, d}, o), at::empty({train ? E : 0, 3}, o)};
}
Tensor egnn_node_image(const std::vector<Tensor>& W0s, const std::vector<Tensor>&,
                       const std::vector<optional<Tensor>>&) {
  const int64_t d = W0s[0].size(0);
  return at::empty({(int64_t)W0s.size(), (int64_t)gmp_egnn_node_image_bytes(d)},
                   W0s[0].options().dtype(at::kByte));
}
std::tuple<Tensor, Tensor, Tensor, Tensor> egnn_node_fwd(const Tensor& h, const Tensor&,
                                                         const std::vector<Tensor>&, const Tensor&,
                                                         bool with_ab, int64_t, bool, double,
                                                         bool train) {
  const int64_t N = h.size(0), d = h.size(1);
  auto o = h.options();
  return {at::empty({N, d}, o), at::empty({with_ab ? N : 0, 2 * d}, o),
          at::empty({train ? 2 : 0, N, d}, o), at::empty({train ? 2 : 0, N}, o)};
}
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor> egnn_edge_bwd(
    const Tensor& pos, const Tensor&, const Tensor& recv, const Tensor&,
    const std::vector<Tensor>&, int64_t, bool, const Tensor& xhat, const Tensor&, const Tensor&,
    const Tensor&, const optional<Tensor>&) {
  const int64_t N = pos.size(0), E = recv.numel(), d = xhat.size(2);
  auto o = pos.options();
  return {at::empty({N, d}, o), at::empty({N, 3}, o), at::empty({E, d}, o), at::empty({E, 3}, o),
          at::empty({E, d}, o), at::empty({E, d}, o),
          at::empty({gmp_egnn_edge_bwd_partials_rows(E, d), 8 * d + 1}, o)};
}
Tensor cfconv_aggregate(const Tensor& x, const Tensor&, const Tensor&, const Tensor&,
                        const Tensor&, int64_t n_seg, const optional<Tensor>&) {
  return at::empty({n_seg, x.size(1)}, x.options());
}
Tensor cfconv_wgrad(const Tensor&, const Tensor& gidx, const Tensor& x, const Tensor&,
                    const optional<Tensor>&) {
  return at::empty({gidx.numel(), x.size(1)}, x.options());
}
Tensor ssp_fwd(const Tensor& x, double) { return at::empty_like(x); }
Tensor ssp_bwd(const Tensor& x, const Tensor&) { return at::empty_like(x); }
std::tuple<Tensor, Tensor, Tensor> ln_act_fwd(const Tensor& x, const Tensor&, const Tensor&, double,
                                              int64_t) {
  return {at::empty_like(x), at::empty_like(x), at::empty({x.numel() / x.size(-1)}, x.options())};
}
std::tuple<Tensor, Tensor> ln_act_bwd(const Tensor&, const Tensor& xhat, const Tensor&,
                                      const Tensor&, const Tensor&, int64_t) {
  return {at::empty_like(xhat), at::empty({2 * xhat.size(-1)}, xhat.options())};
}
Tensor edge_xyz_dot(const Tensor& A, const Tensor&) {
  return at::empty({A.size(1) / 3}, A.options());
}
Tensor vec_norm_fwd(const Tensor& v) { return at::empty_like(v); }
Tensor vec_norm_bwd(const Tensor& v, const Tensor&) { return at::empty_like(v); }
Tensor xyz_norm_fwd(const Tensor& vh) { return at::empty({vh.size(0), vh.size(2)}, vh.options()); }
Tensor xyz_norm_bwd(const Tensor& vh, const Tensor&) { return at::empty_like(vh); }
std::tuple<Tensor, Tensor> edge_featurize(const Tensor& pos, const Tensor& ei,
                                          at::ArrayRef<double> w, double, double, double,
                                          int64_t lmax) {
  return {at::empty({ei.size(1), (lmax + 1) * (lmax + 1)}, pos.options()),
          at::empty({ei.size(1), (int64_t)w.size()}, pos.options())};
}
Tensor edge_featurize_bwd(const Tensor& pos, const Tensor& ei, at::ArrayRef<double>, double,
                          double, double, const optional<Tensor>&, const optional<Tensor>&,
                          int64_t) {
  return at::empty({ei.size(1), 3}, pos.options());
}
std::tuple<Tensor, Tensor> edge_featurize_gvp(const Tensor& pos, const Tensor& ei,
                                              at::ArrayRef<double> w, double, double, double) {
  return {at::empty({ei.size(1), (int64_t)w.size()}, pos.options()),
          at::empty({ei.size(1), 3}, pos.options())};
}
Tensor edge_featurize_gvp_bwd(const Tensor& pos, const Tensor& ei, at::ArrayRef<double>, double,
                              double, double, const optional<Tensor>&, const optional<Tensor>&) {
  return at::empty({ei.size(1), 3}, pos.options());
}
std::tuple<Tensor, Tensor, Tensor> schnet_featurize(const Tensor& pos, const Tensor& ei,
                                                    const Tensor& offsets, double, double) {
  const int64_t E = ei.size(1);
  return {at::empty({E}, pos.options()), at::empty({E, offsets.numel()}, pos.options()),
          at::empty({E}, pos.options())};
}
Tensor schnet_featurize_bwd(const Tensor& pos, const Tensor& ei, const Tensor&, double, double,
                            const optional<Tensor>&, const optional<Tensor>&,
                            const optional<Tensor>&) {
  return at::empty({ei.size(1), 3}, pos.options());
}
Tensor gate_fwd(const Tensor& x, const Tensor& out_map, double, double) {
  return at::empty({x.size(0), out_map.size(0)}, x.options());
}
Tensor gate_bwd(const Tensor& x, const Tensor&, const Tensor&, double, double) {
  return at::empty_like(x);
}
std::tuple<Tensor, Tensor, Tensor> irreps_bn_fwd(const Tensor& x, const Tensor&,
                                                 const Tensor& chan_col, const Tensor&,
                                                 const Tensor&, const optional<Tensor>&, Tensor,
                                                 Tensor, bool, double, double) {
  const int64_t nf = chan_col.size(0);
  return {at::empty_like(x), at::empty({nf}, x.options()), at::empty({nf}, x.options())};
}
std::tuple<Tensor, Tensor, Tensor> irreps_bn_bwd(const Tensor& x, const Tensor&, const Tensor&,
                                                 const Tensor& chan_col, const Tensor&,
                                                 const Tensor&, const Tensor&, const Tensor&,
                                                 bool, int64_t n_scalar) {
  return {at::empty_like(x), at::empty({chan_col.size(0)}, x.options()),
          at::empty({n_scalar}, x.options())};
}
Tensor symmetric_contraction_fwd(const Tensor& x, const Tensor&, int64_t rows, const Tensor&) {
  return at::empty({x.size(0), rows * x.size(1)}, x.options());
}
std::tuple<Tensor, Tensor> symmetric_contraction_bwd(const Tensor& x, const Tensor&, int64_t,
                                                     const Tensor& coef, const Tensor&) {
  return {at::empty_like(x), at::empty({gmp_sc_groups(x.size(0)), coef.size(0), x.size(1)},
                                       x.options())};
}
Tensor tp_edge_z(at::IntArrayRef desc, const Tensor&, const Tensor&, const Tensor& x,
                 const Tensor&, const Tensor&, const Tensor&, int64_t e0, int64_t e1) {
  return at::empty({(e1 - e0 + 1) * desc[5]}, x.options());
}
std::tuple<Tensor, Tensor> tp_edge_z_bwd(at::IntArrayRef desc, const Tensor&, const Tensor&,
                                         const Tensor& x, const Tensor&, const Tensor&,
                                         const Tensor&, int64_t e0, int64_t e1, const Tensor&) {
  return {at::empty({e1 - e0, desc[1]}, x.options()), at::empty({e1 - e0, desc[3]}, x.options())};
}
void tp_conv_fwd(int64_t, at::IntArrayRef, const Tensor&, const Tensor&, const Tensor&,
                 const Tensor&, const Tensor&, const Tensor&, const Tensor&, int64_t, int64_t,
                 Tensor) {}
Tensor tp_conv_bwd(int64_t, at::IntArrayRef, const Tensor&, const Tensor&, const Tensor&,
                   const Tensor&, const Tensor& W, const Tensor&, const Tensor&, const Tensor&,
                   int64_t, int64_t, const Tensor&, Tensor, Tensor) {
  return at::empty_like(W);
}
std::tuple<Tensor, Tensor> tp_node_outer(const Tensor& eoff, const Tensor&, const Tensor& A,
                                         int64_t w) {
  const int64_t c = eoff.numel() - 1;
  return {at::empty({c, w, A.size(1)}, A.options()), at::empty({c, w}, A.options())};
}
void tp_node_apply(const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&,
                   Tensor, Tensor) {}
Tensor tp_split_w2(const Tensor& W2, const Tensor&, int64_t, int64_t mul1, int64_t mo, bool fwd) {
  const int64_t K1 = mul1 * W2.size(1);
  return at::empty({fwd ? 3 * mo * (K1 + mul1) : 3 * K1 * mo}, W2.options().dtype(at::kShort));
}
void tp_gemm_x3(const Tensor&, int64_t, const optional<Tensor>&, int64_t, const Tensor&, int64_t,
                int64_t, Tensor, int64_t, int64_t, int64_t, int64_t, int64_t, bool) {}
Tensor tp_gemm_x3_widen(const Tensor& A, const Tensor&, int64_t N) {
  return at::empty({A.size(0), N}, A.options());
}
Tensor outer_sum_cols(const Tensor& A, const Tensor& B) {
  return at::empty({A.size(1), B.size(1)}, A.options());
}
std::tuple<Tensor, Tensor> edge_outer_sum(const Tensor& A, const Tensor& B) {
  return {at::empty({A.size(1), B.size(1)}, A.options()), at::empty({A.size(1)}, A.options())};
}
void edge_outer_sum_ex(const Tensor&, const Tensor&, Tensor, const optional<Tensor>&, int64_t,
                       const optional<Tensor>&, const optional<Tensor>&) {}
void edge_outer_sum_ex2(const Tensor&, const Tensor&, const Tensor&, Tensor,
                        const optional<Tensor>&) {}
std::tuple<Tensor, Tensor> edge_outer_sum_act(const Tensor& A, const Tensor&, const Tensor&,
                                              const Tensor&, int64_t, const optional<Tensor>&) {
  return {at::empty({A.size(1), A.size(1)}, A.options()), at::empty({A.size(1)}, A.options())};
}
std::tuple<Tensor, Tensor> gvp_layer_fwd(const Tensor& s, const Tensor& v,
                                         const std::vector<Tensor>&, bool) {
  return {at::empty_like(s), at::empty_like(v)};
}
std::vector<Tensor> egnn_node_bwd(const Tensor& g, const Tensor&, const Tensor&, const Tensor&,
                                  const Tensor&, const std::vector<Tensor>&, int64_t, bool) {
  const int64_t N = g.size(0), d = g.size(1);
  auto o = g.options();
  return {at::empty({N, d}, o), at::empty({N, d}, o), at::empty({N, d}, o),
          at::empty({N, d}, o), at::empty({4 * d}, o)};
}
std::vector<Tensor> gvp_ff_fwd(const Tensor& s, const Tensor& v, const std::vector<Tensor>&) {
  const int64_t N = s.size(0);
  auto o = s.options();
  return {at::empty_like(s),       at::empty_like(v),      at::empty({N, 32}, o),
          at::empty({N, 192}, o),  at::empty({N, 576}, o), at::empty({N, 64}, o),
          at::empty({N, 128}, o)};
}
std::vector<Tensor> gvp_ff_bwd(const Tensor& v, const std::vector<Tensor>&, const Tensor&,
                               const Tensor&, const Tensor& s2, const Tensor&, const Tensor&) {
  const int64_t N = s2.size(0);
  auto o = s2.options();
  return {at::empty_like(s2),     at::empty_like(v),      at::empty({N, 576}, o),
          at::empty({N, 192}, o), at::empty({N, 192}, o), at::empty({N, 192}, o)};
}

std::vector<Tensor> gvp_layer_bwd(const Tensor& s, const Tensor& v, const std::vector<Tensor>&,
                                  const Tensor&, const Tensor&, bool, bool want_factors) {
  const int64_t E = s.size(0);
  auto o = s.options();
  const int64_t Ef = want_factors ? E : 0;
  return {at::empty_like(s),      at::empty_like(v),     at::empty({E, 128}, o),
          at::empty({Ef, 128}, o), at::empty({E, 16}, o), at::empty({E, 16}, o),
          at::empty({Ef, 48}, o),  at::empty({E, 48}, o), at::empty({E, 48}, o)};
}
std::vector<Tensor> gvp_layer_bwd_agg(const Tensor& s, const Tensor& v,
                                      const std::vector<Tensor>& W, const Tensor& ds,
                                      const Tensor& dv, const Tensor&, const Tensor&,
                                      const std::string&, bool relu, bool want_factors) {
  return meta::gvp_layer_bwd(s, v, W, ds, dv, relu, want_factors);
}
std::tuple<Tensor, Tensor> gvp_layer_fwd_agg(const Tensor& s, const Tensor&,
                                             const std::vector<Tensor>&, const optional<Tensor>&,
                                             const Tensor&, const Tensor&, int64_t n_nodes,
                                             const std::string&) {
  return {at::empty({n_nodes, 128}, s.options()), at::empty({n_nodes, 16, 3}, s.options())};
}
std::tuple<Tensor, Tensor> gvp_edge_embed_fwd(const Tensor& radial, const Tensor&,
                                              const std::vector<Tensor>& W, double) {
  const int64_t E = radial.size(0);
  return {at::empty({E, W[3].size(0)}, radial.options()), at::empty({E, 1, 3}, radial.options())};
}
Tensor gvp_edge_embed_bwd(const Tensor& radial, const Tensor&, const std::vector<Tensor>& W,
                          double, const Tensor&, const Tensor&) {
  const int64_t R = radial.size(1), so = W[3].size(0);
  return at::empty({2 * R + 3 + so * (R + 3)}, radial.options());
}
std::tuple<Tensor, Tensor> gvp_msg0_fwd(const Tensor& send, const Tensor&, const Tensor& P,
                                        const Tensor&, const Tensor&, const Tensor&,
                                        const std::vector<Tensor>&) {
  const int64_t E = send.numel();
  return {at::empty({E, 128}, P.options()), at::empty({E, 16, 3}, P.options())};
}
std::vector<Tensor> gvp_msg0_bwd(const Tensor& send, const Tensor&, const Tensor& P,
                                 const Tensor&, const Tensor&, const Tensor&,
                                 const std::vector<Tensor>&, const Tensor&, const Tensor&,
                                 bool want_factors) {
  const int64_t E = send.numel(), Ef = want_factors ? E : 0;
  auto o = P.options();
  return {at::empty({E, 128}, o), at::empty({Ef, 128}, o), at::empty({E, 16}, o),
          at::empty({E, 48}, o),  at::empty({Ef, 144}, o), at::empty({E, 48}, o),
          at::empty({E, 144}, o), at::empty({E, 32}, o),  at::empty({E, 3}, o)};
}
std::vector<Tensor> gvp_msg0_bwd_agg(const Tensor& send, const Tensor& recv, const Tensor& P,
                                     const Tensor& Q, const Tensor& es, const Tensor& ev,
                                     const std::vector<Tensor>& W, const Tensor& ds,
                                     const Tensor& dv, const optional<Tensor>&, const Tensor&,
                                     int64_t n_nodes, bool want_factors) {
  auto out = meta::gvp_msg0_bwd(send, recv, P, Q, es, ev, W, ds, dv, want_factors);
  auto o = P.options();
  out.push_back(at::empty({n_nodes, 128}, o));
  out.push_back(at::empty({n_nodes, 144}, o));
  out.push_back(at::empty({n_nodes, 16}, o));
  out.push_back(at::empty({n_nodes, 48}, o));
  return out;
}
}  // namespace meta

}  // namespace

TORCH_LIBRARY(gmp, m) {
  m.def("csr_build(Tensor index, int n_seg, Tensor? payload=None) -> "
        "(Tensor perm, Tensor rowptr, Tensor sorted, Tensor payload_sorted, Tensor err)");
  m.def("gather_rows(Tensor src, Tensor index) -> Tensor");
  m.def("segment_reduce(Tensor src, Tensor? perm, Tensor rowptr, int n_seg, str reduce) -> "
        "(Tensor out, Tensor argmax)");
  m.def("segment_reduce_bwd(Tensor grad_out, Tensor index, Tensor rowptr, str reduce, "
        "Tensor? argmax, int n_items) -> Tensor");
  m.def("egnn_edge_fwd(Tensor AB, Tensor pos, Tensor rowptr, Tensor recv, Tensor send, "
        "Tensor[] params, int act, bool msg_mean, float eps, bool train, int xhat_planes=2) -> "
        "(Tensor m_aggr, Tensor pos_aggr, Tensor xhat, Tensor rstd)");
  m.def("egnn_node_image(Tensor[] W0s, Tensor[] W3s, Tensor?[] W1ns) -> Tensor");
  m.def("egnn_node_fwd(Tensor h, Tensor m_aggr, Tensor[] vecs, Tensor image, bool with_ab, "
        "int act, bool residual, float eps, bool train) -> (Tensor h_out, Tensor ab, "
        "Tensor xhat, Tensor rstd)");
  m.def("egnn_edge_bwd(Tensor pos, Tensor rowptr, Tensor recv, Tensor send, Tensor[] params, "
        "int act, bool msg_mean, Tensor xhat, Tensor rstd, Tensor g_m_aggr, Tensor g_pos_aggr, "
        "Tensor(a!)? amax=None) -> (Tensor dA, Tensor dpos_recv, "
        "Tensor dpre1, Tensor gdiff, Tensor dpre2, Tensor dpre3, Tensor partials)");
  m.def("cfconv_aggregate(Tensor x, Tensor xidx, Tensor w, Tensor perm, Tensor rowptr, "
        "int n_seg, Tensor? escale=None) -> Tensor");
  m.def("cfconv_wgrad(Tensor g, Tensor gidx, Tensor x, Tensor xidx, Tensor? escale=None) -> "
        "Tensor");
  m.def("ssp_fwd(Tensor x, float shift) -> Tensor");
  m.def("ssp_bwd(Tensor x, Tensor grad_y) -> Tensor");
  m.def("ln_act_fwd(Tensor x, Tensor gamma, Tensor beta, float eps, int act) -> "
        "(Tensor y, Tensor xhat, Tensor rstd)");
  m.def("ln_act_bwd(Tensor grad_y, Tensor xhat, Tensor rstd, Tensor gamma, Tensor beta, "
        "int act) -> (Tensor grad_x, Tensor grad_gamma_beta)");
  m.def("vec_norm_fwd(Tensor v) -> Tensor");
  m.def("vec_norm_bwd(Tensor v, Tensor grad_out) -> Tensor");
  m.def("xyz_norm_fwd(Tensor vh) -> Tensor");
  m.def("xyz_norm_bwd(Tensor vh, Tensor grad_out) -> Tensor");
  m.def("edge_featurize(Tensor pos, Tensor edge_index, float[] bessel_weights, float prefactor, "
        "float r_max, float p, int lmax=2) -> (Tensor sh, Tensor radial)");
  m.def("edge_featurize_bwd(Tensor pos, Tensor edge_index, float[] bessel_weights, "
        "float prefactor, float r_max, float p, Tensor? g_sh, Tensor? g_radial, int lmax=2) "
        "-> Tensor");
  m.def("edge_featurize_gvp(Tensor pos, Tensor edge_index, float[] bessel_weights, "
        "float prefactor, float r_max, float p) -> (Tensor radial, Tensor unit)");
  m.def("edge_featurize_gvp_bwd(Tensor pos, Tensor edge_index, float[] bessel_weights, "
        "float prefactor, float r_max, float p, Tensor? g_radial, Tensor? g_unit) -> Tensor");
  m.def("schnet_featurize(Tensor pos, Tensor edge_index, Tensor offsets, float coeff, "
        "float cutoff) -> (Tensor dist, Tensor rbf, Tensor cut)");
  m.def("schnet_featurize_bwd(Tensor pos, Tensor edge_index, Tensor offsets, float coeff, "
        "float cutoff, Tensor? g_dist, Tensor? g_rbf, Tensor? g_cut) -> Tensor");
  m.def("gate_fwd(Tensor x, Tensor out_map, float c_act, float c_gate) -> Tensor");
  m.def("gate_bwd(Tensor x, Tensor grad_y, Tensor in_map, float c_act, float c_gate) -> Tensor");
  m.def("irreps_bn_fwd(Tensor x, Tensor col_chan, Tensor chan_col, Tensor chan_info, "
        "Tensor weight, Tensor? bias, Tensor(a!) running_mean, Tensor(b!) running_var, "
        "bool training, float momentum, float eps) -> (Tensor y, Tensor shift, Tensor invstd)");
  m.def("irreps_bn_bwd(Tensor x, Tensor grad_y, Tensor col_chan, Tensor chan_col, "
        "Tensor chan_info, Tensor weight, Tensor shift, Tensor invstd, bool training, "
        "int n_scalar) -> (Tensor grad_x, Tensor grad_weight, Tensor grad_bias)");
  m.def("symmetric_contraction_fwd(Tensor x, Tensor plan, int rows, Tensor coef) -> Tensor");
  m.def("symmetric_contraction_bwd(Tensor x, Tensor plan, int rows, Tensor coef, Tensor gout) "
        "-> (Tensor dx, Tensor dcoef_partials)");
  m.def("tp_edge_z(int[] desc, Tensor paths, Tensor cg, Tensor x, Tensor sh, Tensor src_sorted, "
        "Tensor perm, int e0, int e1) -> Tensor");
  m.def("tp_edge_z_bwd(int[] desc, Tensor paths, Tensor cg, Tensor x, Tensor sh, "
        "Tensor src_sorted, Tensor perm, int e0, int e1, Tensor dz) -> "
        "(Tensor dx_edge, Tensor dY_edge)");
  m.def("tp_conv_fwd(int layout, int[] desc, Tensor paths, Tensor cg, Tensor x, Tensor sh, "
        "Tensor W, Tensor src_sorted, Tensor perm, int c0, int c1, Tensor(a!) msg) -> ()");
  m.def("tp_conv_bwd(int layout, int[] desc, Tensor paths, Tensor cg, Tensor x, Tensor sh, "
        "Tensor W, Tensor recv_sorted, Tensor src_sorted, Tensor perm, int c0, int c1, "
        "Tensor gout, Tensor(a!) dx_edge, Tensor(b!) dY_edge) -> Tensor dW");
  m.def("tp_node_outer(Tensor eoff, Tensor Z, Tensor A, int w) -> (Tensor S, Tensor Sb)");
  m.def("tp_node_apply(Tensor eoff, Tensor Z, Tensor A, Tensor T, Tensor Tb, Tensor(a!) dA, "
        "Tensor(b!) dZ) -> ()");
  m.def("tp_split_w2(Tensor W2, Tensor b2, int off, int mul1, int mul_out, bool fwd) -> Tensor");
  m.def("tp_gemm_x3(Tensor A1, int K1, Tensor? A2, int K2, Tensor Bp, int ldb, int N, "
        "Tensor(a!) C, int c_offset, int cgrp, int cldg, int cldr, int cldn, bool accumulate) "
        "-> ()");
  m.def("tp_gemm_x3_widen(Tensor A, Tensor Bp, int N) -> Tensor");
  m.def("outer_sum_cols(Tensor A, Tensor B) -> Tensor");
  m.def("edge_outer_sum(Tensor A, Tensor B) -> (Tensor C, Tensor colsum)");
  m.def("edge_outer_sum_ex(Tensor A, Tensor B, Tensor(a!) C, Tensor(b!)? colsum, int act, "
        "Tensor? w, Tensor? b) -> ()");
  m.def("edge_outer_sum_ex2(Tensor A, Tensor B1, Tensor B2, Tensor(a!) C, Tensor(b!)? colsum) "
        "-> ()");
  m.def("edge_outer_sum_act(Tensor A, Tensor X, Tensor w, Tensor b, int act, Tensor? amax=None) "
        "-> (Tensor C, Tensor colsum)");
  m.def("egnn_node_bwd(Tensor g, Tensor xhat, Tensor rstd, Tensor W0, Tensor W3, Tensor[] vecs, "
        "int act, bool residual) -> Tensor[]");
  m.def("gvp_ff_fwd(Tensor s, Tensor v, Tensor[] W) -> Tensor[]");
  m.def("gvp_ff_bwd(Tensor v, Tensor[] W, Tensor gate1, Tensor B2, Tensor s2, Tensor ds, "
        "Tensor dv) -> Tensor[]");
  m.def("gvp_layer_fwd(Tensor s, Tensor v, Tensor[] W, bool relu) -> (Tensor s_out, "
        "Tensor v_out)");
  m.def("gvp_layer_bwd(Tensor s, Tensor v, Tensor[] W, Tensor ds, Tensor dv, bool relu, "
        "bool want_factors=True) -> "
        "Tensor[]");
  m.def("gvp_layer_fwd_agg(Tensor s, Tensor v, Tensor[] W, Tensor? perm, Tensor skey, "
        "Tensor rowptr, int n_nodes, str reduce) -> (Tensor s_agg, Tensor v_agg)");
  m.def("gvp_layer_bwd_agg(Tensor s, Tensor v, Tensor[] W, Tensor ds, Tensor dv, Tensor index, "
        "Tensor rowptr, str reduce, bool relu, bool want_factors=True) -> Tensor[]");
  m.def("edge_xyz_dot(Tensor A, Tensor v) -> Tensor");
  m.def("gvp_edge_embed_fwd(Tensor radial, Tensor unit, Tensor[] W, float eps) "
        "-> (Tensor es, Tensor ev)");
  m.def("gvp_edge_embed_bwd(Tensor radial, Tensor unit, Tensor[] W, float eps, Tensor grad_es, "
        "Tensor grad_ev) -> Tensor");
  m.def("gvp_msg0_fwd(Tensor send, Tensor recv, Tensor P, Tensor Q, Tensor es, Tensor ev, "
        "Tensor[] W) -> (Tensor s_out, Tensor v_out)");
  m.def("gvp_msg0_bwd(Tensor send, Tensor recv, Tensor P, Tensor Q, Tensor es, Tensor ev, "
        "Tensor[] W, Tensor ds, Tensor dv, bool want_factors=True) -> Tensor[]");
  m.def("gvp_msg0_bwd_agg(Tensor send, Tensor recv, Tensor P, Tensor Q, Tensor es, Tensor ev, "
        "Tensor[] W, Tensor ds, Tensor dv, Tensor? perm, Tensor rowptr, int n_nodes, "
        "bool want_factors=True) -> Tensor[]");
}

#define GMP_IMPL(m, ns)                                                    \
  m.impl("csr_build", ns csr_build);                                      \
  m.impl("gather_rows", ns gather_rows);                                  \
  m.impl("segment_reduce", ns segment_reduce);                            \
  m.impl("segment_reduce_bwd", ns segment_reduce_bwd);                    \
  m.impl("egnn_edge_fwd", ns egnn_edge_fwd);                              \
  m.impl("egnn_node_fwd", ns egnn_node_fwd);                              \
  m.impl("egnn_node_image", ns egnn_node_image);                          \
  m.impl("egnn_edge_bwd", ns egnn_edge_bwd);                              \
  m.impl("cfconv_aggregate", ns cfconv_aggregate);                        \
  m.impl("cfconv_wgrad", ns cfconv_wgrad);                                \
  m.impl("ssp_fwd", ns ssp_fwd);                                          \
  m.impl("ssp_bwd", ns ssp_bwd);                                          \
  m.impl("ln_act_fwd", ns ln_act_fwd);                                    \
  m.impl("ln_act_bwd", ns ln_act_bwd);                                    \
  m.impl("edge_xyz_dot", ns edge_xyz_dot);                                \
  m.impl("gvp_edge_embed_fwd", ns gvp_edge_embed_fwd);                    \
  m.impl("gvp_edge_embed_bwd", ns gvp_edge_embed_bwd);                    \
  m.impl("vec_norm_fwd", ns vec_norm_fwd);                                \
  m.impl("vec_norm_bwd", ns vec_norm_bwd);                                \
  m.impl("xyz_norm_fwd", ns xyz_norm_fwd);                                \
  m.impl("xyz_norm_bwd", ns xyz_norm_bwd);                                \
  m.impl("edge_featurize", ns edge_featurize);                            \
  m.impl("edge_featurize_bwd", ns edge_featurize_bwd);                    \
  m.impl("edge_featurize_gvp", ns edge_featurize_gvp);                    \
  m.impl("edge_featurize_gvp_bwd", ns edge_featurize_gvp_bwd);            \
  m.impl("schnet_featurize", ns schnet_featurize);                        \
  m.impl("schnet_featurize_bwd", ns schnet_featurize_bwd);                \
  m.impl("gate_fwd", ns gate_fwd);                                        \
  m.impl("gate_bwd", ns gate_bwd);                                        \
  m.impl("irreps_bn_fwd", ns irreps_bn_fwd);                              \
  m.impl("irreps_bn_bwd", ns irreps_bn_bwd);                              \
  m.impl("symmetric_contraction_fwd", ns symmetric_contraction_fwd);      \
  m.impl("symmetric_contraction_bwd", ns symmetric_contraction_bwd);      \
  m.impl("tp_edge_z", ns tp_edge_z);                                      \
  m.impl("tp_edge_z_bwd", ns tp_edge_z_bwd);                              \
  m.impl("tp_conv_fwd", ns tp_conv_fwd);                                  \
  m.impl("tp_conv_bwd", ns tp_conv_bwd);                                  \
  m.impl("tp_node_outer", ns tp_node_outer);                              \
  m.impl("tp_node_apply", ns tp_node_apply);                              \
  m.impl("tp_split_w2", ns tp_split_w2);                                  \
  m.impl("tp_gemm_x3", ns tp_gemm_x3);                                    \
  m.impl("tp_gemm_x3_widen", ns tp_gemm_x3_widen);                        \
  m.impl("outer_sum_cols", ns outer_sum_cols);                            \
  m.impl("edge_outer_sum", ns edge_outer_sum);                            \
  m.impl("edge_outer_sum_ex", ns edge_outer_sum_ex);                      \
  m.impl("edge_outer_sum_ex2", ns edge_outer_sum_ex2);                    \
  m.impl("edge_outer_sum_act", ns edge_outer_sum_act);                    \
  m.impl("egnn_node_bwd", ns egnn_node_bwd);                              \
  m.impl("gvp_ff_fwd", ns gvp_ff_fwd);                                    \
  m.impl("gvp_ff_bwd", ns gvp_ff_bwd);                                    \
  m.impl("gvp_layer_fwd", ns gvp_layer_fwd);                              \
  m.impl("gvp_layer_bwd", ns gvp_layer_bwd);                              \
  m.impl("gvp_layer_bwd_agg", ns gvp_layer_bwd_agg);                      \
  m.impl("gvp_layer_fwd_agg", ns gvp_layer_fwd_agg);                      \
  m.impl("gvp_msg0_bwd_agg", ns gvp_msg0_bwd_agg);                        \
  m.impl("gvp_msg0_fwd", ns gvp_msg0_fwd);                                \
  m.impl("gvp_msg0_bwd", ns gvp_msg0_bwd);

TORCH_LIBRARY_IMPL(gmp, CUDA, m) { GMP_IMPL(m, ) }
// CPU tensors reach the same implementations, whose device guard rejects them with the
// boundary's message ("... must be HIP device tensors (no CPU fallback)"), as a RuntimeError
TORCH_LIBRARY_IMPL(gmp, CPU, m) { GMP_IMPL(m, ) }
TORCH_LIBRARY_IMPL(gmp, Meta, m) { GMP_IMPL(m, meta::) }
