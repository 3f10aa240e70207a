// Python bindings for the gfx950 kernels (module epfl_megatron_amd._C).
//
// Every op launches on PyTorch's current HIP stream (c10::hip), allocates
// outputs/workspaces through the caching allocator, validates shapes/dtypes
// on the host BEFORE launching (a mis-shaped launch on a shared MI355X node
// can fault the whole machine), and never synchronises.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ema::DT_F32;
    case at::kHalf: return ema::DT_F16;
    case at::kBFloat16: return ema::DT_BF16;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return -1;
}

void check_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}

void check_vec_aligned(const at::Tensor& t, const char* name) {
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name,
              " must be 16-byte aligned");
}

at::Tensor as_dtype(const at::Tensor& w, const at::Tensor& like) {
  return w.scalar_type() == like.scalar_type() ? w.contiguous() : w.to(like.scalar_type()).contiguous();
}

// ---------------------------------------------------------------- norms
// Optional residual: `res` (same shape/dtype as x) -> the norm input is
// s = x + res, returned as the last output; `dres` -> added into dx.
at::Tensor check_res(const c10::optional<at::Tensor>& r, const at::Tensor& x, const char* name) {
  if (!r.has_value() || !r->defined()) return at::Tensor();
  TORCH_CHECK(r->is_contiguous() && r->sizes() == x.sizes() && r->scalar_type() == x.scalar_type(),
              name, " must match x (contiguous, same shape and dtype)");
  check_vec_aligned(*r, name);
  return *r;
}

void check_norm_input(const at::Tensor& x, const at::Tensor& w) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "x must be contiguous [rows, H]");
  const int H = (int)x.size(1);
  const int dt = dtype_code(x);
  TORCH_CHECK(H % (16 / x.element_size()) == 0, "hidden size must be a multiple of 16 bytes");
  TORCH_CHECK(H <= ema::norm_max_hidden(dt), "hidden size too large for the norm kernel");
  TORCH_CHECK(w.numel() == H, "weight size mismatch");
  check_vec_aligned(x, "x");
}

std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps,
                                    const c10::optional<at::Tensor>& res) {
  check_norm_input(x, w);
  const int64_t rows = x.size(0);
  const int H = (int)x.size(1);
  const int dt = dtype_code(x);
  auto r = check_res(res, x, "res");
  auto wc = as_dtype(w, x);
  auto y = at::empty_like(x);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  at::Tensor sum = r.defined() ? at::empty_like(x) : x;
  if (rows > 0)
    ema::rmsnorm_fwd(x.data_ptr(), r.defined() ? r.data_ptr() : nullptr,
                     r.defined() ? sum.data_ptr() : nullptr, wc.data_ptr(), y.data_ptr(),
                     rstd.data_ptr<float>(), rows, H, (float)eps, dt, cur_stream());
  return {y, rstd, sum};
}

// fp32 main_grad a fused norm backward writes its parameter gradient into
static float* grad_acc_ptr(const c10::optional<at::Tensor>& g, int64_t H, const char* what) {
  if (!(g.has_value() && g->defined())) return nullptr;
  TORCH_CHECK(g->scalar_type() == at::kFloat && g->is_contiguous() && g->numel() == H && g->is_cuda(),
              what, " must be a contiguous fp32 CUDA tensor of hidden size");
  return g->data_ptr<float>();
}

std::vector<at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                    const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                                    const c10::optional<at::Tensor>& dw_acc, bool accumulate) {
  check_gpu(x, "x");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes(), "shape mismatch");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "dtype mismatch");
  TORCH_CHECK(rstd.numel() == x.size(0), "rstd size mismatch");
  const int64_t rows = x.size(0);
  const int H = (int)x.size(1);
  const int dt = dtype_code(x);
  auto dr = check_res(dres, x, "dres");
  auto wc = as_dtype(w, x);
  auto dx = at::empty_like(x);
  float* acc = grad_acc_ptr(dw_acc, H, "dw_acc");
  auto dw = acc ? at::Tensor() : at::empty({H}, x.options());
  const int P = ema::norm_bwd_workspace_rows(rows);
  auto part = at::empty({(int64_t)P, H}, x.options().dtype(at::kFloat));
  if (rows > 0) {
    ema::rmsnorm_bwd(dy.data_ptr(), x.data_ptr(), wc.data_ptr(), rstd.data_ptr<float>(),
                     dr.defined() ? dr.data_ptr() : nullptr, dx.data_ptr(),
                     part.data_ptr<float>(), acc ? nullptr : dw.data_ptr(), acc,
                     accumulate ? 1 : 0, rows, H, dt, cur_stream());
  } else if (acc) {
    if (!accumulate) dw_acc->zero_();
  } else {
    dw.zero_();
  }
  return {dx, acc ? at::Tensor() : dw.to(w.scalar_type())};
}

std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const at::Tensor& w,
                                      const c10::optional<at::Tensor>& b, double eps,
                                      const c10::optional<at::Tensor>& res) {
  check_norm_input(x, w);
  const int64_t rows = x.size(0);
  const int H = (int)x.size(1);
  const int dt = dtype_code(x);
  auto r = check_res(res, x, "res");
  auto wc = as_dtype(w, x);
  at::Tensor bc;
  if (b.has_value() && b->defined()) {
    TORCH_CHECK(b->numel() == H, "bias size mismatch");
    bc = as_dtype(*b, x);
  }
  auto y = at::empty_like(x);
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  at::Tensor sum = r.defined() ? at::empty_like(x) : x;
  if (rows > 0)
    ema::layernorm_fwd(x.data_ptr(), r.defined() ? r.data_ptr() : nullptr,
                       r.defined() ? sum.data_ptr() : nullptr, wc.data_ptr(),
                       bc.defined() ? bc.data_ptr() : nullptr, y.data_ptr(),
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, H, (float)eps, dt,
                       cur_stream());
  return {y, mean, rstd, sum};
}

std::vector<at::Tensor> layernorm_bwd(const at::Tensor& dy, const at::Tensor& x,
                                      const at::Tensor& w, const at::Tensor& mean,
                                      const at::Tensor& rstd,
                                      const c10::optional<at::Tensor>& dres,
                                      const c10::optional<at::Tensor>& dw_acc,
                                      const c10::optional<at::Tensor>& db_acc, bool accumulate_w,
                                      bool accumulate_b) {
  check_gpu(x, "x");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.sizes() == x.sizes(), "shape mismatch");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "dtype mismatch");
  TORCH_CHECK(rstd.numel() == x.size(0) && mean.numel() == x.size(0), "stats size mismatch");
  const int64_t rows = x.size(0);
  const int H = (int)x.size(1);
  const int dt = dtype_code(x);
  auto dr = check_res(dres, x, "dres");
  auto wc = as_dtype(w, x);
  auto dx = at::empty_like(x);
  float* wacc = grad_acc_ptr(dw_acc, H, "dw_acc");
  float* bacc = grad_acc_ptr(db_acc, H, "db_acc");
  auto dw = wacc ? at::Tensor() : at::empty({H}, x.options());
  auto db = bacc ? at::Tensor() : at::empty({H}, x.options());
  const int P = ema::norm_bwd_workspace_rows(rows);
  auto pw = at::empty({(int64_t)P, H}, x.options().dtype(at::kFloat));
  auto pb = at::empty({(int64_t)P, H}, x.options().dtype(at::kFloat));
  if (rows > 0) {
    ema::layernorm_bwd(dy.data_ptr(), x.data_ptr(), wc.data_ptr(), mean.data_ptr<float>(),
                       rstd.data_ptr<float>(), dr.defined() ? dr.data_ptr() : nullptr,
                       dx.data_ptr(), pw.data_ptr<float>(), pb.data_ptr<float>(),
                       wacc ? nullptr : dw.data_ptr(), bacc ? nullptr : db.data_ptr(), wacc, bacc,
                       accumulate_w ? 1 : 0, accumulate_b ? 1 : 0, rows, H, dt, cur_stream());
  } else {
    if (wacc) { if (!accumulate_w) dw_acc->zero_(); } else dw.zero_();
    if (bacc) { if (!accumulate_b) db_acc->zero_(); } else db.zero_();
  }
  return {dx, wacc ? at::Tensor() : dw.to(w.scalar_type()),
          bacc ? at::Tensor() : db.to(w.scalar_type())};
}

// ---------------------------------------------------------------- rope
void rope_qkv_inplace(at::Tensor qkv5, const at::Tensor& cos, const at::Tensor& sin,
                      const c10::optional<at::Tensor>& pos, int64_t offset, bool inverse,
                      bool k_only) {
  check_gpu(qkv5, "qkv");
  TORCH_CHECK(qkv5.dim() == 5, "qkv must be [s, b, ng, r+2, hd]");
  TORCH_CHECK(qkv5.stride(4) == 1, "head_dim must be contiguous");
  const int S = (int)qkv5.size(0), B = (int)qkv5.size(1), G = (int)qkv5.size(2);
  const int R = (int)qkv5.size(3) - 2, HD = (int)qkv5.size(4);
  TORCH_CHECK(HD % 8 == 0, "head_dim must be a multiple of 8");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.is_contiguous() && sin.is_contiguous(),
              "rope tables must be contiguous fp32");
  TORCH_CHECK(cos.size(1) == HD / 2, "rope table width must be head_dim / 2");
  TORCH_CHECK((qkv5.stride(3) % 8) == 0 && (qkv5.stride(2) % 8) == 0 && (qkv5.stride(1) % 8) == 0 &&
              (qkv5.stride(0) % 8) == 0, "qkv strides must keep 16-byte alignment");
  const int64_t max_pos = cos.size(0);
  const int64_t* pp = nullptr;
  int64_t psb = 0;
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->dim() == 2 && pos->size(0) == B &&
                pos->size(1) == S, "position_ids must be int64 [b, s]");
    TORCH_CHECK(pos->stride(1) == 1, "position_ids rows must be contiguous");
    pp = pos->data_ptr<int64_t>();
    psb = pos->stride(0);
  } else {
    TORCH_CHECK(offset + S <= max_pos, "rope table too short for sequence");
  }
  ema::rope_qkv_inplace(qkv5.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), pp, psb,
                        S, B, G, R, HD, qkv5.stride(0), qkv5.stride(1), qkv5.stride(2),
                        qkv5.stride(3), (int)offset, inverse ? 1 : 0, k_only ? 1 : 0,
                        dtype_code(qkv5), cur_stream());
}

// ---------------------------------------------------------------- activations
at::Tensor glu_fwd(const at::Tensor& x, int64_t kind) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
  const int64_t two_f = x.size(-1);
  TORCH_CHECK(two_f % 2 == 0, "GLU input width must be even");
  const int F = (int)(two_f / 2);
  TORCH_CHECK(F % (16 / x.element_size()) == 0, "GLU width must be a multiple of 16 bytes");
  const int64_t rows = x.numel() / two_f;
  auto sizes = x.sizes().vec();
  sizes.back() = F;
  auto y = at::empty(sizes, x.options());
  if (rows > 0) ema::glu_fwd(x.data_ptr(), y.data_ptr(), rows, F, (int)kind, dtype_code(x), cur_stream());
  return y;
}

at::Tensor glu_bwd(const at::Tensor& dy, const at::Tensor& x, int64_t kind) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous(), "inputs must be contiguous");
  const int64_t two_f = x.size(-1);
  const int F = (int)(two_f / 2);
  const int64_t rows = x.numel() / two_f;
  TORCH_CHECK(dy.numel() == rows * F, "dy shape mismatch");
  auto dx = at::empty_like(x);
  if (rows > 0)
    ema::glu_bwd(dy.data_ptr(), x.data_ptr(), dx.data_ptr(), rows, F, (int)kind, dtype_code(x),
                 cur_stream());
  return dx;
}

at::Tensor gelu_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& bias, int64_t approx) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
  const int F = (int)x.size(-1);
  TORCH_CHECK(F % (16 / x.element_size()) == 0, "width must be a multiple of 16 bytes");
  const int64_t rows = x.numel() / F;
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = as_dtype(*bias, x);
    TORCH_CHECK(b.numel() == F, "bias size mismatch");
  }
  auto y = at::empty_like(x);
  if (rows > 0)
    ema::gelu_fwd(x.data_ptr(), b.defined() ? b.data_ptr() : nullptr, y.data_ptr(), rows, F,
                  (int)approx, dtype_code(x), cur_stream());
  return y;
}

at::Tensor gelu_bwd(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& bias,
                    int64_t approx) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous() && dy.sizes() == x.sizes(), "shape mismatch");
  const int F = (int)x.size(-1);
  const int64_t rows = x.numel() / F;
  at::Tensor b;
  if (bias.has_value() && bias->defined()) b = as_dtype(*bias, x);
  auto dx = at::empty_like(x);
  if (rows > 0)
    ema::gelu_bwd(dy.data_ptr(), x.data_ptr(), b.defined() ? b.data_ptr() : nullptr,
                  dx.data_ptr(), rows, F, (int)approx, dtype_code(x), cur_stream());
  return dx;
}

// ---------------------------------------------------------------- cross entropy
void check_ce(const at::Tensor& z, const at::Tensor& t) {
  check_gpu(z, "logits");
  TORCH_CHECK(z.dim() == 2 && z.is_contiguous(), "logits must be contiguous [rows, V]");
  TORCH_CHECK(t.scalar_type() == at::kLong && t.is_contiguous() && t.numel() == z.size(0),
              "target must be int64 [rows]");
  TORCH_CHECK(z.size(1) % (16 / z.element_size()) == 0, "vocab shard must be a multiple of 16 bytes");
  check_vec_aligned(z, "logits");
}

std::vector<at::Tensor> ce_fwd_fused(const at::Tensor& z, const at::Tensor& t) {
  check_ce(z, t);
  const int64_t rows = z.size(0);
  auto loss = at::empty({rows}, z.options().dtype(at::kFloat));
  auto lse = at::empty({rows}, z.options().dtype(at::kFloat));
  if (rows > 0)
    ema::ce_fwd_fused(z.data_ptr(), t.data_ptr<int64_t>(), loss.data_ptr<float>(),
                      lse.data_ptr<float>(), rows, (int)z.size(1), dtype_code(z), cur_stream());
  return {loss, lse};
}

at::Tensor ce_row_max(const at::Tensor& z) {
  check_gpu(z, "logits");
  TORCH_CHECK(z.dim() == 2 && z.is_contiguous(), "logits must be contiguous [rows, V]");
  const int64_t rows = z.size(0);
  auto m = at::empty({rows}, z.options().dtype(at::kFloat));
  if (rows > 0) ema::ce_row_max(z.data_ptr(), m.data_ptr<float>(), rows, (int)z.size(1), dtype_code(z), cur_stream());
  return m;
}

std::vector<at::Tensor> ce_sumexp_target(const at::Tensor& z, const at::Tensor& t,
                                         const at::Tensor& rmax, int64_t vstart) {
  check_ce(z, t);
  const int64_t rows = z.size(0);
  auto se = at::empty({rows}, z.options().dtype(at::kFloat));
  auto tl = at::empty({rows}, z.options().dtype(at::kFloat));
  if (rows > 0)
    ema::ce_sumexp_target(z.data_ptr(), t.data_ptr<int64_t>(), rmax.data_ptr<float>(),
                          se.data_ptr<float>(), tl.data_ptr<float>(), rows, (int)z.size(1), vstart,
                          dtype_code(z), cur_stream());
  return {se, tl};
}

at::Tensor ce_bwd(const at::Tensor& z, const at::Tensor& t, const at::Tensor& lse,
                  const at::Tensor& dl, int64_t vstart) {
  check_ce(z, t);
  TORCH_CHECK(lse.numel() == z.size(0) && dl.numel() == z.size(0) && dl.scalar_type() == at::kFloat,
              "lse / dloss must be fp32 [rows]");
  auto dz = at::empty_like(z);
  const int64_t rows = z.size(0);
  if (rows > 0)
    ema::ce_bwd(z.data_ptr(), t.data_ptr<int64_t>(), lse.data_ptr<float>(),
                dl.contiguous().data_ptr<float>(), dz.data_ptr(), rows, (int)z.size(1), vstart,
                dtype_code(z), cur_stream());
  return dz;
}

// ---------------------------------------------------------------- softmax
at::Tensor softmax_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& mask, double scale,
                       int64_t mode) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "scores must be contiguous [b, np, sq, sk]");
  const int64_t B = x.size(0), NP = x.size(1);
  const int SQ = (int)x.size(2), SK = (int)x.size(3);
  TORCH_CHECK(SK <= 8192, "sk must be <= 8192");
  if (mode == 1) TORCH_CHECK(SQ == SK, "causal softmax expects square scores");
  const uint8_t* mp = nullptr;
  at::Tensor m;
  int64_t mask_bs = 0;
  if (mode == 2) {
    TORCH_CHECK(mask.has_value() && mask->defined(), "mask required for mode 2");
    // bool -> uint8 is a reinterpretation (same bytes), no copy
    m = mask->scalar_type() == at::kBool ? mask->view(at::kByte) : mask->to(at::kByte);
    m = m.contiguous();
    TORCH_CHECK(m.dim() == 4 && (m.size(0) == B || m.size(0) == 1) && m.size(1) == 1 &&
                    m.size(2) == SQ && m.size(3) == SK,
                "mask must be [b or 1, 1, sq, sk]");
    mask_bs = m.size(0) == 1 ? 0 : (int64_t)SQ * SK;  // a batch-broadcast mask is never expanded
    mp = m.data_ptr<uint8_t>();
  }
  auto y = at::empty_like(x);
  if (x.numel() > 0)
    ema::softmax_fwd(x.data_ptr(), mp, mask_bs, y.data_ptr(), B, NP, SQ, SK, (float)scale,
                     (int)mode, dtype_code(x), cur_stream());
  return y;
}

at::Tensor softmax_bwd(const at::Tensor& dy, const at::Tensor& y, double scale) {
  check_gpu(y, "y");
  TORCH_CHECK(dy.is_contiguous() && y.is_contiguous() && dy.sizes() == y.sizes(), "shape mismatch");
  const int SK = (int)y.size(-1);
  const int64_t rows = y.numel() / SK;
  auto dx = at::empty_like(y);
  if (rows > 0) ema::softmax_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), rows, SK, (float)scale, dtype_code(y), cur_stream());
  return dx;
}

// ---------------------------------------------------------------- optimizer
void check_table(const at::Tensor& table) {
  check_gpu(table, "table");
  TORCH_CHECK(table.scalar_type() == at::kLong && table.dim() == 2 && table.size(1) == 4 &&
              table.is_contiguous(), "chunk table must be int64 [n, 4]");
}

at::Tensor chunked_sumsq(const at::Tensor& grad, const at::Tensor& table) {
  check_gpu(grad, "grad");
  check_table(table);
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.is_contiguous(), "grad must be fp32 flat");
  check_vec_aligned(grad, "grad");
  const int n = (int)table.size(0);
  auto part = at::empty({n}, grad.options());
  auto out = at::empty({}, grad.options());
  ema::chunked_sumsq(grad.data_ptr<float>(), table.data_ptr<int64_t>(), n, part.data_ptr<float>(),
                     out.data_ptr<float>(), cur_stream());
  return out;
}

void flat_adam(at::Tensor master, const c10::optional<at::Tensor>& model_out, const at::Tensor& grad,
               at::Tensor m, at::Tensor v, const at::Tensor& table, std::vector<double> lrs,
               std::vector<double> wds, double beta1, double beta2, double eps, double bc1,
               double bc2, double grad_scale, bool adam_w_mode,
               const c10::optional<at::Tensor>& dev_state) {
  check_gpu(master, "master");
  check_table(table);
  for (const at::Tensor* t : {&master, &m, &v}) {
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "fp32 flat state expected");
    TORCH_CHECK(t->numel() == master.numel(), "state size mismatch");
    check_vec_aligned(*t, "state");
  }
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.is_contiguous(), "grad must be fp32 flat");
  check_vec_aligned(grad, "grad");
  TORCH_CHECK(lrs.size() == wds.size() && lrs.size() <= 8, "at most 8 param groups");
  ema::AdamArgs a{};
  for (size_t i = 0; i < lrs.size(); ++i) {
    a.lr[i] = (float)lrs[i];
    a.wd[i] = (float)wds[i];
  }
  a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.bc1 = (float)bc1; a.bc2 = (float)bc2; a.grad_scale = (float)grad_scale;
  a.adam_w_mode = adam_w_mode ? 1 : 0;
  a.dev_state = nullptr;
  if (dev_state.has_value() && dev_state->defined()) {
    check_gpu(*dev_state, "dev_state");
    TORCH_CHECK(dev_state->scalar_type() == at::kFloat && dev_state->numel() >= 3 &&
                dev_state->is_contiguous(), "dev_state must be fp32 [>=3]");
    a.dev_state = dev_state->data_ptr<float>();
  }
  void* mo = nullptr;
  int mdt = ema::DT_F32;
  if (model_out.has_value() && model_out->defined()) {
    TORCH_CHECK(model_out->is_contiguous() && model_out->numel() == grad.numel(),
                "model buffer must match the grad buffer layout");
    check_vec_aligned(*model_out, "model params");
    mo = model_out->data_ptr();
    mdt = dtype_code(*model_out);
  }
  ema::flat_adam(master.data_ptr<float>(), mo, mdt, grad.data_ptr<float>(), m.data_ptr<float>(),
                 v.data_ptr<float>(), table.data_ptr<int64_t>(), (int)table.size(0), a, cur_stream());
}

void opt_prep(const at::Tensor& norm_sq, const c10::optional<at::Tensor>& inv_scale, double clip,
              at::Tensor st) {
  check_gpu(norm_sq, "norm_sq");
  check_gpu(st, "st");
  TORCH_CHECK(norm_sq.scalar_type() == at::kFloat && norm_sq.numel() == 1, "norm_sq: fp32 scalar");
  TORCH_CHECK(st.scalar_type() == at::kFloat && st.numel() == 4 && st.is_contiguous(),
              "st: fp32 [4]");
  const float* inv = nullptr;
  if (inv_scale.has_value() && inv_scale->defined()) {
    check_gpu(*inv_scale, "inv_scale");
    TORCH_CHECK(inv_scale->scalar_type() == at::kFloat && inv_scale->numel() == 1,
                "inv_scale: fp32 scalar");
    inv = inv_scale->data_ptr<float>();
  }
  ema::opt_prep(norm_sq.data_ptr<float>(), inv, (float)clip, st.data_ptr<float>(), cur_stream());
}

// ---------------------------------------------------------------- attention
// Diagnostics: a uint64 buffer of 8 stamps per attention workgroup, attached
// to every following launch until cleared (scripts/fa_stamps.py).
// The buffer is kept referenced while attached (no use-after-free) and its
// length travels with the pointer: a workgroup whose 8 stamps would not fit
// writes none.
static at::Tensor g_fa_stamps_buf;
void fa_set_stamps(const c10::optional<at::Tensor>& buf) {
  if (buf.has_value() && buf->defined()) {
    TORCH_CHECK(buf->scalar_type() == at::kLong && buf->is_contiguous() && buf->is_cuda(),
                "stamps: contiguous int64 device buffer");
    g_fa_stamps_buf = *buf;
  } else {
    g_fa_stamps_buf = at::Tensor();
  }
}

ema::AttnParams make_attn(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                          const at::Tensor& out, const at::Tensor& lse, int64_t b, int64_t sq,
                          int64_t sk, int64_t nq, int64_t nkv, int64_t hd,
                          const std::vector<int64_t>& qs, const std::vector<int64_t>& ks,
                          const std::vector<int64_t>& vs, const std::vector<int64_t>& os,
                          bool causal, double scale, bool lse_view = false) {
  TORCH_CHECK(qs.size() == 4 && ks.size() == 3 && vs.size() == 3 && os.size() == 3, "bad strides");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type() &&
              q.scalar_type() == out.scalar_type(), "q/k/v/out dtype mismatch");
  TORCH_CHECK(ema::flash_attn_supported((int)hd, dtype_code(q)), "flash attention supports bf16/fp16 "
              "with head_dim 64 or 128 (got ", hd, ")");
  TORCH_CHECK(nkv > 0 && nq % nkv == 0, "nq must be a multiple of nkv");
  TORCH_CHECK(sq > 0 && sk > 0 && b > 0, "empty attention");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == b * nq * sq &&
                  (lse_view || lse.is_contiguous()),
              "lse must be fp32 [b, nq, sq]");
  for (int64_t s : qs) TORCH_CHECK(s % 8 == 0, "q strides must keep 16-byte alignment");
  for (int64_t s : ks) TORCH_CHECK(s % 8 == 0, "k strides must keep 16-byte alignment");
  for (int64_t s : vs) TORCH_CHECK(s % 8 == 0, "v strides must keep 16-byte alignment");
  for (int64_t s : os) TORCH_CHECK(s % 4 == 0, "o strides must keep 8-byte alignment");
  for (const at::Tensor* t : {&q, &k, &v}) check_vec_aligned(*t, "q/k/v");
  // Every address the kernel can form must lie inside its tensor's storage.
  auto span = [](int64_t b, int64_t s, int64_t n, int64_t sb, int64_t ss, int64_t sn, int64_t hd) {
    return (b - 1) * sb + (s - 1) * ss + (n - 1) * sn + hd;
  };
  const int64_t r = nq / nkv;
  const int64_t qspan = (b - 1) * qs[0] + (sq - 1) * qs[1] + (nkv - 1) * qs[2] + (r - 1) * qs[3] + hd;
  TORCH_CHECK(q.storage_offset() + qspan <= (int64_t)(q.storage().nbytes() / q.element_size()),
              "q strides exceed storage");
  TORCH_CHECK(k.storage_offset() + span(b, sk, nkv, ks[0], ks[1], ks[2], hd) <=
              (int64_t)(k.storage().nbytes() / k.element_size()), "k strides exceed storage");
  TORCH_CHECK(v.storage_offset() + span(b, sk, nkv, vs[0], vs[1], vs[2], hd) <=
              (int64_t)(v.storage().nbytes() / v.element_size()), "v strides exceed storage");
  TORCH_CHECK(out.storage_offset() + span(b, sq, nq, os[0], os[1], os[2], hd) <=
              (int64_t)(out.storage().nbytes() / out.element_size()), "out strides exceed storage");
  ema::AttnParams p{};
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr(); p.o = out.data_ptr();
  p.lse = lse.data_ptr<float>();
  p.b = (int)b; p.sq = (int)sq; p.sk = (int)sk; p.nq = (int)nq; p.nkv = (int)nkv; p.hd = (int)hd;
  p.q_sb = qs[0]; p.q_ss = qs[1]; p.q_sg = qs[2]; p.q_sh = qs[3];
  p.k_sb = ks[0]; p.k_ss = ks[1]; p.k_sg = ks[2];
  p.v_sb = vs[0]; p.v_ss = vs[1]; p.v_sg = vs[2];
  p.o_sb = os[0]; p.o_ss = os[1]; p.o_sh = os[2];
  p.causal = causal ? 1 : 0;
  p.coff = (int)(sk - sq);
  p.scale = (float)scale;
  p.lse_sb = nq * sq;
  p.lse_sh = sq;
  if (g_fa_stamps_buf.defined()) {
    p.stamps = reinterpret_cast<unsigned long long*>(g_fa_stamps_buf.data_ptr<int64_t>());
    p.stamps_n = g_fa_stamps_buf.numel();
  }
  return p;
}

// Fused RoPE tables for the attention kernels (see AttnParams): fp32
// [max_pos, hd/2] cos/sin, optional int64 [b, s] position ids (else the row
// index is the position, sq == sk).
static void set_rope(ema::AttnParams& p, const c10::optional<at::Tensor>& cos,
                     const c10::optional<at::Tensor>& sin, const c10::optional<at::Tensor>& pos) {
  if (!(cos.has_value() && cos->defined())) return;
  TORCH_CHECK(sin.has_value() && sin->defined(), "rope needs both cos and sin");
  TORCH_CHECK(cos->scalar_type() == at::kFloat && sin->scalar_type() == at::kFloat &&
              cos->is_contiguous() && sin->is_contiguous() && cos->dim() == 2 &&
              cos->sizes() == sin->sizes(), "rope tables must be contiguous fp32 [max_pos, hd/2]");
  TORCH_CHECK(cos->size(1) == p.hd / 2, "rope table width must be head_dim / 2");
  TORCH_CHECK(p.sq == p.sk, "fused rope needs sq == sk");
  check_gpu(*cos, "rope_cos");
  p.rope_cos = cos->data_ptr<float>();
  p.rope_sin = sin->data_ptr<float>();
  if (pos.has_value() && pos->defined()) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->dim() == 2 && pos->size(0) == p.b &&
                pos->size(1) == p.sq && pos->stride(1) == 1, "position_ids must be int64 [b, s]");
    p.rope_pos = pos->data_ptr<int64_t>();
    p.rope_pos_sb = pos->stride(0);
  } else {
    TORCH_CHECK(p.sq <= cos->size(0), "rope table too short for sequence");
  }
}

// Document mask (see AttnParams): contiguous int32 [2, b, s] = (doc_start, doc_end).
static void set_docs(ema::AttnParams& p, const c10::optional<at::Tensor>& docs) {
  if (!(docs.has_value() && docs->defined())) return;
  TORCH_CHECK(docs->scalar_type() == at::kInt && docs->is_contiguous() && docs->dim() == 3 &&
              docs->size(0) == 2 && docs->size(1) == p.b && docs->size(2) == p.sq,
              "doc bounds must be contiguous int32 [2, b, s]");
  TORCH_CHECK(p.sq == p.sk && p.causal, "document masking needs causal self-attention (sq == sk)");
  check_gpu(*docs, "doc bounds");
  p.doc_start = docs->data_ptr<int>();
  p.doc_end = p.doc_start + (int64_t)p.b * p.sq;
}

void flash_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor out,
                    at::Tensor lse, int64_t b, int64_t sq, int64_t sk, int64_t nq, int64_t nkv,
                    int64_t hd, std::vector<int64_t> qs, std::vector<int64_t> ks,
                    std::vector<int64_t> vs, std::vector<int64_t> os, bool causal, double scale,
                    const c10::optional<at::Tensor>& rope_cos,
                    const c10::optional<at::Tensor>& rope_sin,
                    const c10::optional<at::Tensor>& rope_pos,
                    const c10::optional<at::Tensor>& docs) {
  check_gpu(q, "q");
  auto p = make_attn(q, k, v, out, lse, b, sq, sk, nq, nkv, hd, qs, ks, vs, os, causal, scale);
  set_rope(p, rope_cos, rope_sin, rope_pos);
  set_docs(p, docs);
  ema::flash_attn_fwd(p, dtype_code(q), cur_stream());
}

// One ring-attention step (parallel/context.py): attention of q over this K/V
// chunk, log-sum-exp combined in place with the running fp32 output o32
// [b, sq, nq, hd] (any strides, head_dim contiguous) and lse [b, nq, sq] (any
// batch / head strides, rows contiguous); merge = false stores instead.
void flash_attn_fwd_merge(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                          at::Tensor o32, at::Tensor lse, int64_t b, int64_t sq, int64_t sk,
                          int64_t nq, int64_t nkv, int64_t hd, std::vector<int64_t> qs,
                          std::vector<int64_t> ks, std::vector<int64_t> vs, bool causal,
                          double scale, bool merge, const c10::optional<at::Tensor>& docs,
                          int64_t coff) {
  check_gpu(q, "q");
  TORCH_CHECK(o32.scalar_type() == at::kFloat && o32.dim() == 4 && o32.size(0) == b &&
                  o32.size(1) == sq && o32.size(2) == nq && o32.size(3) == hd && o32.stride(3) == 1 &&
                  o32.stride(1) % 4 == 0 && o32.stride(2) % 4 == 0 && o32.stride(0) % 4 == 0 &&
                  o32.data_ptr<float>() != nullptr && reinterpret_cast<uintptr_t>(o32.data_ptr()) % 16 == 0,
              "flash_attn_fwd_merge: o32 fp32 [b, sq, nq, hd], head_dim contiguous, 16-B aligned");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.dim() == 3 && lse.size(0) == b &&
                  lse.size(1) == nq && lse.size(2) == sq && lse.stride(2) == 1,
              "flash_attn_fwd_merge: lse fp32 [b, nq, sq], rows contiguous");
  TORCH_CHECK(o32.storage_offset() + (b - 1) * o32.stride(0) + (sq - 1) * o32.stride(1) +
                      (nq - 1) * o32.stride(2) + hd <=
                  (int64_t)(o32.storage().nbytes() / 4),
              "o32 strides exceed storage");
  // make_attn validates q / k / v; no 16-bit output is written in this mode
  // (q stands in for `out` in the validation only)
  TORCH_CHECK(q.dim() == 4 && q.size(0) == b && q.size(1) == sq, "flash_attn_fwd_merge: q [b, sq, ...]");
  std::vector<int64_t> os = {qs[0], qs[1], qs[3]};
  auto p = make_attn(q, k, v, q, lse, b, sq, sk, nq, nkv, hd, qs, ks, vs, os, causal, scale, true);
  p.o = nullptr;
  p.lse_sb = lse.stride(0);
  p.lse_sh = lse.stride(1);
  p.o32 = o32.data_ptr<float>();
  p.o32_sb = o32.stride(0);
  p.o32_ss = o32.stride(1);
  p.o32_sh = o32.stride(2);
  p.merge = merge ? 1 : 0;
  set_docs(p, docs);
  if (coff >= 0) {
    TORCH_CHECK(causal && coff >= sk - sq, "flash_attn_fwd_merge: coff needs the causal kernel");
    p.coff = (int)coff;
  }
  ema::flash_attn_fwd(p, dtype_code(q), cur_stream());
}

void flash_attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k,
                    const at::Tensor& v, const at::Tensor& out, const at::Tensor& lse, at::Tensor dq,
                    at::Tensor dk, at::Tensor dv, int64_t b, int64_t sq, int64_t sk, int64_t nq,
                    int64_t nkv, int64_t hd, std::vector<int64_t> qs, std::vector<int64_t> ks,
                    std::vector<int64_t> vs, std::vector<int64_t> os, bool causal, double scale,
                    const c10::optional<at::Tensor>& rope_cos,
                    const c10::optional<at::Tensor>& rope_sin,
                    const c10::optional<at::Tensor>& rope_pos,
                    const c10::optional<at::Tensor>& docs, int64_t coff) {
  check_gpu(q, "q");
  auto f = make_attn(q, k, v, out, lse, b, sq, sk, nq, nkv, hd, qs, ks, vs, os, causal, scale);
  set_rope(f, rope_cos, rope_sin, rope_pos);
  set_docs(f, docs);
  if (coff >= 0) {
    TORCH_CHECK(causal && coff >= sk - sq, "flash_attn_bwd: coff needs the causal kernel");
    f.coff = (int)coff;
  }
  TORCH_CHECK(dout.scalar_type() == q.scalar_type(), "dout dtype mismatch");
  TORCH_CHECK(dout.stride(-1) == 1, "dout head_dim must be contiguous");
  ema::AttnBwdParams p{};
  p.f = f;
  p.dout = dout.data_ptr();
  p.dq = dq.data_ptr();
  p.dk = dk.data_ptr();
  p.dv = dv.data_ptr();
  auto rowc = at::empty({2 * b * nq * sq}, q.options().dtype(at::kFloat));
  p.ndelta = rowc.data_ptr<float>();
  p.lse2 = p.ndelta + b * nq * sq;
  p.kv_split = ema::flash_attn_kv_split((int)b, (int)sk, (int)nq, (int)nkv);
  at::Tensor ws;
  if (p.kv_split > 1) {
    ws = at::empty({(int64_t)p.kv_split * b * nkv * sk * 2 * hd}, q.options().dtype(at::kFloat));
    p.dkv_ws = ws.data_ptr<float>();
  }
  ema::flash_attn_bwd(p, dtype_code(q), cur_stream());
}

// ---------------------------------------------------------------- skinny GEMM (decode)
bool skinny_gemm_supported(int64_t M, int64_t N, int64_t K) {
  return ema::skinny_gemm_supported(M, N, K);
}

// x [M, K] @ w[N, K]^T -> [M, N]
at::Tensor skinny_gemm(const at::Tensor& x, const at::Tensor& w, bool packed) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "skinny_gemm: shapes");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "skinny_gemm: contiguous operands");
  TORCH_CHECK(x.scalar_type() == w.scalar_type(), "skinny_gemm: dtype mismatch");
  const int dt = dtype_code(x);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16, "skinny_gemm: bf16/fp16 only");
  const int64_t M = x.size(0), N = w.size(0), K = x.size(1);
  TORCH_CHECK(ema::skinny_gemm_supported(M, N, K), "skinny_gemm: unsupported shape");
  check_vec_aligned(x, "x");
  check_vec_aligned(w, "w");
  TORCH_CHECK(!packed || K % 256 == 0, "skinny_gemm: packed weights need K % 256 == 0");
  auto y = at::empty({M, N}, x.options());
  ema::SkinnyArgs p{};
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.y = y.data_ptr();
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.ldy = N;
  p.packed = packed ? 1 : 0;
  ema::skinny_gemm_ex(p, 0, dt, cur_stream());
  return y;
}

// Fused decode projections (csrc/skinny_gemm.hip).  x [M, K] (M <= 16),
// w [N, K] (GLU: [2F, K]); norm_w: RMSNorm of x in the prologue; epi:
// 0 plain, 1 residual add (res [M, N]), 2 GLU (-> [M, F]),
// 3 QKV (-> q [M, nq * hd]; k / v written into the cache slot).
static ema::SkinnyArgs skinny_args(const at::Tensor& x, const at::Tensor& w,
                                   const c10::optional<at::Tensor>& norm_w, double eps,
                                   bool packed) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "skinny: shapes");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "skinny: contiguous operands");
  TORCH_CHECK(x.scalar_type() == w.scalar_type(), "skinny: dtype mismatch");
  const int dt = dtype_code(x);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16, "skinny: bf16/fp16 only");
  check_vec_aligned(x, "x");
  check_vec_aligned(w, "w");
  ema::SkinnyArgs p{};
  p.x = x.data_ptr();
  p.w = w.data_ptr();
  p.M = (int)x.size(0);
  p.K = (int)x.size(1);
  TORCH_CHECK(!packed || p.K % 256 == 0, "skinny: packed weights need K % 256 == 0");
  p.packed = packed ? 1 : 0;
  if (norm_w) {
    TORCH_CHECK(norm_w->is_cuda() && norm_w->is_contiguous() && norm_w->numel() == p.K &&
                norm_w->scalar_type() == x.scalar_type(), "skinny: norm weight must be [K], x dtype");
    p.norm_w = norm_w->data_ptr();
    p.eps = (float)eps;
  }
  return p;
}

at::Tensor skinny_norm_gemm(const at::Tensor& x, const at::Tensor& w,
                            const c10::optional<at::Tensor>& norm_w, double eps,
                            const c10::optional<at::Tensor>& res, bool packed) {
  auto p = skinny_args(x, w, norm_w, eps, packed);
  const int64_t N = w.size(0);
  TORCH_CHECK(ema::skinny_gemm_supported(p.M, N, p.K), "skinny: unsupported shape");
  auto y = at::empty({p.M, N}, x.options());
  p.N = (int)N;
  p.y = y.data_ptr();
  p.ldy = N;
  int epi = 0;
  if (res) {
    TORCH_CHECK(res->is_cuda() && res->scalar_type() == x.scalar_type() && res->dim() == 2 &&
                res->size(0) == p.M && res->size(1) == N && res->stride(1) == 1 &&
                res->stride(0) % 8 == 0, "skinny: residual must be [M, N] rows of the x dtype");
    check_vec_aligned(*res, "res");
    p.res = res->data_ptr();
    p.ldr = res->stride(0);
    epi = 1;
  }
  ema::skinny_gemm_ex(p, epi, dtype_code(x), cur_stream());
  return y;
}

at::Tensor skinny_norm_glu(const at::Tensor& x, const at::Tensor& w1,
                           const c10::optional<at::Tensor>& norm_w, double eps, int64_t kind,
                           bool packed, int64_t packed_tail) {
  auto p = skinny_args(x, w1, norm_w, eps, packed);
  const int64_t F = w1.size(0) / 2;
  TORCH_CHECK(w1.size(0) == 2 * F && F % 8 == 0 &&
              ema::skinny_gemm_supported(p.M, 2 * F, p.K), "skinny glu: unsupported shape");
  TORCH_CHECK(!packed || packed_tail == ema::skinny_glu_half_tail(F, p.K, norm_w.has_value(), p.M),
              "skinny glu: weight packed for another half-unit tail (skinny_glu_half_tail)");
  auto y = at::empty({p.M, F}, x.options());
  p.N = (int)F;
  p.y = y.data_ptr();
  p.ldy = F;
  p.act = (int)kind;
  ema::skinny_gemm_ex(p, 2, dtype_code(x), cur_stream());
  return y;
}


// qkv decode projection: returns the rotated q [M, ng * r * hd]; k / v rows go
// to kcache / vcache [L, B, ng, hd] (views at the batch offset) at the slot
// `slot_t` (int64 device scalar) or `slot`.
at::Tensor skinny_qkv_rope_cache(const at::Tensor& x, const at::Tensor& w,
                                 const c10::optional<at::Tensor>& norm_w, double eps, int64_t ng,
                                 int64_t r, int64_t hd, const at::Tensor& cos,
                                 const at::Tensor& sin, const at::Tensor& pos, at::Tensor kcache,
                                 at::Tensor vcache, const c10::optional<at::Tensor>& slot_t,
                                 int64_t slot, bool packed) {
  auto p = skinny_args(x, w, norm_w, eps, packed);
  const int64_t N = w.size(0);
  TORCH_CHECK(N == ng * (r + 2) * hd && hd % 8 == 0, "skinny qkv: w rows != ng * (r + 2) * hd");
  TORCH_CHECK(ema::skinny_gemm_supported(p.M, N, p.K), "skinny qkv: unsupported shape");
  TORCH_CHECK(cos.is_cuda() && sin.is_cuda() && cos.scalar_type() == at::kFloat &&
              sin.scalar_type() == at::kFloat && cos.is_contiguous() && sin.is_contiguous() &&
              cos.size(-1) == hd / 2, "skinny qkv: rope tables fp32 [max_pos, hd/2]");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kLong && pos.size(0) == p.M,
              "skinny qkv: pos int64 with one row per token");
  for (const at::Tensor* c : {&kcache, &vcache}) {
    TORCH_CHECK(c->is_cuda() && c->scalar_type() == x.scalar_type() && c->dim() == 4 &&
                c->size(1) >= p.M && c->size(2) == ng && c->size(3) == hd && c->stride(3) == 1 &&
                c->stride(2) == hd, "skinny qkv: caches [L, B, ng, hd] with packed heads");
  }
  TORCH_CHECK(kcache.stride(0) == vcache.stride(0) && kcache.stride(1) == vcache.stride(1),
              "skinny qkv: k / v cache strides differ");
  if (slot_t) {
    TORCH_CHECK(slot_t->is_cuda() && slot_t->scalar_type() == at::kLong, "skinny qkv: slot int64");
    p.slot_ptr = slot_t->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(slot >= 0 && slot < kcache.size(0), "skinny qkv: slot out of range");
    p.slot = slot;
  }
  auto q = at::empty({p.M, ng * r * hd}, x.options());
  p.N = (int)N;
  p.y = q.data_ptr();
  p.ldy = ng * r * hd;
  p.r = (int)r;
  p.hd = (int)hd;
  p.cos = cos.data_ptr<float>();
  p.sin = sin.data_ptr<float>();
  p.pos = pos.data_ptr<int64_t>();
  p.pos_sb = pos.stride(0);
  p.kcache = kcache.data_ptr();
  p.vcache = vcache.data_ptr();
  p.c_ss = kcache.stride(0);
  p.c_sb = kcache.stride(1);
  ema::skinny_gemm_ex(p, 3, dtype_code(x), cur_stream());
  return q;
}

// ---------------------------------------------------------------- decode attention
// q [b, 1, nq, hd] (strides qs = (sb, ss, sg, sh)), k/v caches [b, sk, nkv, hd]
// (strides (sb, ss, sg)), out [b, 1, nq, hd] (strides (sb, ss, sh)).
void flash_decode(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor out,
                  int64_t b, int64_t sk, int64_t nq, int64_t nkv, int64_t hd,
                  std::vector<int64_t> qs, std::vector<int64_t> ks, std::vector<int64_t> vs,
                  std::vector<int64_t> os, double scale, const c10::optional<at::Tensor>& kv_len,
                  int64_t kpw) {
  check_gpu(q, "q");
  if (kv_len) {
    TORCH_CHECK(kv_len->is_cuda() && kv_len->scalar_type() == at::kInt && kv_len->numel() >= 1,
                "kv_len must be a device int32 tensor");
    TORCH_CHECK(kv_len->device() == q.device(), "kv_len on another device");
  }
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type() &&
              out.scalar_type() == q.scalar_type(), "q/k/v/out dtype mismatch");
  TORCH_CHECK(ema::flash_attn_supported((int)hd, dtype_code(q)), "decode attention supports "
              "bf16/fp16 with head_dim 64 or 128");
  TORCH_CHECK(nkv > 0 && nq % nkv == 0 && b > 0 && sk > 0, "bad decode shape");
  TORCH_CHECK(q.stride(-1) == 1 && k.stride(-1) == 1 && v.stride(-1) == 1 && out.stride(-1) == 1,
              "head_dim must be contiguous");
  for (int64_t s : ks) TORCH_CHECK(s % 8 == 0, "k strides must keep 16-byte alignment");
  TORCH_CHECK(qs[0] % 8 == 0 && qs[2] % 8 == 0 && qs[3] % 8 == 0,
              "q strides must keep 16-byte alignment");
  for (const at::Tensor* t : {&q, &k, &v}) check_vec_aligned(*t, "q/k/v");
  auto span = [](int64_t b, int64_t s, int64_t n, int64_t sb, int64_t ss, int64_t sn, int64_t hd) {
    return (b - 1) * sb + (s - 1) * ss + (n - 1) * sn + hd;
  };
  TORCH_CHECK(k.storage_offset() + span(b, sk, nkv, ks[0], ks[1], ks[2], hd) <=
              (int64_t)(k.storage().nbytes() / k.element_size()), "k strides exceed storage");
  TORCH_CHECK(v.storage_offset() + span(b, sk, nkv, vs[0], vs[1], vs[2], hd) <=
              (int64_t)(v.storage().nbytes() / v.element_size()), "v strides exceed storage");
  ema::DecodeParams p{};
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr(); p.o = out.data_ptr();
  p.b = (int)b; p.sk = (int)sk; p.nq = (int)nq; p.nkv = (int)nkv; p.hd = (int)hd;
  p.q_sb = qs[0]; p.q_sg = qs[2]; p.q_sh = qs[3];
  p.k_sb = ks[0]; p.k_ss = ks[1]; p.k_sg = ks[2];
  p.v_sb = vs[0]; p.v_ss = vs[1]; p.v_sg = vs[2];
  p.o_sb = os[0]; p.o_sh = os[2];
  p.scale = (float)scale;
  p.kv_len = kv_len ? kv_len->data_ptr<int>() : nullptr;
  // keys per wave: auto (the largest of 64 / 16 / 8 whose grid covers the chip) or forced (A/B)
  if (kpw <= 0) kpw = ema::flash_decode_kpw((int)b, (int)sk, (int)nq, (int)nkv);
  TORCH_CHECK(kpw == 8 || kpw == 16 || kpw == 64, "decode attention: kpw must be 8, 16 or 64");
  p.kpw = (int)kpw;
  const int64_t ns = ema::flash_decode_splits((int)sk, (int)kpw);
  auto ws = at::empty({b * nq * ns * (hd + 2)}, q.options().dtype(at::kFloat));
  p.ws_o = ws.data_ptr<float>();
  p.ws_ml = p.ws_o + b * nq * ns * hd;
  // arrival counters: zeroed once, re-armed by the kernel; one buffer per
  // device that only grows (a hipGraph-captured step keeps its pointer: the
  // eager warm-up before capture sizes it)
  static std::vector<at::Tensor> counters;
  const int dev = q.get_device();
  if ((int)counters.size() <= dev) counters.resize(dev + 1);
  const int64_t nc = ema::flash_decode_counters((int)b, (int)nq, (int)nkv);
  if (!counters[dev].defined() || counters[dev].numel() < nc)
    counters[dev] = at::zeros({std::max<int64_t>(nc, 4096)}, q.options().dtype(at::kInt));
  p.counters = reinterpret_cast<unsigned*>(counters[dev].data_ptr<int>());
  ema::flash_decode(p, dtype_code(q), cur_stream());
}

// ---------------------------------------------------------------- greedy decode tail
// logits [b, V] (a view: rows 16-B aligned, last dim contiguous); tokens /
// pos int64 with b contiguous elements, history int64 [b, H] rows contiguous,
// step_idx / slot int64 [1], kv_len int32 [1], counter int32 [1] (zeroed once).
void greedy_tail(const at::Tensor& logits, at::Tensor tokens, at::Tensor history,
                 at::Tensor step_idx, at::Tensor pos, at::Tensor slot, at::Tensor kv_len,
                 at::Tensor counter) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "greedy_tail: logits [b, V], V contiguous");
  const int dt = dtype_code(logits);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16 || dt == ema::DT_F32, "greedy_tail: dtype");
  const int64_t b = logits.size(0), V = logits.size(1);
  TORCH_CHECK(b >= 1 && V >= 1 && V < (1ll << 31), "greedy_tail: shape");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0 &&
                  (logits.stride(0) * logits.element_size()) % 16 == 0,
              "greedy_tail: logits rows must be 16-byte aligned");
  for (const at::Tensor* t : {&tokens, &history, &step_idx, &pos, &slot})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong, "greedy_tail: int64 state tensors");
  TORCH_CHECK(kv_len.is_cuda() && kv_len.scalar_type() == at::kInt && kv_len.numel() >= 1 &&
                  counter.is_cuda() && counter.scalar_type() == at::kInt && counter.numel() >= 1,
              "greedy_tail: kv_len / counter int32");
  TORCH_CHECK(tokens.is_contiguous() && tokens.numel() == b && pos.is_contiguous() &&
                  pos.numel() == b && history.dim() == 2 && history.size(0) == b &&
                  history.stride(1) == 1 && step_idx.numel() >= 1 && slot.numel() >= 1,
              "greedy_tail: tokens / pos [b], history [b, H]");
  ema::greedy_tail(logits.data_ptr(), logits.stride(0), (int)V, (int)b, dt,
                   tokens.data_ptr<int64_t>(), history.data_ptr<int64_t>(), history.stride(0),
                   step_idx.data_ptr<int64_t>(), pos.data_ptr<int64_t>(), slot.data_ptr<int64_t>(),
                   kv_len.data_ptr<int>(), reinterpret_cast<unsigned*>(counter.data_ptr<int>()),
                   cur_stream());
}

// ---------------------------------------------------------------- bias-dropout-add
at::Tensor bias_dropout_add_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& x2,
                                const c10::optional<at::Tensor>& bias, const at::Tensor& res,
                                double p, int64_t seed, int64_t offset) {
  check_gpu(x, "x");
  check_gpu(res, "residual");
  TORCH_CHECK(x.is_contiguous() && res.is_contiguous(), "x / residual must be contiguous");
  TORCH_CHECK(x.sizes() == res.sizes() && x.scalar_type() == res.scalar_type(), "x / residual mismatch");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "bf16/fp16 only");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout probability must be in [0, 1)");
  const int64_t h = x.size(-1);
  TORCH_CHECK(h % 8 == 0 && x.numel() % 8 == 0, "hidden size must be a multiple of 8");
  const void* x2p = nullptr;
  if (x2.has_value() && x2->defined()) {
    TORCH_CHECK(x2->sizes() == x.sizes() && x2->is_contiguous() &&
                x2->scalar_type() == x.scalar_type(), "x2 must match x");
    check_vec_aligned(*x2, "x2");
    x2p = x2->data_ptr();
  }
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() == h && bias->is_contiguous() && bias->scalar_type() == x.scalar_type(),
                "bias must be [h] of x's dtype");
    check_vec_aligned(*bias, "bias");
    bp = bias->data_ptr();
  }
  auto out = at::empty_like(x);
  check_vec_aligned(x, "x");
  check_vec_aligned(res, "residual");
  check_vec_aligned(out, "out");
  if (x.numel() > 0)
    ema::bias_dropout_add_fwd(x.data_ptr(), x2p, bp, res.data_ptr(), out.data_ptr(), x.numel(), h,
                              (float)p, (uint64_t)seed, (uint64_t)offset, dtype_code(x), cur_stream());
  return out;
}

at::Tensor bias_dropout_add_bwd(const at::Tensor& dout, double p, int64_t seed, int64_t offset) {
  check_gpu(dout, "dout");
  TORCH_CHECK(dout.is_contiguous() && dout.numel() % 8 == 0, "dout must be contiguous, numel % 8 == 0");
  TORCH_CHECK(p > 0.0 && p < 1.0, "dropout probability must be in (0, 1)");
  auto dx = at::empty_like(dout);
  check_vec_aligned(dout, "dout");
  if (dout.numel() > 0)
    ema::bias_dropout_add_bwd(dout.data_ptr(), dx.data_ptr(), dout.numel(), (float)p, (uint64_t)seed,
                              (uint64_t)offset, dtype_code(dout), cur_stream());
  return dx;
}

// ---------------------------------------------------------------- wgrad GEMM
bool wgrad_supported(int64_t M, int64_t N, int64_t K) { return ema::wgrad_supported(M, N, K); }

// main_grad[N,K] (+)= dy[M,N]^T x[M,K]; x_map = [rows, n1, s1, s2]: dY's token
// q pairs with X row ((q / rows) % n1) * s1 + ((q / rows) / n1) * s2 + q % rows
void wgrad_gemm(const at::Tensor& dy, const at::Tensor& x, at::Tensor g, bool accumulate,
                std::vector<int64_t> x_map) {
  check_gpu(dy, "dy");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && g.dim() == 2, "wgrad_gemm: 2-D operands");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && g.is_contiguous(),
              "wgrad_gemm: contiguous operands required");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && g.scalar_type() == at::kFloat,
              "wgrad_gemm: dy/x same 16-bit dtype, g fp32");
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(g.size(0) == N && g.size(1) == K, "wgrad_gemm: shape mismatch");
  ema::TokMap xm;
  if (x_map.empty()) {
    TORCH_CHECK(x.size(0) == M, "wgrad_gemm: shape mismatch");
  } else {
    TORCH_CHECK(x_map.size() == 4, "wgrad_gemm: x_map = [rows, n1, s1, s2]");
    const int64_t R = x_map[0], n1 = x_map[1], s1 = x_map[2], s2 = x_map[3];
    TORCH_CHECK(R > 0 && R % 32 == 0 && n1 > 0 && s1 >= 0 && s2 >= 0 && M % (R * n1) == 0,
                "wgrad_gemm: x_map rows must be a positive multiple of 32 dividing M / n1");
    const int64_t n2 = M / (R * n1);
    TORCH_CHECK((n1 - 1) * s1 + (n2 - 1) * s2 + R <= x.size(0),
                "wgrad_gemm: x_map reaches past the rows of x");
    xm.rows = (int)R;
    xm.n1 = (int)n1;
    xm.s1 = s1;
    xm.s2 = s2;
  }
  TORCH_CHECK(ema::wgrad_supported(M, N, K), "wgrad_gemm: unsupported shape");
  const int dt = dtype_code(dy);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16, "wgrad_gemm: bf16/fp16 only");
  // split-K over tokens where whole tiles leave CUs idle (fp32 partials from
  // the caching allocator, ordered reduce)
  const int64_t wsf = ema::wgrad_workspace_floats(M, N, K);
  at::Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, g.options());
  ema::wgrad_gemm(dy.data_ptr(), x.data_ptr(), g.data_ptr<float>(), M, N, K, accumulate, dt,
                  cur_stream(), wsf > 0 ? ws.data_ptr<float>() : nullptr, xm);
}

// (main_tiles, tail_lin0, tail_tiles, nsplit) of a wgrad shape
std::vector<int64_t> wgrad_plan(int64_t M, int64_t N, int64_t K) {
  const ema::WgradPlan p = ema::wgrad_plan(M, N, K);
  return {p.main_tiles, p.tail_lin0, p.tail_tiles, p.nsplit};
}


// ---------------------------------------------------------------- NT GEMM
// 2-D, row stride multiple of 8 elements, unit column stride, 16-B aligned
static void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) % 8 == 0,
              name, ": 2-D with unit column stride and row stride % 8 == 0 required");
  check_vec_aligned(t, name);
}

bool gemm_nt_supported(const at::Tensor& a, const at::Tensor& b) {
  if (!a.is_cuda() || a.dim() != 2 || b.dim() != 2 || a.stride(1) != 1 || b.stride(1) != 1)
    return false;
  if (a.scalar_type() != b.scalar_type() ||
      (a.scalar_type() != at::kBFloat16 && a.scalar_type() != at::kHalf))
    return false;
  if (reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(b.data_ptr()) % 16)
    return false;
  return a.size(1) == b.size(1) &&
         ema::gemm_nt_supported(a.size(0), b.size(0), a.size(1), a.stride(0), b.stride(0), b.size(0));
}

// Row-group remap from Python: (rows, stride, offset) or rows == 0.  The host
// checks that every physical row of the remapped logical rows [0, M) lies in
// [0, phys_rows) BEFORE launching.
ema::RowMap row_map(const std::vector<int64_t>& m, int64_t M, int64_t phys_rows, const char* what) {
  ema::RowMap r;
  if (m.empty() || m[0] == 0) {
    TORCH_CHECK(M <= phys_rows, what, ": ", M, " logical rows but ", phys_rows, " physical");
    return r;
  }
  TORCH_CHECK(m.size() == 3 && m[0] > 0 && m[1] >= m[0] && m[2] >= 0 && m[0] < (1LL << 31) &&
              M < (1LL << 31), what, ": row map must be (rows > 0, stride >= rows, offset >= 0)");
  r.rows = (int)m[0];
  r.stride = m[1];
  r.offset = m[2];
  const int64_t last = ((M - 1) / m[0]) * m[1] + m[2] + (M - 1) % m[0];
  TORCH_CHECK(m[2] + std::min<int64_t>(m[0], M) - 1 <= last && last < phys_rows, what,
              ": remapped rows exceed the operand (last row ", last, ", ", phys_rows, " rows)");
  return r;
}

// c[M,N] = a[M,K] b[N,K]^T (c allocated unless given).  a_map: logical A row
// q is row map(q) of `a` (M = m if given, else a.size(0)); c_map: output row q
// goes to row map(q) of `out`.
at::Tensor gemm_nt(const at::Tensor& a, const at::Tensor& b, c10::optional<at::Tensor> out,
                   std::vector<int64_t> a_map, std::vector<int64_t> c_map, int64_t m) {
  check_gpu(a, "a");
  check_rows(a, "a");
  check_rows(b, "b");
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "gemm_nt: a/b dtype mismatch");
  const int dt = dtype_code(a);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16, "gemm_nt: bf16/fp16 only");
  const int64_t M = m > 0 ? m : a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt: reduction dims differ");
  const ema::RowMap am = row_map(a_map, M, a.size(0), "gemm_nt a_map");
  at::Tensor c = out.has_value() ? *out : at::empty({M, N}, a.options());
  check_rows(c, "c");
  TORCH_CHECK(c.size(1) == N && c.scalar_type() == a.scalar_type(), "gemm_nt: bad output");
  const ema::RowMap cm = row_map(c_map, M, c.size(0), "gemm_nt c_map");
  TORCH_CHECK(ema::gemm_nt_supported(M, N, K, a.stride(0), b.stride(0), c.stride(0)),
              "gemm_nt: unsupported shape (K % 32, N % 8)");
  // few-tile products split K over fp32 partials (caching allocator, ordered reduce)
  const int64_t wsf = ema::gemm_nt_workspace_floats(M, N, K);
  at::Tensor ws;
  if (wsf > 0) ws = at::empty({wsf}, a.options().dtype(at::kFloat));
  ema::gemm_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, a.stride(0), b.stride(0),
               c.stride(0), dt, cur_stream(), am, cm, wsf > 0 ? ws.data_ptr<float>() : nullptr);
  return c;
}

// fc1 forward with the GLU fused: returns (pre [M, 2F], y [M, F]); with
// c_map the rows go to the given pre / y through the map
std::vector<at::Tensor> gemm_nt_glu(const at::Tensor& a, const at::Tensor& w1, int64_t kind,
                                    c10::optional<at::Tensor> pre_out,
                                    c10::optional<at::Tensor> y_out, std::vector<int64_t> c_map) {
  check_gpu(a, "a");
  check_rows(a, "a");
  check_rows(w1, "w1");
  const int dt = dtype_code(a);
  TORCH_CHECK(a.scalar_type() == w1.scalar_type() && (dt == ema::DT_BF16 || dt == ema::DT_F16),
              "gemm_nt_glu: bf16/fp16 operands of one dtype");
  const int64_t M = a.size(0), K = a.size(1), F = w1.size(0) / 2;
  TORCH_CHECK(w1.size(1) == K && w1.size(0) == 2 * F, "gemm_nt_glu: w1 must be [2F, K]");
  TORCH_CHECK(ema::gemm_nt_supported(M, F, K, a.stride(0), w1.stride(0), 2 * F),
              "gemm_nt_glu: unsupported shape (K % 32, F % 8)");
  TORCH_CHECK(pre_out.has_value() == y_out.has_value(), "gemm_nt_glu: give both outputs or none");
  auto pre = pre_out.has_value() ? *pre_out : at::empty({M, 2 * F}, a.options());
  auto y = y_out.has_value() ? *y_out : at::empty({M, F}, a.options());
  TORCH_CHECK(pre.is_contiguous() && y.is_contiguous() && pre.dim() == 2 && y.dim() == 2 &&
              pre.size(1) == 2 * F && y.size(1) == F && pre.size(0) == y.size(0) &&
              pre.scalar_type() == a.scalar_type() && y.scalar_type() == a.scalar_type(),
              "gemm_nt_glu: outputs must be contiguous [R, 2F] and [R, F] of the operand dtype");
  check_vec_aligned(pre, "pre");
  check_vec_aligned(y, "y");
  const ema::RowMap cm = row_map(c_map, M, pre.size(0), "gemm_nt_glu c_map");
  ema::gemm_nt_glu(a.data_ptr(), w1.data_ptr(), pre.data_ptr(), y.data_ptr(), M, F, K,
                   a.stride(0), w1.stride(0), (int)kind, dt, cur_stream(), cm);
  return {pre, y};
}

// fc2 dgrad with the GLU backward fused: d(pre) [M, 2F] from dy [M, K] and
// w2t = W2^T [F, K] and the saved pre-activation [M, 2F]
at::Tensor gemm_nt_dglu(const at::Tensor& dy, const at::Tensor& w2t, const at::Tensor& pre,
                        int64_t kind, c10::optional<at::Tensor> out) {
  check_gpu(dy, "dy");
  check_rows(dy, "dy");
  check_rows(w2t, "w2t");
  const int dt = dtype_code(dy);
  TORCH_CHECK(dy.scalar_type() == w2t.scalar_type() && pre.scalar_type() == dy.scalar_type() &&
              (dt == ema::DT_BF16 || dt == ema::DT_F16), "gemm_nt_dglu: one bf16/fp16 dtype");
  const int64_t M = dy.size(0), K = dy.size(1), F = w2t.size(0);
  TORCH_CHECK(w2t.size(1) == K, "gemm_nt_dglu: w2t must be [F, K]");
  TORCH_CHECK(pre.is_contiguous() && pre.dim() == 2 && pre.size(0) == M && pre.size(1) == 2 * F,
              "gemm_nt_dglu: pre must be contiguous [M, 2F]");
  check_vec_aligned(pre, "pre");
  TORCH_CHECK(ema::gemm_nt_supported(M, F, K, dy.stride(0), w2t.stride(0), 2 * F),
              "gemm_nt_dglu: unsupported shape (K % 32, F % 8)");
  at::Tensor dpre;
  if (out.has_value()) {
    dpre = *out;
    TORCH_CHECK(dpre.is_contiguous() && dpre.dim() == 2 && dpre.size(0) == M &&
                    dpre.size(1) == 2 * F && dpre.scalar_type() == dy.scalar_type(),
                "gemm_nt_dglu: out must be contiguous [M, 2F] of the operand dtype");
    check_vec_aligned(dpre, "out");
  } else {
    dpre = at::empty({M, 2 * F}, dy.options());
  }
  ema::gemm_nt_dglu(dy.data_ptr(), w2t.data_ptr(), pre.data_ptr(), dpre.data_ptr(), M, F, K,
                    dy.stride(0), w2t.stride(0), (int)kind, dt, cur_stream());
  return dpre;
}

// ---------------------------------------------------------------- transpose
bool transpose16_supported(int64_t rows, int64_t cols) {
  return ema::transpose16_supported(rows, cols);
}

// dst[cols, rows] = src[rows, cols]^T (16-bit dtypes; rows, cols multiples of 64).
void transpose16(const at::Tensor& src, at::Tensor dst) {
  check_gpu(src, "src");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.is_contiguous() && dst.is_contiguous(),
              "transpose16: contiguous 2-D tensors required");
  TORCH_CHECK(src.element_size() == 2 && dst.scalar_type() == src.scalar_type(),
              "transpose16: matching 16-bit dtypes required");
  TORCH_CHECK(dst.device() == src.device(), "transpose16: tensors on different devices");
  const int64_t R = src.size(0), C = src.size(1);
  TORCH_CHECK(dst.size(0) == C && dst.size(1) == R, "transpose16: dst must be [cols, rows]");
  TORCH_CHECK(ema::transpose16_supported(R, C),
              "transpose16: rows and cols must be positive multiples of 64");
  check_vec_aligned(src, "src");
  check_vec_aligned(dst, "dst");
  ema::transpose16(src.data_ptr(), dst.data_ptr(), R, C, cur_stream());
}

}  // namespace

// ---------------------------------------------------------------- xGMI one-shot all-reduce
// (csrc/xgmi_allreduce.hip; parallel/xgmi.py exchanges the handles)
std::tuple<int64_t, at::Tensor> xgmi_create(int64_t rank, int64_t world, int64_t cap) {
  at::Tensor h = at::empty({ema::xgmi_handle_size()}, at::TensorOptions().dtype(at::kByte));
  const int64_t id = ema::xgmi_create((int)rank, (int)world, cap, h.data_ptr());
  return {id, h};
}
void xgmi_open(int64_t id, const at::Tensor& handles) {
  TORCH_CHECK(!handles.is_cuda() && handles.scalar_type() == at::kByte && handles.is_contiguous() &&
                  handles.dim() == 2 && handles.size(1) == ema::xgmi_handle_size(),
              "xgmi_open: handles uint8 [world, handle_size] on the CPU");
  ema::xgmi_open(id, handles.data_ptr());
}
void xgmi_all_reduce(int64_t id, const at::Tensor& inp, at::Tensor out) {
  check_gpu(inp, "inp");
  check_gpu(out, "out");
  const int dt = dtype_code(inp);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16 || dt == ema::DT_F32, "xgmi_all_reduce: dtype");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == inp.numel() &&
                  inp.is_contiguous() && out.is_contiguous(),
              "xgmi_all_reduce: contiguous in / out of one dtype and size");
  const int64_t nbytes = inp.numel() * inp.element_size();
  TORCH_CHECK(nbytes % 16 == 0 && reinterpret_cast<uintptr_t>(inp.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "xgmi_all_reduce: 16-byte aligned, 16-byte sized buffers");
  TORCH_CHECK(nbytes <= ema::xgmi_capacity(id), "xgmi_all_reduce: message exceeds the registered capacity");
  ema::xgmi_all_reduce(id, inp.data_ptr(), out.data_ptr(), nbytes, dt, cur_stream());
}

void xgmi_all_gather(int64_t id, const at::Tensor& inp, at::Tensor out, int64_t world) {
  check_gpu(inp, "inp");
  check_gpu(out, "out");
  const int dt = dtype_code(inp);
  TORCH_CHECK(dt == ema::DT_BF16 || dt == ema::DT_F16 || dt == ema::DT_F32, "xgmi_all_gather: dtype");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type() && out.numel() == world * inp.numel() &&
                  inp.is_contiguous() && out.is_contiguous(),
              "xgmi_all_gather: contiguous in [n] / out [world * n] of one dtype");
  const int64_t nbytes = inp.numel() * inp.element_size();
  const uintptr_t ib = reinterpret_cast<uintptr_t>(inp.data_ptr()),
                  ob = reinterpret_cast<uintptr_t>(out.data_ptr());
  // in disjoint from out, or exactly one of its chunks (the in-place form: every
  // element of in is read and then overwritten by the same thread)
  const bool chunk_alias = ib >= ob && ib < ob + world * nbytes && (ib - ob) % nbytes == 0;
  TORCH_CHECK(ib + nbytes <= ob || ob + world * nbytes <= ib || chunk_alias,
              "xgmi_all_gather: in must be disjoint from out or one of its chunks");
  TORCH_CHECK(nbytes % 16 == 0 && ib % 16 == 0 && ob % 16 == 0,
              "xgmi_all_gather: 16-byte aligned, 16-byte sized buffers");
  TORCH_CHECK(nbytes <= ema::xgmi_capacity(id), "xgmi_all_gather: message exceeds the registered capacity");
  ema::xgmi_all_gather(id, inp.data_ptr(), out.data_ptr(), nbytes, dt, cur_stream());
}

void register_gemm_lt(pybind11::module& m);

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  register_gemm_lt(m);
  m.def("wgrad_gemm", &wgrad_gemm, py::arg("dy"), py::arg("x"), py::arg("g"),
        py::arg("accumulate"), py::arg("x_map") = std::vector<int64_t>{});
  m.def("wgrad_supported", &wgrad_supported);
  m.def("wgrad_set_variant", &ema::wgrad_set_variant);
  m.def("wgrad_plan", &wgrad_plan);
  m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("b"), py::arg("out") = py::none(),
        py::arg("a_map") = std::vector<int64_t>{}, py::arg("c_map") = std::vector<int64_t>{},
        py::arg("m") = 0);
  m.def("gemm_nt_supported", &gemm_nt_supported);
  m.def("gemm_nt_ksplit", [](int64_t M, int64_t N, int64_t K) { return ema::gemm_nt_ksplit(M, N, K); });
  m.def("gemm_nt_set_variant", &ema::gemm_nt_set_variant);
  m.def("gemm_nt_glu", &gemm_nt_glu, py::arg("a"), py::arg("w1"), py::arg("kind"),
        py::arg("pre") = py::none(), py::arg("y") = py::none(),
        py::arg("c_map") = std::vector<int64_t>{});
  m.def("gemm_nt_dglu", &gemm_nt_dglu, py::arg("dy"), py::arg("w2t"), py::arg("pre"),
        py::arg("kind"), py::arg("out") = py::none());
  m.doc() = "epfl_megatron_amd gfx950 (MI355X) HIP kernels";
  m.def("rmsnorm_fwd", &rmsnorm_fwd, py::arg("x"), py::arg("w"), py::arg("eps"),
        py::arg("res") = py::none());
  m.def("rmsnorm_bwd", &rmsnorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("rstd"),
        py::arg("dres") = py::none(), py::arg("dw_acc") = py::none(),
        py::arg("accumulate") = false);
  m.def("layernorm_fwd", &layernorm_fwd, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("eps"),
        py::arg("res") = py::none());
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"),
        py::arg("mean"), py::arg("rstd"), py::arg("dres") = py::none(),
        py::arg("dw_acc") = py::none(), py::arg("db_acc") = py::none(),
        py::arg("accumulate_w") = false, py::arg("accumulate_b") = false);
  m.def("rope_qkv_inplace", &rope_qkv_inplace);
  m.def("glu_fwd", &glu_fwd);
  m.def("glu_bwd", &glu_bwd);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("ce_fwd_fused", &ce_fwd_fused);
  m.def("ce_row_max", &ce_row_max);
  m.def("ce_sumexp_target", &ce_sumexp_target);
  m.def("ce_bwd", &ce_bwd);
  m.def("softmax_fwd", &softmax_fwd);
  m.def("softmax_bwd", &softmax_bwd);
  m.def("chunked_sumsq", &chunked_sumsq);
  m.def("flat_adam", &flat_adam);
  m.def("opt_prep", &opt_prep);
  m.def("bias_dropout_add_fwd", &bias_dropout_add_fwd);
  m.def("bias_dropout_add_bwd", &bias_dropout_add_bwd);
  m.def("flash_attn_fwd", &flash_attn_fwd);
  m.def("flash_attn_fwd_merge", &flash_attn_fwd_merge, py::arg("q"), py::arg("k"), py::arg("v"),
        py::arg("o32"), py::arg("lse"), py::arg("b"), py::arg("sq"), py::arg("sk"), py::arg("nq"),
        py::arg("nkv"), py::arg("hd"), py::arg("qs"), py::arg("ks"), py::arg("vs"),
        py::arg("causal"), py::arg("scale"), py::arg("merge"), py::arg("docs") = py::none(),
        py::arg("coff") = -1);
  m.def("flash_attn_bwd", &flash_attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"),
        py::arg("v"), py::arg("out"), py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"),
        py::arg("b"), py::arg("sq"), py::arg("sk"), py::arg("nq"), py::arg("nkv"), py::arg("hd"),
        py::arg("qs"), py::arg("ks"), py::arg("vs"), py::arg("os"), py::arg("causal"),
        py::arg("scale"), py::arg("rope_cos"), py::arg("rope_sin"), py::arg("rope_pos"),
        py::arg("docs"), py::arg("coff") = -1);
  m.def("fa_set_stamps", &fa_set_stamps);
  m.def("fa_set_pairing", &ema::fa_set_pairing);
  m.def("fa_set_kv2", &ema::fa_set_kv2);
  m.def("greedy_tail", &greedy_tail);
  m.def("xgmi_create", &xgmi_create);
  m.def("xgmi_open", &xgmi_open);
  m.def("xgmi_all_reduce", &xgmi_all_reduce);
  m.def("xgmi_all_gather", &xgmi_all_gather);
  m.def("xgmi_error", [](int64_t id) { return ema::xgmi_error(id); });
  m.def("xgmi_set_timeout", [](int64_t id, int64_t ms) { ema::xgmi_set_timeout(id, ms); });
  m.def("xgmi_get_timeout", [](int64_t id) { return ema::xgmi_get_timeout(id); });
  m.def("xgmi_error_tensor", [](int64_t id) {
    // a view of the communicator's device error word (no ownership: the
    // Python communicator keeps it alive while it holds the view)
    int dev = 0;
    TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "hipGetDevice");
    return at::from_blob(ema::xgmi_error_word(id), {1},
                         at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev));
  });
  m.def("xgmi_destroy", [](int64_t id) { ema::xgmi_destroy(id); });
  m.def("flash_decode", &flash_decode, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("out"),
        py::arg("b"), py::arg("sk"), py::arg("nq"), py::arg("nkv"), py::arg("hd"), py::arg("qs"),
        py::arg("ks"), py::arg("vs"), py::arg("os"), py::arg("scale"), py::arg("kv_len"),
        py::arg("kpw") = 0);
  m.def("skinny_gemm", &skinny_gemm, py::arg("x"), py::arg("w"), py::arg("packed") = false);
  m.def("skinny_gemm_supported", &skinny_gemm_supported);
  m.def("skinny_norm_gemm", &skinny_norm_gemm, py::arg("x"), py::arg("w"), py::arg("norm_w"),
        py::arg("eps"), py::arg("res"), py::arg("packed") = false);
  m.def("skinny_norm_glu", &skinny_norm_glu, py::arg("x"), py::arg("w1"), py::arg("norm_w"),
        py::arg("eps"), py::arg("kind"), py::arg("packed") = false, py::arg("packed_tail") = 0);
  m.def("skinny_glu_half_tail", &ema::skinny_glu_half_tail, py::arg("F"), py::arg("K"),
        py::arg("norm"), py::arg("M") = 1);
  m.def("skinny_qkv_rope_cache", &skinny_qkv_rope_cache, py::arg("x"), py::arg("w"),
        py::arg("norm_w"), py::arg("eps"), py::arg("ng"), py::arg("r"), py::arg("hd"),
        py::arg("cos"), py::arg("sin"), py::arg("pos"), py::arg("kcache"), py::arg("vcache"),
        py::arg("slot_t"), py::arg("slot"), py::arg("packed") = false);
  m.def("transpose16", &transpose16);
  m.def("transpose16_supported", &transpose16_supported);
}
