// PyTorch bindings for the kubedl_amd HIP kernels (module ``kubedl_amd._C``).
//
// Kernels live in the *.hip translation units and take raw pointers plus a
// hipStream_t; this file owns all tensor checks, output allocation (through
// the PyTorch caching allocator) and stream selection.  Every launch goes to
// PyTorch's current HIP stream so the ops compose with autograd, RCCL and
// hipGraph capture.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kdl_api.h"

namespace {

int dtype_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return 1;
  if (t.scalar_type() == at::kFloat) return 0;
  TORCH_CHECK(false, "kubedl_amd: unsupported dtype ", t.scalar_type());
  return -1;
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "kubedl_amd: ", what, " failed: ", hipGetErrorString(e));
}

bool is_nhwc_dense(const at::Tensor& t) {
  if (t.dim() == 4) return t.is_contiguous(at::MemoryFormat::ChannelsLast);
  return t.is_contiguous();
}

// ------------------------------------------------------------------ BN + act
// ``ws``: optional per-layer fp32 workspace (bn_workspace_floats(C) elements,
// zero-initialised once by its owner and kept zero by the kernels); a fresh
// zeroed one is allocated here if absent.
at::Tensor get_acc(const c10::optional<at::Tensor>& acc, int64_t C, const at::Tensor& like) {
  const int64_t n = kdl::bn_workspace_floats(static_cast<int>(C));
  if (acc.has_value() && acc->defined()) {
    TORCH_CHECK(acc->scalar_type() == at::kFloat && acc->is_contiguous() && acc->numel() >= n &&
                    acc->device() == like.device(),
                "bn: workspace must be a contiguous fp32 tensor of >= bn_workspace_floats(C) "
                "elements on x's device");
    return *acc;
  }
  return at::zeros({n}, like.options().dtype(at::kFloat));
}

int64_t bn_ws_floats(int64_t C) { return kdl::bn_workspace_floats(static_cast<int>(C)); }

std::vector<at::Tensor> bn_act_fwd(const at::Tensor& x, const at::Tensor& weight,
                                   const at::Tensor& bias, const at::Tensor& running_mean,
                                   const at::Tensor& running_var,
                                   const c10::optional<at::Tensor>& residual, bool relu,
                                   bool training, double momentum, double eps,
                                   const c10::optional<at::Tensor>& acc, bool want_mask) {
  TORCH_CHECK(x.is_cuda(), "bn_act_fwd: x must be on the GPU");
  TORCH_CHECK(x.dim() == 4 || x.dim() == 2, "bn_act_fwd: x must be NHWC 4-D or [M, C]");
  TORCH_CHECK(is_nhwc_dense(x), "bn_act_fwd: x must be channels_last-dense");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(weight.numel() == C && bias.numel() == C, "bn_act_fwd: affine size mismatch");
  TORCH_CHECK(weight.scalar_type() == bias.scalar_type(), "bn_act_fwd: weight/bias dtype mismatch");
  TORCH_CHECK(running_mean.scalar_type() == at::kFloat && running_var.scalar_type() == at::kFloat,
              "bn_act_fwd: running stats must be fp32");
  TORCH_CHECK(running_mean.numel() == C && running_var.numel() == C, "bn_act_fwd: stats size");
  const at::Tensor* res = nullptr;
  if (residual.has_value() && residual->defined()) {
    res = &residual.value();
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == x.scalar_type() &&
                    is_nhwc_dense(*res),
                "bn_act_fwd: residual must match x (shape, dtype, channels_last)");
  }
  auto y = at::empty_like(x);
  // packed ReLU mask (uint8 [M, C/8]) replaces y in the backward of relu+residual layers
  const bool mask = want_mask && relu && res != nullptr && x.scalar_type() == at::kBFloat16 && C % 8 == 0;
  at::Tensor mbits;
  if (mask) mbits = at::empty({M, C / 8}, x.options().dtype(at::kByte));
  auto fopt = x.options().dtype(at::kFloat);
  auto save_mean = at::empty({C}, fopt);
  auto save_invstd = at::empty({C}, fopt);
  at::Tensor a = get_acc(acc, C, x);
  check_hip(kdl::bn_act_forward(x.data_ptr(), res ? res->data_ptr() : nullptr, y.data_ptr(),
                                mask ? mbits.data_ptr<uint8_t>() : nullptr, weight.data_ptr(), bias.data_ptr(), running_mean.data_ptr<float>(),
                                running_var.data_ptr<float>(), save_mean.data_ptr<float>(),
                                save_invstd.data_ptr<float>(), a.data_ptr<float>(), M,
                                static_cast<int>(C), dtype_code(x), dtype_code(weight), relu,
                                training, static_cast<float>(momentum), static_cast<float>(eps),
                                cur_stream()),
            "bn_act_forward");
  return {y, save_mean, save_invstd, mbits};
}

std::vector<at::Tensor> bn_act_bwd(const at::Tensor& dy, const at::Tensor& x,
                                   const c10::optional<at::Tensor>& y_opt,
                                   const at::Tensor& weight, const at::Tensor& bias,
                                   const at::Tensor& mean, const at::Tensor& invstd, bool relu,
                                   bool has_residual, bool training,
                                   const c10::optional<at::Tensor>& acc,
                                   const c10::optional<at::Tensor>& mask) {
  const bool has_mask = mask.has_value() && mask->defined();
  const bool has_y = y_opt.has_value() && y_opt->defined();
  TORCH_CHECK(has_y || has_mask || !relu, "bn_act_bwd: relu needs y or the packed mask");
  TORCH_CHECK(is_nhwc_dense(dy) && is_nhwc_dense(x) && (!has_y || is_nhwc_dense(*y_opt)),
              "bn_act_bwd: tensors must be channels_last-dense");
  TORCH_CHECK(dy.sizes() == x.sizes() && (!has_y || y_opt->sizes() == x.sizes()),
              "bn_act_bwd: shape mismatch");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "bn_act_bwd: dtype mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t C = x.size(1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(weight.numel() == C && bias.numel() == C && mean.numel() == C && invstd.numel() == C,
              "bn_act_bwd: per-channel tensor size mismatch");
  if (has_mask)
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->is_contiguous() && mask->numel() == M * (C / 8) &&
                    C % 8 == 0 && x.scalar_type() == at::kBFloat16,
                "bn_act_bwd: mask must be uint8 [M, C/8] for bf16 x");
  auto dx = at::empty_like(x);
  at::Tensor dres;
  if (has_residual) dres = at::empty_like(x);
  auto dgamma = at::empty_like(weight);
  auto dbeta = at::empty_like(weight);
  at::Tensor a = get_acc(acc, C, x);
  check_hip(kdl::bn_act_backward(dy.data_ptr(), has_y ? y_opt->data_ptr() : nullptr,
                                 has_mask ? mask->data_ptr<uint8_t>() : nullptr, x.data_ptr(),
                                 weight.data_ptr(),
                                 bias.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                 dx.data_ptr(), has_residual ? dres.data_ptr() : nullptr,
                                 dgamma.data_ptr(), dbeta.data_ptr(), a.data_ptr<float>(), M,
                                 static_cast<int>(C), dtype_code(x), dtype_code(weight), relu,
                                 training, cur_stream()),
            "bn_act_backward");
  return {dx, dgamma, dbeta, has_residual ? dres : at::Tensor()};
}

std::vector<at::Tensor> bn_pool_fwd(const at::Tensor& x, const at::Tensor& weight, const at::Tensor& bias,
                                    const at::Tensor& running_mean, const at::Tensor& running_var,
                                    bool training, double momentum, double eps,
                                    const c10::optional<at::Tensor>& acc) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && is_nhwc_dense(x) && x.scalar_type() == at::kBFloat16,
              "bn_pool_fwd: x must be a channels_last bf16 NCHW tensor");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0, "bn_pool_fwd: C % 8 == 0");
  TORCH_CHECK(weight.numel() == C && bias.numel() == C && running_mean.numel() == C &&
                  running_var.numel() == C && running_mean.scalar_type() == at::kFloat,
              "bn_pool_fwd: per-channel tensors");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t PH = (H - 1) / 2 + 1, PW = (W - 1) / 2 + 1;
  auto y = at::empty({N, C, PH, PW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, PH, PW, C}, x.options().dtype(at::kByte));
  auto fopt = x.options().dtype(at::kFloat);
  auto save_mean = at::empty({C}, fopt);
  auto save_invstd = at::empty({C}, fopt);
  at::Tensor a = get_acc(acc, C, x);
  check_hip(kdl::bn_pool_forward(x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), weight.data_ptr(),
                                 bias.data_ptr(), running_mean.data_ptr<float>(),
                                 running_var.data_ptr<float>(), save_mean.data_ptr<float>(),
                                 save_invstd.data_ptr<float>(), a.data_ptr<float>(), static_cast<int>(N),
                                 static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                 dtype_code(weight), training, static_cast<float>(momentum),
                                 static_cast<float>(eps), cur_stream()),
            "bn_pool_forward");
  return {y, save_mean, save_invstd, idx};
}

std::vector<at::Tensor> bn_pool_bwd(const at::Tensor& dyp, const at::Tensor& idx, const at::Tensor& x,
                                    const at::Tensor& weight, const at::Tensor& bias, const at::Tensor& mean,
                                    const at::Tensor& invstd, bool training,
                                    const c10::optional<at::Tensor>& acc) {
  TORCH_CHECK(is_nhwc_dense(x) && is_nhwc_dense(dyp) && dyp.scalar_type() == at::kBFloat16 &&
                  x.scalar_type() == at::kBFloat16,
              "bn_pool_bwd: channels_last bf16 tensors");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t PH = (H - 1) / 2 + 1, PW = (W - 1) / 2 + 1;
  TORCH_CHECK(dyp.size(0) == N && dyp.size(1) == C && dyp.size(2) == PH && dyp.size(3) == PW,
              "bn_pool_bwd: pooled gradient shape");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.numel() == N * PH * PW * C,
              "bn_pool_bwd: idx");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto dx = at::empty_like(x);
  auto dgamma = at::empty_like(weight);
  auto dbeta = at::empty_like(weight);
  at::Tensor a = get_acc(acc, C, x);
  check_hip(kdl::bn_pool_backward(dyp.data_ptr(), idx.data_ptr<uint8_t>(), x.data_ptr(), weight.data_ptr(),
                                  bias.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                  dx.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), a.data_ptr<float>(),
                                  static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                                  static_cast<int>(C), dtype_code(weight), training, cur_stream()),
            "bn_pool_backward");
  return {dx, dgamma, dbeta};
}

// ------------------------------------------------------------------ optimizers
kdl::OptHyper make_hyper(double lr, double momentum, double dampening, double eps, double bc1,
                         double bc2, double grad_scale, bool nesterov, bool first_step, bool adam_w,
                         const std::vector<double>& wd, const std::vector<double>& lr_scale) {
  kdl::OptHyper h{};
  h.lr = static_cast<float>(lr);
  h.momentum = static_cast<float>(momentum);
  h.dampening = static_cast<float>(dampening);
  h.eps = static_cast<float>(eps);
  h.bc1 = static_cast<float>(bc1);
  h.bc2 = static_cast<float>(bc2);
  h.grad_scale = static_cast<float>(grad_scale);
  h.nesterov = nesterov;
  h.first_step = first_step;
  h.adam_w = adam_w;
  TORCH_CHECK(wd.size() <= 4 && lr_scale.size() <= 4, "at most 4 hyper-parameter groups");
  for (int i = 0; i < 4; ++i) {
    h.wd[i] = i < static_cast<int>(wd.size()) ? static_cast<float>(wd[i]) : 0.f;
    h.lr_scale[i] = i < static_cast<int>(lr_scale.size()) ? static_cast<float>(lr_scale[i]) : 1.f;
  }
  return h;
}

void check_chunks(const at::Tensor& chunks) {
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong && chunks.dim() == 2 &&
                  chunks.size(1) == 2,
              "chunk table must be an int64 [n, 2] GPU tensor");
  static_assert(sizeof(kdl::OptChunk) == 16, "OptChunk layout");
}

void sgd_step(const at::Tensor& chunks, at::Tensor master, at::Tensor mom, const at::Tensor& grad,
              at::Tensor param, double lr, double momentum, double dampening, double grad_scale,
              bool nesterov, bool first_step, const std::vector<double>& wd,
              const std::vector<double>& lr_scale) {
  check_chunks(chunks);
  TORCH_CHECK(master.scalar_type() == at::kFloat && mom.scalar_type() == at::kFloat,
              "sgd_step: master/momentum must be fp32");
  TORCH_CHECK(master.numel() == grad.numel() && grad.numel() == param.numel() &&
                  mom.numel() == master.numel(),
              "sgd_step: flat buffer size mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(master.device());
  auto h = make_hyper(lr, momentum, dampening, 0, 1, 1, grad_scale, nesterov, first_step, false, wd,
                      lr_scale);
  check_hip(kdl::fused_sgd(reinterpret_cast<const kdl::OptChunk*>(chunks.data_ptr<int64_t>()),
                           static_cast<int>(chunks.size(0)), master.data_ptr<float>(),
                           mom.data_ptr<float>(), grad.data_ptr(), param.data_ptr(),
                           dtype_code(grad), dtype_code(param), h, cur_stream()),
            "fused_sgd");
}

void adam_step(const at::Tensor& chunks, at::Tensor master, at::Tensor m1, at::Tensor m2,
               const at::Tensor& grad, at::Tensor param, double lr, double beta1, double beta2,
               double eps, int64_t step, double grad_scale, bool adam_w,
               const std::vector<double>& wd, const std::vector<double>& lr_scale) {
  check_chunks(chunks);
  TORCH_CHECK(master.numel() == grad.numel() && grad.numel() == param.numel() &&
                  m1.numel() == master.numel() && m2.numel() == master.numel(),
              "adam_step: flat buffer size mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(master.device());
  const double bc1 = 1.0 - std::pow(beta1, static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(beta2, static_cast<double>(step));
  auto h = make_hyper(lr, beta1, beta2, eps, bc1, bc2, grad_scale, false, false, adam_w, wd, lr_scale);
  check_hip(kdl::fused_adam(reinterpret_cast<const kdl::OptChunk*>(chunks.data_ptr<int64_t>()),
                            static_cast<int>(chunks.size(0)), master.data_ptr<float>(),
                            m1.data_ptr<float>(), m2.data_ptr<float>(), grad.data_ptr(),
                            param.data_ptr(), dtype_code(grad), dtype_code(param), h, cur_stream()),
            "fused_adam");
}

at::Tensor chunk_sumsq(const at::Tensor& chunks, const at::Tensor& x, double scale) {
  check_chunks(chunks);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto out = at::empty({chunks.size(0)}, x.options().dtype(at::kFloat));
  check_hip(kdl::chunk_sumsq(reinterpret_cast<const kdl::OptChunk*>(chunks.data_ptr<int64_t>()),
                             static_cast<int>(chunks.size(0)), x.data_ptr(), dtype_code(x),
                             static_cast<float>(scale), out.data_ptr<float>(), cur_stream()),
            "chunk_sumsq");
  return out;
}

void cast_copy(const at::Tensor& src, at::Tensor dst) {
  TORCH_CHECK(src.numel() == dst.numel() && src.is_contiguous() && dst.is_contiguous(),
              "cast_copy: size/contiguity mismatch");
  TORCH_CHECK(src.numel() % 8 == 0, "cast_copy: numel must be a multiple of 8");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  check_hip(kdl::cast_copy(src.data_ptr(), dtype_code(src), dst.data_ptr(), dtype_code(dst),
                           src.numel(), cur_stream()),
            "cast_copy");
}

// ------------------------------------------------------------------ multi-tensor pack
void pack_grads(const at::Tensor& chunks, const at::Tensor& src_ptrs, at::Tensor dst, double scale) {
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong && chunks.dim() == 2 &&
                  chunks.size(1) == 3 && chunks.is_contiguous(),
              "pack_grads: chunk table must be a contiguous int64 [n, 3] GPU tensor");
  TORCH_CHECK(src_ptrs.is_cuda() && src_ptrs.scalar_type() == at::kLong && src_ptrs.is_contiguous(),
              "pack_grads: src_ptrs must be a contiguous int64 GPU tensor");
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "pack_grads: dst must be contiguous on GPU");
  static_assert(sizeof(kdl::PackChunk) == 24, "PackChunk layout");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  check_hip(kdl::pack_tensors(reinterpret_cast<const kdl::PackChunk*>(chunks.data_ptr<int64_t>()),
                              static_cast<int>(chunks.size(0)), src_ptrs.data_ptr<int64_t>(),
                              dst.data_ptr(), dtype_code(dst), static_cast<float>(scale),
                              cur_stream()),
            "pack_tensors");
}

// ------------------------------------------------------------------ GBDT
void gbdt_hist(const at::Tensor& bins, const at::Tensor& grad, const at::Tensor& hess, int64_t gh_stride,
               const at::Tensor& rows, const at::Tensor& seg, int64_t max_rows_per_node, int64_t num_bins,
               at::Tensor hist) {
  TORCH_CHECK(bins.is_cuda() && bins.scalar_type() == at::kByte && bins.dim() == 2 && bins.is_contiguous(),
              "gbdt_hist: bins must be a contiguous uint8 [N, F] GPU tensor");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && hess.scalar_type() == at::kFloat, "gbdt_hist: g/h fp32");
  TORCH_CHECK(rows.scalar_type() == at::kInt && seg.scalar_type() == at::kInt && rows.is_contiguous() &&
                  seg.is_contiguous(),
              "gbdt_hist: rows/seg must be contiguous int32");
  const int64_t F = bins.size(1);
  const int64_t nodes = seg.numel() - 1;
  TORCH_CHECK(num_bins >= 2 && num_bins <= 256, "gbdt_hist: 2 <= num_bins <= 256");
  TORCH_CHECK(hist.is_contiguous() && hist.scalar_type() == at::kFloat && hist.numel() == nodes * F * num_bins * 2,
              "gbdt_hist: hist must be contiguous fp32 [nodes, F, B, 2]");
  TORCH_CHECK(grad.numel() >= (bins.size(0) - 1) * gh_stride + 1 && hess.numel() == grad.numel(),
              "gbdt_hist: grad/hess too small for the row stride");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins.device());
  check_hip(kdl::gbdt_hist_build(bins.data_ptr<uint8_t>(), grad.data_ptr<float>(), hess.data_ptr<float>(),
                                 gh_stride, rows.data_ptr<int32_t>(), seg.data_ptr<int32_t>(),
                                 static_cast<int>(nodes), static_cast<int>(max_rows_per_node),
                                 static_cast<int>(F), static_cast<int>(num_bins), hist.data_ptr<float>(),
                                 cur_stream()),
            "gbdt_hist_build");
}

std::vector<at::Tensor> gbdt_split(const at::Tensor& hist, double lambda, double min_child_weight) {
  TORCH_CHECK(hist.is_cuda() && hist.dim() == 4 && hist.size(3) == 2 && hist.is_contiguous() &&
                  hist.scalar_type() == at::kFloat,
              "gbdt_split: hist must be contiguous fp32 [nodes, F, B, 2]");
  TORCH_CHECK(hist.size(2) <= 256, "gbdt_split: at most 256 bins");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(hist.device());
  const int64_t nodes = hist.size(0), F = hist.size(1), B = hist.size(2);
  auto fo = hist.options();
  auto gain = at::empty({nodes, F}, fo);
  auto bin = at::empty({nodes, F}, fo.dtype(at::kInt));
  auto gl = at::empty({nodes, F}, fo);
  auto hl = at::empty({nodes, F}, fo);
  check_hip(kdl::gbdt_split_find(hist.data_ptr<float>(), static_cast<int>(nodes), static_cast<int>(F),
                                 static_cast<int>(B), static_cast<float>(lambda),
                                 static_cast<float>(min_child_weight), gain.data_ptr<float>(),
                                 bin.data_ptr<int32_t>(), gl.data_ptr<float>(), hl.data_ptr<float>(), cur_stream()),
            "gbdt_split_find");
  return {gain, bin, gl, hl};
}

at::Tensor gbdt_route(const at::Tensor& bins, const at::Tensor& rows, const at::Tensor& row_node,
                      const at::Tensor& split_feat, const at::Tensor& split_bin) {
  TORCH_CHECK(bins.is_cuda() && bins.scalar_type() == at::kByte && bins.is_contiguous(), "gbdt_route: bins");
  TORCH_CHECK(rows.scalar_type() == at::kInt && row_node.scalar_type() == at::kInt &&
                  split_feat.scalar_type() == at::kInt && split_bin.scalar_type() == at::kInt,
              "gbdt_route: int32 tensors expected");
  TORCH_CHECK(rows.numel() == row_node.numel(), "gbdt_route: rows/row_node size");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins.device());
  auto out = at::empty_like(rows);
  check_hip(kdl::gbdt_route_rows(bins.data_ptr<uint8_t>(), rows.data_ptr<int32_t>(), row_node.data_ptr<int32_t>(),
                                 split_feat.data_ptr<int32_t>(), split_bin.data_ptr<int32_t>(),
                                 static_cast<int>(bins.size(1)), static_cast<int>(rows.numel()),
                                 out.data_ptr<int32_t>(), cur_stream()),
            "gbdt_route_rows");
  return out;
}

// ------------------------------------------------------------------ CTR
at::Tensor gemm_bias_act(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& bias, bool relu) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "gemm_bias_act: bf16 GPU operands");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1), "gemm_bias_act: A [M,K], W [N,K]");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous(), "gemm_bias_act: contiguous operands");
  TORCH_CHECK(a.size(1) % 8 == 0, "gemm_bias_act: K must be a multiple of 8 (16-byte rows)");
  const int64_t M = a.size(0), N = w.size(0), K = a.size(1);
  const float* bp = nullptr;
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b.numel() == N, "gemm_bias_act: bias size");
    bp = b.data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto c = at::empty({M, N}, a.options());
  check_hip(kdl::gemm_bias_act(a.data_ptr(), w.data_ptr(), bp, c.data_ptr(), static_cast<int>(M),
                               static_cast<int>(N), static_cast<int>(K), relu, cur_stream()),
            "gemm_bias_act");
  return c;
}

std::vector<at::Tensor> relu_bwd_dbias(const at::Tensor& dy, const c10::optional<at::Tensor>& y) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 2 && dy.is_contiguous(),
              "relu_bwd_dbias: dy bf16 [M,N] contiguous");
  TORCH_CHECK(dy.size(1) % 8 == 0, "relu_bwd_dbias: N % 8 == 0");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  const bool has_y = y.has_value() && y->defined();
  at::Tensor dz = has_y ? at::empty_like(dy) : dy;
  if (has_y) TORCH_CHECK(y->sizes() == dy.sizes() && y->is_contiguous(), "relu_bwd_dbias: y shape");
  auto db = at::zeros({dy.size(1)}, dy.options().dtype(at::kFloat));
  check_hip(kdl::relu_bwd_dbias(dy.data_ptr(), has_y ? y->data_ptr() : nullptr, dz.data_ptr(), db.data_ptr<float>(),
                                static_cast<int>(dy.size(0)), static_cast<int>(dy.size(1)), cur_stream()),
            "relu_bwd_dbias");
  return {dz, db};
}

void embed_gather(const at::Tensor& table, const at::Tensor& idx, int64_t F, at::Tensor out, int64_t col0) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.is_contiguous(), "embed_gather: table [V, D]");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous(), "embed_gather: int64 idx");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.scalar_type() == table.scalar_type(), "embed_gather: out");
  const int64_t D = table.size(1), n = idx.numel();
  TORCH_CHECK(n % F == 0 && out.size(0) * F == n && col0 + F * D <= out.size(1), "embed_gather: shapes");
  TORCH_CHECK((D * table.element_size()) % 16 == 0 && (out.stride(0) * out.element_size()) % 16 == 0 &&
                  (col0 * out.element_size()) % 16 == 0,
              "embed_gather: rows must be 16-byte multiples");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  check_hip(kdl::embed_gather(table.data_ptr(), dtype_code(table), idx.data_ptr<int64_t>(), static_cast<int>(n),
                              static_cast<int>(F), static_cast<int>(D), out.data_ptr(),
                              static_cast<int>(out.stride(0)), static_cast<int>(col0), cur_stream()),
            "embed_gather");
}

at::Tensor segment_reduce(const at::Tensor& rows, int64_t F, int64_t col0, int64_t D, const at::Tensor& order,
                          const at::Tensor& seg) {
  TORCH_CHECK(rows.is_cuda() && rows.dim() == 2 && rows.stride(1) == 1, "segment_reduce: rows [B, ld]");
  TORCH_CHECK(order.scalar_type() == at::kLong && seg.scalar_type() == at::kLong && order.is_contiguous() &&
                  seg.is_contiguous(),
              "segment_reduce: int64 order/seg");
  TORCH_CHECK(order.numel() == rows.size(0) * F && col0 + F * D <= rows.size(1), "segment_reduce: shapes");
  const int64_t U = seg.numel() - 1;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(rows.device());
  auto out = at::empty({U, D}, rows.options().dtype(at::kFloat));
  check_hip(kdl::segment_reduce(rows.data_ptr(), dtype_code(rows), static_cast<int>(F), static_cast<int>(rows.stride(0)),
                                static_cast<int>(col0), order.data_ptr<int64_t>(), seg.data_ptr<int64_t>(),
                                static_cast<int>(U), static_cast<int>(D), out.data_ptr<float>(), cur_stream()),
            "segment_reduce");
  return out;
}

void segment_adagrad(const at::Tensor& grads, const at::Tensor& order, const at::Tensor& seg,
                     const at::Tensor& rows_local, at::Tensor table, at::Tensor accum, double lr, double eps,
                     double scale) {
  TORCH_CHECK(grads.is_cuda() && grads.scalar_type() == at::kFloat && grads.is_contiguous(), "segment_adagrad: grads");
  TORCH_CHECK(table.scalar_type() == at::kFloat && accum.scalar_type() == at::kFloat && table.is_contiguous() &&
                  accum.is_contiguous() && table.sizes() == accum.sizes(),
              "segment_adagrad: fp32 table/accum");
  TORCH_CHECK(grads.size(1) == table.size(1), "segment_adagrad: D mismatch");
  TORCH_CHECK(rows_local.numel() == seg.numel() - 1 && order.numel() == grads.size(0), "segment_adagrad: shapes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  check_hip(kdl::segment_adagrad(grads.data_ptr<float>(), order.data_ptr<int64_t>(), seg.data_ptr<int64_t>(),
                                 rows_local.data_ptr<int64_t>(), static_cast<int>(seg.numel() - 1),
                                 static_cast<int>(table.size(1)), table.data_ptr<float>(), accum.data_ptr<float>(),
                                 static_cast<float>(lr), static_cast<float>(eps), static_cast<float>(scale),
                                 cur_stream()),
            "segment_adagrad");
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "kubedl_amd CDNA4 (gfx950) HIP kernels";
  m.def("bn_act_fwd", &bn_act_fwd, "fused BatchNorm(+residual)(+ReLU) forward, NHWC");
  m.def("bn_act_bwd", &bn_act_bwd, "fused BatchNorm(+residual)(+ReLU) backward, NHWC");
  m.def("bn_pool_fwd", &bn_pool_fwd, "stem BatchNorm + ReLU + max-pool(3,2,1) forward, NHWC bf16");
  m.def("bn_pool_bwd", &bn_pool_bwd, "stem BatchNorm + ReLU + max-pool(3,2,1) backward, NHWC bf16");
  m.def("bn_workspace_floats", &bn_ws_floats, "per-layer BN workspace size (fp32 elements)");
  m.def("sgd_step", &sgd_step, "flat chunked fused SGD-momentum with fp32 master weights");
  m.def("adam_step", &adam_step, "flat chunked fused Adam/AdamW with fp32 master weights");
  m.def("chunk_sumsq", &chunk_sumsq, "per-chunk sum of squares");
  m.def("cast_copy", &cast_copy, "flat dtype-casting copy");
  m.def("pack_grads", &pack_grads, "multi-tensor gather of gradient tensors into a flat buffer");
  m.def("gbdt_hist", &gbdt_hist, "GBDT per-node gradient/hessian histograms (LDS atomics)");
  m.def("gbdt_split", &gbdt_split, "GBDT best split per (node, feature)");
  m.def("gbdt_route", &gbdt_route, "GBDT row routing (1 = right child)");
  m.def("gemm_bias_act", &gemm_bias_act, "MFMA bf16 GEMM C = act(A W^T + b)");
  m.def("relu_bwd_dbias", &relu_bwd_dbias, "ReLU backward (mask from output) + bias gradient");
  m.def("embed_gather", &embed_gather, "embedding row gather into a [B, ld] activation");
  m.def("segment_reduce", &segment_reduce, "sorted segment sum of gradient rows");
  m.def("segment_adagrad", &segment_adagrad, "segment sum + fused sparse Adagrad on owned rows");
  m.attr("arch") = "gfx950";
}
