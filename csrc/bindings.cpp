#include <map>
#include <mutex>
// PyTorch bindings for the kubedl_amd HIP kernels (module ``kubedl_amd._C``).
//
// Kernels live in the *.hip translation units and take raw pointers plus a
// hipStream_t; this file owns all tensor checks, output allocation (through
// the PyTorch caching allocator) and stream selection.  Every launch goes to
// PyTorch's current HIP stream so the ops compose with autograd, RCCL and
// hipGraph capture.
#include <cstring>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "bn_fin.h"
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
  // relu without a residual recomputes its mask from x; with a residual it needs y or the bits
  TORCH_CHECK(has_y || has_mask || !relu || !has_residual, "bn_act_bwd: relu+residual needs y or the packed mask");
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
                                    const c10::optional<at::Tensor>& acc, bool gemm_stats, bool want_xam) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && is_nhwc_dense(x) && x.scalar_type() == at::kBFloat16,
              "bn_pool_fwd: x must be a channels_last bf16 NCHW tensor");
  TORCH_CHECK(!gemm_stats || (acc.has_value() && acc->defined()), "bn_pool_fwd: gemm_stats reads the statistics from acc");
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
  auto xam = want_xam ? at::empty_like(y) : at::Tensor();
  check_hip(kdl::bn_pool_forward(x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), weight.data_ptr(),
                                 bias.data_ptr(), running_mean.data_ptr<float>(),
                                 running_var.data_ptr<float>(), save_mean.data_ptr<float>(),
                                 save_invstd.data_ptr<float>(), a.data_ptr<float>(), static_cast<int>(N),
                                 static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                 dtype_code(weight), training, static_cast<float>(momentum),
                                 static_cast<float>(eps), cur_stream(), gemm_stats,
                                 want_xam ? xam.data_ptr() : nullptr),
            "bn_pool_forward");
  return {y, save_mean, save_invstd, idx, xam};
}

std::vector<at::Tensor> bn_pool_bwd(const at::Tensor& dyp, const at::Tensor& idx, const at::Tensor& x,
                                    const at::Tensor& weight, const at::Tensor& bias, const at::Tensor& mean,
                                    const at::Tensor& invstd, bool training,
                                    const c10::optional<at::Tensor>& acc, bool with_dx) {
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
  auto dx = with_dx ? at::empty_like(x) : at::Tensor();
  auto dgamma = at::empty_like(weight);
  auto dbeta = at::empty_like(weight);
  at::Tensor a = get_acc(acc, C, x);
  check_hip(kdl::bn_pool_backward(dyp.data_ptr(), idx.data_ptr<uint8_t>(), x.data_ptr(), weight.data_ptr(),
                                  bias.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                  with_dx ? dx.data_ptr() : nullptr, dgamma.data_ptr(), dbeta.data_ptr(),
                                  a.data_ptr<float>(), static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                                  static_cast<int>(C), dtype_code(weight), training, cur_stream(), with_dx),
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

// the same gather with the source pointers in the kernel arguments (<= kPackArgPtrs
// tensors; 0 = a parameter without a gradient): no device pointer table to upload
void pack_grads_ptrs(const at::Tensor& chunks, const std::vector<int64_t>& ptrs, at::Tensor dst, double scale) {
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong && chunks.dim() == 2 &&
                  chunks.size(1) == 3 && chunks.is_contiguous(),
              "pack_grads_ptrs: chunk table must be a contiguous int64 [n, 3] GPU tensor");
  TORCH_CHECK(static_cast<int>(ptrs.size()) <= kdl::kPackArgPtrs, "pack_grads_ptrs: at most ", kdl::kPackArgPtrs,
              " tensors (use pack_grads with a device pointer table)");
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "pack_grads_ptrs: dst must be contiguous on GPU");
  kdl::PackPtrs a{};
  for (size_t i = 0; i < ptrs.size(); ++i) a.p[i] = reinterpret_cast<const void*>(ptrs[i]);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  check_hip(kdl::pack_tensors(reinterpret_cast<const kdl::PackChunk*>(chunks.data_ptr<int64_t>()),
                              static_cast<int>(chunks.size(0)), nullptr, dst.data_ptr(), dtype_code(dst),
                              static_cast<float>(scale), cur_stream(), &a),
            "pack_tensors");
}

void transpose_tiles(const at::Tensor& table) {
  static_assert(sizeof(kdl::TransposeTile) == 40, "TransposeTile layout");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.dim() == 2 && table.size(1) == 5 &&
                  table.is_contiguous(),
              "transpose_tiles: table must be a contiguous int64 [n, 5] GPU tensor "
              "(src, dst, rows|cols<<32, r0|c0<<32, src_ld|dst_ld<<32)");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  check_hip(kdl::transpose_tiles(reinterpret_cast<const kdl::TransposeTile*>(table.data_ptr<int64_t>()),
                                 static_cast<int>(table.size(0)), cur_stream()),
            "transpose_tiles");
}

// ------------------------------------------------------------------ P2P all-reduce
// IPC plumbing is stateless here: python (kubedl_amd/parallel/p2p.py) owns the
// exchanged handles, the mapped peer pointers and the epoch counter.
py::tuple ipc_handle(const at::Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "ipc_handle: GPU tensor required");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(t.device());
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  check_hip(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(t.data_ptr())),
            "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  check_hip(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)), "hipIpcGetMemHandle");
  const int64_t off = reinterpret_cast<const char*>(t.data_ptr()) - reinterpret_cast<const char*>(base);
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), off);
}

int64_t ipc_open(const std::string& handle, int64_t device) {
  TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "ipc_open: bad handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  check_hip(hipSetDevice(static_cast<int>(device)), "hipSetDevice");
  void* p = nullptr;
  check_hip(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return reinterpret_cast<int64_t>(p);
}

void ipc_close(int64_t base) {
  check_hip(hipIpcCloseMemHandle(reinterpret_cast<void*>(base)), "hipIpcCloseMemHandle");
}

at::Tensor p2p_signal_alloc(int64_t device) {
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, device));
  const size_t bytes = kdl::kP2PSignalWords * sizeof(uint32_t);
  void* p = nullptr;
  // uncached: flags are polled across GPUs
  check_hip(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
  check_hip(hipMemset(p, 0, bytes), "hipMemset");
  check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return at::from_blob(p, {static_cast<int64_t>(bytes)}, [](void* q) { (void)hipFree(q); },
                       at::TensorOptions().dtype(at::kByte).device(c10::DeviceType::CUDA, device));
}

// host-mapped error word: returns (host pointer, device pointer)
py::tuple p2p_error_word() {
  void* h = nullptr;
  check_hip(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
  std::memset(h, 0, 64);
  void* d = nullptr;
  check_hip(hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer");
  return py::make_tuple(reinterpret_cast<int64_t>(h), reinterpret_cast<int64_t>(d));
}

void p2p_error_free(int64_t host) { (void)hipHostFree(reinterpret_cast<void*>(host)); }

void p2p_allreduce(const std::vector<int64_t>& bufs, const std::vector<int64_t>& sigs, int64_t err_dev,
                   int64_t rank, int64_t nbytes, int64_t epoch, double scale, bool bf16, double timeout_s,
                   bool oneshot) {
  const int64_t world = static_cast<int64_t>(bufs.size());
  TORCH_CHECK(world >= 1 && world <= kdl::kP2PMaxRanks && static_cast<int64_t>(sigs.size()) == world,
              "p2p_allreduce: 1..8 ranks, one buffer and one signal pointer per rank");
  TORCH_CHECK(rank >= 0 && rank < world, "p2p_allreduce: rank out of range");
  TORCH_CHECK(nbytes > 0 && nbytes % 16 == 0 && nbytes / 16 < (int64_t(1) << 28),
              "p2p_allreduce: bucket bytes must be a positive multiple of 16 below 4 GiB");
  kdl::P2PArgs a{};
  for (int64_t j = 0; j < world; ++j) {
    TORCH_CHECK(bufs[j] % 16 == 0 && bufs[j] != 0 && sigs[j] != 0, "p2p_allreduce: unaligned or null pointer");
    a.buf[j] = reinterpret_cast<void*>(bufs[j]);
    a.sig[j] = reinterpret_cast<uint32_t*>(sigs[j]);
  }
  a.err = reinterpret_cast<uint32_t*>(err_dev);
  a.timeout_ticks = static_cast<uint64_t>(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  a.units = static_cast<uint32_t>(nbytes / 16);
  a.epoch = static_cast<uint32_t>(epoch);
  a.scale = static_cast<float>(scale);
  a.rank = static_cast<int>(rank);
  a.world = static_cast<int>(world);
  TORCH_CHECK(!oneshot || nbytes / 16 <= kdl::p2p_oneshot_max_units(), "p2p_allreduce: bucket too large for one-shot");
  check_hip(kdl::p2p_allreduce(a, bf16, oneshot, cur_stream()), "p2p_allreduce");
}

// ------------------------------------------------------------------ GBDT
std::vector<at::Tensor> gbdt_grad_hess(const at::Tensor& pred, const at::Tensor& y, int64_t obj) {
  TORCH_CHECK(pred.is_cuda() && pred.scalar_type() == at::kFloat && pred.dim() == 2 && pred.is_contiguous(),
              "gbdt_grad_hess: pred fp32 [n, K] contiguous");
  TORCH_CHECK(y.scalar_type() == at::kFloat && y.is_contiguous() && y.numel() == pred.size(0),
              "gbdt_grad_hess: y fp32 [n]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(pred.device());
  auto g = at::empty_like(pred), h = at::empty_like(pred);
  check_hip(kdl::gbdt_grad_hess(pred.data_ptr<float>(), y.data_ptr<float>(), pred.size(0),
                                static_cast<int>(pred.size(1)), static_cast<int>(obj), g.data_ptr<float>(),
                                h.data_ptr<float>(), cur_stream()),
            "gbdt_grad_hess");
  return {g, h};
}

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

// The device grower's quantised histogram (gbdt_hist_wq) over nodes = consecutive
// row ranges seg[j]..seg[j+1] of ``rows``, with the grower's fixed-point scale
// from {max |g|, max h} of all rows: [nodes, F, B, 2] fp32 (a test hook: the
// grower calls the launcher natively).
at::Tensor gbdt_hist_quant(const at::Tensor& bins, const at::Tensor& grad, const at::Tensor& hess,
                           const at::Tensor& rows, const at::Tensor& seg, int64_t num_bins, int64_t rpb) {
  TORCH_CHECK(bins.is_cuda() && bins.scalar_type() == at::kByte && bins.dim() == 2 && bins.is_contiguous(),
              "gbdt_hist_quant: contiguous uint8 bins [N, F]");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && hess.scalar_type() == at::kFloat && grad.is_contiguous() &&
                  hess.is_contiguous() && grad.numel() == bins.size(0) && hess.numel() == grad.numel(),
              "gbdt_hist_quant: fp32 g/h [N]");
  TORCH_CHECK(rows.scalar_type() == at::kInt && seg.scalar_type() == at::kInt && rows.is_contiguous() &&
                  seg.is_contiguous() && seg.numel() >= 2, "gbdt_hist_quant: int32 rows / seg");
  TORCH_CHECK(num_bins >= 2 && num_bins <= 256 && rpb >= 64 && rpb <= 4096, "gbdt_hist_quant: bins / rpb");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bins.device());
  const int64_t nb = seg.numel() - 1, F = bins.size(1), N = bins.size(0);
  auto ghmax = at::empty({2}, grad.options());
  auto hist = at::zeros({nb, F, num_bins, 2}, grad.options());
  auto blo = seg.slice(0, 0, nb).contiguous(), bhi = seg.slice(0, 1, nb + 1).contiguous();
  auto chunk_off = at::empty({nb + 1}, seg.options());
  check_hip(kdl::gbdt_gh_absmax(grad.data_ptr<float>(), hess.data_ptr<float>(), static_cast<int>(N),
                                ghmax.data_ptr<float>(), cur_stream()), "gbdt_gh_absmax");
  const int max_chunks = static_cast<int>((N + rpb - 1) / rpb + nb);
  check_hip(kdl::gbdt_hist_wq(bins.data_ptr<uint8_t>(), grad.data_ptr<float>(), hess.data_ptr<float>(), 1,
                              rows.data_ptr<int32_t>(), blo.data_ptr<int32_t>(), bhi.data_ptr<int32_t>(),
                              chunk_off.data_ptr<int32_t>(), static_cast<int>(nb), max_chunks, static_cast<int>(rpb),
                              static_cast<int>(F), static_cast<int>(num_bins), ghmax.data_ptr<float>(),
                              hist.data_ptr<float>(), cur_stream()), "gbdt_hist_wq");
  return hist;
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
                                 bin.data_ptr<int32_t>(), gl.data_ptr<float>(), hl.data_ptr<float>(), nullptr,
                                 cur_stream()),
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
at::Tensor gemm_bias_act(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& bias, bool relu,
                         bool trans_w) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "gemm_bias_act: bf16 GPU operands");
  // trans_w: C = A W with W [K, N] (the data gradient through an nn.Linear weight), else C = A W^T, W [N, K]
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(trans_w ? 0 : 1),
              trans_w ? "gemm_bias_act: A [M,K], W [K,N]" : "gemm_bias_act: A [M,K], W [N,K]");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous(), "gemm_bias_act: contiguous operands");
  TORCH_CHECK(a.size(1) % 8 == 0, "gemm_bias_act: K must be a multiple of 8 (16-byte rows)");
  const int64_t M = a.size(0), N = w.size(trans_w ? 1 : 0), K = a.size(1);
  TORCH_CHECK(!trans_w || N % 8 == 0, "gemm_bias_act: W [K, N] needs N % 8 == 0");
// bias read in its own dtype (bf16 or fp32): no conversion launch
  const void* bp = nullptr;
  bool b16 = false;
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->scalar_type() == at::kBFloat16 || bias->scalar_type() == at::kFloat ? bias->contiguous()
                                                                                   : bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b.is_cuda() && b.numel() == N, "gemm_bias_act: bias size");
    b16 = b.scalar_type() == at::kBFloat16;
    bp = b.data_ptr();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto c = at::empty({M, N}, a.options());
  check_hip(kdl::gemm_bias_act(a.data_ptr(), w.data_ptr(), bp, b16, c.data_ptr(), static_cast<int>(M),
                               static_cast<int>(N), static_cast<int>(K), relu, trans_w, cur_stream()),
            "gemm_bias_act");
  return c;
}

// ticket counters of the in-launch reductions (zeroed once; every kernel re-arms
// its own): slot 0 = head_bce_fwd, 1 = head_bce_bwd, 64.. = relu_bwd_dbias.  One
// set per (device, stream): launches on ONE stream are ordered, so they may share
// a counter; two streams running the same kernel at once must not (a block would
// count the other launch's arrivals and reduce partials that are not ready).
static at::Tensor ticket_counters(const at::Tensor& like, int64_t base) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(static_cast<int>(like.get_device()), cur_stream());
  auto it = cache.find(key);
  if (it == cache.end()) it = cache.insert_or_assign(key, at::zeros({1 << 14}, like.options().dtype(at::kInt))).first;
  return it->second.narrow(0, base, (1 << 14) - base);
}

std::vector<at::Tensor> relu_bwd_dbias(const at::Tensor& dy, const c10::optional<at::Tensor>& y, bool db_bf16) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 2 && dy.is_contiguous(),
              "relu_bwd_dbias: dy bf16 [M,N] contiguous");
  TORCH_CHECK(dy.size(1) % 8 == 0, "relu_bwd_dbias: N % 8 == 0");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  const bool has_y = y.has_value() && y->defined();
  at::Tensor dz = has_y ? at::empty_like(dy) : dy;
  if (has_y) TORCH_CHECK(y->sizes() == dy.sizes() && y->is_contiguous(), "relu_bwd_dbias: y shape");
  const int M = static_cast<int>(dy.size(0)), N = static_cast<int>(dy.size(1));
  auto db = at::empty({N}, dy.options().dtype(db_bf16 ? at::kBFloat16 : at::kFloat));
  auto part = at::empty({std::max(1, kdl::relu_bwd_dbias_parts(M, N)), N}, dy.options().dtype(at::kFloat));
  TORCH_CHECK((N + 255) / 256 <= (1 << 14) - 64, "relu_bwd_dbias: N too wide for the ticket slots");
  auto cnt = ticket_counters(dy, 64);
  check_hip(kdl::relu_bwd_dbias(dy.data_ptr(), has_y ? y->data_ptr() : nullptr, dz.data_ptr(), part.data_ptr<float>(),
                                reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), db.data_ptr(), db_bf16, M, N,
                                cur_stream()),
            "relu_bwd_dbias");
  return {dz, db};
}

// dz_prev = (dz W) * [y > 0], db_prev = sum_m dz_prev (bf16): the tower's data gradient through the
// previous layer's ReLU with that layer's bias gradient, in one launch (replaces gemm + relu_bwd_dbias)
std::vector<at::Tensor> gemm_dgrad_relu(const at::Tensor& dz, const at::Tensor& w, const at::Tensor& y) {
  TORCH_CHECK(dz.is_cuda() && dz.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  y.scalar_type() == at::kBFloat16, "gemm_dgrad_relu: bf16 GPU operands");
  TORCH_CHECK(dz.dim() == 2 && w.dim() == 2 && dz.size(1) == w.size(0), "gemm_dgrad_relu: dz [M, K], W [K, N]");
  TORCH_CHECK(dz.is_contiguous() && w.is_contiguous() && y.is_contiguous(), "gemm_dgrad_relu: contiguous operands");
  const int64_t M = dz.size(0), N = w.size(1), K = dz.size(1);
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "gemm_dgrad_relu: K % 8 == 0 and N % 8 == 0");
  TORCH_CHECK(y.dim() == 2 && y.size(0) == M && y.size(1) == N, "gemm_dgrad_relu: y [M, N]");
  TORCH_CHECK((N + 63) / 64 <= (1 << 14) - 8192, "gemm_dgrad_relu: N too wide for the ticket slots");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dz.device());
  auto c = at::empty({M, N}, dz.options());
  auto db = at::empty({N}, dz.options());
  const int tm = kdl::gemm_dgrad_relu_tiles_m(static_cast<int>(M), static_cast<int>(N));
  auto part = at::empty({tm, N}, dz.options().dtype(at::kFloat));
  auto cnt = ticket_counters(dz, 8192);
  check_hip(kdl::gemm_dgrad_relu(dz.data_ptr(), w.data_ptr(), y.data_ptr(), c.data_ptr(), part.data_ptr<float>(),
                                 reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), db.data_ptr(), static_cast<int>(M),
                                 static_cast<int>(N), static_cast<int>(K), cur_stream()),
            "gemm_dgrad_relu");
  return {c, db};
}

static void check_head(const at::Tensor& x, const at::Tensor& w, const char* who) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(),
              who, ": x bf16 [M,K] contiguous");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() == x.size(1), who, ": w bf16 [K]");
  TORCH_CHECK(x.size(1) % 8 == 0, who, ": K % 8 == 0");
}

std::vector<at::Tensor> head_bce_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
                                     const at::Tensor& y) {
  check_head(x, w, "head_bce_fwd");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK((b.scalar_type() == at::kFloat || b.scalar_type() == at::kBFloat16) && b.numel() == 1 && b.is_cuda(),
              "head_bce_fwd: bias f32 / bf16 [1]");
  TORCH_CHECK(y.scalar_type() == at::kFloat && y.numel() == M && y.is_contiguous(), "head_bce_fwd: labels f32 [M]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto opt = x.options().dtype(at::kFloat);
  auto logit = at::empty({M}, opt), dlogit = at::empty({M}, opt), part = at::empty({kdl::head_bce_fwd_blocks(static_cast<int>(M))}, opt);
  auto loss = at::empty({1}, opt);
  auto cnt = ticket_counters(x, 0);
  check_hip(kdl::head_bce_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), b.scalar_type() == at::kBFloat16,
                              y.data_ptr<float>(), static_cast<int>(M), static_cast<int>(K), logit.data_ptr<float>(),
                              dlogit.data_ptr<float>(), part.data_ptr<float>(),
                              reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), loss.data_ptr<float>(), cur_stream()),
            "head_bce_fwd");
  return {logit, dlogit, part, loss};
}

std::vector<at::Tensor> head_bce_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& dlogit,
                                     double scale, const c10::optional<at::Tensor>& gscale, bool relu_x) {
  check_head(x, w, "head_bce_bwd");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(dlogit.scalar_type() == at::kFloat && dlogit.numel() == M && dlogit.is_contiguous(),
              "head_bce_bwd: dlogit f32 [M]");
  const bool has_g = gscale.has_value() && gscale->defined();
  if (has_g)
    TORCH_CHECK(gscale->scalar_type() == at::kFloat && gscale->numel() == 1 && gscale->is_cuda(),
                "head_bce_bwd: gscale f32 [1]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int nb = kdl::head_bce_bwd_blocks(static_cast<int>(M));
  auto opt = x.options().dtype(at::kFloat);
  auto dx = at::empty_like(x), dwp = at::empty({nb, K}, opt), dbp = at::empty({nb}, opt);
  auto dw = at::empty({K}, x.options()), db = at::empty({1}, x.options());  // bf16, summed in block order
  auto cnt = ticket_counters(x, 1);
  // relu_x: x is a ReLU output; dx masked by x > 0 and dbx = its column sums (bf16 [K])
  at::Tensor dbxp, dbx;
  if (relu_x) {
    dbxp = at::empty({nb, K}, opt);
    dbx = at::empty({K}, x.options());
  }
  check_hip(kdl::head_bce_bwd(x.data_ptr(), w.data_ptr(), dlogit.data_ptr<float>(), static_cast<float>(scale),
                              has_g ? gscale->data_ptr<float>() : nullptr, static_cast<int>(M), static_cast<int>(K),
                              dx.data_ptr(), dwp.data_ptr<float>(), dbp.data_ptr<float>(),
                              reinterpret_cast<unsigned*>(cnt.data_ptr<int>()), dw.data_ptr(), db.data_ptr(),
                              cur_stream(), relu_x ? dbxp.data_ptr<float>() : nullptr,
                              relu_x ? dbx.data_ptr() : nullptr),
            "head_bce_bwd");
  if (relu_x) return {dx, dw, db, dwp, dbp, dbx};
  return {dx, dw, db, dwp, dbp};
}

void embed_gather_cast(const at::Tensor& table, const at::Tensor& uniq, const at::Tensor& inv, int64_t F,
                       at::Tensor out, int64_t col0, const c10::optional<at::Tensor>& dense, int64_t tail) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.is_contiguous() &&
                  (table.scalar_type() == at::kFloat || table.scalar_type() == at::kBFloat16),
              "embed_gather_cast: fp32 or bf16 table [V, D]");
  TORCH_CHECK(uniq.scalar_type() == at::kLong && inv.scalar_type() == at::kLong && uniq.is_contiguous() &&
                  inv.is_contiguous() && uniq.numel() >= 1,
              "embed_gather_cast: int64 uniq / inv");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.scalar_type() == at::kBFloat16, "embed_gather_cast: bf16 out");
  const int64_t D = table.size(1), n = inv.numel();
  TORCH_CHECK(F > 0 && n % F == 0 && out.size(0) * F == n && col0 + F * D <= out.size(1), "embed_gather_cast: shapes");
  TORCH_CHECK(D % 8 == 0 && out.stride(0) % 8 == 0 && col0 % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(table.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "embed_gather_cast: 16-byte rows (D, the out row stride and col0 multiples of 8)");
  // tail: the next ``tail`` columns after the last field (dense fp32 [B, nd], then zeros) in the same launch
  const bool has_d = dense.has_value() && dense->defined();
  int64_t nd = 0;
  if (tail > 0) {
    TORCH_CHECK(tail % 8 == 0 && col0 + F * D + tail <= out.size(1), "embed_gather_cast: tail columns");
    if (has_d) {
      TORCH_CHECK(dense->is_cuda() && dense->scalar_type() == at::kFloat && dense->is_contiguous() && dense->dim() == 2 &&
                      dense->size(0) == out.size(0) && dense->size(1) <= tail,
                  "embed_gather_cast: dense fp32 [B, nd <= tail] contiguous");
      nd = dense->size(1);
    }
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  check_hip(kdl::embed_gather_cast(table.data_ptr(), table.scalar_type() == at::kBFloat16, uniq.data_ptr<int64_t>(),
                                   inv.data_ptr<int64_t>(),
                                   static_cast<int>(n), static_cast<int>(F), static_cast<int>(D), out.data_ptr(),
                                   static_cast<int>(out.stride(0)), static_cast<int>(col0), cur_stream(),
                                   has_d && tail > 0 ? dense->data_ptr<float>() : nullptr, static_cast<int>(nd),
                                   static_cast<int>(tail > 0 ? tail : 0)),
            "embed_gather_cast");
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

const int* opt_count(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "ucount: int32 GPU tensor");
  return t->data_ptr<int>();
}

at::Tensor segment_reduce(const at::Tensor& rows, int64_t F, int64_t col0, int64_t D, const at::Tensor& order,
                          const at::Tensor& seg, const c10::optional<at::Tensor>& ucount,
                          const c10::optional<at::Tensor>& out_rows, const c10::optional<at::Tensor>& out_opt) {
  TORCH_CHECK(rows.is_cuda() && rows.dim() == 2 && rows.stride(1) == 1, "segment_reduce: rows [B, ld]");
  TORCH_CHECK(order.scalar_type() == at::kLong && seg.scalar_type() == at::kLong && order.is_contiguous() &&
                  seg.is_contiguous() && order.device() == rows.device() && seg.device() == rows.device(),
              "segment_reduce: int64 order/seg on rows' device");
  TORCH_CHECK(order.numel() == rows.size(0) * F && col0 + F * D <= rows.size(1), "segment_reduce: shapes");
  const int64_t U = seg.numel() - 1;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(rows.device());
  // out_rows / out: segment u's sum lands in out[out_rows[u]] (the exchange send
  // buffer, rows >= out.size(0) dropped) instead of a fresh [U, D] tensor
  const bool mapped = out_rows.has_value() && out_rows->defined();
  TORCH_CHECK(mapped == (out_opt.has_value() && out_opt->defined()), "segment_reduce: out_rows and out go together");
  at::Tensor out;
  if (mapped) {
    out = *out_opt;
    TORCH_CHECK(out_rows->scalar_type() == at::kLong && out_rows->is_contiguous() && out_rows->numel() >= U,
                "segment_reduce: int64 out_rows [U]");
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 2 &&
                    out.size(1) == D,
                "segment_reduce: fp32 out [rows, D]");
  } else {
    out = at::empty({U, D}, rows.options().dtype(at::kFloat));
  }
  check_hip(kdl::segment_reduce(rows.data_ptr(), dtype_code(rows), static_cast<int>(F), static_cast<int>(rows.stride(0)),
                                static_cast<int>(col0), order.data_ptr<int64_t>(), seg.data_ptr<int64_t>(),
                                static_cast<int>(U), static_cast<int>(D), out.data_ptr<float>(), cur_stream(),
                                opt_count(ucount), order.numel(), mapped ? out_rows->data_ptr<int64_t>() : nullptr,
                                mapped ? out.size(0) : 0),
            "segment_reduce");
  return out;
}

// sync-free one-owner push in one launch: the per-id gradient sums of rows
// (segment_reduce) applied by Adagrad to table/accum rows rows_local[u]
void segment_reduce_adagrad(const at::Tensor& rows, int64_t F, int64_t col0, int64_t D, const at::Tensor& order,
                            const at::Tensor& seg, const c10::optional<at::Tensor>& ucount, const at::Tensor& rows_local,
                            at::Tensor table, at::Tensor accum, double lr, double eps, double scale) {
  TORCH_CHECK(rows.is_cuda() && rows.dim() == 2 && rows.stride(1) == 1, "segment_reduce_adagrad: rows [B, ld]");
  TORCH_CHECK(order.scalar_type() == at::kLong && seg.scalar_type() == at::kLong && order.is_contiguous() &&
                  seg.is_contiguous() && order.device() == rows.device() && seg.device() == rows.device(),
              "segment_reduce_adagrad: int64 order/seg on rows' device");
  TORCH_CHECK(order.numel() == rows.size(0) * F && col0 + F * D <= rows.size(1), "segment_reduce_adagrad: shapes");
  const int64_t U = seg.numel() - 1;
  TORCH_CHECK(rows_local.scalar_type() == at::kLong && rows_local.is_contiguous() && rows_local.numel() >= U &&
                  rows_local.device() == rows.device(),
              "segment_reduce_adagrad: int64 rows_local [U] on rows' device");
  TORCH_CHECK(table.device() == rows.device() && accum.device() == rows.device() && table.scalar_type() == at::kFloat && table.is_contiguous() && table.dim() == 2 &&
                  table.size(1) == D && accum.sizes() == table.sizes() && accum.scalar_type() == at::kFloat &&
                  accum.is_contiguous(),
              "segment_reduce_adagrad: fp32 table / accum [rows, D]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(rows.device());
  check_hip(kdl::segment_reduce_adagrad(rows.data_ptr(), dtype_code(rows), static_cast<int>(F),
                                        static_cast<int>(rows.stride(0)), static_cast<int>(col0),
                                        order.data_ptr<int64_t>(), seg.data_ptr<int64_t>(), static_cast<int>(U),
                                        static_cast<int>(D), opt_count(ucount), order.numel(),
                                        rows_local.data_ptr<int64_t>(), table.size(0), table.data_ptr<float>(),
                                        accum.data_ptr<float>(), static_cast<float>(lr), static_cast<float>(eps),
                                        static_cast<float>(scale), cur_stream()),
            "segment_reduce_adagrad");
}

// Fixed-capacity exchange routing (csrc/ctr.hip a2a_route): send [W * (cap + 1)]
// int64 and rslot [n] int64 are written; count: int32 [1] live ids (or None = n)
void a2a_route(const at::Tensor& uniq, const c10::optional<at::Tensor>& count, const at::Tensor& owner_rank,
               int64_t W, int64_t cap, at::Tensor send, at::Tensor rslot) {
  TORCH_CHECK(uniq.is_cuda() && uniq.scalar_type() == at::kLong && uniq.is_contiguous(), "a2a_route: int64 uniq");
  TORCH_CHECK(owner_rank.scalar_type() == at::kLong && owner_rank.is_contiguous() && owner_rank.numel() >= 1,
              "a2a_route: int64 owner_rank");
  TORCH_CHECK(W >= 1 && W <= kdl::a2a_max_world() && cap >= 1, "a2a_route: 1 <= W <= ", kdl::a2a_max_world());
  TORCH_CHECK(send.scalar_type() == at::kLong && send.is_contiguous() && send.numel() >= W * (cap + 1),
              "a2a_route: int64 send [W * (cap + 1)]");
  const int64_t n = uniq.numel();
  TORCH_CHECK(rslot.scalar_type() == at::kLong && rslot.is_contiguous() && rslot.numel() >= n, "a2a_route: rslot [n]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(uniq.device());
  auto cnt = at::empty({kdl::a2a_route_blocks(static_cast<int>(n)) * W}, uniq.options().dtype(at::kInt));
  check_hip(kdl::a2a_route(uniq.data_ptr<int64_t>(), opt_count(count), static_cast<int>(n),
                           owner_rank.data_ptr<int64_t>(), static_cast<int>(owner_rank.numel()), static_cast<int>(W),
                           static_cast<int>(cap), cnt.data_ptr<int>(), send.data_ptr<int64_t>(),
                           rslot.data_ptr<int64_t>(), cur_stream()),
            "a2a_route");
}

// owner side: (rows [n, D] fp32, local [n] int64) for the requested ids req [n]
std::vector<at::Tensor> a2a_serve(const at::Tensor& table, const at::Tensor& req, int64_t n_own, bool rows_bf16,
                                  const c10::optional<at::Tensor>& slotmap, int64_t call, int64_t cap, int64_t W) {
  TORCH_CHECK(table.is_cuda() && table.dim() == 2 && table.is_contiguous() && table.scalar_type() == at::kFloat &&
                  table.size(1) % 4 == 0 && reinterpret_cast<uintptr_t>(table.data_ptr()) % 16 == 0,
              "a2a_serve: fp32 table [V, D], D % 4 == 0");
  TORCH_CHECK(req.scalar_type() == at::kLong && req.is_contiguous(), "a2a_serve: int64 req");
  const int64_t n = req.numel(), D = table.size(1);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  auto rows = at::empty({n, D}, table.options().dtype(rows_bf16 ? at::kBFloat16 : at::kFloat));
  auto local = at::empty({n}, req.options());
  int64_t* sm = nullptr;
  if (slotmap.has_value()) {
    TORCH_CHECK(slotmap->scalar_type() == at::kLong && slotmap->is_contiguous() &&
                    slotmap->numel() >= table.size(0) * W && W >= 1 && cap >= 1 && n == W * cap,
                "a2a_serve: slotmap int64 [nrows * W], n = W * cap");
    sm = slotmap->data_ptr<int64_t>();
  }
  check_hip(kdl::a2a_serve(table.data_ptr<float>(), req.data_ptr<int64_t>(), static_cast<int>(n),
                           static_cast<int>(n_own), static_cast<int>(D), rows.data_ptr(), rows_bf16,
                           local.data_ptr<int64_t>(), cur_stream(), sm, call, static_cast<int>(cap),
                           static_cast<int>(W), table.size(0)),
            "a2a_serve");
  return {rows, local};
}

void segment_adagrad(const at::Tensor& grads, const at::Tensor& order, const at::Tensor& seg,
                     const at::Tensor& rows_local, at::Tensor table, at::Tensor accum, double lr, double eps,
                     double scale, const c10::optional<at::Tensor>& ucount) {
  TORCH_CHECK(grads.is_cuda() && grads.scalar_type() == at::kFloat && grads.is_contiguous(), "segment_adagrad: grads");
  TORCH_CHECK(table.scalar_type() == at::kFloat && accum.scalar_type() == at::kFloat && table.is_contiguous() &&
                  accum.is_contiguous() && table.sizes() == accum.sizes(),
              "segment_adagrad: fp32 table/accum");
  TORCH_CHECK(grads.size(1) == table.size(1), "segment_adagrad: D mismatch");
  TORCH_CHECK(rows_local.numel() == seg.numel() - 1 && order.numel() == grads.size(0), "segment_adagrad: shapes");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  check_hip(kdl::segment_adagrad(grads.data_ptr<float>(), order.data_ptr<int64_t>(), seg.data_ptr<int64_t>(),
                                 rows_local.data_ptr<int64_t>(), static_cast<int>(seg.numel() - 1),
                                 static_cast<int>(table.size(1)), table.size(0), table.data_ptr<float>(),
                                 accum.data_ptr<float>(),
                                 static_cast<float>(lr), static_cast<float>(eps), static_cast<float>(scale),
                                 cur_stream(), opt_count(ucount)),
            "segment_adagrad");
}

// owner update of a fixed exchange (csrc/ctr.hip a2a_stamp + a2a_adagrad): no
// de-duplication pass; slotmap int64 [nrows * W] kept by the caller (zero
// initially), call = 1, 2, ... per update
void a2a_owner_update(const at::Tensor& grads, const at::Tensor& local, int64_t cap, int64_t W, at::Tensor slotmap,
                      int64_t call, at::Tensor table, at::Tensor accum, double lr, double eps, double scale,
                      bool stamped) {
  TORCH_CHECK(grads.is_cuda() && grads.scalar_type() == at::kFloat && grads.is_contiguous() && grads.dim() == 2,
              "a2a_owner_update: fp32 grads [S, D]");
  const int64_t S = grads.size(0), D = grads.size(1);
  TORCH_CHECK(local.scalar_type() == at::kLong && local.is_contiguous() && local.numel() == S,
              "a2a_owner_update: int64 local [S]");
  TORCH_CHECK(W >= 1 && cap >= 1 && S == W * cap && S < (int64_t(1) << 31), "a2a_owner_update: S = W * cap < 2^31");
  TORCH_CHECK(table.scalar_type() == at::kFloat && accum.scalar_type() == at::kFloat && table.is_contiguous() &&
                  accum.is_contiguous() && table.sizes() == accum.sizes() && table.dim() == 2 && table.size(1) == D,
              "a2a_owner_update: fp32 table/accum [nrows, D]");
  const int64_t nrows = table.size(0);
  TORCH_CHECK(slotmap.scalar_type() == at::kLong && slotmap.is_contiguous() && slotmap.numel() >= nrows * W,
              "a2a_owner_update: slotmap int64 [nrows * W]");
  TORCH_CHECK(call >= 1 && call < (int64_t(1) << 31), "a2a_owner_update: call in [1, 2^31)");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  check_hip(kdl::a2a_owner_update(grads.data_ptr<float>(), local.data_ptr<int64_t>(), static_cast<int>(S),
                                  static_cast<int>(cap), static_cast<int>(W), static_cast<int>(D), nrows,
                                  slotmap.data_ptr<int64_t>(), call, table.data_ptr<float>(),
                                  accum.data_ptr<float>(), static_cast<float>(lr), static_cast<float>(eps),
                                  static_cast<float>(scale), cur_stream(), stamped),
            "a2a_owner_update");
}

int64_t dedup_table_slots(int64_t n) { return kdl::dedup_table_slots(static_cast<int>(n)); }

// the CSR half of dedup_csr, later in the step (sizes from that dedup_csr call;
// sizes and cursor are scratch of the long-segment sort afterwards)
void csr_from_inverse_only(const at::Tensor& inv, at::Tensor sizes, const at::Tensor& count, at::Tensor bsum,
                           at::Tensor cursor, at::Tensor seg, at::Tensor order) {
  const int64_t n = inv.numel();
  TORCH_CHECK(n > 0 && inv.is_cuda() && inv.scalar_type() == at::kLong && inv.is_contiguous(), "csr: inv");
  TORCH_CHECK(sizes.scalar_type() == at::kInt && sizes.numel() >= n + 1 && cursor.scalar_type() == at::kInt &&
                  cursor.numel() >= n + 1 && count.scalar_type() == at::kInt && bsum.scalar_type() == at::kInt &&
                  bsum.numel() >= kdl::csr_bsum_slots(static_cast<int>(n)),
              "csr: int32 sizes/cursor/count/bsum");
  TORCH_CHECK(seg.scalar_type() == at::kLong && seg.numel() >= n + 1 && order.scalar_type() == at::kLong &&
                  order.numel() >= n,
              "csr: int64 seg/order");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(inv.device());
  check_hip(kdl::csr_from_inverse(inv.data_ptr<int64_t>(), static_cast<int>(n), sizes.data_ptr<int>(),
                                  count.data_ptr<int>(), bsum.data_ptr<int>(), cursor.data_ptr<int>(),
                                  seg.data_ptr<int64_t>(), order.data_ptr<int64_t>(), cur_stream()),
            "csr_from_inverse");
}

// ws: (keys int64 [T] filled -1, slot_of int32 [n], slot_uid int32 [T], bsum int32 [T/1024 + n/1024 + 2],
//      sizes int32 [n + 1], cursor int32 [n + 1]); returns nothing, fills uniq/inv/count/seg/order
void dedup_csr(const at::Tensor& ids, at::Tensor keys, at::Tensor slot_of, at::Tensor slot_uid, at::Tensor bsum,
               at::Tensor sizes, at::Tensor cursor, at::Tensor uniq, at::Tensor inv, at::Tensor count, at::Tensor seg,
               at::Tensor order, bool with_csr) {
  const int64_t n = ids.numel();
  const int64_t T = kdl::dedup_table_slots(static_cast<int>(n));
  auto chk = [](const at::Tensor& t, at::ScalarType st, int64_t numel, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == st && t.is_contiguous() && t.numel() >= numel, "dedup_csr: ", what);
  };
  chk(ids, at::kLong, n, "ids int64");
  chk(keys, at::kLong, T, "keys int64 [T]");
  chk(slot_of, at::kInt, n, "slot_of");
  chk(slot_uid, at::kInt, T, "slot_uid");
  chk(bsum, at::kInt, T / 1024 + (n + 1) / 1024 + 2, "bsum");
  chk(sizes, at::kInt, n + 1, "sizes");
  chk(cursor, at::kInt, n + 1, "cursor");
  chk(uniq, at::kLong, n, "uniq");
  chk(inv, at::kLong, n, "inv");
  chk(count, at::kInt, 1, "count");
  chk(seg, at::kLong, n + 1, "seg");
  chk(order, at::kLong, n, "order");
  TORCH_CHECK(n > 0 && n < (1 << 30), "dedup_csr: 0 < n < 2^30");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(ids.device());
  check_hip(kdl::dedup_ids(ids.data_ptr<int64_t>(), static_cast<int>(n), keys.data_ptr(), static_cast<int>(T),
                           slot_of.data_ptr<int>(), slot_uid.data_ptr<int>(), bsum.data_ptr<int>(),
                           uniq.data_ptr<int64_t>(), inv.data_ptr<int64_t>(), count.data_ptr<int>(),
                           sizes.data_ptr<int>(), cur_stream()),
            "dedup_ids");
  if (with_csr)
    check_hip(kdl::csr_from_inverse(inv.data_ptr<int64_t>(), static_cast<int>(n), sizes.data_ptr<int>(),
                                    count.data_ptr<int>(), bsum.data_ptr<int>(), cursor.data_ptr<int>(),
                                    seg.data_ptr<int64_t>(), order.data_ptr<int64_t>(), cur_stream()),
              "csr_from_inverse");
}


// ------------------------------------------------------------------ engine ops: fused 1x1 convs + staged BN
// These are the raw building blocks of kubedl_amd.models.resnet_engine (explicit
// forward/backward of the ResNet-50 bottleneck).  Outputs are preallocated by the
// caller; every pointer is checked for device, dtype, density and extent here
// because the kernels trust their shape arguments.
const void* opt_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}
float* opt_fptr(const c10::optional<at::Tensor>& t) {
  if (!(t.has_value() && t->defined())) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "expected a contiguous fp32 tensor");
  return t->data_ptr<float>();
}
void need_bf16(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, what, ": bf16 GPU tensor expected");
  // 4-D activations must be NHWC in memory (row = pixel, channels contiguous)
  TORCH_CHECK(is_nhwc_dense(t), what, ": channels_last-dense (4-D) or contiguous (2-D) tensor expected");
  TORCH_CHECK(t.numel() >= numel, what, ": too small (", t.numel(), " < ", numel, ")");
}
void need_opt_bf16(const c10::optional<at::Tensor>& t, int64_t numel, const char* what) {
  if (t.has_value() && t->defined()) need_bf16(*t, numel, what);
}
void need_opt_f32(const c10::optional<at::Tensor>& t, int64_t numel, const char* what) {
  if (t.has_value() && t->defined())
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() >= numel, what,
                ": fp32 contiguous GPU tensor of >= ", numel, " elements expected");
}

// ------------------------------------------------------------------ classifier head (csrc/head.hip)
std::vector<int64_t> head_splits(int64_t Nb, int64_t C, int64_t L) {
  int s1 = 0, s2 = 0;
  kdl::head_splits(static_cast<int>(Nb), static_cast<int>(C), static_cast<int>(L), &s1, &s2);
  return {s1, s2};
}

void need_f32(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() >= numel, what,
              ": fp32 contiguous GPU tensor of >= ", numel, " elements expected");
}

// x [Nb, C, H, W] channels_last (the last block's output); ws = (feat, part1, lrow, dl, dlT)
void head_forward(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b, const at::Tensor& y,
                  at::Tensor feat, at::Tensor part1, at::Tensor lrow, at::Tensor dl, at::Tensor dlT) {
  TORCH_CHECK(x.dim() == 4 && is_nhwc_dense(x), "head_forward: x must be [Nb, C, H, W] channels_last");
  const int64_t Nb = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == C && w.is_contiguous(), "head_forward: w must be [L, C] contiguous");
  const int64_t L = w.size(0);
  TORCH_CHECK(C % 8 == 0 && L <= 8192, "head_forward: C % 8 == 0, L <= 8192");
  need_bf16(x, Nb * C * HW, "head x");
  need_bf16(w, L * C, "head w");
  need_opt_bf16(b, L, "head b");
  TORCH_CHECK(!b.has_value() || !b->defined() || b->is_contiguous(), "head b: contiguous");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kLong && y.is_contiguous() && y.numel() == Nb, "head y: int64 [Nb]");
  auto sp = head_splits(Nb, C, L);
  need_bf16(feat, Nb * C, "head feat");
  need_f32(part1, sp[0] * Nb * L, "head part1");
  need_f32(lrow, Nb, "head lrow");
  need_bf16(dl, Nb * kdl::head_lpad(static_cast<int>(L)), "head dl");
  need_bf16(dlT, L * Nb, "head dlT");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::head_forward(x.data_ptr(), static_cast<int>(Nb), static_cast<int>(HW), static_cast<int>(C),
                              w.data_ptr(), opt_ptr(b), static_cast<int>(L), y.data_ptr<int64_t>(), feat.data_ptr(),
                              part1.data_ptr<float>(), lrow.data_ptr<float>(), dl.data_ptr(), dlT.data_ptr(),
                              cur_stream()),
            "head_forward");
}

void head_backward(const at::Tensor& feat, const at::Tensor& w, const at::Tensor& dl, const at::Tensor& dlT,
                   at::Tensor part2, at::Tensor dfeat, at::Tensor dW, at::Tensor db, const at::Tensor& lrow,
                   at::Tensor loss) {
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "head_backward: w [L, C] contiguous");
  const int64_t L = w.size(0), C = w.size(1), Nb = feat.numel() / C;
  TORCH_CHECK(Nb % 8 == 0 && C % 8 == 0, "head_backward: Nb, C multiples of 8");
  auto sp = head_splits(Nb, C, L);
  need_bf16(feat, Nb * C, "head feat");
  need_bf16(w, L * C, "head w");
  need_bf16(dl, Nb * kdl::head_lpad(static_cast<int>(L)), "head dl");
  need_bf16(dlT, L * Nb, "head dlT");
  need_f32(part2, sp[1] * Nb * C, "head part2");
  need_bf16(dfeat, Nb * C, "head dfeat");
  need_bf16(dW, L * C, "head dW");
  TORCH_CHECK(dW.is_contiguous() && db.is_contiguous(), "head dW/db: contiguous");
  need_bf16(db, L, "head db");
  need_f32(lrow, Nb, "head lrow");
  need_f32(loss, 1, "head loss");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  check_hip(kdl::head_backward(feat.data_ptr(), w.data_ptr(), dl.data_ptr(), dlT.data_ptr(), static_cast<int>(Nb),
                               static_cast<int>(C), static_cast<int>(L), part2.data_ptr<float>(), dfeat.data_ptr(),
                               dW.data_ptr(), db.data_ptr(), lrow.data_ptr<float>(), loss.data_ptr<float>(),
                               cur_stream()),
            "head_backward");
}

// BN finalize folded into the next conv GEMM launch (csrc/bn_fin.h): bn_fin_arm
// names the workspace(s) whose BN the next conv1x1_gemm / conv3x3_gemm /
// conv3x3_s2_dgrad call on this thread finalizes in its epilogue's last
// arriving blocks; the launch consumes (clears) the arming.
struct FinArm {
  float* ws = nullptr;
  float* ws2 = nullptr;
  float M = 0.f;
  int64_t C = 0;
};
thread_local FinArm g_fin_arm;

void bn_fin_arm(const at::Tensor& ws, const c10::optional<at::Tensor>& ws2, int64_t C, int64_t M) {
  TORCH_CHECK(C > 0 && C <= 2048 && C % 64 == 0, "bn_fin_arm: C in 64..2048, C % 64 == 0");
  auto chk = [&](const at::Tensor& w) {
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() &&
                    w.numel() >= kdl::bn_workspace_floats(static_cast<int>(C)),
                "bn_fin_arm: workspace must be fp32 >= bn_workspace_floats(C)");
  };
  chk(ws);
  g_fin_arm.ws = ws.data_ptr<float>();
  g_fin_arm.ws2 = nullptr;
  if (ws2.has_value() && ws2->defined()) {
    chk(*ws2);
    g_fin_arm.ws2 = ws2->data_ptr<float>();
  }
  g_fin_arm.M = static_cast<float>(M);
  g_fin_arm.C = C;
}

// consumed at the top of every GEMM binding, so a launch that throws still
// disarms; applied to the launch arguments once they are built
FinArm take_fin_arm() {
  const FinArm f = g_fin_arm;
  g_fin_arm = FinArm{};
  return f;
}

// BN-backward-apply prologue armed for the next conv1x1_gemm (on its A operand:
// A' = k A + c1 x + c0, the output of bn_stage_bwd_apply) or conv1x1_wgrad (on
// its G operand) call on this thread, so the consumer GEMM computes that
// tensor while staging it instead of a separate apply pass writing it to HBM
// and the consumers reading it back; ``out`` (optional) receives it, for a
// consumer that still reads it materialised.  Consumed (cleared) by the launch.
struct BwdArm {
  const void* x = nullptr;
  const float* coef = nullptr;
  const float* coef2 = nullptr;  // res 2: the downsample BN's scale | shift
  void* out = nullptr;
  int64_t C = 0, rows = 0;
  int res = 0;              // 1: forward residual-apply prologue (bn_res_pro_arm)
  uint8_t* bits = nullptr;  // its packed ReLU mask out
};
thread_local BwdArm g_bwd_arm;

void bn_bwd_pro_arm(const at::Tensor& x, const at::Tensor& ws, int64_t C, const c10::optional<at::Tensor>& out) {
  TORCH_CHECK(C > 0 && C % 64 == 0 && x.numel() % C == 0, "bn_bwd_pro_arm: C % 64 == 0 dividing x");
  need_bf16(x, x.numel(), "bn_bwd_pro_arm x");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous() &&
                  ws.numel() >= kdl::bn_workspace_floats(static_cast<int>(C)),
              "bn_bwd_pro_arm: workspace must be fp32 >= bn_workspace_floats(C)");
  g_bwd_arm.x = x.data_ptr();
  g_bwd_arm.coef = ws.data_ptr<float>() + 32 * 4 * C + 2 * C;  // ws_bcoef (csrc/bn_act.hip)
  g_bwd_arm.out = nullptr;
  if (out.has_value() && out->defined()) {
    need_bf16(*out, x.numel(), "bn_bwd_pro_arm out");
    g_bwd_arm.out = out->data_ptr();
  }
  g_bwd_arm.C = C;
  g_bwd_arm.rows = x.numel() / C;
}

// The next conv1x1_gemm (forward, STATS) applies the previous block's closing
// BN + residual + ReLU to its A = that block's conv3 output:
// A' = relu(A * coef[k] + coef[K + k] + res), written through to ``out`` with
// its packed ReLU mask in ``bits`` [M, K / 8] -- bit-identical to
// bn_stage_fwd_apply(A, ws, res, ..., out, bits) (csrc/conv1x1.hip PRO_RES).
// coefd (optional) [2C]: ``res`` is a downsample branch's BN input, the residual
// res * coefd[k] + coefd[C + k] (bn_stage_fwd_apply's dual form); coef and coefd
// are read by the kernel from both tables (no concatenated copy)
void bn_res_pro_arm(const at::Tensor& res, const at::Tensor& coef, int64_t C, const at::Tensor& out,
                    const at::Tensor& bits, const c10::optional<at::Tensor>& coefd) {
  TORCH_CHECK(C > 0 && C % 64 == 0 && res.numel() % C == 0, "bn_res_pro_arm: C % 64 == 0 dividing res");
  need_bf16(res, res.numel(), "bn_res_pro_arm res");
  need_bf16(out, res.numel(), "bn_res_pro_arm out");
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() >= 2 * C,
              "bn_res_pro_arm: coef fp32 [2C] (scale | shift)");
  TORCH_CHECK(bits.is_cuda() && bits.scalar_type() == at::kByte && bits.is_contiguous() &&
                  bits.numel() >= res.numel() / 8,
              "bn_res_pro_arm: bits uint8 [M * C / 8]");
  g_bwd_arm.x = res.data_ptr();
  g_bwd_arm.coef = coef.data_ptr<float>();
  g_bwd_arm.res = 1;
  if (coefd.has_value() && coefd->defined()) {
    TORCH_CHECK(coefd->is_cuda() && coefd->scalar_type() == at::kFloat && coefd->is_contiguous() &&
                    coefd->numel() >= 2 * C,
                "bn_res_pro_arm: coefd fp32 [2C]");
    g_bwd_arm.coef2 = coefd->data_ptr<float>();
    g_bwd_arm.res = 2;
  }
  g_bwd_arm.out = out.data_ptr();
  g_bwd_arm.C = C;
  g_bwd_arm.rows = res.numel() / C;
  g_bwd_arm.bits = bits.data_ptr<uint8_t>();
}

BwdArm take_bwd_arm() {
  const BwdArm b = g_bwd_arm;
  g_bwd_arm = BwdArm{};
  return b;
}

void apply_fin_arm(const FinArm& f, kdl::Conv1x1Args& a, int64_t N, int64_t epi) {
  if (!f.ws) return;
  TORCH_CHECK(f.C == N, "bn_fin_arm: armed for C = ", f.C, ", the GEMM has N = ", N);
  TORCH_CHECK(epi == 1 || epi == 2 || epi == 3, "bn_fin_arm: the GEMM's epilogue produces no BN sums");
  a.fin_ws = f.ws;
  a.fin_ws2 = f.ws2;
  a.fin_M = f.M;
}

// the layer's finalize descriptor into the workspace tail (once; the pointers are stable)
void bn_fin_desc(at::Tensor ws, const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                 at::Tensor rm, at::Tensor rv, at::Tensor save_mean, at::Tensor save_invstd,
                 const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta, double momentum,
                 double eps) {
  const int64_t C = rm.numel();
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous() &&
                  ws.numel() >= kdl::bn_workspace_floats(static_cast<int>(C)),
              "bn_fin_desc: workspace");
  for (const at::Tensor* t : {&rm, &rv, &save_mean, &save_invstd})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C,
                "bn_fin_desc: fp32 per-channel tensors");
  kdl::BnFinDesc d{};
  int pt = -1;
  for (const c10::optional<at::Tensor>* t : {&gamma, &beta, &dgamma, &dbeta}) {
    if (!t->has_value() || !(*t)->defined()) continue;
    TORCH_CHECK((*t)->is_cuda() && (*t)->is_contiguous() && (*t)->numel() == C, "bn_fin_desc: affine tensors");
    const int this_pt = (*t)->scalar_type() == at::kBFloat16 ? 1 : 0;
    TORCH_CHECK((*t)->scalar_type() == at::kBFloat16 || (*t)->scalar_type() == at::kFloat, "bn_fin_desc: dtype");
    TORCH_CHECK(pt < 0 || pt == this_pt, "bn_fin_desc: affine tensors of one dtype");
    pt = this_pt;
  }
  d.gamma = opt_ptr(gamma);
  d.beta = opt_ptr(beta);
  d.rm = rm.data_ptr<float>();
  d.rv = rv.data_ptr<float>();
  d.save_mean = save_mean.data_ptr<float>();
  d.save_invstd = save_invstd.data_ptr<float>();
  d.dgamma = const_cast<void*>(opt_ptr(dgamma));
  d.dbeta = const_cast<void*>(opt_ptr(dbeta));
  d.momentum = static_cast<float>(momentum);
  d.eps = static_cast<float>(eps);
  d.C = static_cast<int>(C);
  d.pt_bf16 = pt == 1 ? 1 : 0;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(ws.device());
  check_hip(hipMemcpy(ws.data_ptr<float>() + kdl::fin_desc_off(static_cast<int>(C)), &d, sizeof(d),
                      hipMemcpyHostToDevice),
            "bn_fin_desc");
}

void conv1x1_gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor C, int64_t M, int64_t N, int64_t K,
                  int64_t Hout, int64_t Wout, int64_t Hin, int64_t Win, int64_t stride,
                  const c10::optional<at::Tensor>& pro_coef, int64_t epi, const c10::optional<at::Tensor>& shift,
                  const c10::optional<at::Tensor>& acc, const c10::optional<at::Tensor>& ex,
                  const c10::optional<at::Tensor>& emean, const c10::optional<at::Tensor>& ecoef,
                  const c10::optional<at::Tensor>& eres, int64_t res_stride, int64_t res_H, int64_t res_W,
                  const c10::optional<at::Tensor>& ebits, const c10::optional<at::Tensor>& ex2,
                  const c10::optional<at::Tensor>& emean2, const c10::optional<at::Tensor>& acc2) {
  const FinArm fin = take_fin_arm();
  const BwdArm bw = take_bwd_arm();
  TORCH_CHECK(K % 64 == 0 && N % 64 == 0 && M > 0, "conv1x1_gemm: need K % 64 == 0, N % 64 == 0");
  TORCH_CHECK(epi >= 0 && epi <= 4, "conv1x1_gemm: epi 0 (plain) .. 4 (res)");
  if (bw.x) {
    TORCH_CHECK(bw.C == K && bw.rows == M, "bn_bwd_pro_arm: armed for [", bw.rows, ", ", bw.C,
                "], the GEMM's A is [", M, ", ", K, "]");
    if (bw.res) {
      TORCH_CHECK(stride == 1 && !opt_ptr(pro_coef) && epi == 1 && K <= 2048,
                  "conv1x1_gemm: the residual-apply prologue serves dense forward (STATS) GEMMs, K <= 2048");
    } else {
      TORCH_CHECK(stride == 1 && !opt_ptr(pro_coef) && epi != 1,
                  "conv1x1_gemm: the backward-apply prologue serves dense data-gradient GEMMs");
    }
  }
  const int64_t rows_in = stride > 1 ? (M / (Hout * Wout)) * Hin * Win : M;
  if (stride > 1) TORCH_CHECK(M % (Hout * Wout) == 0 && (Hout - 1) * stride < Hin && (Wout - 1) * stride < Win,
                              "conv1x1_gemm: gather geometry");
  need_bf16(A, rows_in * K, "conv1x1_gemm A");
  need_bf16(B, N * K, "conv1x1_gemm B");
  need_bf16(C, M * N, "conv1x1_gemm C");
  need_opt_f32(pro_coef, 2 * K, "pro_coef");
  const int64_t rep = 32 * 2 * N;
  if (epi == 1) { TORCH_CHECK(opt_ptr(shift) && opt_ptr(acc), "epi STATS needs shift, acc"); need_opt_f32(shift, N, "shift"); need_opt_f32(acc, rep, "acc"); }
  if (epi == 2) {
    TORCH_CHECK(opt_ptr(ex) && opt_ptr(emean) && opt_ptr(ecoef) && opt_ptr(acc), "epi MASKX needs ex, emean, ecoef, acc");
    need_opt_bf16(ex, M * N, "ex"); need_opt_f32(emean, N, "emean"); need_opt_f32(ecoef, 2 * N, "ecoef"); need_opt_f32(acc, rep, "acc");
  }
  if (epi == 3 || epi == 4) {
    TORCH_CHECK(opt_ptr(eres), "epi RES/RESBITS needs eres");
    if (res_stride > 1) {
      TORCH_CHECK(M % (res_H * res_W) == 0, "conv1x1_gemm: residual geometry");
      const int64_t ho = (res_H + res_stride - 1) / res_stride, wo = (res_W + res_stride - 1) / res_stride;
      need_opt_bf16(eres, (M / (res_H * res_W)) * ho * wo * N, "eres");
    } else {
      need_opt_bf16(eres, M * N, "eres");
    }
  }
  if (epi == 3) {
    TORCH_CHECK(opt_ptr(ex) && opt_ptr(emean) && opt_ptr(acc) && opt_ptr(ebits),
                "epi RESBITS needs ex, emean, acc, ebits");
    need_opt_bf16(ex, M * N, "ex");
    need_opt_f32(emean, N, "emean"); need_opt_f32(acc, rep, "acc");
    TORCH_CHECK(ebits->scalar_type() == at::kByte && ebits->is_contiguous() && ebits->numel() >= M * N / 8, "ebits");
    if (opt_ptr(ex2)) {
      need_opt_bf16(ex2, M * N, "ex2"); need_opt_f32(emean2, N, "emean2"); need_opt_f32(acc2, rep, "acc2");
      TORCH_CHECK(opt_ptr(emean2) && opt_ptr(acc2), "ex2 needs emean2, acc2");
    }
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  kdl::Conv1x1Args a{};
  a.A = A.data_ptr(); a.B = B.data_ptr(); a.C = C.data_ptr();
  a.M = static_cast<int>(M); a.N = static_cast<int>(N); a.K = static_cast<int>(K);
  a.Hout = static_cast<int>(Hout); a.Wout = static_cast<int>(Wout); a.Hin = static_cast<int>(Hin);
  a.Win = static_cast<int>(Win); a.stride = static_cast<int>(stride);
  a.pro_coef = opt_fptr(pro_coef);
  a.epi = static_cast<int>(epi);
  a.shift = opt_fptr(shift); a.acc = opt_fptr(acc);
  a.ex = opt_ptr(ex); a.emean = opt_fptr(emean); a.ecoef = opt_fptr(ecoef);
  a.eres = opt_ptr(eres); a.res_stride = static_cast<int>(res_stride); a.res_H = static_cast<int>(res_H);
  a.res_W = static_cast<int>(res_W);
  a.ebits = ebits.has_value() && ebits->defined() ? ebits->data_ptr<uint8_t>() : nullptr;
  a.ex2 = opt_ptr(ex2); a.emean2 = opt_fptr(emean2); a.acc2 = opt_fptr(acc2);
  a.bx = bw.x; a.bcoef = bw.coef; a.bcoef2 = bw.coef2; a.aout = bw.out;
  if (bw.res) { a.bres = bw.res; a.obits = bw.bits; }
  apply_fin_arm(fin, a, N, epi);
  check_hip(kdl::conv1x1_gemm(a, cur_stream()), "conv1x1_gemm");
}

int64_t conv3x3_wgrad_slabs(int64_t Nb, int64_t H, int64_t W, int64_t Cin, int64_t Cout, int64_t stride) {
  return kdl::conv3x3_wgrad_slabs(static_cast<int>(Nb), static_cast<int>(H), static_cast<int>(W),
                                  static_cast<int>(Cin), static_cast<int>(Cout), static_cast<int>(stride));
}

int64_t conv1x1_wgrad_splits(int64_t M, int64_t N, int64_t K, bool solo) {
  return kdl::conv1x1_wgrad_splits(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), solo);
}

// 3x3 / pad 1 convolution as an implicit GEMM on the same MFMA kernel:
// y[Nb, Ho, Wo, Cout] = conv(pro(x)[Nb, H, W, Cin], W[Cout][3][3][Cin]).
//   epi 0 PLAIN, 1 STATS (shift = rm, acc = fwd replicas), 2 MASKX (dgrad:
//   ex = that BN's input [M, Cout], emean, ecoef).  pro_coef [2Cin] applies
//   relu(x*scale + shift) to in-image taps; padding taps are zero.
// conv3x3_aout_arm(a): the next conv3x3_gemm with a BN + ReLU prologue also
// writes relu(B(x)) into ``a`` (the 56x56 halo kernel; elsewhere it fails)
thread_local void* g_aout_arm = nullptr;
thread_local int64_t g_aout_n = 0;
void conv3x3_aout_arm(const c10::optional<at::Tensor>& a) {
  if (a) {
    TORCH_CHECK(a->is_cuda() && a->scalar_type() == at::kBFloat16, "conv3x3_aout_arm: bf16 GPU tensor");
    g_aout_arm = a->data_ptr();
    g_aout_n = a->numel();
  } else {
    g_aout_arm = nullptr;
    g_aout_n = 0;
  }
}

void conv3x3_gemm(const at::Tensor& A, const at::Tensor& W, at::Tensor C, int64_t Nb, int64_t H, int64_t Wd,
                  int64_t Cin, int64_t Cout, int64_t stride, const c10::optional<at::Tensor>& pro_coef, int64_t epi,
                  const c10::optional<at::Tensor>& shift, const c10::optional<at::Tensor>& acc,
                  const c10::optional<at::Tensor>& ex, const c10::optional<at::Tensor>& emean,
                  const c10::optional<at::Tensor>& ecoef) {
  const FinArm fin = take_fin_arm();
  void* aout = g_aout_arm;
  const int64_t aout_n = g_aout_n;
  g_aout_arm = nullptr;
  g_aout_n = 0;
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0 && Nb > 0 && stride >= 1, "conv3x3_gemm: need Cin, Cout % 64 == 0");
  TORCH_CHECK(!aout || (opt_ptr(pro_coef) && epi == 1 && stride == 1 && aout_n == Nb * H * Wd * Cin),
              "conv3x3_gemm: the write-through needs the prologue, STATS, stride 1 and an [N, H, W, Cin] tensor");
  TORCH_CHECK(epi == 0 || epi == 1 || epi == 2, "conv3x3_gemm: epilogue must be PLAIN, STATS or MASKX");
  TORCH_CHECK(!(epi == 2 && opt_ptr(pro_coef)), "conv3x3_gemm: MASKX runs without a prologue");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (Wd - 1) / stride + 1;
  const int64_t M = Nb * Ho * Wo, K = 9 * Cin, N = Cout;
  need_bf16(A, Nb * H * Wd * Cin, "conv3x3_gemm A");
  need_bf16(W, N * K, "conv3x3_gemm W");
  need_bf16(C, M * N, "conv3x3_gemm C");
  need_opt_f32(pro_coef, 2 * Cin, "pro_coef");
  const int64_t rep = 32 * 2 * N;
  if (epi == 1) { TORCH_CHECK(opt_ptr(shift) && opt_ptr(acc), "epi STATS needs shift, acc"); need_opt_f32(shift, N, "shift"); need_opt_f32(acc, rep, "acc"); }
  if (epi == 2) {
    TORCH_CHECK(opt_ptr(ex) && opt_ptr(emean) && opt_ptr(ecoef) && opt_ptr(acc), "epi MASKX needs ex, emean, ecoef, acc");
    need_opt_bf16(ex, M * N, "ex"); need_opt_f32(emean, N, "emean"); need_opt_f32(ecoef, 2 * N, "ecoef"); need_opt_f32(acc, rep, "acc");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  kdl::Conv1x1Args a{};
  a.A = A.data_ptr(); a.B = W.data_ptr(); a.C = C.data_ptr();
  a.M = static_cast<int>(M); a.N = static_cast<int>(N); a.K = static_cast<int>(K);
  a.Hout = static_cast<int>(Ho); a.Wout = static_cast<int>(Wo); a.Hin = static_cast<int>(H);
  a.Win = static_cast<int>(Wd); a.stride = static_cast<int>(stride);
  a.ksize = 3; a.Cin = static_cast<int>(Cin);
  a.pro_coef = opt_fptr(pro_coef);
  a.epi = static_cast<int>(epi);
  a.shift = opt_fptr(shift); a.acc = opt_fptr(acc);
  a.ex = opt_ptr(ex); a.emean = opt_fptr(emean); a.ecoef = opt_fptr(ecoef);
  a.res_stride = 1;
  a.aout = aout;
  apply_fin_arm(fin, a, N, epi);
  check_hip(kdl::conv1x1_gemm(a, cur_stream()), "conv3x3_gemm");
}

// ResNet stem 7x7 / stride 2 / pad 3 conv, [Nb, 3, H, W] -> [Nb, 64, OH, OW] (csrc/stem.hip).
void stem7x7_fwd(const at::Tensor& x, const at::Tensor& wp, at::Tensor y, const c10::optional<at::Tensor>& shift,
                 const c10::optional<at::Tensor>& acc) {
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 3 && is_nhwc_dense(x), "stem7x7_fwd: x must be [Nb, 3, H, W] channels_last");
  const int64_t Nb = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  need_bf16(x, Nb * H * W * 3, "stem7x7_fwd x");
  // wp: the nn.Conv2d weight [64, 3, 7, 7] (reordered inside the kernel) or [64, 224] in K order
  const bool raw_w = wp.numel() == 64 * 3 * 7 * 7;
  need_bf16(wp, raw_w ? 64 * 147 : 64 * 224, "stem7x7_fwd wp");
  TORCH_CHECK(y.dim() == 4 && y.size(0) == Nb && y.size(1) == 64 && y.size(2) == OH && y.size(3) == OW,
              "stem7x7_fwd: y must be [Nb, 64, OH, OW]");
  need_bf16(y, Nb * OH * OW * 64, "stem7x7_fwd y");
  TORCH_CHECK(Nb * OH * OW * 128 < (int64_t(1) << 31), "stem7x7_fwd: 32-bit row offsets");
  TORCH_CHECK(!opt_ptr(acc) || opt_ptr(shift), "stem7x7_fwd: statistics need a shift");
  need_opt_f32(shift, 64, "shift");
  need_opt_f32(acc, 32 * 2 * 64, "acc");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::stem7x7_fwd(x.data_ptr(), wp.data_ptr(), y.data_ptr(), static_cast<int>(Nb), static_cast<int>(H),
                             static_cast<int>(W), opt_fptr(shift), opt_fptr(acc), cur_stream(), raw_w),
            "stem7x7_fwd");
}

// stem weight gradient -> dW [64][224] bf16 (kubedl_amd.ops.conv.stem_weights K order)
// or [64, 3, 7, 7] channels_last (the parameter's own layout)
void stem7x7_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor dw32, at::Tensor dW) {
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 3 && is_nhwc_dense(x), "stem7x7_wgrad: x must be [Nb, 3, H, W] channels_last");
  const int64_t Nb = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == Nb && dy.size(1) == 64 && dy.size(2) == OH && dy.size(3) == OW &&
                  is_nhwc_dense(dy),
              "stem7x7_wgrad: dy must be [Nb, 64, OH, OW] channels_last");
  need_bf16(x, Nb * H * W * 3, "stem7x7_wgrad x");
  need_bf16(dy, Nb * OH * OW * 64, "stem7x7_wgrad dy");
  const bool raw_out = dW.numel() == 64 * 3 * 7 * 7;  // [64, 3, 7, 7] (else [64, 224] K order)
  need_bf16(dW, raw_out ? 64 * 147 : 64 * 224, "stem7x7_wgrad dW");
  const int64_t slabs = kdl::stem7x7_wgrad_slabs(static_cast<int>(Nb), static_cast<int>(H), static_cast<int>(W));
  TORCH_CHECK(dw32.is_cuda() && dw32.scalar_type() == at::kFloat && dw32.is_contiguous() &&
                  dw32.numel() >= slabs * 64 * 224,
              "stem7x7_wgrad: dw32 must hold stem7x7_wgrad_slabs(Nb, H, W) x 64 x 224 fp32");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::stem7x7_wgrad(dy.data_ptr(), x.data_ptr(), dw32.data_ptr<float>(), dW.data_ptr(),
                               static_cast<int>(Nb), static_cast<int>(H), static_cast<int>(W), cur_stream(), raw_out),
            "stem7x7_wgrad");
}

// stem weight gradient with the stem BN + ReLU + max-pool backward folded in
// (after bn_pool_bwd(..., with_dx = false) filled the workspace's coefficients)
void stem7x7_wgrad_bn(const at::Tensor& c0, const at::Tensor& dp, const at::Tensor& idx, const at::Tensor& ws,
                      const at::Tensor& x, at::Tensor dw32, at::Tensor dW) {
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 3 && x.size(2) == 224 && x.size(3) == 224 && is_nhwc_dense(x),
              "stem7x7_wgrad_bn: x must be [Nb, 3, 224, 224] channels_last");
  const int64_t Nb = x.size(0);
  TORCH_CHECK(c0.dim() == 4 && c0.size(0) == Nb && c0.size(1) == 64 && c0.size(2) == 112 && c0.size(3) == 112 &&
                  is_nhwc_dense(c0),
              "stem7x7_wgrad_bn: c0 must be [Nb, 64, 112, 112] channels_last");
  TORCH_CHECK(dp.dim() == 4 && dp.size(0) == Nb && dp.size(1) == 64 && dp.size(2) == 56 && dp.size(3) == 56 &&
                  is_nhwc_dense(dp),
              "stem7x7_wgrad_bn: dp must be [Nb, 64, 56, 56] channels_last");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.numel() == Nb * 56 * 56 * 64,
              "stem7x7_wgrad_bn: idx");
  need_bf16(x, Nb * 224 * 224 * 3, "x");
  need_bf16(c0, Nb * 112 * 112 * 64, "c0");
  need_bf16(dp, Nb * 56 * 56 * 64, "dp");
  const bool raw_out = dW.numel() == 64 * 3 * 7 * 7;
  need_bf16(dW, raw_out ? 64 * 147 : 64 * 224, "dW");
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous() &&
                  ws.numel() >= kdl::bn_workspace_floats(64),
              "stem7x7_wgrad_bn: ws must be the stem BN workspace");
  const int64_t slabs = kdl::stem7x7_wgrad_slabs(static_cast<int>(Nb));
  TORCH_CHECK(dw32.is_cuda() && dw32.scalar_type() == at::kFloat && dw32.is_contiguous() &&
                  dw32.numel() >= slabs * 64 * 224,
              "stem7x7_wgrad_bn: dw32 must hold stem7x7_wgrad_slabs(Nb) x 64 x 224 fp32");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::stem7x7_wgrad_bn(c0.data_ptr(), dp.data_ptr(), idx.data_ptr<uint8_t>(),
                                  ws.data_ptr<float>() + 32 * 4 * 64 /* bn_coef_offset(64) */, x.data_ptr(), dw32.data_ptr<float>(),
                                  dW.data_ptr(), static_cast<int>(Nb), cur_stream(), raw_out),
            "stem7x7_wgrad_bn");
}

// dx of a 3x3 / pad 1 / stride 2 conv: dy [Nb, Hd, Wd, Cd] (channels_last),
// ball = the weights regrouped class-major [N][9 Cd] (kubedl_amd.ops.conv.s2_dgrad_weights),
// dx [Nb, Hx, Wx, N] with Hx = 2 Hd or 2 Hd - 1 (an odd conv input; 0: 2 Hd),
// likewise Wx; epi 0 PLAIN, 2 MASKX (ex = that BN's input [Nb, Hx, Wx, N]).
void conv3x3_s2_dgrad(const at::Tensor& dy, const at::Tensor& ball, at::Tensor dx, int64_t Nb, int64_t Hd,
                      int64_t Wd, int64_t Cd, int64_t N, int64_t epi, const c10::optional<at::Tensor>& acc,
                      const c10::optional<at::Tensor>& ex, const c10::optional<at::Tensor>& emean,
                      const c10::optional<at::Tensor>& ecoef, int64_t Hx, int64_t Wx) {
  const FinArm fin = take_fin_arm();
  TORCH_CHECK(Cd % 64 == 0 && N % 64 == 0 && Nb > 0 && Hd > 0 && Wd > 0, "conv3x3_s2_dgrad: need Cd, N % 64 == 0");
  TORCH_CHECK(epi == 0 || epi == 2, "conv3x3_s2_dgrad: epilogue must be PLAIN or MASKX");
  if (Hx <= 0) Hx = 2 * Hd;
  if (Wx <= 0) Wx = 2 * Wd;
  TORCH_CHECK((Hx == 2 * Hd || Hx == 2 * Hd - 1) && (Wx == 2 * Wd || Wx == 2 * Wd - 1),
              "conv3x3_s2_dgrad: dx must be (2 Hd or 2 Hd - 1) x (2 Wd or 2 Wd - 1)");
  const int64_t Mdx = Nb * Hx * Wx;
  need_bf16(dy, Nb * Hd * Wd * Cd, "conv3x3_s2_dgrad dy");
  need_bf16(ball, N * 9 * Cd, "conv3x3_s2_dgrad ball");
  need_bf16(dx, Mdx * N, "conv3x3_s2_dgrad dx");
  if (epi == 2) {
    TORCH_CHECK(opt_ptr(ex) && opt_ptr(emean) && opt_ptr(ecoef) && opt_ptr(acc), "epi MASKX needs ex, emean, ecoef, acc");
    need_opt_bf16(ex, Mdx * N, "ex"); need_opt_f32(emean, N, "emean"); need_opt_f32(ecoef, 2 * N, "ecoef");
    need_opt_f32(acc, 32 * 2 * N, "acc");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  kdl::Conv1x1Args a{};
  a.A = dy.data_ptr(); a.B = ball.data_ptr(); a.C = dx.data_ptr();
  a.M = static_cast<int>(Nb * Hd * Wd); a.N = static_cast<int>(N); a.K = static_cast<int>(9 * Cd);
  a.Hin = static_cast<int>(Hd); a.Win = static_cast<int>(Wd);
  a.Hout = static_cast<int>(Hx); a.Wout = static_cast<int>(Wx); a.stride = 2;
  a.ksize = 3; a.Cin = static_cast<int>(Cd);
  a.epi = static_cast<int>(epi);
  a.acc = opt_fptr(acc);
  a.ex = opt_ptr(ex); a.emean = opt_fptr(emean); a.ecoef = opt_fptr(ecoef);
  apply_fin_arm(fin, a, N, epi);
  check_hip(kdl::conv3x3_dgrad_s2(a, cur_stream()), "conv3x3_s2_dgrad");
}

void conv1x1_wgrad(const at::Tensor& G, const at::Tensor& A, const c10::optional<at::Tensor>& pro_coef,
                   at::Tensor dw32, const c10::optional<at::Tensor>& dW, double scale, int64_t M, int64_t N, int64_t K,
                   int64_t Hout, int64_t Wout, int64_t Hin, int64_t Win, int64_t stride, bool solo) {
  const BwdArm bw = take_bwd_arm();
  TORCH_CHECK(K % 64 == 0 && N % 64 == 0 && M > 0, "conv1x1_wgrad: need K % 64 == 0, N % 64 == 0");
  if (bw.x) {
    TORCH_CHECK(bw.C == N && bw.rows == M, "bn_bwd_pro_arm: armed for [", bw.rows, ", ", bw.C,
                "], the weight gradient's G is [", M, ", ", N, "]");
    TORCH_CHECK(!bw.out, "conv1x1_wgrad: the G prologue has no write-through");
    TORCH_CHECK(stride == 1 || !opt_ptr(pro_coef), "conv1x1_wgrad: G prologue + A prologue need dense A rows");
  }
  const int64_t rows_in = stride > 1 ? (M / (Hout * Wout)) * Hin * Win : M;
  need_bf16(G, M * N, "conv1x1_wgrad G");
  need_bf16(A, rows_in * K, "conv1x1_wgrad A");
  need_opt_f32(pro_coef, 2 * K, "pro_coef");
  const int64_t slabs =
      kdl::conv1x1_wgrad_splits(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), solo);
  TORCH_CHECK(dw32.is_cuda() && dw32.scalar_type() == at::kFloat && dw32.is_contiguous() &&
                  dw32.numel() >= slabs * N * K,
              "conv1x1_wgrad: dw32 must be fp32 contiguous with conv1x1_wgrad_splits(M, N, K) * N * K elements");
  if (dW.has_value() && dW->defined())
    TORCH_CHECK(dW->is_cuda() && dW->is_contiguous() && dW->numel() == N * K && dW->scalar_type() == at::kBFloat16,
                "conv1x1_wgrad: dW bf16 contiguous [N, K]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(G.device());
  check_hip(kdl::conv1x1_wgrad(G.data_ptr(), A.data_ptr(), opt_fptr(pro_coef), dw32.data_ptr<float>(),
                               dW.has_value() && dW->defined() ? dW->data_ptr() : nullptr, static_cast<float>(scale),
                               static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), static_cast<int>(Hout),
                               static_cast<int>(Wout), static_cast<int>(Hin), static_cast<int>(Win),
                               static_cast<int>(stride), cur_stream(), bw.x, bw.coef, solo),
            "conv1x1_wgrad");
}

// Gram fold (csrc/conv1x1.hip): Q | s of relu(B(X)) into ws, then the folded bf16 dW
int64_t conv1x1_gram_floats(int64_t M, int64_t K) {
  return static_cast<int64_t>(kdl::conv1x1_gram_splits(static_cast<int>(M), static_cast<int>(K))) * (K * K + K);
}

void conv1x1_gram(const at::Tensor& X, const at::Tensor& pro, at::Tensor ws, int64_t M, int64_t K) {
  need_bf16(X, M * K, "conv1x1_gram X");
  need_opt_f32(pro, 2 * K, "conv1x1_gram pro");
  need_opt_f32(ws, conv1x1_gram_floats(M, K), "conv1x1_gram ws");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(X.device());
  check_hip(kdl::conv1x1_gram(X.data_ptr(), pro.data_ptr<float>(), ws.data_ptr<float>(), static_cast<int>(M),
                              static_cast<int>(K), cur_stream()),
            "conv1x1_gram");
}

void gram_fold(const at::Tensor& Gm, const at::Tensor& QS, const at::Tensor& W, const at::Tensor& bcoef, at::Tensor out,
               int64_t N, int64_t K) {
  need_opt_f32(Gm, N * K, "gram_fold G");
  need_opt_f32(QS, K * K + K, "gram_fold Q|s");
  need_opt_f32(bcoef, 3 * N, "gram_fold bcoef");
  need_bf16(W, N * K, "gram_fold W");
  need_bf16(out, N * K, "gram_fold out");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  check_hip(kdl::gram_fold(Gm.data_ptr<float>(), QS.data_ptr<float>(), W.data_ptr(), bcoef.data_ptr<float>(),
                           static_cast<int>(N), static_cast<int>(K), out.data_ptr(), cur_stream()),
            "gram_fold");
}

// fixed-order sum of nsplit fp32 [nk] slabs into the first (fp32, in place)
void slab_reduce_f32(at::Tensor slabs, int64_t nk, int64_t nsplit) {
  TORCH_CHECK(nk % 4 == 0 && nsplit >= 1, "slab_reduce_f32: nk % 4 == 0");
  need_opt_f32(slabs, nk * nsplit, "slab_reduce_f32 slabs");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(slabs.device());
  check_hip(kdl::wgrad_slab_reduce(slabs.data_ptr<float>(), nk, static_cast<int>(nsplit), 1.0f, nullptr,
                                   cur_stream()),
            "slab_reduce_f32");
}

void conv3x3_wgrad(const at::Tensor& G, const at::Tensor& A, const c10::optional<at::Tensor>& pro_coef,
                   at::Tensor dw32, const c10::optional<at::Tensor>& dW, double scale, int64_t Nb, int64_t H,
                   int64_t Wd, int64_t Cin, int64_t Cout, int64_t stride) {
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0 && Nb > 0 && stride >= 1, "conv3x3_wgrad: need Cin, Cout % 64 == 0");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (Wd - 1) / stride + 1, M = Nb * Ho * Wo, K = 9 * Cin;
  need_bf16(G, M * Cout, "conv3x3_wgrad G");
  need_bf16(A, Nb * H * Wd * Cin, "conv3x3_wgrad A");
  need_opt_f32(pro_coef, 2 * Cin, "pro_coef");
  const int64_t slabs = kdl::conv1x1_wgrad_splits(static_cast<int>(M), static_cast<int>(Cout), static_cast<int>(K));
  TORCH_CHECK(dw32.is_cuda() && dw32.scalar_type() == at::kFloat && dw32.is_contiguous() &&
                  dw32.numel() >= slabs * Cout * K,
              "conv3x3_wgrad: dw32 must hold conv1x1_wgrad_splits(M, Cout, 9 Cin) * Cout * 9 Cin fp32");
  if (dW.has_value() && dW->defined()) {
    need_bf16(*dW, Cout * K, "conv3x3_wgrad dW");  // OHWI: channels_last [Cout, Cin, 3, 3] or [Cout, 9 Cin]
    TORCH_CHECK(dW->numel() == Cout * K, "conv3x3_wgrad: dW must have Cout * 9 * Cin elements");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(G.device());
  check_hip(kdl::conv3x3_wgrad(G.data_ptr(), A.data_ptr(), opt_fptr(pro_coef), dw32.data_ptr<float>(), dw32.numel(),
                               dW.has_value() && dW->defined() ? dW->data_ptr() : nullptr, static_cast<float>(scale),
                               static_cast<int>(Nb), static_cast<int>(H), static_cast<int>(Wd), static_cast<int>(Cin),
                               static_cast<int>(Cout), static_cast<int>(stride), cur_stream()),
            "conv3x3_wgrad");
}

int64_t pdtype_of(const at::Tensor& t) { return t.scalar_type() == at::kBFloat16 ? 1 : 0; }

void need_ws(const at::Tensor& ws, int64_t C) {
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous() &&
                  ws.numel() >= kdl::bn_workspace_floats(static_cast<int>(C)),
              "bn stage: workspace must be fp32 >= bn_workspace_floats(C)");
}

int64_t bn_coef_offset(int64_t C) { return 32 * 4 * C; }

void bn_stage_fwd_stats(const at::Tensor& x, at::Tensor ws, int64_t M, int64_t C) {
  need_bf16(x, M * C, "bn_stage_fwd_stats x");
  need_ws(ws, C);
  TORCH_CHECK(C % 8 == 0, "C % 8");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::bn_stage_fwd_stats(x.data_ptr(), ws.data_ptr<float>(), M, static_cast<int>(C), cur_stream()),
            "bn_stage_fwd_stats");
}

void bn_stage_fwd_finalize(const c10::optional<at::Tensor>& x, const c10::optional<at::Tensor>& shift, at::Tensor ws,
                           int64_t M, int64_t C, const at::Tensor& gamma, const at::Tensor& beta, at::Tensor rm,
                           at::Tensor rv, at::Tensor save_mean, at::Tensor save_invstd, bool training,
                           double momentum, double eps) {
  TORCH_CHECK(opt_ptr(x) || opt_ptr(shift), "bn_stage_fwd_finalize: x or shift");
  need_opt_bf16(x, C, "x");
  need_opt_f32(shift, C, "shift");
  need_ws(ws, C);
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && gamma.scalar_type() == beta.scalar_type(), "gamma/beta");
  for (const at::Tensor* t : {&rm, &rv, &save_mean, &save_invstd})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == C && t->is_contiguous(), "fp32 [C] stats");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(ws.device());
  check_hip(kdl::bn_stage_fwd_finalize(opt_ptr(x), opt_fptr(shift), ws.data_ptr<float>(), M, static_cast<int>(C),
                                       gamma.data_ptr(), beta.data_ptr(), rm.data_ptr<float>(), rv.data_ptr<float>(),
                                       save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                                       static_cast<int>(pdtype_of(gamma)), training, static_cast<float>(momentum),
                                       static_cast<float>(eps), cur_stream()),
            "bn_stage_fwd_finalize");
}

void bn_stage_fwd_apply(const at::Tensor& x, const at::Tensor& ws, const c10::optional<at::Tensor>& res,
                        const c10::optional<at::Tensor>& xd, const c10::optional<at::Tensor>& wsd, at::Tensor y,
                        const c10::optional<at::Tensor>& mbits, int64_t M, int64_t C, bool relu) {
  need_bf16(x, M * C, "x");
  need_bf16(y, M * C, "y");
  need_ws(ws, C);
  need_opt_bf16(res, M * C, "res");
  need_opt_bf16(xd, M * C, "xd");
  if (opt_ptr(xd)) need_ws(*wsd, C);
  uint8_t* mb = nullptr;
  if (mbits.has_value() && mbits->defined()) {
    TORCH_CHECK(mbits->scalar_type() == at::kByte && mbits->is_contiguous() && mbits->numel() >= M * C / 8, "mbits");
    mb = mbits->data_ptr<uint8_t>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::bn_stage_fwd_apply(x.data_ptr(), ws.data_ptr<float>(), opt_ptr(res), opt_ptr(xd),
                                    opt_ptr(xd) ? wsd->data_ptr<float>() : nullptr, y.data_ptr(), mb, M,
                                    static_cast<int>(C), relu, cur_stream()),
            "bn_stage_fwd_apply");
}

void bn_stage_bwd_mask_reduce(const at::Tensor& dy, int64_t dy_rows_per_img, double dy_scale, const at::Tensor& mbits,
                              const at::Tensor& x, const at::Tensor& mean, at::Tensor gout, at::Tensor ws, int64_t M,
                              int64_t C, const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& mean2,
                              const c10::optional<at::Tensor>& ws2) {
  if (opt_ptr(x2)) {
    need_opt_bf16(x2, M * C, "x2");
    need_opt_f32(mean2, C, "mean2");
    TORCH_CHECK(opt_ptr(mean2) && opt_ptr(ws2), "x2 needs mean2, ws2");
    need_ws(*ws2, C);
  }
  need_bf16(dy, dy_rows_per_img > 0 ? (M / dy_rows_per_img) * C : M * C, "dy");
  if (dy_rows_per_img > 0) TORCH_CHECK(M % dy_rows_per_img == 0, "dy rows per image");
  need_bf16(x, M * C, "x");
  need_bf16(gout, M * C, "gout");
  need_ws(ws, C);
  TORCH_CHECK(mbits.scalar_type() == at::kByte && mbits.numel() >= M * C / 8, "mbits");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && mean.numel() == C, "mean");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::bn_stage_bwd_mask_reduce(dy.data_ptr(), static_cast<int>(dy_rows_per_img),
                                          static_cast<float>(dy_scale), mbits.data_ptr<uint8_t>(), x.data_ptr(),
                                          mean.data_ptr<float>(), gout.data_ptr(), ws.data_ptr<float>(), M,
                                          static_cast<int>(C), opt_ptr(x2), opt_fptr(mean2),
                                          opt_ptr(x2) ? ws2->data_ptr<float>() : nullptr, cur_stream()),
            "bn_stage_bwd_mask_reduce");
}

void check_bn_params(const at::Tensor& gamma, const at::Tensor& beta, const at::Tensor& mean,
                     const at::Tensor& invstd, int64_t C) {
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && gamma.scalar_type() == beta.scalar_type() &&
                  gamma.is_contiguous() && beta.is_contiguous(),
              "gamma/beta [C], same dtype");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && invstd.scalar_type() == at::kFloat && mean.numel() == C &&
                  invstd.numel() == C,
              "mean/invstd fp32 [C]");
}

void bn_stage_bwd_reduce(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& beta,
                         const at::Tensor& mean, const at::Tensor& invstd, at::Tensor ws, int64_t M, int64_t C,
                         bool relu_mask_x) {
  need_bf16(dy, M * C, "dy");
  need_bf16(x, M * C, "x");
  need_ws(ws, C);
  check_bn_params(gamma, beta, mean, invstd, C);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::bn_stage_bwd_reduce(dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                     mean.data_ptr<float>(), invstd.data_ptr<float>(), ws.data_ptr<float>(), M,
                                     static_cast<int>(C), relu_mask_x, static_cast<int>(pdtype_of(gamma)),
                                     cur_stream()),
            "bn_stage_bwd_reduce");
}

void bn_stage_bwd_apply_maskx(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& gamma,
                              const at::Tensor& beta, const at::Tensor& mean, const at::Tensor& invstd,
                              const at::Tensor& ws, at::Tensor dx, int64_t M, int64_t C) {
  need_bf16(dy, M * C, "dy");
  need_bf16(x, M * C, "x");
  need_bf16(dx, M * C, "dx");
  need_ws(ws, C);
  check_bn_params(gamma, beta, mean, invstd, C);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::bn_stage_bwd_apply_maskx(dy.data_ptr(), x.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                          mean.data_ptr<float>(), invstd.data_ptr<float>(), ws.data_ptr<float>(),
                                          dx.data_ptr(), M, static_cast<int>(C), static_cast<int>(pdtype_of(gamma)),
                                          cur_stream()),
            "bn_stage_bwd_apply_maskx");
}

void bn_stage_bwd_finalize(at::Tensor ws, int64_t M, int64_t C, const at::Tensor& gamma, const at::Tensor& mean,
                           const at::Tensor& invstd, at::Tensor dgamma, at::Tensor dbeta, bool training) {
  need_ws(ws, C);
  TORCH_CHECK(gamma.numel() == C && dgamma.numel() == C && dbeta.numel() == C &&
                  dgamma.scalar_type() == gamma.scalar_type() && dbeta.scalar_type() == gamma.scalar_type() &&
                  dgamma.is_contiguous() && dbeta.is_contiguous(),
              "bn_stage_bwd_finalize: gamma/dgamma/dbeta [C], same dtype");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && invstd.scalar_type() == at::kFloat && mean.numel() == C &&
                  invstd.numel() == C,
              "mean/invstd fp32 [C]");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(ws.device());
  check_hip(kdl::bn_stage_bwd_finalize(ws.data_ptr<float>(), M, static_cast<int>(C), gamma.data_ptr(),
                                       mean.data_ptr<float>(), invstd.data_ptr<float>(), dgamma.data_ptr(),
                                       dbeta.data_ptr(), static_cast<int>(pdtype_of(gamma)), training, cur_stream()),
            "bn_stage_bwd_finalize");
}

void bn_stage_bwd_apply(const at::Tensor& g, const at::Tensor& x, const at::Tensor& ws, at::Tensor dx,
                        const c10::optional<at::Tensor>& xd, const c10::optional<at::Tensor>& wsd,
                        const c10::optional<at::Tensor>& dxd, int64_t M, int64_t C) {
  need_bf16(g, M * C, "g");
  need_bf16(x, M * C, "x");
  need_bf16(dx, M * C, "dx");
  need_ws(ws, C);
  if (opt_ptr(xd)) {
    need_opt_bf16(xd, M * C, "xd");
    need_opt_bf16(dxd, M * C, "dxd");
    need_ws(*wsd, C);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_hip(kdl::bn_stage_bwd_apply(g.data_ptr(), x.data_ptr(), ws.data_ptr<float>(), dx.data_ptr(), opt_ptr(xd),
                                    opt_ptr(xd) ? wsd->data_ptr<float>() : nullptr,
                                    opt_ptr(xd) ? dxd->data_ptr() : nullptr, M, static_cast<int>(C), cur_stream()),
            "bn_stage_bwd_apply");
}

}  // namespace

// ------------------------------------------------------------------ streams
int64_t make_stream_py(bool dedicated, int64_t priority, int64_t cus) {
  hipStream_t s = nullptr;
  check_hip(kdl::make_stream(dedicated, static_cast<int>(priority), &s, static_cast<int>(cus)), "make_stream");
  return reinterpret_cast<int64_t>(s);
}

void destroy_stream_py(int64_t handle) {
  if (handle) check_hip(hipStreamDestroy(reinterpret_cast<hipStream_t>(handle)), "hipStreamDestroy");
}

void spin_py(double microseconds) { check_hip(kdl::spin(cur_stream(), microseconds), "spin"); }


void register_gbdt(pybind11::module& m);  // gbdt_grower.cpp

PYBIND11_MODULE(_C, m) {
  register_gbdt(m);
  m.def("make_stream", &make_stream_py,
        "new HIP stream (dedicated=True: own hardware queue via a full CU mask; cus > 0: that many CUs)",
        py::arg("dedicated"), py::arg("priority") = 0, py::arg("cus") = 0);
  m.def("destroy_stream", &destroy_stream_py, "destroy a stream from make_stream");
  m.def("set_gemm_core", &kdl::set_gemm_core_mode, "conv GEMM main loop: -1 by shape, 0 register-staged, 1 LDS-DMA");
  m.def("set_igemm_cfg", &kdl::set_igemm_cfg, "force an LDS-DMA tile config (-1 = by shape)");
  m.def("set_halo3x3", &kdl::set_halo3x3, "1: stride-1 3x3 convs of the early stages on the halo kernel");
  m.def("get_gemm_core", &kdl::gemm_core_mode, "current conv GEMM main-loop mode");
  m.def("spin", &spin_py, "one wave busy-waiting N microseconds on the current stream");
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
  m.def("transpose_tiles", &transpose_tiles, "batched bf16 2-D transposes from a static 64x64 tile table");
  m.def("ipc_handle", &ipc_handle, "(IPC handle bytes, byte offset) of a GPU tensor's allocation");
  m.def("ipc_open", &ipc_open, "map a peer process's IPC handle; returns the mapped base pointer");
  m.def("ipc_close", &ipc_close, "unmap a pointer returned by ipc_open");
  m.def("p2p_signal_alloc", &p2p_signal_alloc, "zeroed uncached signal buffer for p2p_allreduce");
  m.def("p2p_error_word", &p2p_error_word, "host-mapped error word (host ptr, device ptr)");
  m.def("p2p_error_free", &p2p_error_free, "free a p2p_error_word");
  m.def("p2p_blocks", &kdl::p2p_blocks, "blocks per p2p_allreduce launch for (16-B units, world)");
  m.def("p2p_oneshot_max_units", &kdl::p2p_oneshot_max_units, "largest bucket (16-B units) of the one-shot path");
  m.def("p2p_allreduce", &p2p_allreduce, "in-place two-phase all-reduce over IPC-mapped peer buffers");
  m.def("pack_grads", &pack_grads, "multi-tensor gather of gradient tensors into a flat buffer");
  m.def("pack_grads_ptrs", &pack_grads_ptrs, "pack_grads with the source pointers as kernel arguments");
  m.attr("pack_arg_ptrs") = kdl::kPackArgPtrs;
  m.def("gbdt_grad_hess", &gbdt_grad_hess, "boosting round gradient + hessian in one launch (0 reg, 1 logistic, 2 softmax)");
  m.def("gbdt_hist", &gbdt_hist, "GBDT per-node gradient/hessian histograms (LDS atomics)");
  m.def("gbdt_hist_quant", &gbdt_hist_quant, "the device grower's quantised (fixed-point) histograms (test hook)");
  m.def("set_gbdt_pack64", &kdl::set_gbdt_pack64, "row-per-lane hist: 1 packed 64-bit LDS add, 0 two 32-bit adds, -1 KDL_TUNE");
  m.def("set_gbdt_hist_rows", &kdl::set_gbdt_hist_rows, "quantised hist kernel: 0 slot, 4 / 8 row-per-lane (rows in flight), -2 KDL_TUNE");
  m.def("gbdt_split", &gbdt_split, "GBDT best split per (node, feature)");
  m.def("gbdt_route", &gbdt_route, "GBDT row routing (1 = right child)");
  m.def("gemm_bias_act", &gemm_bias_act, "MFMA bf16 GEMM C = act(A W^T + b) (trans_w: A W, W [K, N])",
        py::arg("a"), py::arg("w"), py::arg("bias"), py::arg("relu"), py::arg("trans_w") = false);
  m.def("set_ctr_tile", &kdl::set_ctr_tile, "gemm_bias_act tile: -1 by shape, 0/1/2 = 128x128 / 128x64 / 64x64");
  m.def("ctr_tile_for", &kdl::ctr_tile_for, "the gemm_bias_act tile picked for an M x N output");
  m.def("set_ctr_igemm", &kdl::set_ctr_igemm, "forward gemm_bias_act on igemm: mode 0 off / 1 by tile count / 2 always; cfg -1 by shape",
        py::arg("mode"), py::arg("cfg") = -1);
  m.def("set_ctr_handoff", &kdl::set_ctr_handoff,
        "split-reduction hand-off: 1 = sc1 partials without fences, 0 = fenced, -1 = the KDL_TUNE value");
  m.def("ctr_igemm_cfg_for", &kdl::ctr_igemm_cfg_for, "igemm cfg serving a forward M x N x K gemm_bias_act (-1: none)");
  m.def("gemm_dgrad_relu", &gemm_dgrad_relu, "(dz W) * [y > 0] and its column sums (bf16): data gradient through a ReLU + bias gradient, one launch");
  m.def("relu_bwd_dbias", &relu_bwd_dbias, "ReLU backward (mask from output) + bias gradient (deterministic; bf16 or fp32)",
        py::arg("dy"), py::arg("y"), py::arg("db_bf16") = false);
  m.def("head_bce_fwd", &head_bce_fwd, "1-wide logit layer + sigmoid BCE: (logit, dlogit, per-block loss sums)");
  m.def("head_bce_bwd", &head_bce_bwd,
        "logit layer backward: (dx, dw, db, per-block dw partials, per-block db partials[, dbx: relu_x])",
        py::arg("x"), py::arg("w"), py::arg("dlogit"), py::arg("scale"), py::arg("gscale"), py::arg("relu_x") = false);
  m.def("embed_gather", &embed_gather, "embedding row gather into a [B, ld] activation");
  m.def("segment_reduce", &segment_reduce, "sorted segment sum of gradient rows", py::arg("rows"), py::arg("F"),
        py::arg("col0"), py::arg("D"), py::arg("order"), py::arg("seg"), py::arg("ucount") = py::none(),
        py::arg("out_rows") = py::none(), py::arg("out") = py::none());
  m.def("a2a_route", &a2a_route, "fixed-capacity exchange: per-owner send blocks + header + rslot of unique ids");
  m.def("a2a_owner_update", &a2a_owner_update, "owner Adagrad update of a fixed exchange without de-duplication",
        py::arg("grads"), py::arg("local"), py::arg("cap"), py::arg("W"), py::arg("slotmap"), py::arg("call"),
        py::arg("table"), py::arg("accum"), py::arg("lr"), py::arg("eps"), py::arg("scale"),
        py::arg("stamped") = false);
  m.def("a2a_serve", &a2a_serve, "owner side of the fixed exchange: requested rows + local row ids (+ the owner "
        "update's slot stamps)",
        py::arg("table"), py::arg("req"), py::arg("n_own"), py::arg("rows_bf16") = false,
        py::arg("slotmap") = py::none(), py::arg("call") = 0, py::arg("cap") = 0, py::arg("W") = 0);
  m.def("embed_gather_cast", &embed_gather_cast,
        "fused one-owner pull: bf16(table[uniq[inv]]) into the tower input (+ tail: dense columns, zero pad)",
        py::arg("table"), py::arg("uniq"), py::arg("inv"), py::arg("F"), py::arg("out"), py::arg("col0"),
        py::arg("dense") = py::none(), py::arg("tail") = 0);
  m.def("segment_adagrad", &segment_adagrad, "segment sum + fused sparse Adagrad on owned rows");
  m.def("dedup_table_slots", &dedup_table_slots, "hash-table slots dedup_csr needs for n ids");
  m.def("segment_reduce_adagrad", &segment_reduce_adagrad,
        "one-owner sync-free push: per-id gradient sums (segment_reduce) applied by Adagrad in the same launch");
  m.def("csr_from_inverse_only", &csr_from_inverse_only, "CSR (seg, order) of a dedup_csr inverse, positions ascending per id");
  m.def("dedup_csr", &dedup_csr, "sync-free id de-duplication (uniq/inv/count on the device) + optional CSR of the inverse");
  m.def("conv1x1_gemm", &conv1x1_gemm, "1x1 conv / dgrad as MFMA GEMM with fused BN prologue/epilogue");
  m.def("set_stem_drop", &kdl::set_stem_drop, "timing-only: skip the stem kernel's MFMAs (1), epilogue (2), input (4)");
  m.def("conv1x1_gram_floats", &conv1x1_gram_floats, "workspace floats of conv1x1_gram(M, K)");
  m.def("conv1x1_gram", &conv1x1_gram, "Q = a^T a | s = 1^T a of a = relu(X*scale+shift) (fp32, into ws[:K*K+K])");
  m.def("gram_fold", &gram_fold, "dW = diag(k) G + diag(c1) W Q + c0 s^T -> bf16 (BN-backward weight gradient, dc never stored)");
  m.def("slab_reduce_f32", &slab_reduce_f32, "fixed-order fp32 sum of slabs into the first");
  m.def("bn_bwd_pro_arm", &bn_bwd_pro_arm, "fuse this BN's backward apply (input x, workspace ws) into the next conv1x1_gemm's A (or conv1x1_wgrad's G) staging; optional write-through tensor");
  m.def("bn_fin_arm", &bn_fin_arm, "fold the BN finalize of this workspace (C channels, M elements) into the next conv GEMM launch");
  m.def("bn_fin_desc", &bn_fin_desc, "write a BN layer's finalize descriptor into its workspace tail");
  m.def("stem7x7_wgrad_bn", &stem7x7_wgrad_bn, "stem weight gradient with the stem BN+ReLU+max-pool backward folded in");
  m.def("stem7x7_wgrad", &stem7x7_wgrad, "ResNet stem 7x7/s2/p3 conv weight gradient -> [64][224] bf16 (stem K order)");
  m.def("stem7x7_wgrad_slabs", [](int64_t nb, int64_t h, int64_t w) {
          return kdl::stem7x7_wgrad_slabs(static_cast<int>(nb), static_cast<int>(h), static_cast<int>(w)); },
        "fp32 slab count of stem7x7_wgrad's workspace", py::arg("nb"), py::arg("h") = 224, py::arg("w") = 224);
  m.def("head_splits", &head_splits, "K splits (fc forward, dfeat) of the classifier head kernels");
  m.def("head_lpad", [](int64_t L) { return kdl::head_lpad(static_cast<int>(L)); }, "row pitch of the head's dl");
  m.def("head_forward", &head_forward, "classifier head forward: mean pool + fc (MFMA) + softmax CE + dlogits");
  m.def("head_backward", &head_backward, "classifier head backward: dfeat, dW, db (MFMA) + mean loss");
  m.def("stem7x7_fwd", &stem7x7_fwd, "ResNet stem 7x7/s2/p3 conv (224 -> 112, 3 -> 64 channels) with BN statistics epilogue");
  m.def("conv3x3_s2_dgrad", &conv3x3_s2_dgrad,
        "stride-2 3x3 pad-1 conv data gradient: four sub-pixel class GEMMs, PLAIN or MASKX epilogue",
        py::arg("dy"), py::arg("ball"), py::arg("dx"), py::arg("Nb"), py::arg("Hd"), py::arg("Wd"), py::arg("Cd"),
        py::arg("N"), py::arg("epi"), py::arg("acc"), py::arg("ex"), py::arg("emean"), py::arg("ecoef"),
        py::arg("Hx") = 0, py::arg("Wx") = 0);
  m.def("bn_res_pro_arm", &bn_res_pro_arm, "next forward conv1x1_gemm applies relu(A*scale+shift+res), written through + mask");
  m.def("conv3x3_aout_arm", &conv3x3_aout_arm, "next prologue conv3x3_gemm also writes relu(B(x)) here (56x56 halo)");
  m.def("conv3x3_gemm", &conv3x3_gemm, "3x3 pad-1 conv (fwd or stride-1 dgrad) as implicit MFMA GEMM with fused BN prologue/epilogue");
  m.def("conv1x1_wgrad", &conv1x1_wgrad, "1x1 conv weight gradient (split-M MFMA into fp32 slabs, fixed-order reduce + bf16 cast); solo: no side stream shares the GPU (more splits)",
        py::arg("G"), py::arg("A"), py::arg("pro_coef"), py::arg("dw32"), py::arg("dW"), py::arg("scale"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("Hout"), py::arg("Wout"), py::arg("Hin"), py::arg("Win"), py::arg("stride"),
        py::arg("solo") = false);
  m.def("conv3x3_wgrad", &conv3x3_wgrad, "3x3 pad-1 conv weight gradient (implicit GEMM, split-M slabs)");
  m.def("conv3x3_wgrad_slabs", &conv3x3_wgrad_slabs, "fp32 [Cout, 9 Cin] slabs conv3x3_wgrad may write (its fastest path)");
  m.def("set_wgrad_big", &kdl::set_wgrad_big, "256x256 weight-gradient tiles: 0 off, 1 3x3 only, 2 3x3 + 1x1");
  m.def("conv1x1_wgrad_splits", &conv1x1_wgrad_splits, "M splits (slab count) of conv1x1_wgrad", py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("solo") = false);
  m.def("bn_coef_offset", &bn_coef_offset, "float offset of the coefficient block in a BN workspace");
  m.def("bn_stage_fwd_stats", &bn_stage_fwd_stats, "BN forward statistics into the workspace replicas");
  m.def("bn_stage_fwd_finalize", &bn_stage_fwd_finalize, "BN forward finalize (mean/invstd/coefs/running stats)");
  m.def("bn_stage_fwd_apply", &bn_stage_fwd_apply, "BN forward apply (+residual | +second BN branch)(+ReLU)(+mask)");
  m.def("bn_stage_bwd_mask_reduce", &bn_stage_bwd_mask_reduce, "masked gradient + BN backward sums");
  m.def("bn_stage_bwd_reduce", &bn_stage_bwd_reduce, "BN backward sums (optional ReLU mask recomputed from x)");
  m.def("bn_stage_bwd_apply_maskx", &bn_stage_bwd_apply_maskx, "BN backward apply with the ReLU mask from x");
  m.def("bn_stage_bwd_finalize", &bn_stage_bwd_finalize, "BN backward finalize (dgamma, dbeta, dx coefs)");
  m.def("bn_stage_bwd_apply", &bn_stage_bwd_apply, "BN backward apply (one or two BN branches)");
  m.attr("arch") = "gfx950";
}
