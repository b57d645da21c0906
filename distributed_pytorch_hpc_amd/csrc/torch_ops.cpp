// PyTorch dispatcher registration of the CDNA4 kernels as `torch.ops.dph.*` (HIP dispatch key = "CUDA"
// on ROCm builds).  Shape/meta functions live in distributed_pytorch_hpc_amd/ops/_meta.py, autograd in
// ops/*.py.  Every op validates its operands on the host (shape, dtype, contiguity, alignment) before a
// launch, so a kernel never sees a layout it was not written for.
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "kernels.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dt_code(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return dph::kBF16;
  if (t.scalar_type() == at::kFloat) return dph::kF32;
  TORCH_CHECK(false, "dph: unsupported dtype ", t.scalar_type(), " (fp32 / bf16 only)");
}
void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "dph: ", name, " must be a GPU tensor");
}
void check_align16(const Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "dph: ", name, " must be 16-byte aligned");
}

// ------------------------------------------------------------------------------------------------ RMSNorm
std::tuple<Tensor, Tensor, Tensor> rmsnorm_fwd(const Tensor& x, const Tensor& w, double eps,
                                               const c10::optional<Tensor>& residual) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "rmsnorm: contiguous operands required");
  const int64_t D = x.size(-1);
  TORCH_CHECK(w.numel() == D && D % 8 == 0, "rmsnorm: dim must match weight and be a multiple of 8");
  const int64_t rows = x.numel() / D;
  auto y = at::empty_like(x);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  Tensor h;
  const void* res = nullptr;
  if (residual.has_value()) {
    TORCH_CHECK(residual->is_contiguous() && residual->sizes() == x.sizes() &&
                residual->scalar_type() == x.scalar_type(), "rmsnorm: residual must match x");
    h = at::empty_like(x);
    res = residual->data_ptr();
  } else {
    h = at::empty({0}, x.options());
  }
  check_align16(x, "x");
  dph::rmsnorm_fwd(x.data_ptr(), w.data_ptr(), res, res ? h.data_ptr() : nullptr, y.data_ptr(),
                   rstd.data_ptr<float>(), rows, (int)D, (float)eps, dt_code(x), dt_code(w), cur_stream());
  return {y, rstd, h};
}

std::tuple<Tensor, Tensor> rmsnorm_bwd(const Tensor& dy, const Tensor& x, const Tensor& w, const Tensor& rstd,
                                       const c10::optional<Tensor>& dres) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && w.is_contiguous(), "rmsnorm_bwd: contiguous required");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "rmsnorm_bwd: dy/x dtype mismatch");
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(w);
  if (rows == 0) return {dx, dw.zero_()};
  const int nblk = dph::rmsnorm_bwd_blocks(rows);
  auto part = at::empty({nblk, D}, x.options().dtype(at::kFloat));
  const void* dr = nullptr;
  if (dres.has_value()) {
    TORCH_CHECK(dres->is_contiguous() && dres->sizes() == x.sizes() && dres->scalar_type() == x.scalar_type(),
                "rmsnorm_bwd: dres must match x");
    dr = dres->data_ptr();
  }
  dph::rmsnorm_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), dr, dx.data_ptr(),
                   part.data_ptr<float>(), dw.data_ptr(), nblk, rows, (int)D, dt_code(x), dt_code(w), cur_stream());
  return {dx, dw};
}

// ------------------------------------------------------------------------------------------------ LayerNorm
std::tuple<Tensor, Tensor, Tensor> layernorm_fwd(const Tensor& x, const Tensor& w, const Tensor& b, double eps) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous() && b.is_contiguous(), "layernorm: contiguous required");
  const int64_t D = x.size(-1);
  TORCH_CHECK(w.numel() == D && b.numel() == D && D % 8 == 0 && D <= 8192, "layernorm: bad dim");
  TORCH_CHECK(w.scalar_type() == b.scalar_type(), "layernorm: weight/bias dtype mismatch");
  const int64_t rows = x.numel() / D;
  auto y = at::empty_like(x);
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  dph::layernorm_fwd(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), rows, (int)D, (float)eps, dt_code(x), dt_code(w), cur_stream());
  return {y, mean, rstd};
}

std::tuple<Tensor, Tensor, Tensor> layernorm_bwd(const Tensor& dy, const Tensor& x, const Tensor& w,
                                                 const Tensor& mean, const Tensor& rstd) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "layernorm_bwd: contiguous required");
  const int64_t D = x.size(-1);
  const int64_t rows = x.numel() / D;
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(w);
  auto db = at::empty_like(w);
  if (rows == 0) return {dx, dw.zero_(), db.zero_()};
  const int nblk = dph::rmsnorm_bwd_blocks(rows);
  auto part = at::empty({nblk, 2 * D}, x.options().dtype(at::kFloat));
  dph::layernorm_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                     dx.data_ptr(), part.data_ptr<float>(), dw.data_ptr(), db.data_ptr(), nblk, rows, (int)D,
                     dt_code(x), dt_code(w), cur_stream());
  return {dx, dw, db};
}

// ------------------------------------------------------------------------------------------------ RoPE
void rope_(Tensor x, const Tensor& cos_t, const Tensor& sin_t, int64_t pos_offset, bool inverse) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.dim() == 4, "rope: x must be [B, S, H, hd]");
  TORCH_CHECK(x.stride(3) == 1, "rope: head dim must be contiguous");
  const int64_t hd = x.size(3);
  TORCH_CHECK(hd % 8 == 0, "rope: head dim must be a multiple of 8");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
              sin_t.is_contiguous() && cos_t.size(-1) == hd / 2, "rope: tables must be fp32 [S, hd/2]");
  TORCH_CHECK(pos_offset + x.size(1) <= cos_t.size(0), "rope: position table too short");
  TORCH_CHECK(x.stride(0) % 8 == 0 && x.stride(1) % 8 == 0 && x.stride(2) % 8 == 0, "rope: strides must be x8");
  check_align16(x, "x");
  dph::rope_apply(x.data_ptr(), cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), x.size(0), x.size(1), x.size(2),
                  (int)hd, x.stride(0), x.stride(1), x.stride(2), pos_offset, inverse ? 1 : 0, dt_code(x),
                  cur_stream());
}

// ------------------------------------------------------------------------------------------------ SwiGLU
Tensor swiglu_fwd(const Tensor& x2) {
  c10::DeviceGuard g(x2.device());
  TORCH_CHECK(x2.is_contiguous(), "swiglu: contiguous input required");
  const int64_t two_f = x2.size(-1);
  TORCH_CHECK(two_f % 16 == 0, "swiglu: hidden must be a multiple of 8");
  const int64_t f = two_f / 2, n = x2.numel() / two_f;
  auto sizes = x2.sizes().vec();
  sizes.back() = f;
  auto y = at::empty(sizes, x2.options());
  dph::swiglu_fwd(x2.data_ptr(), y.data_ptr(), n, f, two_f, dt_code(x2), cur_stream());
  return y;
}
Tensor swiglu_bwd(const Tensor& dy, const Tensor& x2) {
  c10::DeviceGuard g(x2.device());
  TORCH_CHECK(x2.is_contiguous() && dy.is_contiguous(), "swiglu_bwd: contiguous required");
  const int64_t two_f = x2.size(-1), f = two_f / 2, n = x2.numel() / two_f;
  auto dx2 = at::empty_like(x2);
  dph::swiglu_bwd(dy.data_ptr(), x2.data_ptr(), dx2.data_ptr(), n, f, two_f, dt_code(x2), cur_stream());
  return dx2;
}

// ------------------------------------------------------------------------------------------------ GELU
Tensor gelu_fwd(const Tensor& x, bool tanh_form) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_contiguous() && x.numel() % 8 == 0, "gelu: contiguous, numel % 8 == 0 required");
  auto y = at::empty_like(x);
  dph::gelu_fwd(x.data_ptr(), y.data_ptr(), x.numel(), tanh_form ? 1 : 0, dt_code(x), cur_stream());
  return y;
}
Tensor gelu_bwd(const Tensor& dy, const Tensor& x, bool tanh_form) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_contiguous() && dy.is_contiguous(), "gelu_bwd: contiguous required");
  auto dx = at::empty_like(x);
  dph::gelu_bwd(dy.data_ptr(), x.data_ptr(), dx.data_ptr(), x.numel(), tanh_form ? 1 : 0, dt_code(x), cur_stream());
  return dx;
}

// ------------------------------------------------------------------------------------------------ optimizers
// device [lr, step] of a graph-capturable optimizer step (nullptr: the scalar arguments apply)
static const float* hyper_ptr(const c10::optional<Tensor>& hyper, const Tensor& master) {
  if (!hyper.has_value()) return nullptr;
  TORCH_CHECK(hyper->scalar_type() == at::kFloat && hyper->numel() >= 2 && hyper->is_contiguous() &&
                  hyper->device() == master.device(),
              "optimizer hyper: fp32 [lr, step] on the parameters' device expected");
  return hyper->data_ptr<float>();
}

void adamw_step_(Tensor master, Tensor m, Tensor v, const Tensor& grad, const c10::optional<Tensor>& param_out,
                 double lr, double b1, double b2, double eps, double wd, double bc1, double bc2,
                 const c10::optional<Tensor>& grad_scale, const c10::optional<Tensor>& hyper) {
  c10::DeviceGuard g(master.device());
  const int64_t n = master.numel();
  TORCH_CHECK(master.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw: master/m/v must be fp32");
  TORCH_CHECK(m.numel() == n && v.numel() == n && grad.numel() == n, "adamw: size mismatch");
  TORCH_CHECK(master.is_contiguous() && m.is_contiguous() && v.is_contiguous() && grad.is_contiguous(),
              "adamw: contiguous buffers required");
  check_align16(master, "master"); check_align16(m, "m"); check_align16(v, "v");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(grad.data_ptr()) % 8 == 0, "adamw: grad must be 8-byte aligned");
  void* pout = nullptr;
  int pdt = dph::kBF16;
  if (param_out.has_value()) {
    TORCH_CHECK(param_out->numel() == n && param_out->is_contiguous(), "adamw: param_out mismatch");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(param_out->data_ptr()) % 8 == 0, "adamw: param_out alignment");
    pout = param_out->data_ptr();
    pdt = dt_code(*param_out);
  }
  const float* gs = grad_scale.has_value() ? grad_scale->data_ptr<float>() : nullptr;
  const float* hp = hyper_ptr(hyper, master);
  dph::adamw_step(master.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), grad.data_ptr(), pout, n,
                  (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2, gs, hp,
                  dt_code(grad), pdt, cur_stream());
}

void sgd_step_(Tensor master, Tensor buf, const Tensor& grad, const c10::optional<Tensor>& param_out, double lr,
               double momentum, double dampening, double wd, bool nesterov, bool first_step,
               const c10::optional<Tensor>& grad_scale, const c10::optional<Tensor>& hyper) {
  c10::DeviceGuard g(master.device());
  const int64_t n = master.numel();
  TORCH_CHECK(master.scalar_type() == at::kFloat && buf.scalar_type() == at::kFloat, "sgd: fp32 master/buf");
  TORCH_CHECK(grad.numel() == n && master.is_contiguous() && grad.is_contiguous(), "sgd: layout");
  void* pout = nullptr;
  int pdt = dph::kBF16;
  if (param_out.has_value()) {
    pout = param_out->data_ptr();
    pdt = dt_code(*param_out);
  }
  const float* gs = grad_scale.has_value() ? grad_scale->data_ptr<float>() : nullptr;
  const float* hp = hyper_ptr(hyper, master);
  dph::sgd_step(master.data_ptr<float>(), buf.data_ptr<float>(), grad.data_ptr(), pout, n, (float)lr,
                (float)momentum, (float)dampening, (float)wd, nesterov ? 1 : 0, first_step ? 1 : 0, gs, hp,
                dt_code(grad), pdt, cur_stream());
}

void sumsq_(const Tensor& x, Tensor out) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_contiguous() && out.scalar_type() == at::kFloat, "sumsq: layout");
  check_align16(x, "x");
  dph::sumsq(x.data_ptr(), x.numel(), out.data_ptr<float>(), dt_code(x), cur_stream());
}

// ------------------------------------------------------------------------------------------------ cross-entropy
std::tuple<Tensor, Tensor> cross_entropy_fwd(Tensor logits, const Tensor& target, const Tensor& inv_count,
                                             int64_t ignore_index, bool grad_inplace, double smoothing) {
  c10::DeviceGuard g(logits.device());
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent: logits must be [N, V] row-major");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == logits.size(0), "xent: target [N] int64");
  const int64_t n = logits.size(0), v = logits.size(1);
  auto loss = at::empty({n}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({n}, logits.options().dtype(at::kFloat));
  dph::cross_entropy_fwd(logits.data_ptr(), target.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(),
                         inv_count.data_ptr<float>(), n, v, logits.stride(0), ignore_index, grad_inplace ? 1 : 0,
                         (float)smoothing, dt_code(logits), cur_stream());
  return {loss, lse};
}

// ------------------------------------------------------------------------------------------------ attention
void check_attn_operand(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 4, "flash_attn: ", name, " must be [B, S, H, D]");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "flash_attn: ", name, " must be bf16");
  TORCH_CHECK(t.stride(3) == 1, "flash_attn: ", name, " head dim must be contiguous");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              "flash_attn: ", name, " strides must be multiples of 8 elements");
  check_align16(t, name);
}

dph::AttnParams make_params(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, const Tensor& lse,
                            double scale, bool causal, double dropout_p = 0.0, int64_t seed = 0) {
  dph::AttnParams p{};
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr(); p.o = o.data_ptr();
  p.lse = lse.defined() && lse.numel() ? lse.data_ptr<float>() : nullptr;
  p.q_sb = q.stride(0); p.q_ss = q.stride(1); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_ss = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_ss = v.stride(1); p.v_sh = v.stride(2);
  p.o_sb = o.stride(0); p.o_ss = o.stride(1); p.o_sh = o.stride(2);
  p.B = (int)q.size(0); p.Sq = (int)q.size(1); p.Hq = (int)q.size(2); p.D = (int)q.size(3);
  p.Sk = (int)k.size(1); p.Hkv = (int)k.size(2);
  p.scale = (float)scale;
  p.causal = causal ? 1 : 0;
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "flash_attn: dropout_p must be in [0, 1)");
  p.drop_p = (float)dropout_p;
  p.drop_seed = (unsigned)(seed & 0xffffffff);
  return p;
}

std::tuple<Tensor, Tensor> flash_attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, double scale,
                                          bool causal, double dropout_p, int64_t seed) {
  c10::DeviceGuard g(q.device());
  check_attn_operand(q, "q"); check_attn_operand(k, "k"); check_attn_operand(v, "v");
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 32 || D == 64 || D == 128, "flash_attn: head_dim must be 32, 64 or 128");
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && k.sizes() == v.sizes(), "flash_attn: k/v shape mismatch");
  TORCH_CHECK(k.size(0) == q.size(0) && q.size(2) % k.size(2) == 0, "flash_attn: batch / GQA heads mismatch");
  auto o = at::empty({q.size(0), q.size(1), q.size(2), D}, q.options());
  auto lse = at::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  auto p = make_params(q, k, v, o, lse, scale, causal, dropout_p, seed);
  dph::flash_attn_fwd(p, cur_stream());
  return {o, lse};
}

void flash_attn_bwd_impl(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                         const Tensor& lse, double scale, bool causal, Tensor& dq, Tensor& dk, Tensor& dv,
                         double dropout_p, int64_t seed, const c10::optional<Tensor>& rope_cos = c10::nullopt,
                         const c10::optional<Tensor>& rope_sin = c10::nullopt, int64_t rope_offset = 0) {
  c10::DeviceGuard g(q.device());
  check_attn_operand(q, "q"); check_attn_operand(k, "k"); check_attn_operand(v, "v");
  check_attn_operand(o, "o"); check_attn_operand(dout, "dout");
  check_attn_operand(dq, "dq"); check_attn_operand(dk, "dk"); check_attn_operand(dv, "dv");
  TORCH_CHECK(dout.sizes() == o.sizes() && o.sizes() == q.sizes() && dq.sizes() == q.sizes(),
              "flash_attn_bwd: dout/o/dq shape mismatch");
  TORCH_CHECK(dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "flash_attn_bwd: dk/dv shape mismatch");
  const int64_t B = q.size(0), Sq = q.size(1), Hq = q.size(2), D = q.size(3);
  auto delta = at::empty({B, Hq, Sq}, q.options().dtype(at::kFloat));
  dph::AttnBwdParams P{};
  auto lse_c = lse.contiguous();
  P.f = make_params(q, k, v, o, lse_c, scale, causal, dropout_p, seed);
  P.dout = dout.data_ptr(); P.do_sb = dout.stride(0); P.do_ss = dout.stride(1); P.do_sh = dout.stride(2);
  P.delta = delta.data_ptr<float>();
  P.dq = dq.data_ptr(); P.dk = dk.data_ptr(); P.dv = dv.data_ptr();
  P.dq_sb = dq.stride(0); P.dq_ss = dq.stride(1); P.dq_sh = dq.stride(2);
  P.dk_sb = dk.stride(0); P.dk_ss = dk.stride(1); P.dk_sh = dk.stride(2);
  P.dv_sb = dv.stride(0); P.dv_ss = dv.stride(1); P.dv_sh = dv.stride(2);
  if (rope_cos.has_value() && rope_cos->defined()) {
    TORCH_CHECK(rope_sin.has_value() && rope_sin->defined(), "flash_attn_bwd: rope_cos without rope_sin");
    const auto& c = *rope_cos;
    const auto& sn = *rope_sin;
    TORCH_CHECK(c.scalar_type() == at::kFloat && sn.scalar_type() == at::kFloat && c.is_contiguous() &&
                    sn.is_contiguous() && c.dim() == 2 && c.sizes() == sn.sizes() && c.size(1) == D / 2,
                "flash_attn_bwd: rope tables must be contiguous fp32 [max_pos, head_dim / 2]");
    TORCH_CHECK(c.device() == q.device(), "flash_attn_bwd: rope tables on another device");
    TORCH_CHECK(k.size(1) == Sq && rope_offset >= 0 && rope_offset + Sq <= c.size(0),
                "flash_attn_bwd: fused RoPE needs Sq == Sk and positions inside the table");
    P.rope_cos = c.data_ptr<float>();
    P.rope_sin = sn.data_ptr<float>();
    P.rope_off = (int)rope_offset;
  }
  dph::flash_attn_bwd(P, cur_stream());
}

// Ring-attention step: attention of q against this K/V block, merged in the kernel's epilogue into the fp32 running
// output acc_o [B, Sq, Hq, D] and log-sum-exp acc_lse [B, Hq, Sq] (views allowed: unit stride along D / the sequence).
void flash_attn_fwd_merge_(const Tensor& q, const Tensor& k, const Tensor& v, double scale, bool causal, Tensor acc_o,
                           Tensor acc_lse) {
  c10::DeviceGuard g(q.device());
  check_attn_operand(q, "q"); check_attn_operand(k, "k"); check_attn_operand(v, "v");
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 32 || D == 64 || D == 128, "flash_attn_fwd_merge_: head_dim must be 32, 64 or 128");
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && k.sizes() == v.sizes(), "flash_attn_fwd_merge_: k/v mismatch");
  TORCH_CHECK(acc_o.scalar_type() == at::kFloat && acc_o.dim() == 4 && acc_o.sizes() == q.sizes() &&
                  acc_o.stride(3) == 1 && acc_o.device() == q.device(),
              "flash_attn_fwd_merge_: acc_o must be fp32 [B, Sq, Hq, D] with unit stride along D");
  TORCH_CHECK(acc_o.stride(0) % 4 == 0 && acc_o.stride(1) % 4 == 0 && acc_o.stride(2) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(acc_o.data_ptr()) % 16 == 0,
              "flash_attn_fwd_merge_: acc_o rows must be 16-B aligned");
  TORCH_CHECK(acc_lse.scalar_type() == at::kFloat && acc_lse.dim() == 3 && acc_lse.size(0) == q.size(0) &&
                  acc_lse.size(1) == q.size(2) && acc_lse.size(2) == q.size(1) && acc_lse.stride(2) == 1,
              "flash_attn_fwd_merge_: acc_lse must be fp32 [B, Hq, Sq] with unit stride along the sequence");
  auto p = make_params(q, k, v, acc_o, Tensor(), scale, causal);
  p.o = nullptr;
  p.acc_o = acc_o.data_ptr<float>();
  p.ao_sb = acc_o.stride(0); p.ao_ss = acc_o.stride(1); p.ao_sh = acc_o.stride(2);
  p.acc_lse = acc_lse.data_ptr<float>();
  p.al_sb = acc_lse.stride(0); p.al_sh = acc_lse.stride(1);
  dph::flash_attn_fwd(p, cur_stream());
}

std::tuple<Tensor, Tensor, Tensor> flash_attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k,
                                                  const Tensor& v, const Tensor& o, const Tensor& lse, double scale,
                                                  bool causal, double dropout_p, int64_t seed) {
  auto dq = at::empty(q.sizes(), q.options());
  auto dk = at::empty(k.sizes(), k.options());
  auto dv = at::empty(v.sizes(), v.options());
  flash_attn_bwd_impl(dout, q, k, v, o, lse, scale, causal, dq, dk, dv, dropout_p, seed);
  return {dq, dk, dv};
}

void flash_attn_bwd_into(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                         const Tensor& lse, double scale, bool causal, Tensor dq, Tensor dk, Tensor dv,
                         double dropout_p, int64_t seed, const c10::optional<Tensor>& rope_cos,
                         const c10::optional<Tensor>& rope_sin, int64_t rope_offset) {
  flash_attn_bwd_impl(dout, q, k, v, o, lse, scale, causal, dq, dk, dv, dropout_p, seed, rope_cos, rope_sin,
                      rope_offset);
}

// ------------------------------------------------------------------------------------------------ image batches
Tensor image_augment(const Tensor& images, const Tensor& idx, const c10::optional<Tensor>& params,
                     const Tensor& mean, const Tensor& inv_std, int64_t pad, bool channels_last, bool bf16_out) {
  c10::DeviceGuard g(images.device());
  TORCH_CHECK(images.scalar_type() == at::kByte && images.dim() == 4 && images.is_contiguous(),
              "image_augment: images must be contiguous uint8 [N, H, W, C]");
  const int64_t H = images.size(1), W = images.size(2), C = images.size(3);
  TORCH_CHECK(C == 1 || C == 3, "image_augment: 1 or 3 channels");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous(), "image_augment: int64 [B] idx");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && inv_std.scalar_type() == at::kFloat && mean.numel() == C &&
                  inv_std.numel() == C && mean.is_contiguous() && inv_std.is_contiguous(),
              "image_augment: fp32 mean / inv_std of C elements");
  TORCH_CHECK(pad >= 0 && pad <= H && pad <= W, "image_augment: bad padding");
  const int64_t B = idx.size(0);
  const int* prm = nullptr;
  if (params.has_value() && params->defined()) {
    TORCH_CHECK(params->scalar_type() == at::kInt && params->is_contiguous() && params->numel() == 3 * B,
                "image_augment: int32 [B, 3] (dy, dx, flip) params");
    prm = params->data_ptr<int>();
  }
  for (const Tensor* t : {&idx, &mean, &inv_std}) TORCH_CHECK(t->device() == images.device(), "image_augment: device");
  auto opts = images.options().dtype(bf16_out ? at::kBFloat16 : at::kFloat);
  Tensor out = channels_last ? at::empty({B, C, H, W}, opts.memory_format(at::MemoryFormat::ChannelsLast))
                             : at::empty({B, C, H, W}, opts);
  dph::image_augment(images.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(), prm, mean.data_ptr<float>(),
                     inv_std.data_ptr<float>(), out.data_ptr(), B, H, W, C, pad, channels_last,
                     bf16_out ? dph::kBF16 : dph::kF32, cur_stream());
  return out;
}

// ------------------------------------------------------------------------------------------------ fp8
// (y [R, C] or empty, yt [C, R] or empty, dequant fp32 scalar): per-tensor current scaling from max|x|.
std::tuple<Tensor, Tensor, Tensor> fp8_quantize(const Tensor& x, int64_t fmt, bool rowmajor, bool transposed) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(),
              "fp8_quantize: contiguous bf16 [R, C]");
  TORCH_CHECK(fmt == dph::kFP8E4M3 || fmt == dph::kFP8E5M2, "fp8_quantize: fmt 0 (e4m3) or 1 (e5m2)");
  TORCH_CHECK(rowmajor || transposed, "fp8_quantize: nothing to write");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(R % 64 == 0 && C % 64 == 0, "fp8_quantize: R and C must be multiples of 64");
  TORCH_CHECK(x.data_ptr() == nullptr || reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "fp8_quantize: 16-B aligned input");
  const auto f8 = fmt == dph::kFP8E4M3 ? at::kFloat8_e4m3fn : at::kFloat8_e5m2;
  Tensor y = rowmajor ? at::empty({R, C}, x.options().dtype(f8)) : at::empty({0}, x.options().dtype(f8));
  Tensor yt = transposed ? at::empty({C, R}, x.options().dtype(f8)) : at::empty({0}, x.options().dtype(f8));
  // one small fp32 buffer: [amax, scale, dequant | per-block partials]; the dequant scale is returned as a view
  Tensor buf = at::empty({3 + dph::fp8_amax_blocks(R * C)}, x.options().dtype(at::kFloat));
  float* scal = buf.data_ptr<float>();
  auto st = cur_stream();
  dph::fp8_amax(x.data_ptr(), R * C, (int)fmt, scal + 3, scal, st);
  dph::fp8_quant(x.data_ptr(), R, C, scal, (int)fmt, rowmajor ? y.data_ptr() : nullptr,
                 transposed ? yt.data_ptr() : nullptr, st);
  return {y, yt, buf.select(0, 2)};
}

// ------------------------------------------------------------------------------------------------ serving
// returns 1 for OCP e4m3 caches, 0 for bf16
int check_kv_cache(const Tensor& kc, const Tensor& vc) {
  const bool fp8 = kc.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(kc.dim() == 4 && (fp8 || kc.scalar_type() == at::kBFloat16) && kc.sizes() == vc.sizes() &&
                  kc.strides() == vc.strides() && vc.scalar_type() == kc.scalar_type(),
              "kv cache: k and v must be bf16 or float8_e4m3fn [B, Smax, Hkv, D] with equal strides");
  TORCH_CHECK(kc.stride(3) == 1 && kc.stride(0) % 8 == 0 && kc.stride(1) % 8 == 0 && kc.stride(2) % 8 == 0,
              "kv cache: head dim contiguous, strides multiples of 8 elements");
  check_align16(kc, "k_cache"); check_align16(vc, "v_cache");
  return fp8 ? 1 : 0;
}

void check_positions(const Tensor& pos, const Tensor& like, int64_t B) {
  TORCH_CHECK(pos.scalar_type() == at::kInt && pos.dim() == 1 && pos.size(0) == B && pos.is_contiguous() &&
                  pos.device() == like.device(),
              "kv cache: pos must be a contiguous int32 [B] tensor on the cache's device");
}

void kv_append_(Tensor& qkv, Tensor& kc, Tensor& vc, const Tensor& pos, const Tensor& cos, const Tensor& sin,
                int64_t n_heads, int64_t n_kv_heads, double kv_scale) {
  c10::DeviceGuard g(qkv.device());
  const int fp8 = check_kv_cache(kc, vc);
  TORCH_CHECK(kv_scale > 0.0, "kv_append: kv_scale must be positive");
  const int64_t B = qkv.size(0), S = qkv.size(1), D = kc.size(3);
  TORCH_CHECK(qkv.dim() == 3 && qkv.scalar_type() == at::kBFloat16 && qkv.stride(2) == 1 &&
                  qkv.size(2) == (n_heads + 2 * n_kv_heads) * D && qkv.stride(0) % 8 == 0 && qkv.stride(1) % 8 == 0,
              "kv_append: qkv must be bf16 [B, S, (Hq + 2 Hkv) * D] with a contiguous last dim");
  check_align16(qkv, "qkv");
  TORCH_CHECK(kc.size(0) == B && kc.size(2) == n_kv_heads && n_heads % n_kv_heads == 0 && D % 8 == 0,
              "kv_append: cache batch / heads do not match qkv");
  check_positions(pos, qkv, B);
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                  sin.is_contiguous() && cos.dim() == 2 && cos.sizes() == sin.sizes() && cos.size(1) == D / 2 &&
                  cos.size(0) >= kc.size(1) && cos.device() == qkv.device(),
              "kv_append: rope tables must be contiguous fp32 [>= Smax, D / 2] on the same device");
  dph::KVAppendParams p{};
  p.qkv = qkv.data_ptr(); p.qkv_sb = qkv.stride(0); p.qkv_ss = qkv.stride(1);
  p.kc = kc.data_ptr(); p.vc = vc.data_ptr(); p.c_sb = kc.stride(0); p.c_ss = kc.stride(1); p.c_sh = kc.stride(2);
  p.pos = pos.data_ptr<int>(); p.cos = cos.data_ptr<float>(); p.sin = sin.data_ptr<float>();
  p.B = (int)B; p.S = (int)S; p.Hq = (int)n_heads; p.Hkv = (int)n_kv_heads; p.D = (int)D; p.Smax = (int)kc.size(1);
  p.kv_fp8 = fp8; p.kv_scale = (float)kv_scale;
  dph::kv_append(p, cur_stream());
}

Tensor decode_attention(const Tensor& qkv, const Tensor& kc, const Tensor& vc, const Tensor& pos, int64_t n_heads,
                        int64_t n_kv_heads, double scale, int64_t max_len, double kv_scale) {
  c10::DeviceGuard g(qkv.device());
  const int fp8 = check_kv_cache(kc, vc);
  const int64_t B = qkv.size(0), D = kc.size(3), Smax = kc.size(1);
  TORCH_CHECK(D == 32 || D == 64 || D == 128, "decode_attention: head_dim must be 32, 64 or 128");
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(1) == 1 && qkv.scalar_type() == at::kBFloat16 && qkv.stride(2) == 1 &&
                  qkv.size(2) == (n_heads + 2 * n_kv_heads) * D && qkv.stride(0) % 8 == 0,
              "decode_attention: qkv must be bf16 [B, 1, (Hq + 2 Hkv) * D]");
  check_align16(qkv, "qkv");
  TORCH_CHECK(kc.size(0) == B && kc.size(2) == n_kv_heads && n_heads % n_kv_heads == 0,
              "decode_attention: cache batch / heads do not match qkv");
  check_positions(pos, qkv, B);
  TORCH_CHECK(max_len >= 1 && max_len <= Smax, "decode_attention: max_len must be in [1, Smax]");
  const int64_t nch = (max_len + 63) / 64;
  auto out = at::empty({B, n_heads * D}, qkv.options());
  auto opart = at::empty({B, n_heads, nch, D}, qkv.options().dtype(at::kFloat));
  auto ml = at::empty({B, n_heads, nch, 2}, qkv.options().dtype(at::kFloat));
  dph::DecodeParams p{};
  p.q = qkv.data_ptr(); p.q_sb = qkv.stride(0); p.q_sh = D;
  p.kc = kc.data_ptr(); p.vc = vc.data_ptr(); p.c_sb = kc.stride(0); p.c_ss = kc.stride(1); p.c_sh = kc.stride(2);
  p.pos = pos.data_ptr<int>(); p.len_add = 1;
  p.opart = opart.data_ptr<float>(); p.mlpart = ml.data_ptr<float>();
  p.out = out.data_ptr(); p.out_sb = out.stride(0);
  p.B = (int)B; p.Hq = (int)n_heads; p.Hkv = (int)n_kv_heads; p.D = (int)D; p.nch = (int)nch; p.Smax = (int)Smax;
  p.scale = (float)scale;
  p.kv_fp8 = fp8; p.kv_scale = (float)kv_scale;
  dph::decode_attention(p, cur_stream());
  return out;
}

Tensor skinny_linear(const Tensor& x, const Tensor& w) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "skinny_linear: bf16 only");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && x.size(-1) == w.size(1), "skinny_linear: w [N, K] contiguous");
  const int64_t K = w.size(1), N = w.size(0), M = x.numel() / std::max<int64_t>(K, 1);
  TORCH_CHECK(dph::skinny_gemm_supported(M, N, K), "skinny_linear: needs rows <= 64 and (1-2 rows: N % 8, K % 8, K <= 16384; else N % 16, K % 128)");
  auto x2 = x.reshape({M, K});
  TORCH_CHECK(x2.stride(1) == 1 && x2.stride(0) % 8 == 0, "skinny_linear: x rows must be contiguous, 16-B aligned");
  check_align16(x2, "x"); check_align16(w, "w");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  auto y = at::empty(sizes, x.options());
  dph::skinny_gemm(x2.data_ptr(), x2.stride(0), w.data_ptr(), K, y.data_ptr(), N, (int)M, (int)N, (int)K,
                   cur_stream());
  return y;
}

Tensor gemv_swiglu(const Tensor& x2, const Tensor& w) {
  c10::DeviceGuard g(x2.device());
  TORCH_CHECK(x2.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && w.dim() == 2 &&
                  w.is_contiguous(), "gemv_swiglu: bf16, w [N, K] contiguous");
  const int64_t K = w.size(1), N = w.size(0);
  TORCH_CHECK(x2.size(-1) == 2 * K, "gemv_swiglu: x2 must be [..., 2K] (gate | up)");
  const int64_t M = x2.numel() / (2 * K);
  TORCH_CHECK(dph::gemv_supported(M, N, K), "gemv_swiglu: needs 1-2 rows, N % 8, K % 8, K <= 16384");
  auto xr = x2.reshape({M, 2 * K});
  TORCH_CHECK(xr.stride(1) == 1 && xr.stride(0) % 8 == 0, "gemv_swiglu: rows must be contiguous");
  check_align16(xr, "x2"); check_align16(w, "w");
  auto sizes = x2.sizes().vec();
  sizes.back() = N;
  auto y = at::empty(sizes, x2.options());
  dph::GemvArgs a{};
  a.x = xr.data_ptr(); a.ldx = xr.stride(0); a.w = w.data_ptr(); a.ldw = K; a.y = y.data_ptr(); a.ldy = N;
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  dph::gemv(a, 1, cur_stream());
  return y;
}

std::tuple<Tensor, Tensor> gemv_rmsnorm(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& gw, double eps,
                                        const Tensor& w) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 && gw.scalar_type() == at::kBFloat16,
              "gemv_rmsnorm: bf16 x, norm weight and w");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && gw.is_contiguous() && gw.numel() == w.size(1),
              "gemv_rmsnorm: w [N, K] contiguous, norm weight [K]");
  const int64_t K = w.size(1), N = w.size(0);
  TORCH_CHECK(x.size(-1) == K && x.numel() == K, "gemv_rmsnorm: exactly one row of K");
  TORCH_CHECK(dph::gemv_supported(1, N, K), "gemv_rmsnorm: needs N % 8, K % 8, K <= 16384");
  auto xr = x.reshape({1, K}).contiguous();
  check_align16(xr, "x"); check_align16(w, "w"); check_align16(gw, "norm weight");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  auto y = at::empty(sizes, x.options());
  dph::GemvArgs a{};
  a.x = xr.data_ptr(); a.ldx = K; a.g = gw.data_ptr(); a.eps = (float)eps;
  Tensor h;
  if (res.has_value() && res->defined()) {
    TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == at::kBFloat16, "gemv_rmsnorm: residual shape");
    auto rr = res->reshape({1, K}).contiguous();
    check_align16(rr, "res");
    h = at::empty_like(x);
    a.res = rr.data_ptr(); a.ldres = K; a.h_out = h.data_ptr(); a.ldh = K;
  } else {
    h = at::empty({0}, x.options());   // no residual: h is x itself (not returned as an alias)
  }
  a.w = w.data_ptr(); a.ldw = K; a.y = y.data_ptr(); a.ldy = N; a.M = 1; a.N = (int)N; a.K = (int)K;
  dph::gemv(a, 2, cur_stream());
  return {y, h};
}

// ------------------------------------------------------------------------------------------------ embedding
Tensor embedding_fwd(const Tensor& ids, const Tensor& table, int64_t vocab_start) {
  c10::DeviceGuard g(table.device());
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && table.is_contiguous() && table.dim() == 2,
              "embedding: int64 ids, contiguous [V, D] table");
  TORCH_CHECK(table.size(1) % 8 == 0, "embedding: dim must be a multiple of 8");
  auto sizes = ids.sizes().vec();
  sizes.push_back(table.size(1));
  auto out = at::empty(sizes, table.options());
  dph::embedding_fwd(ids.data_ptr<int64_t>(), table.data_ptr(), out.data_ptr(), ids.numel(), table.size(1),
                     vocab_start, table.size(0), dt_code(table), cur_stream());
  return out;
}
Tensor embedding_bwd(const Tensor& ids, const Tensor& dout, int64_t vocab_local, int64_t vocab_start) {
  c10::DeviceGuard g(dout.device());
  TORCH_CHECK(dout.is_contiguous() && ids.is_contiguous(), "embedding_bwd: contiguous required");
  const int64_t dim = dout.size(-1);
  TORCH_CHECK(dim % 8 == 0, "embedding_bwd: dim must be a multiple of 8");
  check_align16(dout, "dout");
  auto dtab = at::zeros({vocab_local, dim}, dout.options().dtype(at::kFloat));
  auto sorted = at::sort(ids.reshape({-1}), /*stable=*/true, /*dim=*/0, /*descending=*/false);
  const Tensor sids = std::get<0>(sorted).contiguous(), perm = std::get<1>(sorted).contiguous();
  dph::embedding_bwd(sids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dout.data_ptr(), dtab.data_ptr<float>(),
                     ids.numel(), dim, vocab_start, vocab_local, dt_code(dout), cur_stream());
  return dtab;
}

// ------------------------------------------------------------------------------------------------ wgrad GEMM
// C[M, N] (+)= A^T B with A [K, M], B [K, N] bf16 row-major (dW = dY^T X).  C bf16 or fp32, row-major.
void gemm_tn_(Tensor C, const Tensor& A, const Tensor& B, bool accumulate) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm_tn: 2-D operands required");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm_tn: bf16 A / B");
  const int64_t K = A.size(0), M = A.size(1), N = B.size(1);
  TORCH_CHECK(B.size(0) == K && C.size(0) == M && C.size(1) == N, "gemm_tn: shape mismatch");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "gemm_tn: row-major operands required");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0, "gemm_tn: leading dims must be multiples of 8");
  TORCH_CHECK(dph::gemm_tn_supported(M, N, K), "gemm_tn: need M, N % 8 == 0 and K % 64 == 0 (got ", M, ", ", N,
              ", ", K, ")");
  check_align16(A, "A");
  check_align16(B, "B");
  const dph::GemmTnPlan plan = dph::gemm_tn_plan(M, N, K);
  Tensor ws;
  if (plan.split) ws = at::empty({plan.workspace_floats}, A.options().dtype(at::kFloat));
  dph::gemm_tn(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), C.stride(0), dt_code(C),
               accumulate, cur_stream(), &plan, plan.split ? ws.data_ptr<float>() : nullptr);
}

// tail split of the wgrad GEMM: n > 0 plans for n CUs (tests), 0 = the device's CU count (default), < 0 = off
void gemm_tn_tail_(int64_t cus) { dph::gemm_tn_set_tail((int)cus); }

std::vector<int64_t> gemm_tn_plan_info(int64_t M, int64_t N, int64_t K) {
  const auto pl = dph::gemm_tn_plan(M, N, K);
  return {pl.split, pl.dim, pl.keep, pl.workspace_floats};
}

// ------------------------------------------------------------------------------------------------ 1x1 conv GEMMs
// C[M, N] = A[M, K] B[N, K]^T, bf16, row-major (channels-last 1x1 convolution forward / input gradient).
// H, W > 0: 3x3 / stride-1 / pad-1 convolution as implicit GEMM, A = channels-last input [n*H*W, Cin],
// B = weights [Cout, 9 * Cin] (tap-major).
// add (optional): C = A B^T + add, add [M, N] bf16 row-major (a residual branch's gradient merged in the epilogue)
// BatchNorm + ReLU prologue coefficients of a 1x1 convolution's input: fp32 [scale K | shift K], K <= 2048
const float* pro_ptr(const c10::optional<Tensor>& pro_ss, int64_t K, int64_t H, const Tensor& like) {
  if (!pro_ss.has_value()) return nullptr;
  TORCH_CHECK(H == 0 && K <= 2048, "ts_gemm: the BatchNorm prologue is a 1x1 (H = 0), K <= 2048 feature");
  TORCH_CHECK(pro_ss->scalar_type() == at::kFloat && pro_ss->is_contiguous() && pro_ss->numel() == 2 * K &&
                  pro_ss->device() == like.device(),
              "ts_gemm: pro_ss must be a contiguous fp32 [2 * K] tensor ([scale | shift])");
  return pro_ss->data_ptr<float>();
}

Tensor ts_gemm_nt(const Tensor& A, const Tensor& B, int64_t H, int64_t W, const c10::optional<Tensor>& add,
                  const c10::optional<Tensor>& bias, const c10::optional<Tensor>& pro_ss) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "ts_gemm_nt: 2-D operands required");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "ts_gemm_nt: bf16 operands");
  const int64_t M = A.size(0), N = B.size(0);
  const int64_t K = H > 0 ? 9 * A.size(1) : A.size(1);
  TORCH_CHECK(B.size(1) == K, "ts_gemm_nt: K mismatch");
  TORCH_CHECK(H == 0 || (W > 0 && M % (H * W) == 0), "ts_gemm_nt: rows must be a multiple of H * W");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "ts_gemm_nt: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::conv1x1_supported(M, N, K), "ts_gemm_nt: need N, K % 64 == 0 (got ", N, ", ", K, ")");
  check_align16(A, "A");
  check_align16(B, "B");
  Tensor C = at::empty({M, N}, A.options());
  const void* D = nullptr;
  if (add.has_value()) {
    TORCH_CHECK(H == 0, "ts_gemm_nt: add is supported for 1x1 (H = 0) only");
    TORCH_CHECK(add->scalar_type() == at::kBFloat16 && add->dim() == 2 && add->size(0) == M && add->size(1) == N &&
                    add->is_contiguous() && add->device() == A.device(),
                "ts_gemm_nt: add must be a contiguous bf16 [M, N] tensor");
    check_align16(*add, "add");
    D = add->data_ptr();
  }
  if (bias.has_value()) {   // 3x3 with a per-output-channel fp32 bias in the LDS-DMA kernel's epilogue
    TORCH_CHECK(H > 0 && !add.has_value() && dph::conv3_supported(M, N, K, A.stride(0), B.stride(0)),
                "ts_gemm_nt: bias is supported on the 3x3 LDS-DMA path only");
    TORCH_CHECK((bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16) && bias->numel() == N &&
                    bias->is_contiguous() && bias->device() == A.device(),
                "ts_gemm_nt: bias must be a contiguous fp32 / bf16 [N] tensor");
    dph::conv3_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), C.stride(0),
                    (int)H, (int)W, cur_stream(), nullptr, bias->data_ptr(), bias->scalar_type() == at::kBFloat16);
    return C;
  }
  const float* pro = pro_ptr(pro_ss, K, H, A);
  TORCH_CHECK(pro == nullptr || D == nullptr, "ts_gemm_nt: add and pro_ss are exclusive");
  dph::ts_gemm_nt(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), C.stride(0),
                  cur_stream(), (int)H, (int)W, D, nullptr, pro);
  return C;
}

// 1x1 input gradient C = A B^T with a stride-2 sub-image gradient added at the even pixels of the H x W grid.
Tensor ts_gemm_nt_add_sub(const Tensor& A, const Tensor& B, const Tensor& add, int64_t H, int64_t W, int64_t s) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16,
              "ts_gemm_nt_add_sub: bf16 2-D operands");
  TORCH_CHECK(s == 2, "ts_gemm_nt_add_sub: stride 2 only");
  const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(B.size(1) == K && H > 0 && W > 0 && M % (H * W) == 0, "ts_gemm_nt_add_sub: shape mismatch");
  const int64_t Ho = (H - 1) / s + 1, Wo = (W - 1) / s + 1;
  TORCH_CHECK(add.scalar_type() == at::kBFloat16 && add.dim() == 2 && add.size(0) == (M / (H * W)) * Ho * Wo &&
                  add.size(1) == N && add.is_contiguous() && add.device() == A.device(),
              "ts_gemm_nt_add_sub: add must be a contiguous bf16 [n * ceil(H/2) * ceil(W/2), N] tensor");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "ts_gemm_nt_add_sub: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::conv1x1_supported(M, N, K), "ts_gemm_nt_add_sub: need N, K % 64 == 0");
  check_align16(A, "A");
  check_align16(B, "B");
  check_align16(add, "add");
  Tensor C = at::empty({M, N}, A.options());
  dph::ts_gemm_nt_add_sub(A.data_ptr(), B.data_ptr(), C.data_ptr(), add.data_ptr(), M, N, K, A.stride(0),
                          B.stride(0), C.stride(0), (int)H, (int)W, (int)s, cur_stream());
  return C;
}

// Input gradient C = A B^T [+ add] of a convolution whose input is a training-mode BatchNorm + ReLU output, with the
// BatchNorm backward's reduction over C in the epilogue (kernels.h BnRed): returns C and the partials
// [cdiv(M, 128), 2N] that bn_act_bwd takes as pre_part.  H, W > 0 and sub = 0: 3x3 stride-1 (A = dY, B = the flipped
// weight [N, 9 * Cout]); sub = 2: add is a stride-2 sub-image gradient over the H x W grid (ts_gemm_nt_add_sub);
// otherwise 1x1 with an optional [M, N] add.  x: the BatchNorm's input ([M, N] rows, channels-last); the ReLU mask
// comes from ss (fp32 [scale N | shift N]) or from bits (the forward's uint8 [M * N / 8]).
std::tuple<Tensor, Tensor> ts_gemm_nt_bnred(const Tensor& A, const Tensor& B, int64_t H, int64_t W,
                                            const c10::optional<Tensor>& add, int64_t sub, const Tensor& x,
                                            const Tensor& mean, const Tensor& invstd, const c10::optional<Tensor>& ss,
                                            const c10::optional<Tensor>& bits,
                                            const c10::optional<Tensor>& add_mask) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16,
              "ts_gemm_nt_bnred: bf16 2-D operands");
  TORCH_CHECK(sub == 0 || sub == 2, "ts_gemm_nt_bnred: sub must be 0 or 2");
  const bool c3 = H > 0 && sub == 0;
  const int64_t M = A.size(0), N = B.size(0), K = c3 ? 9 * A.size(1) : A.size(1);
  TORCH_CHECK(B.size(1) == K && (H == 0 || (W > 0 && M % (H * W) == 0)), "ts_gemm_nt_bnred: shape mismatch");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "ts_gemm_nt_bnred: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::conv1x1_supported(M, N, K), "ts_gemm_nt_bnred: need N, K % 64 == 0");
  TORCH_CHECK(!c3 || (!add.has_value() && dph::conv3_supported(M, N, K, A.stride(0), B.stride(0))),
              "ts_gemm_nt_bnred: 3x3 needs the LDS-DMA kernel's shapes and no add");
  TORCH_CHECK(sub == 0 || (add.has_value() && H > 0 && W > 0), "ts_gemm_nt_bnred: sub = 2 needs add and H, W");
  check_align16(A, "A");
  check_align16(B, "B");
  const void* D = nullptr;
  if (add.has_value()) {
    const int64_t rows = sub == 2 ? (M / (H * W)) * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1) : M;
    TORCH_CHECK(add->scalar_type() == at::kBFloat16 && add->dim() == 2 && add->size(0) == rows &&
                    add->size(1) == N && add->is_contiguous() && add->device() == A.device(),
                "ts_gemm_nt_bnred: add must be a contiguous bf16 [rows, N] tensor");
    check_align16(*add, "add");
    D = add->data_ptr();
  }
  const bool xcl = x.dim() == 4 ? (x.size(1) == N && x.is_contiguous(at::MemoryFormat::ChannelsLast))
                                : (x.dim() == 2 && x.size(1) == N && x.is_contiguous());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.numel() == M * N && xcl && x.device() == A.device(),
              "ts_gemm_nt_bnred: x must be the BatchNorm's bf16 channels-last input with M x N elements");
  check_align16(x, "x");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && invstd.scalar_type() == at::kFloat && mean.numel() == N &&
                  invstd.numel() == N && mean.is_contiguous() && invstd.is_contiguous(),
              "ts_gemm_nt_bnred: fp32 mean / invstd [N]");
  TORCH_CHECK(ss.has_value() != bits.has_value(), "ts_gemm_nt_bnred: exactly one of ss / bits");
  dph::BnRed r;
  r.x = x.data_ptr();
  r.mean = mean.data_ptr<float>();
  r.invstd = invstd.data_ptr<float>();
  if (ss.has_value()) {
    TORCH_CHECK(ss->scalar_type() == at::kFloat && ss->numel() == 2 * N && ss->is_contiguous(),
                "ts_gemm_nt_bnred: ss must be fp32 [scale N | shift N]");
    r.ss = ss->data_ptr<float>();
  } else {
    TORCH_CHECK(bits->scalar_type() == at::kByte && bits->numel() == M * N / 8 && bits->is_contiguous(),
                "ts_gemm_nt_bnred: bits must be the forward's uint8 [M * N / 8]");
    r.bits = bits->data_ptr<uint8_t>();
  }
  const uint8_t* am = nullptr;
  if (add_mask.has_value()) {
    TORCH_CHECK(add.has_value() && sub == 0 && !c3 && add_mask->scalar_type() == at::kByte &&
                    add_mask->numel() == M * N / 8 && add_mask->is_contiguous() && add_mask->device() == A.device(),
                "ts_gemm_nt_bnred: add_mask must be uint8 [M * N / 8] bits of a 1x1 [M, N] add");
    am = add_mask->data_ptr<uint8_t>();
  }
  Tensor C = at::empty({M, N}, A.options());
  Tensor part = at::empty({(M + 127) / 128, 2 * N}, A.options().dtype(at::kFloat));
  r.part = part.data_ptr<float>();
  dph::ts_gemm_nt_bnred(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), N, (int)H,
                        (int)W, D, (int)sub, r, cur_stream(), am);
  return {C, part};
}

// 1x1 input gradient C = A B^T + add * mask: the residual gradient of a BatchNorm + residual + ReLU handed over as its
// output gradient ``add`` [M, N] and the forward's ReLU bits ``add_mask`` (uint8 [M * N / 8]), bitwise the plain add
// of the masked bf16 gradient.
Tensor ts_gemm_nt_addmask(const Tensor& A, const Tensor& B, const Tensor& add, const Tensor& add_mask) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16,
              "ts_gemm_nt_addmask: bf16 2-D operands");
  const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(B.size(1) == K, "ts_gemm_nt_addmask: K mismatch");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "ts_gemm_nt_addmask: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::conv1x1_supported(M, N, K), "ts_gemm_nt_addmask: need N, K % 64 == 0");
  TORCH_CHECK(add.scalar_type() == at::kBFloat16 && add.dim() == 2 && add.size(0) == M && add.size(1) == N &&
                  add.is_contiguous() && add.device() == A.device(),
              "ts_gemm_nt_addmask: add must be a contiguous bf16 [M, N] tensor");
  TORCH_CHECK(add_mask.scalar_type() == at::kByte && add_mask.numel() == M * N / 8 && add_mask.is_contiguous() &&
                  add_mask.device() == A.device(),
              "ts_gemm_nt_addmask: add_mask must be uint8 [M * N / 8]");
  check_align16(A, "A");
  check_align16(B, "B");
  check_align16(add, "add");
  Tensor C = at::empty({M, N}, A.options());
  dph::ts_gemm_nt_bnred(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), N, 0, 0,
                        add.data_ptr(), 0, dph::BnRed{}, cur_stream(), add_mask.data_ptr<uint8_t>());
  return C;
}

// C = A B^T plus the BatchNorm statistics partials of C per 128-row block ([mean | M2 | rows], see conv1x1.hip).
std::tuple<Tensor, Tensor> ts_gemm_nt_stats(const Tensor& A, const Tensor& B, int64_t H, int64_t W,
                                            const c10::optional<Tensor>& pro_ss, const c10::optional<Tensor>& bias) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16,
              "ts_gemm_nt_stats: bf16 2-D operands");
  const int64_t M = A.size(0), N = B.size(0), K = B.size(1);
  TORCH_CHECK(H > 0 ? (W > 0 && K == 9 * A.size(1) && M % (H * W) == 0) : A.size(1) == K,
              "ts_gemm_nt_stats: K mismatch (3x3: B is [N, 9 * Cin], rows a multiple of H * W)");
  TORCH_CHECK(H == 0 || dph::conv3_supported(M, N, K, A.stride(0), B.stride(0)),
              "ts_gemm_nt_stats: 3x3 statistics need the LDS-DMA kernel's shapes");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "ts_gemm_nt_stats: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::conv1x1_supported(M, N, K), "ts_gemm_nt_stats: need N, K % 64 == 0");
  check_align16(A, "A");
  check_align16(B, "B");
  const int64_t nmb = (M + 127) / 128;
  Tensor C = at::empty({M, N}, A.options());
  Tensor st = at::empty({2 * nmb * N + nmb}, A.options().dtype(at::kFloat));
  if (bias.has_value()) {   // 3x3 LDS-DMA kernel: fp32 bias on the accumulators, statistics of the biased output
    TORCH_CHECK(H > 0 && !pro_ss.has_value(), "ts_gemm_nt_stats: bias is a 3x3 (H > 0) feature");
    TORCH_CHECK((bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16) && bias->numel() == N &&
                    bias->is_contiguous() && bias->device() == A.device(),
                "ts_gemm_nt_stats: bias must be a contiguous fp32 / bf16 [N] tensor");
    dph::conv3_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), C.stride(0),
                    (int)H, (int)W, cur_stream(), st.data_ptr<float>(), bias->data_ptr(),
                    bias->scalar_type() == at::kBFloat16);
    return {C, st};
  }
  dph::ts_gemm_nt(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), C.stride(0),
                  cur_stream(), (int)H, (int)W, nullptr, st.data_ptr<float>(), pro_ptr(pro_ss, K, H, A));
  return {C, st};
}

// C[N, K] (+)= A[M, N]^T B[M, K] (1x1 convolution weight gradient, split over pixel chunks).
// H, W > 0: 3x3 weight gradient, C [N, 9 * K_in] tap-major, B = channels-last input [n*H*W, K_in].
void ts_gemm_tn_(Tensor C, const Tensor& A, const Tensor& B, bool accumulate, int64_t H, int64_t W,
                 const c10::optional<Tensor>& pro_ss) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "ts_gemm_tn: 2-D operands required");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "ts_gemm_tn: bf16 A / B");
  const int64_t M = A.size(0), N = A.size(1), K = H > 0 ? 9 * B.size(1) : B.size(1);
  TORCH_CHECK(B.size(0) == M && C.size(0) == N && C.size(1) == K && C.is_contiguous(), "ts_gemm_tn: shape mismatch");
  TORCH_CHECK(H == 0 || (W > 0 && M % (H * W) == 0), "ts_gemm_tn: rows must be a multiple of H * W");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "ts_gemm_tn: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::conv1x1_supported(M, N, K), "ts_gemm_tn: need N, K % 64 == 0 (got ", N, ", ", K, ")");
  TORCH_CHECK(C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat, "ts_gemm_tn: C bf16 or fp32");
  check_align16(A, "A");
  check_align16(B, "B");
  const bool w1 = H == 0 && !pro_ss.has_value() && dph::w1_supported(M, N, K, A.stride(0), B.stride(0));
  const int ns = (H > 0 && dph::c3w_supported(M, N, K, A.stride(0), B.stride(0))) ? dph::c3w_splits(M, N, K)
                 : w1                                                              ? dph::w1_splits(M, N, K)
                                                                                  : dph::ts_gemm_tn_splits(M, N, K);
  Tensor part = at::empty({(int64_t)ns * N * K}, A.options().dtype(at::kFloat));
  dph::ts_gemm_tn(A.data_ptr(), B.data_ptr(), part.data_ptr<float>(), C.data_ptr(), M, N, K, A.stride(0),
                  B.stride(0), ns, dt_code(C), accumulate, cur_stream(), (int)H, (int)W, pro_ptr(pro_ss, K, H, A));
}

// ---------------------------------------------------------------- gathered implicit GEMM (strided convolutions)
// geo = [Hs, Ws, Ho, Wo, sy, sx, by, bx, Hd, Wd, ty, tx, tby, tbx, ntaps, tdy[0..8], tdx[0..8]] (kernels.h ConvGeo)
dph::ConvGeo make_geo(at::IntArrayRef geo, int64_t src_rows, bool chunk_taps = false) {
  TORCH_CHECK(geo.size() == 15 + 18, "conv geometry: 33 integers expected");
  dph::ConvGeo g{};
  int* f[15] = {&g.Hs, &g.Ws, &g.Ho, &g.Wo, &g.sy, &g.sx, &g.by, &g.bx, &g.Hd, &g.Wd, &g.ty, &g.tx, &g.tby, &g.tbx, &g.ntaps};
  for (int i = 0; i < 15; ++i) *f[i] = (int)geo[i];
  for (int t = 0; t < 9; ++t) {
    g.tdy[t] = (int)geo[15 + t];
    g.tdx[t] = (int)geo[24 + t];
  }
  g.src_rows = src_rows;
  TORCH_CHECK(g.Hs > 0 && g.Ws > 0 && g.Ho > 0 && g.Wo > 0 && g.Hd > 0 && g.Wd > 0 && g.ntaps >= 1 &&
                  (chunk_taps ? g.tdx[0] > 0 : g.ntaps <= 9),
              "conv geometry: positive grids and 1..9 taps required (chunk taps: any count, tdx[0] taps per row)");
  TORCH_CHECK(src_rows % ((int64_t)g.Hs * g.Ws) == 0, "conv geometry: source rows must be whole Hs x Ws images");
  // every destination row of every image must land inside the Hd x Wd grid (scatter bound, checked on the host)
  const int64_t ymax = (int64_t)g.ty * (g.Ho - 1) + g.tby, xmax = (int64_t)g.tx * (g.Wo - 1) + g.tbx;
  TORCH_CHECK(g.tby >= 0 && g.tbx >= 0 && ymax < g.Hd && xmax < g.Wd, "conv geometry: destination outside the grid");
  return g;
}

// C[rows(g), N] (rows stored per g's destination map) = A_gathered[M, K] B[N, K]^T; M = images * Ho * Wo.
// out (optional): the destination tensor (parity classes of one input gradient share it); stats: BatchNorm partials;
// bias (optional): a per-output-channel fp32 / bf16 bias added in the epilogue (before the statistics).
std::vector<Tensor> convg_nt(const Tensor& A, const Tensor& B, at::IntArrayRef geo, const c10::optional<Tensor>& out,
                             bool stats, bool chunk_taps, const c10::optional<Tensor>& bias = c10::nullopt) {
  check_cuda(A, "A");
  c10::DeviceGuard dg(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16,
              "convg_nt: bf16 2-D operands");
  const dph::ConvGeo g = make_geo(geo, A.size(0), chunk_taps);
  const int64_t imgs = A.size(0) / ((int64_t)g.Hs * g.Ws);
  const int64_t M = imgs * g.Ho * g.Wo, N = B.size(0), K = B.size(1);
  TORCH_CHECK(chunk_taps ? (A.size(1) == 8 && K % 64 == 0) : K == g.ntaps * A.size(1),
              "convg_nt: B must be [N, ntaps * Cin] (chunk taps: A [rows, 8], K a multiple of 64)");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "convg_nt: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::convg_supported(M, N, K, A.stride(0), B.stride(0), g, chunk_taps),
              "convg_nt: unsupported shape (N % 64, Cin % 64, 32-bit offsets)");
  check_align16(A, "A");
  check_align16(B, "B");
  const int64_t rows = imgs * g.Hd * g.Wd;
  Tensor C;
  if (out.has_value()) {
    C = *out;
    TORCH_CHECK(C.scalar_type() == at::kBFloat16 && C.dim() == 2 && C.size(0) == rows && C.size(1) == N &&
                    C.stride(1) == 1 && C.stride(0) % 8 == 0 && C.device() == A.device(),
                "convg_nt: out must be a bf16 [images * Hd * Wd, N] row-major tensor");
    check_align16(C, "out");
  } else {
    C = at::empty({rows, N}, A.options());
  }
  std::vector<Tensor> res{C};
  float* sp = nullptr;
  if (stats) {
    TORCH_CHECK(rows == M, "convg_nt: statistics need the identity destination map");
    const int64_t nmb = (M + 127) / 128;
    Tensor st = at::empty({2 * nmb * N + nmb}, A.options().dtype(at::kFloat));
    sp = st.data_ptr<float>();
    res.push_back(st);
  }
  const void* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK((bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16) && bias->numel() == N &&
                    bias->is_contiguous() && bias->device() == A.device(),
                "convg_nt: bias must be a contiguous fp32 / bf16 [N] tensor");
    bp = bias->data_ptr();
  }
  dph::convg_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, A.stride(0), B.stride(0), C.stride(0), g,
                  cur_stream(), sp, chunk_taps, bp, bias.has_value() && bias->scalar_type() == at::kBFloat16);
  return res;
}

std::vector<Tensor> convg_nt_fresh(const Tensor& A, const Tensor& B, at::IntArrayRef geo, bool stats, bool chunk_taps,
                                   const c10::optional<Tensor>& bias) {
  return convg_nt(A, B, geo, c10::nullopt, stats, chunk_taps, bias);
}

void convg_nt_out_(const Tensor& A, const Tensor& B, at::IntArrayRef geo, Tensor out) {
  (void)convg_nt(A, B, geo, out, false, false);
}

// C[N, ntaps * Cin] (+)= dY[M, N]^T X_gathered[M, ntaps * Cin]; X = the [images * Hs * Ws, Cin] input.
void convg_tn_(Tensor C, const Tensor& A, const Tensor& B, at::IntArrayRef geo, bool accumulate, bool chunk_taps) {
  check_cuda(A, "A");
  c10::DeviceGuard dg(A.device());
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2 && A.scalar_type() == at::kBFloat16 &&
                  B.scalar_type() == at::kBFloat16,
              "convg_tn_: bf16 2-D operands");
  const dph::ConvGeo g = make_geo(geo, B.size(0), chunk_taps);
  const int64_t imgs = B.size(0) / ((int64_t)g.Hs * g.Ws);
  const int64_t M = A.size(0), N = A.size(1), K = chunk_taps ? C.size(1) : g.ntaps * B.size(1);
  TORCH_CHECK(!chunk_taps || B.size(1) == 8, "convg_tn_: chunk taps need an [rows, 8] input");
  TORCH_CHECK(M == imgs * g.Ho * g.Wo, "convg_tn_: dY rows must be images * Ho * Wo");
  TORCH_CHECK(C.size(0) == N && C.size(1) == K && C.is_contiguous(), "convg_tn_: C must be [N, ntaps * Cin]");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0,
              "convg_tn_: row-major operands with 16-B aligned rows required");
  TORCH_CHECK(dph::c3wg_supported(M, N, K, A.stride(0), B.stride(0), g, chunk_taps),
              "convg_tn_: unsupported shape (N % 64, ntaps * Cin % 192, Cin % 64; one tap: Cin % 64)");
  TORCH_CHECK(C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat, "convg_tn_: C bf16 or fp32");
  check_align16(A, "A");
  check_align16(B, "B");
  const int ns = dph::c3wg_splits(M, N, K, chunk_taps, g.ntaps == 1);
  Tensor part = at::empty({(int64_t)ns * N * K}, A.options().dtype(at::kFloat));
  dph::ts_gemm_tn_geo(A.data_ptr(), B.data_ptr(), part.data_ptr<float>(), C.data_ptr(), M, N, K, A.stride(0),
                      B.stride(0), ns, dt_code(C), accumulate, g, cur_stream(), chunk_taps);
}

// ------------------------------------------------------------------------------------------------ channel sum
// x channels-last [N, C, H, W] or contiguous [M, C] -> [C] in out_dtype (the convolution bias gradient).
Tensor channel_sum(const Tensor& x, at::ScalarType out_dtype) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK((x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast)) || (x.dim() == 2 && x.is_contiguous()),
              "channel_sum: channels-last [N, C, H, W] or contiguous [M, C]");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "channel_sum: fp32 / bf16 output");
  const int64_t C = x.size(1), M = C ? x.numel() / C : 0;
  auto out = at::empty({C}, x.options().dtype(out_dtype));
  if (C == 0) return out;
  auto part = at::empty({(int64_t)dph::chsum_partial_blocks(M, C) * C}, x.options().dtype(at::kFloat));
  dph::chsum(x.data_ptr(), part.data_ptr<float>(), out.data_ptr(), M, C, dt_code(x),
             out_dtype == at::kBFloat16 ? dph::kBF16 : dph::kF32, cur_stream());
  return out;
}

// channel_sum written into an existing [C] buffer (a parameter's gradient-bucket view: no separate copy)
void channel_sum_into_(const Tensor& x, Tensor out) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK((x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast)) || (x.dim() == 2 && x.is_contiguous()),
              "channel_sum_into_: channels-last [N, C, H, W] or contiguous [M, C]");
  const int64_t C = x.size(1), M = C ? x.numel() / C : 0;
  TORCH_CHECK(out.numel() == C && out.is_contiguous() && out.device() == x.device() &&
                  (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16),
              "channel_sum_into_: out must be a contiguous fp32 / bf16 tensor of C elements");
  if (C == 0) return;
  auto part = at::empty({(int64_t)dph::chsum_partial_blocks(M, C) * C}, x.options().dtype(at::kFloat));
  dph::chsum(x.data_ptr(), part.data_ptr<float>(), out.data_ptr(), M, C, dt_code(x),
             out.scalar_type() == at::kBFloat16 ? dph::kBF16 : dph::kF32, cur_stream());
}

// ------------------------------------------------------------------------------------------------ max pooling
// x: channels-last [N, C, H, W], C % 8 == 0; k = 3 (3x3 / 2 / 1) or 2 (2x2 / 2 / 0).
// Returns (y channels-last [N, C, Ho, Wo], tap uint8 [N, Ho, Wo, C]).
std::tuple<Tensor, Tensor> maxpool_s2_fwd(const Tensor& x, int64_t k) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(k == 2 || k == 3, "maxpool_s2: kernel 2 or 3");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_s2: channels-last [N, C, H, W] input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && H >= k - 1 && W >= k - 1, "maxpool_s2: channels must be a multiple of 8");
  check_align16(x, "x");
  const int64_t Ho = dph::maxpool_s2_out(H, (int)k), Wo = dph::maxpool_s2_out(W, (int)k);
  TORCH_CHECK(Ho >= 1 && Wo >= 1, "maxpool_s2: empty output");
  auto y = at::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto tap = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  dph::maxpool_s2_fwd(x.data_ptr(), y.data_ptr(), tap.data_ptr<uint8_t>(), N, H, W, C, (int)k, dt_code(x),
                      cur_stream());
  return {y, tap};
}

// The optional second gradient of a pooling input: channels [add_off, add_off + C) of a channels-last [N, *, H, W]
// tensor of dy's dtype (SimpleUNet: the skip connection's slice of d(concat)).  Returns (pointer, row stride).
static std::pair<const void*, int64_t> pool_add_operand(const c10::optional<Tensor>& add, int64_t add_off,
                                                        const Tensor& dy, int64_t H, int64_t W, const char* what) {
  if (!add.has_value()) return {nullptr, 0};
  const Tensor& a = *add;
  const int64_t C = dy.size(1);
  TORCH_CHECK(a.dim() == 4 && a.size(0) == dy.size(0) && a.size(2) == H && a.size(3) == W && add_off >= 0 &&
                  add_off % 8 == 0 && add_off + C <= a.size(1) && a.scalar_type() == dy.scalar_type() &&
                  a.device() == dy.device() && a.is_contiguous(at::MemoryFormat::ChannelsLast),
              what, ": add must be a channels-last [N, >= add_off + C, H, W] tensor of dy's dtype");
  check_align16(a, "add");
  return {static_cast<const char*>(a.data_ptr()) + add_off * a.element_size(), a.size(1)};
}

Tensor maxpool_s2_bwd(const Tensor& dy, const Tensor& tap, int64_t H, int64_t W, int64_t k,
                      const c10::optional<Tensor>& add, int64_t add_off) {
  check_cuda(dy, "dy");
  c10::DeviceGuard g(dy.device());
  TORCH_CHECK(k == 2 || k == 3, "maxpool_s2_bwd: kernel 2 or 3");
  TORCH_CHECK(dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_s2_bwd: channels-last [N, C, Ho, Wo] gradient");
  const int64_t N = dy.size(0), C = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(C % 8 == 0 && Ho == dph::maxpool_s2_out(H, (int)k) && Wo == dph::maxpool_s2_out(W, (int)k),
              "maxpool_s2_bwd: gradient shape does not match a stride-2 pooling of ", H, "x", W);
  TORCH_CHECK(tap.scalar_type() == at::kByte && tap.is_contiguous() && tap.dim() == 4 && tap.size(0) == N &&
                  tap.size(1) == Ho && tap.size(2) == Wo && tap.size(3) == C && tap.device() == dy.device(),
              "maxpool_s2_bwd: tap must be the forward's uint8 [N, Ho, Wo, C]");
  check_align16(dy, "dy");
  const auto ad = pool_add_operand(add, add_off, dy, H, W, "maxpool_s2_bwd");
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  dph::maxpool_s2_bwd(dy.data_ptr(), tap.data_ptr<uint8_t>(), dx.data_ptr(), N, H, W, C, (int)k, dt_code(dy),
                      cur_stream(), ad.first, ad.second);
  return dx;
}

// maxpool_s2_bwd whose input x is a training-mode BatchNorm + ReLU output (the ResNet stem): also that BatchNorm's
// backward reduction partials [blocks, 2C] (mask from x with the forward's ss = [scale | shift]), for bn_act_bwd's
// pre_part -- the BatchNorm then skips its reduction pass over dx and x.
std::tuple<Tensor, Tensor> maxpool_s2_bwd_bnred(const Tensor& dy, const Tensor& tap, int64_t H, int64_t W, int64_t k,
                                                const Tensor& x, const Tensor& mean, const Tensor& invstd,
                                                const Tensor& ss, const c10::optional<Tensor>& add,
                                                int64_t add_off) {
  check_cuda(dy, "dy");
  c10::DeviceGuard g(dy.device());
  TORCH_CHECK(k == 2 || k == 3, "maxpool_s2_bwd_bnred: kernel 2 or 3");
  TORCH_CHECK(dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy.scalar_type() == at::kBFloat16,
              "maxpool_s2_bwd_bnred: channels-last bf16 [N, C, Ho, Wo] gradient");
  const int64_t N = dy.size(0), C = dy.size(1), Ho = dy.size(2), Wo = dy.size(3);
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0 && Ho == dph::maxpool_s2_out(H, (int)k) &&
                  Wo == dph::maxpool_s2_out(W, (int)k),
              "maxpool_s2_bwd_bnred: gradient shape / channel count (C / 8 must divide 256)");
  TORCH_CHECK(tap.scalar_type() == at::kByte && tap.is_contiguous() && tap.dim() == 4 && tap.size(0) == N &&
                  tap.size(1) == Ho && tap.size(2) == Wo && tap.size(3) == C && tap.device() == dy.device(),
              "maxpool_s2_bwd_bnred: tap must be the forward's uint8 [N, Ho, Wo, C]");
  TORCH_CHECK(x.dim() == 4 && x.size(0) == N && x.size(1) == C && x.size(2) == H && x.size(3) == W &&
                  x.scalar_type() == at::kBFloat16 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  x.device() == dy.device(),
              "maxpool_s2_bwd_bnred: x must be the BatchNorm's bf16 channels-last [N, C, H, W] input");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && invstd.scalar_type() == at::kFloat && ss.scalar_type() == at::kFloat &&
                  mean.numel() == C && invstd.numel() == C && ss.numel() == 2 * C && mean.is_contiguous() &&
                  invstd.is_contiguous() && ss.is_contiguous(),
              "maxpool_s2_bwd_bnred: fp32 mean / invstd [C], ss [2C]");
  check_align16(dy, "dy");
  check_align16(x, "x");
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor part = at::empty({dph::maxpool_s2_bwd_bnred_blocks(N, H, W, C), 2 * C}, dy.options().dtype(at::kFloat));
  dph::BnRed r;
  r.x = x.data_ptr();
  r.mean = mean.data_ptr<float>();
  r.invstd = invstd.data_ptr<float>();
  r.ss = ss.data_ptr<float>();
  r.part = part.data_ptr<float>();
  const auto ad = pool_add_operand(add, add_off, dy, H, W, "maxpool_s2_bwd_bnred");
  dph::maxpool_s2_bwd_bnred(dy.data_ptr(), tap.data_ptr<uint8_t>(), dx.data_ptr(), N, H, W, C, (int)k, r,
                            cur_stream(), ad.first, ad.second);
  return {dx, part};
}

// ------------------------------------------------------------------------------------------------ UNet up-path
// y2: [N*H*W, 4*Co] ConvTranspose2d(2, 2) GEMM output; skip: channels-last [N, Cs, Ho, Wo].
// Returns channels-last [N, Co + Cs, Ho, Wo] = cat([bilinear(pixel_shuffle(y2) + bias, (Ho, Wo)), skip]).
Tensor upcat_fwd(const Tensor& y2, const c10::optional<Tensor>& bias, const Tensor& skip, int64_t H, int64_t W) {
  check_cuda(y2, "y2");
  check_cuda(skip, "skip");
  c10::DeviceGuard g(y2.device());
  TORCH_CHECK(skip.dim() == 4 && skip.is_contiguous(at::MemoryFormat::ChannelsLast), "upcat: channels-last skip");
  TORCH_CHECK(y2.dim() == 2 && y2.is_contiguous() && y2.scalar_type() == skip.scalar_type(),
              "upcat: contiguous [N*H*W, 4*Co] GEMM output of the skip's dtype");
  const int64_t N = skip.size(0), Cs = skip.size(1), Ho = skip.size(2), Wo = skip.size(3);
  TORCH_CHECK(H > 0 && W > 0 && y2.size(0) == N * H * W && y2.size(1) % 32 == 0, "upcat: y2 must be [N*H*W, 4*Co]");
  const int64_t Co = y2.size(1) / 4;
  TORCH_CHECK(Co % 8 == 0 && Cs % 8 == 0, "upcat: channel counts must be multiples of 8");
  TORCH_CHECK(Ho > 0 && Wo > 0 && Ho <= 4 * H && Wo <= 4 * W && 4 * Ho >= 2 * H && 4 * Wo >= 2 * W,
              "upcat: resize ratio outside [0.5, 2]");
  const float* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == Co &&
                    bias->device() == y2.device(),
                "upcat: fp32 bias [Co]");
    bp = bias->data_ptr<float>();
  }
  check_align16(y2, "y2");
  check_align16(skip, "skip");
  auto out = at::empty({N, Co + Cs, Ho, Wo}, skip.options().memory_format(at::MemoryFormat::ChannelsLast));
  dph::upcat_fwd(y2.data_ptr(), bp, skip.data_ptr(), out.data_ptr(), N, H, W, Co, Ho, Wo, Cs, dt_code(skip),
                 cur_stream());
  return out;
}

// dcat: channels-last [N, Co + Cs, Ho, Wo]; returns (dy2 [N*H*W, 4*Co], dskip channels-last [N, Cs, Ho, Wo])
// want_skip false: dskip is an empty tensor and the kernel writes only dy2.
std::tuple<Tensor, Tensor> upcat_bwd(const Tensor& dcat, int64_t H, int64_t W, int64_t Co, bool want_skip) {
  check_cuda(dcat, "dcat");
  c10::DeviceGuard g(dcat.device());
  TORCH_CHECK(dcat.dim() == 4 && dcat.is_contiguous(at::MemoryFormat::ChannelsLast), "upcat_bwd: channels-last dcat");
  const int64_t N = dcat.size(0), Ct = dcat.size(1), Ho = dcat.size(2), Wo = dcat.size(3), Cs = Ct - Co;
  TORCH_CHECK(Co > 0 && Co % 8 == 0 && Cs >= 0 && Cs % 8 == 0 && H > 0 && W > 0, "upcat_bwd: bad channel split");
  TORCH_CHECK(Ho <= 4 * H && Wo <= 4 * W && 4 * Ho >= 2 * H && 4 * Wo >= 2 * W, "upcat_bwd: resize ratio outside [0.5, 2]");
  check_align16(dcat, "dcat");
  auto dy = at::empty({N * H * W, 4 * Co}, dcat.options());
  auto dskip = want_skip ? at::empty({N, Cs, Ho, Wo}, dcat.options().memory_format(at::MemoryFormat::ChannelsLast))
                         : at::empty({0}, dcat.options());
  dph::upcat_bwd(dcat.data_ptr(), dy.data_ptr(), want_skip ? dskip.data_ptr() : nullptr, N, H, W, Co, Ho, Wo, Cs,
                 dt_code(dcat), cur_stream());
  return {dy, dskip};
}

// ------------------------------------------------------------------------------------------------ transpose
// [R, C] bf16 rows (any row stride) -> [R, cols] with zero columns C..cols-1 (cols % 8 == 0)
Tensor pad_cols(const Tensor& x, int64_t cols) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kBFloat16 && x.stride(1) == 1, "pad_cols: bf16 [R, C] rows");
  TORCH_CHECK(cols % 8 == 0 && cols >= x.size(1), "pad_cols: cols must be a multiple of 8 and >= C");
  auto out = at::empty({x.size(0), cols}, x.options());
  dph::pad_cols(x.data_ptr(), out.data_ptr(), x.size(0), x.size(1), x.stride(0), cols, cur_stream());
  return out;
}

Tensor transpose2d(const Tensor& x) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kBFloat16 && x.stride(1) == 1, "transpose2d: bf16 [R, C] rows");
  TORCH_CHECK(x.stride(0) % 8 == 0, "transpose2d: leading dim must be a multiple of 8");
  check_align16(x, "x");
  const int64_t R = x.size(0), C = x.size(1);
  auto out = at::empty({C, R}, x.options());
  TORCH_CHECK(R % 8 == 0, "transpose2d: rows must be a multiple of 8 (16-B output rows)");
  dph::transpose2d(x.data_ptr(), out.data_ptr(), R, C, x.stride(0), R, cur_stream());
  return out;
}

// [cout, cin, 3, 3] channels-last bf16 weight -> [cin, 9 * cout]: the flipped, channel-transposed weight of the 3x3
// convolution's input gradient (what w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, 9 * cout) copies element-wise)
Tensor conv3x3_dgrad_weight(const Tensor& w) {
  c10::DeviceGuard g(w.device());
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.scalar_type() == at::kBFloat16 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_dgrad_weight: channels-last bf16 [cout, cin, 3, 3]");
  const int64_t cout = w.size(0), cin = w.size(1);
  TORCH_CHECK(cout % 8 == 0 && cin % 8 == 0, "conv3x3_dgrad_weight: channels must be multiples of 8");
  check_align16(w, "w");
  auto out = at::empty({cin, 9 * cout}, w.options().memory_format(at::MemoryFormat::Contiguous));
  dph::conv3x3_dgrad_weight(w.data_ptr(), out.data_ptr(), cout, cin, cur_stream());
  return out;
}

// ------------------------------------------------------------------------------------------------ BatchNorm+act
// x: channels-last [N, C, H, W] (or contiguous [M, C]); statistics over everything but C.
int64_t bn_channels(const Tensor& x) {
  TORCH_CHECK(x.dim() == 4 || x.dim() == 2, "bn_act: [N, C, H, W] channels-last or [M, C] input");
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "bn_act: 4-D input must be channels-last");
  } else {
    TORCH_CHECK(x.is_contiguous(), "bn_act: 2-D input must be contiguous");
  }
  const int64_t C = x.size(1);
  TORCH_CHECK(dph::bn_nhwc_supported(C), "bn_act: channels must be a power of two in [8, 2048]");
  check_align16(x, "x");
  return C;
}
void check_like(const Tensor& a, const Tensor& x, const char* name) {
  TORCH_CHECK(a.sizes() == x.sizes() && a.scalar_type() == x.scalar_type() && a.strides() == x.strides(),
              "bn_act: ", name, " must match x (shape, dtype, channels-last layout)");
}

std::tuple<Tensor, Tensor, Tensor, Tensor> bn_act_fwd(const Tensor& x, const c10::optional<Tensor>& res,
                                              const c10::optional<Tensor>& w, const c10::optional<Tensor>& b,
                                              const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar,
                                              double momentum, double eps, bool relu,
                                              const c10::optional<Tensor>& pre_stats,
                                              const c10::optional<Tensor>& num_batches_tracked,
                                              const c10::optional<Tensor>& relu_mask_out, bool apply) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const int64_t C = bn_channels(x), M = x.numel() / C;
  if (res) check_like(*res, x, "residual");
  TORCH_CHECK(!w || (w->numel() == C && w->is_contiguous()), "bn_act: weight [C]");
  TORCH_CHECK(!b || (b->numel() == C && b->is_contiguous()), "bn_act: bias [C]");
  TORCH_CHECK(!w || !b || w->scalar_type() == b->scalar_type(), "bn_act: weight/bias dtype mismatch");
  TORCH_CHECK((!rmean && !rvar) || (rmean && rvar && rmean->numel() == C && rvar->numel() == C &&
                                    rmean->scalar_type() == rvar->scalar_type()),
              "bn_act: running stats [C] (both or none)");
  auto fopt = x.options().dtype(at::kFloat);
  // apply = false: statistics, running-stat update and [scale | shift] only -- the consumer folds the apply into its
  // operand load (ts_gemm_nt / ts_gemm_tn_ pro_ss)
  TORCH_CHECK(apply || (!res.has_value() && !relu_mask_out.has_value()), "bn_act_fwd: apply=False takes no residual");
  auto y = apply ? at::empty_like(x) : at::empty({0}, x.options());
  auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt);
  auto ss = at::empty({2 * C}, fopt);   // [scale | shift]: the backward recomputes the ReLU mask from them
  const Tensor* pre = pre_stats.has_value() ? &*pre_stats : nullptr;
  int64_t* nbt = nullptr;   // incremented by the finalize kernel (nn.BatchNorm2d's num_batches_tracked += 1)
  if (num_batches_tracked.has_value()) {
    TORCH_CHECK(num_batches_tracked->scalar_type() == at::kLong && num_batches_tracked->numel() == 1 &&
                    num_batches_tracked->device() == x.device(),
                "bn_act_fwd: num_batches_tracked must be an int64 scalar on x's device");
    nbt = num_batches_tracked->data_ptr<int64_t>();
  }
  int pre_groups = 0;
  if (pre) {
    TORCH_CHECK(pre->scalar_type() == at::kFloat && pre->is_contiguous() && pre->numel() % (2 * C + 1) == 0 &&
                    pre->device() == x.device(),
                "bn_act_fwd: pre_stats must be fp32 [mean G*C | M2 G*C | rows G]");
    pre_groups = (int)(pre->numel() / (2 * C + 1));
  }
  uint8_t* rmask = nullptr;   // [y > 0] bits for the backward (ReLU after a residual add: y is not re-read)
  if (relu_mask_out.has_value()) {
    // the kernel writes the mask on the residual + ReLU path only (bn_apply): without a residual the bits would
    // stay uninitialised and bn_act_bwd would read them as the ReLU mask
    TORCH_CHECK(relu && res.has_value() && relu_mask_out->scalar_type() == at::kByte &&
                    relu_mask_out->is_contiguous() && relu_mask_out->numel() == M * C / 8 &&
                    relu_mask_out->device() == x.device(),
                "bn_act_fwd: relu_mask_out must be a contiguous uint8 [M * C / 8], with relu set and a residual");
    rmask = relu_mask_out->data_ptr<uint8_t>();
  }
  const int G = dph::bn_partial_blocks(M, C);
  auto ws = at::empty({2 * (int64_t)G * C + G}, fopt);
  const int pdt = w ? dt_code(*w) : (b ? dt_code(*b) : dph::kF32);
  const int rdt = rmean ? dt_code(*rmean) : dph::kF32;
  dph::bn_fwd_train(x.data_ptr(), res ? res->data_ptr() : nullptr, apply ? y.data_ptr() : nullptr,
                    w ? w->data_ptr() : nullptr,
                    b ? b->data_ptr() : nullptr, rmean ? rmean->data_ptr() : nullptr,
                    rvar ? rvar->data_ptr() : nullptr, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                    ss.data_ptr<float>(), ss.data_ptr<float>() + C, ws.data_ptr<float>(), M, C, (float)momentum,
                    (float)eps, relu, dt_code(x), pdt, rdt, cur_stream(), pre ? pre->data_ptr<float>() : nullptr,
                    pre_groups, nbt, rmask);
  return {y, mean, invstd, ss};
}

// relu(BN_a(x) + BN_b(z)) from both BatchNorms' forward [scale | shift] (bn_act_fwd with apply=False), plus the
// [y > 0] bits into relu_mask (uint8 [M * C / 8]).
Tensor bn_act_apply_resbn(const Tensor& x, const Tensor& ss, const Tensor& z, const Tensor& zss, Tensor relu_mask) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const int64_t C = bn_channels(x), M = x.numel() / C;
  check_like(z, x, "z");
  TORCH_CHECK(ss.scalar_type() == at::kFloat && zss.scalar_type() == at::kFloat && ss.numel() == 2 * C &&
                  zss.numel() == 2 * C && ss.is_contiguous() && zss.is_contiguous(),
              "bn_act_apply_resbn: fp32 [scale | shift] of 2C each");
  TORCH_CHECK(relu_mask.scalar_type() == at::kByte && relu_mask.is_contiguous() && relu_mask.numel() == M * C / 8 &&
                  relu_mask.device() == x.device(),
              "bn_act_apply_resbn: relu_mask must be a contiguous uint8 [M * C / 8]");
  auto y = at::empty_like(x);
  dph::bn_apply_resbn(x.data_ptr(), z.data_ptr(), ss.data_ptr<float>(), zss.data_ptr<float>(), y.data_ptr(),
                      relu_mask.data_ptr<uint8_t>(), M, C, dt_code(x), cur_stream());
  return y;
}

Tensor bn_act_apply(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& scale, const Tensor& shift,
                    bool relu) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const int64_t C = bn_channels(x), M = x.numel() / C;
  if (res) check_like(*res, x, "residual");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && shift.scalar_type() == at::kFloat && scale.numel() == C &&
                  shift.numel() == C && scale.is_contiguous() && shift.is_contiguous(),
              "bn_act_apply: fp32 scale/shift [C]");
  auto y = at::empty_like(x);
  dph::bn_apply(x.data_ptr(), res ? res->data_ptr() : nullptr, scale.data_ptr<float>(), shift.data_ptr<float>(),
                y.data_ptr(), M, C, relu, dt_code(x), cur_stream());
  return y;
}

std::tuple<Tensor, Tensor, Tensor, Tensor> bn_act_bwd(const Tensor& dy, const Tensor& y, const Tensor& x,
                                                      const Tensor& mean, const Tensor& invstd,
                                                      const c10::optional<Tensor>& w, bool relu, bool need_dres,
                                                      bool need_dwb, const c10::optional<Tensor>& xmask_ss,
                                                      const c10::optional<Tensor>& dw_out,
                                                      const c10::optional<Tensor>& db_out,
                                                      const c10::optional<Tensor>& relu_mask,
                                                      const c10::optional<Tensor>& pre_part) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const int64_t C = bn_channels(x), M = x.numel() / C;
  check_like(dy, x, "dy");
  const bool bm = relu && relu_mask.has_value();
  if (bm) {
    TORCH_CHECK(relu_mask->scalar_type() == at::kByte && relu_mask->is_contiguous() &&
                    relu_mask->numel() == M * C / 8 && relu_mask->device() == x.device(),
                "bn_act_bwd: relu_mask must be the forward's uint8 [M * C / 8] bits");
  }
  const bool xm = relu && !bm && xmask_ss.has_value();
  if (bm) {
  } else if (xm) {
    TORCH_CHECK(xmask_ss->scalar_type() == at::kFloat && xmask_ss->numel() == 2 * C && xmask_ss->is_contiguous(),
                "bn_act_bwd: xmask_ss must be the forward's fp32 [scale | shift]");
  } else {
    check_like(y, x, "y");
  }
  auto fopt = x.options().dtype(at::kFloat);
  auto dx = at::empty_like(x);
  Tensor dres = need_dres ? at::empty_like(x) : at::empty({0}, x.options());
  const at::ScalarType pt = w ? w->scalar_type() : at::kFloat;
  // dw_out / db_out: write the parameter gradients straight into caller buffers (the engine's gradient bucket)
  auto out_or_new = [&](const c10::optional<Tensor>& o, const char* name) {
    if (!need_dwb) return at::empty({0}, fopt);
    if (o.has_value()) {
      TORCH_CHECK(o->numel() == C && o->is_contiguous() && o->scalar_type() == pt && o->device() == x.device(),
                  "bn_act_bwd: ", name, " must be a contiguous [C] tensor of the weight dtype");
      return *o;
    }
    return at::empty({C}, x.options().dtype(pt));
  };
  Tensor dw = out_or_new(dw_out, "dw_out");
  Tensor db = out_or_new(db_out, "db_out");
  const int G = dph::bn_partial_blocks(M, C);
  auto ws = at::empty({2 * (int64_t)G * C + 3 * C}, fopt);
  int pre_groups = 0;
  if (pre_part.has_value()) {   // the producer's epilogue reduced dy (ts_gemm_nt_bnred)
    TORCH_CHECK(pre_part->scalar_type() == at::kFloat && pre_part->dim() == 2 && pre_part->size(1) == 2 * C &&
                    pre_part->is_contiguous() && pre_part->device() == x.device() && (bm || xm),
                "bn_act_bwd: pre_part must be fp32 [G, 2C] partials of a ReLU BatchNorm");
    pre_groups = (int)pre_part->size(0);
  }
  dph::bn_bwd(dy.data_ptr(), y.data_ptr(), x.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
              w ? w->data_ptr() : nullptr, dx.data_ptr(), need_dres ? dres.data_ptr() : nullptr,
              need_dwb ? dw.data_ptr() : nullptr, need_dwb ? db.data_ptr() : nullptr, ws.data_ptr<float>(), M, C, relu,
              dt_code(x), w ? dt_code(*w) : dph::kF32, cur_stream(), xm ? xmask_ss->data_ptr<float>() : nullptr,
              bm ? relu_mask->data_ptr<uint8_t>() : nullptr,
              pre_part.has_value() ? pre_part->data_ptr<float>() : nullptr, pre_groups);
  return {dx, dres, dw, db};
}

// relu(bn_a(x) + bn_b(z)) backward (the projection shortcut, ops/batchnorm.py _BNDualActFn): both BatchNorms from dy
// and the forward's ReLU bits, one fused dx pass.  Returns (dx, dz, dw_a, db_a, dw_b, db_b); *_out write the parameter
// gradients into caller buffers (the engine's buckets), pre_part_a = bn_a's partials from its consumer's epilogue.
std::vector<Tensor> bn_act_bwd_dual(const Tensor& dy, const Tensor& x, const Tensor& z, const Tensor& relu_mask,
                                    const Tensor& mean_a, const Tensor& invstd_a, const Tensor& w_a,
                                    const Tensor& mean_b, const Tensor& invstd_b, const Tensor& w_b, bool need_a,
                                    bool need_b, const c10::optional<Tensor>& dw_a_out,
                                    const c10::optional<Tensor>& db_a_out, const c10::optional<Tensor>& dw_b_out,
                                    const c10::optional<Tensor>& db_b_out, const c10::optional<Tensor>& pre_part_a) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const int64_t C = bn_channels(x), M = x.numel() / C;
  check_like(dy, x, "dy");
  check_like(z, x, "z");
  TORCH_CHECK(relu_mask.scalar_type() == at::kByte && relu_mask.is_contiguous() && relu_mask.numel() == M * C / 8 &&
                  relu_mask.device() == x.device(),
              "bn_act_bwd_dual: relu_mask must be the forward's uint8 [M * C / 8] bits");
  for (const Tensor* t : {&mean_a, &invstd_a, &mean_b, &invstd_b})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == C && t->is_contiguous(), "bn_act_bwd_dual: fp32 [C]");
  TORCH_CHECK(w_a.numel() == C && w_b.numel() == C && w_a.is_contiguous() && w_b.is_contiguous() &&
                  w_a.scalar_type() == w_b.scalar_type(),
              "bn_act_bwd_dual: weights [C] of one dtype");
  auto fopt = x.options().dtype(at::kFloat);
  const at::ScalarType pt = w_a.scalar_type();
  auto out_or_new = [&](bool need, const c10::optional<Tensor>& o, const char* name) {
    if (!need) return at::empty({0}, fopt);
    if (o.has_value()) {
      TORCH_CHECK(o->numel() == C && o->is_contiguous() && o->scalar_type() == pt && o->device() == x.device(),
                  "bn_act_bwd_dual: ", name, " must be a contiguous [C] tensor of the weight dtype");
      return *o;
    }
    return at::empty({C}, x.options().dtype(pt));
  };
  Tensor dwa = out_or_new(need_a, dw_a_out, "dw_a_out"), dba = out_or_new(need_a, db_a_out, "db_a_out");
  Tensor dwb = out_or_new(need_b, dw_b_out, "dw_b_out"), dbb = out_or_new(need_b, db_b_out, "db_b_out");
  int pre_groups = 0;
  if (pre_part_a.has_value()) {
    TORCH_CHECK(pre_part_a->scalar_type() == at::kFloat && pre_part_a->dim() == 2 && pre_part_a->size(1) == 2 * C &&
                    pre_part_a->is_contiguous() && pre_part_a->device() == x.device(),
                "bn_act_bwd_dual: pre_part_a must be fp32 [G, 2C]");
    pre_groups = (int)pre_part_a->size(0);
  }
  const int G = dph::bn_partial_blocks(M, C);
  auto wsa = at::empty({2 * (int64_t)G * C + 3 * C}, fopt), wsb = at::empty({2 * (int64_t)G * C + 3 * C}, fopt);
  auto dx = at::empty_like(x), dz = at::empty_like(z);
  dph::bn_bwd_dual(dy.data_ptr(), relu_mask.data_ptr<uint8_t>(), x.data_ptr(), z.data_ptr(), mean_a.data_ptr<float>(),
                   invstd_a.data_ptr<float>(), w_a.data_ptr(), mean_b.data_ptr<float>(), invstd_b.data_ptr<float>(),
                   w_b.data_ptr(), dx.data_ptr(), dz.data_ptr(), need_a ? dwa.data_ptr() : nullptr,
                   need_a ? dba.data_ptr() : nullptr, need_b ? dwb.data_ptr() : nullptr,
                   need_b ? dbb.data_ptr() : nullptr, wsa.data_ptr<float>(), wsb.data_ptr<float>(), M, C, dt_code(x),
                   dt_code(w_a), cur_stream(), pre_part_a.has_value() ? pre_part_a->data_ptr<float>() : nullptr,
                   pre_groups);
  return {dx, dz, dwa, dba, dwb, dbb};
}

// ------------------------------------------------------------------------------ latitude-weighted MSE
// Row step of the latitude axis in the flat storage order: W (NCHW) or W*C (channels-last).
int64_t latmse_check(const Tensor& p, const Tensor& t) {
  check_cuda(p, "pred");
  TORCH_CHECK(p.dim() == 4 && p.sizes() == t.sizes() && p.strides() == t.strides() &&
                  p.scalar_type() == t.scalar_type(),
              "latmse: [B, C, H, W] pred / target of equal shape, layout and dtype");
  check_align16(p, "pred");
  check_align16(t, "target");
  if (p.is_contiguous()) return p.size(3);
  TORCH_CHECK(p.is_contiguous(at::MemoryFormat::ChannelsLast), "latmse: NCHW- or channels-last-contiguous operands");
  return p.size(3) * p.size(1);
}
Tensor latmse_fwd(const Tensor& p, const Tensor& t, int64_t n_global, int64_t lat_offset) {
  const int64_t step = latmse_check(p, t);
  c10::DeviceGuard g(p.device());
  const int64_t n = p.numel();
  auto fopt = p.options().dtype(at::kFloat);
  auto out = at::empty({}, fopt);
  auto part = at::empty({dph::latmse_partial_blocks(n)}, fopt);
  dph::latmse_fwd(p.data_ptr(), t.data_ptr(), part.data_ptr<float>(), out.data_ptr<float>(), n, p.size(2), step,
                  n_global, lat_offset, dt_code(p), cur_stream());
  return out;
}
std::tuple<Tensor, Tensor> latmse_bwd(const Tensor& gloss, const Tensor& p, const Tensor& t, int64_t n_global,
                                      int64_t lat_offset, bool need_dtarget) {
  const int64_t step = latmse_check(p, t);
  c10::DeviceGuard g(p.device());
  TORCH_CHECK(gloss.is_cuda() && gloss.scalar_type() == at::kFloat && gloss.numel() == 1, "latmse_bwd: fp32 scalar grad");
  auto dp = at::empty_like(p);
  Tensor dtg = need_dtarget ? at::empty_like(t) : at::empty({0}, p.options());
  dph::latmse_bwd(p.data_ptr(), t.data_ptr(), gloss.contiguous().data_ptr<float>(), dp.data_ptr(),
                  need_dtarget ? dtg.data_ptr() : nullptr, p.numel(), p.size(2), step, n_global, lat_offset,
                  dt_code(p), cur_stream());
  return {dp, dtg};
}

// ------------------------------------------------------------------------------ custom xGMI all-reduce
int64_t car_create_op(int64_t rank, int64_t world, int64_t max_bytes, double timeout_s) {
  return dph::car_create((int)rank, (int)world, max_bytes, timeout_s);
}
Tensor car_ipc_handle_op(int64_t ctx) {
  auto h = at::zeros({64}, at::TensorOptions().dtype(at::kByte));
  dph::car_ipc_handle(ctx, h.data_ptr());
  return h;
}
void car_open_op(int64_t ctx, const Tensor& handles) {
  TORCH_CHECK(!handles.is_cuda() && handles.scalar_type() == at::kByte && handles.dim() == 2 &&
                  handles.size(1) == 64 && handles.is_contiguous(),
              "car_open: handles must be a contiguous CPU uint8 [world, 64] tensor");
  dph::car_open(ctx, handles.data_ptr());
}
void car_allreduce_op(int64_t ctx, const Tensor& inp, Tensor& out, int64_t algo, double scale, int64_t max_blocks) {
  check_cuda(inp, "inp");
  c10::DeviceGuard g(inp.device());
  TORCH_CHECK(inp.is_contiguous() && out.is_contiguous() && inp.sizes() == out.sizes() &&
                  inp.scalar_type() == out.scalar_type(),
              "car_allreduce: contiguous inp/out of equal shape and dtype");
  check_align16(inp, "inp");
  check_align16(out, "out");
  const int64_t bytes = inp.numel() * inp.element_size();
  TORCH_CHECK(bytes % 16 == 0 && bytes <= dph::car_max_bytes(ctx), "car_allreduce: ", bytes,
              " B is not a multiple of 16 or exceeds the staging buffer");
  TORCH_CHECK(algo >= 0 && algo <= 2, "car_allreduce: algo 0 (auto), 1 (one-shot) or 2 (two-shot)");
  dph::car_allreduce(ctx, inp.data_ptr(), out.data_ptr(), bytes, dt_code(inp), (int)algo, (float)scale,
                     (int)max_blocks, cur_stream());
}
int64_t car_status_op(int64_t ctx) { return dph::car_status(ctx); }
void car_flag_op(int64_t ctx, Tensor& flag) {
  check_cuda(flag, "flag");
  TORCH_CHECK(flag.scalar_type() == at::kInt && flag.numel() >= 1, "car_flag: int32 device tensor");
  c10::DeviceGuard g(flag.device());
  dph::car_flag(ctx, flag.data_ptr<int>(), cur_stream());
}
void car_poison_op(int64_t ctx, const Tensor& flag, Tensor& gscale) {
  check_cuda(flag, "flag");
  check_cuda(gscale, "gscale");
  TORCH_CHECK(flag.scalar_type() == at::kInt && gscale.scalar_type() == at::kFloat && gscale.numel() >= 1,
              "car_poison: int32 flag and float32 gscale device tensors");
  c10::DeviceGuard g(flag.device());
  dph::car_poison(ctx, flag.data_ptr<int>(), gscale.data_ptr<float>(), cur_stream());
}
int64_t car_agreed_op(int64_t ctx) { return dph::car_agreed(ctx); }
int64_t attn_variant_op(int64_t v) { return dph::attn_set_variant((int)v); }
int64_t gemm_nt_variant_op(int64_t v) { return dph::gemm_nt_set_variant((int)v); }
int64_t gemm1_lds_op(int64_t on) { return dph::gemm1_lds_set(on != 0) ? 1 : 0; }
int64_t c3w_round_op(int64_t slots) { return dph::c3w_round_set(slots); }
void car_destroy_op(int64_t ctx) { dph::car_destroy(ctx); }

}  // namespace


// ---- forward / input-gradient GEMM with fused epilogues (csrc/gemm_nt.hip) ----
namespace {
Tensor rows2d(const Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, ": bf16 required");
  Tensor r = t.reshape({-1, t.size(-1)});
  TORCH_CHECK(r.stride(1) == 1 && r.stride(0) % 8 == 0, name, ": rows must be contiguous with 16-B aligned starts");
  check_align16(r, name);
  return r;
}
dph::GemmNtParams nt_params(const Tensor& A, const Tensor& B) {
  dph::GemmNtParams p{};
  p.A = A.data_ptr();
  p.B = B.data_ptr();
  p.M = (int)A.size(0);
  p.K = (int)A.size(1);
  p.lda = A.stride(0);
  p.ldb = B.stride(0);
  return p;
}
std::vector<int64_t> out_sizes(const Tensor& x, int64_t n) {
  auto s = x.sizes().vec();
  s.back() = n;
  return s;
}
}  // namespace

// select the gemm_nt pipeline variant (v < 0: back to the env / default); returns the active one

// C = A B^T (A [..., K], B [N, K]) -> [..., N]
Tensor gemm_nt(const Tensor& A, const Tensor& B) {
  check_cuda(A, "A");
  c10::DeviceGuard g(A.device());
  const Tensor a = rows2d(A, "gemm_nt A"), b = rows2d(B, "gemm_nt B");
  TORCH_CHECK(B.dim() == 2 && b.size(1) == a.size(1), "gemm_nt: B must be [N, K] with A's K");
  TORCH_CHECK(dph::gemm_nt_supported(dph::kNtStore, a.size(0), b.size(0), a.size(1)),
              "gemm_nt: need rows % 256, N % 8, K % 8 (got ", a.size(0), ", ", b.size(0), ", ", a.size(1), ")");
  Tensor C = at::empty(out_sizes(A, b.size(0)), A.options());
  auto p = nt_params(a, b);
  p.N = (int)b.size(0);
  p.C = C.data_ptr();
  p.ldc = b.size(0);
  dph::gemm_nt(dph::kNtStore, p, cur_stream());
  return C;
}

// x13 = x [W1; W3]^T ([..., 2H]) and h = silu(x13[:, :H]) * x13[:, H:] ([..., H]) in one pass
std::tuple<Tensor, Tensor> gemm_nt_swiglu(const Tensor& x, const Tensor& w13) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const Tensor a = rows2d(x, "gemm_nt_swiglu x"), b = rows2d(w13, "gemm_nt_swiglu w13");
  TORCH_CHECK(w13.dim() == 2 && b.size(1) == a.size(1) && b.size(0) % 2 == 0, "gemm_nt_swiglu: w13 [2H, K]");
  const int64_t H = b.size(0) / 2;
  TORCH_CHECK(dph::gemm_nt_supported(dph::kNtSwiglu, a.size(0), H, a.size(1)),
              "gemm_nt_swiglu: need rows % 256, H % 8, K % 8 (got ", a.size(0), ", ", H, ", ", a.size(1), ")");
  Tensor x13 = at::empty(out_sizes(x, 2 * H), x.options());
  Tensor h = at::empty(out_sizes(x, H), x.options());
  auto p = nt_params(a, b);
  p.N = (int)H;
  p.H = (int)H;
  p.C = x13.data_ptr();
  p.ldc = 2 * H;
  p.C2 = h.data_ptr();
  p.ldc2 = H;
  dph::gemm_nt(dph::kNtSwiglu, p, cur_stream());
  return {x13, h};
}

// gemm_nt_swiglu into caller-owned row blocks (x13_out [rows, 2H], h_out [rows, H], row-major, 16-B aligned rows):
// async tensor parallelism writes each round of the token deal straight into its slice of the full activations
void gemm_nt_swiglu_into(const Tensor& x, const Tensor& w13, Tensor x13_out, Tensor h_out) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const Tensor a = rows2d(x, "gemm_nt_swiglu_into x"), b = rows2d(w13, "gemm_nt_swiglu_into w13");
  TORCH_CHECK(w13.dim() == 2 && b.size(1) == a.size(1) && b.size(0) % 2 == 0, "gemm_nt_swiglu_into: w13 [2H, K]");
  const int64_t H = b.size(0) / 2;
  TORCH_CHECK(dph::gemm_nt_supported(dph::kNtSwiglu, a.size(0), H, a.size(1)),
              "gemm_nt_swiglu_into: need rows % 256, H % 8, K % 8");
  TORCH_CHECK(x13_out.scalar_type() == at::kBFloat16 && h_out.scalar_type() == at::kBFloat16 && x13_out.dim() == 2 &&
                  h_out.dim() == 2 && x13_out.size(0) == a.size(0) && x13_out.size(1) == 2 * H &&
                  h_out.size(0) == a.size(0) && h_out.size(1) == H && x13_out.stride(1) == 1 && h_out.stride(1) == 1 &&
                  x13_out.stride(0) % 8 == 0 && h_out.stride(0) % 8 == 0,
              "gemm_nt_swiglu_into: outputs must be bf16 [rows, 2H] / [rows, H] with unit column stride");
  check_align16(x13_out, "x13_out");
  check_align16(h_out, "h_out");
  auto p = nt_params(a, b);
  p.N = (int)H;
  p.H = (int)H;
  p.C = x13_out.data_ptr();
  p.ldc = x13_out.stride(0);
  p.C2 = h_out.data_ptr();
  p.ldc2 = h_out.stride(0);
  dph::gemm_nt(dph::kNtSwiglu, p, cur_stream());
}

// gemm_nt_dswiglu into a caller-owned row block d13_out [rows, 2H]
void gemm_nt_dswiglu_into(const Tensor& dy, const Tensor& w2t, const Tensor& x13, Tensor d13_out) {
  check_cuda(dy, "dy");
  c10::DeviceGuard g(dy.device());
  const Tensor a = rows2d(dy, "gemm_nt_dswiglu_into dy"), b = rows2d(w2t, "gemm_nt_dswiglu_into w2t");
  const Tensor xr = rows2d(x13, "gemm_nt_dswiglu_into x13");
  const int64_t H = b.size(0);
  TORCH_CHECK(w2t.dim() == 2 && b.size(1) == a.size(1) && xr.size(0) == a.size(0) && xr.size(1) == 2 * H,
              "gemm_nt_dswiglu_into: w2t [H, K], x13 [rows, 2H]");
  TORCH_CHECK(dph::gemm_nt_supported(dph::kNtDswiglu, a.size(0), H, a.size(1)),
              "gemm_nt_dswiglu_into: need rows % 256, H % 8, K % 8");
  TORCH_CHECK(d13_out.scalar_type() == at::kBFloat16 && d13_out.dim() == 2 && d13_out.size(0) == a.size(0) &&
                  d13_out.size(1) == 2 * H && d13_out.stride(1) == 1 && d13_out.stride(0) % 8 == 0,
              "gemm_nt_dswiglu_into: d13_out must be bf16 [rows, 2H] with unit column stride");
  check_align16(d13_out, "d13_out");
  auto p = nt_params(a, b);
  p.N = (int)H;
  p.H = (int)H;
  p.C = d13_out.data_ptr();
  p.ldc = d13_out.stride(0);
  p.X = xr.data_ptr();
  p.ldx = xr.stride(0);
  dph::gemm_nt(dph::kNtDswiglu, p, cur_stream());
}

// d13 = SwiGLU-backward(dh = dy W2, x13): dy [..., K], w2t = W2^T [H, K], x13 [..., 2H] -> [..., 2H]
Tensor gemm_nt_dswiglu(const Tensor& dy, const Tensor& w2t, const Tensor& x13) {
  check_cuda(dy, "dy");
  c10::DeviceGuard g(dy.device());
  const Tensor a = rows2d(dy, "gemm_nt_dswiglu dy"), b = rows2d(w2t, "gemm_nt_dswiglu w2t");
  const Tensor xr = rows2d(x13, "gemm_nt_dswiglu x13");
  const int64_t H = b.size(0);
  TORCH_CHECK(w2t.dim() == 2 && b.size(1) == a.size(1) && xr.size(0) == a.size(0) && xr.size(1) == 2 * H,
              "gemm_nt_dswiglu: w2t [H, K], x13 [rows, 2H]");
  TORCH_CHECK(dph::gemm_nt_supported(dph::kNtDswiglu, a.size(0), H, a.size(1)),
              "gemm_nt_dswiglu: need rows % 256, H % 8, K % 8 (got ", a.size(0), ", ", H, ", ", a.size(1), ")");
  Tensor d13 = at::empty(out_sizes(dy, 2 * H), dy.options());
  auto p = nt_params(a, b);
  p.N = (int)H;
  p.H = (int)H;
  p.C = d13.data_ptr();
  p.ldc = 2 * H;
  p.X = xr.data_ptr();
  p.ldx = xr.stride(0);
  dph::gemm_nt(dph::kNtDswiglu, p, cur_stream());
  return d13;
}

// C = x W^T with interleaved RoPE on columns [0, n_rot) (heads of hd), position = row % S + pos_off
Tensor gemm_nt_rope(const Tensor& x, const Tensor& w, const Tensor& cos_t, const Tensor& sin_t, int64_t S,
                    int64_t hd, int64_t n_rot, int64_t pos_off) {
  check_cuda(x, "x");
  c10::DeviceGuard g(x.device());
  const Tensor a = rows2d(x, "gemm_nt_rope x"), b = rows2d(w, "gemm_nt_rope w");
  TORCH_CHECK(w.dim() == 2 && b.size(1) == a.size(1), "gemm_nt_rope: w [N, K]");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(-1) * 2 == hd && hd % 4 == 0,
              "gemm_nt_rope: fp32 contiguous cos / sin tables [positions, hd / 2]");
  TORCH_CHECK(n_rot % hd == 0 && n_rot <= b.size(0) && S > 0 && a.size(0) % S == 0 &&
                  cos_t.size(0) >= S + pos_off, "gemm_nt_rope: bad rotary layout");
  TORCH_CHECK(dph::gemm_nt_supported(dph::kNtRope, a.size(0), b.size(0), a.size(1)),
              "gemm_nt_rope: need rows % 256, N % 8, K % 8");
  Tensor C = at::empty(out_sizes(x, b.size(0)), x.options());
  auto p = nt_params(a, b);
  p.N = (int)b.size(0);
  p.C = C.data_ptr();
  p.ldc = b.size(0);
  p.rope_cos = cos_t.data_ptr<float>();
  p.rope_sin = sin_t.data_ptr<float>();
  p.S = (int)S;
  p.hd = (int)hd;
  p.n_rot = (int)n_rot;
  p.pos_off = (int)pos_off;
  dph::gemm_nt(dph::kNtRope, p, cur_stream());
  return C;
}

TORCH_LIBRARY(dph, m) {
  m.def("rmsnorm_fwd(Tensor x, Tensor w, float eps, Tensor? residual=None) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres=None) -> (Tensor, Tensor)");
  m.def("layernorm_fwd(Tensor x, Tensor w, Tensor b, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("layernorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd) -> (Tensor, Tensor, Tensor)");
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, int pos_offset, bool inverse) -> ()");
  m.def("swiglu_fwd(Tensor x2) -> Tensor");
  m.def("swiglu_bwd(Tensor dy, Tensor x2) -> Tensor");
  m.def("gelu_fwd(Tensor x, bool tanh_form) -> Tensor");
  m.def("gelu_bwd(Tensor dy, Tensor x, bool tanh_form) -> Tensor");
  m.def("adamw_step_(Tensor(a!) master, Tensor(b!) m, Tensor(c!) v, Tensor grad, Tensor(d!)? param_out, float lr, "
        "float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2, Tensor? grad_scale, "
        "Tensor? hyper=None) -> ()");
  m.def("sgd_step_(Tensor(a!) master, Tensor(b!) buf, Tensor grad, Tensor(d!)? param_out, float lr, float momentum, "
        "float dampening, float weight_decay, bool nesterov, bool first_step, Tensor? grad_scale, "
        "Tensor? hyper=None) -> ()");
  m.def("sumsq_(Tensor x, Tensor(a!) out) -> ()");
  m.def("cross_entropy_fwd(Tensor(a!) logits, Tensor target, Tensor inv_count, int ignore_index, bool grad_inplace, "
        "float smoothing) -> (Tensor, Tensor)");
  m.def("flash_attn_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal, float dropout_p=0., int seed=0) "
        "-> (Tensor, Tensor)");
  m.def("flash_attn_fwd_merge_(Tensor q, Tensor k, Tensor v, float scale, bool causal, Tensor(a!) acc_o, "
        "Tensor(b!) acc_lse) -> ()");
  m.def("flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, float scale, bool causal, "
        "float dropout_p=0., int seed=0) -> (Tensor, Tensor, Tensor)");
  m.def("flash_attn_bwd_into(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, float scale, "
        "bool causal, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, float dropout_p=0., int seed=0, "
        "Tensor? rope_cos=None, Tensor? rope_sin=None, int rope_offset=0) -> ()");
  m.def("image_augment(Tensor images, Tensor idx, Tensor? params, Tensor mean, Tensor inv_std, int pad, "
        "bool channels_last, bool bf16_out) -> Tensor");
  m.def("fp8_quantize(Tensor x, int fmt, bool rowmajor, bool transposed) -> (Tensor, Tensor, Tensor)");
  m.def("kv_append_(Tensor(a!) qkv, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor pos, Tensor cos, Tensor sin, "
        "int n_heads, int n_kv_heads, float kv_scale=1.) -> ()");
  m.def("decode_attention(Tensor qkv, Tensor k_cache, Tensor v_cache, Tensor pos, int n_heads, int n_kv_heads, "
        "float scale, int max_len, float kv_scale=1.) -> Tensor");
  m.def("skinny_linear(Tensor x, Tensor w) -> Tensor");
  m.def("gemv_swiglu(Tensor x2, Tensor w) -> Tensor");
  m.def("gemv_rmsnorm(Tensor x, Tensor? res, Tensor norm_weight, float eps, Tensor w) -> (Tensor, Tensor)");
  m.def("embedding_fwd(Tensor ids, Tensor table, int vocab_start) -> Tensor");
  m.def("embedding_bwd(Tensor ids, Tensor dout, int vocab_local, int vocab_start) -> Tensor");
  m.def("gemm_tn_(Tensor(a!) C, Tensor A, Tensor B, bool accumulate) -> ()");
  m.def("gemm_nt(Tensor A, Tensor B) -> Tensor");
  m.def("gemm_nt_swiglu(Tensor x, Tensor w13) -> (Tensor, Tensor)");
  m.def("gemm_nt_swiglu_into(Tensor x, Tensor w13, Tensor(a!) x13_out, Tensor(b!) h_out) -> ()");
  m.def("gemm_nt_dswiglu_into(Tensor dy, Tensor w2t, Tensor x13, Tensor(a!) d13_out) -> ()");
  m.def("gemm_nt_dswiglu(Tensor dy, Tensor w2t, Tensor x13) -> Tensor");
  m.def("gemm_nt_rope(Tensor x, Tensor w, Tensor cos, Tensor sin, int S, int hd, int n_rot, int pos_off) -> Tensor");
  m.def("gemm_tn_tail_(int cus) -> ()", &gemm_tn_tail_);                          // catch-all kernels
  m.def("gemm_tn_plan_info(int M, int N, int K) -> int[]", &gemm_tn_plan_info);
  m.def("ts_gemm_nt(Tensor A, Tensor B, int H=0, int W=0, Tensor? add=None, Tensor? bias=None, Tensor? pro_ss=None) "
        "-> Tensor");
  m.def("ts_gemm_nt_stats(Tensor A, Tensor B, int H=0, int W=0, Tensor? pro_ss=None, Tensor? bias=None) -> (Tensor, Tensor)");
  m.def("ts_gemm_tn_(Tensor(a!) C, Tensor A, Tensor B, bool accumulate, int H=0, int W=0, Tensor? pro_ss=None) -> ()");
  m.def("transpose2d(Tensor x) -> Tensor");
  m.def("pad_cols(Tensor x, int cols) -> Tensor");
  m.def("conv3x3_dgrad_weight(Tensor w) -> Tensor");
  m.def("convg_nt(Tensor A, Tensor B, int[] geo, bool stats=False, bool chunk_taps=False, Tensor? bias=None) -> Tensor[]");
  // the parity classes of one strided input gradient write disjoint rows of one shared dx: an in-place op
  m.def("convg_nt_out_(Tensor A, Tensor B, int[] geo, Tensor(a!) out) -> ()");
  m.def("convg_tn_(Tensor(a!) C, Tensor A, Tensor B, int[] geo, bool accumulate, bool chunk_taps=False) -> ()");
  m.def("ts_gemm_nt_add_sub(Tensor A, Tensor B, Tensor add, int H, int W, int s) -> Tensor");
  m.def("ts_gemm_nt_bnred(Tensor A, Tensor B, int H, int W, Tensor? add, int sub, Tensor x, Tensor mean, "
        "Tensor invstd, Tensor? ss=None, Tensor? bits=None, Tensor? add_mask=None) -> (Tensor, Tensor)");
  m.def("ts_gemm_nt_addmask(Tensor A, Tensor B, Tensor add, Tensor add_mask) -> Tensor");
  m.def("maxpool_s2_fwd(Tensor x, int k) -> (Tensor, Tensor)");
  m.def("channel_sum(Tensor x, ScalarType out_dtype) -> Tensor");
  m.def("channel_sum_into_(Tensor x, Tensor(a!) out) -> ()");
  m.def("maxpool_s2_bwd(Tensor dy, Tensor tap, int H, int W, int k, Tensor? add=None, int add_off=0) -> Tensor");
  m.def("maxpool_s2_bwd_bnred(Tensor dy, Tensor tap, int H, int W, int k, Tensor x, Tensor mean, Tensor invstd, "
        "Tensor ss, Tensor? add=None, int add_off=0) -> (Tensor, Tensor)");
  m.def("upcat_fwd(Tensor y2, Tensor? bias, Tensor skip, int H, int W) -> Tensor");
  m.def("upcat_bwd(Tensor dcat, int H, int W, int Co, bool want_skip=True) -> (Tensor, Tensor)");
  m.def("bn_act_fwd(Tensor x, Tensor? res, Tensor? w, Tensor? b, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
        "float momentum, float eps, bool relu, Tensor? pre_stats=None, Tensor(c!)? num_batches_tracked=None, "
        "Tensor(d!)? relu_mask_out=None, bool apply=True) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("bn_act_apply(Tensor x, Tensor? res, Tensor scale, Tensor shift, bool relu) -> Tensor");
  m.def("bn_act_apply_resbn(Tensor x, Tensor ss, Tensor z, Tensor zss, Tensor(a!) relu_mask) -> Tensor");
  m.def("bn_act_bwd_dual(Tensor dy, Tensor x, Tensor z, Tensor relu_mask, Tensor mean_a, Tensor invstd_a, "
        "Tensor w_a, Tensor mean_b, Tensor invstd_b, Tensor w_b, bool need_a, bool need_b, Tensor(a!)? dw_a_out=None, "
        "Tensor(b!)? db_a_out=None, Tensor(c!)? dw_b_out=None, Tensor(d!)? db_b_out=None, Tensor? pre_part_a=None) "
        "-> Tensor[]");
  m.def("bn_act_bwd(Tensor dy, Tensor y, Tensor x, Tensor mean, Tensor invstd, Tensor? w, bool relu, bool need_dres, "
        "bool need_dwb, Tensor? xmask_ss=None, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None, "
        "Tensor? relu_mask=None, Tensor? pre_part=None) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("latmse_fwd(Tensor pred, Tensor target, int n_global, int lat_offset) -> Tensor");
  m.def("latmse_bwd(Tensor gloss, Tensor pred, Tensor target, int n_global, int lat_offset, bool need_dtarget) -> "
        "(Tensor, Tensor)");
  // custom all-reduce: resource management ops carry no device tensor, so they get catch-all kernels
  m.def("car_create(int rank, int world, int max_bytes, float timeout_s) -> int", &car_create_op);
  m.def("car_ipc_handle(int ctx) -> Tensor", &car_ipc_handle_op);
  m.def("car_open(int ctx, Tensor handles) -> ()", &car_open_op);
  m.def("car_status(int ctx) -> int", &car_status_op);
  m.def("car_agreed(int ctx) -> int", &car_agreed_op);
  m.def("attn_variant(int v) -> int", &attn_variant_op);
  m.def("gemm_nt_variant(int v) -> int", &gemm_nt_variant_op);
  m.def("gemm1_lds(int on) -> int", &gemm1_lds_op);
  m.def("c3w_round(int slots) -> int", &c3w_round_op);
  m.def("car_flag(int ctx, Tensor(a!) flag) -> ()");
  m.def("car_poison(int ctx, Tensor flag, Tensor(a!) gscale) -> ()");
  m.def("car_destroy(int ctx) -> ()", &car_destroy_op);
  m.def("car_allreduce(int ctx, Tensor inp, Tensor(a!) out, int algo, float scale, int max_blocks) -> ()");
}

TORCH_LIBRARY_IMPL(dph, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("layernorm_fwd", &layernorm_fwd);
  m.impl("layernorm_bwd", &layernorm_bwd);
  m.impl("rope_", &rope_);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("gelu_fwd", &gelu_fwd);
  m.impl("gelu_bwd", &gelu_bwd);
  m.impl("adamw_step_", &adamw_step_);
  m.impl("sgd_step_", &sgd_step_);
  m.impl("sumsq_", &sumsq_);
  m.impl("cross_entropy_fwd", &cross_entropy_fwd);
  m.impl("image_augment", &image_augment);
  m.impl("flash_attn_fwd", &flash_attn_fwd);
  m.impl("flash_attn_fwd_merge_", &flash_attn_fwd_merge_);
  m.impl("flash_attn_bwd", &flash_attn_bwd);
  m.impl("flash_attn_bwd_into", &flash_attn_bwd_into);
  m.impl("fp8_quantize", &fp8_quantize);
  m.impl("kv_append_", &kv_append_);
  m.impl("decode_attention", &decode_attention);
  m.impl("skinny_linear", &skinny_linear);
  m.impl("gemv_swiglu", &gemv_swiglu);
  m.impl("gemv_rmsnorm", &gemv_rmsnorm);
  m.impl("embedding_fwd", &embedding_fwd);
  m.impl("embedding_bwd", &embedding_bwd);
  m.impl("gemm_tn_", &gemm_tn_);
  m.impl("gemm_nt", &gemm_nt);
  m.impl("gemm_nt_swiglu", &gemm_nt_swiglu);
  m.impl("gemm_nt_swiglu_into", &gemm_nt_swiglu_into);
  m.impl("gemm_nt_dswiglu_into", &gemm_nt_dswiglu_into);
  m.impl("gemm_nt_dswiglu", &gemm_nt_dswiglu);
  m.impl("gemm_nt_rope", &gemm_nt_rope);
  m.impl("ts_gemm_nt", &ts_gemm_nt);
  m.impl("ts_gemm_nt_stats", &ts_gemm_nt_stats);
  m.impl("ts_gemm_tn_", &ts_gemm_tn_);
  m.impl("transpose2d", &transpose2d);
  m.impl("pad_cols", &pad_cols);
  m.impl("conv3x3_dgrad_weight", &conv3x3_dgrad_weight);
  m.impl("convg_nt", &convg_nt_fresh);
  m.impl("convg_nt_out_", &convg_nt_out_);
  m.impl("convg_tn_", &convg_tn_);
  m.impl("ts_gemm_nt_add_sub", &ts_gemm_nt_add_sub);
  m.impl("ts_gemm_nt_bnred", &ts_gemm_nt_bnred);
  m.impl("ts_gemm_nt_addmask", &ts_gemm_nt_addmask);
  m.impl("maxpool_s2_fwd", &maxpool_s2_fwd);
  m.impl("channel_sum", &channel_sum);
  m.impl("channel_sum_into_", &channel_sum_into_);
  m.impl("maxpool_s2_bwd", &maxpool_s2_bwd);
  m.impl("maxpool_s2_bwd_bnred", &maxpool_s2_bwd_bnred);
  m.impl("upcat_fwd", &upcat_fwd);
  m.impl("upcat_bwd", &upcat_bwd);
  m.impl("bn_act_fwd", &bn_act_fwd);
  m.impl("bn_act_apply", &bn_act_apply);
  m.impl("bn_act_bwd", &bn_act_bwd);
  m.impl("bn_act_bwd_dual", &bn_act_bwd_dual);
  m.impl("bn_act_apply_resbn", &bn_act_apply_resbn);
  m.impl("car_allreduce", &car_allreduce_op);
  m.impl("car_flag", &car_flag_op);
  m.impl("car_poison", &car_poison_op);
  m.impl("latmse_fwd", &latmse_fwd);
  m.impl("latmse_bwd", &latmse_bwd);
}
