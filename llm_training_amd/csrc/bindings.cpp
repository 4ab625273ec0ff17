// Torch operator registrations for the gfx950 kernels (namespace `llmt`, loaded with
// torch.ops.load_library). Every op runs on torch's current HIP stream, validates shapes on the host
// before launching (a mis-shaped launch can fault the GPU), and raises if a launch fails.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

extern "C" {
hipError_t llmt_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* res_out, float* rstd,
                            int T, int H, float eps, hipStream_t stream);
int llmt_rmsnorm_bwd_nblocks(int T, int H);
hipError_t llmt_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dres,
                            void* dx, float* dw_part, void* dw, int dw_is_fp32, int accumulate, int T, int H,
                            hipStream_t stream);
hipError_t llmt_swiglu_fwd(const void* gu, void* c, int64_t T, int I, hipStream_t stream);
hipError_t llmt_swiglu_bwd(const void* gu, const void* dc, void* dgu, int64_t T, int I, hipStream_t stream);
hipError_t llmt_swiglu_bwd_tr(const void* gu, const void* dc, void* dgu, void* dguT, int64_t T, int I,
                              hipStream_t stream);
hipError_t llmt_transpose2d(const void* in, void* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo,
                            hipStream_t stream);
hipError_t llmt_splitk_reduce(const float* slabs, int nsplit, int64_t n, void* out, int out_is_fp32, int accumulate,
                              hipStream_t stream);
hipError_t llmt_rope(void* qkv, const void* pos, int pos_is_64, const float* cos_t, const float* sin_t, int64_t T,
                     int nheads, int D, int64_t stride_t, int stride_h, int inverse, int64_t P, int* err, hipStream_t stream);
hipError_t llmt_cross_entropy(void* logits, int64_t N, int64_t ld, int V, const int64_t* labels,
                              int64_t vocab_start, int64_t ignore_index, const float* lse_in, float* lse_out,
                              float* tgt_out, float* loss_out, const float* coef_row, const float* coef_scalar,
                              int write_grad, int64_t vocab_total, int* err, float* rowsum_out, hipStream_t stream);
hipError_t llmt_adamw(float* p, float* m, float* v, const void* g, int grad_is_fp32, void* pout, int64_t n,
                      float lr, float b1, float b2, float eps, float wd, int64_t step, const float* gscale,
                      hipStream_t stream);
hipError_t llmt_sumsq(const void* x, int is_fp32, int64_t n, float* out, float* ws, hipStream_t stream);
hipError_t llmt_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const int* seg,
                               int B, int S, int Hq, int Hkv, int D, int64_t q_sb, int64_t q_ss, int64_t q_sh,
                               int64_t k_sb, int64_t k_ss, int64_t k_sh, int64_t v_sb, int64_t v_ss, int64_t v_sh,
                               int64_t o_sb, int64_t o_ss, int64_t o_sh, float scale, int causal, int window,
                               int seg_runs, float drop_p, uint32_t drop_seed, const void* rpos, int rpos64,
                               int64_t rp_sb, int64_t rp_ss, const float* rcos, const float* rsin, int64_t rP,
                               void* qrot, hipStream_t stream);
int llmt_flash_attn_fwd_rope_inkernel(int D, float drop_p, int has_seg, int seg_runs);
int llmt_flash_attn_bwd_generic(int D, float drop_p);
int llmt_attn_diag_build();
hipError_t llmt_gemm(const void* x, const void* y, void* c, int x_mn, int y_mn, int out_mode, int M, int N, int K,
                     int64_t ldx, int64_t ldy, int64_t ldc, hipStream_t stream);
hipError_t llmt_gemm_swiglu_bwd(const void* dy, const void* w, const void* gu, void* dgu, void* dgu_t, int M, int N,
                                int K, int64_t ldx, int64_t ldy, hipStream_t stream);
hipError_t llmt_gemm_splitk(const void* x, const void* y, float* slabs, int x_mn, int y_mn, int M, int N, int K,
                            int64_t ldx, int64_t ldy, int64_t ldc, int nsplit, hipStream_t stream);
int64_t llmt_flash_attn_bwd_ws(int B, int S, int Hq, int D);
hipError_t llmt_quant_int8(const void* x, int x_fp32, int8_t* q, float* scale, int64_t n, hipStream_t stream);
hipError_t llmt_dequant_int8(const int8_t* q, const float* scale, void* y, int64_t n, hipStream_t stream);
hipError_t llmt_dequant_sum(const int8_t* q, const float* scale, void* out, int out_fp32, int64_t n, int k,
                            int accumulate, hipStream_t stream);
hipError_t llmt_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                               const float* lse, float* delta, const int* seg, void* dq, void* dk, void* dv,
                               float* work, int B, int S, int Hq, int Hkv, int D, int64_t q_sb, int64_t q_ss,
                               int64_t q_sh, int64_t k_sb, int64_t k_ss, int64_t k_sh, int64_t v_sb, int64_t v_ss,
                               int64_t v_sh, int64_t o_sb, int64_t o_ss, int64_t o_sh, int64_t dq_sb, int64_t dq_ss,
                               int64_t dq_sh, int64_t dk_sb, int64_t dk_ss, int64_t dk_sh, int64_t dv_sb,
                               int64_t dv_ss, int64_t dv_sh, float scale, int causal, int window, int seg_runs,
                               float drop_p, uint32_t drop_seed, const void* rpos, int rpos64, int64_t rp_sb,
                               int64_t rp_ss, const float* rcos, const float* rsin, int64_t rP, void* qrot,
                               hipStream_t stream);
}

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

inline void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "llmt kernel '", what, "' failed: ", hipGetErrorString(e));
}

inline void check_bf16_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}

inline void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
}

// ---------------------------------------------------------------- RMSNorm
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& res,
                                                           const at::Tensor& w, double eps) {
  check_bf16_cuda(x, "x");
  check_bf16_cuda(w, "weight");
  check_rows(x, "x");
  const int64_t H = x.size(-1);
  TORCH_CHECK(w.numel() == H && w.is_contiguous(), "weight shape mismatch");
  TORCH_CHECK(H % 8 == 0 && H <= 8192, "rmsnorm: hidden size must be a multiple of 8 and <= 8192");
  const int64_t T = x.numel() / H;
  auto y = at::empty_like(x);
  auto rstd = at::empty({T}, x.options().dtype(at::kFloat));
  at::Tensor res_out;
  const void* rp = nullptr;
  void* rop = nullptr;
  if (res.has_value() && res->defined()) {
    check_bf16_cuda(*res, "residual");
    check_rows(*res, "residual");
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch");
    res_out = at::empty_like(x);
    rp = res->data_ptr();
    rop = res_out.data_ptr();
  }
  check(llmt_rmsnorm_fwd(x.data_ptr(), rp, w.data_ptr(), y.data_ptr(), rop, rstd.data_ptr<float>(), (int)T, (int)H,
                         (float)eps, cur_stream()),
        "rmsnorm_fwd");
  return {y, res_out.defined() ? res_out : at::Tensor(), rstd};
}

// dw_out: if given (bf16 or fp32, numel H) the weight gradient is written (accumulate=false) or added
// (accumulate=true) into it in place; otherwise a new fp32 tensor is returned.
std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                               const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                                               const c10::optional<at::Tensor>& dw_out, bool accumulate,
                                               bool compute_dw) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(x, "x");
  check_rows(dy, "dy");
  check_rows(x, "x");
  const int64_t H = x.size(-1);
  const int64_t T = x.numel() / H;
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy shape mismatch");
  TORCH_CHECK(rstd.numel() == T && rstd.scalar_type() == at::kFloat, "rstd mismatch");
  auto dx = at::empty_like(x);
  const void* drp = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_bf16_cuda(*dres, "dres");
    check_rows(*dres, "dres");
    TORCH_CHECK(dres->sizes() == x.sizes(), "dres shape mismatch");
    drp = dres->data_ptr();
  }
  at::Tensor dw;
  void* dwp = nullptr;
  int dw_fp32 = 1;
  if (compute_dw) {
    if (dw_out.has_value() && dw_out->defined()) {
      dw = *dw_out;
      TORCH_CHECK(dw.numel() == H && dw.is_contiguous() && dw.is_cuda(), "dw_out mismatch");
      TORCH_CHECK(dw.scalar_type() == at::kFloat || dw.scalar_type() == at::kBFloat16, "dw_out dtype");
      dw_fp32 = dw.scalar_type() == at::kFloat;
    } else {
      dw = at::empty({H}, x.options().dtype(at::kFloat));
      accumulate = false;
    }
    dwp = dw.data_ptr();
  }
  const int nblk = llmt_rmsnorm_bwd_nblocks((int)T, (int)H);
  // the kernels write nblk x H fp32 partials only when a weight gradient is wanted (null otherwise)
  at::Tensor part;
  if (compute_dw) part = at::empty({(int64_t)nblk * H}, x.options().dtype(at::kFloat));
  check(llmt_rmsnorm_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), drp, dx.data_ptr(),
                         compute_dw ? part.data_ptr<float>() : nullptr, dwp, dw_fp32, accumulate ? 1 : 0, (int)T,
                         (int)H, cur_stream()),
        "rmsnorm_bwd");
  return {dx, dw};
}

// ---------------------------------------------------------------- SwiGLU
at::Tensor swiglu_fwd(const at::Tensor& gu) {
  check_bf16_cuda(gu, "gate_up");
  check_rows(gu, "gate_up");
  const int64_t I2 = gu.size(-1);
  TORCH_CHECK(I2 % 16 == 0, "swiglu: intermediate size must be a multiple of 8");
  auto sizes = gu.sizes().vec();
  sizes.back() = I2 / 2;
  auto c = at::empty(sizes, gu.options());
  check(llmt_swiglu_fwd(gu.data_ptr(), c.data_ptr(), gu.numel() / I2, (int)(I2 / 2), cur_stream()), "swiglu_fwd");
  return c;
}

at::Tensor swiglu_bwd(const at::Tensor& gu, const at::Tensor& dc) {
  check_bf16_cuda(gu, "gate_up");
  check_bf16_cuda(dc, "grad");
  check_rows(gu, "gate_up");
  check_rows(dc, "grad");
  const int64_t I2 = gu.size(-1);
  TORCH_CHECK(dc.numel() * 2 == gu.numel() && dc.size(-1) * 2 == I2, "swiglu_bwd shape mismatch");
  auto dgu = at::empty_like(gu);
  check(llmt_swiglu_bwd(gu.data_ptr(), dc.data_ptr(), dgu.data_ptr(), gu.numel() / I2, (int)(I2 / 2), cur_stream()),
        "swiglu_bwd");
  return dgu;
}

// SwiGLU backward that also returns dgu^T [2I, T] (T, I multiples of 64)
std::tuple<at::Tensor, at::Tensor> swiglu_bwd_tr(const at::Tensor& gu, const at::Tensor& dc) {
  check_bf16_cuda(gu, "gate_up");
  check_bf16_cuda(dc, "dc");
  TORCH_CHECK(gu.is_contiguous() && dc.is_contiguous(), "swiglu_bwd_tr: contiguous inputs");
  const int64_t I2 = gu.size(-1), T = gu.numel() / I2;
  TORCH_CHECK(dc.numel() == T * (I2 / 2), "swiglu_bwd_tr: dc must be [T, I]");
  auto dgu = at::empty_like(gu);
  auto dguT = at::empty({I2, T}, gu.options());
  check(llmt_swiglu_bwd_tr(gu.data_ptr(), dc.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), T, (int)(I2 / 2),
                           cur_stream()),
        "swiglu_bwd_tr");
  return {dgu, dguT};
}

// ---------------------------------------------------------------- RoPE (in place)
// qkv: [..., T, nh_total, D] with unit stride on D; rotates the first `nheads` heads.
// out[C, R] = x[R, C]^T for bf16 matrices with R, C multiples of 64 (row-major, unit inner stride)
void transpose_(const at::Tensor& x, at::Tensor out) {
  TORCH_CHECK(x.is_cuda() && out.is_cuda() && x.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
              "transpose_: bf16 GPU tensors");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.stride(1) == 1 && out.stride(1) == 1, "transpose_: 2-D, unit stride");
  TORCH_CHECK(out.size(0) == x.size(1) && out.size(1) == x.size(0), "transpose_: out must be [C, R]");
  check(llmt_transpose2d(x.data_ptr(), out.data_ptr(), x.size(0), x.size(1), x.stride(0), out.stride(0), cur_stream()),
        "transpose2d");
}

// out (+)= slabs.sum(0): split-K partials of a weight gradient (slabs fp32 [nsplit, *out.shape])
void splitk_reduce_(const at::Tensor& slabs, at::Tensor out, bool accumulate) {
  TORCH_CHECK(slabs.is_cuda() && out.is_cuda() && slabs.scalar_type() == at::kFloat && slabs.is_contiguous() &&
                  out.is_contiguous(), "splitk_reduce_: contiguous GPU tensors, fp32 slabs");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "splitk_reduce_: out fp32/bf16");
  TORCH_CHECK(slabs.dim() >= 1 && slabs.numel() == slabs.size(0) * out.numel(), "splitk_reduce_: slabs [k, *out]");
  check(llmt_splitk_reduce(slabs.data_ptr<float>(), (int)slabs.size(0), out.numel(), out.data_ptr(),
                           out.scalar_type() == at::kFloat, accumulate, cur_stream()),
        "splitk_reduce");
}

// ---------------------------------------------------------------- device-side index checks
// Per-device int32 words the kernels set when a data-dependent index is out of range (the kernels clamp or
// skip, so memory stays safe): [0] a RoPE position outside the cos/sin table, [1] a cross-entropy label
// that is neither ignore_index nor a vocabulary id. Read (one host sync) by llm_training_amd.ops.native.
// check_kernel_errors() at the trainer's logging steps.
at::Tensor kernel_errors() {
  static std::mutex mu;
  static std::map<int, at::Tensor> words;
  const int dev = c10::hip::current_device();
  std::lock_guard<std::mutex> lock(mu);
  auto it = words.find(dev);
  if (it == words.end())
    it = words.emplace(dev, at::zeros({4}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, dev))).first;
  return it->second;
}
static int* err_words() { return kernel_errors().data_ptr<int>(); }

// 1 when this library is the diagnostic build (_C_diag.so, -DLLMT_DIAG: wrong-result probes compiled in)
int64_t diag_build() { return llmt_attn_diag_build(); }

void rope_(at::Tensor qkv, const at::Tensor& pos, const at::Tensor& cos_t, const at::Tensor& sin_t, int64_t nheads,
           bool inverse) {
  check_bf16_cuda(qkv, "qkv");
  TORCH_CHECK(qkv.dim() >= 3, "rope: qkv must be [T, H, D]");
  const int64_t D = qkv.size(-1);
  TORCH_CHECK(qkv.stride(-1) == 1, "rope: head dim must be contiguous");
  TORCH_CHECK(D % 16 == 0, "rope: head dim must be a multiple of 16");
  TORCH_CHECK(nheads <= qkv.size(-2), "rope: nheads out of range");
  // flatten all leading dims into T (they must be uniformly strided)
  const int64_t T = qkv.numel() / (qkv.size(-1) * qkv.size(-2));
  const int64_t stride_t = qkv.stride(-3);
  for (int d = 0; d < qkv.dim() - 3; ++d)
    TORCH_CHECK(qkv.stride(d) == qkv.stride(d + 1) * qkv.size(d + 1), "rope: leading dims not flattenable");
  TORCH_CHECK(pos.numel() == T && pos.is_contiguous() && pos.is_cuda(), "rope: positions must be [T] contiguous");
  TORCH_CHECK(pos.scalar_type() == at::kLong || pos.scalar_type() == at::kInt, "rope: positions must be int");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(-1) * 2 == D,
              "rope: cos/sin tables must be fp32 [max_pos, D/2]");
  check(llmt_rope(qkv.data_ptr(), pos.data_ptr(), pos.scalar_type() == at::kLong, cos_t.data_ptr<float>(),
                  sin_t.data_ptr<float>(), T, (int)nheads, (int)D, stride_t, (int)qkv.stride(-2), inverse ? 1 : 0,
                  cos_t.size(0), err_words(), cur_stream()),
        "rope");
}

// ---------------------------------------------------------------- cross entropy
// vocab_total: upper bound of a valid label for the error word (-1: the row width when vocab_start == 0, the
// whole-vocabulary logits of the non-parallel losses; 0: lower bound only, a vocab-parallel shard)
std::tuple<at::Tensor, at::Tensor, at::Tensor> cross_entropy_(at::Tensor logits, const at::Tensor& labels,
                                                             int64_t vocab_start, int64_t ignore_index,
                                                             const c10::optional<at::Tensor>& lse_in,
                                                             const c10::optional<at::Tensor>& coef_row,
                                                             const c10::optional<at::Tensor>& coef_scalar,
                                                             bool write_grad, int64_t vocab_total,
                                                             const c10::optional<at::Tensor>& rowsum) {
  check_bf16_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N, V] with unit column stride");
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(labels.numel() == N && labels.scalar_type() == at::kLong && labels.is_contiguous(), "labels mismatch");
  auto opts = logits.options().dtype(at::kFloat);
  auto lse = at::empty({N}, opts), tgt = at::empty({N}, opts), loss = at::empty({N}, opts);
  auto fptr = [&](const c10::optional<at::Tensor>& t, int64_t n) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == n && t->is_cuda(),
                "cross_entropy: fp32 side input mismatch");
    return t->data_ptr<float>();
  };
  check(llmt_cross_entropy(logits.data_ptr(), N, logits.stride(0), (int)V, labels.data_ptr<int64_t>(), vocab_start,
                           ignore_index, fptr(lse_in, N), lse.data_ptr<float>(), tgt.data_ptr<float>(),
                           loss.data_ptr<float>(), fptr(coef_row, N), fptr(coef_scalar, 1), write_grad ? 1 : 0,
                           vocab_total >= 0 ? vocab_total : (vocab_start == 0 ? V : 0), err_words(),
                           (rowsum.has_value() && rowsum->defined() && !lse_in.has_value())
                               ? const_cast<float*>(fptr(rowsum, N)) : nullptr,
                           cur_stream()),
        "cross_entropy");
  return {lse, tgt, loss};
}

// ---------------------------------------------------------------- optimizer
void adamw_(at::Tensor p, at::Tensor m, at::Tensor v, const at::Tensor& g, const c10::optional<at::Tensor>& pout,
            double lr, double b1, double b2, double eps, double wd, int64_t step,
            const c10::optional<at::Tensor>& gscale) {
  const int64_t n = p.numel();
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw: master/m/v must be fp32");
  TORCH_CHECK(p.is_contiguous() && m.is_contiguous() && v.is_contiguous() && g.is_contiguous(), "adamw: contiguous");
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n, "adamw: size mismatch");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "adamw: grad dtype");
  TORCH_CHECK(n % 4 == 0, "adamw: flat buffers must be padded to a multiple of 4");
  void* po = nullptr;
  if (pout.has_value() && pout->defined()) {
    TORCH_CHECK(pout->numel() == n && pout->scalar_type() == at::kBFloat16 && pout->is_contiguous(), "adamw: pout");
    po = pout->data_ptr();
  }
  const float* gs = nullptr;
  if (gscale.has_value() && gscale->defined()) {
    TORCH_CHECK(gscale->scalar_type() == at::kFloat && gscale->numel() == 1, "adamw: gscale");
    gs = gscale->data_ptr<float>();
  }
  check(llmt_adamw(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr(),
                   g.scalar_type() == at::kFloat, po, n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, step,
                   gs, cur_stream()),
        "adamw");
}

void sumsq_(const at::Tensor& x, at::Tensor out) {
  TORCH_CHECK(x.is_contiguous() && x.numel() % 4 == 0, "sumsq: contiguous, numel % 4 == 0");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "sumsq dtype");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 1, "sumsq out");
  auto ws = at::empty({1024}, out.options());
  check(llmt_sumsq(x.data_ptr(), x.scalar_type() == at::kFloat, x.numel(), out.data_ptr<float>(),
                   ws.data_ptr<float>(), cur_stream()),
        "sumsq");
}

// ---------------------------------------------------------------- int8 blockwise quantisation (ZeRO++)
// one fp32 scale per 64 elements; n must be a multiple of 64
void quant_int8_(const at::Tensor& x, at::Tensor q, at::Tensor scale) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "quant_int8: x must be a contiguous bf16/fp32 GPU tensor");
  const int64_t n = x.numel();
  TORCH_CHECK(n % 64 == 0, "quant_int8: numel % 64");
  TORCH_CHECK(q.scalar_type() == at::kChar && q.numel() == n && q.is_contiguous(), "quant_int8: q");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == n / 64 && scale.is_contiguous(), "quant_int8: scale");
  check(llmt_quant_int8(x.data_ptr(), x.scalar_type() == at::kFloat, (int8_t*)q.data_ptr(), scale.data_ptr<float>(), n,
                        cur_stream()),
        "quant_int8");
}

void dequant_int8_(const at::Tensor& q, const at::Tensor& scale, at::Tensor y) {
  const int64_t n = y.numel();
  TORCH_CHECK(y.is_cuda() && y.is_contiguous() && y.scalar_type() == at::kBFloat16 && n % 64 == 0, "dequant_int8: y");
  TORCH_CHECK(q.scalar_type() == at::kChar && q.numel() == n && q.is_contiguous(), "dequant_int8: q");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == n / 64 && scale.is_contiguous(), "dequant_int8: scale");
  check(llmt_dequant_int8((const int8_t*)q.data_ptr(), scale.data_ptr<float>(), y.data_ptr(), n, cur_stream()),
        "dequant_int8");
}

// out (+)= sum over the k chunks of q [k, n] (scales [k, n/64])
void dequant_sum_(const at::Tensor& q, const at::Tensor& scale, at::Tensor out, int64_t k, bool accumulate) {
  const int64_t n = out.numel();
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && n % 64 == 0 &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "dequant_sum: out");
  TORCH_CHECK(q.scalar_type() == at::kChar && q.numel() == k * n && q.is_contiguous(), "dequant_sum: q");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == k * n / 64 && scale.is_contiguous(),
              "dequant_sum: scale");
  check(llmt_dequant_sum((const int8_t*)q.data_ptr(), scale.data_ptr<float>(), out.data_ptr(),
                         out.scalar_type() == at::kFloat, n, (int)k, accumulate ? 1 : 0, cur_stream()),
        "dequant_sum");
}

// ---------------------------------------------------------------- GEMM
// c (+)= X . Y^T with X = a ([M, K], or [K, M] when a_mn) and Y = b ([N, K], or [K, N] when b_mn);
// bf16 operands, c bf16 or fp32 [M, N] with unit column stride.
inline int64_t row_ld(const at::Tensor& t) {
  // a single row's stride is arbitrary in torch: any multiple of 8 covering the row works
  return t.size(0) > 1 ? t.stride(0) : (t.size(1) + 7) / 8 * 8;
}

void gemm_(const at::Tensor& a, const at::Tensor& b, at::Tensor c, bool a_mn, bool b_mn, bool accumulate) {
  check_bf16_cuda(a, "a");
  check_bf16_cuda(b, "b");
  TORCH_CHECK(c.is_cuda() && (c.scalar_type() == at::kBFloat16 || c.scalar_type() == at::kFloat),
              "gemm: c must be a bf16 or fp32 GPU tensor");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm: operands must be 2-D");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1 && c.stride(1) == 1, "gemm: unit column stride required");
  const int64_t M = a_mn ? a.size(1) : a.size(0), K = a_mn ? a.size(0) : a.size(1);
  const int64_t N = b_mn ? b.size(1) : b.size(0), Kb = b_mn ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "gemm: contraction sizes differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(b_mn || !a_mn, "gemm: an MN-major a needs an MN-major b");
  TORCH_CHECK(c.size(0) == M && c.size(1) == N, "gemm: output must be [", M, ", ", N, "]");
  TORCH_CHECK(K > 0 && K % 32 == 0, "gemm: K must be a positive multiple of 32");
  TORCH_CHECK(N % 4 == 0, "gemm: N must be a multiple of 4");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "gemm: dimension too large");
  const int64_t lda = row_ld(a), ldb = row_ld(b), ldc = c.size(0) > 1 ? c.stride(0) : (N + 3) / 4 * 4;
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "gemm: leading dimensions must be 16-byte multiples");
  TORCH_CHECK(256 * lda * 2 < 0x7fffffffLL && 256 * ldb * 2 < 0x7fffffffLL, "gemm: leading dimension too large");
  for (const at::Tensor* t : {&a, &b, static_cast<const at::Tensor*>(&c)})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "gemm: operands must be 16-byte aligned");
  const int out_mode = c.scalar_type() == at::kFloat ? (accumulate ? 2 : 1) : (accumulate ? 3 : 0);
  if (M == 0 || N == 0) return;
  check(llmt_gemm(a.data_ptr(), b.data_ptr(), c.data_ptr(), a_mn ? 1 : 0, b_mn ? 1 : 0, out_mode, (int)M, (int)N,
                  (int)K, lda, ldb, ldc, cur_stream()),
        "gemm");
}

// Down-projection input gradient with the SwiGLU backward fused into the GEMM epilogue (csrc/gemm.hip
// SwiArgs): dy [M, K] @ w_down [K, N] -> dc (never stored) -> dgu [M, 2N] (and dgu^T [2N, M] when transposed)
// from gu [M, 2N] = [gate | up].
std::vector<at::Tensor> gemm_swiglu_bwd(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& gu, bool transposed) {
  check_bf16_cuda(dy, "dy");
  check_bf16_cuda(w, "w");
  check_bf16_cuda(gu, "gu");
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && gu.dim() == 2, "gemm_swiglu_bwd: 2-D operands");
  TORCH_CHECK(dy.stride(1) == 1 && w.stride(1) == 1 && gu.is_contiguous(), "gemm_swiglu_bwd: layouts");
  const int64_t M = dy.size(0), K = dy.size(1), N = w.size(1);
  TORCH_CHECK(w.size(0) == K && gu.size(0) == M && gu.size(1) == 2 * N, "gemm_swiglu_bwd: shapes");
  TORCH_CHECK(K % 32 == 0 && N % 64 == 0 && M % 64 == 0, "gemm_swiglu_bwd: K % 32, N % 64, M % 64");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 30) && K < (1LL << 31), "gemm_swiglu_bwd: dimension too large");
  const int64_t lda = row_ld(dy), ldb = row_ld(w);
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm_swiglu_bwd: leading dimensions must be 16-byte multiples");
  TORCH_CHECK(256 * lda * 2 < 0x7fffffffLL && 256 * ldb * 2 < 0x7fffffffLL, "gemm_swiglu_bwd: leading dimension too large");
  auto dgu = at::empty_like(gu);
  at::Tensor dgu_t;
  if (transposed) dgu_t = at::empty({2 * N, M}, gu.options());
  for (const at::Tensor* t : {&dy, &w, &gu, static_cast<const at::Tensor*>(&dgu)})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "gemm_swiglu_bwd: 16-byte aligned operands");
  if (M > 0)
    check(llmt_gemm_swiglu_bwd(dy.data_ptr(), w.data_ptr(), gu.data_ptr(), dgu.data_ptr(),
                               transposed ? dgu_t.data_ptr() : nullptr, (int)M, (int)N, (int)K, lda, ldb, cur_stream()),
          "gemm_swiglu_bwd");
  if (transposed) return {dgu, dgu_t};
  return {dgu};
}

// slabs [nsplit, M, N] fp32 (contiguous): slab s = a . b^T over contraction slice s (layouts as gemm_)
void gemm_splitk_(const at::Tensor& a, const at::Tensor& b, at::Tensor slabs, bool a_mn, bool b_mn) {
  check_bf16_cuda(a, "a");
  check_bf16_cuda(b, "b");
  TORCH_CHECK(slabs.is_cuda() && slabs.scalar_type() == at::kFloat && slabs.dim() == 3 && slabs.is_contiguous(),
              "gemm_splitk: slabs must be a contiguous fp32 [nsplit, M, N] GPU tensor");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1, "gemm_splitk: 2-D operands with unit column stride");
  const int64_t M = a_mn ? a.size(1) : a.size(0), K = a_mn ? a.size(0) : a.size(1);
  const int64_t N = b_mn ? b.size(1) : b.size(0), Kb = b_mn ? b.size(0) : b.size(1);
  const int64_t ns = slabs.size(0);
  TORCH_CHECK(K == Kb && (b_mn || !a_mn), "gemm_splitk: contraction sizes / layouts");
  TORCH_CHECK(slabs.size(1) == M && slabs.size(2) == N, "gemm_splitk: slabs must be [nsplit, ", M, ", ", N, "]");
  TORCH_CHECK(ns >= 1 && K % (32 * ns) == 0 && N % 4 == 0, "gemm_splitk: K must be a multiple of 32 * nsplit, N of 4");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "gemm_splitk: dimension too large");
  const int64_t lda = row_ld(a), ldb = row_ld(b);
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm_splitk: leading dimensions must be 16-byte multiples");
  TORCH_CHECK(256 * lda * 2 < 0x7fffffffLL && 256 * ldb * 2 < 0x7fffffffLL, "gemm_splitk: leading dimension too large");
  for (const at::Tensor* t : {&a, &b, static_cast<const at::Tensor*>(&slabs)})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "gemm_splitk: operands must be 16-byte aligned");
  if (M == 0 || N == 0) return;
  check(llmt_gemm_splitk(a.data_ptr(), b.data_ptr(), slabs.data_ptr<float>(), a_mn ? 1 : 0, b_mn ? 1 : 0, (int)M,
                         (int)N, (int)K, lda, ldb, N, (int)ns, cur_stream()),
        "gemm_splitk");
}

// ---------------------------------------------------------------- flash attention
// q: [B, S, Hq, D], k/v: [B, S, Hkv, D] (any batch/seq/head strides, unit stride on D).
// seg: optional int32 segment ids (0 = padding): attention is restricted to the token's contiguous run of
// equal ids. [B, S] = ids only (every tile compares ids); [3, B, S] = ids, run start, run end per token:
// key tiles outside a query block's runs are skipped and tiles inside one run take the unmasked path;
// ops/fused.py segment_info appends the work orders of the query and key blocks (heaviest first).
static int seg_layout(const c10::optional<at::Tensor>& seg, int64_t B, int64_t S, const int** sp) {
  *sp = nullptr;
  if (!seg.has_value() || !seg->defined()) return 0;
  TORCH_CHECK(seg->scalar_type() == at::kInt && seg->is_contiguous() && seg->is_cuda(), "flash_attn: seg must be "
              "contiguous int32 on the GPU");
  const int64_t nord = 2 * B * ((S + 127) / 128);  // query- and key-block work orders (segment_info)
  TORCH_CHECK(seg->numel() == B * S || seg->numel() == 3 * B * S || seg->numel() == 3 * B * S + nord,
              "flash_attn: seg must be [B, S], [3, B, S] or segment_info's [3 B S + 2 B ceil(S / 128)]");
  *sp = seg->data_ptr<int>();
  return seg->numel() == 3 * B * S + nord ? 2 : seg->numel() == 3 * B * S ? 1 : 0;
}
// fused RoPE operands of the attention ops: positions of token (b, s) at pos[b * sb + s * ss] (int32 / int64),
// fp32 half-width tables [P, D/2] (the standalone rope_'s contract)
struct RopeIn {
  const void* pos = nullptr;
  int pos64 = 0;
  const float* cos = nullptr;
  const float* sin = nullptr;
  int64_t P = 0, sb = 0, ss = 0;
};
RopeIn rope_in(const c10::optional<at::Tensor>& pos, const c10::optional<at::Tensor>& cos_t,
               const c10::optional<at::Tensor>& sin_t, int64_t sb, int64_t ss, int64_t B, int64_t S, int64_t D) {
  RopeIn r;
  if (!cos_t.has_value()) {
    TORCH_CHECK(!pos.has_value() && !sin_t.has_value(), "flash_attn rope: cos / sin tables required");
    return r;
  }
  TORCH_CHECK(sin_t.has_value(), "flash_attn rope: cos / sin tables required");
  TORCH_CHECK(cos_t->scalar_type() == at::kFloat && sin_t->scalar_type() == at::kFloat && cos_t->is_contiguous() &&
                  sin_t->is_contiguous() && cos_t->dim() == 2 && cos_t->size(1) * 2 == D && sin_t->sizes() == cos_t->sizes() &&
                  cos_t->is_cuda() && sin_t->is_cuda(),
              "flash_attn rope: cos/sin tables must be fp32 [rows, D/2] on the GPU");
  TORCH_CHECK(sb >= 0 && ss >= 0, "flash_attn rope: row strides");
  if (pos.has_value()) {  // position ids index the tables
    TORCH_CHECK(pos->is_cuda() && pos->is_contiguous() &&
                    (pos->scalar_type() == at::kLong || pos->scalar_type() == at::kInt),
                "flash_attn rope: positions must be contiguous int32 / int64 on the GPU");
    TORCH_CHECK((B - 1) * sb + (S - 1) * ss < pos->numel(), "flash_attn rope: position strides");
    r.pos = pos->data_ptr();
    r.pos64 = pos->scalar_type() == at::kLong;
  } else {  // per-token tables: row b * sb + s * ss is token (b, s)'s own
    TORCH_CHECK((B - 1) * sb + (S - 1) * ss < cos_t->size(0), "flash_attn rope: token-table strides");
  }
  r.cos = cos_t->data_ptr<float>();
  r.sin = sin_t->data_ptr<float>();
  r.P = cos_t->size(0);
  r.sb = sb;
  r.ss = ss;
  return r;
}

std::tuple<at::Tensor, at::Tensor> flash_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                  const c10::optional<at::Tensor>& seg, double scale, bool causal,
                                                  int64_t window, double dropout_p, int64_t seed,
                                                  const c10::optional<at::Tensor>& rope_pos,
                                                  const c10::optional<at::Tensor>& rope_cos,
                                                  const c10::optional<at::Tensor>& rope_sin, int64_t rope_sb,
                                                  int64_t rope_ss) {
  check_bf16_cuda(q, "q");
  check_bf16_cuda(k, "k");
  check_bf16_cuda(v, "v");
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "flash_attn: q/k/v must be [B, S, H, D]");
  const int64_t B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && k.size(1) == S && k.size(3) == D && v.sizes() == k.sizes(), "flash_attn: k/v shape");
  TORCH_CHECK(Hq % Hkv == 0, "flash_attn: Hq must be a multiple of Hkv");
  TORCH_CHECK(D == 64 || D == 96 || D == 128, "flash_attn: head dim must be 64, 96 or 128");
  TORCH_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1, "flash_attn: unit stride on head dim");
  // O keeps q's batch/sequence memory order (seq-major activations stay seq-major: no copies)
  auto o = (q.stride(0) >= q.stride(1)) ? at::empty({B, S, Hq, D}, q.options())
                                        : at::empty({S, B, Hq, D}, q.options()).transpose(0, 1);
  auto lse = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  const int* sp = nullptr;
  const int runs = seg_layout(seg, B, S, &sp);
  // fused RoPE: q arrives unrotated and is never written; kernels without the in-kernel rotation read a
  // rotated copy (qrot)
  const RopeIn rp = rope_in(rope_pos, rope_cos, rope_sin, rope_sb, rope_ss, B, S, D);
  at::Tensor qrot;
  if (rp.cos && !llmt_flash_attn_fwd_rope_inkernel((int)D, (float)dropout_p, sp != nullptr, runs))
    qrot = at::empty({B, S, Hq, D}, q.options());
  check(llmt_flash_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), sp, (int)B,
                            (int)S, (int)Hq, (int)Hkv, (int)D, q.stride(0), q.stride(1), q.stride(2), k.stride(0),
                            k.stride(1), k.stride(2), v.stride(0), v.stride(1), v.stride(2), o.stride(0), o.stride(1),
                            o.stride(2), (float)scale, causal ? 1 : 0, (int)window, runs, (float)dropout_p,
                            (uint32_t)seed, rp.pos, rp.pos64, rp.sb, rp.ss, rp.cos, rp.sin, rp.P,
                            qrot.defined() ? qrot.data_ptr() : nullptr, cur_stream()),
        "flash_attn_fwd");
  return {o, lse};
}

// dq/dk/dv are written into caller-provided tensors (so they can be views of one fused dQKV buffer).
void flash_attn_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
                    const at::Tensor& dout, const at::Tensor& lse, const c10::optional<at::Tensor>& seg, at::Tensor dq,
                    at::Tensor dk, at::Tensor dv, double scale, bool causal, int64_t window, double dropout_p,
                    int64_t seed, const c10::optional<at::Tensor>& rope_pos, const c10::optional<at::Tensor>& rope_cos,
                    const c10::optional<at::Tensor>& rope_sin, int64_t rope_sb, int64_t rope_ss,
                    bool rope_q_rotated) {
  const int64_t B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(2);
  check_bf16_cuda(dout, "dout");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes(), "flash_attn_bwd: o/dout shape");
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "flash_attn_bwd: grads");
  TORCH_CHECK(dout.stride(3) == 1 && o.stride(3) == 1 && dq.stride(3) == 1 && dk.stride(3) == 1 && dv.stride(3) == 1,
              "flash_attn_bwd: unit stride on head dim");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == B * Hq * S, "flash_attn_bwd: lse");
  const int* sp = nullptr;
  const int runs = seg_layout(seg, B, S, &sp);
  auto delta = at::empty({llmt_flash_attn_bwd_ws((int)B, (int)S, (int)Hq, (int)D)}, q.options().dtype(at::kFloat));
  TORCH_CHECK(dout.strides() == o.strides(), "flash_attn_bwd: dout must share O's layout");
  at::Tensor work;  // fp32 per-q-head dK/dV partials, only needed for GQA
  // only the generic kernels (dropout, LLMT_FA_GENERIC=1) reduce GQA through partials
  if (Hq != Hkv && llmt_flash_attn_bwd_generic((int)D, (float)dropout_p))
    work = at::empty({2, B, S, Hq, D}, q.options().dtype(at::kFloat));
  // fused RoPE: dq / dk come back for the unrotated q / k. q holds the UNROTATED queries (k rotated) unless
  // rope_q_rotated (both rotated in memory: only the inverse rotation of the gradients is fused); qrot
  // receives the rotated queries the dK/dV pass stages through LDS.
  const RopeIn rp = rope_in(rope_pos, rope_cos, rope_sin, rope_sb, rope_ss, B, S, D);
  at::Tensor qrot;
  if (rp.cos && !rope_q_rotated) qrot = at::empty({B, S, Hq, D}, q.options());
  check(llmt_flash_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                            lse.data_ptr<float>(), delta.data_ptr<float>(), sp, dq.data_ptr(), dk.data_ptr(),
                            dv.data_ptr(), work.defined() ? work.data_ptr<float>() : nullptr, (int)B, (int)S, (int)Hq, (int)Hkv, (int)D,
                            q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2), v.stride(0),
                            v.stride(1), v.stride(2), dout.stride(0), dout.stride(1), dout.stride(2), dq.stride(0),
                            dq.stride(1), dq.stride(2), dk.stride(0), dk.stride(1), dk.stride(2), dv.stride(0),
                            dv.stride(1), dv.stride(2), (float)scale, causal ? 1 : 0, (int)window, runs,
                            (float)dropout_p, (uint32_t)seed, rp.pos, rp.pos64, rp.sb, rp.ss, rp.cos, rp.sin, rp.P,
                            qrot.defined() ? qrot.data_ptr() : nullptr, cur_stream()),
        "flash_attn_bwd");
}

}  // namespace

TORCH_LIBRARY(llmt, m) {
  m.def("rmsnorm_fwd(Tensor x, Tensor? res, Tensor w, float eps) -> (Tensor, Tensor, Tensor)");
  m.def(
      "rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres, Tensor(a!)? dw_out, bool accumulate, "
      "bool compute_dw) -> (Tensor, Tensor)");
  m.def("swiglu_fwd(Tensor gu) -> Tensor");
  m.def("swiglu_bwd(Tensor gu, Tensor dc) -> Tensor");
  m.def("transpose_(Tensor x, Tensor(a!) out) -> ()");
  m.def("splitk_reduce_(Tensor slabs, Tensor(a!) out, bool accumulate) -> ()");
  m.def("swiglu_bwd_tr(Tensor gu, Tensor dc) -> (Tensor, Tensor)");
  m.def("rope_(Tensor(a!) qkv, Tensor pos, Tensor cos, Tensor sin, int nheads, bool inverse) -> ()");
  m.def(
      "cross_entropy_(Tensor(a!) logits, Tensor labels, int vocab_start, int ignore_index, Tensor? lse_in, "
      "Tensor? coef_row, Tensor? coef_scalar, bool write_grad, int vocab_total=-1, Tensor(b!)? rowsum=None) -> "
      "(Tensor, Tensor, Tensor)");
  m.def("kernel_errors() -> Tensor", &kernel_errors);
  m.def("diag_build() -> int", &diag_build);
  m.def(
      "adamw_(Tensor(a!) p, Tensor(b!) m, Tensor(c!) v, Tensor g, Tensor(d!)? pout, float lr, float b1, float b2, "
      "float eps, float wd, int step, Tensor? gscale) -> ()");
  m.def("sumsq_(Tensor x, Tensor(a!) out) -> ()");
  m.def("quant_int8_(Tensor x, Tensor(a!) q, Tensor(b!) scale) -> ()");
  m.def("dequant_int8_(Tensor q, Tensor scale, Tensor(a!) y) -> ()");
  m.def("dequant_sum_(Tensor q, Tensor scale, Tensor(a!) out, int k, bool accumulate) -> ()");
  m.def("gemm_(Tensor a, Tensor b, Tensor(a!) c, bool a_mn, bool b_mn, bool accumulate) -> ()");
  m.def("gemm_splitk_(Tensor a, Tensor b, Tensor(a!) slabs, bool a_mn, bool b_mn) -> ()");
  m.def("gemm_swiglu_bwd(Tensor dy, Tensor w, Tensor gu, bool transposed) -> Tensor[]");
  m.def(
      "flash_attn_fwd(Tensor q, Tensor k, Tensor v, Tensor? seg, float scale, bool causal, int window, "
      "float dropout_p=0., int seed=0, Tensor? rope_pos=None, Tensor? rope_cos=None, Tensor? rope_sin=None, "
      "int rope_sb=0, int rope_ss=0) -> (Tensor, Tensor)");
  m.def(
      "flash_attn_bwd(Tensor q, Tensor k, Tensor v, Tensor o, Tensor dout, Tensor lse, Tensor? seg, Tensor(a!) dq, "
      "Tensor(b!) dk, Tensor(c!) dv, float scale, bool causal, int window, float dropout_p=0., int seed=0, "
      "Tensor? rope_pos=None, Tensor? rope_cos=None, Tensor? rope_sin=None, int rope_sb=0, int rope_ss=0, "
      "bool rope_q_rotated=False) -> ()");
}

TORCH_LIBRARY_IMPL(llmt, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("transpose_", &transpose_);
  m.impl("splitk_reduce_", &splitk_reduce_);
  m.impl("swiglu_bwd_tr", &swiglu_bwd_tr);
  m.impl("rope_", &rope_);
  m.impl("cross_entropy_", &cross_entropy_);
  m.impl("adamw_", &adamw_);
  m.impl("sumsq_", &sumsq_);
  m.impl("quant_int8_", &quant_int8_);
  m.impl("dequant_int8_", &dequant_int8_);
  m.impl("dequant_sum_", &dequant_sum_);
  m.impl("gemm_", &gemm_);
  m.impl("gemm_splitk_", &gemm_splitk_);
  m.impl("gemm_swiglu_bwd", &gemm_swiglu_bwd);
  m.impl("flash_attn_fwd", &flash_attn_fwd);
  m.impl("flash_attn_bwd", &flash_attn_bwd);
}
