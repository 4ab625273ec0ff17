// Host-side AdamW for optimizer-state offload (DeepSpeed `offload_optimizer`, FSDP2 `offload_policy`;
// reference knobs: src/llm_training/lightning/strategy/deepspeed/deepspeed_strategy.py:22-27,94-102 and
// lightning/strategy/fsdp2/fsdp2_strategy.py:58). The reference forwards these to DeepSpeed's CPU-Adam;
// here the engine keeps the fp32 master / exp_avg / exp_avg_sq shards in pinned host memory, streams the
// bf16 gradient shard down, runs this kernel and streams the bf16 parameter shard back up.
//
// One pass per element: read g (bf16 or fp32) + p/m/v (fp32), write p/m/v and the bf16 copy of p.
// Same math as the GPU kernel (csrc/optim.hip adamw_kernel): decoupled weight decay, bias-corrected
// step, gradient pre-scaled by the clip/accumulation factor. Split over at::get_num_threads() std::threads
// in contiguous ranges (ATen's header-inline parallel_for is OpenMP pragmas, which an extension built
// without -fopenmp runs on one thread); the inner loop is branch-free so the compiler vectorises it.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

template <typename F>
void parallel_ranges(int64_t n, int64_t grain, F&& f) {
  const int64_t want = std::max<int64_t>(1, std::min<int64_t>(at::get_num_threads(), (n + grain - 1) / grain));
  if (want == 1) {
    f(0, n);
    return;
  }
  const int64_t chunk = (n + want - 1) / want;
  std::vector<std::thread> pool;
  pool.reserve(want - 1);
  for (int64_t t = 1; t < want; ++t) {
    const int64_t b = t * chunk, e = std::min(n, b + chunk);
    if (b < e) pool.emplace_back([&f, b, e] { f(b, e); });
  }
  f(0, std::min(n, chunk));
  for (auto& th : pool) th.join();
}

inline float bf16_to_f32(uint16_t h) {
  uint32_t u = static_cast<uint32_t>(h) << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f32_to_bf16(float f) {  // round to nearest even; NaN stays NaN
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <bool kOut, typename LoadG>
void adamw_span(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v, LoadG load_g,
                uint16_t* __restrict__ pout, int64_t b, int64_t e, float lr, float b1, float b2, float eps, float wd,
                float step_size, float inv_sqrt_bc2, float sc) {
  const float decay = 1.f - lr * wd;
  for (int64_t i = b; i < e; ++i) {
    const float g = load_g(i) * sc;
    const float mi = b1 * m[i] + (1.f - b1) * g;
    const float vi = b2 * v[i] + (1.f - b2) * g * g;
    const float pi = p[i] * decay - step_size * mi / (std::sqrt(vi) * inv_sqrt_bc2 + eps);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
  // separate pass: the NaN-preserving rounding would keep the update loop from vectorising
  if constexpr (kOut)
    for (int64_t i = b; i < e; ++i) pout[i] = f32_to_bf16(p[i]);
}

template <typename LoadG>
void adamw_range(float* p, float* m, float* v, LoadG load_g, uint16_t* pout, int64_t b, int64_t e, float lr, float b1,
                 float b2, float eps, float wd, float step_size, float inv_sqrt_bc2, float sc) {
  if (pout)
    adamw_span<true>(p, m, v, load_g, pout, b, e, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, sc);
  else
    adamw_span<false>(p, m, v, load_g, pout, b, e, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, sc);
}

void adamw_cpu_(at::Tensor p, at::Tensor m, at::Tensor v, const at::Tensor& g, const c10::optional<at::Tensor>& pout,
                double lr, double b1, double b2, double eps, double wd, int64_t step, double gscale) {
  TORCH_CHECK(p.device().is_cpu() && m.device().is_cpu() && v.device().is_cpu() && g.device().is_cpu(),
              "adamw_cpu_: all operands must be host tensors");
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw_cpu_: p, exp_avg, exp_avg_sq must be fp32");
  TORCH_CHECK(p.is_contiguous() && m.is_contiguous() && v.is_contiguous() && g.is_contiguous(),
              "adamw_cpu_: operands must be contiguous");
  const int64_t n = p.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n, "adamw_cpu_: size mismatch");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat, "adamw_cpu_: grad must be bf16/fp32");
  uint16_t* po = nullptr;
  if (pout.has_value() && pout->defined()) {
    TORCH_CHECK(pout->device().is_cpu() && pout->scalar_type() == at::kBFloat16 && pout->is_contiguous() &&
                    pout->numel() == n,
                "adamw_cpu_: pout must be a contiguous host bf16 tensor of the same size");
    po = reinterpret_cast<uint16_t*>(pout->data_ptr());
  }
  TORCH_CHECK(step >= 1, "adamw_cpu_: step counts from 1");
  const float fb1 = static_cast<float>(b1), fb2 = static_cast<float>(b2);
  const double bc1 = 1.0 - std::pow(b1, static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(b2, static_cast<double>(step));
  const float step_size = static_cast<float>(lr / bc1);
  const float inv_sqrt_bc2 = static_cast<float>(1.0 / std::sqrt(bc2));
  float* pp = p.data_ptr<float>();
  float* mm = m.data_ptr<float>();
  float* vv = v.data_ptr<float>();
  const float sc = static_cast<float>(gscale);
  constexpr int64_t kGrain = 1 << 16;  // below 64K elements per thread the spawn cost dominates
  if (g.scalar_type() == at::kBFloat16) {
    const uint16_t* gg = reinterpret_cast<const uint16_t*>(g.data_ptr());
    parallel_ranges(n, kGrain, [&](int64_t b, int64_t e) {
      adamw_range(pp, mm, vv, [gg](int64_t i) { return bf16_to_f32(gg[i]); }, po, b, e, static_cast<float>(lr), fb1,
                 fb2, static_cast<float>(eps), static_cast<float>(wd), step_size, inv_sqrt_bc2, sc);
    });
  } else {
    const float* gg = g.data_ptr<float>();
    parallel_ranges(n, kGrain, [&](int64_t b, int64_t e) {
      adamw_range(pp, mm, vv, [gg](int64_t i) { return gg[i]; }, po, b, e, static_cast<float>(lr), fb1, fb2,
                 static_cast<float>(eps), static_cast<float>(wd), step_size, inv_sqrt_bc2, sc);
    });
  }
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(llmt, m) {
  m.def(
      "adamw_cpu_(Tensor(a!) p, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor g, Tensor(d!)? pout, float lr, "
      "float b1, float b2, float eps, float wd, int step, float gscale) -> ()");
}

TORCH_LIBRARY_IMPL(llmt, CPU, m) { m.impl("adamw_cpu_", &adamw_cpu_); }
