// Host-side AdamW for optimizer-state offload (DeepSpeed `offload_optimizer`, FSDP2 `offload_policy`;
// reference knobs: src/llm_training/lightning/strategy/deepspeed/deepspeed_strategy.py:22-27,94-102 and
// lightning/strategy/fsdp2/fsdp2_strategy.py:58). The reference forwards these to DeepSpeed's CPU-Adam;
// here the engine keeps the fp32 master / exp_avg / exp_avg_sq shards in pinned host memory, streams the
// bf16 gradient shard down, runs this kernel and streams the bf16 parameter shard back up.
//
// The element loop lives in cpu_adam_core.h (plain C++, also built under ASan / UBSan / TSan by the host
// sanitizer test); it is split over at::get_num_threads() std::threads (ATen's header-inline parallel_for
// is OpenMP pragmas, which an extension built without -fopenmp runs on one thread).
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include "cpu_adam_core.h"

namespace {

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
  const bool bf = g.scalar_type() == at::kBFloat16;
  llmt::adamw_host(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                   bf ? reinterpret_cast<const uint16_t*>(g.data_ptr()) : nullptr, bf ? nullptr : g.data_ptr<float>(),
                   po, n, lr, b1, b2, eps, wd, step, gscale, at::get_num_threads());
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(llmt, m) {
  m.def(
      "adamw_cpu_(Tensor(a!) p, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor g, Tensor(d!)? pout, float lr, "
      "float b1, float b2, float eps, float wd, int step, float gscale) -> ()");
}

TORCH_LIBRARY_IMPL(llmt, CPU, m) { m.impl("adamw_cpu_", &adamw_cpu_); }
