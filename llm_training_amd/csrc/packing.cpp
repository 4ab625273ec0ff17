// Host-side (C++) sequence packing for the data pipeline, registered as CPU torch ops.
//
// Replaces the reference's pure-Python O(n * bins) best-fit scan
// (src/llm_training/data/pre_training/pre_training_datamodule.py:156-179) and the instruction-tuning
// group-by-length grouping (data/instruction_tuning/instruction_tuning_datamodule.py:102-145) with
// O(n log n) C++ implementations that return exactly the same assignment (packing_core.h).
#include <ATen/ATen.h>
#include <torch/library.h>

#include "packing_core.h"

namespace {

at::Tensor bfd_pack(const at::Tensor& lengths_in, int64_t capacity) {
  auto lengths = lengths_in.to(at::kLong).contiguous();
  auto out = at::empty({lengths.numel()}, at::kLong);
  llmt::bfd_assign(lengths.data_ptr<int64_t>(), lengths.numel(), capacity, out.data_ptr<int64_t>());
  return out;
}

at::Tensor group_by_length(const at::Tensor& lengths_in, int64_t max_length) {
  auto lengths = lengths_in.to(at::kLong).contiguous();
  auto out = at::empty({lengths.numel()}, at::kLong);
  llmt::group_by_length_assign(lengths.data_ptr<int64_t>(), lengths.numel(), max_length, out.data_ptr<int64_t>());
  return out;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(llmt, m) {
  m.def("bfd_pack(Tensor lengths, int capacity) -> Tensor");
  m.def("group_by_length(Tensor lengths, int max_length) -> Tensor");
}

TORCH_LIBRARY_IMPL(llmt, CPU, m) {
  m.impl("bfd_pack", &bfd_pack);
  m.impl("group_by_length", &group_by_length);
}
