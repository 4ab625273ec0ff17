// Host-side (C++) sequence packing for the data pipeline, registered as CPU torch ops.
//
// Replaces the reference's pure-Python O(n * bins) best-fit scan
// (src/llm_training/data/pre_training/pre_training_datamodule.py:156-179) and the instruction-tuning
// group-by-length grouping (data/instruction_tuning/instruction_tuning_datamodule.py:102-145) with
// O(n log n) C++ implementations that return exactly the same assignment:
//  * best-fit decreasing: items in stable descending-length order; each goes to the open bin with the
//    least remaining space that still fits it (ties -> lowest bin index), else a new bin;
//  * group-by-length: items in stable ascending-length order, greedily appended while
//    sum(lengths) + (#items in group) + length <= max_length.
#include <ATen/ATen.h>
#include <torch/library.h>

#include <algorithm>
#include <numeric>
#include <set>
#include <utility>
#include <vector>

namespace {

at::Tensor bfd_pack(const at::Tensor& lengths_in, int64_t capacity) {
  auto lengths = lengths_in.to(at::kLong).contiguous();
  const int64_t n = lengths.numel();
  const int64_t* len = lengths.data_ptr<int64_t>();
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return len[a] > len[b]; });
  // (remaining space, bin index): lower_bound({L, -1}) = least remaining >= L, lowest index on ties
  std::set<std::pair<int64_t, int64_t>> open;
  std::vector<int64_t> remaining;
  auto out = at::empty({n}, at::kLong);
  int64_t* bin = out.data_ptr<int64_t>();
  for (int64_t i : order) {
    const int64_t L = len[i];
    auto it = open.lower_bound({L, -1});
    if (it != open.end()) {
      const int64_t b = it->second;
      open.erase(it);
      remaining[b] -= L;
      open.insert({remaining[b], b});
      bin[i] = b;
    } else {
      const int64_t b = (int64_t)remaining.size();
      remaining.push_back(capacity - L);
      open.insert({capacity - L, b});
      bin[i] = b;
    }
  }
  return out;
}

at::Tensor group_by_length(const at::Tensor& lengths_in, int64_t max_length) {
  auto lengths = lengths_in.to(at::kLong).contiguous();
  const int64_t n = lengths.numel();
  const int64_t* len = lengths.data_ptr<int64_t>();
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return len[a] < len[b]; });
  auto out = at::empty({n}, at::kLong);
  int64_t* grp = out.data_ptr<int64_t>();
  int64_t g = 0, sum = 0, cnt = 0;
  for (int64_t i : order) {
    const int64_t L = len[i];
    if (cnt == 0 || sum + L + cnt <= max_length) {
      sum += L;
      ++cnt;
    } else {
      ++g;
      sum = L;
      cnt = 1;
    }
    grp[i] = g;
  }
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
