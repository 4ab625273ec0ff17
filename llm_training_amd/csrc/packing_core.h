// Sequence-packing assignments in plain C++ (no ATen): shared by the torch ops in packing.cpp and the
// host sanitizer harness (tests/native/host_sanitize.cpp).
//  * best-fit decreasing: items in stable descending-length order; each goes to the open bin with the
//    least remaining space that still fits it (ties -> lowest bin index), else a new bin;
//  * group-by-length: items in stable ascending-length order, greedily appended while
//    sum(lengths) + (#items in group) + length <= max_length.
#pragma once

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <set>
#include <utility>
#include <vector>

namespace llmt {

// bin[i] = bin of item i (n items of lengths len[0..n))
inline void bfd_assign(const int64_t* len, int64_t n, int64_t capacity, int64_t* bin) {
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return len[a] > len[b]; });
  // (remaining space, bin index): lower_bound({L, -1}) = least remaining >= L, lowest index on ties
  std::set<std::pair<int64_t, int64_t>> open;
  std::vector<int64_t> remaining;
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
}

// grp[i] = group of item i
inline void group_by_length_assign(const int64_t* len, int64_t n, int64_t max_length, int64_t* grp) {
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return len[a] < len[b]; });
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
}

}  // namespace llmt
