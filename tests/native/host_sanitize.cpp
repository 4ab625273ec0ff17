// Host sanitizer harness for the framework's native host code: the packing assignments
// (csrc/packing_core.h) and the threaded host AdamW (csrc/cpu_adam_core.h), built without ATen under
// AddressSanitizer + UndefinedBehaviorSanitizer, and ThreadSanitizer for the threaded optimizer
// (tests/test_host_sanitizers.py compiles and runs it). Each check compares against a naive reference;
// any sanitizer report or mismatch exits non-zero.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "cpu_adam_core.h"
#include "packing_core.h"

static int failures = 0;
#define CHECK(cond, ...)                  \
  do {                                    \
    if (!(cond)) {                        \
      std::fprintf(stderr, __VA_ARGS__);  \
      std::fprintf(stderr, "\n");         \
      ++failures;                         \
    }                                     \
  } while (0)

// the reference's O(n * bins) best fit over lengths already sorted descending (stable)
static std::vector<int64_t> naive_bfd(const std::vector<int64_t>& len, int64_t cap) {
  std::vector<int64_t> order(len.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int64_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return len[a] > len[b]; });
  std::vector<int64_t> bins, out(len.size());
  for (int64_t i : order) {
    int64_t best = -1, space = INT64_MAX;
    for (size_t j = 0; j < bins.size(); ++j)
      if (bins[j] >= len[i] && bins[j] - len[i] < space) best = (int64_t)j, space = bins[j] - len[i];
    if (best >= 0) {
      bins[best] -= len[i];
      out[i] = best;
    } else {
      bins.push_back(cap - len[i]);
      out[i] = (int64_t)bins.size() - 1;
    }
  }
  return out;
}

static void check_packing(std::mt19937_64& rng) {
  for (int trial = 0; trial < 200; ++trial) {
    const int64_t cap = 16 + (int64_t)(rng() % 512);
    const int64_t n = (int64_t)(rng() % 300);
    std::vector<int64_t> len(n), bin(n, -7), grp(n, -7);
    for (auto& x : len) x = 1 + (int64_t)(rng() % cap);
    llmt::bfd_assign(len.data(), n, cap, bin.data());
    CHECK(bin == naive_bfd(len, cap), "bfd mismatch (trial %d, n %lld)", trial, (long long)n);
    std::vector<int64_t> used;
    for (int64_t i = 0; i < n; ++i) {
      if (bin[i] >= (int64_t)used.size()) used.resize(bin[i] + 1, 0);
      used[bin[i]] += len[i];
    }
    for (int64_t u : used) CHECK(u <= cap, "bin over capacity");
    llmt::group_by_length_assign(len.data(), n, cap, grp.data());
    std::vector<int64_t> sum, cnt;
    for (int64_t i = 0; i < n; ++i) {
      if (grp[i] >= (int64_t)sum.size()) sum.resize(grp[i] + 1, 0), cnt.resize(grp[i] + 1, 0);
      sum[grp[i]] += len[i];
      cnt[grp[i]] += 1;
    }
    for (size_t g = 0; g < sum.size(); ++g)
      CHECK(cnt[g] == 1 || sum[g] + cnt[g] - 1 <= cap, "group %zu over max_length", g);
  }
}

static void check_adamw(std::mt19937_64& rng, int64_t nthreads) {
  std::normal_distribution<float> nd(0.f, 1.f);
  for (int64_t n : {int64_t(1), int64_t(1000), int64_t(3 << 16) + 17}) {
    for (int use_bf16 = 0; use_bf16 < 2; ++use_bf16) {
      std::vector<float> p(n), m(n), v(n), gf(n);
      std::vector<uint16_t> gb(n), pout(n);
      for (int64_t i = 0; i < n; ++i) {
        p[i] = nd(rng);
        m[i] = 0.1f * nd(rng);
        v[i] = std::abs(0.01f * nd(rng));
        gb[i] = llmt::f32_to_bf16(nd(rng));
        gf[i] = use_bf16 ? llmt::bf16_to_f32(gb[i]) : nd(rng);
      }
      std::vector<double> rp(p.begin(), p.end()), rm(m.begin(), m.end()), rv(v.begin(), v.end());
      const double lr = 1e-3, b1 = 0.9, b2 = 0.95, eps = 1e-8, wd = 0.1, sc = 0.5;
      const int64_t step = 3;
      llmt::adamw_host(p.data(), m.data(), v.data(), use_bf16 ? gb.data() : nullptr, use_bf16 ? nullptr : gf.data(),
                       pout.data(), n, lr, b1, b2, eps, wd, step, sc, nthreads);
      const double bc1 = 1 - std::pow(b1, step), bc2 = 1 - std::pow(b2, step);
      double worst = 0;
      for (int64_t i = 0; i < n; ++i) {
        const double g = gf[i] * sc;
        rm[i] = b1 * rm[i] + (1 - b1) * g;
        rv[i] = b2 * rv[i] + (1 - b2) * g * g;
        rp[i] = rp[i] * (1 - lr * wd) - lr / bc1 * rm[i] / (std::sqrt(rv[i]) / std::sqrt(bc2) + eps);
        worst = std::max(worst, std::abs(rp[i] - p[i]) / (1e-3 + std::abs(rp[i])));
        CHECK(pout[i] == llmt::f32_to_bf16(p[i]), "bf16 copy of p differs at %lld", (long long)i);
      }
      CHECK(worst < 1e-5, "adamw (n %lld, bf16 %d, threads %lld) rel err %g", (long long)n, use_bf16,
            (long long)nthreads, worst);
    }
  }
  CHECK(llmt::f32_to_bf16(NAN) != llmt::f32_to_bf16(INFINITY), "NaN must stay NaN");
}

int main(int argc, char** argv) {
  const int64_t threads = argc > 1 ? std::atoll(argv[1]) : 4;
  std::mt19937_64 rng(1234);
  check_packing(rng);
  check_adamw(rng, 1);
  check_adamw(rng, threads);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host sanitize harness: ok\n");
  return 0;
}
