// Host AdamW in plain C++ (no ATen): shared by the torch op in cpu_adam.cpp and the host sanitizer
// harness (tests/native/host_sanitize.cpp). One pass per element: read g (bf16 or fp32) + p/m/v (fp32),
// write p/m/v and optionally the bf16 copy of p. Same math as the GPU kernel (csrc/optim.hip
// adamw_kernel): decoupled weight decay, bias-corrected step, gradient pre-scaled by the clip /
// accumulation factor. Split over `nthreads` std::threads in contiguous ranges; the inner loop is
// branch-free so the compiler vectorises it.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace llmt {

template <typename F>
void parallel_ranges(int64_t n, int64_t grain, int64_t nthreads, F&& f) {
  const int64_t want = std::max<int64_t>(1, std::min<int64_t>(nthreads, (n + grain - 1) / grain));
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

// One AdamW step over n elements. g_bf16 xor g_f32 is non-null; pout may be null.
inline void adamw_host(float* p, float* m, float* v, const uint16_t* g_bf16, const float* g_f32, uint16_t* pout,
                       int64_t n, double lr, double b1, double b2, double eps, double wd, int64_t step, double gscale,
                       int64_t nthreads) {
  const double bc1 = 1.0 - std::pow(b1, static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(b2, static_cast<double>(step));
  const float step_size = static_cast<float>(lr / bc1);
  const float inv_sqrt_bc2 = static_cast<float>(1.0 / std::sqrt(bc2));
  const float flr = static_cast<float>(lr), fb1 = static_cast<float>(b1), fb2 = static_cast<float>(b2);
  const float feps = static_cast<float>(eps), fwd = static_cast<float>(wd), sc = static_cast<float>(gscale);
  constexpr int64_t kGrain = 1 << 16;  // below 64K elements per thread the spawn cost dominates
  auto run = [&](auto load_g) {
    parallel_ranges(n, kGrain, nthreads, [&](int64_t b, int64_t e) {
      if (pout)
        adamw_span<true>(p, m, v, load_g, pout, b, e, flr, fb1, fb2, feps, fwd, step_size, inv_sqrt_bc2, sc);
      else
        adamw_span<false>(p, m, v, load_g, pout, b, e, flr, fb1, fb2, feps, fwd, step_size, inv_sqrt_bc2, sc);
    });
  };
  if (g_bf16)
    run([g_bf16](int64_t i) { return bf16_to_f32(g_bf16[i]); });
  else
    run([g_f32](int64_t i) { return g_f32[i]; });
}

}  // namespace llmt
