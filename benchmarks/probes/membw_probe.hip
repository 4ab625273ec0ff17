// Bandwidth probe for the streaming kernels of the optimizer step (standalone, hipcc):
// AdamW access-pattern variants on one Llama-3-8B decoder-layer unit (218 M parameters, 28 B moved per
// parameter) next to a float4 copy, so the kernel in csrc/optim.hip is chosen by measurement.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/membw_probe benchmarks/membw_probe.hip && /tmp/membw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#include "../llm_training_amd/csrc/rmsnorm.hip"

using namespace llmt;
typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

__global__ __launch_bounds__(256) void copy_kernel(const f4* __restrict__ a, f4* __restrict__ b, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

struct Hp {
  float b1, b2, eps, decay, step_size, inv_sqrt_bc2;
};

__device__ __forceinline__ void adam1(float& p, float& m, float& v, float g, const Hp& h) {
  m = h.b1 * m + (1.f - h.b1) * g;
  v = h.b2 * v + (1.f - h.b2) * g * g;
  const float denom = sqrtf(v) * h.inv_sqrt_bc2 + h.eps;
  p = p * h.decay - h.step_size * m / denom;
}

// A: the shipped adamw8 (8 per thread, two adjacent float4 per stream, nt stores, grid-stride)
template <bool NT>
__global__ __launch_bounds__(256) void adam_a(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                              const bf16* __restrict__ g, bf16* __restrict__ po, int64_t n8, Hp h) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float gg[8];
    unpack8(reinterpret_cast<const bf16x8*>(g)[i], gg);
    f4 pp[2], mm[2], vv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      pp[k] = reinterpret_cast<const f4*>(p)[2 * i + k];
      mm[k] = reinterpret_cast<const f4*>(m)[2 * i + k];
      vv[k] = reinterpret_cast<const f4*>(v)[2 * i + k];
    }
    float out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float pk = pp[k / 4][k % 4], mk = mm[k / 4][k % 4], vk = vv[k / 4][k % 4];
      adam1(pk, mk, vk, gg[k], h);
      pp[k / 4][k % 4] = pk;
      mm[k / 4][k % 4] = mk;
      vv[k / 4][k % 4] = vk;
      out[k] = pk;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (NT) {
        __builtin_nontemporal_store(pp[k], reinterpret_cast<f4*>(p) + 2 * i + k);
        __builtin_nontemporal_store(mm[k], reinterpret_cast<f4*>(m) + 2 * i + k);
        __builtin_nontemporal_store(vv[k], reinterpret_cast<f4*>(v) + 2 * i + k);
      } else {
        reinterpret_cast<f4*>(p)[2 * i + k] = pp[k];
        reinterpret_cast<f4*>(m)[2 * i + k] = mm[k];
        reinterpret_cast<f4*>(v)[2 * i + k] = vv[k];
      }
    }
    reinterpret_cast<bf16x8*>(po)[i] = pack8(out);
  }
}

// B: every wave instruction covers contiguous bytes: float4 index = chunk*256*U + u*256 + tid, grad / param
// copy as 8-byte accesses on the same index; U chunks' loads issued before any math
template <int U, bool NT>
__global__ __launch_bounds__(256) void adam_b(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                              const bf16* __restrict__ g, bf16* __restrict__ po, int64_t n4, Hp h) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
    f4 pp[U], mm[U], vv[U];
    uint2 gw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) {
        gw[u] = reinterpret_cast<const uint2*>(g)[i];
        pp[u] = reinterpret_cast<const f4*>(p)[i];
        mm[u] = reinterpret_cast<const f4*>(m)[i];
        vv[u] = reinterpret_cast<const f4*>(v)[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * 256;
      if (i < n4) {
        const float gg[4] = {bf16_lo(gw[u].x), bf16_hi(gw[u].x), bf16_lo(gw[u].y), bf16_hi(gw[u].y)};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float pk = pp[u][k], mk = mm[u][k], vk = vv[u][k];
          adam1(pk, mk, vk, gg[k], h);
          pp[u][k] = pk;
          mm[u][k] = mk;
          vv[u][k] = vk;
        }
        if (NT) {
          __builtin_nontemporal_store(pp[u], reinterpret_cast<f4*>(p) + i);
          __builtin_nontemporal_store(mm[u], reinterpret_cast<f4*>(m) + i);
          __builtin_nontemporal_store(vv[u], reinterpret_cast<f4*>(v) + i);
        } else {
          reinterpret_cast<f4*>(p)[i] = pp[u];
          reinterpret_cast<f4*>(m)[i] = mm[u];
          reinterpret_cast<f4*>(v)[i] = vv[u];
        }
        uint2 o;
        o.x = pack_bf16x2(pp[u][0], pp[u][1]);
        o.y = pack_bf16x2(pp[u][2], pp[u][3]);
        reinterpret_cast<uint2*>(po)[i] = o;
      }
    }
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int64_t n = 218112000;  // one Llama-3-8B decoder layer
  float *p, *m, *v, *src, *dst;
  bf16 *g, *po;
  CK(hipMalloc(&p, n * 4));
  CK(hipMalloc(&m, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&g, n * 2));
  CK(hipMalloc(&po, n * 2));
  CK(hipMalloc(&src, n * 4));
  CK(hipMalloc(&dst, n * 4));
  CK(hipMemset(p, 0, n * 4));
  CK(hipMemset(m, 0, n * 4));
  CK(hipMemset(v, 0, n * 4));
  CK(hipMemset(g, 0x3c, n * 2));
  CK(hipMemset(src, 0, n * 4));
  Hp h{0.9f, 0.95f, 1e-8f, 1.f - 3e-6f, 3e-5f, 1.f};
  const int reps = 20;
  const double adam_bytes = 28.0 * n;
  const int64_t n4 = n / 4, n8 = n / 8;
  int cus = 256;
  for (int gmul : {8, 16, 32}) {
    const int grid = cus * gmul;
    float ms = timeit([&] { copy_kernel<<<grid, 256>>>((const f4*)src, (f4*)dst, n4); }, reps);
    printf("{\"kernel\": \"copy_f4\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, 8.0 * n / ms / 1e9);
  }
  for (int gmul : {8, 16, 32}) {
    const int grid = cus * gmul;
    float ms = timeit([&] { adam_a<true><<<grid, 256>>>(p, m, v, g, po, n8, h); }, reps);
    printf("{\"kernel\": \"adam_a_nt\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
    ms = timeit([&] { adam_a<false><<<grid, 256>>>(p, m, v, g, po, n8, h); }, reps);
    printf("{\"kernel\": \"adam_a\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
  }
  for (int gmul : {4, 8, 16}) {
    const int grid = cus * gmul;
    float ms = timeit([&] { adam_b<1, true><<<grid, 256>>>(p, m, v, g, po, n4, h); }, reps);
    printf("{\"kernel\": \"adam_b1_nt\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
    ms = timeit([&] { adam_b<2, true><<<grid, 256>>>(p, m, v, g, po, n4, h); }, reps);
    printf("{\"kernel\": \"adam_b2_nt\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
    ms = timeit([&] { adam_b<2, false><<<grid, 256>>>(p, m, v, g, po, n4, h); }, reps);
    printf("{\"kernel\": \"adam_b2\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
    ms = timeit([&] { adam_b<4, true><<<grid, 256>>>(p, m, v, g, po, n4, h); }, reps);
    printf("{\"kernel\": \"adam_b4_nt\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
  }
  {  // one chunk per thread, no grid-stride loop
    const int grid = (int)((n4 + 255) / 256);
    float ms = timeit([&] { adam_b<1, true><<<grid, 256>>>(p, m, v, g, po, n4, h); }, reps);
    printf("{\"kernel\": \"adam_b1_nt_flat\", \"grid\": %d, \"ms\": %.3f, \"tb_s\": %.2f}\n", grid, ms, adam_bytes / ms / 1e9);
  }
  {  // RMSNorm + residual at the bench shape (T = 4 x 8192, H = 4096): 4 x T x H x 2 bytes forward
    const int T = 32768, H = 4096;
    bf16 *x = (bf16*)src, *res = (bf16*)dst, *y = g, *ro = po;
    float* rstd = p;
    float ms = timeit([&] { llmt_rmsnorm_fwd(x, res, x, y, ro, rstd, T, H, 1e-5f, 0); }, reps);
    printf("{\"kernel\": \"rmsnorm_fwd_res\", \"ms\": %.3f, \"tb_s\": %.2f}\n", ms, 8.0 * T * H / ms / 1e9);
    ms = timeit([&] { llmt_rmsnorm_bwd(y, x, x, rstd, res, ro, m, v, 1, 0, T, H, 0); }, reps);
    printf("{\"kernel\": \"rmsnorm_bwd_res\", \"ms\": %.3f, \"tb_s\": %.2f}\n", ms, 8.0 * T * H / ms / 1e9);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
