// Fused AdamW step and gradient-norm reduction on flat (sharded) buffers, gfx950.
//
// Replaces DeepSpeed FusedAdam (reference configs
// config/examples/llama-3.1/llama-3.1-8b_pt_example.yaml:44) together with the 3-pass Python master-
// weight wrapper (reference src/llm_training/optim/master_weight_wrapper.py:63-80: grad.float() copy ->
// inner step -> copy back). One pass per element: read bf16 (or fp32) grad, fp32 master, m, v; write
// master, m, v and the bf16 model parameter. The gradient-clipping coefficient is read from device
// memory, so clipping never synchronises with the host.
#include "common.h"

namespace llmt {

template <typename GradT>
__device__ __forceinline__ void load4(const GradT* g, int64_t i, float* out);
template <>
__device__ __forceinline__ void load4<float>(const float* g, int64_t i, float* out) {
  *reinterpret_cast<float4*>(out) = reinterpret_cast<const float4*>(g)[i];
}
template <>
__device__ __forceinline__ void load4<bf16>(const bf16* g, int64_t i, float* out) {
  const uint2 w = reinterpret_cast<const uint2*>(g)[i];
  out[0] = bf16_lo(w.x);
  out[1] = bf16_hi(w.x);
  out[2] = bf16_lo(w.y);
  out[3] = bf16_hi(w.y);
}

// One float4 group per thread and no grid-stride loop: every wave instruction covers contiguous bytes
// (fp32 streams 1 KiB, bf16 grad / param copy 512 B) and the grid is as large as the unit. Measured on
// one Llama-3-8B layer unit (218 M params, 28 B/param, benchmarks/membw_probe.hip): 1.14 ms = 5.4 TB/s
// vs 1.33 ms (4.6 TB/s) for the earlier 8-per-thread grid-stride form (two adjacent float4 per stream).
template <typename GradT>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ m,
                                                    float* __restrict__ v, const GradT* __restrict__ g,
                                                    bf16* __restrict__ pout, int64_t n4, float lr, float b1,
                                                    float b2, float eps, float wd, float step_size,
                                                    float inv_sqrt_bc2, const float* __restrict__ gscale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float sc = gscale ? gscale[0] : 1.f;
  const float decay = 1.f - lr * wd;
  typedef float f4 __attribute__((ext_vector_type(4)));
  float gg[4];
  load4<GradT>(g, i, gg);
  f4 pp = reinterpret_cast<const f4*>(p)[i];
  f4 mm = reinterpret_cast<const f4*>(m)[i];
  f4 vv = reinterpret_cast<const f4*>(v)[i];
  float pf[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gk = gg[k] * sc;
    const float mk = b1 * mm[k] + (1.f - b1) * gk;
    const float vk = b2 * vv[k] + (1.f - b2) * gk * gk;
    const float denom = sqrtf(vk) * inv_sqrt_bc2 + eps;
    pf[k] = pp[k] * decay - step_size * mk / denom;
    mm[k] = mk;
    vv[k] = vk;
    pp[k] = pf[k];
  }
  __builtin_nontemporal_store(pp, reinterpret_cast<f4*>(p) + i);
  __builtin_nontemporal_store(mm, reinterpret_cast<f4*>(m) + i);
  __builtin_nontemporal_store(vv, reinterpret_cast<f4*>(v) + i);
  if (pout) {
    uint2 o;
    o.x = pack_bf16x2(pf[0], pf[1]);
    o.y = pack_bf16x2(pf[2], pf[3]);
    reinterpret_cast<uint2*>(pout)[i] = o;
  }
}

// Deterministic sum of squares (the clipping norm must not depend on atomic ordering, so two runs of
// the same step produce the same update): pass 1 writes one partial per block, pass 2 adds the
// partials in a fixed order and accumulates into out[0] (units are summed in launch order).
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, int64_t n4, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float f[4];
    load4<T>(x, i, f);
    s += f[0] * f[0] + f[1] * f[1] + f[2] * f[2] + f[3] * f[3];
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// bf16 form with 16-byte loads, two per thread in flight per iteration (the 8-byte, one-load form read a
// 218 M-element gradient at 3.7 TB/s with its 1024 partial blocks); the partials stay one per block
__global__ __launch_bounds__(256) void sumsq8_kernel(const bf16* __restrict__ x, int64_t n8, float* __restrict__ part) {
  __shared__ float red[4];
  float s0 = 0.f, s1 = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < n8; i += 2 * stride) {
    const bf16x8 a = reinterpret_cast<const bf16x8*>(x)[i];
    const bf16x8 b = reinterpret_cast<const bf16x8*>(x)[i + stride];
    float fa[8], fb[8];
    unpack8(a, fa);
    unpack8(b, fb);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s0 += fa[k] * fa[k];
      s1 += fb[k] * fb[k];
    }
  }
  if (i < n8) {
    float fa[8];
    unpack8(reinterpret_cast<const bf16x8*>(x)[i], fa);
#pragma unroll
    for (int k = 0; k < 8; ++k) s0 += fa[k] * fa[k];
  }
  const float s = block_sum<4>(s0 + s1, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) out[0] += s;
}

}  // namespace llmt

using namespace llmt;

extern "C" hipError_t llmt_adamw(float* p, float* m, float* v, const void* g, int grad_is_fp32, void* pout,
                                 int64_t n, float lr, float b1, float b2, float eps, float wd, int64_t step,
                                 const float* gscale, hipStream_t stream) {
  if (n % 4) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  if (n4 == 0) return hipSuccess;
  const double bc1 = 1.0 - pow((double)b1, (double)step);
  const double bc2 = 1.0 - pow((double)b2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float inv_sqrt_bc2 = (float)(1.0 / sqrt(bc2));
  const int64_t blocks = (n4 + 255) / 256;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  if (grad_is_fp32)
    adamw_kernel<float><<<(unsigned)blocks, 256, 0, stream>>>(p, m, v, (const float*)g, (bf16*)pout, n4, lr, b1, b2,
                                                             eps, wd, step_size, inv_sqrt_bc2, gscale);
  else
    adamw_kernel<bf16><<<(unsigned)blocks, 256, 0, stream>>>(p, m, v, (const bf16*)g, (bf16*)pout, n4, lr, b1, b2,
                                                            eps, wd, step_size, inv_sqrt_bc2, gscale);
  return hipGetLastError();
}

// ws: >= 1024 floats of scratch
extern "C" hipError_t llmt_sumsq(const void* x, int is_fp32, int64_t n, float* out, float* ws, hipStream_t stream) {
  if (n % 4) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  if (n4 == 0) return hipSuccess;
  const int grid = stream_grid(n4, 256) > 1024 ? 1024 : stream_grid(n4, 256);
  if (!is_fp32 && n % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    sumsq8_kernel<<<grid, 256, 0, stream>>>((const bf16*)x, n / 8, ws);
    sum_partials_kernel<<<1, 256, 0, stream>>>(ws, grid, out);
    return hipGetLastError();
  }
  if (is_fp32)
    sumsq_kernel<float><<<grid, 256, 0, stream>>>((const float*)x, n4, ws);
  else
    sumsq_kernel<bf16><<<grid, 256, 0, stream>>>((const bf16*)x, n4, ws);
  sum_partials_kernel<<<1, 256, 0, stream>>>(ws, grid, out);
  return hipGetLastError();
}
