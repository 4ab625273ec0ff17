// Blockwise int8 quantisation for the ZeRO++ communication knobs (reference
// deepspeed_strategy.py:70-72 zero_quantized_weights / zero_quantized_gradients):
//  * quant_int8   : x (bf16 or fp32) -> int8 q + one fp32 scale per 64 elements (absmax / 127)
//  * dequant_int8 : q, scale -> bf16
//  * dequant_sum  : sum_k dequant(q[k], scale[k]) -> bf16 / fp32 out (optionally += out), the reduce
//                   step after an all-to-all of quantised gradient chunks
// Each thread owns 8 consecutive elements (one 16-byte bf16 load / 8-byte int8 store); the 8 threads of
// a 64-element block reduce their absmax with three xor-shuffles inside the wave.
#include "common.h"

namespace llmt {

constexpr int kQB = 64;  // elements per scale

template <typename T>
__device__ __forceinline__ void load8(const T* x, int64_t i, float* f);
template <>
__device__ __forceinline__ void load8<bf16>(const bf16* x, int64_t i, float* f) {
  unpack8(*reinterpret_cast<const bf16x8*>(x + i), f);
}
template <>
__device__ __forceinline__ void load8<float>(const float* x, int64_t i, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(x + i), b = *reinterpret_cast<const float4*>(x + i + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

template <typename T>
__global__ __launch_bounds__(256) void quant_int8_kernel(const T* __restrict__ x, int8_t* __restrict__ q,
                                                         float* __restrict__ scale, int64_t n8) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n8; t += (int64_t)gridDim.x * 256) {
    float f[8];
    load8<T>(x, t * 8, f);
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(f[i]));
    // the 8 threads of one 64-element block are consecutive lanes (t = 8 * block + j)
    am = fmaxf(am, __shfl_xor(am, 1, kWave));
    am = fmaxf(am, __shfl_xor(am, 2, kWave));
    am = fmaxf(am, __shfl_xor(am, 4, kWave));
    const float s = am / 127.f;
    const float inv = am > 0.f ? 127.f / am : 0.f;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo |= (uint32_t)(uint8_t)(int8_t)__float2int_rn(f[i] * inv) << (8 * i);
      hi |= (uint32_t)(uint8_t)(int8_t)__float2int_rn(f[4 + i] * inv) << (8 * i);
    }
    *reinterpret_cast<uint2*>(q + t * 8) = make_uint2(lo, hi);
    if ((t & 7) == 0) scale[t >> 3] = s;
  }
}

__device__ __forceinline__ void deq8(const int8_t* q, float s, float* f) {
  const uint2 v = *reinterpret_cast<const uint2*>(q);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = (float)(int8_t)(v.x >> (8 * i)) * s;
    f[4 + i] = (float)(int8_t)(v.y >> (8 * i)) * s;
  }
}

__global__ __launch_bounds__(256) void dequant_int8_kernel(const int8_t* __restrict__ q,
                                                           const float* __restrict__ scale, bf16* __restrict__ y,
                                                           int64_t n8) {
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n8; t += (int64_t)gridDim.x * 256) {
    float f[8];
    deq8(q + t * 8, scale[t >> 3], f);
    *reinterpret_cast<bf16x8*>(y + t * 8) = pack8(f);
  }
}

// out[i] (+)= sum_k q[k * n + i] * scale[k * n / 64 + i / 64]
template <typename T>
__global__ __launch_bounds__(256) void dequant_sum_kernel(const int8_t* __restrict__ q,
                                                          const float* __restrict__ scale, T* __restrict__ out,
                                                          int64_t n8, int k, int accumulate) {
  const int64_t n = n8 * 8;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n8; t += (int64_t)gridDim.x * 256) {
    float acc[8];
    if (accumulate) {
      if constexpr (sizeof(T) == 2) {
        unpack8(*reinterpret_cast<const bf16x8*>(out + t * 8), acc);
      } else {
        load8<float>(reinterpret_cast<const float*>(out), t * 8, acc);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    }
    for (int j = 0; j < k; ++j) {
      float f[8];
      deq8(q + j * n + t * 8, scale[(j * n) / kQB + (t >> 3)], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<bf16x8*>(out + t * 8) = pack8(acc);
    } else {
      float* o = reinterpret_cast<float*>(out) + t * 8;
      *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
  }
}

}  // namespace llmt

using namespace llmt;

extern "C" hipError_t llmt_quant_int8(const void* x, int x_fp32, int8_t* q, float* scale, int64_t n,
                                      hipStream_t stream) {
  if (n % kQB) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  if (x_fp32)
    quant_int8_kernel<float><<<stream_grid(n8, 256), 256, 0, stream>>>((const float*)x, q, scale, n8);
  else
    quant_int8_kernel<bf16><<<stream_grid(n8, 256), 256, 0, stream>>>((const bf16*)x, q, scale, n8);
  return hipGetLastError();
}

extern "C" hipError_t llmt_dequant_int8(const int8_t* q, const float* scale, void* y, int64_t n, hipStream_t stream) {
  if (n % kQB) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  dequant_int8_kernel<<<stream_grid(n8, 256), 256, 0, stream>>>(q, scale, (bf16*)y, n8);
  return hipGetLastError();
}

extern "C" hipError_t llmt_dequant_sum(const int8_t* q, const float* scale, void* out, int out_fp32, int64_t n,
                                       int k, int accumulate, hipStream_t stream) {
  if (n % kQB) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  if (out_fp32)
    dequant_sum_kernel<float><<<stream_grid(n8, 256), 256, 0, stream>>>(q, scale, (float*)out, n8, k, accumulate);
  else
    dequant_sum_kernel<bf16><<<stream_grid(n8, 256), 256, 0, stream>>>(q, scale, (bf16*)out, n8, k, accumulate);
  return hipGetLastError();
}
