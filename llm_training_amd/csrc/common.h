// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of llm_training_amd.
//
// Conventions used by every kernel in this directory:
//  * wave64 everywhere (warpSize folds to 64 on gfx950) — reductions use __shfl_xor over 64 lanes;
//  * 16-byte vector accesses (8 x bf16 / 4 x fp32) for every streaming load/store;
//  * fp32 accumulation for every reduction, bf16 storage for activations;
//  * every launcher takes an explicit hipStream_t (the caller passes torch's current stream) so the
//    kernels compose with HIP graphs and with the side streams of the ZeRO engine.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace llmt {

constexpr int kWave = 64;

using bf16 = __hip_bfloat16;

// 8 x bf16 packed in 16 bytes.
struct alignas(16) bf16x8 {
  uint32_t w[4];
};

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Round-to-nearest-even fp32 -> bf16 (keeps NaN a NaN through the compiler's v_cvt_pk_bf16_f32).
__device__ __forceinline__ uint16_t f2bf_bits(float f) {
  bf16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf_bits(lo) | ((uint32_t)f2bf_bits(hi) << 16);
}

__device__ __forceinline__ void unpack8(const bf16x8& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf16_lo(v.w[i]);
    f[2 * i + 1] = bf16_hi(v.w[i]);
  }
}
__device__ __forceinline__ bf16x8 pack8(const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v.w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

__device__ __forceinline__ float bf2f(bf16 x) { return __bfloat162float(x); }
__device__ __forceinline__ float bfbits2f(uint16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blocks of NW waves; `red` must hold NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  __syncthreads();
  return t;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Grid size for grid-stride memory-bound kernels: ≥ 8 blocks per CU on 256 CUs, capped.
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace llmt

#define LLMT_HIP_CHECK(expr)                                                     \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) return _e;                                             \
  } while (0)
