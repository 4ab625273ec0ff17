// Does the MFMA shape change the clock the chip holds under load? Bare loops of bf16 MFMAs on random operands
// (one wave per SIMD, every CU busy), the 32x32x16 form (the attention kernels) against the 16x16x32 form
// (the GEMMs), equal FLOPs per iteration, with NV v_exp_f32 fillers per 32-cycle MFMA slot as an
// attention-softmax stand-in. Prints TF/s per variant after a 2 s warm-up of the same variant.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_shape_probe benchmarks/probes/mfma_shape_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

// asm MFMAs with the accumulator pinned to the AGPR file (the builtin form had hipcc rotate the 16x16
// accumulators through copies every iteration); the loop's end pads the MFMA-write -> read wait states
#define MF32(c, x, y) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y))
#define MF16(c, x, y) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y))

template <int SHAPE, int NV>
__global__ __launch_bounds__(256, 1) void probe(const bf8* in, float* out, int iters) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bf8* p = in + (blockIdx.x * 4 + w) * 256 + lane;  // 4 fragments of 64 lanes per wave
  bf8 a0 = p[0], a1 = p[64], b0 = p[128], b1 = p[192];
  float e[4] = {(float)a0[0] * 0.01f, (float)a0[1] * 0.01f, (float)a1[0] * 0.01f, (float)a1[1] * 0.01f};
  float tot = 0.f;
  if constexpr (SHAPE == 32) {
    f16v c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int it = 0; it < iters; ++it) {
      MF32(c0, a0, b0);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
      MF32(c1, a1, b0);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
      MF32(c2, a0, b1);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
      MF32(c3, a1, b1);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3");
    for (int i = 0; i < 16; ++i) tot += c0[i] + c1[i] + c2[i] + c3[i];
  } else {
    f4v c0 = {}, c1 = {}, c2 = {}, c3 = {}, c4 = {}, c5 = {}, c6 = {}, c7 = {};
    for (int it = 0; it < iters; ++it) {
      MF16(c0, a0, b0);
      MF16(c1, a1, b0);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
      MF16(c2, a0, b1);
      MF16(c3, a1, b1);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
      MF16(c4, a1, b0);
      MF16(c5, a0, b1);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
      MF16(c6, a1, b1);
      MF16(c7, a0, b0);
      for (int v = 0; v < NV; ++v) e[v & 3] = __builtin_amdgcn_exp2f(e[v & 3]) * 0.5f;
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3");
    const f4v cs = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
    tot = cs[0] + cs[1] + cs[2] + cs[3];
  }
  out[(blockIdx.x * 4 + w) * 64 + lane] = tot + e[0] + e[1] + e[2] + e[3];
}

template <int SHAPE, int NV>
double run(const bf8* in, float* out, int iters, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // warm-up: ~2 s of the same variant, so the clock settles where this body holds it
  hipEventRecord(a);
  int n = 0;
  float ms = 0.f;
  while (ms < 2000.f) {
    probe<SHAPE, NV><<<grid, 256>>>(in, out, iters);
    ++n;
    if (n % 8 == 0) {
      hipEventRecord(b);
      hipEventSynchronize(b);
      hipEventElapsedTime(&ms, a, b);
    }
  }
  hipEventRecord(a);
  for (int i = 0; i < 16; ++i) probe<SHAPE, NV><<<grid, 256>>>(in, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  const double flops = 16.0 * grid * 4 * (double)iters * 4 * 32768.0;
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  const int grid = 256 * 2, iters = 20000;  // 2 workgroups per CU -> 2 waves per SIMD
  const size_t n = (size_t)grid * 4 * 256 * 8;  // bf16 elements: 256 bf8 per wave
  std::vector<__bf16> h(n);
  srand(1);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (__bf16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  bf8* in;
  float* out;
  hipMalloc(&in, h.size() * 2);
  hipMalloc(&out, (size_t)grid * 256 * 4);
  hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  printf("{\"variant\": \"32x32x16 nv0\", \"tflops\": %.1f}\n", run<32, 0>(in, out, iters, grid));
  printf("{\"variant\": \"16x16x32 nv0\", \"tflops\": %.1f}\n", run<16, 0>(in, out, iters, grid));
  printf("{\"variant\": \"32x32x16 nv2\", \"tflops\": %.1f}\n", run<32, 2>(in, out, iters, grid));
  printf("{\"variant\": \"16x16x32 nv2\", \"tflops\": %.1f}\n", run<16, 2>(in, out, iters, grid));
  printf("{\"variant\": \"32x32x16 nv0\", \"tflops\": %.1f}\n", run<32, 0>(in, out, iters, grid));
  printf("{\"variant\": \"16x16x32 nv0\", \"tflops\": %.1f}\n", run<16, 0>(in, out, iters, grid));
  hipFree(in);
  hipFree(out);
  return 0;
}
