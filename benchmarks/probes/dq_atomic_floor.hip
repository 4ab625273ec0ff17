// The dQ-accumulation floor of a single-pass (dK, dV, dQ) attention backward on MI355X.
//
// A one-kernel backward (key-parallel workgroups that also produce dQ) must sum each query row's dQ
// over every key block that sees it. With fp32 atomics that is, per (batch, q head), S x D floats added
// (S / KB + 1) / 2 times on average under the causal mask. This program issues EXACTLY that atomic
// traffic — same workgroup grid (one workgroup per (batch, kv head, key block of KB keys), looping over
// the group's q heads and the visible 32-row query tiles), same instruction shape (one register of a
// 32x32 fp32 accumulator per wave-instruction: two 128-byte row segments) — with no compute, so its time
// is a lower bound for the fused kernel's time. Compared against the two-kernel backward
// (fa_bwd_dkdv128 + fa_bwd_dq3) at Llama-3-8B shapes.
//
//   hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics benchmarks/dq_atomic_floor.hip -o /tmp/dq_floor
//   /tmp/dq_floor [B S Hq Hkv]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));         \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int D = 128;

// grid: (S / KB) * Hkv * B workgroups, KB / 32 waves of 32 keys each (KB = 128: 4 waves, 256: 8 waves).
// Per visible 32-row query tile every wave adds a 32 x 32 fp32 block (its D-quarter / eighth of the
// workgroup's dQ tile after an LDS reduction would be the same bytes): 16 wave-instructions, each one
// accumulator register = rows (r, r + 4) x 32 contiguous floats.
template <int KB>
__global__ __launch_bounds__(KB * 2) void dq_atomics(float* dq, int B, int S, int Hq, int Hkv) {
  constexpr int NW = KB / 32;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int L = blockIdx.x;
  const int hk = L % Hkv;
  L /= Hkv;
  const int b = L % B;
  const int kb = L / B;
  const int grp = Hq / Hkv;
  const int q0 = kb * KB;  // causal: query rows from the block's first key on
  // the workgroup's dQ tile is 32 rows x 128 columns; wave w owns columns (w % 4) * 32.., and with 8 waves
  // the two wave halves split the rows of each register (each still a 2 x 128-byte shape)
  const int col = (wid % 4) * 32 + (lane & 31);
  const int hh = lane >> 5;
  for (int g = 0; g < grp; ++g) {
    const int h = hk * grp + g;
    float* base = dq + ((int64_t)b * S * Hq + h) * D;  // [B, S, Hq, D]
    for (int t = q0; t < S; t += 32) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (NW == 8 && ((j >> 3) != (wid >> 2))) continue;  // 8 waves: each register added by one wave half
        const int row = t + 8 * (j >> 2) + 4 * hh + (j & 3);
        atomicAdd(base + (int64_t)row * Hq * D + col, 1.0f);
      }
    }
  }
}

template <int KB>
static float run(float* dq, int B, int S, int Hq, int Hkv, int iters) {
  const int nblk = (S / KB) * Hkv * B;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  dq_atomics<KB><<<nblk, KB * 2>>>(dq, B, S, Hq, Hkv);  // warm-up
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) dq_atomics<KB><<<nblk, KB * 2>>>(dq, B, S, Hq, Hkv);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  int B = 4, S = 8192, Hq = 32, Hkv = 8;
  if (argc == 5) {
    B = atoi(argv[1]);
    S = atoi(argv[2]);
    Hq = atoi(argv[3]);
    Hkv = atoi(argv[4]);
  }
  if (S % 256 != 0 || Hq % Hkv != 0) {
    fprintf(stderr, "S must be a multiple of 256 and Hq of Hkv\n");
    return 1;
  }
  float* dq;
  const size_t n = (size_t)B * S * Hq * D;
  CHECK(hipMalloc(&dq, n * sizeof(float)));
  CHECK(hipMemset(dq, 0, n * sizeof(float)));
  for (int kb : {128, 256}) {
    const float ms = kb == 128 ? run<128>(dq, B, S, Hq, Hkv, 5) : run<256>(dq, B, S, Hq, Hkv, 5);
    // added bytes: per (b, h) sum over key blocks of (S - q0) rows x D floats
    double bytes = 0;
    for (int q0 = 0; q0 < S; q0 += kb) bytes += (double)(S - q0) * D * 4;
    bytes *= (double)B * Hq;
    printf("{\"B\": %d, \"S\": %d, \"Hq\": %d, \"Hkv\": %d, \"key_block\": %d, \"ms\": %.3f, \"atomic_GB\": %.2f, "
           "\"TB_per_s\": %.3f}\n",
           B, S, Hq, Hkv, kb, ms, bytes / 1e9, bytes / ms / 1e9);
  }
  CHECK(hipFree(dq));
  return 0;
}
