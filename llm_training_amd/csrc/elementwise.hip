// Fused elementwise kernels for gfx950: SwiGLU (SiLU·mul) and rotary position embedding.
//
// SwiGLU replaces the reference's LigerSiLUMulFunction (reference call sites
// src/llm_training/ops/liger_kernel/swiglu_op.py:36-39 <- models/llama/llama_model.py:427). Our MLP
// keeps gate and up projections in ONE fused GEMM whose output row is [gate(I) | up(I)], so the
// kernel reads the fused [T, 2I] buffer directly (no torch.chunk views, no copies).
//
// RoPE replaces src/llm_training/ops/rope_op.py:10-20. It runs IN PLACE on the
// fused QKV GEMM output [T, Hq+2Hkv, D] for the q and k heads, gathering cos/sin from a
// precomputed fp32 table by position id (packed-sequence aware: any position layout works).
// Backward is the same kernel with the rotation negated (rotate by -theta).
#include "common.h"

#include <cstdlib>

namespace llmt {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// c[t, j] = silu(gu[t, j]) * gu[t, I + j]
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16x8* __restrict__ gu, bf16x8* __restrict__ c,
                                                         int64_t n8, int I8) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n8; e += (int64_t)gridDim.x * 256) {
    const int64_t t = e / I8;
    const int j = (int)(e - t * I8);
    float a[8], b[8], o[8];
    unpack8(gu[t * 2 * I8 + j], a);
    unpack8(gu[t * 2 * I8 + I8 + j], b);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = a[i] * sigmoidf_(a[i]) * b[i];
    c[e] = pack8(o);
  }
}

// d gate = dc * b * s * (1 + a * (1 - s)),  d up = dc * a * s
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16x8* __restrict__ gu, const bf16x8* __restrict__ dc,
                                                         bf16x8* __restrict__ dgu, int64_t n8, int I8) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n8; e += (int64_t)gridDim.x * 256) {
    const int64_t t = e / I8;
    const int j = (int)(e - t * I8);
    float a[8], b[8], g[8], da[8], db[8];
    unpack8(gu[t * 2 * I8 + j], a);
    unpack8(gu[t * 2 * I8 + I8 + j], b);
    unpack8(dc[e], g);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float s = sigmoidf_(a[i]);
      const float silu = a[i] * s;
      da[i] = g[i] * b[i] * s * (1.f + a[i] * (1.f - s));
      db[i] = g[i] * silu;
    }
    dgu[t * 2 * I8 + j] = pack8(da);
    dgu[t * 2 * I8 + I8 + j] = pack8(db);
  }
}

// Row-blocked forms (default): grid (ceil(I8 / 256), T), one 16-byte group per thread, no grid-stride loop
// and no 64-bit index division (the flat grid-stride forms above divide a 64-bit element index by I8 per
// item). T = 32768, I = 14336: forward 0.563 -> 0.496 ms (5.0 -> 5.7 TB/s), backward 0.962 -> 0.857 ms,
// bitwise-equal outputs (profiles/r3_elementwise_kernels.jsonl)
__global__ __launch_bounds__(256) void swiglu_fwd_rows_kernel(const bf16x8* __restrict__ gu, bf16x8* __restrict__ c,
                                                              int I8) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= I8) return;
  const int64_t t = blockIdx.y;
  float a[8], b[8], o[8];
  unpack8(gu[t * 2 * I8 + j], a);
  unpack8(gu[t * 2 * I8 + I8 + j], b);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = a[i] * sigmoidf_(a[i]) * b[i];
  c[t * I8 + j] = pack8(o);
}

__global__ __launch_bounds__(256) void swiglu_bwd_rows_kernel(const bf16x8* __restrict__ gu, const bf16x8* __restrict__ dc,
                                                              bf16x8* __restrict__ dgu, int I8) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= I8) return;
  const int64_t t = blockIdx.y;
  float a[8], b[8], g[8], da[8], db[8];
  unpack8(gu[t * 2 * I8 + j], a);
  unpack8(gu[t * 2 * I8 + I8 + j], b);
  unpack8(dc[t * I8 + j], g);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float s = sigmoidf_(a[i]);
    const float silu = a[i] * s;
    da[i] = g[i] * b[i] * s * (1.f + a[i] * (1.f - s));
    db[i] = g[i] * silu;
  }
  dgu[t * 2 * I8 + j] = pack8(da);
  dgu[t * 2 * I8 + I8 + j] = pack8(db);
}

// In-place rotary embedding (HF rotate_half convention): for i < D/2,
//   y[i]       = x[i] * cos - x[i+D/2] * sin
//   y[i+D/2]   = x[i+D/2] * cos + x[i] * sin
// One thread owns 8 consecutive pairs of one (token, head). sign = -1 applies the inverse rotation.
template <typename PosT>
__global__ __launch_bounds__(256) void rope_kernel(bf16* __restrict__ qkv, const PosT* __restrict__ pos,
                                                   const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                                                   int64_t T, int nheads, int D, int64_t stride_t, int stride_h,
                                                   float sign, int64_t P, int* __restrict__ err) {
  const int half = D >> 1;
  const int groups = half >> 3;  // 8 pairs per thread
  const int64_t total = T * nheads * groups;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int g = (int)(e % groups);
    const int64_t th = e / groups;
    const int h = (int)(th % nheads);
    const int64_t t = th / nheads;
    int64_t p = (int64_t)pos[t];
    if (p < 0 || p >= P) {  // position outside the cos/sin table: flag it, read a valid row
      if (err) err[0] = 1;
      p = p < 0 ? 0 : P - 1;
    }
    bf16* base = qkv + t * stride_t + (int64_t)h * stride_h + g * 8;
    bf16x8* lo = reinterpret_cast<bf16x8*>(base);
    bf16x8* hi = reinterpret_cast<bf16x8*>(base + half);
    const float4* cp = reinterpret_cast<const float4*>(cos_t + p * half + g * 8);
    const float4* sp = reinterpret_cast<const float4*>(sin_t + p * half + g * 8);
    float c[8], s[8];
    *reinterpret_cast<float4*>(c) = cp[0];
    *reinterpret_cast<float4*>(c + 4) = cp[1];
    *reinterpret_cast<float4*>(s) = sp[0];
    *reinterpret_cast<float4*>(s + 4) = sp[1];
    float x1[8], x2[8], y1[8], y2[8];
    unpack8(*lo, x1);
    unpack8(*hi, x2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sn = sign * s[i];
      y1[i] = x1[i] * c[i] - x2[i] * sn;
      y2[i] = x2[i] * c[i] + x1[i] * sn;
    }
    *lo = pack8(y1);
    *hi = pack8(y2);
  }
}

// Token-blocked form (default): a 64 x 4 block rotates 4 tokens, the 64 lanes of a row walking that
// token's (head, 8-pair group) items; the position and its table row are read once per item from L1
// and there is no 64-bit division per item (the flat form divides a 64-bit index three times)
template <typename PosT>
__global__ __launch_bounds__(256) void rope_rows_kernel(bf16* __restrict__ qkv, const PosT* __restrict__ pos,
                                                        const float* __restrict__ cos_t,
                                                        const float* __restrict__ sin_t, int64_t T, int nheads, int D,
                                                        int64_t stride_t, int stride_h, float sign, int64_t P,
                                                        int* __restrict__ err) {
  const int64_t t = (int64_t)blockIdx.x * 4 + threadIdx.y;
  if (t >= T) return;
  const int half = D >> 1;
  const int groups = half >> 3;
  int64_t p = (int64_t)pos[t];
  if (p < 0 || p >= P) {
    if (err && threadIdx.x == 0) err[0] = 1;
    p = p < 0 ? 0 : P - 1;
  }
  bf16* row = qkv + t * stride_t;
  const float* crow = cos_t + p * half;
  const float* srow = sin_t + p * half;
  for (int it = threadIdx.x; it < nheads * groups; it += 64) {
    const int h = it / groups;
    const int g = it - h * groups;
    bf16* base = row + h * stride_h + g * 8;
    bf16x8* lo = reinterpret_cast<bf16x8*>(base);
    bf16x8* hi = reinterpret_cast<bf16x8*>(base + half);
    float c[8], s[8];
    *reinterpret_cast<float4*>(c) = reinterpret_cast<const float4*>(crow + g * 8)[0];
    *reinterpret_cast<float4*>(c + 4) = reinterpret_cast<const float4*>(crow + g * 8)[1];
    *reinterpret_cast<float4*>(s) = reinterpret_cast<const float4*>(srow + g * 8)[0];
    *reinterpret_cast<float4*>(s + 4) = reinterpret_cast<const float4*>(srow + g * 8)[1];
    float x1[8], x2[8], y1[8], y2[8];
    unpack8(*lo, x1);
    unpack8(*hi, x2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sn = sign * s[i];
      y1[i] = x1[i] * c[i] - x2[i] * sn;
      y2[i] = x2[i] * c[i] + x1[i] * sn;
    }
    *lo = pack8(y1);
    *hi = pack8(y2);
  }
}

// LDS-staged form: a block copies the q / k part of TPB token rows into LDS with contiguous 16-byte
// loads, rotates there, and writes the rows back with contiguous 16-byte stores. With a head dim whose
// half is not a whole number of 128-byte lines (D = 96: 96-byte halves) the direct kernels' lo / hi
// accesses split every line between two instructions; staged, every global access is a full line.
// Requires heads contiguous in the row (stride_h == D). Opt-in (LLMT_ROPE_KERNEL=lds): 0.177 -> 0.167 ms
// standalone for Phi-3 (D96) but slower for Llama (D128) and 1-2 ms slower in the Phi-3 IT step
// (profiles/r3_elementwise_kernels.jsonl), so the token-blocked kernel stays the default.
constexpr int ROPE_TPB = 2;
template <typename PosT>
__global__ __launch_bounds__(256) void rope_lds_kernel(bf16* __restrict__ qkv, const PosT* __restrict__ pos,
                                                       const float* __restrict__ cos_t,
                                                       const float* __restrict__ sin_t, int64_t T, int nheads, int D,
                                                       int64_t stride_t, float sign, int64_t P,
                                                       int* __restrict__ err) {
  extern __shared__ bf16x8 rows[];  // [ROPE_TPB][nheads * D / 8]
  const int64_t t0 = (int64_t)blockIdx.x * ROPE_TPB;
  const int ntok = (int)(T - t0 < ROPE_TPB ? T - t0 : ROPE_TPB);
  const int C = nheads * D / 8;  // 16-byte chunks per token
  for (int i = threadIdx.x; i < ntok * C; i += 256) {
    const int k = i / C;
    rows[i] = reinterpret_cast<const bf16x8*>(qkv + (t0 + k) * stride_t)[i - k * C];
  }
  __syncthreads();
  const int half = D >> 1;
  const int groups = half >> 3;
  const int items = nheads * groups;
  bf16* lrow = reinterpret_cast<bf16*>(rows);
  for (int it = threadIdx.x; it < ntok * items; it += 256) {
    const int k = it / items;
    const int r = it - k * items;
    const int h = r / groups;
    const int g = r - h * groups;
    int64_t p = (int64_t)pos[t0 + k];
    if (p < 0 || p >= P) {
      if (err) err[0] = 1;
      p = p < 0 ? 0 : P - 1;
    }
    bf16* base = lrow + (int64_t)k * nheads * D + h * D + g * 8;
    bf16x8* lo = reinterpret_cast<bf16x8*>(base);
    bf16x8* hi = reinterpret_cast<bf16x8*>(base + half);
    const float* crow = cos_t + p * half + g * 8;
    const float* srow = sin_t + p * half + g * 8;
    float c[8], sn8[8];
    *reinterpret_cast<float4*>(c) = reinterpret_cast<const float4*>(crow)[0];
    *reinterpret_cast<float4*>(c + 4) = reinterpret_cast<const float4*>(crow)[1];
    *reinterpret_cast<float4*>(sn8) = reinterpret_cast<const float4*>(srow)[0];
    *reinterpret_cast<float4*>(sn8 + 4) = reinterpret_cast<const float4*>(srow)[1];
    float x1[8], x2[8], y1[8], y2[8];
    unpack8(*lo, x1);
    unpack8(*hi, x2);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float sn = sign * sn8[i];
      y1[i] = x1[i] * c[i] - x2[i] * sn;
      y2[i] = x2[i] * c[i] + x1[i] * sn;
    }
    *lo = pack8(y1);
    *hi = pack8(y2);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ntok * C; i += 256) {
    const int k = i / C;
    reinterpret_cast<bf16x8*>(qkv + (t0 + k) * stride_t)[i - k * C] = rows[i];
  }
}

}  // namespace llmt

using namespace llmt;

// LLMT_ROPE_ROWS=0 selects the flat grid-stride RoPE kernel (read per call, for A/B runs)
static bool rope_rows() {
  const char* e = getenv("LLMT_ROPE_ROWS");
  return !(e && e[0] == '0');
}

// LLMT_ROPE_KERNEL=lds|rows|flat (read per call, for A/B runs) overrides LLMT_ROPE_ROWS
static int rope_kind() {
  const char* k = getenv("LLMT_ROPE_KERNEL");
  if (k && k[0] == 'l') return 2;
  if (k && k[0] == 'f') return 0;
  if (k && k[0] == 'r') return 1;
  return rope_rows() ? 1 : 0;
}

// rows of one row-blocked launch: grid.y holds at most 65535, so T is split into equal launches (65536 tokens:
// two of 32768, not 65535 + a one-row launch)
static int64_t rows_per_launch(int64_t T) {
  const int64_t n = (T + 65534) / 65535;
  return (T + n - 1) / n;
}

// LLMT_EW_ROWS=0 selects the flat grid-stride SwiGLU kernels (read per call, for A/B runs)
static bool ew_rows(int64_t T) {
  const char* e = getenv("LLMT_EW_ROWS");
  return T <= 65535 * 16 && !(e && e[0] == '0');
}

extern "C" hipError_t llmt_swiglu_fwd(const void* gu, void* c, int64_t T, int I, hipStream_t stream) {
  if (I % 8) return hipErrorInvalidValue;
  const int64_t n8 = T * (I / 8);
  if (n8 == 0) return hipSuccess;
  if (ew_rows(T)) {
    const int64_t rows = rows_per_launch(T);
    for (int64_t t0 = 0; t0 < T; t0 += rows) {
      const int64_t nt = T - t0 < rows ? T - t0 : rows;
      swiglu_fwd_rows_kernel<<<dim3((I / 8 + 255) / 256, (unsigned)nt), 256, 0, stream>>>(
          (const bf16x8*)gu + t0 * (I / 4), (bf16x8*)c + t0 * (I / 8), I / 8);
    }
    return hipGetLastError();
  }
  swiglu_fwd_kernel<<<stream_grid(n8, 256), 256, 0, stream>>>((const bf16x8*)gu, (bf16x8*)c, n8, I / 8);
  return hipGetLastError();
}

extern "C" hipError_t llmt_swiglu_bwd(const void* gu, const void* dc, void* dgu, int64_t T, int I,
                                      hipStream_t stream) {
  if (I % 8) return hipErrorInvalidValue;
  const int64_t n8 = T * (I / 8);
  if (n8 == 0) return hipSuccess;
  if (ew_rows(T)) {
    const int64_t rows = rows_per_launch(T);
    for (int64_t t0 = 0; t0 < T; t0 += rows) {
      const int64_t nt = T - t0 < rows ? T - t0 : rows;
      swiglu_bwd_rows_kernel<<<dim3((I / 8 + 255) / 256, (unsigned)nt), 256, 0, stream>>>(
          (const bf16x8*)gu + t0 * (I / 4), (const bf16x8*)dc + t0 * (I / 8), (bf16x8*)dgu + t0 * (I / 4), I / 8);
    }
    return hipGetLastError();
  }
  swiglu_bwd_kernel<<<stream_grid(n8, 256), 256, 0, stream>>>((const bf16x8*)gu, (const bf16x8*)dc, (bf16x8*)dgu,
                                                               n8, I / 8);
  return hipGetLastError();
}

// qkv: bf16, element strides stride_t (token) / stride_h (head); pos: int32 (pos_is_64=0) or int64.
extern "C" hipError_t llmt_rope(void* qkv, const void* pos, int pos_is_64, const float* cos_t, const float* sin_t,
                                int64_t T, int nheads, int D, int64_t stride_t, int stride_h, int inverse,
                                int64_t P, int* err, hipStream_t stream) {
  if (D % 16 || P <= 0) return hipErrorInvalidValue;
  const int64_t total = T * nheads * (D / 16);
  if (total == 0) return hipSuccess;
  const float sign = inverse ? -1.f : 1.f;
  const int kind = rope_kind();
  const size_t lds = (size_t)ROPE_TPB * nheads * D * 2;
  if (kind == 2 && stride_h == D && lds <= 64 * 1024 && stride_t % 8 == 0) {
    const unsigned grid = (unsigned)((T + ROPE_TPB - 1) / ROPE_TPB);
    if (pos_is_64)
      rope_lds_kernel<int64_t><<<grid, 256, lds, stream>>>((bf16*)qkv, (const int64_t*)pos, cos_t, sin_t, T, nheads, D,
                                                           stride_t, sign, P, err);
    else
      rope_lds_kernel<int32_t><<<grid, 256, lds, stream>>>((bf16*)qkv, (const int32_t*)pos, cos_t, sin_t, T, nheads, D,
                                                           stride_t, sign, P, err);
    return hipGetLastError();
  }
  if (kind >= 1) {  // 4 tokens per 256-thread block; grid.x <= 2^31 - 1 holds for any T we address
    const dim3 grid((unsigned)((T + 3) / 4)), block(64, 4);
    if (pos_is_64)
      rope_rows_kernel<int64_t><<<grid, block, 0, stream>>>((bf16*)qkv, (const int64_t*)pos, cos_t, sin_t, T, nheads,
                                                            D, stride_t, stride_h, sign, P, err);
    else
      rope_rows_kernel<int32_t><<<grid, block, 0, stream>>>((bf16*)qkv, (const int32_t*)pos, cos_t, sin_t, T, nheads,
                                                            D, stride_t, stride_h, sign, P, err);
    return hipGetLastError();
  }
  const int grid = stream_grid(total, 256);
  if (pos_is_64)
    rope_kernel<int64_t><<<grid, 256, 0, stream>>>((bf16*)qkv, (const int64_t*)pos, cos_t, sin_t, T, nheads, D,
                                                   stride_t, stride_h, sign, P, err);
  else
    rope_kernel<int32_t><<<grid, 256, 0, stream>>>((bf16*)qkv, (const int32_t*)pos, cos_t, sin_t, T, nheads, D,
                                                   stride_t, stride_h, sign, P, err);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- 2-D bf16 transpose
// out[C, R] = in[R, C]^T (row-major, leading dims ldi / ldo in elements). 64 x 64 tiles through LDS:
// every global access is a 16-byte vector (two per thread each way); the LDS tile rows are padded to
// 66 elements so the eight 2-byte column reads of one output vector land on distinct banks across the
// wave. Used to hand hipBLASLt its fastest (TN: both operands contraction-contiguous) layout for the
// linear-layer input / weight gradients.
namespace llmt {
__global__ __launch_bounds__(256) void transpose64_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                          int64_t ldi, int64_t ldo) {
  __shared__ uint16_t tile[64][66];
  const int tid = threadIdx.x, cv = (tid & 7) * 8, rr = tid >> 3;
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = rr + 32 * h;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(in + (r0 + r) * ldi + c0 + cv);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<uint32_t*>(&tile[r][cv + 2 * j]) = w[j];
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int oc = rr + 32 * h;  // output row = input column
    bf16x8 v;
    uint16_t* e = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[cv + j][oc];
    *reinterpret_cast<bf16x8*>(out + (c0 + oc) * ldo + r0 + cv) = v;
  }
}
}  // namespace llmt

extern "C" hipError_t llmt_transpose2d(const void* in, void* out, int64_t R, int64_t C, int64_t ldi, int64_t ldo,
                                       hipStream_t stream) {
  if (R % 64 || C % 64 || ldi % 8 || ldo % 8 || ldi < C || ldo < R) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return hipErrorInvalidValue;
  if (R == 0 || C == 0) return hipSuccess;
  if (R / 64 > 65535) return hipErrorInvalidValue;
  llmt::transpose64_kernel<<<dim3((unsigned)(C / 64), (unsigned)(R / 64)), 256, 0, stream>>>(
      (const llmt::bf16*)in, (llmt::bf16*)out, ldi, ldo);
  return hipGetLastError();
}

// Split-K reduction of the weight-gradient GEMM (ops/fused.py wgrad_into): out (+)= sum of `nsplit` fp32
// slabs of n elements each, out bf16 or fp32. One float4 group per thread: reads 16 * nsplit bytes and
// writes 8 (bf16) / 16 (fp32) per group.
namespace llmt {
template <typename OutT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float4* __restrict__ slabs, int nsplit, int64_t n4,
                                                            OutT* __restrict__ out, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 s = slabs[i];
  for (int k = 1; k < nsplit; ++k) {
    const float4 t = slabs[k * n4 + i];
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  if constexpr (sizeof(OutT) == 4) {
    float4* o = reinterpret_cast<float4*>(out) + i;
    if (accumulate) {
      const float4 t = *o;
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    *o = s;
  } else {
    uint2* o = reinterpret_cast<uint2*>(out) + i;
    if (accumulate) {
      const uint2 t = *o;
      s.x += bf16_lo(t.x); s.y += bf16_hi(t.x); s.z += bf16_lo(t.y); s.w += bf16_hi(t.y);
    }
    uint2 w;
    w.x = pack_bf16x2(s.x, s.y);
    w.y = pack_bf16x2(s.z, s.w);
    *o = w;
  }
}
}  // namespace llmt

extern "C" hipError_t llmt_splitk_reduce(const float* slabs, int nsplit, int64_t n, void* out, int out_is_fp32,
                                         int accumulate, hipStream_t stream) {
  if (n % 4 || nsplit < 1) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(slabs) | reinterpret_cast<uintptr_t>(out)) & 15) return hipErrorInvalidValue;
  const int64_t n4 = n / 4, blocks = (n4 + 255) / 256;
  if (n4 == 0) return hipSuccess;
  if (out_is_fp32)
    llmt::splitk_reduce_kernel<float><<<(unsigned)blocks, 256, 0, stream>>>((const float4*)slabs, nsplit, n4,
                                                                           (float*)out, accumulate);
  else
    llmt::splitk_reduce_kernel<llmt::bf16><<<(unsigned)blocks, 256, 0, stream>>>((const float4*)slabs, nsplit, n4,
                                                                                (llmt::bf16*)out, accumulate);
  return hipGetLastError();
}

// SwiGLU backward that also writes dgu^T [2I, T]: the token-contiguous copy the gate_up weight gradient
// needs for hipBLASLt's TN kernel (4.81 vs 5.58 ms for the TT form at T = 32768, I = 14336), produced while
// the tile is in registers instead of by a separate transpose pass that re-reads dgu (0.82 ms). One block
// per 64 tokens x 64 intermediate columns: gate / up / dc rows in, dgu rows out, both halves transposed
// through LDS (rows padded to 66 elements) and written as 128-byte token runs. T and I multiples of 64.
namespace llmt {
__global__ __launch_bounds__(256) void swiglu_bwd_tr_kernel(const bf16* __restrict__ gu, const bf16* __restrict__ dc,
                                                            bf16* __restrict__ dgu, bf16* __restrict__ dguT,
                                                            int64_t T, int I) {
  // LDS tiles of 32-bit words: word [col][p] = (token 2p, token 2p+1) of one output column, so the
  // transposed rows come out as 16-byte reads (4 words = 8 tokens); rows padded to 36 words
  constexpr int PW = 36;
  __shared__ uint32_t tg[64 * PW];
  __shared__ uint32_t tu[64 * PW];
  const int j0 = blockIdx.x * 64;
  const int64_t t0 = (int64_t)blockIdx.y * 64;
  const int tid = threadIdx.x;
  const int cc = tid & 7, p = tid >> 3;  // 8 lanes cover a 128-byte row run; 32 token pairs
  const int c = cc * 8;
  uint32_t wg[8], wu[8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t t = t0 + 2 * p + h;
    const bf16* grow = gu + t * 2 * I;
    bf16* drow = dgu + t * 2 * I;
    float a[8], b[8], g[8], da[8], db[8];
    unpack8(*reinterpret_cast<const bf16x8*>(grow + j0 + c), a);
    unpack8(*reinterpret_cast<const bf16x8*>(grow + I + j0 + c), b);
    unpack8(*reinterpret_cast<const bf16x8*>(dc + t * I + j0 + c), g);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // the swiglu_bwd_kernel math, element for element
      const float sg = sigmoidf_(a[i]);
      const float silu = a[i] * sg;
      da[i] = g[i] * b[i] * sg * (1.f + a[i] * (1.f - sg));
      db[i] = g[i] * silu;
    }
    const bf16x8 pa = pack8(da), pb = pack8(db);
    *reinterpret_cast<bf16x8*>(drow + j0 + c) = pa;
    *reinterpret_cast<bf16x8*>(drow + I + j0 + c) = pb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo_g = pa.w[i] & 0xffffu, hi_g = pa.w[i] >> 16;
      const uint32_t lo_u = pb.w[i] & 0xffffu, hi_u = pb.w[i] >> 16;
      if (h == 0) {
        wg[2 * i] = lo_g; wg[2 * i + 1] = hi_g;
        wu[2 * i] = lo_u; wu[2 * i + 1] = hi_u;
      } else {
        wg[2 * i] |= lo_g << 16; wg[2 * i + 1] |= hi_g << 16;
        wu[2 * i] |= lo_u << 16; wu[2 * i + 1] |= hi_u << 16;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    tg[(c + i) * PW + p] = wg[i];
    tu[(c + i) * PW + p] = wu[i];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k;
    const int j = idx >> 3, ch = idx & 7;  // output row j, tokens 8ch .. 8ch+7
    const uint4 vg = *reinterpret_cast<const uint4*>(tg + j * PW + 4 * ch);
    const uint4 vu = *reinterpret_cast<const uint4*>(tu + j * PW + 4 * ch);
    *reinterpret_cast<uint4*>(dguT + (int64_t)(j0 + j) * T + t0 + ch * 8) = vg;
    *reinterpret_cast<uint4*>(dguT + (int64_t)(I + j0 + j) * T + t0 + ch * 8) = vu;
  }
}
}  // namespace llmt

extern "C" hipError_t llmt_swiglu_bwd_tr(const void* gu, const void* dc, void* dgu, void* dguT, int64_t T, int I,
                                         hipStream_t stream) {
  if (T % 64 || I % 64 || T == 0) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(gu) | reinterpret_cast<uintptr_t>(dc) | reinterpret_cast<uintptr_t>(dgu) |
       reinterpret_cast<uintptr_t>(dguT)) & 15)
    return hipErrorInvalidValue;
  if (T / 64 > 65535) return hipErrorInvalidValue;
  llmt::swiglu_bwd_tr_kernel<<<dim3((unsigned)(I / 64), (unsigned)(T / 64)), 256, 0, stream>>>(
      (const llmt::bf16*)gu, (const llmt::bf16*)dc, (llmt::bf16*)dgu, (llmt::bf16*)dguT, T, I);
  return hipGetLastError();
}
