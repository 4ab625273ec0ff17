// RMSNorm forward/backward (+ fused residual add) for gfx950.
//
// Replaces the reference's Liger/Triton RMSNorm (reference call sites
// src/llm_training/ops/liger_kernel/rms_norm_op.py:15-19, models/llama/llama_model.py:271-286).
// Semantics follow src/llm_training/ops/rms_norm_op.py:4-14 ("llama" casting): the normalised
// row is rounded to the input dtype before the weight multiply.
//
// Forward: one wave64 per row (4 rows per 256-thread block). A lane owns NC 16-byte chunks of the
// row (8 bf16 each, columns (c*64+lane)*8), so the whole row lives in registers between the
// reduction and the write — one HBM read and one write per element, no LDS round trip.
// Backward: two waves per row (see rmsnorm_bwd_kernel). dW: each block accumulates its rows' dy*n in
// registers, combines its waves through LDS and writes one fp32 partial row; a second kernel reduces the
// partials column-wise and writes (or accumulates into) the bf16/fp32 weight gradient.
#include "common.h"

#include <cstdlib>

namespace llmt {

template <int NC, bool RES>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(
    const bf16x8* __restrict__ x, const bf16x8* __restrict__ res, const bf16x8* __restrict__ w,
    bf16x8* __restrict__ y, bf16x8* __restrict__ res_out, float* __restrict__ rstd_out,
    int T, int H8, float inv_h, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const int64_t base = (int64_t)row * H8;
  float v[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 64 + lane;
    if (col < H8) {
      unpack8(x[base + col], v[c]);
      if constexpr (RES) {
        float r[8];
        unpack8(res[base + col], r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] += r[i];
        // the residual stream is kept in bf16: round the sum before normalising (matches torch x + r)
        bf16x8 s = pack8(v[c]);
        res_out[base + col] = s;
        unpack8(s, v[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss * inv_h + eps);
  if (lane == 0 && rstd_out) rstd_out[row] = r;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 64 + lane;
    if (col < H8) {
      float wf[8], o[8];
      unpack8(w[col], wf);
      float nf[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) nf[i] = v[c][i] * r;
      unpack8(pack8(nf), nf);  // round the normalised row to bf16 ("llama" casting)
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = nf[i] * wf[i];
      y[base + col] = pack8(o);
    }
  }
}

// dx = rstd * (dn - xhat * mean(dn * xhat)),  dn = dy * w,  xhat = x * rstd; plus the optional residual-stream
// gradient `dres`. Two waves per row, each owning half of the row's 16-byte chunks, and two rows in flight per
// 4-wave block; the halves' dot products meet in LDS behind one barrier per row pair. The residual gradient is
// read after that barrier and the weight row re-read per row, so a wave holds half a row of x / dy plus its dW
// accumulators: 128 VGPRs at H = 4096, four waves per SIMD. (The round-1 kernel, one wave per row with the whole
// row and dres in registers, took 240 VGPRs, two waves per SIMD: 0.260 -> 0.250 ms at T = 32768, H = 4096 and
// 0.385 -> 0.365 ms at T = 65536, H = 3072, profiles/r6_rmsnorm_bwd_ab.jsonl.)
// Per-block partial dW (sum over the block's rows of dy * bf16(xhat)) goes to dw_part[blockIdx] unless null.
template <int NH, bool DRES>
__global__ __launch_bounds__(256, NH <= 4 ? 4 : 2) void rmsnorm_bwd_kernel(
    const bf16x8* __restrict__ dy, const bf16x8* __restrict__ x, const bf16x8* __restrict__ w,
    const float* __restrict__ rstd, const bf16x8* __restrict__ dres, bf16x8* __restrict__ dx,
    float* __restrict__ dw_part, int T, int H8, float inv_h, int rows_per_block) {
  __shared__ float dots[2][2][2];             // [iteration parity][row of the pair][half]
  __shared__ float4 red[2][2 * NH][64];       // the odd rows' dW partials: [half][chunk, quad][lane]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, pr = wid >> 1, hf = wid & 1;
  float dwacc[NH][8];
#pragma unroll
  for (int c = 0; c < NH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) dwacc[c][i] = 0.f;
  const int row0 = blockIdx.x * rows_per_block;
  const int row1 = min(T, row0 + rows_per_block);
  const int iters = (rows_per_block + 1) / 2;  // the same for every wave: the loop holds a barrier
  for (int it = 0; it < iters; ++it) {
    const int row = row0 + 2 * it + pr;
    const bool live = row < row1;
    const int64_t base = (int64_t)(live ? row : 0) * H8;
    const float r = live ? rstd[row] : 0.f;
    // the weight row is re-read (L1 / L2 hits) per row instead of hoisted out of the loop as floats
    const bf16x8* wl = w;
    asm volatile("" : "+s"(wl));
    bf16x8 xv[NH], gv[NH], rv[NH];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (hf * NH + c) * 64 + lane;
      if (live && col < H8) {
        xv[c] = x[base + col];
        gv[c] = dy[base + col];
                float xf[8], g[8], wf[8], nf[8];
        unpack8(xv[c], xf);
        unpack8(gv[c], g);
        unpack8(wl[col], wf);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          nf[i] = xf[i] * r;
          dot += g[i] * wf[i] * nf[i];
        }
        unpack8(pack8(nf), nf);
#pragma unroll
        for (int i = 0; i < 8; ++i) dwacc[c][i] += g[i] * nf[i];
      }
    }
    dot = wave_sum(dot);
    if (lane == 0) dots[it & 1][pr][hf] = dot;
    // (parity-indexed slots: the slot written next was last read before this barrier)
    __syncthreads();
    dot = (dots[it & 1][pr][0] + dots[it & 1][pr][1]) * inv_h;
    // keep the row as packed bf16 across the barrier (re-unpacked below) rather than as the first loop's floats
#pragma unroll
    for (int c = 0; c < NH; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(xv[c].w[i]), "+v"(gv[c].w[i]));
    if constexpr (DRES) {
#pragma unroll
      for (int c = 0; c < NH; ++c) {
        const int col = (hf * NH + c) * 64 + lane;
        if (live && col < H8) rv[c] = dres[base + col];
      }
    }
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (hf * NH + c) * 64 + lane;
      if (live && col < H8) {
        float xf[8], g[8], wf[8], o[8];
        unpack8(xv[c], xf);
        unpack8(gv[c], g);
        unpack8(wl[col], wf);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = r * (g[i] * wf[i] - xf[i] * r * dot);
        if constexpr (DRES) {
          float d2[8];
          unpack8(rv[c], d2);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += d2[i];
        }
        dx[base + col] = pack8(o);
      }
    }
  }
  if (!dw_part) return;  // no weight gradient wanted (frozen weight): no partials
  // the odd rows' waves hand their partials to the even rows' waves of the same half through LDS
  if (pr == 1) {
#pragma unroll
    for (int c = 0; c < NH; ++c)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        red[hf][2 * c + q][lane] = make_float4(dwacc[c][4 * q], dwacc[c][4 * q + 1], dwacc[c][4 * q + 2], dwacc[c][4 * q + 3]);
  }
  __syncthreads();
  if (pr == 0) {
    float* out = dw_part + (int64_t)blockIdx.x * H8 * 8;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (hf * NH + c) * 64 + lane;
      if (col < H8) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float4 o = red[hf][2 * c + q][lane];
          *reinterpret_cast<float4*>(out + col * 8 + 4 * q) = make_float4(
              o.x + dwacc[c][4 * q], o.y + dwacc[c][4 * q + 1], o.z + dwacc[c][4 * q + 2], o.w + dwacc[c][4 * q + 3]);
        }
      }
    }
  }
}

// Column reduction of the per-block dW partials: out[j] (+)= sum_b part[b][j].
// 256 threads = 16 columns x 16 row groups (64-byte row runs), LDS combine of the groups: H / 16 blocks (256 at
// H = 4096) spread the 1024 partial rows over the chip (64 columns x 4 groups per block ran 64 blocks: 21 us a
// call at 1024 partials, r6_llama8b_1gpu_mb4_final3_kernel_stats.md).
template <typename OutT>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, OutT* __restrict__ out,
                                                     int nparts, int H, int accumulate) {
  __shared__ float red[16][17];
  const int cx = threadIdx.x & 15, gy = threadIdx.x >> 4;
  const int j = blockIdx.x * 16 + cx;
  float s = 0.f;
  if (j < H) {
#pragma unroll 4
    for (int b = gy; b < nparts; b += 16) s += part[(int64_t)b * H + j];
  }
  red[gy][cx] = s;
  __syncthreads();
  if (gy == 0 && j < H) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += red[g][cx];
    if (accumulate) t += (float)out[j];
    out[j] = (OutT)t;
  }
}

}  // namespace llmt

using namespace llmt;

#define FWD_CASE(NC)                                                                                   \
  case NC:                                                                                             \
    if (res)                                                                                           \
      rmsnorm_fwd_kernel<NC, true><<<grid, 256, 0, stream>>>((const bf16x8*)x, (const bf16x8*)res,     \
                                                            (const bf16x8*)w, (bf16x8*)y,              \
                                                            (bf16x8*)res_out, rstd, T, H8, inv_h, eps); \
    else                                                                                               \
      rmsnorm_fwd_kernel<NC, false><<<grid, 256, 0, stream>>>((const bf16x8*)x, nullptr,               \
                                                             (const bf16x8*)w, (bf16x8*)y, nullptr,    \
                                                             rstd, T, H8, inv_h, eps);                 \
    break;

extern "C" hipError_t llmt_rmsnorm_fwd(const void* x, const void* res, const void* w, void* y, void* res_out,
                                       float* rstd, int T, int H, float eps, hipStream_t stream) {
  if (H % 8 != 0 || H > 8192) return hipErrorInvalidValue;
  const int H8 = H / 8;
  const int nc = (H8 + 63) / 64;
  const int grid = (T + 3) / 4;
  const float inv_h = 1.f / H;
  if (T == 0) return hipSuccess;
  switch (nc <= 8 ? nc : (nc + 1) / 2 * 2) {
    FWD_CASE(1) FWD_CASE(2) FWD_CASE(3) FWD_CASE(4) FWD_CASE(5) FWD_CASE(6) FWD_CASE(7) FWD_CASE(8)
    FWD_CASE(10) FWD_CASE(12) FWD_CASE(14) FWD_CASE(16)
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#define BWD_CASE(NH)                                                                                   \
  case NH:                                                                                             \
    if (dres)                                                                                          \
      rmsnorm_bwd_kernel<NH, true><<<nblk, 256, 0, stream>>>(                                          \
          (const bf16x8*)dy, (const bf16x8*)x, (const bf16x8*)w, rstd, (const bf16x8*)dres,            \
          (bf16x8*)dx, dw_part, T, H8, inv_h, rpb);                                                    \
    else                                                                                               \
      rmsnorm_bwd_kernel<NH, false><<<nblk, 256, 0, stream>>>(                                         \
          (const bf16x8*)dy, (const bf16x8*)x, (const bf16x8*)w, rstd, nullptr, (bf16x8*)dx, dw_part,  \
          T, H8, inv_h, rpb);                                                                          \
    break;

// dw_part must hold nblocks*H floats where nblocks = llmt_rmsnorm_bwd_nblocks(T, H).
extern "C" int llmt_rmsnorm_bwd_nblocks(int T, int H) {
  // >= 16 rows per block, and as many 4-wave blocks as the kernel's occupancy keeps resident on the 256 CUs
  // (H <= 4096: four waves per SIMD -> 1024 blocks; wider rows: two -> 512). More blocks only add partial rows
  // (round 3, one-wave-per-row kernel at two waves per SIMD: 512 blocks 0.270 ms, 1024 0.286, 2048 0.325).
  // LLMT_RMSNORM_BWD_BLOCKS overrides the cap (read once).
  static const int env_cap = [] {
    const char* e = getenv("LLMT_RMSNORM_BWD_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 0;
  }();
  const int cap = env_cap ? env_cap : ((H / 8 + 127) / 128 <= 4 ? 1024 : 512);
  int nblk = (T + 15) / 16;
  if (nblk > cap) nblk = cap;
  if (nblk < 1) nblk = 1;
  return nblk;
}

extern "C" hipError_t llmt_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                                       const void* dres, void* dx, float* dw_part, void* dw, int dw_is_fp32,
                                       int accumulate, int T, int H, hipStream_t stream) {
  if (H % 8 != 0 || H > 8192) return hipErrorInvalidValue;
  const int H8 = H / 8;
  const int nblk = llmt_rmsnorm_bwd_nblocks(T, H);
  const int rpb = (T + nblk - 1) / nblk;
  const float inv_h = 1.f / H;
  if (T > 0) {
    switch ((H8 + 127) / 128) {  // 16-byte chunks per lane in each half-row
      BWD_CASE(1) BWD_CASE(2) BWD_CASE(3) BWD_CASE(4) BWD_CASE(5) BWD_CASE(6) BWD_CASE(7) BWD_CASE(8)
      default:
        return hipErrorInvalidValue;
    }
  }
  if (dw) {
    const int g = (H + 15) / 16;
    if (dw_is_fp32)
      colsum_kernel<float><<<g, 256, 0, stream>>>(dw_part, (float*)dw, T > 0 ? nblk : 0, H, accumulate);
    else
      colsum_kernel<bf16><<<g, 256, 0, stream>>>(dw_part, (bf16*)dw, T > 0 ? nblk : 0, H, accumulate);
  }
  return hipGetLastError();
}
