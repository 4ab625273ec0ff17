// Flash attention forward / backward for gfx950 (CDNA4) with MFMA 32x32x16 bf16.
//
// Replaces flash-attn 2 (CUDA) `flash_attn_func` / `flash_attn_varlen_func` (SURVEY K6/K7/K8;
// reference call sites src/llm_training/ops/attention_op.py:538-654 <- models/llama/llama_model.py:570-663).
// Instead of unpad -> varlen -> pad (attention_op.py:415-485) the kernels take the padded [B, S, H, D]
// layout directly plus optional per-token segment ids (the reference's packed attention-mask contract,
// SURVEY Q1): a key is visible to a query iff seg[q] == seg[k] (and k <= q when causal, and
// k >= q - window when a sliding window is set). GQA is native (kv head = q head / (Hq/Hkv)).
// q/k/v may be arbitrary strided views (e.g. slices of one fused QKV GEMM output) — no copies.
//
// Layout choices (all wave64, MFMA v_mfma_f32_32x32x16_bf16):
//  * forward / dQ: "swapped" S^T = K·Q^T, so each lane owns ONE query (the MFMA column) and holds its
//    scores for 16 keys in registers: softmax max / sum are lane-local plus one cross-half shuffle.
//    The S^T accumulator is directly the B operand of O^T += V^T·P^T (accumulator-as-operand: registers
//    8s..8s+7 = k-step s), and V^T comes from LDS via ds_read_b64_tr_b16 (hardware transpose read).
//  * dK/dV: S = Q·K^T with the KEY on the lane; P and dS accumulators are directly the B operands of
//    dV^T += dO^T·P and dK^T += Q^T·dS; dO^T / Q^T come from transposed LDS reads.
//  * dQ is a separate query-parallel pass (recomputes S and dP) so the backward needs no atomics and
//    is bitwise deterministic (the reference only offers determinism via FLASH_ATTENTION_DETERMINISTIC,
//    attention_op.py:590-592).
//  * LDS row pitches are chosen per read kind: (2D+16) bytes makes 16 consecutive rows hit distinct
//    16-byte bank slots for ds_read_b128; 320/192 bytes put the 4 rows of a tr-read block in disjoint
//    16-bank ranges.
//  * K/V (or Q/dO) tiles are register-staged: the next tile's global loads are issued before the
//    current tile's MFMAs and written to LDS after the barrier (async-stage split).
//  * query blocks are scheduled heaviest-first (reverse order) so the causal triangle load-balances.
//  * packed sequences (varlen): segments are contiguous runs of equal ids. With the run
//    boundaries of every token (rs = first, re = last index of its run; `seg` then points at a
//    [3][B][S] int32 block: ids, rs, re) a query block only visits key tiles from the run start of its
//    first query (and, non-causal, up to the run end of its last query) — the reference's
//    flash_attn_varlen_func cost, attention_op.py:606-619 — and a tile lying inside the block's single
//    run takes the unmasked fast path; only tiles that straddle a run boundary pay for the
//    per-element segment compare. The same bounds drive the key-parallel dK/dV passes.
#include "common.h"

#include <cstdlib>
#include <initializer_list>
#include <type_traits>
#include <utility>

namespace llmt {

typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
typedef short s16v4 __attribute__((ext_vector_type(4)));
typedef short s16v8 __attribute__((ext_vector_type(8)));
typedef float f32v16 __attribute__((ext_vector_type(16)));
typedef float f32v8 __attribute__((ext_vector_type(8)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32v16 mfma32(const bfv8& a, const bfv8& b, const f32v16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int D>
struct FaGeom {
  static constexpr int KP = 2 * D + 16;           // pitch (bytes) of row-read images
  static constexpr int TP = (D == 128) ? 320 : 192;  // pitch (bytes) of transposed-read images
  static constexpr int NKK = D / 16;              // k-steps of a D-deep product
  static constexpr int NDT = D / 32;              // 32-wide output tiles along D
  static constexpr int V8 = D / 8;                // 16-byte vectors per row
};

__device__ __forceinline__ bfv8 lds_b128(const char* p) { return *reinterpret_cast<const bfv8*>(p); }

__device__ __forceinline__ s16v4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16v4*)(p));
}

// A operand (rows = 32 consecutive columns c0.. of an LDS image, k = image rows) for the
// accumulator-as-B product: element j of lane half hh <-> image row
//   rbase + 8*(j>>2) + 4*hh + (j&3)
// and column c0 + (lane & 31). Two transposed reads, 4 rows each.
__device__ __forceinline__ bfv8 lds_trA(const char* img, int pitch, int rbase, int c0, int lane) {
  const int g = lane >> 4, i16 = lane & 15;
  const int row = rbase + 4 * (g >> 1) + (i16 >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (i16 & 3);
  const char* p = img + row * pitch + col * 2;
  const s16v4 lo = lds_tr(p);
  const s16v4 hi = lds_tr(p + 8 * pitch);
  const s16v8 x = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bfv8, x);
}

// registers 8s..8s+7 of an accumulator tile as a bf16 B operand (k-step s)
__device__ __forceinline__ bfv8 acc_as_b(const f32v16& a, int s) {
  f32v8 f;
  if (s == 0)
    f = __builtin_shufflevector(a, a, 0, 1, 2, 3, 4, 5, 6, 7);
  else
    f = __builtin_shufflevector(a, a, 8, 9, 10, 11, 12, 13, 14, 15);
  return __builtin_convertvector(f, bfv8);
}

// 16-byte buffer load; rows past the descriptor's num_records come back as zeros (no selects).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// The descriptor words must stay scalar, or hipcc wraps every buffer op in a readfirstlane/saveexec
// waterfall loop (cdna guide T20). Build it from kernel-argument / blockIdx values with plain integer
// ops only: HIP's min<int64_t> (lowered through f64) or a readfirstlane round trip both pushed the
// descriptor into VGPRs and produced the waterfall in every K/V load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const int n = (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, n, 0x00020000);
}
__device__ __forceinline__ bfv8 bload8(__amdgpu_buffer_rsrc_t r, int off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return __builtin_bit_cast(bfv8, v);
}

// one-time fragment loads (outside the tile loops): plain global loads, zero rows past the end
__device__ __forceinline__ bfv8 gload8(const bf16* p, bool ok) {
  bfv8 v = *reinterpret_cast<const bfv8*>(p);  // callers clamp p to a valid row
  if (!ok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (__bf16)0.f;
  }
  return v;
}

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Dual-use LDS image of a [rows][D] bf16 tile: for D = 128 one XOR-swizzled image of 256-byte rows
// serves both ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads conflict-free
// (chunk' = chunk ^ ((r&3)<<2 | (r>>2)&3)); other D use a padded row image plus a padded tr image.
template <int D>
struct Img {
  static constexpr bool kDual = (D == 128);
  static constexpr int RP = kDual ? 256 : 2 * D + 16;
  static constexpr int TPb = kDual ? 256 : ((D == 128) ? 320 : 192);
  static constexpr int bytes(int rows) { return kDual ? rows * 256 : rows * (RP + TPb); }
  __device__ static __forceinline__ int swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
  // row image: byte offset of 16-byte chunk ch of row r
  __device__ static __forceinline__ int roff(int r, int ch) {
    if constexpr (kDual) return 256 * r + 16 * (ch ^ swz(r));
    else return r * RP + 16 * ch;
  }
  // transposed-read image: byte offset of element `col` (multiple of 4) of row r
  __device__ static __forceinline__ int toff(int rows, int r, int col) {
    if constexpr (kDual) return 256 * r + 16 * ((col >> 3) ^ swz(r)) + 2 * (col & 7);
    else return rows * RP + r * TPb + 2 * col;
  }
  __device__ static __forceinline__ void store(char* base, int rows, int r, int ch, const bfv8& v) {
    *reinterpret_cast<bfv8*>(base + roff(r, ch)) = v;
    if constexpr (!kDual) *reinterpret_cast<bfv8*>(base + rows * RP + r * TPb + 16 * ch) = v;
  }
  __device__ static __forceinline__ bfv8 row_read(const char* base, int r, int ch) {
    return *reinterpret_cast<const bfv8*>(base + roff(r, ch));
  }
  // A operand of the accumulator-as-B product (see lds_trA): rows rbase.., columns c0 + (lane & 31)
  __device__ static __forceinline__ bfv8 trA(const char* base, int rows, int rbase, int c0, int lane) {
    const int g = lane >> 4, i16 = lane & 15;
    const int row = rbase + 4 * (g >> 1) + (i16 >> 2);
    const int col = c0 + 16 * (g & 1) + 4 * (i16 & 3);
    const s16v4 lo = lds_tr(base + toff(rows, row, col));
    const s16v4 hi = lds_tr(base + toff(rows, row + 8, col));
    return __builtin_bit_cast(bfv8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
};

struct AttnArgs {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  const bf16* o;
  const bf16* dout;
  bf16* out;  // forward: O;  backward: dq
  float* lse;
  const float* delta;
  const int* seg;
  const int* rs;  // run start / end of each token (packed segments), or null
  const int* re;
  // packed segments: (b, 128-row block) pairs in descending order of their work (key tiles of a query
  // block / query tiles of a key block, causal), so the query- / key-parallel kernels start the heaviest
  // blocks first as they do for dense causal rows (ops/fused.py segment_info); null otherwise
  const int* qord;
  const int* kord;
  bf16* dk;
  bf16* dv;
  float* dk_part;
  float* dv_part;
  int B, S, Hq, Hkv;
  int q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh;  // element strides (host-checked < 2^31)
  int d_sb, d_ss, d_sh;    // dout strides
  int dq_sb, dq_ss, dq_sh, dk_sb, dk_ss, dk_sh, dv_sb, dv_ss, dv_sh;
  float scale;
  int causal, window;
  // attention dropout (reference attention_dropout, FA2 dropout_p): a probability is kept iff
  // drop_hash(seed, b * Hq + h, q, k) >= drop_thresh (= p * 2^32) and then scaled by 1 / (1 - p); the
  // backward regenerates the same mask from the same counters. drop_thresh = 0: no dropout.
  uint32_t drop_seed, drop_thresh;
  float drop_scale;
  // dense rows: 1 = a batch row's blocks back to back in the 1-D grids (block_of), so the workgroups
  // co-resident on an XCD share one row's K / V (or Q / dO) stream in L2; 0 = batch-interleaved
  int bmajor;
  // 1: masks from per-row index ranges (the run of a packed row, causal, window, sequence end) instead of
  // per-element segment-id compares; needs run bounds (rs / re) whenever `seg` is set
  int rmask;
  // 1: the query-parallel / dK/dV kernels issue their first K/V (Q/dO) tile DMAs before their own row loads,
  // so the two prologue latencies overlap instead of adding up (short packed documents: the prologue is a
  // large share of a block); 0: rows first (A/B reference, LLMT_FA_EARLY_DMA=0)
  int early;
  // diagnostic probes (LLMT_FA_PROBE, wrong results by design; benchmarks/probes/attn_block_probe.py): forward
  // 1 = no tiles, 2 = no Q row loads, 4 = no O / LSE stores; backward 8 = no tiles in the dQ and dK/dV kernels.
  // Only the diagnostic library (_C_diag.so, built with -DLLMT_DIAG) reads it; in the production library
  // FA_PROBE is the constant 0, so no environment variable can change what the kernels compute.
  int probe;
  // backward (dq3 / dkdv5, always set): the dQ kernel computes delta = rowsum(dO * O) itself and writes the
  // packed per-tile row constants the dK/dV kernel reads here (no separate prep pass)
  float* ldw;
  // RoPE fused into the kernels (ops/fused.py _RopeFlashAttnFn; the reference applies it as its own op,
  // src/llm_training/ops/rope_op.py:10-20 <- models/llama/llama_model.py:553). Token (b, s) sits at position
  // rpos[b * rp_sb + s * rp_ss] (int64 when rpos64) of the half-width fp32 tables rcos / rsin [rP, D/2].
  //  * rope_q: the forward / dQ kernels rotate their Q rows as they load them (q holds UNROTATED queries;
  //    k is rotated by the caller); the dQ kernel also writes the rotated rows to qrot for the dK/dV pass.
  //  * rope_dq / rope_dk: the dQ / dK epilogues apply the inverse rotation, so the kernels return the
  //    gradient of the unrotated q / k.
  const void* rpos;
  const float* rcos;
  const float* rsin;
  int rp_sb, rp_ss, rpos64, rP;
  int rope_q, rope_dq, rope_dk;
  bf16* qrot;
  int qr_sb, qr_ss, qr_sh;
};

#ifdef LLMT_DIAG
#define FA_PROBE(a, m) ((a).probe & (m))
#else
#define FA_PROBE(a, m) 0
#endif

// ---------------------------------------------------------------------------- fused RoPE helpers
// table row of token (b, s): through the position ids, or (rpos null) per-token tables whose row b * rp_sb +
// s * rp_ss holds the token's own cos / sin (one gather per forward, shared by every layer: no dependent
// position load in front of the table read)
__device__ __forceinline__ int rope_pos(const AttnArgs& a, int b, int s) {
  const int64_t i = (int64_t)b * a.rp_sb + (int64_t)s * a.rp_ss;
  const int64_t p = !a.rpos ? i
                    : a.rpos64 ? reinterpret_cast<const int64_t*>(a.rpos)[i]
                               : (int64_t)reinterpret_cast<const int*>(a.rpos)[i];
  return (int)(p < 0 ? 0 : (p >= a.rP ? a.rP - 1 : p));  // out-of-table positions were flagged by the K pass
}
// rotate one row's fragments (lane half hh holds element 16 kk + 8 hh + j in f[kk][j]; the partner of
// element e < D/2 is e + D/2, i.e. fragment kk + NKK/2 in the same lane) with the row's tables cr / sr;
// sign -1 = inverse. Same arithmetic and bf16 rounding as the standalone kernel (csrc/elementwise.hip).
template <int NKK>
__device__ __forceinline__ void rope_frags(bfv8 (&f)[NKK], const float* cr, const float* sr, int hh) {
  constexpr int H = NKK / 2;
#pragma unroll
  for (int kk = 0; kk < H; ++kk) {
    float c[8], s[8];
    *reinterpret_cast<float4*>(c) = *reinterpret_cast<const float4*>(cr + 16 * kk + 8 * hh);
    *reinterpret_cast<float4*>(c + 4) = *reinterpret_cast<const float4*>(cr + 16 * kk + 8 * hh + 4);
    *reinterpret_cast<float4*>(s) = *reinterpret_cast<const float4*>(sr + 16 * kk + 8 * hh);
    *reinterpret_cast<float4*>(s + 4) = *reinterpret_cast<const float4*>(sr + 16 * kk + 8 * hh + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x1 = (float)f[kk][j], x2 = (float)f[kk + H][j];
      f[kk][j] = (__bf16)(x1 * c[j] - x2 * s[j]);
      f[kk + H][j] = (__bf16)(x2 * c[j] + x1 * s[j]);
    }
  }
}
// inverse rotation of one row's fp32 gradient in the row-per-lane store layout (element 32 dt + 8 c + 4 hh + j
// in acc[dt][4 c + j]): 8-column group g = 4 dt + c pairs with group g + D/16 in the same lane
template <int D>
__device__ __forceinline__ void rope_acc_inv(f32v16 (&acc)[D / 32], const float* cr, const float* sr, int hh) {
  constexpr int NG = D / 16;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int g2 = g + NG;
    const float4 c4 = *reinterpret_cast<const float4*>(cr + 8 * g + 4 * hh);
    const float4 s4 = *reinterpret_cast<const float4*>(sr + 8 * g + 4 * hh);
    const float c[4] = {c4.x, c4.y, c4.z, c4.w}, s[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x1 = acc[g >> 2][4 * (g & 3) + j], x2 = acc[g2 >> 2][4 * (g2 & 3) + j];
      acc[g >> 2][4 * (g & 3) + j] = x1 * c[j] + x2 * s[j];
      acc[g2 >> 2][4 * (g2 & 3) + j] = x2 * c[j] - x1 * s[j];
    }
  }
}
// RoPE outside the attention kernels, for the launch paths without the fused form (dropout, the generic
// kernels, opt-in variants): strided [B, S, H, D] rows x -> y (y may alias x), one thread per 8 pairs
__global__ __launch_bounds__(256) void rope_bshd_kernel(AttnArgs a, const bf16* x, int x_sb, int x_ss, int x_sh, bf16* y,
                                                        int y_sb, int y_ss, int y_sh, int H, int D, float sign) {
  const int G = D / 16, half = D / 2;
  const int64_t n = (int64_t)a.B * a.S * H * G;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int g = (int)(e % G);
    int64_t t = e / G;
    const int h = (int)(t % H);
    t /= H;
    const int s = (int)(t % a.S), b = (int)(t / a.S);
    const int p = rope_pos(a, b, s);
    const float* cr = a.rcos + (int64_t)p * half + 8 * g;
    const float* sr = a.rsin + (int64_t)p * half + 8 * g;
    const bf16* xr = x + (int64_t)b * x_sb + (int64_t)s * x_ss + (int64_t)h * x_sh + 8 * g;
    bf16* yr = y + (int64_t)b * y_sb + (int64_t)s * y_ss + (int64_t)h * y_sh + 8 * g;
    bfv8 lo = *reinterpret_cast<const bfv8*>(xr), hi = *reinterpret_cast<const bfv8*>(xr + half);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = cr[j], sn = sign * sr[j], x1 = (float)lo[j], x2 = (float)hi[j];
      lo[j] = (__bf16)(x1 * c - x2 * sn);
      hi[j] = (__bf16)(x2 * c + x1 * sn);
    }
    *reinterpret_cast<bfv8*>(yr) = lo;
    *reinterpret_cast<bfv8*>(yr + half) = hi;
  }
}

__device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint32_t bh, uint32_t q, uint32_t k) {
  uint32_t x = seed ^ (bh * 0x9E3779B1u);
  x ^= q * 0x85EBCA6Bu;
  x = (x ^ (x >> 15)) * 0x2C1B3C6Du;
  x ^= k * 0xC2B2AE35u;
  x = (x ^ (x >> 12)) * 0x297A2D39u;
  return x ^ (x >> 15);
}
// dropout multiplier of probability (q, k): 0 or 1 / (1 - p)
__device__ __forceinline__ float drop_z(const AttnArgs& a, uint32_t bh, int q, int k) {
  return drop_hash(a.drop_seed, bh, (uint32_t)q, (uint32_t)k) >= a.drop_thresh ? a.drop_scale : 0.f;
}

constexpr float kThr = 6.0f;  // defer-max threshold (log2 units): P <= 2^6 before a forced rescale

// The contiguous segment run of a block's first token [lo] and whether the whole block [lo, hi] lies in
// it (uni). Without run information (no segments, or ids only) rs = 0, re = S - 1, uni = !seg: every
// tile then keeps the per-element compare whenever segment ids are present.
struct RunInfo {
  int rs, re;
  bool uni;
};
__device__ __forceinline__ RunInfo block_run(const AttnArgs& a, int b, int lo, int hi) {
  RunInfo ri{0, a.S - 1, a.seg == nullptr};
  if (a.rs) {
    const int64_t base = (int64_t)b * a.S;
    ri.rs = a.rs[base + lo];
    ri.re = a.re[base + lo];
    ri.uni = ri.re >= hi;
  }
  return ri;
}
// Range masks (AttnArgs::rmask). Every mask of a row is an index interval: the keys of query row q are
// [max(rs[q], q - window), causal ? q : re[q]] within [0, S) (documents are contiguous runs: the
// reference's varlen cu_seqlens), and the queries of key row k are [causal ? k : rs[k], min(re[k], k + window)].
// A tile then tests element o (a compile-time offset from the lane's first index i0) with one unsigned
// compare, (i0 - lo + o) <= hi - lo, instead of up to five compares and a segment-id load per element.
struct IdxRange {
  unsigned base, span;  // element o is inside iff base + o <= span (unsigned)
};
__device__ __forceinline__ IdxRange idx_range(int lo, int hi, int i0) {
  if (hi < lo) return {1u, 0u};  // empty: base + o >= 1 > span for every o in [0, 2^31)
  return {(unsigned)(i0 - lo), (unsigned)(hi - lo)};
}
__device__ __forceinline__ bool in_range(const IdxRange& r, int o) { return r.base + (unsigned)o <= r.span; }
// [lo, hi] of the keys of query row q (q >= S: empty)
__device__ __forceinline__ void key_interval(const AttnArgs& a, int b, int q, int& lo, int& hi) {
  lo = 0;
  hi = a.S - 1;
  if (q >= a.S) {
    hi = -1;
    return;
  }
  if (a.rs) {
    lo = a.rs[(int64_t)b * a.S + q];
    hi = a.re[(int64_t)b * a.S + q];
  }
  if (a.causal) hi = min(hi, q);
  if (a.window >= 0) lo = max(lo, q - a.window);
}
// [lo, hi] of the queries of key row k (k >= S: empty)
__device__ __forceinline__ void query_interval(const AttnArgs& a, int b, int k, int& lo, int& hi) {
  lo = 0;
  hi = a.S - 1;
  if (k >= a.S) {
    hi = -1;
    return;
  }
  if (a.rs) {
    lo = a.rs[(int64_t)b * a.S + k];
    hi = a.re[(int64_t)b * a.S + k];
  }
  if (a.causal) lo = max(lo, k);
  if (a.window >= 0) hi = min(hi, k + a.window);
}

// does the segment compare matter for the tile [t0, t1] against a block described by ri?
__device__ __forceinline__ bool seg_mask(const AttnArgs& a, const RunInfo& ri, int t0, int t1) {
  return a.seg && !(ri.uni && t0 >= ri.rs && t1 <= ri.re);
}

// (batch row, 128-row block) of the i-th block of a 1-D grid (i counts blocks of one head): heaviest first.
// Dense rows: query blocks from the last (most key tiles under the causal mask), key blocks from the first.
// Packed rows: the order segment_info sorted by work (qord / kord), which the run layout decides.
__device__ __forceinline__ void block_of(const AttnArgs& a, int i, int nblk, bool query, int& b, int& blk) {
  const int* ord = query ? a.qord : a.kord;
  if (ord) {
    const int bm = ord[i];
    b = bm / nblk;
    blk = bm - b * nblk;
  } else if (a.bmajor) {
    b = i / nblk;
    blk = i - b * nblk;
    if (query) blk = nblk - 1 - blk;
  } else {
    b = i % a.B;
    blk = query ? nblk - 1 - i / a.B : i / a.B;
  }
}

// ============================================================================ forward
// grid: (ceil(S/128), Hq, B), block 256 = 4 waves x 32 queries; KV tiles of 64 keys, double-buffered LDS
// (one barrier per tile), next tile's buffer loads in flight during the current tile's MFMAs.
template <int D>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(AttnArgs a) {
  using G = FaGeom<D>;
  constexpr int BN = 64;
  constexpr int NV = BN * G::V8 / 256;  // staged 16-B vectors per thread per tensor
  constexpr int BUF = BN * G::KP + BN * G::TP + BN * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + 127) / 128;
  const int mb = nqb - 1 - (int)blockIdx.x;
  const int h = blockIdx.y, b = blockIdx.z, hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int qs = mb * 128, qw = qs + wid * 32, qrow = qw + r;
  const bf16* qp = a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh, (int64_t)S * a.k_ss * 2);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh, (int64_t)S * a.v_ss * 2);
  const int* seg = a.seg ? a.seg + (int64_t)b * S : nullptr;
  const int sq = (seg && qrow < S) ? seg[qrow] : 0;
  const float sl2 = a.scale * kLog2e;

  bfv8 qf[G::NKK];
#pragma unroll
  for (int kk = 0; kk < G::NKK; ++kk)
    qf[kk] = gload8(qp + (int64_t)min(qrow, S - 1) * a.q_ss + kk * 16 + hh * 8, qrow < S);

  f32v16 ot[G::NDT];
#pragma unroll
  for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) ot[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  const RunInfo qr = block_run(a, b, qs, min(qs + 127, S - 1));
  int kv_end = a.causal ? min(S, qs + 128) : S;
  if (!a.causal && a.rs) kv_end = min(kv_end, a.re[(int64_t)b * S + min(qs + 127, S - 1)] + 1);
  int kv_beg = a.window >= 0 ? max(0, qs - a.window) : 0;
  kv_beg = max(kv_beg, qr.rs) / BN * BN;

  bfv8 kst[NV], vst[NV];
  int sst = 0;
  auto load_tile = [&, krs, vrs](int n0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, row = e / G::V8, c8 = e % G::V8, kr = n0 + row;
      kst[i] = bload8(krs, (int)(kr * a.k_ss + c8 * 8) * 2);
      vst[i] = bload8(vrs, (int)(kr * a.v_ss + c8 * 8) * 2);
    }
    if (seg && tid < BN) sst = (n0 + tid < S) ? seg[n0 + tid] : -1;
  };
  auto store_tile = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, row = e / G::V8, c8 = e % G::V8;
      *reinterpret_cast<bfv8*>(buf + row * G::KP + c8 * 16) = kst[i];
      *reinterpret_cast<bfv8*>(buf + BN * G::KP + row * G::TP + c8 * 16) = vst[i];
    }
    if (seg && tid < BN) reinterpret_cast<int*>(buf + BN * G::KP + BN * G::TP)[tid] = sst;
  };

  if (kv_beg < kv_end) {
    load_tile(kv_beg);
    store_tile(smem);
  }
  __syncthreads();
  int cur = 0;
  for (int n0 = kv_beg; n0 < kv_end; n0 += BN, cur ^= 1) {
    const bool has_next = n0 + BN < kv_end;
    if (has_next) load_tile(n0 + BN);
    const char* Ks = smem + cur * BUF;
    const char* Vs = Ks + BN * G::KP;
    const int* Ss = reinterpret_cast<const int*>(Vs + BN * G::TP);

    f32v16 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) st[t][i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < G::NKK; ++kk)
        st[t] = mfma32(lds_b128(Ks + (32 * t + r) * G::KP + (kk * 16 + hh * 8) * 2), qf[kk], st[t]);
    }
    // masking only where needed: diagonal (causal), window edge, sequence end, packed segments
    const bool m_causal = a.causal && (n0 + BN - 1 > qw);
    const bool m_window = a.window >= 0 && (n0 < qw + 31 - a.window);
    const bool m_end = n0 + BN > S;
    const bool m_seg = seg_mask(a, qr, n0, n0 + BN - 1);
    float smax = -INFINITY;
    if (m_causal || m_window || m_end || m_seg || qrow >= S) {
      const int lim = qrow - n0 - 4 * hh;         // causal: key offset <= lim
      const int lo = qrow - a.window - n0 - 4 * hh;  // window: key offset >= lo
      const int hi = S - 1 - n0 - 4 * hh;            // bounds
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int4 sk = make_int4(sq, sq, sq, sq);
          if (m_seg) sk = *reinterpret_cast<const int4*>(Ss + 32 * t + 8 * c + 4 * hh);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * c + j, ko = 32 * t + 8 * c + j;
            bool ok = (ko <= hi) && (qrow < S);
            if (a.causal) ok = ok && (ko <= lim);
            if (a.window >= 0) ok = ok && (ko >= lo);
            if (m_seg) ok = ok && ((&sk.x)[j] == sq);
            const float s = ok ? st[t][i] * sl2 : -INFINITY;
            st[t][i] = s;
            smax = fmaxf(smax, s);
          }
        }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          st[t][i] *= sl2;
          smax = fmaxf(smax, st[t][i]);
        }
    }
    smax = fmaxf(smax, __shfl_xor(smax, 32, 64));
    // deferred rescale: keep the running max unless some row grew by more than kThr
    if (__any(smax > m + kThr)) {
      const float mnew = fmaxf(m, smax);
      const float alpha = (mnew == -INFINITY) ? 1.f : fexp2(m - mnew);  // m = -inf -> 0
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) ot[dt][i] *= alpha;
    }
    const float muse = (m == -INFINITY) ? 0.f : m;
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = fexp2(st[t][i] - muse);
        st[t][i] = p;
        rs += p;
      }
    l += rs;  // the normaliser sums the undropped probabilities
    if (a.drop_thresh) {
      const uint32_t bh = (uint32_t)(b * a.Hq + h);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          st[t][i] *= drop_z(a, bh, qrow, n0 + 32 * t + 8 * (i >> 2) + 4 * hh + (i & 3));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bfv8 pb = acc_as_b(st[t], s2);
#pragma unroll
        for (int dt = 0; dt < G::NDT; ++dt)
          ot[dt] = mfma32(lds_trA(Vs, G::TP, 32 * t + 16 * s2, dt * 32, lane), pb, ot[dt]);
      }
    if (has_next) store_tile(smem + (cur ^ 1) * BUF);
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (qrow < S) {
    bf16* op = a.out + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * a.o_sh;
#pragma unroll
    for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint2 w;
        w.x = pack_bf16x2(ot[dt][4 * c] * inv, ot[dt][4 * c + 1] * inv);
        w.y = pack_bf16x2(ot[dt][4 * c + 2] * inv, ot[dt][4 * c + 3] * inv);
        *reinterpret_cast<uint2*>(op + dt * 32 + 8 * c + 4 * hh) = w;
      }
    if (hh == 0) {
      const float muse = (m == -INFINITY) ? 0.f : m;
      a.lse[((int64_t)(int64_t)b * a.Hq + h) * S + qrow] = lt > 0.f ? (muse + __log2f(lt)) * kLn2 : -INFINITY;
    }
  }
}

// ============================================================================ backward: delta = rowsum(dO * O)
template <int D>
__global__ __launch_bounds__(256) void fa_bwd_delta_kernel(AttnArgs a) {
  const int64_t nrows = (int64_t)a.B * a.S * a.Hq;
  for (int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x; row < nrows; row += (int64_t)gridDim.x * 256) {
    const int64_t h = row % a.Hq;
    const int64_t bs = row / a.Hq;
    const int64_t sidx = bs % a.S;
    const int64_t b = bs / a.S;
    const bf16x8* op = reinterpret_cast<const bf16x8*>(a.o + (int64_t)b * a.o_sb + sidx * a.o_ss + (int64_t)h * a.o_sh);
    const bf16x8* dp = reinterpret_cast<const bf16x8*>(a.dout + (int64_t)b * a.d_sb + sidx * a.d_ss + (int64_t)h * a.d_sh);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D / 8; ++c) {
      float x[8], y[8];
      unpack8(op[c], x);
      unpack8(dp[c], y);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += x[i] * y[i];
    }
    ((float*)a.delta)[((int64_t)b * a.Hq + h) * a.S + sidx] = s;
  }
}

// ============================================================================ backward: dQ (query-parallel)
// grid: (ceil(S/128), Hq, B); 4 waves x 32 queries; KV tiles of 64 keys, double-buffered.
template <int D>
__global__ __launch_bounds__(256, 1) void fa_bwd_dq_kernel(AttnArgs a) {
  using G = FaGeom<D>;
  using KI = Img<D>;
  constexpr int BN = 64;
  constexpr int NV = BN * G::V8 / 256;
  constexpr int KB = KI::bytes(BN);
  constexpr int BUF = KB + BN * G::KP + BN * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int nqb = (a.S + 127) / 128;
  const int mb = nqb - 1 - (int)blockIdx.x;
  const int h = blockIdx.y, b = blockIdx.z, hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int qs = mb * 128, qw = qs + wid * 32, qrow = qw + r;
  const bf16* qp = a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh;
  const bf16* dop = a.dout + (int64_t)b * a.d_sb + (int64_t)h * a.d_sh;
  const __amdgpu_buffer_rsrc_t krs = make_rsrc(a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh, (int64_t)S * a.k_ss * 2);
  const __amdgpu_buffer_rsrc_t vrs = make_rsrc(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh, (int64_t)S * a.v_ss * 2);
  const int* seg = a.seg ? a.seg + (int64_t)b * S : nullptr;
  const int sq = (seg && qrow < S) ? seg[qrow] : 0;
  const float sl2 = a.scale * kLog2e;
  const int64_t lrow = ((int64_t)(int64_t)b * a.Hq + h) * S + qrow;
  const float lse2 = qrow < S ? a.lse[lrow] * kLog2e : INFINITY;
  const float dlt = qrow < S ? a.delta[lrow] : 0.f;

  bfv8 qf[G::NKK], df[G::NKK];
#pragma unroll
  for (int kk = 0; kk < G::NKK; ++kk) {
    qf[kk] = gload8(qp + (int64_t)min(qrow, S - 1) * a.q_ss + kk * 16 + hh * 8, qrow < S);
    df[kk] = gload8(dop + (int64_t)min(qrow, S - 1) * a.d_ss + kk * 16 + hh * 8, qrow < S);
  }
  f32v16 dqt[G::NDT];
#pragma unroll
  for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dqt[dt][i] = 0.f;

  const RunInfo qr = block_run(a, b, qs, min(qs + 127, S - 1));
  int kv_end = a.causal ? min(S, qs + 128) : S;
  if (!a.causal && a.rs) kv_end = min(kv_end, a.re[(int64_t)b * S + min(qs + 127, S - 1)] + 1);
  int kv_beg = a.window >= 0 ? max(0, qs - a.window) : 0;
  kv_beg = max(kv_beg, qr.rs) / BN * BN;

  bfv8 kst[NV], vst[NV];
  int sst = 0;
  auto load_tile = [&, krs, vrs](int n0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, row = e / G::V8, c8 = e % G::V8, kr = n0 + row;
      kst[i] = bload8(krs, (int)(kr * a.k_ss + c8 * 8) * 2);
      vst[i] = bload8(vrs, (int)(kr * a.v_ss + c8 * 8) * 2);
    }
    if (seg && tid < BN) sst = (n0 + tid < S) ? seg[n0 + tid] : -1;
  };
  auto store_tile = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, row = e / G::V8, c8 = e % G::V8;
      KI::store(buf, BN, row, c8, kst[i]);
      *reinterpret_cast<bfv8*>(buf + KB + row * G::KP + c8 * 16) = vst[i];
    }
    if (seg && tid < BN) reinterpret_cast<int*>(buf + KB + BN * G::KP)[tid] = sst;
  };
  if (kv_beg < kv_end) {
    load_tile(kv_beg);
    store_tile(smem);
  }
  __syncthreads();
  int cur = 0;
  for (int n0 = kv_beg; n0 < kv_end; n0 += BN, cur ^= 1) {
    const bool has_next = n0 + BN < kv_end;
    if (has_next) load_tile(n0 + BN);
    const char* Ks = smem + cur * BUF;
    const char* Vs = Ks + KB;
    const int* Ss = reinterpret_cast<const int*>(Vs + BN * G::KP);
    const bool m_seg = seg_mask(a, qr, n0, n0 + BN - 1);
    const bool need_mask = m_seg || (n0 + BN > S) || (a.causal && n0 + BN - 1 > qw) ||
                           (a.window >= 0 && n0 < qw + 31 - a.window) || qw + 31 >= S;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32v16 st, dpt;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] = 0.f;
        dpt[i] = 0.f;
      }
#pragma unroll
      for (int kk = 0; kk < G::NKK; ++kk) {
        st = mfma32(KI::row_read(Ks, 32 * t + r, 2 * kk + hh), qf[kk], st);
        dpt = mfma32(lds_b128(Vs + (32 * t + r) * G::KP + (kk * 16 + hh * 8) * 2), df[kk], dpt);
      }
      if (need_mask || a.drop_thresh) {
        // dropout: dS = P * (Z * dP - delta), Z the forward's keep mask / (1 - p)
        const uint32_t bh = (uint32_t)(b * a.Hq + h);
        const int lim = qrow - n0 - 32 * t - 4 * hh;
        const int lo = qrow - a.window - n0 - 32 * t - 4 * hh;
        const int hi = S - 1 - n0 - 32 * t - 4 * hh;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int4 sk = make_int4(sq, sq, sq, sq);
          if (m_seg) sk = *reinterpret_cast<const int4*>(Ss + 32 * t + 8 * c + 4 * hh);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * c + j, ko = 8 * c + j;
            bool ok = (ko <= hi) && (qrow < S);
            if (a.causal) ok = ok && (ko <= lim);
            if (a.window >= 0) ok = ok && (ko >= lo);
            if (m_seg) ok = ok && ((&sk.x)[j] == sq);
            const float p = ok ? fexp2(st[i] * sl2 - lse2) : 0.f;
            const float dp = a.drop_thresh ? dpt[i] * drop_z(a, bh, qrow, n0 + 32 * t + 4 * hh + ko) : dpt[i];
            st[i] = p * (dp - dlt);
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) st[i] = fexp2(st[i] * sl2 - lse2) * (dpt[i] - dlt);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bfv8 db = acc_as_b(st, s2);
#pragma unroll
        for (int dt = 0; dt < G::NDT; ++dt)
          dqt[dt] = mfma32(KI::trA(Ks, BN, 32 * t + 16 * s2, dt * 32, lane), db, dqt[dt]);
      }
    }
    if (has_next) store_tile(smem + (cur ^ 1) * BUF);
    __syncthreads();
  }
  if (qrow < S) {
    bf16* dqp = a.out + (int64_t)b * a.dq_sb + (int64_t)qrow * a.dq_ss + (int64_t)h * a.dq_sh;
#pragma unroll
    for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint2 w;
        w.x = pack_bf16x2(dqt[dt][4 * c] * a.scale, dqt[dt][4 * c + 1] * a.scale);
        w.y = pack_bf16x2(dqt[dt][4 * c + 2] * a.scale, dqt[dt][4 * c + 3] * a.scale);
        *reinterpret_cast<uint2*>(dqp + dt * 32 + 8 * c + 4 * hh) = w;
      }
  }
}

// ============================================================================ backward: dK, dV (key-parallel)
// grid: (ceil(S/128), Hq, B); 4 waves x 32 keys; query tiles of 32 rows, double-buffered.
// Hq == Hkv: writes bf16 dk/dv directly.  GQA: writes fp32 per-q-head partials, reduced afterwards.
template <int D, bool GQA>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv_kernel(AttnArgs a) {
  using G = FaGeom<D>;
  using QI = Img<D>;
  constexpr int BM = 32;
  constexpr int NV = (BM * G::V8 + 255) / 256;
  constexpr int IB = QI::bytes(BM);
  constexpr int BUF = 2 * IB + 3 * BM * 4;  // Q image, dO image, lse*log2e, delta, segment ids
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int kb = (int)blockIdx.x;  // early key blocks see the most queries: launched first
  const int h = blockIdx.y, b = blockIdx.z, hk = h / (a.Hq / a.Hkv);
  const int S = a.S;
  const int ks = kb * 128, kw = ks + wid * 32, kr = kw + r;
  const __amdgpu_buffer_rsrc_t qrs = make_rsrc(a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh, (int64_t)S * a.q_ss * 2);
  const __amdgpu_buffer_rsrc_t drs = make_rsrc(a.dout + (int64_t)b * a.d_sb + (int64_t)h * a.d_sh, (int64_t)S * a.d_ss * 2);
  const bf16* kp = a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh;
  const bf16* vp = a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh;
  const float* lsep = a.lse + ((int64_t)(int64_t)b * a.Hq + h) * S;
  const float* dlp = a.delta + ((int64_t)(int64_t)b * a.Hq + h) * S;
  const int* seg = a.seg ? a.seg + (int64_t)b * S : nullptr;
  const int sk = (seg && kr < S) ? seg[kr] : 0;
  const float sl2 = a.scale * kLog2e;

  bfv8 kf[G::NKK], vf[G::NKK];
#pragma unroll
  for (int kk = 0; kk < G::NKK; ++kk) {
    kf[kk] = gload8(kp + (int64_t)min(kr, S - 1) * a.k_ss + kk * 16 + hh * 8, kr < S);
    vf[kk] = gload8(vp + (int64_t)min(kr, S - 1) * a.v_ss + kk * 16 + hh * 8, kr < S);
  }
  f32v16 dkt[G::NDT], dvt[G::NDT];
#pragma unroll
  for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      dkt[dt][i] = 0.f;
      dvt[dt][i] = 0.f;
    }

  const RunInfo kr_run = block_run(a, b, min(ks, S - 1), min(ks + 127, S - 1));
  int q_beg = a.causal ? ks : 0;
  if (!a.causal) q_beg = max(q_beg, kr_run.rs);
  q_beg = q_beg / BM * BM;
  int q_end = a.window >= 0 ? min(S, ks + 128 + a.window) : S;
  if (a.rs) q_end = min(q_end, a.re[(int64_t)b * S + min(ks + 127, S - 1)] + 1);

  bfv8 qst[NV], dst_[NV];
  float lst = 0.f, dls = 0.f;
  int sst = 0;
  auto load_tile = [&, qrs, drs](int q0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, row = e / G::V8, c8 = e % G::V8, qi = q0 + row;
      if (e < BM * G::V8) {
        qst[i] = bload8(qrs, (int)(qi * a.q_ss + c8 * 8) * 2);
        dst_[i] = bload8(drs, (int)(qi * a.d_ss + c8 * 8) * 2);
      }
    }
    if (tid < BM) {
      const int qi = q0 + tid;
      lst = qi < S ? lsep[qi] * kLog2e : INFINITY;
      dls = qi < S ? dlp[qi] : 0.f;
      if (seg) sst = qi < S ? seg[qi] : -1;
    }
  };
  auto store_tile = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, row = e / G::V8, c8 = e % G::V8;
      if (e < BM * G::V8) {
        QI::store(buf, BM, row, c8, qst[i]);
        QI::store(buf + IB, BM, row, c8, dst_[i]);
      }
    }
    if (tid < BM) {
      float* L = reinterpret_cast<float*>(buf + 2 * IB);
      L[tid] = lst;
      L[BM + tid] = dls;
      reinterpret_cast<int*>(L)[2 * BM + tid] = sst;
    }
  };
  if (q_beg < q_end) {
    load_tile(q_beg);
    store_tile(smem);
  }
  __syncthreads();
  int cur = 0;
  for (int q0 = q_beg; q0 < q_end; q0 += BM, cur ^= 1) {
    const bool has_next = q0 + BM < q_end;
    if (has_next) load_tile(q0 + BM);
    const char* Qs = smem + cur * BUF;
    const char* Ds = Qs + IB;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * IB);
    const float* Dl = Ls + BM;
    const int* Sg = reinterpret_cast<const int*>(Ls + 2 * BM);
    f32v16 sacc, dpacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      sacc[i] = 0.f;
      dpacc[i] = 0.f;
    }
#pragma unroll
    for (int kk = 0; kk < G::NKK; ++kk) {
      sacc = mfma32(QI::row_read(Qs, r, 2 * kk + hh), kf[kk], sacc);
      dpacc = mfma32(QI::row_read(Ds, r, 2 * kk + hh), vf[kk], dpacc);
    }
    const bool m_seg = seg_mask(a, kr_run, q0, q0 + BM - 1);
    const bool need_mask = m_seg || (q0 + BM > S) || (kw + 31 >= S) || (a.causal && kw + 31 > q0) ||
                           (a.window >= 0 && q0 + BM - 1 > kw + a.window);
    const uint32_t bh = (uint32_t)(b * a.Hq + h);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float4 l4 = *reinterpret_cast<const float4*>(Ls + 8 * c + 4 * hh);
      const float4 d4 = *reinterpret_cast<const float4*>(Dl + 8 * c + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * c + j;
        const int qloc = 8 * c + 4 * hh + j;
        float p = fexp2(sacc[i] * sl2 - (&l4.x)[j]);
        if (need_mask) {
          const int qi = q0 + qloc;
          bool ok = kr < S && qi < S;
          if (a.causal) ok = ok && (kr <= qi);
          if (a.window >= 0) ok = ok && (kr >= qi - a.window);
          if (m_seg) ok = ok && (Sg[qloc] == sk);
          p = ok ? p : 0.f;
        }
        if (a.drop_thresh) {  // dV takes the dropped P, dS = P * (Z * dP - delta)
          const float z = drop_z(a, bh, q0 + qloc, kr);
          sacc[i] = p * z;
          dpacc[i] = p * (dpacc[i] * z - (&d4.x)[j]);
        } else {
          sacc[i] = p;                                 // P
          dpacc[i] = p * (dpacc[i] - (&d4.x)[j]);      // dS
        }
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bfv8 pb = acc_as_b(sacc, s2);
      const bfv8 db = acc_as_b(dpacc, s2);
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt) {
        dvt[dt] = mfma32(QI::trA(Ds, BM, 16 * s2, dt * 32, lane), pb, dvt[dt]);
        dkt[dt] = mfma32(QI::trA(Qs, BM, 16 * s2, dt * 32, lane), db, dkt[dt]);
      }
    }
    if (has_next) store_tile(smem + (cur ^ 1) * BUF);
    __syncthreads();
  }
  if (kr < S) {
    if constexpr (GQA) {
      float* dkp = a.dk_part + (((int64_t)b * S + kr) * a.Hq + h) * D;
      float* dvp = a.dv_part + (((int64_t)b * S + kr) * a.Hq + h) * D;
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int d = dt * 32 + 8 * c + 4 * hh;
          *reinterpret_cast<float4*>(dkp + d) =
              make_float4(dkt[dt][4 * c] * a.scale, dkt[dt][4 * c + 1] * a.scale, dkt[dt][4 * c + 2] * a.scale,
                          dkt[dt][4 * c + 3] * a.scale);
          *reinterpret_cast<float4*>(dvp + d) =
              make_float4(dvt[dt][4 * c], dvt[dt][4 * c + 1], dvt[dt][4 * c + 2], dvt[dt][4 * c + 3]);
        }
    } else {
      bf16* dkp = a.dk + (int64_t)b * a.dk_sb + (int64_t)kr * a.dk_ss + (int64_t)hk * a.dk_sh;
      bf16* dvp = a.dv + (int64_t)b * a.dv_sb + (int64_t)kr * a.dv_ss + (int64_t)hk * a.dv_sh;
#pragma unroll
      for (int dt = 0; dt < G::NDT; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int d = dt * 32 + 8 * c + 4 * hh;
          uint2 wk, wv;
          wk.x = pack_bf16x2(dkt[dt][4 * c] * a.scale, dkt[dt][4 * c + 1] * a.scale);
          wk.y = pack_bf16x2(dkt[dt][4 * c + 2] * a.scale, dkt[dt][4 * c + 3] * a.scale);
          wv.x = pack_bf16x2(dvt[dt][4 * c], dvt[dt][4 * c + 1]);
          wv.y = pack_bf16x2(dvt[dt][4 * c + 2], dvt[dt][4 * c + 3]);
          *reinterpret_cast<uint2*>(dkp + d) = wk;
          *reinterpret_cast<uint2*>(dvp + d) = wv;
        }
    }
  }
}

// GQA: dk[b, s, hk, :] = sum over the group's q heads of dk_part[b, s, h, :]  (same for dv)
template <int D>
__global__ __launch_bounds__(256) void fa_gqa_reduce_kernel(AttnArgs a) {
  const int grp = a.Hq / a.Hkv;
  const int64_t total = (int64_t)a.B * a.S * a.Hkv * (D / 4);
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int c4 = (int)(e % (D / 4));
    const int64_t t = e / (D / 4);
    const int hk = (int)(t % a.Hkv);
    const int64_t bs = t / a.Hkv;
    const int s = (int)(bs % a.S);
    const int64_t b = bs / a.S;
    float4 sk = make_float4(0.f, 0.f, 0.f, 0.f), sv = sk;
    for (int g = 0; g < grp; ++g) {
      const int64_t off = ((bs)*a.Hq + hk * grp + g) * D + c4 * 4;
      const float4 x = *reinterpret_cast<const float4*>(a.dk_part + off);
      const float4 y = *reinterpret_cast<const float4*>(a.dv_part + off);
      sk.x += x.x; sk.y += x.y; sk.z += x.z; sk.w += x.w;
      sv.x += y.x; sv.y += y.y; sv.z += y.z; sv.w += y.w;
    }
    uint2 wk, wv;
    wk.x = pack_bf16x2(sk.x, sk.y);
    wk.y = pack_bf16x2(sk.z, sk.w);
    wv.x = pack_bf16x2(sv.x, sv.y);
    wv.y = pack_bf16x2(sv.z, sv.w);
    *reinterpret_cast<uint2*>(a.dk + (int64_t)b * a.dk_sb + (int64_t)s * a.dk_ss + (int64_t)hk * a.dk_sh + c4 * 4) = wk;
    *reinterpret_cast<uint2*>(a.dv + (int64_t)b * a.dv_sb + (int64_t)s * a.dv_ss + (int64_t)hk * a.dv_sh + c4 * 4) = wv;
  }
}

// ============================================================================ backward, D = 128 pipeline
// The D = 64 / 96 / 128 backward (every Llama-family and Phi-3 model) is: the query-parallel dQ kernel
// (fa_bwd_dq3_kernel, two workgroups per CU), which also computes delta and writes the packed per-row
// constants below, and this key-parallel dK/dV kernel, built for one wave per SIMD (512 registers per lane):
//  * Q / dO tiles arrive by LDS-DMA (`buffer_load ... lds`, zero-filled past the end) into a ring of NS
//    slots, several tiles ahead, behind counted `s_waitcnt vmcnt` and a raw barrier.
//  * one wave per SIMD issues one instruction per issue slot, so the loop is instruction-bound, not
//    MFMA-bound (profiles/r2_dkdv_issue_bound.md): descriptors are built once per head, S / dP start
//    from the MFMA's inline zero and the row constants enter the softmax (P = exp2(fma(S, scale*log2e,
//    -lse*log2e)), dS = P (dP - delta), packed fp32), masks only on diagonal / window / packed tiles.
//  * each iteration overlaps the S/dP MFMAs of tile t with the softmax VALU and transposed LDS reads of
//    tile t-1, and the dV/dK MFMAs of tile t-1 with the row reads of tile t+1.
//  * the dK/dV workgroup loops over every query head of its kv-head group, so GQA needs no fp32
//    partials and no reduction kernel; blocks are ordered kv-head-fastest (an XCD per kv head at
//    Hkv = 8), heaviest key blocks first.
// Per-row constants, packed per 32-row tile for the DMA:
//   ld[((b*Hq + h)*nT + t)*128 + {0..31: -lse/scale | 32..63: -delta | 64..95: segment id |
//                                  96..127: -lse*log2(e)}]
constexpr int kLdTile = 128;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// LDS-DMA issued from inline asm: hipcc cannot see these as LDS writes, so it does not put a
// `vmcnt(0)` in front of every ds_read that follows one (it did with the builtin form, draining the
// ring each iteration); the ring's counted waits below are the only synchronisation.
struct Rsrc {
  u32x4 w;
};
__device__ __forceinline__ Rsrc make_rsrc4(const void* base, int64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  Rsrc r;
  r.w[0] = (uint32_t)p;
  r.w[1] = (uint32_t)(p >> 32) & 0xffffu;
  r.w[2] = (uint32_t)(bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes);
  r.w[3] = 0x00020000u;
  return r;
}
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)(lds_ptr_t)(const_cast<char*>(p));
}
__device__ __forceinline__ void dma16(const Rsrc& r, const char* lds, int voff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(lds_addr(lds)), "v"(voff), "s"(r.w) : "memory");
}
__device__ __forceinline__ void dma4(const Rsrc& r, const char* lds, int voff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(lds_addr(lds)), "v"(voff), "s"(r.w) : "memory");
}
// the five LDS-DMAs of one dK/dV ring tile (Q rows x2, dO rows x2, row constants) in one statement: M0 is
// saved and restored once instead of around every load
__device__ __forceinline__ void dma_tile5(const Rsrc& q, const Rsrc& d, const Rsrc& l, const char* lq0,
                                          const char* lq1, const char* ld0, const char* ld1, const char* ll,
                                          int vq0, int vq1, int vd0, int vd1, int vl) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %6, %11, 0 offen lds\n\t"
      "s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %7, %11, 0 offen lds\n\t"
      "s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %8, %12, 0 offen lds\n\t"
      "s_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %9, %12, 0 offen lds\n\t"
      "s_mov_b32 m0, %5\n\ts_nop 0\n\tbuffer_load_dword %10, %13, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_addr(lq0)), "s"(lds_addr(lq1)), "s"(lds_addr(ld0)), "s"(lds_addr(ld1)), "s"(lds_addr(ll)), "v"(vq0),
        "v"(vq1), "v"(vd0), "v"(vd1), "v"(vl), "s"(q.w), "s"(d.w), "s"(l.w)
      : "memory");
}
// the nine LDS-DMAs of one K/V ring tile of the forward / dQ kernels (K rows x4, V rows x4, segment ids) in
// one statement, M0 saved once; `lds` = the wave's first K row in the slot, rows 4 apart, V `img` bytes on
__device__ __forceinline__ void dma_tile9(const Rsrc& k, const Rsrc& v, const Rsrc& sg, const char* lds, int img,
                                          const char* lseg, const int (&vk)[4], const int (&vv)[4], int vs) {
  uint32_t keep;
  // (wave-uniform; readfirstlane so hipcc's divergence analysis cannot leave it in a VGPR for the "s" operand)
  const uint32_t l0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %12, 0 offen lds\n\t"
      "s_add_u32 m0, %1, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %7, %13, 0 offen lds\n\t"
      "s_add_u32 m0, %1, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %12, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %8, %13, 0 offen lds\n\t"
      "s_add_u32 m0, %1, 0x800\n\ts_nop 0\n\tbuffer_load_dwordx4 %5, %12, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %9, %13, 0 offen lds\n\t"
      "s_add_u32 m0, %1, 0xc00\n\ts_nop 0\n\tbuffer_load_dwordx4 %6, %12, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %10, %13, 0 offen lds\n\t"
      "s_mov_b32 m0, %15\n\ts_nop 0\n\tbuffer_load_dword %11, %14, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(l0), "s"(img), "v"(vk[0]), "v"(vk[1]), "v"(vk[2]), "v"(vk[3]), "v"(vv[0]), "v"(vv[1]), "v"(vv[2]),
        "v"(vv[3]), "v"(vs), "s"(k.w), "s"(v.w), "s"(sg.w), "s"(__builtin_amdgcn_readfirstlane(lds_addr(lseg)))
      : "memory");
}
// the same with the descriptor forced to SGPRs (a kernel under SGPR pressure may keep it in VGPRs,
// which the asm's "s" operand does not accept)
__device__ __forceinline__ Rsrc sgpr_rsrc(const Rsrc& r) {
  Rsrc o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o.w[i] = __builtin_amdgcn_readfirstlane(r.w[i]);
  return o;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// every wave's LDS reads retired, then a barrier that does NOT drain the DMA ring (no vmcnt(0))
__device__ __forceinline__ void ring_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// the same without the LDS drain, for loops in which every read of the slot the next DMA overwrites has
// already been consumed (so retired) before the barrier in program order, and the only reads still in
// flight are the prefetched rows of a slot the next DMA does not touch
__device__ __forceinline__ void ring_barrier_nodrain() { asm volatile("s_barrier" ::: "memory"); }

// Widened row-per-lane store tail (cdna guide T21). w[g] holds this lane's 4 bf16 of 8-column group g
// of its row: the lower lane half columns 8g..8g+3, the upper half 8g+4..8g+7. One permlane32_swap per
// dword of each group pair (g, g+1) leaves the lower half 16 contiguous bytes of group g and the upper
// half those of group g+1, so a lane issues NG / 2 dwordx4 stores instead of NG dwordx2. Run on every
// lane (a pair's two halves share one row), store where the row exists.
template <int NG>
__device__ __forceinline__ void widen_pairs(uint2 (&w)[NG]) {
#pragma unroll
  for (int g = 0; g < NG; g += 2) {
    const auto sx = __builtin_amdgcn_permlane32_swap(w[g].x, w[g + 1].x, false, false);
    const auto sy = __builtin_amdgcn_permlane32_swap(w[g].y, w[g + 1].y, false, false);
    w[g].x = sx[0];
    w[g + 1].x = sx[1];
    w[g].y = sy[0];
    w[g + 1].y = sy[1];
  }
}
// row = the row's first element + 8 * (lane >> 5) (16-byte aligned)
template <int NG>
__device__ __forceinline__ void store_pairs(bf16* row, const uint2 (&w)[NG]) {
#pragma unroll
  for (int g = 0; g < NG; g += 2) *reinterpret_cast<uint4*>(row + 8 * g) = make_uint4(w[g].x, w[g].y, w[g + 1].x, w[g + 1].y);
}

// ============================================================================ backward dK/dV, v5
// grid: ceil(S/128) * Hkv * B blocks (1-D), 4 waves x 32 keys; query tiles of 32 rows over all q heads of
// the kv group through an NSL-slot LDS-DMA ring. D = 96 (Phi-3) runs the same structure on 256-byte LDS rows:
// the DMA rows read 64 bytes past each 192-byte row (never past the tensor: the descriptors end at the last
// row's D elements) and only the first D / 16 k-steps / D / 32 output tiles are used. The loop is a software
// pipeline for one wave per SIMD (profiles/r4_dkdv_pipeline.md; the earlier un-pipelined kernel and the
// 64-keys-per-wave / hand-allocated variants lost their A/Bs and were removed, profiles/r5_dkdv6.md). Per
// iteration t (one 32-row query tile):
//  * phase A issues the 2*NKK S / dP MFMAs of tile t; in their gaps the Q / dO row fragments of tile t
//    arrive just in time (two k-steps ahead), and the transposed Q^T / dO^T fragments of tile t-1 and the
//    row constants of tile t are read for phase B;
//  * phase B issues the 4*NDT dV / dK MFMAs of tile t-1 (operands P, dS of tile t-1 as bf16) while the
//    softmax of tile t (P = exp2(S*scale*log2e - lse*log2e), dS = P (dP - delta)) runs in their gaps.
// Only the bf16 P / dS operands (16 VGPRs) cross the iteration; the fp32 scores are produced and consumed
// inside one iteration, so they never get parked in accumulator registers (the v3 loop opened every tile
// with 32 serial accumulator reads, and a scores-carrying pipeline had hipcc copy them through AGPRs).
// The MFMAs are inline asm with pinned register files: scores in VGPRs where the softmax reads them, the
// kernel-resident K / V fragments in AGPRs (freeing 64 VGPRs), accumulators dK / dV left to hipcc (AGPRs).
// An asm MFMA's result is read by VALU only in the next phase, behind at least one full MFMA chain.
__device__ __forceinline__ void mfma_v0(f32v16& c, const bfv8& x, const bfv8& y) {  // c (VGPR) = x . y (AGPR)
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(c) : "v"(x), "a"(y));
}
__device__ __forceinline__ void mfma_vv(f32v16& c, const bfv8& x, const bfv8& y) {  // c (VGPR) += x . y (AGPR)
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(x), "a"(y));
}

// P = exp2(x) and dS = P (dP + nd) as single-lane asm (see exp_ds in the dQ kernel)
__device__ __forceinline__ void exp_pds(float x, float dp, float nd, float& p, float& ds) {
  asm("v_exp_f32 %0, %2\n\tv_add_f32 %1, %3, %4\n\tv_mul_f32 %1, %0, %1" : "=&v"(p), "=&v"(ds) : "v"(x), "v"(dp), "v"(nd));
}

// TRJ = 1: the transposed Q^T / dO^T fragments of phase B are read just in time inside phase B (two MFMAs
// ahead; the first two at the end of phase A) instead of all in phase A. With every wave of the CU in the same
// phase (one barrier per tile), phase A carried ~40 KB of LDS reads per wave against 16 MFMAs, more than the
// LDS array serves in their time, while phase B read nothing; split by phase, each fits under its MFMAs.
template <int D, bool OM = false, int NSL = 6, int TRJ = 0>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv5_kernel(AttnArgs a, const float* ld) {
  constexpr int NKK = D / 16, NDT = D / 32;
  // NSL ring slots: tiles issued NSL - 2 ahead, each given NSL - 4 iterations to land
  constexpr int BM = 32, IMG = BM * 256, SLOT = 2 * IMG + 2 * 256, NS = NSL;
  constexpr int NDMA = 5;
  constexpr int NB = 4 * NDT;  // phase-B MFMAs (dV then dK, s2-major)
  using QI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = a.S, grp = a.Hq / a.Hkv;
  int L = (int)blockIdx.x;
  const int hk = L % a.Hkv;
  L /= a.Hkv;
  int b, kb;
  block_of(a, L, (S + 127) / 128, false, b, kb);
  const int ks = kb * 128, kw = ks + wid * 32, kr = kw + r;
  const int nT = (S + 31) / 32;
  const bf16* kp = a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh;
  const bf16* vp = a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh;
  const int sk = (OM && a.seg && kr < S) ? a.seg[(int64_t)b * S + kr] : 0;  // OM: see fa_fwd3_kernel
  int qlo = 0, qhi = -1;
  if (!OM) query_interval(a, b, kr, qlo, qhi);
  const float sl2 = a.scale * kLog2e;

  bfv8 kf[NKK], vf[NKK];
  // the block's K / V rows: loaded after the first ring tiles were issued when a.early (their latencies
  // overlap: one workgroup per CU leaves the prologue exposed), else first
  auto load_kv = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      kf[kk] = gload8(kp + (int64_t)min(kr, S - 1) * a.k_ss + kk * 16 + hh * 8, kr < S);
      vf[kk] = gload8(vp + (int64_t)min(kr, S - 1) * a.v_ss + kk * 16 + hh * 8, kr < S);
    }
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(kf[kk]), "+v"(vf[kk]));
    // move K / V into the accumulator file here, with the VALU-write -> MFMA-read wait states behind them
    // (the asm MFMAs that read them are invisible to the hazard recognizer)
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+a"(kf[kk]), "+a"(vf[kk]));
    asm volatile("s_nop 7");
  };
  if (!a.early) load_kv();
  f32v16 dkt[NDT], dvt[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      dkt[dt][i] = 0.f;
      dvt[dt][i] = 0.f;
    }

  const RunInfo kr_run = block_run(a, b, min(ks, S - 1), min(ks + 127, S - 1));
  const int q_beg = a.causal ? ks : max(0, kr_run.rs) / 32 * 32;
  int q_end = a.window >= 0 ? min(S, ks + 128 + a.window) : S;
  if (a.rs) q_end = min(q_end, a.re[(int64_t)b * S + min(ks + 127, S - 1)] + 1);
  const int nq = q_end > q_beg ? (q_end - q_beg + BM - 1) / BM : 0;
  const int T = FA_PROBE(a, 8) ? 0 : nq * grp;

  if (T > 0) {
    int dq_off[2], dd_off[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int row = 8 * wid + 4 * n + (lane >> 4);
      const int ch = (lane & 15) ^ QI::swz(row);
      dq_off[n] = (row * a.q_ss + ch * 8) * 2;
      dd_off[n] = (row * a.d_ss + ch * 8) * 2;
    }
    const int ld_off = ((wid & 1) * 64 + lane) * 4;
    asm volatile("" : "+v"(dq_off[0]), "+v"(dq_off[1]), "+v"(dd_off[0]), "+v"(dd_off[1]));
    const int64_t q_rows = S - q_beg;
    const int64_t nrec_q = ((q_rows - 1) * a.q_ss + D) * 2, nrec_d = ((q_rows - 1) * a.d_ss + D) * 2;
    const int64_t nrec_l = (int64_t)nq * kLdTile * 4;
    const bf16* qh0 = a.q + (int64_t)b * a.q_sb + (int64_t)(hk * grp) * a.q_sh + (int64_t)q_beg * a.q_ss;
    const bf16* dh0 = a.dout + (int64_t)b * a.d_sb + (int64_t)(hk * grp) * a.d_sh + (int64_t)q_beg * a.d_ss;
    const float* lh0 = ld + (((int64_t)b * a.Hq + hk * grp) * nT + (q_beg >> 5)) * kLdTile;
    const int step_q = BM * a.q_ss * 2, step_d = BM * a.d_ss * 2;
    Rsrc qrs = make_rsrc4(qh0, nrec_q), drs = make_rsrc4(dh0, nrec_d), lrs = make_rsrc4(lh0, nrec_l);
    int iss_g = 0, iss_q = 0, iss_n = 0, toff_q = 0, toff_d = 0, toff_l = 0;
    auto advance = [&]() {  // offsets (and head descriptors) of the next tile in load order
      if (++iss_n < T) {
        toff_q += step_q;
        toff_d += step_d;
        toff_l += kLdTile * 4;
        if (++iss_q == nq) {
          iss_q = 0;
          ++iss_g;
          toff_q = toff_d = toff_l = 0;
          qrs = make_rsrc4(qh0 + (int64_t)iss_g * a.q_sh, nrec_q);
          drs = make_rsrc4(dh0 + (int64_t)iss_g * a.d_sh, nrec_d);
          lrs = make_rsrc4(lh0 + (int64_t)iss_g * nT * kLdTile, nrec_l);
        }
      }
    };
    auto issue = [&](const char* slot) {
      const char* q0 = slot + 8 * wid * 256;
      dma_tile5(qrs, drs, lrs, q0, q0 + 4 * 256, q0 + IMG, q0 + IMG + 4 * 256, slot + 2 * IMG + (wid & 1) * 256,
                dq_off[0] + toff_q, dq_off[1] + toff_q, dd_off[0] + toff_d, dd_off[1] + toff_d, ld_off + toff_l);
      advance();
    };
    int cur_q = 0;
    const bool seg_or_window = a.seg != nullptr || a.window >= 0;
    struct TileMask {
      int q0;
      bool need, m_seg;
    };
    auto tile_mask = [&]() {
      TileMask m;
      m.q0 = q_beg + cur_q * BM;
      m.need = a.causal && kw + 31 > m.q0;
      m.m_seg = false;
      if (seg_or_window) {
        m.m_seg = seg_mask(a, kr_run, m.q0, m.q0 + 31);
        m.need = m.need || m.m_seg || (a.window >= 0 && m.q0 + 31 - a.window > kw);
      }
      if (++cur_q == nq) cur_q = 0;
      return m;
    };
    int ro[NKK], to[NDT][2];
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) ro[kk] = QI::roff(r, 2 * kk + hh);
    {
      const int g = lane >> 4, i16 = lane & 15;
      const int row = 4 * (g >> 1) + (i16 >> 2), col = 16 * (g & 1) + 4 * (i16 & 3);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        to[dt][0] = QI::toff(BM, row, dt * 32 + col);
        to[dt][1] = QI::toff(BM, row + 8, dt * 32 + col);
      }
    }
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(ro[kk]));
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) asm volatile("" : "+v"(to[dt][0]), "+v"(to[dt][1]));

    // transposed fragment i of phase B: i < 2*NDT -> dO^T (dV product), else Q^T (dK product);
    // s2 = (i / NDT) & 1, dt = i % NDT
    auto trf = [&](const char* slot, int i) -> bfv8 {
      const int s2 = (i / NDT) & 1, dt = i % NDT;
      const char* base = slot + (i < 2 * NDT ? IMG : 0) + 4096 * s2;
      const s16v4 lo = lds_tr(base + to[dt][0]), hi = lds_tr(base + to[dt][1]);
      return __builtin_bit_cast(bfv8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    // S / dP of the tile in `cs` (first two k-steps prefetched in qa / da); with `ps` != null the
    // transposed fragments of the previous tile are read into tf in the MFMA gaps
    auto phase_a = [&](auto with_tr, const char* cs, const char* ps, bfv8 (&qa)[2], bfv8 (&da)[2], f32v16& sc,
                       f32v16& dc, bfv8 (&tf)[NB], float (&lq)[16], float (&nd)[16]) {
      bfv8 qf[NKK], df[NKK];
      qf[0] = qa[0]; df[0] = da[0]; qf[1] = qa[1]; df[1] = da[1];
      const float* Ls = reinterpret_cast<const float*>(cs + 2 * IMG);
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        if (kk + 2 < NKK) {
          qf[kk + 2] = lds_b128(cs + ro[kk + 2]);
          df[kk + 2] = lds_b128(cs + ro[kk + 2] + IMG);
        }
        // row constants of this tile (-lse*log2e at floats 96.., -delta at 32..), one 16-byte read per k-step
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if ((2 * c) * NKK / 8 == kk) {
            const float4 l4 = *reinterpret_cast<const float4*>(Ls + 96 + 8 * c + 4 * hh);
            lq[4 * c] = l4.x; lq[4 * c + 1] = l4.y; lq[4 * c + 2] = l4.z; lq[4 * c + 3] = l4.w;
          }
          if ((2 * c + 1) * NKK / 8 == kk) {
            const float4 d4 = *reinterpret_cast<const float4*>(Ls + 32 + 8 * c + 4 * hh);
            nd[4 * c] = d4.x; nd[4 * c + 1] = d4.y; nd[4 * c + 2] = d4.z; nd[4 * c + 3] = d4.w;
          }
        }
        if constexpr (decltype(with_tr)::value && TRJ == 0) {
#pragma unroll
          for (int i = kk * NB / NKK; i < (kk + 1) * NB / NKK; ++i) tf[i] = trf(ps, i);
        }
        if constexpr (decltype(with_tr)::value && TRJ == 1) {
          if (kk >= NKK - 2) tf[kk - (NKK - 2)] = trf(ps, kk - (NKK - 2));
        }
        if (kk == 0) {
          mfma_v0(sc, qf[0], kf[0]);
          mfma_v0(dc, df[0], vf[0]);
        } else {
          mfma_vv(sc, qf[kk], kf[kk]);
          mfma_vv(dc, df[kk], vf[kk]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // hipcc's hazard recognizer does not see the asm MFMAs: the XDL-write -> VALU read / write wait states
      // (8-pass 32x32x16: 11, +1 on gfx950) before the mask / softmax touch the scores, with margin
      asm volatile("s_nop 7\n\ts_nop 7");
      __builtin_amdgcn_sched_barrier(0);
    };
    // masked elements (diagonal / window / packed tiles only) get S = -inf, so P = exp2(-inf) = 0 (the row
    // constant is never +inf: rows past S or without keys carry -inf)
    auto apply_mask = [&](const char* cs, const TileMask& m, f32v16& sc) {
      if constexpr (!OM) {
        const IdxRange rg = idx_range(qlo, qhi, m.q0 + 4 * hh);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (!in_range(rg, 8 * (i >> 2) + (i & 3))) sc[i] = -INFINITY;
        return;
      }
      const int* Sg = reinterpret_cast<const int*>(cs + 2 * IMG) + 64;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        int4 s4 = make_int4(sk, sk, sk, sk);
        if (m.m_seg) s4 = *reinterpret_cast<const int4*>(Sg + 8 * c + 4 * hh);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qi = m.q0 + 8 * c + 4 * hh + j;
          bool o = true;
          if (a.causal) o = o && (kr <= qi);
          if (a.window >= 0) o = o && (qi - kr <= a.window);
          if (m.m_seg) o = o && ((&s4.x)[j] == sk);
          if (!o) sc[4 * c + j] = -INFINITY;
        }
      }
    };
    // softmax element v of a tile into the bf16 operands pn / dn
    auto smx = [&](int v, const f32v16& sc, const f32v16& dc, const float (&lq)[16], const float (&nd)[16],
                   bfv8 (&pn)[2], bfv8 (&dn)[2]) {
      // single-lane asm: with plain C++ hipcc paired neighbouring elements into v_pk_add_f32 / v_pk_mul_f32
      // and padded the phase with 16 s_nop; this form took the B4 S8192 backward from 7.996 to 7.545 ms in
      // one process, bitwise-equal gradients
      float p, ds;
      exp_pds(fmaf(sc[v], sl2, lq[v]), dc[v], nd[v], p, ds);
      pn[v >> 3][v & 7] = (__bf16)p;
      dn[v >> 3][v & 7] = (__bf16)ds;
    };
    // dV / dK of the previous tile (operands po / dso, fragments tf) || softmax of this tile into pn / dsn;
    // with `ns` the first two k-steps of the next tile's rows are read at the end
    auto phase_b = [&](auto smax, const bfv8 (&po)[2], const bfv8 (&dso)[2], bfv8 (&tf)[NB],
                       const f32v16& sc, const f32v16& dc, const float (&lq)[16], const float (&nd)[16],
                       bfv8 (&pn)[2], bfv8 (&dsn)[2], const char* ns, bfv8 (&qa)[2], bfv8 (&da)[2], const char* ps) {
      constexpr bool SMAX = decltype(smax)::value;  // softmax of a next tile (and its rows) to interleave
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        if constexpr (TRJ == 1) {
          if (i + 2 < NB) tf[i + 2] = trf(ps, i + 2);
        }
        const int s2 = (i / NDT) & 1, dt = i % NDT;
        if (i < 2 * NDT)
          dvt[dt] = mfma32(tf[i], po[s2], dvt[dt]);
        else
          dkt[dt] = mfma32(tf[i], dso[s2], dkt[dt]);
        if constexpr (SMAX) {
#pragma unroll
          for (int v = i * 16 / NB; v < (i + 1) * 16 / NB; ++v) smx(v, sc, dc, lq, nd, pn, dsn);
        }
        if (SMAX && i == NB - 3) {
          qa[0] = lds_b128(ns + ro[0]);
          da[0] = lds_b128(ns + ro[0] + IMG);
          qa[1] = lds_b128(ns + ro[1]);
          da[1] = lds_b128(ns + ro[1] + IMG);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    int sl_m2 = (NS - 1) * SLOT, sl_m1 = 0, sl_0 = SLOT, sl_p1 = 2 * SLOT;
    // early: the tiles the first wait covers, then the rows (hipcc's wait for its own younger loads covers
    // those tiles too: loads retire in order), then the rest of the ring
#pragma unroll
    for (int t = 0; t < 3; ++t) issue(smem + t * SLOT);
    if (a.early) load_kv();
#pragma unroll
    for (int t = 3; t < NS - 1; ++t) issue(smem + t * SLOT);
    static_assert(NS - 1 - (NS - 4) == 3, "first wait covers three tiles");
    wait_vm<NDMA * (NS - 4)>();
    ring_barrier();

    bfv8 qa[2], da[2], pb[2], db[2];
    bfv8 tf[NB];
    float lq[16], nd[16];
    {  // tile 0: S / dP and its softmax
      qa[0] = lds_b128(smem + ro[0]);
      da[0] = lds_b128(smem + ro[0] + IMG);
      qa[1] = lds_b128(smem + ro[1]);
      da[1] = lds_b128(smem + ro[1] + IMG);
      f32v16 sc, dc;
      const TileMask m0 = tile_mask();
      phase_a(std::false_type{}, smem, smem, qa, da, sc, dc, tf, lq, nd);
      if (m0.need) apply_mask(smem, m0, sc);
#pragma unroll
      for (int v = 0; v < 16; ++v) smx(v, sc, dc, lq, nd, pb, db);
      qa[0] = lds_b128(smem + SLOT + ro[0]);
      da[0] = lds_b128(smem + SLOT + ro[0] + IMG);
      qa[1] = lds_b128(smem + SLOT + ro[1]);
      da[1] = lds_b128(smem + SLOT + ro[1] + IMG);
    }
    for (int t = 1; t < T; ++t) {
      issue(smem + sl_m2);
      const TileMask mcur = tile_mask();
      f32v16 sc, dc;
      phase_a(std::true_type{}, smem + sl_0, smem + sl_m1, qa, da, sc, dc, tf, lq, nd);
      if (mcur.need) apply_mask(smem + sl_0, mcur, sc);
      bfv8 pn[2], dsn[2];
      phase_b(std::true_type{}, pb, db, tf, sc, dc, lq, nd, pn, dsn, smem + sl_p1, qa, da, smem + sl_m1);
      pb[0] = pn[0]; pb[1] = pn[1]; db[0] = dsn[0]; db[1] = dsn[1];
      sl_m2 = sl_m1;
      sl_m1 = sl_0;
      sl_0 = sl_p1;
      sl_p1 = (sl_p1 + SLOT == NS * SLOT) ? 0 : sl_p1 + SLOT;
      wait_vm<NDMA * (NS - 4)>();
      ring_barrier_nodrain();
    }
    {  // dV / dK of the last tile
#pragma unroll
      for (int i = 0; i < (TRJ == 1 ? 2 : NB); ++i) tf[i] = trf(smem + sl_m1, i);
      f32v16 z = {};
      bfv8 pn[2], dsn[2];
      phase_b(std::false_type{}, pb, db, tf, z, z, lq, nd, pn, dsn, smem, qa, da, smem + sl_m1);
    }
    wait_vm<0>();  // no LDS-DMA may outlive the workgroup
  }

  if (a.rope_dk && kr < S) {  // fused RoPE: gradient of the unrotated k
    const int p = rope_pos(a, b, kr);
    rope_acc_inv<D>(dkt, a.rcos + (int64_t)p * (D / 2), a.rsin + (int64_t)p * (D / 2), hh);
  }
  uint2 wk[4 * NDT], wv[4 * NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int g = 4 * dt + c;
      wk[g].x = pack_bf16x2(dkt[dt][4 * c] * a.scale, dkt[dt][4 * c + 1] * a.scale);
      wk[g].y = pack_bf16x2(dkt[dt][4 * c + 2] * a.scale, dkt[dt][4 * c + 3] * a.scale);
      wv[g].x = pack_bf16x2(dvt[dt][4 * c], dvt[dt][4 * c + 1]);
      wv[g].y = pack_bf16x2(dvt[dt][4 * c + 2], dvt[dt][4 * c + 3]);
    }
  widen_pairs(wk);
  widen_pairs(wv);
  if (kr < S) {
    store_pairs(a.dk + (int64_t)b * a.dk_sb + (int64_t)kr * a.dk_ss + (int64_t)hk * a.dk_sh + 8 * hh, wk);
    store_pairs(a.dv + (int64_t)b * a.dv_sb + (int64_t)kr * a.dv_ss + (int64_t)hk * a.dv_sh + 8 * hh, wv);
  }
}

// ============================================================================ forward, D = 128, v3
// grid: ceil(S/128) * Hq * B blocks (1-D, kv-head-major, heaviest query blocks first), 4 waves x 32
// queries, two workgroups per CU. Differences from fa_fwd_kernel<128>, each aimed at the exposed LDS
// latency that capped it near 600 TF/s (its ISA waited on every K read one MFMA ahead):
//  * K / V tiles arrive by LDS-DMA (no staging registers) into a 2-slot ring of dual-use swizzled
//    images; the DMA of tile t+1 flies under tile t's compute, one raw barrier per tile.
//  * all 16 K row fragments of a tile are read in one batch ahead of the 16 S^T MFMAs, and the 32
//    V^T transposed reads are issued right behind those MFMAs (into the same registers) so they land
//    while the softmax runs; the P.V MFMAs then run back to back.
//  * the softmax works on raw scores: row max first, then p = exp2(fma(s, scale*log2e, -m)) — one
//    FMA + one exp per score instead of mul + sub + exp.
// single-instruction VALU helpers for MFMA-output math: plain fmaxf makes hipcc canonicalise each MFMA
// result with an extra v_max first, and adjacent f32 adds get SLP-packed into v_pk_add_f32 (slower
// than two v_add_f32 beside MFMAs, cdna guide T12 / cycle constants)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// The leading s_nop is the trans-use wait state: its inputs are v_exp_f32 results, and hipcc's hazard
// recognizer does not look inside inline asm. Without it the D=96 instantiation (which schedules an
// add right behind the exp that produces its operand) read stale values in 4 of every 8 lanes and
// lost terms of the softmax row sum.
__device__ __forceinline__ float vadd(float a, float b) {
  float r;
  asm("s_nop 0\n\tv_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// DMA of one 64-key K/V tile (+ its 64 segment ids) of the query-parallel kernels into ring slot `slot`:
// with NW = 4 waves each wave fetches 16 K and 16 V rows (4 + 4 one-KB pieces), with NW = 8 eight of each
// (2 + 2); every wave also fetches the segment ids (the same 256 bytes)
template <int NW>
__device__ __forceinline__ void kv_tile_dma(const char* slot, int n0, int wid, int lane, const AttnArgs& a,
                                            const Rsrc& krs, const Rsrc& vrs, const Rsrc& srs) {
  constexpr int IMG = 64 * 256;
  using KI = Img<128>;
  constexpr int RPW = 64 / NW;  // rows per wave
  int vk[RPW / 4], vv[RPW / 4];
#pragma unroll
  for (int n = 0; n < RPW / 4; ++n) {
    const int row = RPW * wid + 4 * n + (lane >> 4);
    const int ch = (lane & 15) ^ KI::swz(row);
    vk[n] = ((n0 + row) * a.k_ss + ch * 8) * 2;
    vv[n] = ((n0 + row) * a.v_ss + ch * 8) * 2;
  }
  const char* k0 = slot + RPW * wid * 256;
  if constexpr (NW == 4)
    dma_tile9(krs, vrs, srs, k0, IMG, slot + 2 * IMG, vk, vv, (n0 + lane) * 4);
  else
    dma_tile5(krs, vrs, srs, k0, k0 + 4 * 256, k0 + IMG, k0 + IMG + 4 * 256, slot + 2 * IMG, vk[0], vk[1], vv[0], vv[1],
              (n0 + lane) * 4);
}

// NW = 8: two query heads of one kv group per workgroup, side by side (waves 0-3 head h, waves 4-7 head
// h + 1, 32 queries each): every K/V tile of the LDS-DMA ring then serves 256 query rows instead of 128,
// crossing L2 -> LDS half as often, and each wave issues half the DMA pieces (2 K + 2 V rows groups).
template <int D, int RS = 0, int WS = 0, int NW = 4, bool OM = false>
__global__ __launch_bounds__(NW * 64, 2) void fa_fwd3_kernel(AttnArgs a) {
  constexpr int NKK = D / 16, NDT = D / 32;  // k-steps of a D-deep product, 32-wide output tiles
  constexpr int BN = 64, IMG = BN * 256, SLOT = 2 * IMG + 256;
  using KI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), wq = wid & 3;
  const int S = a.S, grp = a.Hq / a.Hkv;
  const int nqb = (S + 127) / 128;
  int L = (int)blockIdx.x;
  const int hk = L % a.Hkv;
  L /= a.Hkv;
  const int hpb = NW / 4;  // query heads per workgroup
  const int h = hk * grp + (L % (grp / hpb)) * hpb + (wid >> 2);
  L /= grp / hpb;
  int b, mb;
  block_of(a, L, nqb, true, b, mb);
  const int qs = mb * 128, qw = qs + wq * 32, qrow = qw + r;
  const bf16* qp = a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh;
  const float sl2 = a.scale * kLog2e;
  // OM: the per-element segment-id compares (A/B reference; rows without run bounds); else range masks
  int sq = (OM && a.seg && qrow < S) ? a.seg[(int64_t)b * S + qrow] : -2;
  int klo = 0, khi = -1;
  if (!OM) key_interval(a, b, qrow, klo, khi);

  const RunInfo qr = block_run(a, b, qs, min(qs + 127, S - 1));
  int kv_end = a.causal ? min(S, qs + 128) : S;
  if (!a.causal && a.rs) kv_end = min(kv_end, a.re[(int64_t)b * S + min(qs + 127, S - 1)] + 1);
  int kv_beg = a.window >= 0 ? max(0, qs - a.window) : 0;
  kv_beg = max(kv_beg, qr.rs) / BN * BN;
  const int T = (kv_end > kv_beg && !FA_PROBE(a, 1)) ? (kv_end - kv_beg + BN - 1) / BN : 0;
  // records end with the last row's D elements: the 256-byte DMA rows of D < 128 read past a row,
  // and past the tensor on the last row of the last head -> zeros instead of a fault
  const Rsrc krs = make_rsrc4(a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh, ((int64_t)(S - 1) * a.k_ss + D) * 2);
  const Rsrc vrs = make_rsrc4(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh, ((int64_t)(S - 1) * a.v_ss + D) * 2);
  const Rsrc srs = make_rsrc4(a.seg ? a.seg + (int64_t)b * S : nullptr, a.seg ? (int64_t)S * 4 : 0);
  auto issue = [&](int t) { kv_tile_dma<NW>(smem + __builtin_amdgcn_readfirstlane((t & 1) * SLOT), kv_beg + t * BN, wid,
                                            lane, a, krs, vrs, srs); };
  // early: tile 0 is in flight while the Q rows load (hipcc's waits for its own, younger loads then cover
  // it too: loads retire in order)
  if (a.early && T > 0) issue(0);

  bfv8 qf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk)
    qf[kk] = gload8(qp + (int64_t)min(qrow, S - 1) * a.q_ss + kk * 16 + hh * 8, qrow < S && !FA_PROBE(a, 2));
  if (a.rope_q && qrow < S) {  // fused RoPE: the rows arrive unrotated
    const int p = rope_pos(a, b, qrow);
    rope_frags<NKK>(qf, a.rcos + (int64_t)p * (D / 2), a.rsin + (int64_t)p * (D / 2), hh);
  }
  // hipcc does not count the asm DMAs: retire its own loads before the first one is issued
  asm volatile("" : "+v"(sq), "+v"(klo), "+v"(khi));
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(qf[kk]));
  f32v16 ot[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) ot[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;  // running max in scaled log2 units

  if (T > 0) {
    // loop-invariant LDS offsets: K row reads (two 32-key halves) and V^T transposed reads
    int ro[NKK], to[NDT][2];
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) ro[kk] = KI::roff(r, 2 * kk + hh);
    {
      const int g = lane >> 4, i16 = lane & 15;
      const int row = 4 * (g >> 1) + (i16 >> 2), col = 16 * (g & 1) + 4 * (i16 & 3);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        to[dt][0] = KI::toff(BN, row, dt * 32 + col);
        to[dt][1] = KI::toff(BN, row + 8, dt * 32 + col);
      }
    }

    if (!a.early) issue(0);
    wait_vm<0>();
    ring_barrier();
    // the tile loop unrolled by the ring's two slots: each slot's LDS offsets are compile-time constants
    // (folded into the ds_read offset fields instead of one v_add per read and tile)
    auto tile = [&](auto sidx, int t) {
      const char* slot = smem + decltype(sidx)::value * SLOT;
      const int n0 = kv_beg + t * BN;
      if (t + 1 < T) issue(t + 1);
      bfv8 fr[16];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) fr[8 * tt + kk] = lds_b128(slot + 8192 * tt + ro[kk]);
      __builtin_amdgcn_sched_barrier(0);  // keep the batch: one LDS latency per tile, not per MFMA
      f32v16 st[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) st[tt][i] = 0.f;
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) st[tt] = mfma32(fr[8 * tt + kk], qf[kk], st[tt]);
      }
      // V^T operands of the P.V product (keys 32tt + 16s2 .., columns 32dt ..) into the same registers
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const char* base = slot + IMG + 256 * (32 * tt + 16 * s2);
            const s16v4 lo = lds_tr(base + to[dt][0]), hi = lds_tr(base + to[dt][1]);
            fr[8 * tt + 4 * s2 + dt] = __builtin_bit_cast(bfv8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
      __builtin_amdgcn_sched_barrier(0);
      // masking only where needed: diagonal (causal), window edge, sequence end, packed segments
      const bool m_causal = a.causal && (n0 + BN - 1 > qw);
      const bool m_window = a.window >= 0 && (n0 < qw + 31 - a.window);
      const bool m_end = n0 + BN > S;
      const bool m_seg = seg_mask(a, qr, n0, n0 + BN - 1);
      if ((m_causal || m_window || m_end || m_seg || qw + 31 >= S) && !OM) {
        const IdxRange rg = idx_range(klo, khi, n0 + 4 * hh);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (!in_range(rg, 32 * tt + 8 * c + j)) st[tt][4 * c + j] = -INFINITY;
      } else if (OM && (m_causal || m_window || m_end || m_seg || qw + 31 >= S)) {
        const int* Ss = reinterpret_cast<const int*>(slot + 2 * IMG);
        const int lim = qrow - n0 - 4 * hh, lo = qrow - a.window - n0 - 4 * hh, hi = S - 1 - n0 - 4 * hh;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            int4 sk = make_int4(sq, sq, sq, sq);
            if (m_seg) sk = *reinterpret_cast<const int4*>(Ss + 32 * tt + 8 * c + 4 * hh);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int ko = 32 * tt + 8 * c + j;
              bool ok = (ko <= hi) && (qrow < S);
              if (a.causal) ok = ok && (ko <= lim);
              if (a.window >= 0) ok = ok && (ko >= lo);
              if (m_seg) ok = ok && ((&sk.x)[j] == sq);
              if (!ok) st[tt][4 * c + j] = -INFINITY;
            }
          }
      }
      float mx0 = vmax3(st[0][0], st[0][1], st[0][2]), mx1 = vmax3(st[1][0], st[1][1], st[1][2]);
#pragma unroll
      for (int i = 3; i < 15; i += 2) {
        mx0 = vmax3(mx0, st[0][i], st[0][i + 1]);
        mx1 = vmax3(mx1, st[1][i], st[1][i + 1]);
      }
      float smax = vmax3(mx0, st[0][15], vmax3(mx1, st[1][15], mx1));
      if constexpr (RS == 2) {  // the two half-waves' maxima through one permlane32 swap (no LDS round trip)
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(smax), __float_as_uint(smax), false, false);
        smax = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * sl2;
      } else {
        smax = fmaxf(smax, __shfl_xor(smax, 32, 64)) * sl2;
      }
      // deferred rescale: keep the running max unless some row grew by more than kThr
      if (__any(smax > m + kThr)) {
        const float mnew = fmaxf(m, smax);
        const float alpha = (mnew == -INFINITY) ? 1.f : fexp2(m - mnew);
        m = mnew;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) ot[dt][i] *= alpha;
      }
      const float nm = (m == -INFINITY) ? 0.f : -m;
      float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          if constexpr (RS == 2) {
            // exp pair + row-sum adds in one asm block: each add sits one instruction behind the exp it reads
            // (the trans-use wait state, by placement instead of an s_nop), and hipcc cannot pair the adds
            // into v_pk_add_f32 (an anti-lever beside MFMAs, cdna guide cycle constants)
            const float x0 = fmaf(st[tt][i], sl2, nm), x1 = fmaf(st[tt][i + 1], sl2, nm);
            float e0, e1;
            asm("v_exp_f32 %0, %4\n\tv_exp_f32 %1, %5\n\tv_add_f32 %2, %2, %0\n\tv_add_f32 %3, %3, %1"
                : "=&v"(e0), "=&v"(e1), "+v"(rs0), "+v"(rs1)
                : "v"(x0), "v"(x1));
            st[tt][i] = e0;
            st[tt][i + 1] = e1;
            continue;
          }
          st[tt][i] = fexp2(fmaf(st[tt][i], sl2, nm));
          st[tt][i + 1] = fexp2(fmaf(st[tt][i + 1], sl2, nm));
          if constexpr (RS == 0) {
            rs0 = vadd(rs0, st[tt][i]);
            rs1 = vadd(rs1, st[tt][i + 1]);
          } else {  // plain adds: the compiler places the trans-use wait states (and may pack the pair)
            rs0 += st[tt][i];
            rs1 += st[tt][i + 1];
          }
        }
      l += rs0 + rs1;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bfv8 pb = acc_as_b(st[tt], s2);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) ot[dt] = mfma32(fr[8 * tt + 4 * s2 + dt], pb, ot[dt]);
        }
      __builtin_amdgcn_sched_barrier(0);  // the P.V work stays ahead of the wait: the DMA flies under it
      wait_vm<0>();  // this wave's DMA of tile t + 1
      ring_barrier();
        };
    for (int t = 0; t < T; t += 2) {
      tile(std::integral_constant<int, 0>{}, t);
      if (t + 1 < T) tile(std::integral_constant<int, 1>{}, t + 1);
    }
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if constexpr (WS) {
    uint2 w[4 * NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        w[4 * dt + c].x = pack_bf16x2(ot[dt][4 * c] * inv, ot[dt][4 * c + 1] * inv);
        w[4 * dt + c].y = pack_bf16x2(ot[dt][4 * c + 2] * inv, ot[dt][4 * c + 3] * inv);
      }
    widen_pairs(w);
    if (qrow < S && !FA_PROBE(a, 4)) store_pairs(a.out + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * a.o_sh + 8 * hh, w);
  }
  if (qrow < S && !FA_PROBE(a, 4)) {
    if constexpr (!WS) {
      bf16* op = a.out + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * a.o_sh;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint2 w;
          w.x = pack_bf16x2(ot[dt][4 * c] * inv, ot[dt][4 * c + 1] * inv);
          w.y = pack_bf16x2(ot[dt][4 * c + 2] * inv, ot[dt][4 * c + 3] * inv);
          *reinterpret_cast<uint2*>(op + dt * 32 + 8 * c + 4 * hh) = w;
        }
    }
    if (hh == 0) {
      const float mu = (m == -INFINITY) ? 0.f : m;
      a.lse[((int64_t)b * a.Hq + h) * S + qrow] = lt > 0.f ? (mu + __log2f(lt)) * kLn2 : -INFINITY;
    }
  }
}

// ============================================================================ backward dQ, D = 128, v3
// The forward v3 structure applied to the query-parallel dQ pass (grid, block order, K/V LDS-DMA ring,
// two workgroups per CU): per 32-key half of a 64-key tile, batched K row reads -> S^T = K.Q^T, batched
// V row reads -> dP^T = V.dO^T, dS = P (dP - delta) with P = exp2(S * scale * log2e - lse * log2e)
// (the forward's LSE: no online max), then batched K^T transposed reads -> dQ^T += K^T . dS^T.
// dQ = scale * sum; the row constants come straight from lse / delta. delta = rowsum(O * dO) is computed
// here from the wave's own O and dO rows (and written, with -lse/scale, the segment ids and -lse*log2e, as
// the ld tiles the dK/dV kernel reads next).
// NW = 8: two query heads of one kv group per workgroup sharing the K/V ring (as fa_fwd3_kernel)
// dS = P (dP - delta) with P = exp2(x): the exp, the subtraction and the product as three single-lane VALU
// instructions in one asm block (the product reads the exp result one instruction later: its trans-use wait
// state), so hipcc cannot pair neighbouring elements into v_pk_add_f32 / v_pk_mul_f32 beside the MFMAs
__device__ __forceinline__ float exp_ds(float x, float dp, float dlt) {
  float p, t;
  asm("v_exp_f32 %0, %2\n\tv_sub_f32 %1, %3, %4\n\tv_mul_f32 %0, %0, %1" : "=&v"(p), "=&v"(t) : "v"(x), "v"(dp), "v"(dlt));
  return p;
}

template <int D, bool IL = true, bool WS = false, int NW = 4, bool OM = false, bool XS = true>
__global__ __launch_bounds__(NW * 64, 2) void fa_bwd_dq3_kernel(AttnArgs a) {
  constexpr int NKK = D / 16, NDT = D / 32;
  constexpr int BN = 64, IMG = BN * 256, SLOT = 2 * IMG + 256;
  using KI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6), wq = wid & 3;
  const int S = a.S, grp = a.Hq / a.Hkv;
  const int nqb = (S + 127) / 128;
  int L = (int)blockIdx.x;
  const int hk = L % a.Hkv;
  L /= a.Hkv;
  const int hpb = NW / 4;  // query heads per workgroup
  const int h = hk * grp + (L % (grp / hpb)) * hpb + (wid >> 2);
  L /= grp / hpb;
  int b, mb;
  block_of(a, L, nqb, true, b, mb);
  const int qs = mb * 128, qw = qs + wq * 32, qrow = qw + r;
  const bf16* qp = a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh;
  const bf16* dop = a.dout + (int64_t)b * a.d_sb + (int64_t)h * a.d_sh;
  const float sl2 = a.scale * kLog2e;
  const int64_t lrow = ((int64_t)b * a.Hq + h) * S + min(qrow, S - 1);
  float lse2 = qrow < S ? a.lse[lrow] * kLog2e : INFINITY;
  float dlt = (qrow < S && !a.ldw) ? a.delta[lrow] : 0.f;
  int sq = (OM && a.seg && qrow < S) ? a.seg[(int64_t)b * S + qrow] : -2;  // OM: see fa_fwd3_kernel
  int klo = 0, khi = -1;
  if (!OM) key_interval(a, b, qrow, klo, khi);

  const RunInfo qr = block_run(a, b, qs, min(qs + 127, S - 1));
  int kv_end = a.causal ? min(S, qs + 128) : S;
  if (!a.causal && a.rs) kv_end = min(kv_end, a.re[(int64_t)b * S + min(qs + 127, S - 1)] + 1);
  int kv_beg = a.window >= 0 ? max(0, qs - a.window) : 0;
  kv_beg = max(kv_beg, qr.rs) / BN * BN;
  const int T = (kv_end > kv_beg && !FA_PROBE(a, 8)) ? (kv_end - kv_beg + BN - 1) / BN : 0;
  // records end with the last row's D elements: the 256-byte DMA rows of D < 128 read past a row,
  // and past the tensor on the last row of the last head -> zeros instead of a fault
  const Rsrc krs = make_rsrc4(a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh, ((int64_t)(S - 1) * a.k_ss + D) * 2);
  const Rsrc vrs = make_rsrc4(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh, ((int64_t)(S - 1) * a.v_ss + D) * 2);
  const Rsrc srs = make_rsrc4(a.seg ? a.seg + (int64_t)b * S : nullptr, a.seg ? (int64_t)S * 4 : 0);
  auto issue = [&](int t) { kv_tile_dma<NW>(smem + __builtin_amdgcn_readfirstlane((t & 1) * SLOT), kv_beg + t * BN, wid,
                                            lane, a, krs, vrs, srs); };
  if (a.early && T > 0) issue(0);  // tile 0 in flight under the row loads (see fa_fwd3_kernel)

  bfv8 qf[NKK], df[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    qf[kk] = gload8(qp + (int64_t)min(qrow, S - 1) * a.q_ss + kk * 16 + hh * 8, qrow < S);
    df[kk] = gload8(dop + (int64_t)min(qrow, S - 1) * a.d_ss + kk * 16 + hh * 8, qrow < S);
  }
  if (a.rope_q && qrow < S) {
    // fused RoPE: rotate the unrotated rows on load and hand them to the dK/dV pass (which stages Q through
    // LDS-DMA, so it needs them rotated in memory)
    const int p = rope_pos(a, b, qrow);
    rope_frags<NKK>(qf, a.rcos + (int64_t)p * (D / 2), a.rsin + (int64_t)p * (D / 2), hh);
  }
  if (a.ldw) {
    // the backward prep fused in: delta = rowsum(dO * O) from this lane's half row (64 of D elements, the
    // other half in lane r + 32), then the row constants of this wave's 32-row tile for the dK/dV kernel
    // (per 32-row tile: -lse / scale, -delta, segment id, -lse * log2e)
    const bf16* opr = a.o + (int64_t)b * a.o_sb + (int64_t)h * a.o_sh + (int64_t)min(qrow, S - 1) * a.o_ss;
    float dl = 0.f;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      const bfv8 o8 = gload8(opr + kk * 16 + hh * 8, qrow < S);
#pragma unroll
      for (int i = 0; i < 8; ++i) dl = fmaf((float)o8[i], (float)df[kk][i], dl);
    }
    dl += __shfl_xor(dl, 32, 64);
    dlt = qrow < S ? dl : 0.f;
    if (hh == 0 && qw < S) {  // (the last block's waves past the sequence end have no tile)
      float* blk = a.ldw + (((int64_t)b * a.Hq + h) * ((S + 31) / 32) + (qw >> 5)) * kLdTile;
      const float l = qrow < S ? a.lse[lrow] : -INFINITY;
      blk[r] = l == -INFINITY ? -INFINITY : -l / a.scale;
      blk[32 + r] = -dlt;
      reinterpret_cast<int*>(blk)[64 + r] = qrow < S ? (a.seg ? a.seg[(int64_t)b * S + qrow] : 0) : -1;
      blk[96 + r] = l == -INFINITY ? -INFINITY : -l * kLog2e;
    }
  }
  // hipcc does not count the asm DMAs: retire its own loads before the first one is issued
  asm volatile("" : "+v"(sq), "+v"(lse2), "+v"(dlt), "+v"(klo), "+v"(khi));
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(qf[kk]), "+v"(df[kk]));
  f32v16 dqt[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) dqt[dt][i] = 0.f;

  if (T > 0) {
    int ro[NKK], to[NDT][2];
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) ro[kk] = KI::roff(r, 2 * kk + hh);
    {
      const int g = lane >> 4, i16 = lane & 15;
      const int row = 4 * (g >> 1) + (i16 >> 2), col = 16 * (g & 1) + 4 * (i16 & 3);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        to[dt][0] = KI::toff(BN, row, dt * 32 + col);
        to[dt][1] = KI::toff(BN, row + 8, dt * 32 + col);
      }
    }

    if (!a.early) issue(0);
    wait_vm<0>();
    ring_barrier();
    // the tile loop unrolled by the ring's two slots: each slot's LDS offsets are compile-time constants
    // (folded into the ds_read offset fields instead of one v_add per read and tile)
    auto tile = [&](auto sidx, int t) {
      const char* slot = smem + decltype(sidx)::value * SLOT;
      const int n0 = kv_beg + t * BN;
      if (t + 1 < T) issue(t + 1);
      const bool m_seg = seg_mask(a, qr, n0, n0 + BN - 1);
      const bool need_mask = (a.causal && (n0 + BN - 1 > qw)) || (a.window >= 0 && (n0 < qw + 31 - a.window)) ||
                             (n0 + BN > S) || m_seg || qw + 31 >= S;
#pragma unroll 1
      for (int tt = 0; tt < 2; ++tt) {
        bfv8 fr[8];
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) fr[kk] = lds_b128(slot + 8192 * tt + ro[kk]);
        __builtin_amdgcn_sched_barrier(0);
        f32v16 st, dpt;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          st[i] = 0.f;
          dpt[i] = 0.f;
        }
        if constexpr (IL) {
          // V row kk reloads fr[kk] right behind the S^T MFMA that consumed it: the V reads fly under the
          // rest of the S^T chain instead of starting after it
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) {
            st = mfma32(fr[kk], qf[kk], st);
            fr[kk] = lds_b128(slot + IMG + 8192 * tt + ro[kk]);
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) st = mfma32(fr[kk], qf[kk], st);
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk) fr[kk] = lds_b128(slot + IMG + 8192 * tt + ro[kk]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) dpt = mfma32(fr[kk], df[kk], dpt);
        // K^T operands of the dQ product (keys 32tt + 16s2 .., columns 32dt ..), issued before the VALU
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const char* base = slot + 256 * (32 * tt + 16 * s2);
            const s16v4 lo = lds_tr(base + to[dt][0]), hi = lds_tr(base + to[dt][1]);
            fr[4 * s2 + dt] = __builtin_bit_cast(bfv8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
        __builtin_amdgcn_sched_barrier(0);
        if (need_mask && !OM) {
          const IdxRange rg = idx_range(klo, khi, n0 + 32 * tt + 4 * hh);
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            // masked: x = -inf -> exp2 = 0 -> dS = 0
            const float x0 = in_range(rg, 8 * (i >> 2) + (i & 3)) ? fmaf(st[i], sl2, -lse2) : -INFINITY;
            const float x1 = in_range(rg, 8 * (i >> 2) + (i & 3) + 1) ? fmaf(st[i + 1], sl2, -lse2) : -INFINITY;
            const float t0 = dpt[i] - dlt, t1 = dpt[i + 1] - dlt;
            asm("v_exp_f32 %0, %2\n\tv_exp_f32 %1, %3\n\tv_mul_f32 %0, %0, %4\n\tv_mul_f32 %1, %1, %5"
                : "=&v"(st[i]), "=&v"(st[i + 1]) : "v"(x0), "v"(x1), "v"(t0), "v"(t1));
          }
        } else if (OM && need_mask) {
          const int* Ss = reinterpret_cast<const int*>(slot + 2 * IMG);
          const int k0 = n0 + 32 * tt + 4 * hh;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            int4 sk = make_int4(sq, sq, sq, sq);
            if (m_seg) sk = *reinterpret_cast<const int4*>(Ss + 32 * tt + 8 * c + 4 * hh);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int kx = k0 + 8 * c + j;
              bool ok = kx < S && qrow < S;
              if (a.causal) ok = ok && (kx <= qrow);
              if (a.window >= 0) ok = ok && (qrow - kx <= a.window);
              if (m_seg) ok = ok && ((&sk.x)[j] == sq);
              const int i = 4 * c + j;
              const float pr = ok ? fexp2(fmaf(st[i], sl2, -lse2)) : 0.f;
              st[i] = pr * (dpt[i] - dlt);
            }
          }
        } else {  // (single-lane asm: B4 S8192 backward 7.978 -> 7.955 ms against hipcc's packed form)
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            if constexpr (!XS) {  // (A/B reference: the asm block reads the MFMA results itself)
              st[i] = exp_ds(fmaf(st[i], sl2, -lse2), dpt[i], dlt);
              st[i + 1] = exp_ds(fmaf(st[i + 1], sl2, -lse2), dpt[i + 1], dlt);
              continue;
            }
            // the MFMA results are read by compiler-visible VALU (fma, sub: hipcc places the minimal XDL
            // wait states instead of padding every asm block that reads them), the exp pair and the products
            // in one asm block (trans-use wait by placement)
            const float x0 = fmaf(st[i], sl2, -lse2), x1 = fmaf(st[i + 1], sl2, -lse2);
            const float t0 = dpt[i] - dlt, t1 = dpt[i + 1] - dlt;
            asm("v_exp_f32 %0, %2\n\tv_exp_f32 %1, %3\n\tv_mul_f32 %0, %0, %4\n\tv_mul_f32 %1, %1, %5"
                : "=&v"(st[i]), "=&v"(st[i + 1]) : "v"(x0), "v"(x1), "v"(t0), "v"(t1));
          }
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bfv8 db = acc_as_b(st, s2);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) dqt[dt] = mfma32(fr[4 * s2 + dt], db, dqt[dt]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      wait_vm<0>();  // this wave's DMA of tile t + 1
      ring_barrier();
        };
    for (int t = 0; t < T; t += 2) {
      tile(std::integral_constant<int, 0>{}, t);
      if (t + 1 < T) tile(std::integral_constant<int, 1>{}, t + 1);
    }
  }

  if (a.rope_q && qrow < S) {
    // the rotated rows for the dK/dV pass, stored after the loop (the wave's vmcnt counts stores: at the start
    // they held up its first DMA wait)
    bf16* qo = a.qrot + (int64_t)b * a.qr_sb + (int64_t)h * a.qr_sh + (int64_t)qrow * a.qr_ss + hh * 8;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) *reinterpret_cast<bfv8*>(qo + kk * 16) = qf[kk];
  }
  if (a.rope_dq && qrow < S) {  // fused RoPE: gradient of the unrotated q
    const int p = rope_pos(a, b, qrow);
    rope_acc_inv<D>(dqt, a.rcos + (int64_t)p * (D / 2), a.rsin + (int64_t)p * (D / 2), hh);
  }
  if constexpr (WS) {
    uint2 w[4 * NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        w[4 * dt + c].x = pack_bf16x2(dqt[dt][4 * c] * a.scale, dqt[dt][4 * c + 1] * a.scale);
        w[4 * dt + c].y = pack_bf16x2(dqt[dt][4 * c + 2] * a.scale, dqt[dt][4 * c + 3] * a.scale);
      }
    widen_pairs(w);
    if (qrow < S) store_pairs(a.out + (int64_t)b * a.dq_sb + (int64_t)qrow * a.dq_ss + (int64_t)h * a.dq_sh + 8 * hh, w);
  } else if (qrow < S) {
    bf16* dqp = a.out + (int64_t)b * a.dq_sb + (int64_t)qrow * a.dq_ss + (int64_t)h * a.dq_sh;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint2 w;
        w.x = pack_bf16x2(dqt[dt][4 * c] * a.scale, dqt[dt][4 * c + 1] * a.scale);
        w.y = pack_bf16x2(dqt[dt][4 * c + 2] * a.scale, dqt[dt][4 * c + 3] * a.scale);
        *reinterpret_cast<uint2*>(dqp + dt * 32 + 8 * c + 4 * hh) = w;
      }
  }
}

}  // namespace llmt

using namespace llmt;

// Kernel selection. One kernel family per pass and head dim (D = 64 / 96 / 128):
//   forward  fa_fwd3_kernel      (LDS-DMA K/V ring, fused Q rotation, range masks)
//   dQ       fa_bwd_dq3_kernel   (also computes delta and the per-tile row constants for the dK/dV pass)
//   dK/dV    fa_bwd_dkdv5_kernel (software-pipelined, one wave per SIMD, GQA heads looped in-kernel)
// plus the generic kernels (fa_fwd_kernel / fa_bwd_{delta,dq,dkdv}_kernel) for dropout and other head dims.
// Losing variants of earlier rounds (one-wave-per-SIMD hand-allocated forward / dK/dV, head chains, GQA head
// pairs, the un-pipelined dK/dV loop, the separate prep pass) were removed after their A/Bs
// (profiles/r5_attention_fwd4.md, r5_dkdv6.md, r3_attention_head_pairs_ab.jsonl, r4_negative_probes.jsonl).
// Knobs, read per launch (recorded by ops/native.py llmt_env() into run metadata):
//   LLMT_FA_GENERIC=1     the generic kernels for every launch (numerics reference);
//   LLMT_FA_RANGE_MASK=0  per-element mask compares instead of range masks (A/B reference);
//   LLMT_FA_EARLY_DMA=0   row loads before the first ring tiles in the prologues (A/B reference);
//   LLMT_FA_BMAJOR=0      batch-interleaved block order of dense rows (A/B reference; B4 S8192 Hq32 Hkv8 with
//                         the default batch-major order: forward 2.102 -> 2.068 ms, backward 7.795 -> 7.732 ms).
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static bool generic_only() { return env_int("LLMT_FA_GENERIC", 0) == 1; }
static int range_masks() { return env_int("LLMT_FA_RANGE_MASK", 1); }
static int early_dma() { return env_int("LLMT_FA_EARLY_DMA", 1); }
static int bmajor_order() { return env_int("LLMT_FA_BMAJOR", 1); }
#ifdef LLMT_DIAG
static int attn_probe() { return env_int("LLMT_FA_PROBE", 0); }
#else
static int attn_probe() { return 0; }
#endif

// 1 in the diagnostic library (probes compiled in), 0 in the production one
extern "C" int llmt_attn_diag_build() {
#ifdef LLMT_DIAG
  return 1;
#else
  return 0;
#endif
}

static void set_dropout(AttnArgs& a, float p, uint32_t seed) {
  if (p <= 0.f) {
    a.drop_thresh = 0;
    return;
  }
  const double t = (double)p * 4294967296.0;
  a.drop_thresh = (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : (t < 1.0 ? 1.0 : t));
  a.drop_seed = seed;
  a.drop_scale = 1.f / (1.f - p);
}

// buffer-load offsets are 32-bit: every row of one (batch, head) slice must be addressable
static bool fits32(int64_t S, int64_t row_stride) { return S * row_stride * 2 < 0x7fffffffLL; }
static bool strides32(std::initializer_list<int64_t> xs) {
  for (int64_t x : xs)
    if (x < 0 || x >= 0x7fffffffLL) return false;
  return true;
}

static bool aligned16(const void* p, int64_t s0, int64_t s1, int64_t s2) {
  return ((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (s0 % 8 == 0) && (s1 % 8 == 0) && (s2 % 8 == 0);
}

// fused-RoPE arguments (AttnArgs::rpos ...); qrot: contiguous [B, S, Hq, D] scratch for rotated queries
static void set_rope(AttnArgs& a, const void* rpos, int rpos64, int64_t rp_sb, int64_t rp_ss, const float* rcos,
                     const float* rsin, int64_t rP, void* qrot, int D) {
  a.rpos = rpos; a.rpos64 = rpos64; a.rp_sb = (int)rp_sb; a.rp_ss = (int)rp_ss;
  a.rcos = rcos; a.rsin = rsin; a.rP = (int)rP;
  a.qrot = (bf16*)qrot;
  a.qr_sh = D; a.qr_ss = a.Hq * D; a.qr_sb = a.S * a.Hq * D;
}
static void rope_launch(const AttnArgs& a, const bf16* x, int x_sb, int x_ss, int x_sh, bf16* y, int y_sb, int y_ss,
                        int y_sh, int H, int D, float sign, hipStream_t stream) {
  const int64_t n = (int64_t)a.B * a.S * H * (D / 16);
  rope_bshd_kernel<<<stream_grid(n, 256), 256, 0, stream>>>(a, x, x_sb, x_ss, x_sh, y, y_sb, y_ss, y_sh, H, D, sign);
}
// the rotated queries in qrot become the kernels' q
static void use_qrot(AttnArgs& a) {
  a.q = a.qrot; a.q_sb = a.qr_sb; a.q_ss = a.qr_ss; a.q_sh = a.qr_sh;
}
static bool rope_ok(const void* rpos, const float* rcos, const float* rsin, int64_t rP, int64_t rp_sb, int64_t rp_ss) {
  if (!rcos) return rpos == nullptr && rsin == nullptr;
  return rsin && rP > 0 && rP < 0x7fffffffLL && ((reinterpret_cast<uintptr_t>(rcos) | reinterpret_cast<uintptr_t>(rsin)) & 15) == 0 &&
         strides32({rp_sb, rp_ss});
}

// does the forward launch for this problem go to fa_fwd3_kernel (the kernel with the fused Q rotation)?
static bool fwd_uses_fwd3(int D, bool drop) { return !drop && !generic_only() && (D == 64 || D == 96 || D == 128); }

extern "C" hipError_t llmt_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                                          const int* seg, int B, int S, int Hq, int Hkv, int D, int64_t q_sb,
                                          int64_t q_ss, int64_t q_sh, int64_t k_sb, int64_t k_ss, int64_t k_sh,
                                          int64_t v_sb, int64_t v_ss, int64_t v_sh, int64_t o_sb, int64_t o_ss,
                                          int64_t o_sh, float scale, int causal, int window, int seg_runs,
                                          float drop_p, uint32_t drop_seed, const void* rpos, int rpos64,
                                          int64_t rp_sb, int64_t rp_ss, const float* rcos, const float* rsin,
                                          int64_t rP, void* qrot, hipStream_t stream) {
  if (Hkv <= 0 || Hq % Hkv) return hipErrorInvalidValue;
  if (!aligned16(q, q_sb, q_ss, q_sh) || !aligned16(k, k_sb, k_ss, k_sh) || !aligned16(v, v_sb, v_ss, v_sh) ||
      !aligned16(o, o_sb, o_ss, o_sh))
    return hipErrorInvalidValue;
  if (!rope_ok(rpos, rcos, rsin, rP, rp_sb, rp_ss)) return hipErrorInvalidValue;
  const bool rope = rcos != nullptr;
  if (!(drop_p >= 0.f && drop_p < 1.f)) return hipErrorInvalidValue;
  if (B == 0 || S == 0) return hipSuccess;
  if (!fits32(S, q_ss) || !fits32(S, k_ss) || !fits32(S, v_ss)) return hipErrorInvalidValue;
  if (!strides32({q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh})) return hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.out = (bf16*)o; a.lse = lse; a.seg = seg;
  if (seg && seg_runs) {
    a.rs = seg + (int64_t)B * S;
    a.re = seg + 2 * (int64_t)B * S;
    if (seg_runs == 2) {  // + the work orders of the query / key blocks
      a.qord = seg + 3 * (int64_t)B * S;
      a.kord = a.qord + (int64_t)B * ((S + 127) / 128);
    }
  }
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv;
  a.q_sb = q_sb; a.q_ss = q_ss; a.q_sh = q_sh; a.k_sb = k_sb; a.k_ss = k_ss; a.k_sh = k_sh;
  a.v_sb = v_sb; a.v_ss = v_ss; a.v_sh = v_sh; a.o_sb = o_sb; a.o_ss = o_ss; a.o_sh = o_sh;
  a.scale = scale; a.causal = causal; a.window = window;
  set_dropout(a, drop_p, drop_seed);
  a.bmajor = bmajor_order();
  a.rmask = range_masks() && (seg == nullptr || a.rs != nullptr);
  a.early = early_dma();
  a.probe = attn_probe();
  const bool v3 = fwd_uses_fwd3(D, a.drop_thresh != 0);
  if (rope) {
    // fused RoPE: q holds unrotated queries (k is already rotated). fa_fwd3_kernel rotates its rows on load;
    // the generic kernel gets the rotated rows in the qrot scratch (q itself is never written)
    set_rope(a, rpos, rpos64, rp_sb, rp_ss, rcos, rsin, rP, qrot, D);
    if (v3) {
      a.rope_q = 1;
    } else {
      if (!qrot) return hipErrorInvalidValue;
      rope_launch(a, a.q, a.q_sb, a.q_ss, a.q_sh, a.qrot, a.qr_sb, a.qr_ss, a.qr_sh, Hq, D, 1.f, stream);
      use_qrot(a);
    }
  }
  const dim3 grid((S + 127) / 128, Hq, B);
  // fa_fwd3: B1 S8192 Hq32 Hkv8 0.659 ms (834 TF/s; 977 TF/s at B4) vs 0.907 for the generic kernel;
  // RS = 2 (rmask): permlane32 row max, asm exp / row-sum pairs (2.091 -> 2.054 ms at B4 S8192); the widened
  // O store tail (T21) pays at short rows (B64 S512 0.343 -> 0.314 ms; profiles/r3_attention_wide_store_ab.jsonl)
  const unsigned nb1 = (unsigned)((S + 127) / 128 * Hq * B);
#define LLMT_FWD(DD)                                                  \
  if (!v3)                                                            \
    fa_fwd_kernel<DD><<<grid, 256, 0, stream>>>(a);                   \
  else if (a.rmask)                                                   \
    fa_fwd3_kernel<DD, 2, 1><<<nb1, 256, 0, stream>>>(a);             \
  else                                                                \
    fa_fwd3_kernel<DD, 1, 1, 4, true><<<nb1, 256, 0, stream>>>(a);
  switch (D) {
    case 64: { LLMT_FWD(64) } break;    // the v3 structure on 128-byte rows (256-byte LDS pitch)
    case 96: { LLMT_FWD(96) } break;    // Phi-3: 192-byte rows (256-byte LDS pitch)
    case 128: { LLMT_FWD(128) } break;
    default: return hipErrorInvalidValue;
  }
#undef LLMT_FWD
  return hipGetLastError();
}

// 1: a forward with fused RoPE needs no qrot scratch (the launch goes to fa_fwd3_kernel)
extern "C" int llmt_flash_attn_fwd_rope_inkernel(int D, float drop_p, int has_seg, int seg_runs) {
  (void)has_seg;
  (void)seg_runs;
  return fwd_uses_fwd3(D, drop_p > 0.f) ? 1 : 0;
}

// 1: the backward of this problem runs the generic kernels (GQA then needs the fp32 partials workspace)
extern "C" int llmt_flash_attn_bwd_generic(int D, float drop_p) {
  return (drop_p > 0.f || generic_only() || !(D == 64 || D == 96 || D == 128)) ? 1 : 0;
}

// floats of the `delta` workspace llmt_flash_attn_bwd needs
extern "C" int64_t llmt_flash_attn_bwd_ws(int B, int S, int Hq, int D) {
  const int64_t n = (int64_t)B * Hq * S;
  return (D == 128 || D == 96 || D == 64) ? n + (int64_t)B * Hq * ((S + 31) / 32) * kLdTile : n;
}

extern "C" hipError_t llmt_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                          const void* dout, const float* lse, float* delta, const int* seg, void* dq,
                                          void* dk, void* dv, float* work, int B, int S, int Hq, int Hkv, int D,
                                          int64_t q_sb, int64_t q_ss, int64_t q_sh, int64_t k_sb, int64_t k_ss,
                                          int64_t k_sh, int64_t v_sb, int64_t v_ss, int64_t v_sh, int64_t o_sb,
                                          int64_t o_ss, int64_t o_sh, int64_t dq_sb, int64_t dq_ss, int64_t dq_sh,
                                          int64_t dk_sb, int64_t dk_ss, int64_t dk_sh, int64_t dv_sb, int64_t dv_ss,
                                          int64_t dv_sh, float scale, int causal, int window, int seg_runs,
                                          float drop_p, uint32_t drop_seed, const void* rpos, int rpos64,
                                          int64_t rp_sb, int64_t rp_ss, const float* rcos, const float* rsin,
                                          int64_t rP, void* qrot, hipStream_t stream) {
  if (!(drop_p >= 0.f && drop_p < 1.f)) return hipErrorInvalidValue;
  if (!rope_ok(rpos, rcos, rsin, rP, rp_sb, rp_ss)) return hipErrorInvalidValue;
  // rope: dq / dk are returned for the unrotated q / k. qun: q holds UNROTATED queries (the forward rotated
  // them on load; qrot = scratch for the rotated rows); otherwise (qrot null) q / k are both rotated in
  // memory and only the inverse rotation of the gradients is fused
  const bool rope = rcos != nullptr, qun = rope && qrot != nullptr;
  if (Hkv <= 0 || Hq % Hkv) return hipErrorInvalidValue;
  if (!aligned16(q, q_sb, q_ss, q_sh) || !aligned16(k, k_sb, k_ss, k_sh) || !aligned16(v, v_sb, v_ss, v_sh) ||
      !aligned16(o, o_sb, o_ss, o_sh) || !aligned16(dout, o_sb, o_ss, o_sh) || !aligned16(dq, dq_sb, dq_ss, dq_sh) ||
      !aligned16(dk, dk_sb, dk_ss, dk_sh) || !aligned16(dv, dv_sb, dv_ss, dv_sh))
    return hipErrorInvalidValue;
  if (B == 0 || S == 0) return hipSuccess;
  if (!fits32(S, q_ss) || !fits32(S, k_ss) || !fits32(S, v_ss) || !fits32(S, o_ss)) return hipErrorInvalidValue;
  if (!strides32({q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh, o_sb, o_ss, o_sh, dq_sb, dq_ss, dq_sh, dk_sb,
                  dk_ss, dk_sh, dv_sb, dv_ss, dv_sh}))
    return hipErrorInvalidValue;
  AttnArgs a{};
  a.q = (const bf16*)q; a.k = (const bf16*)k; a.v = (const bf16*)v; a.o = (const bf16*)o;
  a.dout = (const bf16*)dout; a.out = (bf16*)dq; a.lse = (float*)lse; a.delta = delta; a.seg = seg;
  if (seg && seg_runs) {
    a.rs = seg + (int64_t)B * S;
    a.re = seg + 2 * (int64_t)B * S;
    if (seg_runs == 2) {  // + the work orders of the query / key blocks
      a.qord = seg + 3 * (int64_t)B * S;
      a.kord = a.qord + (int64_t)B * ((S + 127) / 128);
    }
  }
  a.dk = (bf16*)dk; a.dv = (bf16*)dv;
  const int64_t part = (int64_t)B * S * Hq * D;
  a.dk_part = work; a.dv_part = work ? work + part : nullptr;
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv;
  a.q_sb = q_sb; a.q_ss = q_ss; a.q_sh = q_sh; a.k_sb = k_sb; a.k_ss = k_ss; a.k_sh = k_sh;
  a.v_sb = v_sb; a.v_ss = v_ss; a.v_sh = v_sh; a.o_sb = o_sb; a.o_ss = o_ss; a.o_sh = o_sh;
  a.d_sb = o_sb; a.d_ss = o_ss; a.d_sh = o_sh;  // dout shares O's layout (checked by the caller)
  a.dq_sb = dq_sb; a.dq_ss = dq_ss; a.dq_sh = dq_sh; a.dk_sb = dk_sb; a.dk_ss = dk_ss; a.dk_sh = dk_sh;
  a.dv_sb = dv_sb; a.dv_ss = dv_ss; a.dv_sh = dv_sh;
  a.scale = scale; a.causal = causal; a.window = window;
  set_dropout(a, drop_p, drop_seed);
  a.bmajor = bmajor_order();
  a.rmask = range_masks() && (seg == nullptr || a.rs != nullptr);
  a.early = early_dma();
  a.probe = attn_probe();
  const bool gqa = Hq != Hkv;
  const int64_t nrows = (int64_t)B * S * Hq;
  const dim3 grid((S + 127) / 128, Hq, B);
  const int dgrid = stream_grid(nrows, 256);
  // fused RoPE: with qun the dQ kernel rotates its rows on load and writes them to qrot for the dK/dV
  // kernel; the dQ / dK epilogues apply the inverse rotation. Generic kernels: qrot by the standalone
  // rotation, inverse passes after.
  if (rope) set_rope(a, rpos, rpos64, rp_sb, rp_ss, rcos, rsin, rP, qrot, D);
  if ((D == 128 || D == 96 || D == 64) && !a.drop_thresh && !generic_only()) {
    if (rope) {
      a.rope_q = qun;
      a.rope_dq = 1;
    }
    // delta buffer = [B, Hq, S] delta, then the packed per-tile row constants (llmt_flash_attn_bwd_ws),
    // written by the dQ kernel (its waves cover every 32-row tile of every head; the dK/dV kernel runs after
    // it on this stream)
    float* ld = delta + nrows;
    a.ldw = ld;
    const unsigned gq = (unsigned)((S + 127) / 128 * Hq * B), gk = (unsigned)((S + 127) / 128 * Hkv * B);
    // dK/dV ring: 8 slots for D = 128 (tiles 6 ahead; B4 S8192 backward 7.605 -> 7.544 ms in one process;
    // packed 32 docs/row 1.546 -> 1.511 ms), 6 for D = 96 / 64 (dense 3.635 vs 3.649 ms;
    // profiles/r5_dkdv_ring_ab.jsonl)
#define LLMT_BWD3(DD, RING)                                                       \
  if (a.rmask)                                                                    \
    fa_bwd_dq3_kernel<DD, true, true><<<gq, 256, 0, stream>>>(a);                 \
  else                                                                            \
    fa_bwd_dq3_kernel<DD, true, true, 4, true><<<gq, 256, 0, stream>>>(a);        \
  if (rope) {                                                                     \
    if (qun) use_qrot(a);                                                         \
    a.rope_q = a.rope_dq = 0;                                                     \
    a.rope_dk = 1;                                                                \
  }                                                                               \
  if (a.rmask)                                                                    \
    fa_bwd_dkdv5_kernel<DD, false, RING><<<gk, 256, 0, stream>>>(a, ld);          \
  else                                                                            \
    fa_bwd_dkdv5_kernel<DD, true><<<gk, 256, 0, stream>>>(a, ld);
    switch (D) {
      case 64: { LLMT_BWD3(64, 6) } break;
      case 96: { LLMT_BWD3(96, 6) } break;
      default: { LLMT_BWD3(128, 8) } break;
    }
#undef LLMT_BWD3
    return hipGetLastError();
  }
  if (gqa && !work) return hipErrorInvalidValue;
  if (qun) {  // the generic kernels: rotated queries in qrot, inverse passes over dq / dk below
    rope_launch(a, a.q, a.q_sb, a.q_ss, a.q_sh, a.qrot, a.qr_sb, a.qr_ss, a.qr_sh, Hq, D, 1.f, stream);
    use_qrot(a);
  }
#define LLMT_BWD(DD)                                                                              \
  fa_bwd_delta_kernel<DD><<<dgrid, 256, 0, stream>>>(a);                                          \
  fa_bwd_dq_kernel<DD><<<grid, 256, 0, stream>>>(a);                                              \
  if (gqa) {                                                                                      \
    fa_bwd_dkdv_kernel<DD, true><<<grid, 256, 0, stream>>>(a);                                    \
    fa_gqa_reduce_kernel<DD><<<stream_grid((int64_t)B * S * Hkv * (DD / 4), 256), 256, 0, stream>>>(a); \
  } else {                                                                                        \
    fa_bwd_dkdv_kernel<DD, false><<<grid, 256, 0, stream>>>(a);                                   \
  }
  switch (D) {
    case 64: { LLMT_BWD(64) } break;
    case 96: { LLMT_BWD(96) } break;
    case 128: { LLMT_BWD(128) } break;
    default: return hipErrorInvalidValue;
  }
#undef LLMT_BWD
  if (rope) {
    rope_launch(a, a.out, a.dq_sb, a.dq_ss, a.dq_sh, a.out, a.dq_sb, a.dq_ss, a.dq_sh, Hq, D, -1.f, stream);
    rope_launch(a, a.dk, a.dk_sb, a.dk_ss, a.dk_sh, a.dk, a.dk_sb, a.dk_ss, a.dk_sh, Hkv, D, -1.f, stream);
  }
  return hipGetLastError();
}
