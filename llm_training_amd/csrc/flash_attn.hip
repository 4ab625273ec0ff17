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
  // diagnostic probes (LLMT_FA_PROBE, wrong results by design; benchmarks/attn_block_probe.py): forward 1 = no
  // tiles, 2 = no Q row loads, 4 = no O / LSE stores; backward 8 = no tiles in the dQ and dK/dV kernels
  int probe;
  // backward: non-null -> the dQ kernel computes delta = rowsum(dO * O) itself and writes the packed per-tile
  // row constants the dK/dV kernel reads here (no separate prep pass); null -> the prep kernel ran
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
// constants below (fa_bwd_prep128_kernel is the separate-pass form, LLMT_FA_PREP=1), and this key-parallel
// dK/dV kernel, built for one wave per SIMD (512 registers per lane):
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

// 16 lanes per row: each reads one 16-byte chunk of the row of O and of dO, so a wave instruction covers
// four contiguous 256-byte rows (one row per lane read 64 scattered 16-byte pieces: 2.7 TB/s); the
// partial dot products meet through three xor shuffles inside the 16-lane group.
template <int D>
__global__ __launch_bounds__(256) void fa_bwd_prep128_kernel(AttnArgs a, float* ld) {
  const int nT = (a.S + 31) / 32;
  const int64_t nrows = (int64_t)a.B * a.Hq * nT * 32;
  const float inv_scale = 1.f / a.scale;
  const int c = threadIdx.x & 15;
  for (int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; row < nrows; row += (int64_t)gridDim.x * 16) {
    const int i = (int)(row & 31);
    const int64_t tt = row >> 5;
    const int t = (int)(tt % nT);
    const int64_t bh = tt / nT;
    const int h = (int)(bh % a.Hq);
    const int b = (int)(bh / a.Hq);
    const int s = t * 32 + i;
    float dl = 0.f;
    if (s < a.S && c < D / 8) {
      const bf16x8* op = reinterpret_cast<const bf16x8*>(a.o + (int64_t)b * a.o_sb + (int64_t)s * a.o_ss + (int64_t)h * a.o_sh);
      const bf16x8* dp = reinterpret_cast<const bf16x8*>(a.dout + (int64_t)b * a.d_sb + (int64_t)s * a.d_ss + (int64_t)h * a.d_sh);
      float x[8], y[8];
      unpack8(op[c], x);
      unpack8(dp[c], y);
#pragma unroll
      for (int j = 0; j < 8; ++j) dl += x[j] * y[j];
    }
    dl += __shfl_xor(dl, 8, 16);
    dl += __shfl_xor(dl, 4, 16);
    dl += __shfl_xor(dl, 2, 16);
    dl += __shfl_xor(dl, 1, 16);
    if (c == 0) {
      float ls = -INFINITY, l2 = -INFINITY;
      int sg = -1;
      if (s < a.S) {
        const int64_t lr = ((int64_t)b * a.Hq + h) * a.S + s;
        ((float*)a.delta)[lr] = dl;
        const float l = a.lse[lr];
        ls = (l == -INFINITY) ? -INFINITY : -l * inv_scale;
        l2 = (l == -INFINITY) ? -INFINITY : -l * kLog2e;
        sg = a.seg ? a.seg[(int64_t)b * a.S + s] : 0;
      } else {
        dl = 0.f;
      }
      float* blk = ld + (bh * nT + t) * kLdTile;
      blk[i] = ls;
      blk[32 + i] = -dl;
      reinterpret_cast<int*>(blk)[64 + i] = sg;
      blk[96 + i] = l2;
    }
  }
}

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

// grid: ceil(S/128) * Hkv * B blocks (1-D), 4 waves x 32 keys; query tiles of 32 rows over all q heads of
// the kv group; NS-slot LDS-DMA ring.
// D = 96 (Phi-3) runs the same structure on 256-byte LDS rows: the DMA rows read 64 bytes past each
// 192-byte row (never past the tensor: the descriptors end at the last row's D elements) and only the
// first D / 16 k-steps / D / 32 output tiles are used.
template <int V, int D = 128, bool WS = false>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv128_kernel(AttnArgs a, const float* ld) {
  constexpr int NKK = D / 16, NDT = D / 32;
  constexpr int BM = 32, IMG = BM * 256, SLOT = 2 * IMG + 2 * 256, NS = 6;
  constexpr int NDMA = 5;  // DMA instructions per wave per tile: Q 2, dO 2, row constants 1
  using QI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases go to M0
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
  const int sk = (a.seg && kr < S) ? a.seg[(int64_t)b * S + kr] : 0;
  const float sl2 = a.scale * kLog2e;

  bfv8 kf[NKK], vf[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) {
    kf[kk] = gload8(kp + (int64_t)min(kr, S - 1) * a.k_ss + kk * 16 + hh * 8, kr < S);
    vf[kk] = gload8(vp + (int64_t)min(kr, S - 1) * a.v_ss + kk * 16 + hh * 8, kr < S);
  }
  // hipcc's load counting does not see the asm DMAs below: make it retire its own loads here
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(kf[kk]), "+v"(vf[kk]));
  f32v16 dkt[NDT], dvt[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      dkt[dt][i] = 0.f;
      dvt[dt][i] = 0.f;
    }

  const RunInfo kr_run = block_run(a, b, min(ks, S - 1), min(ks + 127, S - 1));
  const int q_beg = a.causal ? ks : max(0, kr_run.rs) / 32 * 32;  // multiple of 32
  int q_end = a.window >= 0 ? min(S, ks + 128 + a.window) : S;
  if (a.rs) q_end = min(q_end, a.re[(int64_t)b * S + min(ks + 127, S - 1)] + 1);
  const int nq = q_end > q_beg ? (q_end - q_beg + BM - 1) / BM : 0;
  const int T = nq * grp;

  if (T > 0) {
    // ---- DMA of the next tile (tiles past T-1 repeat the last one) into the ring. The tile sequence
    // is walked with scalar counters. Each descriptor covers one head from row q_beg on (rows past S
    // fall outside it and read as zeros) and is rebuilt only when the walk enters the next head; the
    // tile's byte offset inside the head rides in the lane offsets (one VALU add per DMA instead of
    // three 64-bit descriptor builds per tile: the old per-tile descriptors were ~90 SALU per tile
    // in a loop that issues one instruction per cycle from its single wave per SIMD).
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
    auto issue = [&](const char* slot) {
      // row constants: waves 0/2 fetch floats 0..63, waves 1/3 floats 64..127 (same bytes twice)
      const char* q0 = slot + 8 * wid * 256;
      dma_tile5(qrs, drs, lrs, q0, q0 + 4 * 256, q0 + IMG, q0 + IMG + 4 * 256, slot + 2 * IMG + (wid & 1) * 256,
                dq_off[0] + toff_q, dq_off[1] + toff_q, dd_off[0] + toff_d, dd_off[1] + toff_d, ld_off + toff_l);
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
    // mask state of a tile: first query row, and whether any element of it needs the compare
    int cur_q = 0;  // tile index inside its head of the tile whose S/dP is being computed
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
    // lane-constant LDS byte offsets inside a 32-row image, computed once and kept opaque so hipcc
    // does not re-derive the swizzle for every read inside the loop (it did: ~5 VALU per read)
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
    auto rows = [&](const char* slot, bfv8* qr, bfv8* dr) {
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const char* p = slot + ro[kk];  // one VGPR address; the dO image is an immediate offset away
        qr[kk] = lds_b128(p);
        dr[kk] = lds_b128(p + IMG);
      }
    };
    // A operands of the accumulator-as-B products from tile image pair `slot`: rows 16*s2..,
    // columns 32*dt.. of Q (dK) and dO (dV); 8 VGPR addresses per tile, everything else immediates
    auto trA2 = [&](const char* slot, bfv8 (&tq)[2][NDT], bfv8 (&td)[2][NDT]) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const char* p0 = slot + to[dt][0];
        const char* p1 = slot + to[dt][1];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const s16v4 ql = lds_tr(p0 + 4096 * s2), qh = lds_tr(p1 + 4096 * s2);
          const s16v4 dl = lds_tr(p0 + IMG + 4096 * s2), dh = lds_tr(p1 + IMG + 4096 * s2);
          tq[s2][dt] = __builtin_bit_cast(bfv8, __builtin_shufflevector(ql, qh, 0, 1, 2, 3, 4, 5, 6, 7));
          td[s2][dt] = __builtin_bit_cast(bfv8, __builtin_shufflevector(dl, dh, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
    };
    // S = Q.K^T and dP = dO.V^T of the tile in `qr` / `dr`, accumulated from zero (the MFMA's inline 0)
    auto sdp = [&](const bfv8* qr, const bfv8* dr, f32v16& s, f32v16& d) {
      const f32v16 z = {};
      s = mfma32(qr[0], kf[0], z);
      d = mfma32(dr[0], vf[0], z);
#pragma unroll
      for (int kk = 1; kk < NKK; ++kk) {
        s = mfma32(qr[kk], kf[kk], s);
        d = mfma32(dr[kk], vf[kk], d);
      }
    };
    // P = exp2(S * scale * log2e - lse * log2e) and dS = P (dP - delta) of the tile in `slot` (its row
    // constants: -lse*log2e at floats 96.., -delta at 32..; rows past S / without keys carry -inf);
    // masked elements (diagonal / window / segment tiles only) get P = 0
    auto softmax = [&](const char* slot, const TileMask& m, const f32v16& s, const f32v16& d, bfv8 (&pb)[2],
                       bfv8 (&db)[2]) {
      const float* Ls = reinterpret_cast<const float*>(slot + 2 * IMG);
      float lq[16], nd[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 l4 = *reinterpret_cast<const float4*>(Ls + 96 + 8 * c + 4 * hh);
        const float4 d4 = *reinterpret_cast<const float4*>(Ls + 32 + 8 * c + 4 * hh);
        lq[4 * c] = l4.x; lq[4 * c + 1] = l4.y; lq[4 * c + 2] = l4.z; lq[4 * c + 3] = l4.w;
        nd[4 * c] = d4.x; nd[4 * c + 1] = d4.y; nd[4 * c + 2] = d4.z; nd[4 * c + 3] = d4.w;
      }
      // packed fp32 math (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32: two lanes' worth per instruction)
      // wherever two neighbouring elements take the same operation: the loop issues one instruction per
      // cycle from its single wave per SIMD, so halving the VALU count of the softmax shortens it
      typedef float f2 __attribute__((ext_vector_type(2)));
      float p[16];
      const f2 sl2v = {sl2, sl2};
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        if constexpr (V == 1) {  // scalar form (A/B reference)
          p[i] = fexp2(fmaf(s[i], sl2, lq[i]));
          p[i + 1] = fexp2(fmaf(s[i + 1], sl2, lq[i + 1]));
        } else {
          const f2 sv = {s[i], s[i + 1]}, lv = {lq[i], lq[i + 1]};
          const f2 x = __builtin_elementwise_fma(sv, sl2v, lv);
          p[i] = fexp2(x[0]);
          p[i + 1] = fexp2(x[1]);
        }
      }
      if (m.need) {
        const int* Sg = reinterpret_cast<const int*>(Ls + 64);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int4 s4 = make_int4(sk, sk, sk, sk);
          if (m.m_seg) s4 = *reinterpret_cast<const int4*>(Sg + 8 * c + 4 * hh);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int qi = m.q0 + 8 * c + 4 * hh + j;
            bool ok = true;
            if (a.causal) ok = ok && (kr <= qi);
            if (a.window >= 0) ok = ok && (qi - kr <= a.window);
            if (m.m_seg) ok = ok && ((&s4.x)[j] == sk);
            p[4 * c + j] = ok ? p[4 * c + j] : 0.f;
          }
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int i = 8 * s2 + j;
          const f2 pv = {p[i], p[i + 1]}, dv = {d[i], d[i + 1]}, nv = {nd[i], nd[i + 1]};
          f2 ds;
          if constexpr (V == 1) {
            ds[0] = p[i] * (d[i] + nd[i]);
            ds[1] = p[i + 1] * (d[i + 1] + nd[i + 1]);
          } else {
            ds = pv * (dv + nv);
          }
          pb[s2][j] = (__bf16)p[i];
          pb[s2][j + 1] = (__bf16)p[i + 1];
          db[s2][j] = (__bf16)ds[0];
          db[s2][j + 1] = (__bf16)ds[1];
        }
    };

    // ring slots (byte offsets) of tiles t-2 (the DMA target of iteration t), t-1, t, t+1
    int sl_m2 = (NS - 1) * SLOT, sl_m1 = 0, sl_0 = SLOT, sl_p1 = 2 * SLOT;
    // prologue: tiles 0..NS-2 in flight, wait for 0..2
#pragma unroll
    for (int t = 0; t < NS - 1; ++t) issue(smem + t * SLOT);
    wait_vm<NDMA * (NS - 4)>();
    ring_barrier();

    bfv8 qr[NKK], dr[NKK];
    f32v16 sacc, dacc;
    rows(smem, qr, dr);
    TileMask mprev = tile_mask();
    sdp(qr, dr, sacc, dacc);
    rows(smem + SLOT, qr, dr);

    for (int t = 1; t <= T; ++t) {
      issue(smem + sl_m2);
      // ---- region A: S/dP of tile t  ||  softmax of tile t-1 + its transposed reads
      const TileMask mcur = tile_mask();
      const char* pslot = smem + sl_m1;
      bfv8 trd[2][NDT], trq[2][NDT];
      trA2(pslot, trq, trd);
      f32v16 sn, dn;
      sdp(qr, dr, sn, dn);
      bfv8 pb[2], db[2];
      softmax(pslot, mprev, sacc, dacc, pb, db);
      // ---- region B: dV/dK of tile t-1  ||  row reads of tile t+1
      rows(smem + sl_p1, qr, dr);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          dvt[dt] = mfma32(trd[s2][dt], pb[s2], dvt[dt]);
          dkt[dt] = mfma32(trq[s2][dt], db[s2], dkt[dt]);
        }
      sacc = sn;
      dacc = dn;
      mprev = mcur;
      sl_m2 = sl_m1;
      sl_m1 = sl_0;
      sl_0 = sl_p1;
      sl_p1 = (sl_p1 + SLOT == NS * SLOT) ? 0 : sl_p1 + SLOT;
      wait_vm<NDMA * (NS - 4)>();
      if constexpr (V == 3)
        ring_barrier_nodrain();
      else
        ring_barrier();
    }
    wait_vm<0>();  // no LDS-DMA may outlive the workgroup
  }

  if constexpr (WS) {  // widened store tail (widen_pairs): 16-byte stores of dK / dV rows
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
  } else if (kr < S) {
    bf16* dkp = a.dk + (int64_t)b * a.dk_sb + (int64_t)kr * a.dk_ss + (int64_t)hk * a.dk_sh;
    bf16* dvp = a.dv + (int64_t)b * a.dv_sb + (int64_t)kr * a.dv_ss + (int64_t)hk * a.dv_sh;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
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

// ============================================================================ backward dK/dV, v5
// The dK/dV pass of fa_bwd_dkdv128_kernel (same grid, ring, DMA, masks and fragment layouts) with the
// loop rebuilt as a software pipeline for its one wave per SIMD (profiles/r4_dkdv_pipeline.md). Per
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
  const int T = (a.probe & 8) ? 0 : nq * grp;

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
  const int T = (kv_end > kv_beg && !(a.probe & 1)) ? (kv_end - kv_beg + BN - 1) / BN : 0;
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
    qf[kk] = gload8(qp + (int64_t)min(qrow, S - 1) * a.q_ss + kk * 16 + hh * 8, qrow < S && !(a.probe & 2));
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
    if (qrow < S && !(a.probe & 4)) store_pairs(a.out + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * a.o_sh + 8 * hh, w);
  }
  if (qrow < S && !(a.probe & 4)) {
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

// ============================================================================ forward, D = 128, v4
// One wave per SIMD with 64 query rows per wave (two 32-row halves that share every K and V^T fragment
// read, so a tile's LDS reads feed twice the MFMAs of fa_fwd3_kernel), 256-row blocks of 4 waves, 64-key
// K/V tiles by LDS-DMA into a 4-slot ring (one barrier per tile, tile t+2 in flight under tile t).
// Register files by role, allocated by hand (cdna guide §B, the 4-wave one-wave-per-SIMD structure): the
// accumulator file holds O^T (a[0:127]), Q (a[128:191]) and the current K tile (a[192:255]) under literal
// register names in the asm MFMAs and asm LDS reads (hipcc's allocator moved "a"-constrained copies of
// them between registers and spilled when it owned them); the arch VGPRs hold two 64-score sets, bf16 P,
// the V^T fragments and the softmax state, compiler-allocated. Each tile t is two phases of 32 MFMAs:
//  * phase A: S^T(t) = K(t) Q^T, while the softmax of tile t-1 finishes (exps of its second key half, row
//    sums, bf16 P) and the first V^T(t-1) fragments are read;
//  * phase B: O^T += V^T(t-1) P^T(t-1), while the softmax of tile t starts (mask on diagonal / window / end
//    tiles, row max, defer-max decision, exps of the first key half), the rest of V^T(t-1) is read just in
//    time and K(t+1) is read into the accumulator file.
// A rescale (a row max growing past kThr) multiplies O^T and l after phase B, when every P at the old max
// (tile t-1) has been added and none at the new one. Dense rows (no segment ids), D = 128, no dropout.
#define LLMT_ACLOB "a0","a1","a2","a3","a4","a5","a6","a7","a8","a9","a10","a11","a12","a13","a14","a15","a16","a17","a18","a19","a20","a21","a22","a23","a24","a25","a26","a27","a28","a29","a30","a31","a32","a33","a34","a35","a36","a37","a38","a39","a40","a41","a42","a43","a44","a45","a46","a47","a48","a49","a50","a51","a52","a53","a54","a55","a56","a57","a58","a59","a60","a61","a62","a63","a64","a65","a66","a67","a68","a69","a70","a71","a72","a73","a74","a75","a76","a77","a78","a79","a80","a81","a82","a83","a84","a85","a86","a87","a88","a89","a90","a91","a92","a93","a94","a95","a96","a97","a98","a99","a100","a101","a102","a103","a104","a105","a106","a107","a108","a109","a110","a111","a112","a113","a114","a115","a116","a117","a118","a119","a120","a121","a122","a123","a124","a125","a126","a127","a128","a129","a130","a131","a132","a133","a134","a135","a136","a137","a138","a139","a140","a141","a142","a143","a144","a145","a146","a147","a148","a149","a150","a151","a152","a153","a154","a155","a156","a157","a158","a159","a160","a161","a162","a163","a164","a165","a166","a167","a168","a169","a170","a171","a172","a173","a174","a175","a176","a177","a178","a179","a180","a181","a182","a183","a184","a185","a186","a187","a188","a189","a190","a191","a192","a193","a194","a195","a196","a197","a198","a199","a200","a201","a202","a203","a204","a205","a206","a207","a208","a209","a210","a211","a212","a213","a214","a215","a216","a217","a218","a219","a220","a221","a222","a223","a224","a225","a226","a227","a228","a229","a230","a231","a232","a233","a234","a235","a236","a237","a238","a239","a240","a241","a242","a243","a244","a245","a246","a247","a248","a249","a250","a251","a252","a253","a254","a255"

template <int... Is, class F>
__device__ __forceinline__ void sfor_seq(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
// f(std::integral_constant<int, i>) for i = 0 .. N-1: compile-time indices for "i" asm operands
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_seq(std::make_integer_sequence<int, N>{}, f);
}
constexpr int fa4_ao(int dt, int qh) { return (dt * 2 + qh) * 16; }  // O^T tile (d tile, query half)
constexpr int fa4_aq(int qh, int kk) { return 128 + (qh * 8 + kk) * 4; }  // Q fragment (query half, k-step)
constexpr int fa4_ak(int kh, int kk) { return 192 + (kh * 8 + kk) * 4; }  // K fragment (key half, k-step)
// phase B of fa_fwd4 exponentiates the first key half's 32 scores in gaps 10 .. 31: one in gaps 10 .. 21, two
// in gaps 22 .. 31 (score index of the gap's first exp, and how many)
constexpr int fa4_nexp(int g) { return g < 10 ? 0 : (g < 22 ? 1 : 2); }
constexpr int fa4_exp0(int g) { return g < 22 ? g - 10 : 12 + 2 * (g - 22); }

// two floats -> packed bf16 pair, issued where it stands (hipcc lowered element-wise bf16 inserts as one
// block of conversions in front of the first MFMA that reads them)
__device__ __forceinline__ uint32_t cvt_pk(float lo, float hi) {
  uint32_t r;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
// exp2(x) with its row-sum add one instruction behind (the trans-use wait state by placement, see fwd3)
__device__ __forceinline__ float exp_sum(float x, float& rs) {
  float e;
  asm volatile("v_exp_f32 %0, %2\n\ts_nop 0\n\tv_add_f32 %1, %1, %0" : "=&v"(e), "+v"(rs) : "v"(x));
  return e;
}

// LDS-DMA of one 64-key K/V tile (no segment ids) for fa_fwd4: this wave's 16 K and 16 V rows, 4 per
// instruction; the per-lane byte offsets (voffset: range-checked against the descriptor, so rows past the
// sequence end read zeros) hold the tile's first row. The leading s_nop covers descriptor words written by
// a VALU just before (VALU write of an SGPR -> VMEM read of it: 5 wait states; hipcc does not look inside
// the statement).
__device__ __forceinline__ void dma_tile8(const Rsrc& k, const Rsrc& v, uint32_t lds, int img, const int (&vk)[4],
                                          const int (&vv)[4]) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %11, 0 offen lds\n\t"
      "s_add_u32 m0, %1, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %7, %12, 0 offen lds\n\t"
      "s_add_u32 m0, %1, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %11, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %8, %12, 0 offen lds\n\t"
      "s_add_u32 m0, %1, 0x800\n\ts_nop 0\n\tbuffer_load_dwordx4 %5, %11, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %9, %12, 0 offen lds\n\t"
      "s_add_u32 m0, %1, 0xc00\n\ts_nop 0\n\tbuffer_load_dwordx4 %6, %11, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %10, %12, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "s"(img), "v"(vk[0]), "v"(vk[1]), "v"(vk[2]), "v"(vk[3]), "v"(vv[0]), "v"(vv[1]), "v"(vv[2]),
        "v"(vv[3]), "s"(k.w), "s"(v.w)
      : "memory", "scc");
}
// x if key offset o is inside the row's range (base + o <= span, unsigned: idx_range), else -inf, in place;
// VCC only (hipcc's 64-bit compare masks for a whole masked tile ran the kernel out of scalar registers)
template <int O>
__device__ __forceinline__ float range_or_ninf(float x, uint32_t base, uint32_t span) {
  uint32_t t;
  asm("v_add_u32 %1, %c3, %2\n\tv_cmp_le_u32 vcc, %1, %4\n\tv_cndmask_b32 %0, %5, %0, vcc"
      : "+v"(x), "=&v"(t)
      : "v"(base), "i"(O), "v"(span), "v"(-INFINITY)
      : "vcc");
  return x;
}
// single VALU instructions for the hand-spaced softmax gaps (hipcc would pair or fuse neighbours)
__device__ __forceinline__ float v_exp1(float x) {
  float r;
  asm volatile("v_exp_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ void v_add_ip(float& acc, float x) { asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc) : "v"(x)); }
__device__ __forceinline__ float v_fma1(float x, float c, float d) {
  float r;
  asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(c), "v"(d));
  return r;
}

template <int D = 128>
__global__ __launch_bounds__(256, 1) void fa_fwd4_kernel(AttnArgs a) {
  static_assert(D == 128, "fa_fwd4 is the D = 128 kernel");
  constexpr int BN = 64, IMG = BN * 256, SLOT = 2 * IMG, NSL = 4;
  using KI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[NSL * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = a.S, grp = a.Hq / a.Hkv;
  const int nqb = (S + 255) / 256;
  int L = (int)blockIdx.x;
  const int hk = L % a.Hkv;
  L /= a.Hkv;
  const int h = hk * grp + L % grp;
  L /= grp;
  int b, mb;
  block_of(a, L, nqb, true, b, mb);
  const int qs = mb * 256, qw = qs + wid * 64;
  const int qrow0 = qw + r, qrow1 = qw + 32 + r;
  const float sl2 = a.scale * kLog2e;

  // O^T = 0 and Q into the accumulator file; this statement also claims all 256 accumulator registers for
  // the kernel descriptor (the clobbers), so hipcc neither allocates nor spills into them
  asm volatile(
#define Z4(n) "v_accvgpr_write_b32 a" #n ", 0\n\t"
      Z4(0) Z4(1) Z4(2) Z4(3) Z4(4) Z4(5) Z4(6) Z4(7) Z4(8) Z4(9) Z4(10) Z4(11) Z4(12) Z4(13) Z4(14) Z4(15)
      Z4(16) Z4(17) Z4(18) Z4(19) Z4(20) Z4(21) Z4(22) Z4(23) Z4(24) Z4(25) Z4(26) Z4(27) Z4(28) Z4(29) Z4(30)
      Z4(31) Z4(32) Z4(33) Z4(34) Z4(35) Z4(36) Z4(37) Z4(38) Z4(39) Z4(40) Z4(41) Z4(42) Z4(43) Z4(44) Z4(45)
      Z4(46) Z4(47) Z4(48) Z4(49) Z4(50) Z4(51) Z4(52) Z4(53) Z4(54) Z4(55) Z4(56) Z4(57) Z4(58) Z4(59) Z4(60)
      Z4(61) Z4(62) Z4(63) Z4(64) Z4(65) Z4(66) Z4(67) Z4(68) Z4(69) Z4(70) Z4(71) Z4(72) Z4(73) Z4(74) Z4(75)
      Z4(76) Z4(77) Z4(78) Z4(79) Z4(80) Z4(81) Z4(82) Z4(83) Z4(84) Z4(85) Z4(86) Z4(87) Z4(88) Z4(89) Z4(90)
      Z4(91) Z4(92) Z4(93) Z4(94) Z4(95) Z4(96) Z4(97) Z4(98) Z4(99) Z4(100) Z4(101) Z4(102) Z4(103) Z4(104)
      Z4(105) Z4(106) Z4(107) Z4(108) Z4(109) Z4(110) Z4(111) Z4(112) Z4(113) Z4(114) Z4(115) Z4(116) Z4(117)
      Z4(118) Z4(119) Z4(120) Z4(121) Z4(122) Z4(123) Z4(124) Z4(125) Z4(126) Z4(127)
#undef Z4
      ::: LLMT_ACLOB);
  {
    const bf16* qp = a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh;
    sfor<2>([&](auto qc) {
      constexpr int qh = decltype(qc)::value;
      const int q = qh ? qrow1 : qrow0;
      sfor<8>([&](auto kc) {
        constexpr int kk = decltype(kc)::value;
        const bfv8 x = gload8(qp + (int64_t)min(q, S - 1) * a.q_ss + kk * 16 + hh * 8, q < S);
        const u32x4 w = __builtin_bit_cast(u32x4, x);
        asm volatile("v_accvgpr_write_b32 a%c0, %4\n\tv_accvgpr_write_b32 a%c1, %5\n\t"
                     "v_accvgpr_write_b32 a%c2, %6\n\tv_accvgpr_write_b32 a%c3, %7"
                     :: "i"(fa4_aq(qh, kk)), "i"(fa4_aq(qh, kk) + 1), "i"(fa4_aq(qh, kk) + 2), "i"(fa4_aq(qh, kk) + 3),
                     "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
      });
    });
  }
  // per-row key ranges as IdxRange pieces relative to key 0 of the tile: base0 + n0 is added per tile
  int klo0, khi0, klo1, khi1;
  key_interval(a, b, qrow0, klo0, khi0);
  key_interval(a, b, qrow1, klo1, khi1);
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f}, nm[2] = {0.f, 0.f}, alpha[2] = {1.f, 1.f};

  int kv_end = a.causal ? min(S, qs + 256) : S;
  int kv_beg = a.window >= 0 ? max(0, qs - a.window) : 0;
  kv_beg = kv_beg / BN * BN;
  const int T = kv_end > kv_beg ? (kv_end - kv_beg + BN - 1) / BN : 0;
  // this wave's tiles with any visible key: [wt0, wt1] (wave-uniform)
  int wt1 = T - 1, wt0 = 0;
  if (a.causal) wt1 = min(wt1, (min(qw + 63, S - 1) - kv_beg) / BN);
  if (a.window >= 0) wt0 = max(0, (qw - a.window - kv_beg) / BN);
  if (qw >= S) wt1 = -1;

  if (T > 0) {
    const Rsrc krs = make_rsrc4(a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh, ((int64_t)(S - 1) * a.k_ss + D) * 2);
    const Rsrc vrs = make_rsrc4(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh, ((int64_t)(S - 1) * a.v_ss + D) * 2);
    int vk[4], vv[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = 16 * wid + 4 * n + (lane >> 4);
      const int ch = (lane & 15) ^ KI::swz(row);
      vk[n] = (row * a.k_ss + ch * 8) * 2;
      vv[n] = (row * a.v_ss + ch * 8) * 2;
    }
    const uint32_t lds0 = lds_addr(smem) + 16 * wid * 256;
    const int kstep = BN * a.k_ss * 2, vstep = BN * a.v_ss * 2;
    auto issue = [&](int t) {
      int kr = (kv_beg / BN + t) * kstep, vr = (kv_beg / BN + t) * vstep;
      // opaque: otherwise hipcc keeps the per-lane offsets of every unrolled step's tile precomputed in
      // registers (it then parked some in the accumulator file, which the asm owns)
      asm volatile("" : "+s"(kr), "+s"(vr));
      const int ko[4] = {vk[0] + kr, vk[1] + kr, vk[2] + kr, vk[3] + kr};
      const int vo[4] = {vv[0] + vr, vv[1] + vr, vv[2] + vr, vv[3] + vr};
      dma_tile8(krs, vrs, lds0 + (t & 3) * SLOT, IMG, ko, vo);
    };
    int ro[8], to[4][2];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) ro[kk] = lds_addr(smem) + KI::roff(r, 2 * kk + hh);
    {
      const int g = lane >> 4, i16 = lane & 15;
      const int row = 4 * (g >> 1) + (i16 >> 2), col = 16 * (g & 1) + 4 * (i16 & 3);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        to[dt][0] = lds_addr(smem) + KI::toff(BN, row, dt * 32 + col) + IMG;
        to[dt][1] = lds_addr(smem) + KI::toff(BN, row + 8, dt * 32 + col) + IMG;
      }
    }
    // K fragments (both key halves, k-step kk) of the tile in ring slot `sl` into the accumulator file
    auto read_k = [&](int sl, auto kc) {
      constexpr int kk = decltype(kc)::value;
      const int addr = ro[kk] + sl * SLOT;
      asm volatile("ds_read_b128 a[%c0:%c1], %4\n\tds_read_b128 a[%c2:%c3], %4 offset:8192"
                   :: "i"(fa4_ak(0, kk)), "i"(fa4_ak(0, kk) + 3), "i"(fa4_ak(1, kk)), "i"(fa4_ak(1, kk) + 3), "v"(addr)
                   : "memory");
    };
    // V^T fragment (keys 32kh + 16s2 .., columns 32dt ..) of the tile in ring slot `sl`
    auto read_v = [&](int sl, int kh, int s2, int dt) -> bfv8 {
      const int off = sl * SLOT + 256 * (32 * kh + 16 * s2);
      using lp = __attribute__((address_space(3))) s16v4*;
      const s16v4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(uintptr_t)(uint32_t)(to[dt][0] + off));
      const s16v4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(uintptr_t)(uint32_t)(to[dt][1] + off));
      return __builtin_bit_cast(bfv8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };

    // ring slot 3 holds the "previous tile" V^T of a wave's first step when that is tile 0: P = 0 there, but
    // 0 * (stale NaN / inf bits) would not be 0 — zero it once
#pragma unroll
    for (int i = 0; i < IMG / (16 * 256); ++i)
      *reinterpret_cast<uint4*>(smem + 3 * SLOT + IMG + 16 * (tid + 256 * i)) = make_uint4(0, 0, 0, 0);
    issue(0);
    if (T > 1) issue(1);
    wait_vm<0>();
    ring_barrier();
    sfor<8>([&](auto kc) { read_k(0, kc); });

    // score sets of alternate steps ([key half][query half]); the set the wave's first step finishes as "the
    // previous tile" starts at -inf (exp -> P = 0, row sums 0), so every step runs the same two phases
    f32v16 sA[2][2], sB[2][2];
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int x = 0; x < 4; ++x) sB[x >> 1][x & 1][i] = -INFINITY;
    uint32_t pw[2][2][2][4];  // bf16 P of the previous tile: [key half][query half][k-step][pair]
#pragma unroll
    for (int i = 0; i < 32; ++i) (&pw[0][0][0][0])[i] = 0u;  // the wave's first step has no previous tile
    bool resc = false;

    // phase A of tile t: S^T(t) into sc || finish the softmax of tile t-1: exps of its second key half sp[1]
    // (the first half was exponentiated, summed and converted in phase B of the previous step), their row
    // sums, bf16 P of that half
    auto phase_a = [&](f32v16 (&sc)[2][2], f32v16 (&sp)[2][2], int vsl, bfv8 (&vr)[16]) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the K tile in the accumulator file
      __builtin_amdgcn_sched_barrier(0);
      float rs0 = 0.f, rs1 = 0.f;
      sfor<32>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        constexpr int kk = g >> 2, kh = (g >> 1) & 1, qh = g & 1;
        if constexpr (kk == 0)
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], 0"
                       : "=v"(sc[kh][qh])
                       : "i"(fa4_ak(kh, kk)), "i"(fa4_ak(kh, kk) + 3), "i"(fa4_aq(qh, kk)), "i"(fa4_aq(qh, kk) + 3));
        else
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, a[%c1:%c2], a[%c3:%c4], %0"
                       : "+v"(sc[kh][qh])
                       : "i"(fa4_ak(kh, kk)), "i"(fa4_ak(kh, kk) + 3), "i"(fa4_aq(qh, kk)), "i"(fa4_aq(qh, kk) + 3));
        // the second key half's 32 scores e = 16 fq + fi, three gap-stages apart so no gap waits on its own
        // results: gap g scales (fma) and exponentiates score g, adds score g - 2 to its row sum and packs
        // pair (g - 4, g - 3)
        {
          constexpr int fq = g >> 4, fi = g & 15;
          sp[1][fq][fi] = v_exp1(v_fma1(sp[1][fq][fi], sl2, nm[fq]));
        }
        if constexpr (g >= 2) {
          constexpr int e = g - 2;
          v_add_ip((e >> 4) ? rs1 : rs0, sp[1][e >> 4][e & 15]);
        }
        if constexpr (g >= 4 && (g & 1) == 0) {
          constexpr int e = g - 4, pq = e >> 4, ei = e & 15;
          pw[1][pq][ei >> 3][(ei & 7) >> 1] = cvt_pk(sp[1][pq][ei], sp[1][pq][ei + 1]);
        }
        if constexpr (g == 30) {  // the first V^T fragments of phase B
          vr[0] = read_v(vsl, 0, 0, 0);
          vr[1] = read_v(vsl, 0, 0, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      // the tail: scores 30, 31 into the sum, pairs 28 and 30 (a VALU pad after the last exp)
      asm volatile("s_nop 1");
      v_add_ip(rs1, sp[1][1][14]);
      v_add_ip(rs1, sp[1][1][15]);
      pw[1][1][1][2] = cvt_pk(sp[1][1][12], sp[1][1][13]);
      pw[1][1][1][3] = cvt_pk(sp[1][1][14], sp[1][1][15]);
      l[0] += rs0;
      l[1] += rs1;
      // the asm MFMAs are invisible to hipcc's hazard recognizer: XDL write -> VALU read (and VALU write ->
      // MFMA operand read) wait states before the next phase touches their registers
      asm volatile("s_nop 7\n\ts_nop 7");
      __builtin_amdgcn_sched_barrier(0);
    };

    // phase B of tile t: O^T += V^T(t-1) P^T(t-1) || start the softmax of tile t in sc (mask, row max,
    // defer-max decision, exps + row sums of the first key half, its bf16 P into pw[0] once the P.V MFMAs of
    // tile t-1 no longer read that half); K(t+1) into the accumulator file (a stale slot past the last tile is
    // read and never used). `dummy`: the drain step past the wave's last tile, whose scores are all masked.
    // Returns the first half's row sums (added to l after a rescale)
    auto phase_b = [&](f32v16 (&sc)[2][2], int vsl, bfv8 (&vr)[16], int t, bool dummy, float (&rsn)[2]) {
      const int n0 = kv_beg + t * BN;
      const bool need_mask = dummy || (a.causal && n0 + BN - 1 > qw) || (a.window >= 0 && n0 < qw + 63 - a.window) ||
                             n0 + BN > S || qw + 63 >= S;
      if (need_mask) {  // diagonal / window / sequence-end tiles: out-of-range keys -> -inf
        const IdxRange r0 = dummy ? IdxRange{1u, 0u} : idx_range(klo0, khi0, n0 + 4 * hh);
        const IdxRange r1 = dummy ? IdxRange{1u, 0u} : idx_range(klo1, khi1, n0 + 4 * hh);
        sfor<32>([&](auto ec) {
          constexpr int e = decltype(ec)::value, kh = e >> 4, i = e & 15;
          constexpr int o = 32 * kh + 8 * (i >> 2) + (i & 3);
          sc[kh][0][i] = range_or_ninf<o>(sc[kh][0][i], r0.base, r0.span);
          sc[kh][1][i] = range_or_ninf<o>(sc[kh][1][i], r1.base, r1.span);
        });
      }
      __builtin_amdgcn_sched_barrier(0);
      float mx[2] = {0.f, 0.f}, mxa[2] = {0.f, 0.f}, mxb[2] = {0.f, 0.f}, u1 = 0.f, u2 = 0.f, u3 = 0.f;
      rsn[0] = rsn[1] = 0.f;
      sfor<32>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        // MFMA g: V^T fragment f = g / 2 (k-step f / 4 = (key half, s2), d tile f % 4), query half g % 2
        constexpr int f = g >> 1, ks = f >> 2, dt = f & 3, qh = g & 1;
        {
          const uint32_t(&pp)[4] = pw[ks >> 1][qh][ks & 1];
          const u32x4 pb = {pp[0], pp[1], pp[2], pp[3]};
          asm volatile("v_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                       :: "i"(fa4_ao(dt, qh)), "i"(fa4_ao(dt, qh) + 15), "v"(vr[f]), "v"(pb));
        }
        if constexpr (qh == 0 && f + 2 < 16) {  // fragment f + 2, three MFMAs ahead of its first use
          constexpr int f2 = f + 2, k2 = f2 >> 2;
          vr[f2] = read_v(vsl, k2 >> 1, k2 & 1, f2 & 3);
        }
        if constexpr (g < 9) {  // row maxima: 32 scores per query half, 8 per gap in three independent max3,
          // folded into two running maxima one gap later
          if constexpr (g >= 1) {
            constexpr int q2 = (g - 1) >> 2;
            mxa[q2] = (((g - 1) & 3) == 0) ? vmax3(u1, u2, u2) : vmax3(mxa[q2], u1, u2);
            mxb[q2] = (((g - 1) & 3) == 0) ? u3 : fmaxf(mxb[q2], u3);
          }
          if constexpr (g < 8) {
            constexpr int q2 = g >> 2, part = g & 3, k2 = part >> 1, i0 = (part & 1) * 8;
            u1 = vmax3(sc[k2][q2][i0], sc[k2][q2][i0 + 1], sc[k2][q2][i0 + 2]);
            u2 = vmax3(sc[k2][q2][i0 + 3], sc[k2][q2][i0 + 4], sc[k2][q2][i0 + 5]);
            u3 = vmax3(sc[k2][q2][i0 + 6], sc[k2][q2][i0 + 7], sc[k2][q2][i0 + 7]);
          }
        }
        if constexpr (g == 9) {  // both lane halves' maxima, then the defer-max decision
#pragma unroll
          for (int q2 = 0; q2 < 2; ++q2) {
            mx[q2] = fmaxf(mxa[q2], mxb[q2]);
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx[q2]), __float_as_uint(mx[q2]),
                                                            false, false);
            mx[q2] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * sl2;
          }
          resc = __any(mx[0] > m[0] + kThr || mx[1] > m[1] + kThr);
#pragma unroll
          for (int q2 = 0; q2 < 2; ++q2) {
            const float mnew = resc ? fmaxf(m[q2], mx[q2]) : m[q2];
            alpha[q2] = (mnew == -INFINITY || mnew == m[q2]) ? 1.f : fexp2(m[q2] - mnew);
            m[q2] = mnew;
            nm[q2] = (mnew == -INFINITY) ? 0.f : -mnew;
          }
        }
        if constexpr (g >= 10) {  // exps of the first key half: 32 scores over gaps 10 .. 31; row sums 2 gaps later
          constexpr int n = fa4_nexp(g), e0 = fa4_exp0(g);
          sfor<n>([&](auto jc) {
            constexpr int s = e0 + decltype(jc)::value, sq = s >> 4, si = s & 15;
            sc[0][sq][si] = v_exp1(v_fma1(sc[0][sq][si], sl2, nm[sq]));
          });
        }
        if constexpr (g >= 12) {
          constexpr int n = fa4_nexp(g - 2), e0 = fa4_exp0(g - 2);
          sfor<n>([&](auto jc) {
            constexpr int s = e0 + decltype(jc)::value, sq = s >> 4, si = s & 15;
            v_add_ip(rsn[sq], sc[0][sq][si]);
          });
        }
        // bf16 pair p = g - 18 of the first half (its exps done, tile t-1's first-half P no longer read)
        if constexpr (g >= 18) {
          constexpr int p = g - 18, s = 2 * p, sq = s >> 4, si = s & 15;
          pw[0][sq][si >> 3][(si & 7) >> 1] = cvt_pk(sc[0][sq][si], sc[0][sq][si + 1]);
        }
        if constexpr (g >= 4 && g < 12) read_k((t + 1) & 3, std::integral_constant<int, g - 4>{});
        __builtin_amdgcn_sched_barrier(0);
      });
      asm volatile("s_nop 1");  // the last exps -> their row-sum adds and packs
      sfor<4>([&](auto jc) {  // row sums of the last two gaps' scores (28 .. 31)
        constexpr int s = 28 + decltype(jc)::value;
        v_add_ip(rsn[1], sc[0][1][s - 16]);
      });
      pw[0][1][1][2] = cvt_pk(sc[0][1][12], sc[0][1][13]);
      pw[0][1][1][3] = cvt_pk(sc[0][1][14], sc[0][1][15]);
    };

    // the rare rescale of O^T (a[0:127]) after phase B: every P at the old max is in it, none at the new one
    auto rescale = [&]() {
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // the last P.V MFMAs' results
      // (tile t-1's P is all in O^T: phase B issued its last P.V MFMA before this)
      sfor<8>([&](auto tc) {
        constexpr int tile = decltype(tc)::value, qh = tile & 1;
        sfor<16>([&](auto ic) {
          constexpr int reg = tile * 16 + decltype(ic)::value;
          float x;
          asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(reg));
          x *= alpha[qh];
          asm volatile("v_accvgpr_write_b32 a%c1, %0" :: "v"(x), "i"(reg));
        });
      });
      asm volatile("s_nop 3" ::: "memory");  // accumulator write -> MFMA C read
      l[0] *= alpha[0];
      l[1] *= alpha[1];
    };
    auto finish_step = [&]() {
      wait_vm<0>();  // this wave's DMA of tile t + 2
      ring_barrier();
    };
    // a step with nothing to compute for this wave: its share of the ring traffic only
    auto step_idle = [&](int t) {
      if (t + 2 < T) issue(t + 2);
      sfor<8>([&](auto kc) { read_k((t + 1) & 3, kc); });
      finish_step();
    };
    // a compute step; sc = tile t's score set, sp = tile t-1's
    auto step = [&](f32v16 (&sc)[2][2], f32v16 (&sp)[2][2], int t) {
      if (t + 2 < T) issue(t + 2);
      bfv8 vr[16];
      float rsn[2];
      phase_a(sc, sp, (t - 1) & 3, vr);
      phase_b(sc, (t - 1) & 3, vr, t, t > wt1, rsn);
      if (resc) rescale();
      l[0] += rsn[0];  // tile t's first-half row sums, at the new scale
      l[1] += rsn[1];
      finish_step();
    };

    int t = 0;
    if (wt0 <= wt1) {
      for (; t < wt0; ++t) step_idle(t);
      // steps wt0 .. wt1 + 1 (the last one drains P.V of tile wt1), score sets alternating A, B
      for (; t <= wt1 + 1; t += 2) {
        step(sA, sB, t);
        if (t + 1 <= wt1 + 1) step(sB, sA, t + 1);
      }
      t = wt1 + 2;
    }
    for (; t <= T; ++t) step_idle(t);
  }
  // the last asm MFMAs' results are read by the epilogue
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

  sfor<2>([&](auto qc) {
    constexpr int qh = decltype(qc)::value;
    const float lt = l[qh] + __shfl_xor(l[qh], 32, 64);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    uint2 w[16];
    sfor<4>([&](auto dc) {
      constexpr int dt = decltype(dc)::value;
      float ov[16];
      sfor<16>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        float x;
        asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(fa4_ao(dt, qh) + i));
        ov[i] = x;
      });
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        w[4 * dt + c].x = pack_bf16x2(ov[4 * c] * inv, ov[4 * c + 1] * inv);
        w[4 * dt + c].y = pack_bf16x2(ov[4 * c + 2] * inv, ov[4 * c + 3] * inv);
      }
    });
    widen_pairs(w);
    const int q = qh ? qrow1 : qrow0;
    if (q < S) {
      store_pairs(a.out + (int64_t)b * a.o_sb + (int64_t)q * a.o_ss + (int64_t)h * a.o_sh + 8 * hh, w);
      if (hh == 0) {
        const float mu = (m[qh] == -INFINITY) ? 0.f : m[qh];
        a.lse[((int64_t)b * a.Hq + h) * S + q] = lt > 0.f ? (mu + __log2f(lt)) * kLn2 : -INFINITY;
      }
    }
  });
}
// ============================================================================ backward dK/dV, v6
// 64 keys per wave (two 32-key halves), dV^T and dK^T of both halves in the 256 accumulator registers
// (asm-owned, like fa_fwd4: a[0:127] dV^T, a[128:255] dK^T). Every operand fragment read from LDS (Q / dO
// rows, Q^T / dO^T transposed) feeds the two halves' MFMAs back to back, so a tile needs 1.1 LDS reads per
// MFMA against fa_bwd_dkdv5's 1.75, and a 256-key workgroup of 4 waves moves each Q / dO tile through the
// LDS-DMA ring for twice the keys (cdna guide, 'Attention backward': 64 keys per wave in 256 accumulator
// registers). The wave's K fragments stay in VGPRs (64 registers); V of the workgroup's 256 keys sits in LDS
// (a 64 KB swizzled image, the dP operand) next to a 5-slot Q / dO ring (tiles issued 3 ahead). Per 32-row
// query tile t, four phases of 16 MFMAs:
//   1  S(t), both halves (one accumulation chain each, interleaved per k-step: one Q row read per pair)
//                                          || dS(t-1) of k-step 1 and its bf16 pairs
//   2  dP(t), both halves                  || P = exp2(S scale log2e - lse log2e) of k-step 0, bf16 pairs
//   3  dK(t-1) from Q^T(t-1) and dS(t-1)   || P of k-step 1, bf16 pairs
//      (ring wait + barrier: tile t+1 landed, tile t-1's slot free)
//   4  dV(t) from dO^T(t) and P(t)         || dS(t) of k-step 0 and its bf16 pairs
// (diagnostic probes with everything but the MFMAs and the packs removed put the MFMA floor of this loop at
// ~55 % of its time: the softmax VALU must spread over all four phases to hide under the MFMAs)
// The fp32 scores of both halves (S / P, dP / dS: 64 registers) live from phase 1 to phase 4; the bf16 P and
// dS operands (32 registers) from their pack to their MFMAs. Operand reads run two to three MFMAs ahead (LDS
// latency under load); one accumulation chain needs no interleaving for throughput (MI355X_MICROARCH: 32
// cycles back to back on one accumulator). Dense rows only (D = 128, causal / window, no segments).
constexpr int d6_av(int h, int dt) { return (h * 4 + dt) * 16; }        // dV^T accumulator (key half, d tile)
constexpr int d6_ak(int h, int dt) { return 128 + (h * 4 + dt) * 16; }  // dK^T accumulator

template <int D = 128, int PF = 3, int PR = 0, bool DI = false>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv6_kernel(AttnArgs a, const float* ld) {
  static_assert(D == 128, "fa_bwd_dkdv6 is the D = 128 kernel");
  constexpr int NKK = 8, NDT = 4, NB = 16;
  constexpr int BM = 32, IMG = BM * 256, SLOT = 2 * IMG + 512, NS = 5, NDMA = 5;
  constexpr int VIMG = 256 * 256;  // V of the workgroup's 256 keys
  using QI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[VIMG + NS * SLOT];
  char* const ring = smem + VIMG;

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = a.S, grp = a.Hq / a.Hkv;
  int L = (int)blockIdx.x;
  const int hk = L % a.Hkv;
  L /= a.Hkv;
  int b, kb;
  block_of(a, L, (S + 255) / 256, false, b, kb);
  const int ks = kb * 256, kw = ks + wid * 64;
  const int nT = (S + 31) / 32;
  const float sl2 = a.scale * kLog2e;

  // dV^T = dK^T = 0; the clobbers claim all 256 accumulator registers for the kernel descriptor, so hipcc
  // neither allocates nor spills into them
  asm volatile("s_nop 0" ::: LLMT_ACLOB);
  sfor<256>([&](auto ic) __attribute__((always_inline)) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(ic)::value)); });

  // the wave's K fragments (lane: key kw + 32 h + r, columns 16 kk + 8 hh ..), rows past S read as zeros
  bfv8 kf[2][NKK];
  {
    const bf16* kp = a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int key = kw + 32 * h + r;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) kf[h][kk] = gload8(kp + (int64_t)min(key, S - 1) * a.k_ss + kk * 16 + hh * 8, key < S);
    }
  }
  // the block's query tiles (dense rows: the range masks' query intervals are recomputed where a tile needs them)
  const int q_beg = a.causal ? ks : 0;
  const int q_end = a.window >= 0 ? min(S, ks + 256 + a.window) : S;
  const int nq = q_end > q_beg ? (q_end - q_beg + BM - 1) / BM : 0;
  const int T = nq * grp;
  // hipcc does not count the asm DMAs: retire its own loads before the first one is issued
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(kf[0][kk]), "+v"(kf[1][kk]));

  if (T > 0) {
    // per-lane DMA offsets, recomputed per tile (a handful of VALU ops beside the MFMAs; held across the loop they
    // cost five of the registers the pipeline needs)
    auto dma_offs = [&](int (&dq)[2], int (&dd)[2], int& dl) __attribute__((always_inline)) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int row = 8 * wid + 4 * n + (lane >> 4);
        const int ch = (lane & 15) ^ QI::swz(row);
        dq[n] = (row * a.q_ss + ch * 8) * 2;
        dd[n] = (row * a.d_ss + ch * 8) * 2;
      }
      dl = ((wid & 1) * 64 + lane) * 4;
    };
    const int64_t q_rows = S - q_beg;
    const int64_t nrec_q = ((q_rows - 1) * a.q_ss + D) * 2, nrec_d = ((q_rows - 1) * a.d_ss + D) * 2;
    const int64_t nrec_l = (int64_t)nq * kLdTile * 4;
    const bf16* qh0 = a.q + (int64_t)b * a.q_sb + (int64_t)(hk * grp) * a.q_sh + (int64_t)q_beg * a.q_ss;
    const bf16* dh0 = a.dout + (int64_t)b * a.d_sb + (int64_t)(hk * grp) * a.d_sh + (int64_t)q_beg * a.d_ss;
    const float* lh0 = ld + (((int64_t)b * a.Hq + hk * grp) * nT + (q_beg >> 5)) * kLdTile;
    const int step_q = BM * a.q_ss * 2, step_d = BM * a.d_ss * 2;
    Rsrc qrs = make_rsrc4(qh0, nrec_q), drs = make_rsrc4(dh0, nrec_d), lrs = make_rsrc4(lh0, nrec_l);
    int iss_g = 0, iss_q = 0, iss_n = 0, toff_q = 0, toff_d = 0, toff_l = 0;
    // one tile's DMA into ring slot `sl`; past the last tile the last one is loaded again (every iteration
    // issues the same number of pieces, so one counted wait fits every iteration)
    auto issue = [&](int sl) __attribute__((always_inline)) {
      const char* q0 = ring + sl * SLOT + 8 * wid * 256;
      int dq_off[2], dd_off[2], ld_off;
      dma_offs(dq_off, dd_off, ld_off);
      asm volatile("" : "+v"(dq_off[0]), "+v"(dq_off[1]), "+v"(dd_off[0]), "+v"(dd_off[1]), "+v"(ld_off));
      dma_tile5(qrs, drs, lrs, q0, q0 + 4 * 256, q0 + IMG, q0 + IMG + 4 * 256, ring + sl * SLOT + 2 * IMG + (wid & 1) * 256,
                dq_off[0] + toff_q, dq_off[1] + toff_q, dd_off[0] + toff_d, dd_off[1] + toff_d, ld_off + toff_l);
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
    // tiles 0 .. NS-3, then V of the workgroup's keys (16 pieces of 4 rows per wave, swizzled like QI)
#pragma unroll
    for (int t = 0; t < NS - 2; ++t) issue(t);
    {
      const Rsrc vrs = make_rsrc4(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh + (int64_t)ks * a.v_ss,
                                  S > ks ? ((int64_t)(S - 1 - ks) * a.v_ss + D) * 2 : 0);
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        const int row = 64 * wid + 4 * n + (lane >> 4);
        const int ch = (lane & 15) ^ QI::swz(row);
        dma16(vrs, smem + (64 * wid + 4 * n) * 256, (row * a.v_ss + ch * 8) * 2);
      }
    }
    wait_vm<0>();
    ring_barrier();

    // LDS offsets: row reads of k-step kk at ro0 ^ (32 kk) (the swizzle moves 16-byte chunks within bits 4-7
    // of the offset, disjoint from the row's bits), transposed reads of d tile dt at to0[x] ^ (64 dt)
    const int ro0 = QI::roff(r, hh);
    int to0[2];
    {
      const int g = lane >> 4, i16 = lane & 15;
      const int row = 4 * (g >> 1) + (i16 >> 2), col = 16 * (g & 1) + 4 * (i16 & 3);
      to0[0] = QI::toff(BM, row, col);
      to0[1] = QI::toff(BM, row + 8, col);
    }
    const char* vimg = smem + 64 * wid * 256;
    auto rd_q = [&](int sl, int kk) __attribute__((always_inline)) {
      if constexpr (PR & 8) return kf[1][kk & 7];
      return lds_b128(ring + sl * SLOT + (ro0 ^ (32 * kk)));
    };
    auto rd_d = [&](int sl, int kk) __attribute__((always_inline)) {
      if constexpr (PR & 8) return kf[0][kk & 7];
      return lds_b128(ring + sl * SLOT + IMG + (ro0 ^ (32 * kk)));
    };
    auto rd_v = [&](int h, int kk) __attribute__((always_inline)) {
      if constexpr (PR & 8) return kf[h][(kk + 1) & 7];
      return lds_b128(vimg + 32 * 256 * h + (ro0 ^ (32 * kk)));
    };
    // transposed fragment i of a dV / dK phase: i < 8 -> dO^T (dV product), else Q^T (dK); s2 = (i / 4) & 1
    auto rd_t = [&](int sl, int i) __attribute__((always_inline)) -> bfv8 {
      if constexpr (PR & 8) return kf[i & 1][i & 7];
      const int s2 = (i / NDT) & 1, dt = i % NDT;
      const char* base = ring + sl * SLOT + (i < 2 * NDT ? IMG : 0) + 4096 * s2;
      const s16v4 lo = lds_tr(base + (to0[0] ^ (64 * dt))), hi = lds_tr(base + (to0[1] ^ (64 * dt)));
      return __builtin_bit_cast(bfv8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };

    f32v16 sc[2], dc[2];       // S and dP - delta of both key halves (the MFMA chains' accumulators)
    f32v16 cdc;                // DI: -delta of the lane's 16 query rows, the dP chains' initial accumulator
    const float* nds = nullptr;  // !DI: -delta of the tile whose dS is computed (LDS)
    float pv[2][16], dsv[2][16];  // P and dS element-wise (scalars: no vector re-assembly around the updates)
    u32x4 pw[2][2], dw[2][2];  // bf16 P / dS operands [key half][k-step]
    const float* lqs = nullptr;  // the tile's row constants in LDS: -lse log2e (floats 96 ..), -delta (32 ..)
    bfv8 qf[NKK], df[NKK], vf[2][NKK], tf[8];
    auto q0_of = [&](int t) __attribute__((always_inline)) { return q_beg + (t % nq) * BM; };
    auto need_mask = [&](int q0) __attribute__((always_inline)) {
      return (a.causal && q0 < kw + 63) || (a.window >= 0 && q0 + 31 - kw > a.window);
    };
    // exp element e of a tile (k-step e >> 4, half (e >> 3) & 1, value 8 k-step + (e & 7))
    // row constant pair of values v, v + 1 (v even): rows 8 (v >> 2) + 4 hh + (v & 3), adjacent floats
    auto cpair = [&](const float* base, int v) __attribute__((always_inline)) {
      return *reinterpret_cast<const float2*>(base + 8 * (v >> 2) + 4 * hh + (v & 3));
    };
    // exps of the element pair e, e + 1 (e even)
    auto ex2 = [&](auto ec) __attribute__((always_inline)) {
      constexpr int e = decltype(ec)::value, h = (e >> 3) & 1, v = 8 * (e >> 4) + (e & 7);
      if constexpr (PR & 4) return;
      const float2 l = cpair(lqs, v);
      float e0, e1;
      asm volatile("v_fma_f32 %0, %2, %4, %5\n\tv_fma_f32 %1, %3, %4, %6\n\tv_exp_f32 %0, %0\n\tv_exp_f32 %1, %1"
                   : "=&v"(e0), "=&v"(e1)
                   : "v"(pv[h][v]), "v"(pv[h][v + 1]), "v"(sl2), "v"(l.x), "v"(l.y));
      pv[h][v] = e0;
      pv[h][v + 1] = e1;
    };
    // dS = P (dP - delta) of the pair e, e + 1
    auto ds2 = [&](auto ec) __attribute__((always_inline)) {
      constexpr int e = decltype(ec)::value, h = (e >> 3) & 1, v = 8 * (e >> 4) + (e & 7);
      if constexpr (PR & 4) {
        dsv[h][v] = dc[h][v];
        dsv[h][v + 1] = dc[h][v + 1];
        return;
      }
      float t0, t1;
      if constexpr (DI) {  // dc already holds dP - delta (the dP chains start from -delta, see ph_s)
        asm volatile("v_mul_f32 %0, %2, %3\n\tv_mul_f32 %1, %4, %5"
                     : "=&v"(t0), "=&v"(t1) : "v"(dc[h][v]), "v"(pv[h][v]), "v"(dc[h][v + 1]), "v"(pv[h][v + 1]));
      } else {
        const float2 n = cpair(nds, v);
        asm volatile("v_add_f32 %0, %2, %3\n\tv_add_f32 %1, %4, %5\n\tv_mul_f32 %0, %6, %0\n\tv_mul_f32 %1, %7, %1"
                     : "=&v"(t0), "=&v"(t1)
                     : "v"(dc[h][v]), "v"(n.x), "v"(dc[h][v + 1]), "v"(n.y), "v"(pv[h][v]), "v"(pv[h][v + 1]));
      }
      dsv[h][v] = t0;
      dsv[h][v + 1] = t1;
    };
    // bf16 pair w of a tile's operands (k-step w >> 3, half (w >> 2) & 1, word w & 3)
    auto pk_p = [&](auto wc) __attribute__((always_inline)) {
      constexpr int w = decltype(wc)::value, s2 = w >> 3, h = (w >> 2) & 1, j = w & 3, v = 8 * s2 + 2 * j;
      pw[h][s2][j] = cvt_pk(pv[h][v], pv[h][v + 1]);
    };
    auto pk_d = [&](auto wc) __attribute__((always_inline)) {
      constexpr int w = decltype(wc)::value, s2 = w >> 3, h = (w >> 2) & 1, j = w & 3, v = 8 * s2 + 2 * j;
      dw[h][s2][j] = cvt_pk(dsv[h][v], dsv[h][v + 1]);
    };
    auto consts_of = [&](int sl, int off) __attribute__((always_inline)) {
      return reinterpret_cast<const float*>(ring + sl * SLOT + 2 * IMG) + off;
    };
    // phase 1: S(t) of both halves (tile in slot sl; Q rows 0, 1 prefetched), the dP operands' first k-steps
    // and -lse log2e fetched in its gaps
    auto ph_s = [&](int sl, auto&& valu) __attribute__((always_inline)) {
      lqs = consts_of(sl, 96);
      sfor<16>([&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value, kk = g >> 1, h = g & 1;
        valu(gc);
        if constexpr (kk == 0)
          if constexpr (PR & 64) asm volatile("" : "=&v"(sc[h]) : "v"(qf[0]), "v"(kf[h][0]));
          else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(sc[h]) : "v"(qf[0]), "v"(kf[h][0]));
        else
          if constexpr (PR & 64) asm volatile("" : "+v"(sc[h]) : "v"(qf[kk]), "v"(kf[h][kk]));
          else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(sc[h]) : "v"(qf[kk]), "v"(kf[h][kk]));
        if constexpr (h == 0 && kk + 2 < NKK) qf[kk + 2] = rd_q(sl, kk + 2);
        if constexpr (DI && g >= 14) {  // -delta of the tile's rows (floats 32 ..): the dP chains' initial value
#pragma unroll
          for (int c = 2 * (g - 14); c < 2 * (g - 13); ++c) {
            const float4 x = *reinterpret_cast<const float4*>(consts_of(sl, 32) + 8 * c + 4 * hh);
            cdc[4 * c] = x.x; cdc[4 * c + 1] = x.y; cdc[4 * c + 2] = x.z; cdc[4 * c + 3] = x.w;
          }
        }
        if constexpr (g >= 13) {  // dP operands of k-step 0: dO row, V of both halves
          constexpr int y = g - 13;
          if constexpr (y == 0) df[0] = rd_d(sl, 0);
          else vf[y - 1][0] = rd_v(y - 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    // VALU of the four phases (P and dS of a tile spread over all of them; one exp pair, dS pair or two packs
    // per gap beside the MFMA and its operand reads):
    //   phase 1 (S(t)):        dS of tile t-1, k-step 1 (gaps 0 .. 7), its bf16 pairs (2 .. 9)
    //   phase 2 (dP(t)):       exps 0 .. 15 (gaps 2 .. 9), P k-step 0 (10 .. 15)
    //   phase 3 (dK(t-1)):     exps 16 .. 31 (gaps 0 .. 7), P k-step 1 (8 .. 15)
    //   phase 4 (dV(t)):       dS k-step 0 (gaps 0 .. 7), its bf16 pairs (8 .. 15)
    auto v1 = [&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g < 8) ds2(std::integral_constant<int, 16 + 2 * g>{});
      if constexpr (g >= 2 && g < 10) pk_d(std::integral_constant<int, g + 6>{});  // words 8 .. 15, a gap behind
    };
    auto v3 = [&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g < 8) ex2(std::integral_constant<int, 16 + 2 * g>{});
      else pk_p(std::integral_constant<int, g>{});
    };
    auto v4 = [&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      if constexpr (g < 8) ds2(std::integral_constant<int, 2 * g>{});
      else pk_d(std::integral_constant<int, g - 8>{});
    };
    // phase 2: dP(t) of both halves || exps 0 .. 19 (from gap 2: two MFMAs behind the last S MFMA, the
    // XDL-write -> VALU-read wait states), P k-step 0 packed; MSK: the range mask on every score first
    auto ph_dp = [&](auto mc, int sl, int q0) __attribute__((always_inline)) {
      constexpr bool MSK = decltype(mc)::value;
      sfor<16>([&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value, kk = g >> 1, h = g & 1;
        if constexpr (kk == 0)
          if constexpr (DI)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(dc[h]) : "v"(df[0]), "v"(vf[h][0]), "v"(cdc));
          else
            if constexpr (PR & 64) asm volatile("" : "=&v"(dc[h]) : "v"(df[0]), "v"(vf[h][0]));
            else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(dc[h]) : "v"(df[0]), "v"(vf[h][0]));
        else
          if constexpr (PR & 64) asm volatile("" : "+v"(dc[h]) : "v"(df[kk]), "v"(vf[h][kk]));
          else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(dc[h]) : "v"(df[kk]), "v"(vf[h][kk]));
        // next k-step's operands one k-step (two MFMAs) ahead: deeper would not fit the register file
        if constexpr (h == 0 && kk + 1 < NKK) df[kk + 1] = rd_d(sl, kk + 1);
        if constexpr (kk + 1 < NKK) vf[h][kk + 1] = rd_v(h, kk + 1);
        if constexpr (g == 1) {  // the scores as scalars; MSK: out-of-range queries -> -inf (P = 0, dS = 0)
          sfor<2>([&](auto hc) __attribute__((always_inline)) {
            constexpr int hm = decltype(hc)::value;
            if constexpr (MSK) {
              int qlo, qhi;
              query_interval(a, b, kw + 32 * hm + r, qlo, qhi);
              const IdxRange rg = idx_range(qlo, qhi, q0 + 4 * hh);
              sfor<16>([&](auto vc) __attribute__((always_inline)) {
                constexpr int v = decltype(vc)::value, o = 8 * (v >> 2) + (v & 3);
                pv[hm][v] = range_or_ninf<o>(sc[hm][v], rg.base, rg.span);
              });
            } else {
#pragma unroll
              for (int v = 0; v < 16; ++v) pv[hm][v] = sc[hm][v];
            }
          });
        }
        if constexpr (!(PR & 16)) {
          if constexpr (g >= 2 && g < 10) ex2(std::integral_constant<int, 2 * (g - 2)>{});  // exps 0 .. 15
          if constexpr (g >= 10) {  // P k-step 0
            pk_p(std::integral_constant<int, g - 10>{});
            if constexpr (g >= 14) pk_p(std::integral_constant<int, g - 8>{});
          }
        }
        if constexpr (PR & 32) {  // probe: phases 3 and 4's VALU here too
          v3(gc);
          v4(gc);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    // phases 3 / 4: dK (KQ = true: Q^T fragments, dS operands) or dV (dO^T, P) of both halves from the slot
    // `sl` (transposed fragments 0, 1 prefetched), || valu(gap); `qsl` >= 0: the next tile's first Q rows at
    // gaps 14, 15
    auto ph_g = [&](auto kc, int sl, auto&& valu, int qsl) __attribute__((always_inline)) {
      constexpr bool KQ = decltype(kc)::value;
      sfor<16>([&](auto gc) __attribute__((always_inline)) {
        constexpr int i = decltype(gc)::value, f = i >> 1, h = i & 1, s2 = f >> 2, dt = f & 3;
        if constexpr (PR & 64)
          asm volatile("" :: "v"(tf[f]), "v"(KQ ? dw[h][s2] : pw[h][s2]));
        else if constexpr (KQ)
          asm volatile("v_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                       :: "i"(d6_ak(h, dt)), "i"(d6_ak(h, dt) + 15), "v"(tf[f]), "v"(dw[h][s2]));
        else
          asm volatile("v_mfma_f32_32x32x16_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
                       :: "i"(d6_av(h, dt)), "i"(d6_av(h, dt) + 15), "v"(tf[f]), "v"(pw[h][s2]));
        if constexpr (h == 0 && f + 2 < 8) tf[f + 2] = rd_t(sl, (KQ ? 8 : 0) + f + 2);
        valu(gc);
        if constexpr (i >= 14) {
          if (qsl >= 0) qf[i - 14] = rd_q(qsl, i - 14);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    auto pref_t = [&](int sl, bool kq) __attribute__((always_inline)) {
      tf[0] = rd_t(sl, kq ? 8 : 0);
      tf[1] = rd_t(sl, kq ? 9 : 1);
    };
    auto dp = [&](int sl, int q0) __attribute__((always_inline)) {
      if (need_mask(q0))
        ph_dp(std::true_type{}, sl, q0);
      else
        ph_dp(std::false_type{}, sl, q0);
    };
    auto no_valu = [](auto) __attribute__((always_inline)) {};

    int sl_c = 0;  // ring slot of tile t
    qf[0] = rd_q(0, 0);
    qf[1] = rd_q(0, 1);
    {  // tile 0: phase 3 without dK(t-1)
      const int q0 = q0_of(0);
      issue(NS - 2);
      ph_s(0, no_valu);
      dp(0, q0);
      nds = consts_of(0, 32);
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // no MFMA between dP's chains and their reads
      sfor<16>([&](auto gc) __attribute__((always_inline)) { v3(gc); });
      pref_t(0, false);
      wait_vm<2 * NDMA>();
      ring_barrier();
      ph_g(std::false_type{}, 0, v4, T > 1 ? 1 % NS : -1);
    }
    for (int t = 1; t < T; ++t) {
      const int sl_p = sl_c;
      sl_c = sl_c + 1 == NS ? 0 : sl_c + 1;
      const int q0 = q0_of(t);
      if constexpr (!(PR & 1)) issue(sl_c + NS - 2 >= NS ? sl_c - 2 : sl_c + NS - 2);
      if constexpr (PR & 16) ph_s(sl_c, no_valu);
      else ph_s(sl_c, v1);  // with dS(t-1) k-step 1 (nds still tile t-1's)
      dp(sl_c, q0);
      pref_t(sl_p, true);
      nds = consts_of(sl_c, 32);  // -delta of tile t, whose dS phases 4 and 1 compute
      if constexpr (PR & 16) {  // probe: every VALU of the tile beside the accumulator-destination MFMAs
        ph_g(std::true_type{}, sl_p, [&](auto gc) __attribute__((always_inline)) {
          constexpr int g = decltype(gc)::value;
          v1(gc);
          v3(gc);
          if constexpr (g < 8) ex2(std::integral_constant<int, 2 * g>{});
          else pk_p(std::integral_constant<int, g - 8>{});
        }, -1);
      } else if constexpr (PR & 32) {
        ph_g(std::true_type{}, sl_p, no_valu, -1);
      } else {
        ph_g(std::true_type{}, sl_p, v3, -1);
      }
      pref_t(sl_c, false);
      if constexpr (PR & 1) {
        wait_vm<0>();
      } else {
        wait_vm<2 * NDMA>();  // tile t + 1 (issued three iterations ago) landed; slot t - 1 read for the last time
      }
      if constexpr (!(PR & 2)) ring_barrier();
      const int sl_n = sl_c + 1 == NS ? 0 : sl_c + 1;
      if constexpr (PR & 32) ph_g(std::false_type{}, sl_c, no_valu, t + 1 < T ? sl_n : -1);
      else ph_g(std::false_type{}, sl_c, v4, t + 1 < T ? sl_n : -1);
    }
    {  // drain: dS k-step 1 and dK of the last tile
      sfor<16>([&](auto gc) __attribute__((always_inline)) { v1(gc); });
      pref_t(sl_c, true);
      asm volatile("s_nop 7" ::: "memory");  // the last packs -> MFMA operand reads
      ph_g(std::true_type{}, sl_c, no_valu, -1);
    }
    wait_vm<0>();  // no LDS-DMA may outlive the workgroup
  }
  // the last asm MFMAs' accumulator writes -> the reads below
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32v16 dkt[NDT], dvt[NDT];
    sfor<NDT>([&](auto dc_) __attribute__((always_inline)) {
      constexpr int dt = decltype(dc_)::value;
      sfor<16>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        float x, y;
        if (h == 0) {
          asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(d6_ak(0, dt) + i));
          asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(y) : "i"(d6_av(0, dt) + i));
        } else {
          asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(d6_ak(1, dt) + i));
          asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(y) : "i"(d6_av(1, dt) + i));
        }
        dkt[dt][i] = x;
        dvt[dt][i] = y;
      });
    });
    const int kr = kw + 32 * h + r;
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
}

#undef LLMT_ACLOB

// ============================================================================ forward, head-chained
// fa_fwd3 with NH query heads per workgroup (same batch row and query block, so the same key-tile range,
// masks and segment runs): the NH heads' tiles form one sequence through the K/V LDS-DMA ring, so the
// first tile of head j+1 is in flight under the last tile of head j and its Q fragments are loaded there
// too; head j's O / LSE are written at the boundary. A block then pays the prologue (Q + first K/V tile
// latency with nothing to hide it) once per NH heads: that fixed cost is ~6.5 tiles' worth per block,
// the whole kernel at short sequences / packed documents (profiles/r3_attention_bwd_atomic_floor.md).
// Grid: ceil(S/128) * (Hq / NH) * B blocks, head chains fastest, heaviest query blocks first.
template <int D, int NH>
__global__ __launch_bounds__(256, 2) void fa_fwd3c_kernel(AttnArgs a) {
  constexpr int NKK = D / 16, NDT = D / 32;
  constexpr int BN = 64, IMG = BN * 256, SLOT = 2 * IMG + 256;
  using KI = Img<128>;
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = a.S, grp = a.Hq / a.Hkv;
  const int nqb = (S + 127) / 128;
  int L = (int)blockIdx.x;
  int h0;
  if (grp % NH == 0) {  // GQA: kv head fastest (the blocks of one XCD share a kv head's K/V in its L2)
    const int hk = L % a.Hkv;
    L /= a.Hkv;
    h0 = hk * grp + (L % (grp / NH)) * NH;
    L /= grp / NH;
  } else {  // chains span kv heads (MHA): consecutive heads
    const int nch = a.Hq / NH;
    h0 = (L % nch) * NH;
    L /= nch;
  }
  int b, mb;
  block_of(a, L, nqb, true, b, mb);
  const int qs = mb * 128, qw = qs + wid * 32, qrow = qw + r;
  const float sl2 = a.scale * kLog2e;
  int sq = (a.seg && qrow < S) ? a.seg[(int64_t)b * S + qrow] : -2;

  auto load_q = [&](int h, bfv8 (&qd)[NKK]) {
    const bf16* qp = a.q + (int64_t)b * a.q_sb + (int64_t)h * a.q_sh;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) qd[kk] = gload8(qp + (int64_t)min(qrow, S - 1) * a.q_ss + kk * 16 + hh * 8, qrow < S);
  };
  bfv8 qf[NKK];
  load_q(h0, qf);
  // hipcc does not count the asm DMAs: retire its own loads before the first one is issued
  asm volatile("" : "+v"(sq));
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(qf[kk]));
  f32v16 ot[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) ot[dt][i] = 0.f;
  float m = -INFINITY, l = 0.f;

  // O / LSE of head h from the running state, then the state reset for the next head
  auto finish = [&](int h) {
    const float lt = l + __shfl_xor(l, 32, 64);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    uint2 w[4 * NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        w[4 * dt + c].x = pack_bf16x2(ot[dt][4 * c] * inv, ot[dt][4 * c + 1] * inv);
        w[4 * dt + c].y = pack_bf16x2(ot[dt][4 * c + 2] * inv, ot[dt][4 * c + 3] * inv);
      }
    widen_pairs(w);
    if (qrow < S) {
      store_pairs(a.out + (int64_t)b * a.o_sb + (int64_t)qrow * a.o_ss + (int64_t)h * a.o_sh + 8 * hh, w);
      if (hh == 0) {
        const float mu = (m == -INFINITY) ? 0.f : m;
        a.lse[((int64_t)b * a.Hq + h) * S + qrow] = lt > 0.f ? (mu + __log2f(lt)) * kLn2 : -INFINITY;
      }
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) ot[dt][i] = 0.f;
    m = -INFINITY;
    l = 0.f;
  };

  const RunInfo qr = block_run(a, b, qs, min(qs + 127, S - 1));
  int kv_end = a.causal ? min(S, qs + 128) : S;
  if (!a.causal && a.rs) kv_end = min(kv_end, a.re[(int64_t)b * S + min(qs + 127, S - 1)] + 1);
  int kv_beg = a.window >= 0 ? max(0, qs - a.window) : 0;
  kv_beg = max(kv_beg, qr.rs) / BN * BN;
  const int T = kv_end > kv_beg ? (kv_end - kv_beg + BN - 1) / BN : 0;

  if (T == 0) {
#pragma unroll
    for (int j = 0; j < NH; ++j) finish(h0 + j);
    return;
  }
  // K/V descriptors of the chain head being fetched, rebuilt when the fetch moves to the next kv head;
  // records end with the last row's D elements (the 256-byte DMA rows of D < 128 read past a row -> zeros
  // instead of a fault)
  const int64_t krec = ((int64_t)(S - 1) * a.k_ss + D) * 2, vrec = ((int64_t)(S - 1) * a.v_ss + D) * 2;
  int fhk = h0 / grp;
  Rsrc krs = make_rsrc4(a.k + (int64_t)b * a.k_sb + (int64_t)fhk * a.k_sh, krec);
  Rsrc vrs = make_rsrc4(a.v + (int64_t)b * a.v_sb + (int64_t)fhk * a.v_sh, vrec);
  const Rsrc srs = make_rsrc4(a.seg ? a.seg + (int64_t)b * S : nullptr, a.seg ? (int64_t)S * 4 : 0);
  // tile u of the chain = tile u % T of head u / T, in ring slot u & 1
  auto issue = [&](int u, int j, int t) {
    const char* slot = smem + __builtin_amdgcn_readfirstlane((u & 1) * SLOT);
    const int n0 = kv_beg + t * BN;
    int vk[4], vv[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int row = 16 * wid + 4 * n + (lane >> 4);
      const int ch = (lane & 15) ^ KI::swz(row);
      vk[n] = ((n0 + row) * a.k_ss + ch * 8) * 2;
      vv[n] = ((n0 + row) * a.v_ss + ch * 8) * 2;
    }
    const int hk = (h0 + j) / grp;
    if (hk != fhk) {  // wave-uniform: a new kv head (MHA, or a chain crossing a GQA group)
      fhk = hk;
      krs = make_rsrc4(a.k + (int64_t)b * a.k_sb + (int64_t)hk * a.k_sh, krec);
      vrs = make_rsrc4(a.v + (int64_t)b * a.v_sb + (int64_t)hk * a.v_sh, vrec);
    }
    dma_tile9(krs, vrs, srs, slot + 16 * wid * 256, IMG, slot + 2 * IMG, vk, vv, (n0 + lane) * 4);
  };
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

  issue(0, 0, 0);
  wait_vm<0>();
  ring_barrier();
  int j = 0, t = 0;
  const int U = NH * T;
  for (int u = 0; u < U; ++u) {
    const char* slot = smem + __builtin_amdgcn_readfirstlane((u & 1) * SLOT);
    const int n0 = kv_beg + t * BN;
    const bool last = t == T - 1;
    if (u + 1 < U) {
      if (last)
        issue(u + 1, j + 1, 0);
      else
        issue(u + 1, j, t + 1);
    }
    bfv8 fr[16];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) fr[8 * tt + kk] = lds_b128(slot + 8192 * tt + ro[kk]);
    __builtin_amdgcn_sched_barrier(0);
    f32v16 st[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) st[tt][i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) st[tt] = mfma32(fr[8 * tt + kk], qf[kk], st[tt]);
    }
    // the next head's Q into the registers the S^T chain just consumed: the loads fly under the rest of
    // the tile (softmax, P.V)
    if (last && j + 1 < NH) load_q(h0 + j + 1, qf);
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
    const bool m_causal = a.causal && (n0 + BN - 1 > qw);
    const bool m_window = a.window >= 0 && (n0 < qw + 31 - a.window);
    const bool m_end = n0 + BN > S;
    const bool m_seg = seg_mask(a, qr, n0, n0 + BN - 1);
    if (m_causal || m_window || m_end || m_seg || qw + 31 >= S) {
      const int* Ss = reinterpret_cast<const int*>(slot + 2 * IMG);
      const int lim = qrow - n0 - 4 * hh, lo = qrow - a.window - n0 - 4 * hh, hi = S - 1 - n0 - 4 * hh;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          int4 sk = make_int4(sq, sq, sq, sq);
          if (m_seg) sk = *reinterpret_cast<const int4*>(Ss + 32 * tt + 8 * c + 4 * hh);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int ko = 32 * tt + 8 * c + jj;
            bool ok = (ko <= hi) && (qrow < S);
            if (a.causal) ok = ok && (ko <= lim);
            if (a.window >= 0) ok = ok && (ko >= lo);
            if (m_seg) ok = ok && ((&sk.x)[jj] == sq);
            if (!ok) st[tt][4 * c + jj] = -INFINITY;
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
    smax = fmaxf(smax, __shfl_xor(smax, 32, 64)) * sl2;
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
        st[tt][i] = fexp2(fmaf(st[tt][i], sl2, nm));
        st[tt][i + 1] = fexp2(fmaf(st[tt][i + 1], sl2, nm));
        rs0 += st[tt][i];
        rs1 += st[tt][i + 1];
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
    __builtin_amdgcn_sched_barrier(0);
    wait_vm<0>();  // this wave's DMA of tile u + 1 (and the next head's Q loads)
    if (last) {
      finish(h0 + j);
      if (j + 1 < NH) {
        // the asm wait above retired the Q loads; this statement makes hipcc place its own wait for
        // them here (already satisfied) instead of in front of the next tile's MFMAs, after the DMA
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) asm volatile("" : "+v"(qf[kk]));
      }
      ++j;
      t = 0;
    } else {
      ++t;
    }
    ring_barrier();
  }
  wait_vm<0>();  // the last head's O stores
}

// ============================================================================ backward dQ, D = 128, v3
// The forward v3 structure applied to the query-parallel dQ pass (grid, block order, K/V LDS-DMA ring,
// two workgroups per CU): per 32-key half of a 64-key tile, batched K row reads -> S^T = K.Q^T, batched
// V row reads -> dP^T = V.dO^T, dS = P (dP - delta) with P = exp2(S * scale * log2e - lse * log2e)
// (the forward's LSE: no online max), then batched K^T transposed reads -> dQ^T += K^T . dS^T.
// dQ = scale * sum; the row constants come straight from lse / delta. delta = rowsum(O * dO) is computed
// here from the wave's own O and dO rows (and written, with -lse/scale, the segment ids and -lse*log2e, as
// the ld tiles the dK/dV kernel reads next); with LLMT_FA_PREP=1 it comes from the prep kernel instead.
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
  const int T = (kv_end > kv_beg && !(a.probe & 8)) ? (kv_end - kv_beg + BN - 1) / BN : 0;
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
    // (fa_bwd_prep128_kernel's layout: -lse / scale, -delta, segment id, -lse * log2e)
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

// GQA head pairs (two query heads per 8-wave workgroup sharing the K/V ring, fa_fwd3_kernel /
// fa_bwd_dq3_kernel NW = 8) against one head per 4-wave workgroup, in one process
// (profiles/r3_attention_head_pairs_ab.jsonl): B4 S8192 Hq32 Hkv8 forward 2.183 -> 2.111 ms, backward
// 8.146 -> 7.889 ms (dQ); B2 S4096 equal; B32 S1024 forward 0.446 -> 0.486, backward 1.483 -> 1.532 (one
// workgroup per CU exposes the per-block prologue that two independent workgroups hide). In the Llama-3-8B
// step, though, pairs on every dense S8192 call lost 5 ms/step (1497.5 / 1498.7 vs 1492.6 / 1493.0 ms,
// alternating runs on one box): an 8-wave workgroup waits for a whole CU's worth of free slots while the
// optimizer stream's kernels overlap the forward. Opt-in only (forward variant 7, dQ variant 3).
static bool pairs_pay(const int*, int) { return false; }

// dK/dV kernel variant, read on every launch so one process can A/B them (LLMT_FA_BWD_VARIANT):
//   1 = end-of-tile barrier after an LDS drain and scalar softmax (A/B reference), 3 = barrier without
//   the drain (rows prefetched for the next tile stay in flight across it) and packed softmax. (A
//   sched-group pinned schedule of the same loop measured 9.17 vs 8.12 ms at B4 S8192 and was removed.)
static int dkdv_variant() {
  const char* e = getenv("LLMT_FA_BWD_VARIANT");
  // 4 = 3 with the widened dK / dV store tail: B32 S1024 1.496 -> 1.476 ms, B64 S512 1.058 -> 1.029 ms,
  // S8192 unchanged, bitwise-equal gradients (profiles/r3_attention_wide_store_ab.jsonl)
  // 5 = the software-pipelined loop (fa_bwd_dkdv5_kernel): B4 S8192 Hq32 Hkv8 backward 8.150 -> 8.017 ms in
  // one process, bitwise-equal gradients on every checked shape (benchmarks/attn_variant_check.py)
  return e ? atoi(e) : 5;  // 3 vs 1, in-process A/B: B4 S8192 8.117 vs 8.186 ms, bitwise-equal gradients
}

// range masks (AttnArgs::rmask; LLMT_FA_RANGE_MASK=0: per-element compares, the A/B reference)
static int range_masks() {
  const char* e = getenv("LLMT_FA_RANGE_MASK");
  return e ? atoi(e) : 1;
}

// prologue order (AttnArgs::early), read per launch for A/B (LLMT_FA_EARLY_DMA)
static int early_dma() {
  const char* e = getenv("LLMT_FA_EARLY_DMA");
  return e ? atoi(e) : 1;
}

// ring slots of the dK/dV kernel (fa_bwd_dkdv5_kernel NSL), read per launch for A/B (LLMT_FA_D5_RING): 8 for
// D=128 (packed Llama rows, same process: 8 docs 2.900 -> 2.890 ms, 32 docs 1.546 -> 1.511 ms fwd+bwd; dense
// unchanged), 6 for D=96 (dense 3.635 vs 3.649 ms, packed 2.183 vs 2.189; profiles/r5_dkdv_ring_ab.jsonl)
static int d5_ring(bool seg, int D = 128) {
  (void)seg;
  const char* e = getenv("LLMT_FA_D5_RING");
  if (e) return atoi(e) == 8 ? 8 : 6;
  return D == 128 ? 8 : 6;
}

static int attn_probe() {
  const char* e = getenv("LLMT_FA_PROBE");
  return e ? atoi(e) : 0;
}

// block order of the 1-D attention grids (AttnArgs::bmajor), read per launch for A/B (LLMT_FA_BMAJOR)
// (B4 S8192 Hq32 Hkv8: forward 2.102 -> 2.068 ms, backward 7.795 -> 7.732 ms in one process)
static int bmajor_order() {
  const char* e = getenv("LLMT_FA_BMAJOR");
  return e ? atoi(e) : 1;
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

static int fwd_variant() {
  const char* fve = getenv("LLMT_FA_FWD_VARIANT");
  return fve ? atoi(fve) : 4;
}
// does the forward launch for this problem go to fa_fwd3_kernel (the kernel with the fused Q rotation)?
static bool fwd_uses_fwd3(int D, int variant, bool drop, bool rmask, bool seg) {
  if (drop) return false;
  const bool chain = variant == 5 || variant == 6;
  if (D == 64 || D == 96) return variant != 0 && !chain;
  return !chain && !(variant == 10 && rmask && !seg) && (variant == 2 || variant == 3 || variant >= 4);
}

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
  dim3 grid((S + 127) / 128, Hq, B);
  // B1 S8192 Hq32 Hkv8: fwd3 0.659 ms (834 TF/s; 977 TF/s at B4), fa_fwd_kernel 0.907 (variant 0), the
  // removed one-wave-per-SIMD ring forward 1.043; 3 = fwd3 with compiler-placed row-sum adds, 2 = with the
  // inline-asm adds (A/B reference); read per launch
  // 4 = 3 with the widened O store tail (T21), in one process: B4 S8192 2.199 vs 2.203 ms, B32 S1024 0.429
  // vs 0.458, B64 S512 0.314 vs 0.343 ms (the per-block cost of short sequences / packed documents),
  // bitwise-equal output (profiles/r3_attention_wide_store_ab.jsonl)
  const int variant = fwd_variant();  // 3 vs 2 in one process: B4 S8192 2.145 vs 2.168 ms, same output
  if (rope) {
    // fused RoPE: q holds unrotated queries (k is already rotated). fa_fwd3_kernel rotates its rows on load;
    // every other kernel gets the rotated rows in the qrot scratch (q itself is never written)
    set_rope(a, rpos, rpos64, rp_sb, rp_ss, rcos, rsin, rP, qrot, D);
    if (fwd_uses_fwd3(D, variant, a.drop_thresh != 0, a.rmask, seg != nullptr)) {
      a.rope_q = 1;
    } else {
      if (!qrot) return hipErrorInvalidValue;
      rope_launch(a, a.q, a.q_sb, a.q_ss, a.q_sh, a.qrot, a.qr_sb, a.qr_ss, a.qr_sh, Hq, D, 1.f, stream);
      use_qrot(a);
    }
  }
  // head chains (fa_fwd3c: 4 query heads per workgroup, bitwise-equal output) pay standalone where a
  // block's heads have their own K/V: MHA B8 S4096 H32 D128 1.567 -> 1.391 ms, D96 1.631 -> 1.245 ms; with
  // GQA they lose (B4 S8192 Hq32 Hkv8 2.230 -> 2.507 ms; profiles/r3_attention_head_chain_ab.jsonl). In the
  // Phi-3 IT step (packed MHA) they cost 3 ms/step (688.4 / 690.3 vs 685.9 / 686.2 ms alternating on one
  // box), so chains are opt-in: variants 5 / 6 = chains of 2 / 4; 8 = one head per workgroup. Against the
  // round-5 forward they lose standalone too (B8 S4096 H32 D96 dense 0.983 vs 1.131 / 1.241 ms, packed
  // document-major 0.431 vs 0.752 / 1.016 ms; profiles/r4_negative_probes.jsonl).
  const int grp = Hq / Hkv;
  const int chain = variant == 5 ? (Hq % 2 == 0 ? 2 : 0) : variant == 6 ? (Hq % 4 == 0 ? 4 : 0) : 0;
  const unsigned nb1 = (unsigned)((S + 127) / 128 * Hq * B);
  switch (D) {
    case 64:  // the v3 structure on 128-byte rows (256-byte LDS pitch)
      if (a.drop_thresh || variant == 0)
        fa_fwd_kernel<64><<<grid, 256, 0, stream>>>(a);
      else if (chain == 4)
        fa_fwd3c_kernel<64, 4><<<nb1 / 4, 256, 0, stream>>>(a);
      else if (chain == 2)
        fa_fwd3c_kernel<64, 2><<<nb1 / 2, 256, 0, stream>>>(a);
      else if (a.rmask)
        fa_fwd3_kernel<64, 2, 1><<<nb1, 256, 0, stream>>>(a);
      else
        fa_fwd3_kernel<64, 1, 1, 4, true><<<nb1, 256, 0, stream>>>(a);
      break;
    case 96:  // Phi-3: the v3 structure on 192-byte rows (256-byte LDS pitch)
      if (a.drop_thresh || variant == 0)
        fa_fwd_kernel<96><<<grid, 256, 0, stream>>>(a);
      else if (chain == 4)
        fa_fwd3c_kernel<96, 4><<<nb1 / 4, 256, 0, stream>>>(a);
      else if (chain == 2)
        fa_fwd3c_kernel<96, 2><<<nb1 / 2, 256, 0, stream>>>(a);
      else if (a.rmask)
        fa_fwd3_kernel<96, 2, 1><<<nb1, 256, 0, stream>>>(a);
      else
        fa_fwd3_kernel<96, 1, 1, 4, true><<<nb1, 256, 0, stream>>>(a);
      break;
    case 128: {
      if (a.drop_thresh)  // dropout lives in the generic kernels
        fa_fwd_kernel<128><<<grid, 256, 0, stream>>>(a);
      else if (variant == 10 && a.rmask && !seg)  // one wave per SIMD, 64 rows per wave (fa_fwd4_kernel)
        fa_fwd4_kernel<128><<<(S + 255) / 256 * Hq * B, 256, 0, stream>>>(a);
      else if (variant == 2)  // row sums through the inline-asm add (each behind its own wait state)
        fa_fwd3_kernel<128><<<nb1, 256, 0, stream>>>(a);
      else if (variant == 3)  // dwordx2 O store tail (A/B reference)
        fa_fwd3_kernel<128, 1><<<nb1, 256, 0, stream>>>(a);
      else if (chain == 4)
        fa_fwd3c_kernel<128, 4><<<nb1 / 4, 256, 0, stream>>>(a);
      else if (chain == 2)
        fa_fwd3c_kernel<128, 2><<<nb1 / 2, 256, 0, stream>>>(a);
      else if (grp % 2 == 0 && (variant == 7 || (variant == 4 && pairs_pay(seg, S))))  // GQA head pairs
        fa_fwd3_kernel<128, 1, 1, 8><<<nb1 / 2, 512, 0, stream>>>(a);
      else if (variant == 9 && a.rmask)  // compiler-placed row-sum adds, bpermute row max (A/B reference)
        fa_fwd3_kernel<128, 1, 1><<<nb1, 256, 0, stream>>>(a);
      else if (variant >= 4 && a.rmask)  // permlane32 row max, asm exp / row-sum pairs: 2.091 -> 2.054 ms
        fa_fwd3_kernel<128, 2, 1><<<nb1, 256, 0, stream>>>(a);
      else if (variant >= 4)
        fa_fwd3_kernel<128, 1, 1, 4, true><<<nb1, 256, 0, stream>>>(a);
      else
        fa_fwd_kernel<128><<<grid, 256, 0, stream>>>(a);
    } break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// 1: a forward with fused RoPE needs no qrot scratch (the launch goes to fa_fwd3_kernel)
extern "C" int llmt_flash_attn_fwd_rope_inkernel(int D, float drop_p, int has_seg, int seg_runs) {
  const bool rmask = range_masks() && (!has_seg || seg_runs);
  return fwd_uses_fwd3(D, fwd_variant(), drop_p > 0.f, rmask, has_seg != 0) ? 1 : 0;
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
  dim3 grid((S + 127) / 128, Hq, B);
  const int dgrid = stream_grid(nrows, 256);
  static const bool small_v3 = getenv("LLMT_FA_D96_GENERIC") == nullptr;  // A/B switch for D = 64 / 96
  // fused RoPE: with qun the dQ kernel rotates its rows on load and writes them to qrot for the dK/dV
  // kernel; the dQ / dK epilogues (dq3, dkdv5 / dkdv6) apply the inverse rotation. Other kernels: qrot by
  // the standalone rotation, inverse passes after.
  if (rope) set_rope(a, rpos, rpos64, rp_sb, rp_ss, rcos, rsin, rP, qrot, D);
  auto rope_to_dkdv = [&](bool fused_dk) {  // after the dQ kernel: the dK/dV kernel reads qrot
    if (!rope) return;
    if (qun) use_qrot(a);
    a.rope_q = a.rope_dq = 0;
    a.rope_dk = fused_dk;
  };
  auto rope_finish_dk = [&](bool fused_dk) {
    if (rope && !fused_dk) rope_launch(a, a.dk, a.dk_sb, a.dk_ss, a.dk_sh, a.dk, a.dk_sb, a.dk_ss, a.dk_sh, Hkv, D, -1.f, stream);
  };
  if ((D == 128 || ((D == 96 || D == 64) && small_v3)) && !a.drop_thresh) {
    if (rope) {
      a.rope_q = qun;
      a.rope_dq = 1;
    }
    // delta buffer = [B, Hq, S] delta, then the packed per-tile row constants (llmt_flash_attn_bwd_ws)
    float* ld = delta + nrows;
    const int64_t nT = (S + 31) / 32;
    // the dQ kernel computes delta and writes the row constants itself (its waves cover every 32-row tile
    // of every head, and the dK/dV kernel runs after it on this stream); LLMT_FA_PREP=1: the separate prep
    // pass (A/B reference, read per launch)
    const char* pe = getenv("LLMT_FA_PREP");
    const bool fused_prep = !(pe && atoi(pe) == 1);
    if (fused_prep) a.ldw = ld;
    auto prep = [&](auto d_c) {
      if (!fused_prep)
        fa_bwd_prep128_kernel<decltype(d_c)::value><<<stream_grid((int64_t)B * Hq * nT * 32 * 16, 256), 256, 0, stream>>>(a, ld);
    };
    if (D == 96) {  // Phi-3: prep, v3 dQ, ring dK/dV (GQA inside the kernel: no partial buffers)
      prep(std::integral_constant<int, 96>{});
      if (a.rmask)
        fa_bwd_dq3_kernel<96, true, true><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      else
        fa_bwd_dq3_kernel<96, true, true, 4, true><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      const bool f5 = dkdv_variant() == 5;
      rope_to_dkdv(f5);
      if (dkdv_variant() == 5 && a.rmask && d5_ring(seg != nullptr, 96) == 8)
        fa_bwd_dkdv5_kernel<96, false, 8><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else if (dkdv_variant() == 5 && a.rmask)
        fa_bwd_dkdv5_kernel<96><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else if (dkdv_variant() == 5)
        fa_bwd_dkdv5_kernel<96, true><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else if (dkdv_variant() >= 3)
        fa_bwd_dkdv128_kernel<3, 96, true><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else
        fa_bwd_dkdv128_kernel<1, 96><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      rope_finish_dk(f5);
      return hipGetLastError();
    }
    if (D == 64) {
      prep(std::integral_constant<int, 64>{});
      if (a.rmask)
        fa_bwd_dq3_kernel<64, true, true><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      else
        fa_bwd_dq3_kernel<64, true, true, 4, true><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      const bool f5 = dkdv_variant() == 5;
      rope_to_dkdv(f5);
      if (dkdv_variant() == 5 && a.rmask)
        fa_bwd_dkdv5_kernel<64><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else if (dkdv_variant() == 5)
        fa_bwd_dkdv5_kernel<64, true><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else if (dkdv_variant() >= 3)
        fa_bwd_dkdv128_kernel<3, 64, true><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      else
        fa_bwd_dkdv128_kernel<1, 64><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
      rope_finish_dk(f5);
      return hipGetLastError();
    }
    prep(std::integral_constant<int, 128>{});
    // dQ: B4 S8192 Hq32 Hkv8 backward 9.16 ms with dq3 vs 9.66 ms with the earlier one-wave-per-SIMD ring
    // kernel (removed, like the 8-wave role-split dK/dV kernel: 10.81 vs 9.89 ms, and the ring forward)
    {
      // LLMT_FA_DQ_VARIANT=0: V reads after the whole S^T chain (A/B reference, read per launch); the
      // default interleaves them: B4 S8192 backward 8.00 -> 7.93 ms in one process, same gradients.
      // 1 = the dwordx2 dQ store tail; the default (2) widens it (T21): B32 S1024 backward 1.541 ->
      // 1.522 ms, B4 S8192 unchanged, same gradients
      const char* dqe = getenv("LLMT_FA_DQ_VARIANT");
      const int dqv = dqe ? atoi(dqe) : 2;
      if ((Hq / Hkv) % 2 == 0 && (dqv == 3 || (dqv == 2 && pairs_pay(seg, S))))  // GQA head pairs
        fa_bwd_dq3_kernel<128, true, true, 8><<<(S + 127) / 128 * (Hq / 2) * B, 512, 0, stream>>>(a);
      else if (dqv == 0)
        fa_bwd_dq3_kernel<128, false><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      else if (dqv == 1)
        fa_bwd_dq3_kernel<128><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      else if (dqv == 4 && a.rmask)  // asm reading the MFMA results (A/B reference)
        fa_bwd_dq3_kernel<128, true, true, 4, false, false><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      else if (a.rmask)
        fa_bwd_dq3_kernel<128, true, true><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
      else
        fa_bwd_dq3_kernel<128, true, true, 4, true><<<(S + 127) / 128 * Hq * B, 256, 0, stream>>>(a);
    }
    const int variant = dkdv_variant();
    // 7 = 64 keys per wave with asm-owned accumulators (fa_bwd_dkdv6_kernel), dense rows
    const bool v6 = variant == 7 && a.rmask && !seg;
    const bool f5 = variant == 5 || (variant == 6 && a.rmask) || v6;
    rope_to_dkdv(f5);
    // dense rows: an 8-slot Q / dO ring (tiles 6 ahead; B4 S8192 backward 7.605 -> 7.544 ms in one process,
    // 7 slots 7.572); packed rows keep 6 (their key blocks often visit only a few tiles)
    // LLMT_FA_D6_PROBE (diagnostic builds, wrong results): 1 = no ring DMA in the loop, 2 = no loop barrier,
    // 4 = no softmax VALU, 8 = no operand LDS reads, 16 = all VALU beside the accumulator-destination MFMAs,
    // 64 = no MFMAs (profiles/r5_dkdv6.md)
    static const int d6p = getenv("LLMT_FA_D6_PROBE") ? atoi(getenv("LLMT_FA_D6_PROBE")) : 0;
    const unsigned g6 = (S + 255) / 256 * Hkv * B;
    if (v6 && d6p == 1)
      fa_bwd_dkdv6_kernel<128, 3, 1><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 2)
      fa_bwd_dkdv6_kernel<128, 3, 2><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 4)
      fa_bwd_dkdv6_kernel<128, 3, 4><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 8)
      fa_bwd_dkdv6_kernel<128, 3, 8><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 15)
      fa_bwd_dkdv6_kernel<128, 3, 15><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 12)
      fa_bwd_dkdv6_kernel<128, 3, 12><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 64)
      fa_bwd_dkdv6_kernel<128, 3, 64><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 68)
      fa_bwd_dkdv6_kernel<128, 3, 68><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6 && d6p == 16)
      fa_bwd_dkdv6_kernel<128, 3, 16><<<g6, 256, 0, stream>>>(a, ld);
    else if (v6)
      fa_bwd_dkdv6_kernel<128><<<g6, 256, 0, stream>>>(a, ld);
    else if (variant == 6 && a.rmask && !seg)
      fa_bwd_dkdv5_kernel<128, false, 8, 1><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else if (variant == 6 && a.rmask)
      fa_bwd_dkdv5_kernel<128, false, 6, 1><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else if (variant == 5 && a.rmask && d5_ring(seg != nullptr) == 8)
      fa_bwd_dkdv5_kernel<128, false, 8><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else if (variant == 5 && a.rmask)
      fa_bwd_dkdv5_kernel<128><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else if (variant == 5)
      fa_bwd_dkdv5_kernel<128, true><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else if (variant == 3)
      fa_bwd_dkdv128_kernel<3><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else if (variant == 4)
      fa_bwd_dkdv128_kernel<3, 128, true><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    else
      fa_bwd_dkdv128_kernel<1><<<(S + 127) / 128 * Hkv * B, 256, 0, stream>>>(a, ld);
    rope_finish_dk(f5);
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
    rope_finish_dk(false);
  }
  return hipGetLastError();
}
