// bf16 GEMM for gfx950 (CDNA4) with fp32 accumulation, in all three layouts of a linear layer:
//
//   C[M, N] (+)= X . Y^T,   X(m, k) and Y(n, k) read from row-major bf16 matrices, each either
//   K-major (element (i, k) at P[i * ld + k]) or MN-major (element (i, k) at P[k * ld + i]).
//
//   forward  y  = x . W^T   : X = x  [T, K]  K-major,   Y = W [N, K]   K-major
//   dgrad    dx = dy . W    : X = dy [T, N]  K-major,   Y = W [N, K]   MN-major (contraction = W's rows)
//   wgrad    dW = dy^T . x  : X = dy [T, N]  MN-major,  Y = x [T, K]   MN-major (contraction = tokens)
//
// The projections and the lm_head of the models are these GEMMs. The kernel is the
// two-group ping-pong kernel gemm_pp_kernel (1.23-1.28 PF/s on the Llama-3-8B shapes at 32768 tokens; a
// single-group ring kernel, 1.10-1.16, was removed in round 6). hipBLASLt reaches 1.41-1.61 on the forward
// layout, so the framework uses this kernel as a timed weight-gradient candidate (it reads both token-major
// operands without transposes) and for the opt-in SwiGLU-backward epilogue (profiles/r3_gemm_pingpong.md,
// profiles/r6_gemm_pmc.md).
//
// Operand staging:
//  * K advances in 32-deep stages. Each stage's X and Y tiles (16 KB each) arrive by LDS-DMA
//    (`buffer_load_dwordx4 ... lds`, one 1-KB piece per wave-instruction) into a ring of LDS slots, several
//    stages ahead of the MFMAs, behind a counted `s_waitcnt vmcnt` and raw barriers: the loads never drain
//    inside the loop.
//  * LDS images are lane-linear (the DMA writes base + 16 * lane); bank conflicts are removed by
//    permuting the SOURCE address and reading through the same involution:
//      K-major image [256 rows][32 k] (64-B rows): 16-B chunk c of row r at chunk c ^ (-(r >> 2) & 3);
//        fragments by ds_read_b128, every 16-lane group on 16 distinct bank slots.
//      MN-major image [32 k][256 mn] (512-B rows): 32-B unit u of k-row k at unit u ^ ((k & 3) | (k >> 1 & 4));
//        fragments by two ds_read_b64_tr_b16 (hardware transpose: 4 k-rows x 16 columns per 16 lanes),
//        the 8 k-rows read by each 32-lane half land on 8 distinct 32-B bank units.
//  * MFMA v_mfma_f32_16x16x32_bf16 with the operands swapped (Y as the MFMA A operand), so each lane's
//    accumulator holds 4 consecutive OUTPUT COLUMNS of one row: 8-byte row stores, no transpose.
//  * blockIdx -> tile: bijective XCD remap (blocks b and b+8 share an XCD, so each XCD gets a contiguous
//    run of tiles), then a grouped order of kGM row tiles: the 32 workgroups resident on one XCD share
//    4 X panels and 8 Y panels through that XCD's L2.
//  * the stage base is rebased every stage (scalar descriptor), so only offsets inside one stage's
//    window must fit 32 bits; reads past the end of an operand come back as zeros (descriptor range
//    check). K must be a multiple of 32; rows / columns past M / N are computed on padding and not stored.
#include "common.h"

#include <cstring>

namespace llmt {
namespace {

typedef __bf16 gbf8 __attribute__((ext_vector_type(8)));
typedef short gs4 __attribute__((ext_vector_type(4)));
typedef float gf4 __attribute__((ext_vector_type(4)));
typedef unsigned int gu4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 256, kBN = 256, kBK = 32;
constexpr int kImg = kBM * kBK * 2;  // 16 KB: one operand's image of one stage
constexpr int kSlot = 2 * kImg;      // X image + Y image
constexpr int kPieces = 2 * kBM * kBK * 2 / 1024;  // 1-KB DMA pieces per stage (both operands)
constexpr int kGM = 4;               // row tiles per group of the tile order

__device__ __forceinline__ int kswz(int r) { return (-(r >> 2)) & 3; }
__device__ __forceinline__ int mswz(int k) { return (k & 3) | ((k >> 1) & 4); }

struct GRsrc {
  gu4 w;
};

// Raw buffer descriptor (no swizzle, range-checked): loads past `bytes` return zeros. Offsets never
// exceed one stage's window, so clamping a larger extent to 2^31 - 1 cuts nothing that is read.
__device__ __forceinline__ GRsrc g_rsrc(const char* base, int64_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  GRsrc r;
  r.w[0] = (uint32_t)p;
  r.w[1] = (uint32_t)(p >> 32) & 0xffffu;
  r.w[2] = (uint32_t)(bytes > 0x7fffffffLL ? 0x7fffffffLL : (bytes < 0 ? 0 : bytes));
  r.w[3] = 0x00020000u;
  return r;
}

__device__ __forceinline__ uint32_t g_lds(const char* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(const_cast<char*>(p));
}

// 16 bytes per lane global -> LDS (lds_base + 16 * lane). Issued from inline asm so hipcc does not treat
// it as an LDS write it must drain before every ds_read; the counted waits below order it.
__device__ __forceinline__ void g_dma16(const GRsrc& r, uint32_t lds_base, int voff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "s"(lds_base), "v"(voff), "s"(r.w)
               : "memory");
}

template <int N>
__device__ __forceinline__ void g_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// This wave's LDS reads retired, then a barrier that leaves the DMA ring in flight (no vmcnt(0)). The
// lgkmcnt(0) is the builtin (vmcnt/expcnt fields at their maxima) so hipcc's wait bookkeeping knows
// every earlier fragment read has landed and does not stall the next MFMAs on the reads issued after
// the barrier; the barrier itself is asm with a memory clobber so no LDS access moves across it.
__device__ __forceinline__ void g_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0
  asm volatile("s_barrier" ::: "memory");
}

__device__ __forceinline__ gs4 lds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) gs4*)(p));
}

// One operand (X or Y): where this lane's DMA pieces of a stage come from, how the stage base
// advances, and how MFMA fragments are read back from the stage image. The operand's stage image is
// 16 pieces of 1 KB; with NW waves, wave w loads pieces w, w + NW, ... (NP = 16 / NW of them).
template <bool MN, int NW>
struct Opnd {
  static constexpr int NP = 16 / NW;
  const char* base;  // stage 0 tile origin
  int64_t extent;    // readable bytes from `base`
  int64_t step;      // bytes per stage
  int off[NP];       // this lane's source byte offsets of its wave's pieces
  int frag_off;      // lane-constant part of the fragment read address

  // P: row-major matrix with leading dimension ld; rows = its row count; cols = its column count
  // (K-major: rows = output rows/cols of C, cols = K; MN-major: rows = K, cols = output rows/cols).
  __device__ __forceinline__ void init(const bf16* P, int64_t ld, int64_t rows, int64_t cols, int tile0, int w,
                                       int lane) {
    if constexpr (!MN) {
      base = reinterpret_cast<const char*>(P + (int64_t)tile0 * ld);
      extent = ((rows - 1 - tile0) * ld + cols) * 2;
      step = kBK * 2;
#pragma unroll
      for (int i = 0; i < NP; ++i) {  // piece j = rows 16j .. 16j+15
        const int row = (w + NW * i) * 16 + (lane >> 2);
        const int ch = (lane & 3) ^ kswz(row);
        off[i] = row * (int)ld * 2 + ch * 16;
      }
      const int fr = lane & 15;
      frag_off = fr * 64 + (((lane >> 4) ^ kswz(fr)) * 16);
    } else {
      base = reinterpret_cast<const char*>(P + tile0);
      extent = ((rows - 1) * ld + cols - tile0) * 2;
      step = (int64_t)kBK * ld * 2;
#pragma unroll
      for (int i = 0; i < NP; ++i) {  // piece j = k-rows 2j, 2j+1
        const int krow = 2 * (w + NW * i) + (lane >> 5);
        const int pc = lane & 31;
        const int lc = 2 * ((pc >> 1) ^ mswz(krow)) + (pc & 1);
        off[i] = krow * (int)ld * 2 + lc * 16;
      }
      const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
      frag_off = (8 * g + q) * 512 + 8 * p;  // + 32 * (unit ^ h) per fragment, h = q | (g & 1) << 2
    }
  }

  __device__ __forceinline__ GRsrc rsrc(int t) const { return g_rsrc(base + t * step, extent - t * step); }

  // fragment of the 16-row (output index) tile starting at `tile` (multiple of 16) of the stage image
  __device__ __forceinline__ gbf8 frag(const char* img, int tile, int lane) const {
    if constexpr (!MN) {
      return *reinterpret_cast<const gbf8*>(img + tile * 64 + frag_off);
    } else {
      const int h = ((lane & 15) >> 2) | (((lane >> 4) & 1) << 2);
      const char* p = img + frag_off + (((tile >> 4) ^ h) << 5);
      const gs4 lo = lds_tr16(p), hi = lds_tr16(p + 4 * 512);
      return __builtin_bit_cast(gbf8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

struct GemmArgs {
  const bf16* x;
  const bf16* y;
  void* c;
  int M, N, K;
  int64_t ldx, ldy, ldc;
};

// SwiGLU-backward epilogue (OUT = 4, gemm_pp_kernel): C = dc = dy . W_down is not stored; with g = gu[m, n],
// u = gu[m, I + n] (I = N) the epilogue writes dgu[m, n] = dc u silu'(g), dgu[m, I + n] = dc silu(g) and, when
// dgu_t is set, the same values transposed into dgu_t [2I, M] (the token-contiguous operand of the gate_up
// weight-gradient GEMM). Replaces the standalone swiglu_bwd_tr pass (csrc/elementwise.hip), which read dc back.
struct SwiArgs {
  const bf16* gu;  // [M, 2N]
  bf16* dgu;       // [M, 2N]
  bf16* dgu_t;     // [2N, M] or null
};

__device__ __forceinline__ float g_sigmoid(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ void tile_coords(int M, int N, int& tm, int& tn) {
  const int nbm = (M + kBM - 1) / kBM, nbn = (N + kBN - 1) / kBN, nwg = nbm * nbn;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int per = kGM * nbn;
  const int g = wg / per;
  const int first = g * kGM;
  const int gsz = min(nbm - first, kGM);
  const int in = wg - g * per;
  tm = first + in % gsz;
  tn = in / gsz;
}

// ---------------------------------------------------------------- SwiGLU-backward epilogue
// Runs after the main loop of a 256 x 256 tile, in four passes of 64 output columns (the columns of waves
// wq = q of both row groups). Per pass, through the (now free) LDS ring:
//   1. the owning waves write their dc accumulators as bf16 into D [256 rows][64 cols];
//   2. all 512 threads take 2 rows x 8 columns per step (two steps): D from LDS, g / u from global (16-byte
//      loads issued before step 1, so their latency overlaps the LDS staging), dg / du in fp32 with the
//      swiglu_bwd_kernel math, 16-byte row-major stores of dgu, and the bf16 results as 32-bit row-pair
//      words into the transposed images G^T / U^T [64 cols][128 row pairs];
//   3. 16-byte stores of 8 tokens of one dgu_t row from G^T / U^T (32 threads cover a 512-byte row run).
// The staged dc is rounded to bf16 first: the same numerics as the unfused GEMM (bf16 dc) + swiglu_bwd_tr.
constexpr int kSwDP = 144;             // D row pitch (bytes): 128 + 16
constexpr int kSwTW = 132;             // G^T / U^T row pitch (32-bit words): 128 + 4
constexpr int kSwD = 256 * kSwDP;      // 36 KB
constexpr int kSwT = 64 * kSwTW * 4;   // 33 KB each

__device__ __forceinline__ void swiglu_bwd_epilogue(const GemmArgs& g, const SwiArgs& sw, gf4 (&acc)[8][4],
                                                    char* smem, int row0, int col0, int grp, int wq, int fr, int fc,
                                                    int tid) {
  const int M = g.M, N = g.N;
  const int64_t ld2 = 2 * (int64_t)N;
  char* dimg = smem;
  uint32_t* gt = reinterpret_cast<uint32_t*>(smem + kSwD);
  uint32_t* ut = reinterpret_cast<uint32_t*>(smem + kSwD + kSwT);
  const int cch = tid & 7, rp = tid >> 3;  // 8-column chunk, row pair (per step)
  // every wave's DMAs have landed and every fragment read retired before the ring is reused
  g_barrier();
#pragma unroll 1
  for (int q = 0; q < 4; ++q) {
    const int c0 = col0 + q * 64;
    if (c0 >= N) break;  // workgroup-uniform
    // (2) operands of this thread's two steps, loaded first (rows 2 rp, 2 rp + 1 and + 128)
    bf16x8 gv[2][2], uv[2][2];
    const int n = c0 + cch * 8;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = row0 + st * 128 + 2 * rp + h;
        if (m < M && n < N) {
          const bf16* pr = sw.gu + (int64_t)m * ld2 + n;
          gv[st][h] = *reinterpret_cast<const bf16x8*>(pr);
          uv[st][h] = *reinterpret_cast<const bf16x8*>(pr + N);
        } else {
          gv[st][h] = bf16x8{{0u, 0u, 0u, 0u}};
          uv[st][h] = gv[st][h];
        }
      }
    // (1) the owning waves stage dc (bf16) in D
    if (wq == q) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int r = grp * 128 + i * 16 + fr, c = jj * 16 + fc * 4;
          uint2 w;
          w.x = pack_bf16x2(acc[i][jj][0], acc[i][jj][1]);
          w.y = pack_bf16x2(acc[i][jj][2], acc[i][jj][3]);
          *reinterpret_cast<uint2*>(dimg + r * kSwDP + c * 2) = w;
        }
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      uint32_t wg[8], wu[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = st * 128 + 2 * rp + h, m = row0 + r;
        float dcv[8], a[8], b[8], da[8], db[8];
        unpack8(*reinterpret_cast<const bf16x8*>(dimg + r * kSwDP + cch * 16), dcv);
        unpack8(gv[st][h], a);
        unpack8(uv[st][h], b);
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // the swiglu_bwd_kernel math, element for element
          const float sg = g_sigmoid(a[i]);
          const float silu = a[i] * sg;
          da[i] = dcv[i] * b[i] * sg * (1.f + a[i] * (1.f - sg));
          db[i] = dcv[i] * silu;
        }
        const bf16x8 pa = pack8(da), pb = pack8(db);
        if (m < M && n < N) {
          bf16* drow = sw.dgu + (int64_t)m * ld2 + n;
          *reinterpret_cast<bf16x8*>(drow) = pa;
          *reinterpret_cast<bf16x8*>(drow + N) = pb;
        }
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
      if (sw.dgu_t) {
        const int pw = st * 64 + rp;  // row-pair word index
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          gt[(cch * 8 + i) * kSwTW + pw] = wg[i];
          ut[(cch * 8 + i) * kSwTW + pw] = wu[i];
        }
      }
    }
    __syncthreads();
    if (sw.dgu_t) {
      // (3) 64 columns x 32 chunks of 8 tokens per image: 4 chunks of each image per thread
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = tid + 512 * k;
        const int c = idx >> 5, ch = idx & 31;
        const int nn = c0 + c, m = row0 + ch * 8;
        if (nn < N && m < M) {
          const uint4 vg = *reinterpret_cast<const uint4*>(gt + c * kSwTW + 4 * ch);
          const uint4 vu = *reinterpret_cast<const uint4*>(ut + c * kSwTW + 4 * ch);
          *reinterpret_cast<uint4*>(sw.dgu_t + (int64_t)nn * M + m) = vg;
          *reinterpret_cast<uint4*>(sw.dgu_t + (int64_t)(N + nn) * M + m) = vu;
        }
      }
      __syncthreads();  // the images are rewritten by the next pass
    }
  }
}

// ---------------------------------------------------------------- ping-pong kernel
// The same tile (256 x 256, 8 waves as 2 (M) x 4 (N), wave tile 128 x 64, 32-deep stages in a ring of NS
// 32-KB LDS slots filled by LDS-DMA) with the waves split into two groups that alternate roles between
// barriers (cdna guide §5 'The 256² 8-phase template', MI355X_MICROARCH 'Two waves per SIMD'): waves 0-3
// (output rows 0..127) and waves 4-7 (rows 128..255) share each SIMD pairwise, and while one group runs
// its 32 MFMAs of a stage the other reads its fragments of the stage from LDS and issues its share of the
// DMA NS-1 stages ahead (group 0 fetches the X image, group 1 the Y image: 4 one-KB pieces per wave per
// stage). Group 1 starts one barrier late, so every interval between two barriers pairs one group's
// matrix work with the other group's LDS / DMA work on every SIMD.
// Ordering (per wave, stage j): [read fragments of j; DMA of stage j+NS-1 into the slot of stage j-1;
// vmcnt(4 (NS-2)) -> this wave's pieces of stage j+1 have landed; lgkmcnt(0); barrier] [32 MFMAs;
// barrier]. A slot is rewritten only after both groups' reads of it retired before an earlier barrier, and
// a stage is read only after every wave's pieces of it were waited for before an earlier barrier. DMAs
// past the last stage read an empty descriptor range (zeros into slots no one reads) so the wait counts
// stay constant. Split-K: blockIdx.y selects a contiguous slice of the stages, written as an fp32 slab.
// OUT: 0 = bf16 store, 1 = fp32 store (split-K slab), 2 = fp32 accumulate, 3 = bf16 accumulate
// (C = bf16(C + X.Y^T)), 4 = SwiGLU-backward epilogue (no C)
template <bool XMN, bool YMN, int OUT, int NS>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs g, int nk, int64_t slab, SwiArgs sw) {
  constexpr int AH = NS - 1;  // stages in flight ahead of the one being read
  __shared__ __attribute__((aligned(16))) char smem[NS * kSlot];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, wq = w & 3;
  int tm, tn;
  tile_coords(g.M, g.N, tm, tn);
  const int row0 = tm * kBM, col0 = tn * kBN;
  const int64_t k0 = (int64_t)blockIdx.y * nk * kBK;  // first contraction index of this split

  Opnd<XMN, 4> X;
  Opnd<YMN, 4> Y;
  if constexpr (!XMN)
    X.init(g.x + k0, g.ldx, g.M, g.K - k0, row0, wq, lane);
  else
    X.init(g.x + k0 * g.ldx, g.ldx, g.K - k0, g.M, row0, wq, lane);
  if constexpr (!YMN)
    Y.init(g.y + k0, g.ldy, g.N, g.K - k0, col0, wq, lane);
  else
    Y.init(g.y + k0 * g.ldy, g.ldy, g.K - k0, g.N, col0, wq, lane);
  const uint32_t lbase = g_lds(smem);

  auto issue = [&](int t, int slot) {
    const uint32_t sb = lbase + (uint32_t)(slot * kSlot);
    if (grp == 0) {
      const GRsrc r = X.rsrc(t);
#pragma unroll
      for (int i = 0; i < 4; ++i) g_dma16(r, sb + (wq + 4 * i) * 1024, X.off[i]);
    } else {
      const GRsrc r = Y.rsrc(t);
#pragma unroll
      for (int i = 0; i < 4; ++i) g_dma16(r, sb + kImg + (wq + 4 * i) * 1024, Y.off[i]);
    }
  };

  gbf8 fy[4], fx[8];
  gf4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = gf4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < AH; ++t) issue(t, t);
  g_wait_vm<4 * (AH - 1)>();
  g_barrier();
  if (grp == 1) g_barrier();  // the stagger: group 1 runs one interval behind

  int slot = 0, islot = AH;
  for (int j = 0; j < nk; ++j) {
    // ---- load segment: fragments of stage j, DMA of stage j + AH
    const char* img = smem + slot * kSlot;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) fy[jj] = Y.frag(img + kImg, wq * 64 + jj * 16, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) fx[i] = X.frag(img, grp * 128 + i * 16, lane);
    issue(j + AH, islot);
    g_wait_vm<4 * (AH - 1)>();
    g_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- compute segment
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fy[jj], fx[i], acc[i][jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    g_barrier();
    slot = slot + 1 == NS ? 0 : slot + 1;
    islot = islot + 1 == NS ? 0 : islot + 1;
  }
  if (grp == 0) g_barrier();  // equal barrier counts in both groups
  g_wait_vm<0>();             // no LDS-DMA outlives the workgroup

  const int fr = lane & 15, fc = lane >> 4;
  if constexpr (OUT == 4) {
    swiglu_bwd_epilogue(g, sw, acc, smem, row0, col0, grp, wq, fr, fc, tid);
    return;
  }
  char* cbase = reinterpret_cast<char*>(g.c) + (int64_t)blockIdx.y * slab * (OUT == 0 || OUT == 3 ? 2 : 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = row0 + grp * 128 + i * 16 + fr;
    if (m >= g.M) continue;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int n = col0 + wq * 64 + jj * 16 + fc * 4;
      if (n >= g.N) continue;
      const gf4 v = acc[i][jj];
      if constexpr (OUT == 0 || OUT == 3) {
        uint2* p = reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(cbase) + (int64_t)m * g.ldc + n);
        float a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
        if constexpr (OUT == 3) {
          const uint2 o = *p;
          a0 += bf16_lo(o.x);
          a1 += bf16_hi(o.x);
          a2 += bf16_lo(o.y);
          a3 += bf16_hi(o.y);
        }
        uint2 o;
        o.x = pack_bf16x2(a0, a1);
        o.y = pack_bf16x2(a2, a3);
        *p = o;
      } else {
        float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(cbase) + (int64_t)m * g.ldc + n);
        float4 o = make_float4(v[0], v[1], v[2], v[3]);
        if constexpr (OUT == 2) {
          const float4 c = *p;
          o.x += c.x;
          o.y += c.y;
          o.z += c.z;
          o.w += c.w;
        }
        *p = o;
      }
    }
  }
}

template <bool XMN, bool YMN>
hipError_t launch_pp(const GemmArgs& a, int out_mode, int ksplit, int64_t slab, hipStream_t stream,
                     const SwiArgs& sw = SwiArgs{nullptr, nullptr, nullptr}) {
  const int64_t nwg = (int64_t)((a.M + kBM - 1) / kBM) * ((a.N + kBN - 1) / kBN);
  const int nk = a.K / kBK / ksplit;
  const dim3 grid((unsigned)nwg, (unsigned)ksplit), block(512);
  switch (out_mode) {
    case 0: gemm_pp_kernel<XMN, YMN, 0, 5><<<grid, block, 0, stream>>>(a, nk, slab, sw); break;
    case 1: gemm_pp_kernel<XMN, YMN, 1, 5><<<grid, block, 0, stream>>>(a, nk, slab, sw); break;
    case 2: gemm_pp_kernel<XMN, YMN, 2, 5><<<grid, block, 0, stream>>>(a, nk, slab, sw); break;
    case 3: gemm_pp_kernel<XMN, YMN, 3, 5><<<grid, block, 0, stream>>>(a, nk, slab, sw); break;
    default:
      if constexpr (!XMN && YMN) {  // the down-projection input gradient: dy [M, K] . W_down [K, N]
        gemm_pp_kernel<false, true, 4, 5><<<grid, block, 0, stream>>>(a, nk, slab, sw);
        break;
      }
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace
}  // namespace llmt

// Host launcher: C[M, N] (+)= X . Y^T. x_mn / y_mn select MN-major operands (x is [K, M] / y is [K, N]);
// otherwise x is [M, K] and y is [N, K]. Preconditions (checked by the binding): K % 32 == 0, N % 4 == 0,
// ldx / ldy % 8 == 0, ldc % 4 == 0, 16-byte aligned x / y / c, 256 * ld * 2 < 2^31.
extern "C" hipError_t llmt_gemm(const void* x, const void* y, void* c, int x_mn, int y_mn, int out_mode, int M, int N,
                                int K, int64_t ldx, int64_t ldy, int64_t ldc, hipStream_t stream) {
  using namespace llmt;
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % kBK != 0 || N % 4 != 0 || out_mode < 0 || out_mode > 3) return hipErrorInvalidValue;
  if (ldx % 8 || ldy % 8 || ldc % 4) return hipErrorInvalidValue;
  if (256 * ldx * 2 >= 0x7fffffffLL || 256 * ldy * 2 >= 0x7fffffffLL) return hipErrorInvalidValue;
  GemmArgs a{reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(y), c, M, N, K, ldx, ldy, ldc};
  if (!x_mn && !y_mn) return launch_pp<false, false>(a, out_mode, 1, 0, stream);
  if (!x_mn && y_mn) return launch_pp<false, true>(a, out_mode, 1, 0, stream);
  if (x_mn && y_mn) return launch_pp<true, true>(a, out_mode, 1, 0, stream);
  return hipErrorInvalidValue;  // X MN-major with Y K-major: no linear-layer GEMM has this layout
}

// Split-K form of the ping-pong kernel: slabs[s] (fp32 [M, N], row stride ldc, slab stride M * ldc) gets
// X . Y^T over contraction slice s of nsplit equal slices (summed by llmt_splitk_reduce). K must be a
// multiple of 32 * nsplit.
extern "C" hipError_t llmt_gemm_splitk(const void* x, const void* y, float* slabs, int x_mn, int y_mn, int M, int N,
                                       int K, int64_t ldx, int64_t ldy, int64_t ldc, int nsplit, hipStream_t stream) {
  using namespace llmt;
  if (M <= 0 || N <= 0) return hipSuccess;
  if (nsplit < 1 || K <= 0 || K % (kBK * nsplit) != 0 || N % 4 != 0) return hipErrorInvalidValue;
  if (ldx % 8 || ldy % 8 || ldc % 4) return hipErrorInvalidValue;
  if (256 * ldx * 2 >= 0x7fffffffLL || 256 * ldy * 2 >= 0x7fffffffLL) return hipErrorInvalidValue;
  GemmArgs a{reinterpret_cast<const bf16*>(x), reinterpret_cast<const bf16*>(y), slabs, M, N, K, ldx, ldy, ldc};
  const int64_t slab = (int64_t)M * ldc;
  if (!x_mn && !y_mn) return launch_pp<false, false>(a, 1, nsplit, slab, stream);
  if (!x_mn && y_mn) return launch_pp<false, true>(a, 1, nsplit, slab, stream);
  if (x_mn && y_mn) return launch_pp<true, true>(a, 1, nsplit, slab, stream);
  return hipErrorInvalidValue;
}

// Down-projection input gradient with the SwiGLU backward in the epilogue (see SwiArgs): dy [M, K] (row stride
// ldx), w_down [K, N] (row stride ldy), gu / dgu [M, 2N] contiguous, dgu_t [2N, M] or null. Preconditions
// (checked by the binding): K % 32 == 0, N % 64 == 0, M % 64 == 0, 16-byte aligned operands.
extern "C" hipError_t llmt_gemm_swiglu_bwd(const void* dy, const void* w, const void* gu, void* dgu, void* dgu_t, int M,
                                           int N, int K, int64_t ldx, int64_t ldy, hipStream_t stream) {
  using namespace llmt;
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K <= 0 || K % kBK != 0 || N % 64 != 0 || M % 64 != 0) return hipErrorInvalidValue;
  if (ldx % 8 || ldy % 8) return hipErrorInvalidValue;
  if (256 * ldx * 2 >= 0x7fffffffLL || 256 * ldy * 2 >= 0x7fffffffLL) return hipErrorInvalidValue;
  GemmArgs a{reinterpret_cast<const bf16*>(dy), reinterpret_cast<const bf16*>(w), nullptr, M, N, K, ldx, ldy, 0};
  SwiArgs sw{reinterpret_cast<const bf16*>(gu), reinterpret_cast<bf16*>(dgu), reinterpret_cast<bf16*>(dgu_t)};
  return launch_pp<false, true>(a, 4, 1, 0, stream, sw);
}
