// Cross-entropy / log-softmax statistics with in-place gradient for gfx950.
//
// Replaces the reference's LigerCrossEntropyFunction (grad-in-forward online softmax,
// reference src/llm_training/ops/liger_kernel/cross_entropy_op.py:10-33) and the torch
// loss_parallel / log_softmax().gather() paths of DPO/ORPO (reference
// src/llm_training/lms/dpo/dpo.py:73-114, lms/orpo/orpo.py:61-93).
//
// One 1024-thread workgroup per row of bf16 logits [N, V_local] holding the row in registers (ce_reg_kernel,
// rows of up to 131072 logits in 16-byte chunks), else one 256-thread workgroup streaming the row in 16-byte
// vectors (ce_kernel). Pass 1: max / sum-exp, block-reduced -> lse. Pass 2 (optional):
// overwrite the row with coef * (softmax - onehot(label)), i.e. the gradient of
//   coef * (lse - logit[label])
// w.r.t. the logits, so the logits buffer doubles as the dlogits buffer (no extra [N, V] tensor).
//
// Vocab-parallel (TP) use: `vocab_start` offsets the label into this rank's vocab shard; pass 1 is
// run alone (write_grad=0) to produce the LOCAL lse and target logit, the caller combines lse across
// ranks (one small RCCL all-gather/all-reduce), then pass 2 is run with lse_in = the global lse.
#include "common.h"

namespace llmt {

template <bool VEC>
__global__ __launch_bounds__(256) void ce_kernel(bf16* __restrict__ logits, int64_t ld, int V,
                                                 const int64_t* __restrict__ labels, int64_t vocab_start,
                                                 int64_t ignore_index, const float* __restrict__ lse_in,
                                                 float* __restrict__ lse_out, float* __restrict__ tgt_out,
                                                 float* __restrict__ loss_out, const float* __restrict__ coef_row,
                                                 const float* __restrict__ coef_scalar, int write_grad,
                                                 int64_t vocab_total, int* __restrict__ err,
                                                 float* __restrict__ rowsum_out) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  bf16* x = logits + row * ld;
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index;
  const int64_t lloc = lab - vocab_start;
  const bool local_hit = valid && lloc >= 0 && lloc < V;
  const int tid = threadIdx.x;
  // a label that is neither ignore_index nor a vocabulary entry: flag it (the row then trains on lse alone)
  if (err && tid == 0 && valid && (lab < 0 || (vocab_total > 0 && lab >= vocab_total))) err[1] = 1;

  float lse;
  if (lse_in) {
    lse = lse_in[row];
  } else {
    float m = -INFINITY, s = 0.f, rsum = 0.f;  // rsum: plain sum of the row's logits (ORPO metrics)
    if constexpr (VEC) {
      const bf16x8* xv = reinterpret_cast<const bf16x8*>(x);
      const int V8 = V >> 3;
      for (int j = tid; j < V8; j += 256) {
        float f[8];
        unpack8(xv[j], f);
        float lm = f[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) lm = fmaxf(lm, f[i]);
        if (lm > m) {
          s *= __expf(m - lm);
          m = lm;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s += __expf(f[i] - m);
          rsum += f[i];
        }
      }
      for (int j = (V8 << 3) + tid; j < V; j += 256) {
        const float f = bf2f(x[j]);
        if (f > m) {
          s *= __expf(m - f);
          m = f;
        }
        s += __expf(f - m);
        rsum += f;
      }
    } else {
      for (int j = tid; j < V; j += 256) {
        const float f = bf2f(x[j]);
        if (f > m) {
          s *= __expf(m - f);
          m = f;
        }
        s += __expf(f - m);
        rsum += f;
      }
    }
    const float gm = block_max<4>(m, red);
    s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
    const float gs = block_sum<4>(s, red);
    lse = gm + __logf(gs);
    if (rowsum_out) {  // uniform branch: every thread takes part in the block reduction
      const float rs = block_sum<4>(rsum, red);
      if (tid == 0) rowsum_out[row] = rs;
    }
  }
  const float tgt = local_hit ? bf2f(x[lloc]) : 0.f;
  if (tid == 0) {
    if (lse_out) lse_out[row] = lse;
    if (tgt_out) tgt_out[row] = tgt;
    if (loss_out) loss_out[row] = valid ? (lse - tgt) : 0.f;
  }
  if (!write_grad) return;
  __syncthreads();  // every thread has read x[lloc] before anyone overwrites it
  float coef = valid ? 1.f : 0.f;
  if (coef_row) coef *= coef_row[row];
  if (coef_scalar) coef *= coef_scalar[0];
  if constexpr (VEC) {
    bf16x8* xv = reinterpret_cast<bf16x8*>(x);
    const int V8 = V >> 3;
    for (int j = tid; j < V8; j += 256) {
      float f[8];
      unpack8(xv[j], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float g = __expf(f[i] - lse);
        if (local_hit && (int64_t)(j * 8 + i) == lloc) g -= 1.f;
        f[i] = coef * g;
      }
      xv[j] = pack8(f);
    }
    for (int j = (V8 << 3) + tid; j < V; j += 256) {
      float g = __expf(bf2f(x[j]) - lse);
      if (local_hit && j == lloc) g -= 1.f;
      x[j] = __float2bfloat16(coef * g);
    }
  } else {
    for (int j = tid; j < V; j += 256) {
      float g = __expf(bf2f(x[j]) - lse);
      if (local_hit && j == lloc) g -= 1.f;
      x[j] = __float2bfloat16(coef * g);
    }
  }
}

// The same for rows of up to 1024 * NCH 16-byte chunks (V <= 131072 at NCH = 16) with V % 8 == 0 and aligned
// rows: one 1024-thread workgroup per row holds the whole row in registers (NCH chunks per thread), so the row
// is read from HBM once; the two-pass kernel above reads it again for the gradient, and with 8 rows of
// 256 KB in flight per CU that second read misses the caches.
template <int NCH>
__global__ __launch_bounds__(1024) void ce_reg_kernel(bf16* __restrict__ logits, int64_t ld, int V,
                                                      const int64_t* __restrict__ labels, int64_t vocab_start,
                                                      int64_t ignore_index, const float* __restrict__ lse_in,
                                                      float* __restrict__ lse_out, float* __restrict__ tgt_out,
                                                      float* __restrict__ loss_out, const float* __restrict__ coef_row,
                                                      const float* __restrict__ coef_scalar, int write_grad,
                                                      int64_t vocab_total, int* __restrict__ err,
                                                      float* __restrict__ rowsum_out) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  bf16* x = logits + row * ld;
  bf16x8* xv = reinterpret_cast<bf16x8*>(x);
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index;
  const int64_t lloc = lab - vocab_start;
  const bool local_hit = valid && lloc >= 0 && lloc < V;
  const int tid = threadIdx.x;
  if (err && tid == 0 && valid && (lab < 0 || (vocab_total > 0 && lab >= vocab_total))) err[1] = 1;
  const int V8 = V >> 3;
  bf16x8 c[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int j = tid + 1024 * k;
    if (j < V8) c[k] = xv[j];
  }
  float lse;
  if (lse_in) {
    lse = lse_in[row];
  } else {
    // the row is in registers: its max first, then the sum of exp against it (no online rescaling)
    float m = -INFINITY, rsum = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (tid + 1024 * k < V8) {
        float f[8];
        unpack8(c[k], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          m = fmaxf(m, f[i]);
          rsum += f[i];
        }
      }
    }
    const float gm = block_max<16>(m, red);
    float s = 0.f;
    if (gm != -INFINITY) {
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        if (tid + 1024 * k < V8) {
          float f[8];
          unpack8(c[k], f);
#pragma unroll
          for (int i = 0; i < 8; ++i) s += __expf(f[i] - gm);
        }
      }
    }
    const float gs = block_sum<16>(s, red);
    lse = gm + __logf(gs);
    if (rowsum_out) {
      const float rs = block_sum<16>(rsum, red);
      if (tid == 0) rowsum_out[row] = rs;
    }
  }
  const float tgt = local_hit ? bf2f(x[lloc]) : 0.f;
  if (tid == 0) {
    if (lse_out) lse_out[row] = lse;
    if (tgt_out) tgt_out[row] = tgt;
    if (loss_out) loss_out[row] = valid ? (lse - tgt) : 0.f;
  }
  if (!write_grad) return;
  __syncthreads();  // every thread has read x[lloc] before anyone overwrites it
  float coef = valid ? 1.f : 0.f;
  if (coef_row) coef *= coef_row[row];
  if (coef_scalar) coef *= coef_scalar[0];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int j = tid + 1024 * k;
    if (j < V8) {
      float f[8];
      unpack8(c[k], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float g = __expf(f[i] - lse);
        if (local_hit && (int64_t)(j * 8 + i) == lloc) g -= 1.f;
        f[i] = coef * g;
      }
      xv[j] = pack8(f);
    }
  }
}

}  // namespace llmt

using namespace llmt;

extern "C" hipError_t llmt_cross_entropy(void* logits, int64_t N, int64_t ld, int V, const int64_t* labels,
                                         int64_t vocab_start, int64_t ignore_index, const float* lse_in,
                                         float* lse_out, float* tgt_out, float* loss_out, const float* coef_row,
                                         const float* coef_scalar, int write_grad, int64_t vocab_total, int* err,
                                         float* rowsum_out, hipStream_t stream) {
  if (N == 0) return hipSuccess;
  const bool vec = (ld % 8 == 0) && ((reinterpret_cast<uintptr_t>(logits) & 15) == 0);
  // rows of up to 131072 logits in 16-byte chunks: the one-pass kernel (8192 x 128256: 1.222 -> 0.920 ms,
  // 8192 x 32064: 0.202 -> 0.156 ms against the two-pass one, profiles/r6_ce_ab.jsonl)
  const bool reg_ok = vec && V % 8 == 0;
  const int nch = (V / 8 + 1023) / 1024;
#define CE_REG(NCH)                                                                                          \
  ce_reg_kernel<NCH><<<(unsigned)N, 1024, 0, stream>>>((bf16*)logits, ld, V, labels, vocab_start, ignore_index,  \
                                                      lse_in, lse_out, tgt_out, loss_out, coef_row, coef_scalar,  \
                                                      write_grad, vocab_total, err, rowsum_out)
  if (reg_ok && nch <= 4)
    CE_REG(4);
  else if (reg_ok && nch <= 8)
    CE_REG(8);
  else if (reg_ok && nch <= 16)
    CE_REG(16);
  else if (vec)
    ce_kernel<true><<<(unsigned)N, 256, 0, stream>>>((bf16*)logits, ld, V, labels, vocab_start, ignore_index, lse_in,
                                                     lse_out, tgt_out, loss_out, coef_row, coef_scalar, write_grad,
                                                     vocab_total, err, rowsum_out);
  else
    ce_kernel<false><<<(unsigned)N, 256, 0, stream>>>((bf16*)logits, ld, V, labels, vocab_start, ignore_index,
                                                      lse_in, lse_out, tgt_out, loss_out, coef_row, coef_scalar,
                                                      write_grad, vocab_total, err, rowsum_out);
  return hipGetLastError();
}
