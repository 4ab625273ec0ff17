// hipBLASLt GEMMs with per-shape solution selection measured on the device (host-only C++).
//
// The projections and the lm_head are plain bf16 GEMMs: they belong on the vendor library, but its
// default heuristic picks a DepthU-32 MT256x256 kernel for the forward `x @ W^T` layout that runs at
// ~1.1 PF/s inside the Llama-3-8B step while the backward layouts run 1.3-1.5 PF/s
// (profiles/r2_llama8b_1gpu_forced_zero2_kernel_stats.md). This op asks hipBLASLt for its top
// candidates for the exact problem, times each on the live operands (random-like training data, not
// constant fill — constant data makes every kernel look faster through DVFS) writing into a scratch
// output, and caches the winner per problem key for the process (timing is opt-in: LLMT_GEMM_TUNE=1). Winners can be exported / imported
// as "key -> rank in the heuristic list" lines, which are stable for one library build.
//
// Column-major convention (hipBLASLt's): D[m, n] = alpha * op(A)[m, k] * op(B)[k, n] + beta * C.
// bf16 A/B, fp32 compute, bf16 or fp32 C = D.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <torch/library.h>

#include <algorithm>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

namespace {

// heuristic candidates timed per new problem (LLMT_GEMM_TUNE_TOPK overrides)
const int kCandidates = [] {
  const char* e = std::getenv("LLMT_GEMM_TUNE_TOPK");
  const int v = e ? std::atoi(e) : 24;
  return v > 0 ? v : 24;
}();
constexpr size_t kWorkspace = 128ull << 20;      // stream-K / split-K scratch

#define LT_CHECK(expr)                                                                    \
  do {                                                                                    \
    hipblasStatus_t _s = (expr);                                                          \
    TORCH_CHECK(_s == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #expr, " failed (", (int)_s, ")"); \
  } while (0)

struct Choice {
  hipblasLtMatmulAlgo_t algo;
  int rank;
  float ms;
  int gsu;  // 0: the solution as it is (hipblasLtMatmul); > 0: run through hipblaslt_ext::Gemm with GemmTuning splitK
};

// Split-K counts (hipBLASLt "GSU": the solution splits the contraction itself and reduces the partial tiles in
// the library, no fp32 slabs of ours) tried beside every timed candidate whose output has fewer than
// kGsuMaxTiles 256 x 256 tiles: the weight gradients of the projections fill the 256 CUs in 1-4 waves of tiles
// over a 32768-token contraction. LLMT_GEMM_GSU = comma-separated counts ("" or 0: off).
const std::vector<int> kGsu = [] {
  std::vector<int> v;
  const char* e = std::getenv("LLMT_GEMM_GSU");
  std::string t = e ? e : "";
  std::stringstream ss(t);
  std::string item;
  while (std::getline(ss, item, ',')) {
    const int x = std::atoi(item.c_str());
    if (x > 1) v.push_back(x);
  }
  return v;
}();
constexpr int64_t kGsuMaxTiles = 1024;

// interleaved timing rounds per timed problem (LLMT_GEMM_TUNE_ROUNDS, default 1)
const int kTuneRounds = [] {
  const char* e = std::getenv("LLMT_GEMM_TUNE_ROUNDS");
  const int v = e ? std::atoi(e) : 1;
  return v > 0 ? v : 1;
}();

// Problems restricted to non-stream-K solutions (dp > 1 / tp > 1, and the layout table's "/nosk" twins) take
// the heuristic's first non-stream-K solution (default), or time their candidates on first sight
// (LLMT_GEMM_NOSK_TIME=1). Alternating step runs on one box: the multi-GPU schedule on one GPU (every GEMM
// non-stream-K) 1462.0 / 1462.3 / 1466.7 ms heuristic vs 1461.9 / 1464.7 / 1463.8 timed, the one-GPU step
// 1451.5 / 1451.2 vs 1453.3 / 1453.7 (profiles/r6_nosk_time_ab.jsonl): the same speed, and the heuristic's
// choice is the same on every rank by construction, with no first-sight timing under collectives.
const bool kTimeNoSk = [] {
  const char* e = std::getenv("LLMT_GEMM_NOSK_TIME");
  return e && e[0] == '1';
}();

struct State {
  std::mutex mu;
  std::map<int, hipblasLtHandle_t> handles;
  std::map<std::string, Choice> cache;
  std::map<std::string, std::pair<int, int>> preset;  // imported winners: key -> (heuristic rank, GSU split)
  // Timing the candidates is opt-in (LLMT_GEMM_TUNE=1): on the Llama-3-8B shapes the heuristic's first
  // choice won every problem (benchmarks/bench_gemm_paths.py), and timing ~15 problems x 24 candidates
  // costs seconds of start-up.
  bool tune = [] {
    const char* e = std::getenv("LLMT_GEMM_TUNE");
    return e != nullptr && e[0] == '1';
  }();
};

State& st() {
  static State s;
  return s;
}

hipblasLtHandle_t handle_for(int dev) {
  auto& s = st();
  auto it = s.handles.find(dev);
  if (it != s.handles.end()) return it->second;
  hipblasLtHandle_t h;
  LT_CHECK(hipblasLtCreate(&h));
  s.handles[dev] = h;
  return h;
}

struct Desc {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  ~Desc() {
    if (op) hipblasLtMatmulDescDestroy(op);
    if (a) hipblasLtMatrixLayoutDestroy(a);
    if (b) hipblasLtMatrixLayoutDestroy(b);
    if (c) hipblasLtMatrixLayoutDestroy(c);
  }
};

void make_desc(Desc& d, bool ta, bool tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldc,
               hipDataType ctype) {
  LT_CHECK(hipblasLtMatmulDescCreate(&d.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.a, HIP_R_16BF, ta ? k : m, ta ? m : k, lda));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.b, HIP_R_16BF, tb ? n : k, tb ? k : n, ldb));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d.c, ctype, m, n, ldc));
}

// split-K as a strided batch: batch i multiplies the i-th contraction slice (A and B offsets along k) into
// its own [m, n] fp32 slab of C (batch stride m * n); the caller sums the slabs
void set_batch(Desc& d, bool ta, bool tb, int64_t m, int64_t n, int64_t kc, int64_t lda, int64_t ldb, int batch) {
  const int32_t bc = batch;
  const int64_t sa = ta ? kc : kc * lda, sb = tb ? kc * ldb : kc, sc = m * n;
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(d.a, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(d.b, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(d.c, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(d.a, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sa, sizeof(sa)));
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(d.b, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sb, sizeof(sb)));
  LT_CHECK(hipblasLtMatrixLayoutSetAttribute(d.c, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &sc, sizeof(sc)));
}

std::string key_of(bool ta, bool tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldc,
                   hipDataType ctype, bool beta, bool streamk, int batch = 1, bool bias = false) {
  std::ostringstream o;
  o << (ta ? 't' : 'n') << (tb ? 't' : 'n') << "_" << m << "_" << n << "_" << k << "_ld" << lda << "_" << ldb << "_"
    << ldc << (ctype == HIP_R_32F ? "_f32" : "_bf16") << (beta ? "_acc" : "") << (streamk ? "" : "_nosk");
  if (batch > 1) o << "_b" << batch;
  if (bias) o << "_bias";
  return o.str();
}

// Stream-K solutions (kernel names with "_SK") split a tile's K range over workgroups that hand partial
// sums to each other through the workspace, spinning until the partner's flag appears: they assume
// every workgroup of the launch (one per CU) is resident. When another kernel holds CUs at the same
// time (an RCCL collective or an AdamW on a side stream) the spin can wait on a workgroup that cannot
// start — one forward GEMM of a ZeRO-3 step was measured at 2.37 s instead of 3.7 ms
// (profiles/r2_zero3_streamk_stall.md). Callers that overlap communication ask for non-stream-K solutions.
bool is_streamk(hipblasLtHandle_t h, hipblasLtMatmulAlgo_t& algo) {
  const std::string name = hipblaslt_ext::getKernelNameFromAlgo(h, algo);
  return name.find("_SK") != std::string::npos;
}

// C (m x n, column-major) = op(A) . op(B) (+ C when accumulate); batch > 1: split-K into `batch` fp32 slabs
// of C (C is then [batch, n, m] fp32 with ldc = m, k divisible by batch)
// bias (optional, length m, bf16 or fp32): the BIAS epilogue, D = op(A) op(B) + bias broadcast over the n
// columns — for a linear layer's forward (column-major y^T = W . x^T) the bias of every output feature, added
// inside the GEMM instead of by a separate pass over y
void gemm_lt_impl(const at::Tensor& A, const at::Tensor& B, at::Tensor C, bool ta, bool tb, int64_t m, int64_t n,
                  int64_t k, int64_t lda, int64_t ldb, int64_t ldc, bool accumulate, bool streamk, int batch,
                  const c10::optional<at::Tensor>& bias = c10::nullopt) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm_lt: GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm_lt: bf16 A/B");
  TORCH_CHECK(C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kFloat, "gemm_lt: C bf16/fp32");
  if (m == 0 || n == 0) return;
  const hipDataType ctype = C.scalar_type() == at::kFloat ? HIP_R_32F : HIP_R_16BF;
  const int dev = C.get_device();
  hipStream_t stream = at::hip::getCurrentHIPStream(dev).stream();
  auto& s = st();
  std::lock_guard<std::mutex> lock(s.mu);
  hipblasLtHandle_t h = handle_for(dev);
  Desc d;
  TORCH_CHECK(batch >= 1 && k % batch == 0, "gemm_lt: k must divide into the split-K batch");
  make_desc(d, ta, tb, m, n, k / batch, lda, ldb, ldc, ctype);
  if (batch > 1) {
    TORCH_CHECK(ctype == HIP_R_32F && ldc == m && C.numel() >= batch * m * n, "gemm_lt: split-K slabs are fp32 [batch, n, m]");
    set_batch(d, ta, tb, m, n, k / batch, lda, ldb, batch);
  }
  const bool has_bias = bias.has_value() && bias->defined();
  if (has_bias) {
    TORCH_CHECK(batch == 1 && bias->is_cuda() && bias->is_contiguous() && bias->numel() == m &&
                    (bias->scalar_type() == at::kBFloat16 || bias->scalar_type() == at::kFloat),
                "gemm_lt: bias must be a contiguous bf16 / fp32 vector of length m");
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const void* bp = bias->data_ptr();
    const hipDataType bt = bias->scalar_type() == at::kFloat ? HIP_R_32F : HIP_R_16BF;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(d.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  const float alpha = 1.f, beta = accumulate ? 1.f : 0.f;
  auto ws = at::empty({(int64_t)kWorkspace}, C.options().dtype(at::kByte));
  const std::string key = key_of(ta, tb, m, n, k, lda, ldb, ldc, ctype, accumulate, streamk, batch, has_bias) +
                          (has_bias && bias->scalar_type() == at::kFloat ? "32" : "");
  auto it = s.cache.find(key);
  if (it == s.cache.end()) {
    hipblasLtMatmulPreference_t pref;
    LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsz = kWorkspace;
    LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz, sizeof(wsz)));
    // without stream-K the heuristic's first candidates can all be stream-K: ask for the whole list
    const int want = streamk ? kCandidates : 512;
    std::vector<hipblasLtMatmulHeuristicResult_t> res(want);
    int got = 0;
    LT_CHECK(hipblasLtMatmulAlgoGetHeuristic(h, d.op, d.a, d.b, d.c, d.c, pref, want, res.data(), &got));
    hipblasLtMatmulPreferenceDestroy(pref);
    if (!streamk) {  // drop stream-K solutions, keeping the heuristic order of the rest
      std::vector<hipblasLtMatmulHeuristicResult_t> keep;
      for (int i = 0; i < got; ++i)
        if (!is_streamk(h, res[i].algo)) keep.push_back(res[i]);
      if (!keep.empty()) {  // (on gfx950 some layouts have stream-K solutions only: then they stay)
        std::copy(keep.begin(), keep.end(), res.begin());
        got = (int)keep.size();
      }
      got = std::min(got, kCandidates);
    }
    TORCH_CHECK(got > 0, "gemm_lt: no hipBLASLt solution for ", key);
    Choice best{res[0].algo, 0, -1.f, 0};
    auto pre = s.preset.find(key);
    const bool gsu_try = !kGsu.empty() && batch == 1 && ((m + 255) / 256) * ((n + 255) / 256) < kGsuMaxTiles;
    if (pre != s.preset.end() && pre->second.first < got) {
      best = Choice{res[pre->second.first].algo, pre->second.first, 0.f, pre->second.second};
    } else if ((s.tune || (!streamk && kTimeNoSk) || gsu_try) && (got > 1 || gsu_try)) {
      // time every candidate on the live operands; the output goes to a scratch tensor so an
      // accumulating call (beta = 1) is not disturbed
      auto scratch = at::empty_like(C);
      if (accumulate) scratch.copy_(C);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      constexpr int kReps = 3;
      auto run_i = [&](int i) {
        return hipblasLtMatmul(h, d.op, &alpha, A.data_ptr(), d.a, B.data_ptr(), d.b, &beta, scratch.data_ptr(), d.c,
                               scratch.data_ptr(), d.c, &res[i].algo, ws.data_ptr(), kWorkspace, stream);
      };
      // kTuneRounds interleaved rounds of kReps runs per candidate, summed: more rounds time the candidates
      // under a longer, sustained load instead of one burst each
      std::vector<int> ok;
      for (int i = 0; i < got; ++i)
        if (res[i].state == HIPBLAS_STATUS_SUCCESS && run_i(i) == HIPBLAS_STATUS_SUCCESS) ok.push_back(i);  // warm-up
      std::vector<float> tot(got, 0.f);
      for (int rnd = 0; rnd < kTuneRounds; ++rnd)
        for (int i : ok) {
          (void)hipEventRecord(e0, stream);
          for (int r = 0; r < kReps; ++r) run_i(i);
          (void)hipEventRecord(e1, stream);
          (void)hipEventSynchronize(e1);
          float ms = 0.f;
          (void)hipEventElapsedTime(&ms, e0, e1);
          tot[i] += ms / kReps / kTuneRounds;
        }
      for (int i : ok)
        if (best.ms < 0.f || tot[i] < best.ms) best = Choice{res[i].algo, i, tot[i], 0};
      for (int i : ok) {
        if (!gsu_try) break;
        for (int gs : kGsu) {  // the same solution with the library's own split-K
          hipblaslt_ext::Gemm eg(h, d.op, &alpha, A.data_ptr(), d.a, B.data_ptr(), d.b, &beta, scratch.data_ptr(), d.c,
                                 scratch.data_ptr(), d.c);
          hipblaslt_ext::GemmTuning tun;
          tun.setSplitK((uint16_t)gs);
          size_t wsz = 0;
          if (eg.isAlgoSupported(res[i].algo, tun, wsz) != HIPBLAS_STATUS_SUCCESS || wsz > kWorkspace) continue;
          if (eg.initialize(res[i].algo, tun, ws.data_ptr(), false, stream) != HIPBLAS_STATUS_SUCCESS) continue;
          if (eg.run(stream) != HIPBLAS_STATUS_SUCCESS) continue;  // warm-up
          (void)hipEventRecord(e0, stream);
          for (int r = 0; r < kReps; ++r) (void)eg.run(stream);
          (void)hipEventRecord(e1, stream);
          (void)hipEventSynchronize(e1);
          float gms = 0.f;
          (void)hipEventElapsedTime(&gms, e0, e1);
          gms /= kReps;
          if (gms < best.ms) best = Choice{res[i].algo, i, gms, gs};
        }
      }
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
    }
    it = s.cache.emplace(key, best).first;
  }
  if (it->second.gsu > 0) {  // the library's split-K form of the chosen solution
    hipblaslt_ext::Gemm eg(h, d.op, &alpha, A.data_ptr(), d.a, B.data_ptr(), d.b, &beta, C.data_ptr(), d.c,
                           C.data_ptr(), d.c);
    hipblaslt_ext::GemmTuning tun;
    tun.setSplitK((uint16_t)it->second.gsu);
    size_t wsz = 0;
    hipblasLtMatmulAlgo_t algo = it->second.algo;
    LT_CHECK(eg.isAlgoSupported(algo, tun, wsz));
    LT_CHECK(eg.initialize(algo, tun, ws.data_ptr(), false, stream));
    LT_CHECK(eg.run(stream));
    return;
  }
  LT_CHECK(hipblasLtMatmul(h, d.op, &alpha, A.data_ptr(), d.a, B.data_ptr(), d.b, &beta, C.data_ptr(), d.c,
                           C.data_ptr(), d.c, &it->second.algo, ws.data_ptr(), kWorkspace, stream));
}

void gemm_lt(const at::Tensor& A, const at::Tensor& B, at::Tensor C, bool ta, bool tb, int64_t m, int64_t n,
             int64_t k, int64_t lda, int64_t ldb, int64_t ldc, bool accumulate, bool streamk) {
  gemm_lt_impl(A, B, C, ta, tb, m, n, k, lda, ldb, ldc, accumulate, streamk, 1);
}

void gemm_lt_bias(const at::Tensor& A, const at::Tensor& B, at::Tensor C, const at::Tensor& bias, bool ta, bool tb,
                  int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb, int64_t ldc, bool streamk) {
  gemm_lt_impl(A, B, C, ta, tb, m, n, k, lda, ldb, ldc, false, streamk, 1, bias);
}

// split-K form: C fp32 [batch, n, m] slabs, no accumulation (the caller reduces them)
void gemm_lt_splitk(const at::Tensor& A, const at::Tensor& B, at::Tensor C, bool ta, bool tb, int64_t m, int64_t n,
                    int64_t k, int64_t lda, int64_t ldb, int64_t batch, bool streamk) {
  gemm_lt_impl(A, B, C, ta, tb, m, n, k, lda, ldb, m, false, streamk, (int)batch);
}

// "key rank ms" lines of every problem tuned / used so far
std::string gemm_lt_export() {
  auto& s = st();
  std::lock_guard<std::mutex> lock(s.mu);
  std::ostringstream o;
  for (auto& kv : s.cache) {
    hipblasLtMatmulAlgo_t a = kv.second.algo;
    o << kv.first << " " << kv.second.rank << " " << kv.second.ms << " "
      << hipblaslt_ext::getKernelNameFromAlgo(s.handles.begin()->second, a) << " gsu" << kv.second.gsu << "\n";
  }
  return o.str();
}

// parses "key rank [ms kernel gsuN]" lines (gemm_lt_export's format) into the preset map; with `replace`, a
// cached choice of this process that differs is dropped, so the next call of that problem re-resolves to the
// imported one. Returns the number of lines read (replace = false) or of cached choices replaced.
int64_t read_presets(State& s, const std::string& text, bool replace) {
  std::istringstream in(text);
  std::string line;
  int64_t n = 0, replaced = 0;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    std::string key, ms, name, g;
    int rank;
    if (!(ls >> key >> rank)) continue;
    int gsu = 0;
    if (ls >> ms >> name >> g && g.rfind("gsu", 0) == 0) gsu = std::atoi(g.c_str() + 3);
    s.preset[key] = {rank, gsu};
    ++n;
    if (!replace) continue;
    auto it = s.cache.find(key);
    if (it != s.cache.end() && (it->second.rank != rank || it->second.gsu != gsu)) {
      s.cache.erase(it);
      ++replaced;
    }
  }
  return replace ? replaced : n;
}

int64_t gemm_lt_import(const std::string& text, bool tune_unknown) {
  auto& s = st();
  std::lock_guard<std::mutex> lock(s.mu);
  const int64_t n = read_presets(s, text, false);
  s.tune = tune_unknown;
  return n;
}

// Adopt another process's solution choices (rank 0's, broadcast by ops.fused.agree_layouts): every rank then
// runs the same hipBLASLt kernel per problem instead of the one its own first-sight timing picked (the
// non-stream-K candidates are timed per rank at dp > 1, under that rank's collectives). Problems not met yet
// take the adopted choice on first sight. Returns the number of this process's choices replaced.
int64_t gemm_lt_adopt(const std::string& text) {
  auto& s = st();
  std::lock_guard<std::mutex> lock(s.mu);
  return read_presets(s, text, true);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(llmt, m) {
  m.def(
      "gemm_lt(Tensor a, Tensor b, Tensor(a!) c, bool ta, bool tb, int m, int n, int k, int lda, int ldb, int ldc, "
      "bool accumulate, bool streamk=True) -> ()");
  m.def(
      "gemm_lt_splitk(Tensor a, Tensor b, Tensor(a!) c, bool ta, bool tb, int m, int n, int k, int lda, int ldb, "
      "int batch, bool streamk=True) -> ()");
  m.def(
      "gemm_lt_bias(Tensor a, Tensor b, Tensor(a!) c, Tensor bias, bool ta, bool tb, int m, int n, int k, int lda, "
      "int ldb, int ldc, bool streamk=True) -> ()");
  m.def("gemm_lt_export() -> str", &gemm_lt_export);
  m.def("gemm_lt_import(str text, bool tune_unknown) -> int", &gemm_lt_import);
  m.def("gemm_lt_adopt(str text) -> int", &gemm_lt_adopt);
}

TORCH_LIBRARY_IMPL(llmt, CUDA, m) {
  m.impl("gemm_lt", &gemm_lt);
  m.impl("gemm_lt_splitk", &gemm_lt_splitk);
  m.impl("gemm_lt_bias", &gemm_lt_bias);
}
