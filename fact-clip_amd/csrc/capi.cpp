// C-ABI entry points of libfactmx.so (declared in include/factmx.h).
//
// Composite ops (Linear fwd/bwd, the whole MS-TCN stack, the MHA core) are
// orchestrated here in C++ so one Python call launches the whole sequence on
// the caller's stream; kernels live in gemm_f32.hip, rowops.hip, segments.hip.
#include <algorithm>
#include <atomic>
#include <tuple>
#include <map>
#include <mutex>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "fx_common.h"
#include "ops.h"

namespace fx {

// ---- error state ------------------------------------------------------------
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// ---- profiling (opt-in diagnostic used by bench.py) ---------------------------
namespace {
struct ProfState {
  int max_events = 0;
  std::vector<hipEvent_t> ev;
  std::vector<double> flops, bytes;
  std::vector<int> launches;   // launches an event pair brackets (back-to-back chains: one pair)
  int used = 0;
  // kernel-time pairs (hipExtLaunchKernel) of the kernels launched inside this kind's brackets
  std::vector<hipEvent_t> kev;
  int kused = 0;
  int kdropped = 0;            // kernels launched in a bracket after the pool ran out (not timed)
  hipStream_t open_stream = nullptr;
};
constexpr int kProfKinds = 15;  // 0 conv GEMM, 1 / 2 attention over T fwd / bwd, 3-6 X2Y cores of frame-level
                                // calls (a2f fwd, a2f bwd, f2a fwd, f2a bwd), 7 fused MS-TCN layer, 8 persistent
                                // token-kernel launches (tokdec.hip), 9 SCA frame-memory K/V projection GEMM,
                                // 10 X2Y input projections (k, v, q), 11-14 X2Y cores of segment-level calls
std::mutex g_prof_mu;
ProfState g_prof[kProfKinds];
std::atomic<int> g_spin_override[2] = {{-1}, {-1}};   // fx_debug_set_spin: 0 token kernel, 1 X2Y f2a backward

void prof_reset(ProfState& p) {
  for (auto& e : p.ev) (void)hipEventDestroy(e);
  for (auto& e : p.kev) (void)hipEventDestroy(e);
  p = ProfState{};
}
}  // namespace

thread_local int g_prof_open = -1;

void prof_begin(int kind, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (kind < 0 || kind >= kProfKinds) return;
  ProfState& p = g_prof[kind];
  if (p.used >= p.max_events) return;
  (void)hipEventRecord(p.ev[2 * p.used], s);
  p.open_stream = s;
  g_prof_open = kind;
}

void prof_end(int kind, hipStream_t s, double flops, double bytes, int launches) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (kind < 0 || kind >= kProfKinds) return;
  if (g_prof_open == kind) g_prof_open = -1;
  ProfState& p = g_prof[kind];
  if (p.used >= p.max_events) return;
  (void)hipEventRecord(p.ev[2 * p.used + 1], s);
  p.flops[p.used] = flops;
  p.bytes[p.used] = bytes;
  p.launches[p.used] = launches;
  p.used++;
}

bool prof_kernel_events(hipStream_t s, hipEvent_t* e0, hipEvent_t* e1) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  const int kind = g_prof_open;
  if (kind < 0 || kind >= kProfKinds) return false;
  ProfState& p = g_prof[kind];
  if (s != p.open_stream) return false;   // (side / aux stream work launched from inside the call)
  if (2 * (size_t)(p.kused + 1) > p.kev.size()) {
    p.kdropped++;
    return false;
  }
  *e0 = p.kev[2 * p.kused];
  *e1 = p.kev[2 * p.kused + 1];
  p.kused++;
  return true;
}

unsigned tok_spin_max() {
  const int o = g_spin_override[0].load(std::memory_order_relaxed);
  if (o > 0) return (unsigned)o;
  return knobs().tok_spin > 0 ? (unsigned)knobs().tok_spin : (1u << 20);
}

unsigned x2y_spin_max() {
  const int o = g_spin_override[1].load(std::memory_order_relaxed);
  return o > 0 ? (unsigned)o : (1u << 22);
}

int coresident_blocks(const void* kernel, int threads, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, int, size_t>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_tuple(dev, kernel, threads, lds);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const int n = std::max(per_cu, 0) * std::max(cus, 0);
  cache[key] = n;
  return n;
}

// ---- helpers -------------------------------------------------------------------
namespace {

__global__ void relu_bwd_kernel(const float* dy, long long lddy, const float* y, long long ldy, int rows, int cols,
                                float* dz, long long lddz) {
  const long long total = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols, c = i % cols;
    dz[r * lddz + c] = y[r * ldy + c] > 0.f ? dy[r * lddy + c] : 0.f;
  }
}

__global__ void add2_kernel(const float* a, long long lda, const float* b, long long ldb, int rows, int cols,
                            float* o, long long ldo, int accumulate, int bcols) {
  const long long total = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols, c = i % cols;
    const float v = a[r * lda + c] + (b && c < bcols ? b[r * ldb + c] : 0.f);
    o[r * ldo + c] = accumulate ? o[r * ldo + c] + v : v;
  }
}

struct PackArgs {
  const float* w[32];
  float* wf[32];
  float* wb[32];
  const float* wpw[32];   // 1x1 weights (F_out, F_in) -> wpt = transposed (fused backward chain)
  float* wpt[32];
  int F;
};

// Conv1d weight (F_out=F, F_in=F, 3) -> Wf[n][j*F+c] (forward B) and Wb[c][j*F+n] (dX B);
// 1x1 weight W[o][c] -> Wt[c][o].  One 32 (out) x 32 (in) x 3 (tap) tile per workgroup through LDS:
// coalesced reads of the (F, F, 3) rows and coalesced 32-float writes of both packed images (the
// element-wise version scattered every Wb write: 85 us per 10-layer F = 512 stack).
__global__ __launch_bounds__(256) void pack_conv_kernel(PackArgs p) {
  const int l = blockIdx.z, F = p.F;
  const int c0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  __shared__ float t[3][32][33];                              // [tap][out - n0][in - c0]
  const float* w = p.w[l];
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r;
    for (int e = tx; e < 96; e += 32) {
      const int cl = e / 3, j = e - cl * 3;
      t[j][r][cl] = (n < F && c0 + cl < F) ? w[(long long)n * 3 * F + (long long)(c0 + cl) * 3 + j] : 0.f;
    }
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r, c = c0 + r;
    if (n < F && c0 + tx < F)
#pragma unroll
      for (int j = 0; j < 3; ++j) p.wf[l][(long long)n * 3 * F + j * F + c0 + tx] = t[j][r][tx];
    if (c < F && n0 + tx < F)
#pragma unroll
      for (int j = 0; j < 3; ++j) p.wb[l][(long long)c * 3 * F + j * F + n0 + tx] = t[j][tx][r];
  }
  if (p.wpt[l]) {
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
      const int o = n0 + r;
      t[0][r][tx] = (o < F && c0 + tx < F) ? p.wpw[l][(long long)o * F + c0 + tx] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
      const int c = c0 + r;
      if (c < F && n0 + tx < F) p.wpt[l][(long long)c * F + n0 + tx] = t[0][tx][r];
    }
  }
}

}  // namespace

int ew_grid(long long total) { return (int)std::min<long long>(std::max<long long>(cdiv(total, 256), 1), 4096); }

int relu_bwd(const float* dy, long long lddy, const float* y, long long ldy, int rows, int cols, float* dz,
             long long lddz, hipStream_t s) {
  if ((long long)rows * cols == 0) return FX_OK;
  fx_launch(relu_bwd_kernel, dim3(ew_grid((long long)rows * cols)), dim3(256), 0, s, dy, lddy, y, ldy, rows,
                     cols, dz, lddz);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int add2(const float* a, long long lda, const float* b, long long ldb, int rows, int cols, float* o, long long ldo,
         int accumulate, hipStream_t s, int bcols) {
  if ((long long)rows * cols == 0) return FX_OK;
  fx_launch(add2_kernel, dim3(ew_grid((long long)rows * cols)), dim3(256), 0, s, a, lda, b, ldb, rows, cols,
                     o, ldo, accumulate, bcols < 0 ? cols : bcols);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

// split-K factor for small-output / long-K products (dW over frames, token x frame)
int pick_split(int M, int N, int K, int batch) {
  const int nkt = cdiv(K, 64);   // 64-deep K stages of the GEMM kernel
  if (nkt < 4) return 1;
  // whole 64-deep stages and >= 128 rows: the launch can take the 128x64 tile (8 waves), so count
  // those tiles; one block per CU: keep tiles*split within the 256 CUs, no straggler round
  const bool wide = M >= 128 && K % 64 == 0;
  const long long tiles = (long long)cdiv(M, wide ? 128 : 64) * cdiv(N, 64) * batch;
  if (tiles >= 160) return 1;
  int sp = (int)std::min<long long>(nkt / 2, 256 / tiles);
  return std::max(sp, 1);
}

long long split_ws(int M, int N, int K, int batch) {
  const int sp = pick_split(M, N, K, batch);
  return sp > 1 ? (long long)sp * M * N * batch : 0;
}

// y = (x [+pos on the first pos_cols columns]) . w^T (+b) (+relu);  w (N,K) with row stride ldw
int linear_fwd(const float* x, long long ldx, int M, int K, const float* w, const float* b, float* y, long long ldy,
               int N, int relu, hipStream_t s, long long ldw, const float* pos, long long ldpos, int pos_cols) {
  fx_gemm_desc d = gemm_desc(M, N, K, op_rows(x, ldx), op_rows(w, ldw < 0 ? K : ldw), y, ldy);
  d.a.pos = pos;
  d.a.ld_pos = ldpos;
  d.a.pos_cols = pos ? pos_cols : 0;
  d.bias = b;
  d.relu = relu;
  return launch_gemm(d, s);
}

// dx (+)= dy . w  [* (gate > 0)];  w (N,K)
fx_gemm_desc desc_linear_dx(const float* dy, long long lddy, const float* w, int M, int K, int N, float* dx,
                            long long lddx, int accumulate, const float* gate, long long ld_gate, float* ws,
                            long long ldw) {
  fx_gemm_desc d = gemm_desc(M, K, N, op_rows(dy, lddy), op_cols(w, ldw < 0 ? K : ldw), dx, lddx);
  d.beta = accumulate ? 1.f : 0.f;
  d.gate = gate;
  d.ld_gate = ld_gate;
  d.split_k = pick_split(M, K, N);
  d.workspace = ws;
  return d;
}

int linear_dx(const float* dy, long long lddy, const float* w, int M, int K, int N, float* dx, long long lddx,
              int accumulate, const float* gate, long long ld_gate, float* ws, hipStream_t s, long long ldw) {
  return launch_gemm(desc_linear_dx(dy, lddy, w, M, K, N, dx, lddx, accumulate, gate, ld_gate, ws, ldw), s);
}

// dw (+)= dy^T . x  and  db (+)= colsum(dy)  in ONE GEMM: x gets a virtual all-ones column K
// whose output column (the bias gradient) is routed to db.  dy (M,N), x (M,K) -> dw (N,K), ld lddw.
// (no dw and no db: an empty desc, M = 0, that launch_gemm / launch_gemm_group skip)
fx_gemm_desc desc_linear_dwdb(const float* dy, long long lddy, const float* x, long long ldx, int M, int K, int N,
                              float* dw, float* db, int accumulate, float* ws, long long lddw) {
  if (!dw) {
    fx_gemm_desc e{};
    e.batch = 1;
    e.c_last_col = db;   // (a bias-only request: linear_bwd_pair refuses it like linear_dwdb)
    return e;
  }
  fx_operand b = op_cols(x, ldx);
  const int Kc = K + (db ? 1 : 0);
  if (db) b.ones_col = K + 1;
  fx_gemm_desc d = gemm_desc(N, Kc, M, op_cols(dy, lddy), b, dw, lddw < 0 ? K : lddw);
  d.c_last_col = db;
  d.beta = accumulate ? 1.f : 0.f;
  // split sized for the K+1 columns dwdb_ws() reserves, with or without the bias column: counting
  // only K columns can pick a larger split (fewer tiles) than the reservation holds
  d.split_k = pick_split(N, K + 1, M);
  d.workspace = ws;
  return d;
}

int linear_dwdb(const float* dy, long long lddy, const float* x, long long ldx, int M, int K, int N, float* dw,
                float* db, int accumulate, float* ws, hipStream_t s, long long lddw) {
  if (!dw && !db) return FX_OK;
  FX_REQUIRE(dw, "linear_dwdb: bias-only gradient needs dw");
  return launch_gemm(desc_linear_dwdb(dy, lddy, x, ldx, M, K, N, dw, db, accumulate, ws, lddw), s);
}

// The two independent backward GEMMs of one linear layer (dW/db = dY^T X, dX = dY W): one launch
// when both take the direct kernel (token-level shapes), else two.
int linear_bwd_pair(const fx_gemm_desc& dwdb, const fx_gemm_desc& dx, hipStream_t s) {
  FX_REQUIRE(!(dwdb.c_last_col && !dwdb.c), "linear_dwdb: bias-only gradient needs dw");
  const fx_gemm_desc pr[2] = {dwdb, dx};
  return launch_gemm_group(pr, 2, s);
}

int linear_dw(const float* dy, long long lddy, const float* x, long long ldx, int M, int K, int N, float* dw,
              int accumulate, float* ws, hipStream_t s, long long lddw) {
  return linear_dwdb(dy, lddy, x, ldx, M, K, N, dw, nullptr, accumulate, ws, s, lddw);
}

long long dwdb_ws(int M, int K, int N) { return split_ws(N, K + 1, M); }

namespace {

// ---- side stream for overlapping independent GEMMs (one per device, created on first use) ----
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t to_side[3] = {};
  hipEvent_t layer_done[4] = {};
  hipEvent_t join = nullptr;
  // a second, short-lived helper stream for work whose result the caller's stream needs before the
  // entry point returns (no backlog of deferred weight gradients in front of it)
  hipStream_t aux = nullptr;
  hipEvent_t aux_fork = nullptr, aux_done = nullptr;
};

SideStream* side_stream() {
  if (!knobs().side_stream) return nullptr;   // FX_SIDE_STREAM=0: everything on the caller's stream
  static std::mutex mu;
  static std::map<int, SideStream*> pool;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = pool.find(dev);
  if (it != pool.end()) return it->second;
  SideStream* ss = new SideStream();
  // normal priority (the side stream at low priority measured slower: round 3).  FX_SIDE_PRIO_BUILD (a
  // diagnostic build define, -1 low / 1 high) builds the other priorities for A/B runs
#ifndef FX_SIDE_PRIO_BUILD
#define FX_SIDE_PRIO_BUILD 0
#endif
  int prio = 0, least = 0, greatest = 0;
  if (FX_SIDE_PRIO_BUILD != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
    prio = FX_SIDE_PRIO_BUILD < 0 ? least : greatest;
  bool ok = hipStreamCreateWithPriority(&ss->s, hipStreamNonBlocking, prio) == hipSuccess;
  for (auto& e : ss->to_side) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  for (auto& e : ss->layer_done) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&ss->join, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipStreamCreateWithPriority(&ss->aux, hipStreamNonBlocking, prio) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&ss->aux_fork, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&ss->aux_done, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    delete ss;   // (a partially created set leaks its handles; the caller falls back to one stream)
    return nullptr;
  }
  pool[dev] = ss;
  return ss;
}

// ---- MS-TCN layout of saved activations / workspace --------------------------------
struct MstcnLayout {
  // every per-layer row slot holds rows_pad = rows rounded up to the 64-deep GEMM stage; the pad rows of
  // the h / z slots (forward) and of the deferred dZ / dH / dB slots (backward) are zero, so the deferred
  // weight-gradient GEMMs run over K = rows_pad on the FAST loaders (ragged batches included)
  long long rows_pad;
  long long rowsF;
  // saved
  long long h, z, xh, rs, wbs, wpts, wk1b, wk2b, total_saved;
  // workspace
  long long wf, wk1, wk2, buf0, buf1, buf2, buf3, buf4, buf5, split, split2, colsum, dzall, dhall, dball, csb, bsl,
      total_ws;
};

// Split of the deferred batched weight-gradient GEMMs (fx_mstcn_bwd): each workgroup of a batched
// launch otherwise walks all K = rows and holds its CU for the whole launch, so the main stream's
// next kernels wait for CUs; 16 caps a workgroup's share at K / 16 (16 vs 8: 15.78 vs 15.95 ms, median
// of 6 pairs, round 3)
#ifndef FX_DEFER_SPLIT_BUILD
#define FX_DEFER_SPLIT_BUILD 16   // (a diagnostic build define for A/B runs)
#endif
int defer_split_impl(int rows) { return std::max(1, std::min(FX_DEFER_SPLIT_BUILD, rows / 512)); }

MstcnLayout mstcn_layout(const fx_mstcn_params* p, int rows) {
  MstcnLayout L{};
  const long long F = p->F;
  const int NL = p->num_layers;
  L.rows_pad = (long long)cdiv(rows, 64) * 64;
  L.rowsF = L.rows_pad * F;
  L.h = 0;                                   // h_0 .. h_NL
  L.z = L.h + (NL + 1) * L.rowsF;            // z_0 .. z_{NL-1}
  L.xh = L.z + NL * L.rowsF;                 // LN xhat_i
  L.rs = L.xh + (p->layernorm ? NL * L.rowsF : 0);
  L.wbs = L.rs + (p->layernorm ? (long long)NL * rows : 0);   // dX-packed conv weights (fwd packs, bwd reads)
  const long long wsz = 3 * F * F;
  L.wpts = L.wbs + NL * wsz;                 // transposed 1x1 weights (fwd packs, bwd dZ GEMM reads)
  L.wk1b = L.wpts + NL * F * F;              // fused layers: the backward chain's weights (the two above) in
  L.wk2b = L.wk1b + (p->fused_layers ? NL * wsz : 0);   // MFMA fragment order, packed by the forward
  L.total_saved = L.wk2b + (p->fused_layers ? NL * F * F : 0);
  L.wf = 0;
  L.wk1 = L.wf + NL * wsz;                   // fused layers: conv weights in MFMA fragment order
  L.wk2 = L.wk1 + (p->fused_layers ? NL * wsz : 0);   // ... and the 1x1 weights
  L.buf0 = L.wk2 + (p->fused_layers ? NL * F * F : 0);
  L.buf1 = L.buf0 + L.rowsF;
  L.buf2 = L.buf1 + L.rowsF;
  L.buf3 = L.buf2 + L.rowsF;                 // backward: third dH buffer, second dZ buffer (side stream)
  L.buf4 = L.buf3 + L.rowsF;
  L.buf5 = L.buf4 + L.rowsF;                 // third dZ buffer (fused backward chain)
  L.split = L.buf5 + L.rowsF;
  long long sp = 0;
  sp = std::max(sp, split_ws(p->F, 3 * p->F + 1, rows));      // conv dW (+ bias column)
  sp = std::max(sp, dwdb_ws(rows, p->F, p->F));               // pointwise dW
  sp = std::max(sp, split_ws(rows, p->F, p->F));              // pointwise dX (few rows: split K)
  sp = std::max(sp, dwdb_ws(rows, p->F, p->cout));            // out dW
  if (p->in_map) sp = std::max(sp, dwdb_ws(rows, p->cin, p->F));  // in dW
  sp = std::max(sp, split_ws(rows, p->F, p->cout));           // dH_L
  if (p->in_map) sp = std::max(sp, split_ws(rows, p->cin, p->F));
  sp = std::max(sp, layernorm_bwd_ws_floats(rows, p->F));
  L.split2 = L.split + sp;                   // split-K partials of the main stream's GEMMs
  L.colsum = L.split2 + sp;
  long long cs = colsum_workspace_floats(rows, std::max(std::max(p->F, p->cout), p->cin));
  // deferred weight gradients (fx_mstcn_bwd): every layer's dZ_i and dH_i+1 kept for the batched
  // dW GEMMs, and the batched conv-bias column sums
  L.dzall = L.colsum + cs;
  L.dhall = L.dzall + NL * L.rowsF;
  L.dball = L.dhall + NL * L.rowsF;          // training dropout: dB_i = dropout_i(dH_i+1), the 1x1 branch's gradient
  L.csb = L.dball + (p->dropout > 0.f ? NL * L.rowsF : 0);
  L.bsl = L.csb + (long long)NL * colsum_workspace_floats(rows, p->F);
  const int dsp = defer_split_impl(rows);
  L.total_ws = L.bsl + std::max(split_ws(p->F, p->F + 1, rows, std::max(NL, 1)),
                                dsp > 1 ? (long long)dsp * std::max(NL, 1) * p->F * (3LL * p->F) : 0LL);
  return L;
}

int pack_conv_weights(const fx_mstcn_params* p, float* ws, float* wbdst, float* wptdst, const MstcnLayout& L,
                      hipStream_t s) {
  PackArgs a{};
  a.F = p->F;
  const long long wsz = 3LL * p->F * p->F;
  for (int l = 0; l < p->num_layers; ++l) {
    a.w[l] = p->w_dil[l];
    a.wf[l] = ws + L.wf + l * wsz;
    a.wb[l] = wbdst + l * wsz;
    a.wpw[l] = p->w_pw[l];
    a.wpt[l] = wptdst ? wptdst + (long long)l * p->F * p->F : nullptr;
  }
  fx_launch(pack_conv_kernel, dim3(cdiv(p->F, 32), cdiv(p->F, 32), p->num_layers), dim3(256), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

// the fused layer kernel's weights: every layer's conv matrix (ld 3F) and 1x1 matrix (ld F) in fragment
// order, appended to a job list; the 1x1 sources are a per-layer pointer list or a base with a uniform
// stride
void frag_layer_jobs(std::vector<FragJob>& J, int NL, int F, const float* w1, long long w1_stride,
                     const float* const* w2list, const float* w2, long long w2_stride, float* dst1, float* dst2) {
  for (int l = 0; l < NL; ++l) {
    J.push_back({w1 + (long long)l * w1_stride, dst1 + (long long)l * frl_packed_floats(3 * F), 3 * F, 3 * F});
    J.push_back({w2list ? w2list[l] : w2 + (long long)l * w2_stride, dst2 + (long long)l * frl_packed_floats(F), F, F});
  }
}

int launch_frag_jobs(const std::vector<FragJob>& J, hipStream_t s) {
  for (size_t i = 0; i < J.size(); i += FRAG_JOBS)
    FX_TRY(launch_pack_frag(J.data() + i, (int)std::min<size_t>(FRAG_JOBS, J.size() - i), s));
  return FX_OK;
}

// whether fx_mstcn_fwd ran the fused layers (and so packed the backward chain's weights into `saved`)
bool mstcn_fwd_fused(const fx_mstcn_params* p, int nvid, bool ragged, int rows, const float* saved) {
  return p->fused_layers && !p->layernorm && frl_supported(p->F, saved, p->F, p->F) && (!ragged || nvid <= 16) &&
         (p->fused_layers == 2 || frl_fills_device(rows));
}

int layer_dilation(const fx_mstcn_params* p, int i) {
  long long d = p->dil0 > 0 ? p->dil0 : 1;
  const int f = p->dil_factor > 0 ? p->dil_factor : 2;
  for (int k = 0; k < i; ++k) d *= f;
  return (int)d;
}

// The batched weight-gradient GEMMs of fx_mstcn_bwd address layer i's gradients as layer 0's plus
// i times one stride: true for views of one flat gradient buffer in parameter order (FlatGradReducer).
// FX_MSTCN_DEFER=0 keeps the per-layer interleaved GEMMs (A/B).
bool mstcn_defer_ok(const fx_mstcn_params* p, const fx_mstcn_grads* g) {
  if (!knobs().mstcn_defer) return false;
  const int NL = p->num_layers;
  for (int i = 0; i < NL; ++i)
    if (!g->w_dil[i] || !g->b_dil[i] || !g->w_pw[i] || !g->b_pw[i]) return false;
  auto uniform = [&](float* const* v) {
    for (int i = 2; i < NL; ++i)
      if (v[i] - v[i - 1] != v[1] - v[0]) return false;
    return true;
  };
  return uniform(g->w_dil) && uniform(g->b_dil) && uniform(g->w_pw) && uniform(g->b_pw);
}

// The videos of a frame-level call: nvid of T rows each, or ragged host offsets off (nvid + 1).
struct Seqs {
  int T, nvid;
  const int* off;
  int rows() const { return off ? off[nvid] : T * nvid; }
  int start(int v) const { return off ? off[v] : v * T; }
  int len(int v) const { return off ? off[v + 1] - off[v] : T; }
};

int check_seqs(const Seqs& q) {
  FX_REQUIRE(q.nvid >= 1, "frame branch: nvid >= 1");
  if (!q.off) {
    FX_REQUIRE(q.T >= 1, "frame branch: T >= 1");
    return FX_OK;
  }
  FX_REQUIRE(q.nvid <= 16 && q.off[0] == 0, "frame branch: ragged offsets start at 0, <= 16 videos");
  for (int v = 0; v < q.nvid; ++v) FX_REQUIRE(q.off[v + 1] > q.off[v], "frame branch: empty video");
  return FX_OK;
}

// dilated-conv operand over the call's videos (zero outside each video).  The column-major (weight-
// gradient) form of a ragged call needs K padded to whole 64-deep stages (gemm_f32.hip COLS_CONVR): the
// per-layer weight gradients (K = rows) run video by video instead.
fx_operand conv_operand(const float* h, long long ld, int cin, int dil, int dir, const Seqs& q, bool trans) {
  fx_operand o = trans ? op_cols(h, ld) : op_rows(h, ld);
  o.conv_taps = 3;
  o.conv_cin = cin;
  o.conv_dil = dil;
  o.conv_dir = dir;
  if (q.off) {   // (column-major: FAST loaders only, K padded to whole stages -- the deferred dW GEMMs)
    o.seq_off = q.off;
    o.nseq = q.nvid;
  } else {
    o.seq_len = q.T;
  }
  return o;
}

// fn(row0, rows, seqs) once over all rows (uniform videos) or once per video (ragged): the weight-
// gradient GEMMs whose K runs over frames
template <typename Fn>
int per_video(const Seqs& q, Fn fn) {
  if (!q.off) return fn(0, q.rows(), q);
  for (int v = 0; v < q.nvid; ++v) FX_TRY(fn(q.start(v), q.len(v), Seqs{q.len(v), 1, nullptr}));
  return FX_OK;
}

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

int fx_version(void) { return FX_ABI_VERSION; }

}  // extern "C"

namespace fx {
const Knobs& knobs() {
  static Knobs k;
  static std::once_flag once;
  std::call_once(once, [] {
    auto env = [](const char* n) -> const char* { return std::getenv(n); };
    if (const char* p = env("FX_GEMM_PATH")) k.gemm_path = std::string(p) == "tiled" ? 1 : std::string(p) == "direct" ? 2 : 0;
    if (const char* p = env("FX_GEMM_W8")) k.gemm_w8 = p[0] == '1';
    if (const char* p = env("FX_GEMM_WIDE")) k.gemm_wide = p[0] == '1' ? 1 : 0;
    if (const char* p = env("FX_GEMM_XCDPLANES")) k.gemm_xcd_planes = p[0] != '0';
    if (const char* p = env("FX_GEMM_GROUP")) k.gemm_group = p[0] != '0';
    if (const char* p = env("FX_GEMM_KTAIL")) k.gemm_ktail = p[0] != '0';
    if (const char* p = env("FX_DEC_TOK")) k.dec_tok = p[0] != '0';
    if (const char* p = env("FX_TOK_SPIN")) k.tok_spin = std::max(0, std::atoi(p));
    if (const char* p = env("FX_SIDE_STREAM")) k.side_stream = p[0] != '0';
    if (const char* p = env("FX_MSTCN_DEFER")) k.mstcn_defer = p[0] != '0';
    if (const char* p = env("FX_GEMM_ROWPERM")) k.gemm_row_perm = p[0] != '0';
    if (const char* p = env("FX_GEMM_GROUPM")) k.gemm_group_m = p[0] != '0';
    if (const char* p = env("FX_GEMM_PERSIST")) k.gemm_persist = p[0] != '0';
    if (const char* p = env("FX_FRL_XCD")) k.frl_xcd = std::atoi(p);
    if (const char* p = env("FX_FRL_PAIR")) k.frl_pair = p[0] != '0';
    if (const char* p = env("FX_FRL_MIN_FILL")) k.frl_min_fill = std::atoi(p);
    if (const char* p = env("FX_AUX_STREAM")) k.aux_stream = p[0] != '0';
    if (const char* p = env("FX_GRU_POLL2")) k.gru_poll2 = p[0] != '0';
    if (const char* p = env("FX_GRU_STORE_WAVE")) k.gru_store_wave = std::max(0, std::min(2, std::atoi(p)));
    if (const char* p = env("FX_TATTN_RR")) k.tattn_rr = p[0] != '0';
    if (const char* p = env("FX_X2Y_A2F_DW")) k.x2y_a2f_dw = p[0] != '0';
    if (const char* p = env("FX_TATTN_FOLD")) k.tattn_fold = p[0] != '0';
    if (const char* p = env("FX_X2Y_FUSED")) k.x2y_fused = p[0] != '0';
    if (const char* p = env("FX_X2Y_F2A_BWD")) k.x2y_f2a_bwd = std::atoi(p);
    if (const char* p = env("FX_X2Y_F2A_ONE")) k.x2y_f2a_one = p[0] != '0';
  });
  return k;
}
}  // namespace fx

extern "C" {
const char* fx_last_error(void) { return g_last_error.c_str(); }

int fx_dropout(const float* x, long long ldx, int rows, int cols, long long idx_ld, long long idx_col0, float p,
               unsigned long long seed, float* y, long long ldy, void* stream) {
  FX_REQUIRE(x && y && rows >= 0 && cols >= 0, "dropout: bad arguments");
  return launch_dropout(x, ldx, rows, cols, idx_ld, idx_col0, p, seed, y, ldy, (hipStream_t)stream);
}

long long fx_struct_size(int which) {
  switch (which) {
    case 0: return (long long)sizeof(fx_gemm_desc);
    case 1: return (long long)sizeof(fx_decoder_params);
    case 2: return (long long)sizeof(fx_mstcn_params);
    case 3: return (long long)sizeof(fx_loss_term);
    case 4: return (long long)sizeof(fx_video_attn);
    case 5: return (long long)sizeof(fx_mstcn2_params);
    default: return -1;
  }
}

int fx_gemm(const fx_gemm_desc* desc, void* stream) {
  FX_REQUIRE(desc, "fx_gemm: null descriptor");
  // implicit dilated-conv GEMMs (A = shifted-tap operand: conv forward / conv dX, e.g. MSTCN2) are
  // the same kernel class the bench times inside fx_mstcn_*
  const bool conv = desc->a.conv_taps && !desc->a.trans;
  if (conv) prof_begin(0, (hipStream_t)stream);
  const int st = launch_gemm(*desc, (hipStream_t)stream);
  if (conv) prof_end(0, (hipStream_t)stream, 2.0 * desc->M * desc->N * desc->K * desc->batch, 0.0);
  return st;
}

long long fx_gemm_workspace_floats(const fx_gemm_desc* desc) { return desc ? gemm_workspace_floats(*desc) : 0; }

// ---------------------------------------------------------------- Linear
int fx_linear_fwd(const float* x, long long ldx, const float* pos, long long ldpos, int pos_cols, int M, int K,
                  const float* w, long long ldw, const float* b, float* y, long long ldy, int N, int relu,
                  void* stream) {
  return linear_fwd(x, ldx, M, K, w, b, y, ldy, N, relu, (hipStream_t)stream, ldw, pos, ldpos, pos_cols);
}

long long fx_linear_bwd_workspace_floats(int M, int K, int N) {
  return (long long)M * N + split_ws(M, K, N) + dwdb_ws(M, K, N) + colsum_workspace_floats(M, N);
}

int fx_linear_bwd(const float* dy, long long lddy, const float* x, long long ldx, const float* w, long long ldw,
                  const float* relu_out, long long ld_relu, int M, int K, int N, float* dx, long long lddx,
                  float* dw, long long lddw, float* db, int accumulate_dx, int accumulate_w, float* workspace,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  FX_REQUIRE(workspace || (!relu_out && split_ws(M, K, N) == 0 && dwdb_ws(M, K, N) == 0 && !(db && !dw)),
             "fx_linear_bwd: workspace required");
  float* wz = workspace;
  float* wsx = wz + (long long)M * N;
  float* wsw = wsx + split_ws(M, K, N);
  float* wsc = wsw + dwdb_ws(M, K, N);
  const float* g = dy;
  long long ldg = lddy;
  if (relu_out) {
    FX_TRY(relu_bwd(dy, lddy, relu_out, ld_relu, M, N, wz, N, s));
    g = wz;
    ldg = N;
  }
  if (dx) {
    WsBound wb(wsx, split_ws(M, K, N));
    FX_TRY(linear_dx(g, ldg, w, M, K, N, dx, lddx, accumulate_dx, nullptr, 0, wsx, s, ldw));
  }
  if (dw) {
    WsBound wb(wsw, dwdb_ws(M, K, N));
    FX_TRY(linear_dwdb(g, ldg, x, ldx, M, K, N, dw, db, accumulate_w, wsw, s, lddw));
  }
  else if (db) FX_TRY(launch_colsum(g, ldg, M, N, db, accumulate_w, wsc, s));
  return FX_OK;
}

// ---------------------------------------------------------------- MS-TCN
long long fx_mstcn_saved_floats(const fx_mstcn_params* p, int rows) { return mstcn_layout(p, rows).total_saved; }
long long fx_mstcn_workspace_floats(const fx_mstcn_params* p, int rows) { return mstcn_layout(p, rows).total_ws; }

int fx_mstcn_fwd(const fx_mstcn_params* p, const float* x, long long ldx, int T, int nvid, float* y, long long ldy,
                 float* saved, float* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  FX_REQUIRE(p && p->num_layers >= 0 && p->num_layers <= 32, "mstcn: 0..32 layers");
  FX_REQUIRE(p->in_map || p->cin == p->F, "mstcn: in_map=0 needs cin == F");
  const Seqs q{T, nvid, p->seq_off};
  FX_TRY(check_seqs(q));
  const int rows = q.rows();
  const int F = p->F;
  const MstcnLayout L = mstcn_layout(p, rows);
  FX_TRY(pack_conv_weights(p, workspace, saved + L.wbs, saved + L.wpts, L, s));
  if (L.rows_pad > rows && p->num_layers > 0)   // pad rows of h_0 .. h_NL, z_0 .. z_NL-1 (adjacent slots)
    FX_CHECK_HIP(hipMemset2DAsync(saved + L.h + (long long)rows * F, L.rowsF * sizeof(float), 0,
                                  (L.rows_pad - rows) * F * sizeof(float), 2 * p->num_layers + 1, s));
  float* h0 = saved + L.h;
  if (p->in_map) {
    FX_TRY(linear_fwd(x, ldx, rows, p->cin, p->w_in, p->b_in, h0, F, F, 0, s));
  } else {
    FX_CHECK_HIP(hipMemcpy2DAsync(h0, F * sizeof(float), x, ldx * sizeof(float), F * sizeof(float), rows,
                                  hipMemcpyDeviceToDevice, s));
  }
  const bool fused = mstcn_fwd_fused(p, q.nvid, q.off != nullptr, rows, saved);
  if (fused && p->num_layers > 0) {
    // one launch: this pass's weights (conv from the pack above, 1x1 as given) and the backward chain's
    // (the dX-packed conv and transposed 1x1 weights packed above into `saved`), so the backward packs none
    std::vector<FragJob> J;
    frag_layer_jobs(J, p->num_layers, F, workspace + L.wf, 3LL * F * F, p->w_pw, nullptr, 0, workspace + L.wk1,
                    workspace + L.wk2);
    frag_layer_jobs(J, p->num_layers, F, saved + L.wbs, 3LL * F * F, nullptr, saved + L.wpts, (long long)F * F,
                    saved + L.wk1b, saved + L.wk2b);
    FX_TRY(launch_frag_jobs(J, s));
  }
  for (int i = 0; i < p->num_layers; ++i) {
    const float* hi = saved + L.h + i * L.rowsF;
    float* hn = saved + L.h + (i + 1) * L.rowsF;
    float* zi = saved + L.z + i * L.rowsF;
    if (fused) {   // z = relu(conv(h) + b); h' = h + dropout(z . Wpw^T + b): one kernel (mstcn_fused.hip)
      // (timed as one chain: an event pair around every launch would add its own dispatch gap)
      if (i == 0) prof_begin(7, s);
      FX_TRY(launch_frl(hi, F, rows, T, layer_dilation(p, i), 1, q.off, q.nvid,
                        workspace + L.wk1 + (long long)i * 3 * F * F, p->b_dil[i], 1, nullptr, 0, zi, F,
                        workspace + L.wk2 + (long long)i * F * F, p->b_pw[i], hi, F, nullptr, 0, hn, F, p->dropout,
                        fx_drop_subseed(p->seed, i), s));
      if (i == p->num_layers - 1)
        prof_end(7, s, p->num_layers * 2.0 * rows * F * 4.0 * F, p->num_layers * 4.0 * (3.0 * rows * F + 4.0 * F * F),
                 p->num_layers);
      continue;
    }
    // z = relu(dilated_conv(h) + b)      (basic.py:158)
    fx_gemm_desc d = gemm_desc(rows, F, 3 * F, conv_operand(hi, F, F, layer_dilation(p, i), 1, q, false),
                               op_rows(workspace + L.wf + (long long)i * 3 * F * F, 3 * F), zi, F);
    d.bias = p->b_dil[i];
    d.relu = 1;
    prof_begin(0, s);
    FX_TRY(launch_gemm(d, s));
    prof_end(0, s, 2.0 * rows * F * 3.0 * F, 4.0 * (2.0 * rows * F + 3.0 * F * F));
    // h' = h + z . Wpw^T + b   [then LN]   (basic.py:159-169)
    float* u = p->layernorm ? workspace + L.buf0 : hn;
    fx_gemm_desc e = gemm_desc(rows, F, F, op_rows(zi, F), op_rows(p->w_pw[i], F), u, F);
    e.bias = p->b_pw[i];
    e.resid = hi;
    e.ld_resid = F;
    e.drop_p = p->dropout;   // h' = h + dropout(z . Wpw^T + b)   (basic.py:160)
    e.drop_seed = fx_drop_subseed(p->seed, i);
    FX_TRY(launch_gemm(e, s));
    if (p->layernorm)
      FX_TRY(launch_layernorm_fwd(u, F, nullptr, 0, p->ln_w[i], p->ln_b[i], 1e-5f, rows, F, 0, hn, F, nullptr,
                                  saved + L.rs + (long long)i * rows, saved + L.xh + i * L.rowsF, F, s));
  }
  const float* hL = saved + L.h + p->num_layers * L.rowsF;
  return linear_fwd(hL, F, rows, F, p->w_out, p->b_out, y, ldy, p->cout, 0, s);
}

int fx_mstcn_bwd(const fx_mstcn_params* p, const fx_mstcn_grads* g, const float* x, long long ldx, int T, int nvid,
                 const float* dy, long long lddy, float* dx, long long lddx, const float* saved, float* workspace,
                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const Seqs q{T, nvid, p->seq_off};
  FX_TRY(check_seqs(q));
  const int rows = q.rows();
  const int F = p->F;
  const int NL = p->num_layers;
  const MstcnLayout L = mstcn_layout(p, rows);
  float* ws = workspace;
  FX_REQUIRE(p->dropout >= 0.f && p->dropout < 1.f, "mstcn: dropout must be in [0, 1)");
  const bool drop = p->dropout > 0.f;
  // deferred batched weight gradients (below); with training dropout the chain also keeps every layer's
  // masked dB_i for the 1x1 weight gradient.  (The input block's stack is the LAST work of the backward
  // pass, so its batched dW runs after the chain with nothing left to overlap, a ~0.7 ms side-stream tail;
  // giving it the per-layer schedule, or launching the upper layers' dW mid-chain, measured even: the
  // overlapped GEMMs slow the chain by as much, rounds 3 and 5)
  const bool defer = !p->layernorm && NL > 0 && mstcn_defer_ok(p, g);
  // Fused chain (no LayerNorm, <= 16 ragged videos, FX_MSTCN_FUSED=1; dropout on the deferred schedule): see below
  const bool fchain = p->fused_layers && !p->layernorm && (!drop || defer) && NL > 0 &&
                      frl_supported(F, ws + L.buf0, F, F) && (!q.off || q.nvid <= 16) &&
                      (p->fused_layers == 2 || frl_fills_device(rows));
  // the dX-packed conv weights and the transposed 1x1 weights come from the forward (saved); the fused
  // chain reads both in fragment order, which the fused forward packed too (else packed here)
  const float* wk1 = saved + L.wk1b;
  const float* wk2 = saved + L.wk2b;
  if (fchain && !mstcn_fwd_fused(p, q.nvid, q.off != nullptr, rows, saved)) {
    std::vector<FragJob> J;
    frag_layer_jobs(J, NL, F, saved + L.wbs, 3LL * F * F, nullptr, saved + L.wpts, (long long)F * F, ws + L.wk1,
                    ws + L.wk2);
    FX_TRY(launch_frag_jobs(J, s));
    wk1 = ws + L.wk1;
    wk2 = ws + L.wk2;
  }
  const float* wbp = saved + L.wbs;
  float* spl = ws + L.split;     // split-K partials of the weight-gradient GEMMs (side stream)
  float* spm = ws + L.split2;    // ... of the main stream's GEMMs / LN backward
  // dZ_i = (g . W_pw,i) * (z_i > 0) with W_pw,i^T packed row-major by the forward: the B operand
  // loads as k-contiguous rows (b128 fragment reads) instead of the column-major weight
  auto pw_dx = [&](const float* g, int i, float* dZ, const float* zi) -> int {
    fx_gemm_desc d = gemm_desc(rows, F, F, op_rows(g, F), op_rows(saved + L.wpts + (long long)i * F * F, F), dZ, F);
    d.gate = zi;
    d.ld_gate = F;
    d.split_k = pick_split(rows, F, F);
    d.workspace = spm;
    return launch_gemm(d, s);
  };
  WsBound wb(spl, L.colsum - L.split);
  // Weight-gradient GEMMs (dW_out, per layer dW_pw and the dilated-conv dW, dW_in) depend on the
  // input-gradient chain but nothing in the chain depends on them: they run on a side stream,
  // overlapping the chain's GEMMs (each alone leaves the matrix pipes ~45 % idle in its prologue,
  // barriers and epilogue).  Without LayerNorm the chain's buffers rotate (dH over 3, dZ over 2)
  // so the side stream reads a layer's gU / dZ while the main stream computes the next layer;
  // a main-stream write waits for the side stream's layer that last read that buffer.
  SideStream* ss = (p->layernorm || (drop && !defer)) ? nullptr : side_stream();
  hipStream_t sd = ss ? ss->s : s;
  // deferred: the pad rows of the dZ / dH (/ dB) slots are zero, so the batched dW GEMMs run over K = rows_pad
  if (defer && L.rows_pad > rows)
    FX_CHECK_HIP(hipMemset2DAsync(ws + L.dzall + (long long)rows * F, L.rowsF * sizeof(float), 0,
                                  (L.rows_pad - rows) * F * sizeof(float), (drop ? 3 : 2) * NL, s));
  auto fork = [&](int e) -> int {   // side stream waits for the main stream's work so far
    if (!ss) return FX_OK;
    FX_CHECK_HIP(hipEventRecord(ss->to_side[e], s));
    FX_CHECK_HIP(hipStreamWaitEvent(sd, ss->to_side[e], 0));
    return FX_OK;
  };
  auto side_done = [&](int i) -> int {
    if (!ss) return FX_OK;
    FX_CHECK_HIP(hipEventRecord(ss->layer_done[i & 3], sd));
    return FX_OK;
  };
  auto wait_side = [&](int i) -> int {   // main waits until the side stream finished layer i
    if (!ss || i >= NL) return FX_OK;
    FX_CHECK_HIP(hipStreamWaitEvent(s, ss->layer_done[i & 3], 0));
    return FX_OK;
  };
  float* Hb[3] = {ws + L.buf0, ws + L.buf1, ws + L.buf3};
  float* Zb[3] = {ws + L.buf2, ws + L.buf4, ws + L.buf5};
  float* dU = ws + L.buf1;   // LN path (single stream): gradient at the residual sum (pre-LN)
  // weight/bias gradients ACCUMULATE (+=) into g->* (caller zeroes them once per step);
  // every bias gradient rides in its weight-gradient GEMM (virtual ones column).
  const float* hL = saved + L.h + NL * L.rowsF;
  FX_TRY(fork(0));
  FX_TRY(linear_dwdb(dy, lddy, hL, F, rows, F, p->cout, g->w_out, g->b_out, 1, spl, sd));
  float* dH = defer ? ws + L.dhall + (NL - 1) * L.rowsF : Hb[0];   // (deferred: dH_NL kept for the 1x1 dW)
  FX_TRY(linear_dx(dy, lddy, p->w_out, rows, F, p->cout, dH, F, 0, nullptr, 0, spm, s));
  // Fused chain: dH_i = gU_i + conv^T(dZ_i) and the next layer's dZ_i-1 = (dH_i . W_pw,i-1) *
  // (z_i-1 > 0) in ONE kernel per layer (mstcn_fused.hip).  dH_i lives in Hb[(NL - i) % 3], dZ_i in
  // Zb[(NL - 1 - i) % 3]; a kernel overwriting a buffer first waits for the side stream's layer
  // that last read it (layer i + 2 for both).
  auto conv_dw = [&](int i, const float* dZi) -> int {
    return per_video(q, [&](int r0, int nr, const Seqs& qv) -> int {
      fx_operand b = conv_operand(saved + L.h + i * L.rowsF + (long long)r0 * F, F, F, layer_dilation(p, i), 1, qv,
                                  true);
      b.ones_col = 3 * F + 1;
      fx_gemm_desc d = gemm_desc(F, 3 * F + 1, nr, op_cols(dZi + (long long)r0 * F, F), b, g->w_dil[i], 3 * F);
      d.c_tap_cin = F;
      d.c_last_col = g->b_dil[i];
      d.beta = 1.f;
      d.split_k = pick_split(F, 3 * F + 1, nr);
      d.workspace = spl;
      return launch_gemm(d, sd);
    });
  };
  for (int i = NL - 1; fchain && !defer && i >= NL - 1; --i) {   // top layer: dZ by the 1x1 backward GEMM
    const float* zi = saved + L.z + i * L.rowsF;
    FX_TRY(fork(1));
    FX_TRY(linear_dwdb(dH, F, zi, F, rows, F, F, g->w_pw[i], g->b_pw[i], 1, spl, sd));
    FX_TRY(linear_dx(dH, F, p->w_pw[i], rows, F, F, Zb[0], F, 0, zi, F, spm, s));
    FX_TRY(fork(2));
    FX_TRY(conv_dw(i, Zb[0]));
    FX_TRY(side_done(i));
  }
  for (int i = NL - 1; fchain && !defer && i >= 0; --i) {
    float* gU = Hb[(NL - 1 - i) % 3];           // dH_{i+1}
    float* dZi = Zb[(NL - 1 - i) % 3];
    float* dHi = Hb[(NL - i) % 3];
    FX_TRY(wait_side(i + 2));
    if (i == 0) {   // the bottom layer: conv backward only
      fx_gemm_desc d = gemm_desc(rows, F, 3 * F, conv_operand(dZi, F, F, layer_dilation(p, 0), -1, q, false),
                                 op_rows(wbp, 3 * F), dHi, F);
      d.resid = gU;
      d.ld_resid = F;
      prof_begin(0, s);
      FX_TRY(launch_gemm(d, s));
      prof_end(0, s, 2.0 * rows * F * 3.0 * F, 4.0 * (3.0 * rows * F + 3.0 * F * F));
    } else {
      float* dZn = Zb[(NL - i) % 3];
      const float* zn = saved + L.z + (i - 1) * L.rowsF;
      prof_begin(7, s);
      FX_TRY(launch_frl(dZi, F, rows, T, layer_dilation(p, i), -1, q.off, q.nvid,
                        wk1 + (long long)i * 3 * F * F, nullptr, 0, gU, F, dHi, F,
                        wk2 + (long long)(i - 1) * F * F, nullptr, nullptr, 0, zn, F, dZn, F, 0.f, 0, s));
      prof_end(7, s, 2.0 * rows * F * 4.0 * F, 4.0 * (4.0 * rows * F + 4.0 * F * F));
      FX_TRY(fork(1));
      FX_TRY(linear_dwdb(dHi, F, zn, F, rows, F, F, g->w_pw[i - 1], g->b_pw[i - 1], 1, spl, sd));
      FX_TRY(conv_dw(i - 1, dZn));
      FX_TRY(side_done(i - 1));
    }
    dH = dHi;
  }
  // Deferred weight gradients (default when the gradient buffers are uniformly strided, as views of
  // one flat buffer are): the chain keeps every layer's dZ_i and dH_i+1, and the weight gradients of
  // ALL layers follow it as two batched GEMMs on the side stream -- the dilated-conv dW of every layer
  // in one launch (per-layer dilation via b_dil_growth; NL x 24 tiles of 128x64 over the full K = rows,
  // no split-K slabs) and the 1x1 dW + db in another -- plus one batched column sum for the conv
  // biases.  Per layer the interleaved version paid two split-K GEMMs and their reduce launches,
  // competing with the chain for the CUs.
  if (defer) {
    float* dZall = ws + L.dzall;
    float* dHall = ws + L.dhall;   // dHall[i] = dH_{i+1} (gradient at layer i's output)
    // the 1x1 branch's gradient: dB_i = dropout_i(dH_i+1) with the forward's mask (basic.py:160), else dH_i+1
    float* dBall = drop ? ws + L.dball : dHall;
    const int Kp = (int)L.rows_pad;
    // the batched weight gradients of layers [base, base + nb) on the side stream
    auto batched_dw = [&](int base, int nb) -> int {
      if (nb <= 0) return FX_OK;
      FX_TRY(fork(1));
      {   // 1x1: dW_pw,i += dH_{i+1}^T z_i, db_pw,i += colsum(dH_{i+1})   (batched over layers)
        fx_operand b = op_cols(saved + L.z + (long long)base * L.rowsF, F);
        b.batch_stride = L.rowsF;
        b.ones_col = F + 1;
        fx_operand a = op_cols(dBall + (long long)base * L.rowsF, F);
        a.batch_stride = L.rowsF;
        fx_gemm_desc d = gemm_desc(F, F + 1, Kp, a, b, g->w_pw[base], F);
        d.batch = nb;
        d.c_batch_stride = NL > 1 ? g->w_pw[1] - g->w_pw[0] : 0;
        d.c_last_col = g->b_pw[base];
        d.c_last_batch_stride = NL > 1 ? g->b_pw[1] - g->b_pw[0] : 0;
        d.beta = 1.f;
        d.split_k = std::max(pick_split(F, F + 1, rows, nb), defer_split_impl(rows));
        d.workspace = ws + L.bsl;
        WsBound wbb(ws + L.bsl, L.total_ws - L.bsl);
        FX_TRY(launch_gemm(d, sd));
      }
      {   // dilated conv: dW_i += dZ_i^T taps(h_i) stored straight into (F, F, 3)   (batched over layers;
          // ragged videos in the same launch: the B loader finds each frame's video, gemm_f32.hip COLS_CONVR)
        WsBound wbb(ws + L.bsl, L.total_ws - L.bsl);
        fx_operand b = conv_operand(saved + L.h + (long long)base * L.rowsF, F, F, layer_dilation(p, base), 1, q, true);
        b.batch_stride = L.rowsF;
        fx_operand a = op_cols(dZall + (long long)base * L.rowsF, F);
        a.batch_stride = L.rowsF;
        fx_gemm_desc d = gemm_desc(F, 3 * F, Kp, a, b, g->w_dil[base], 3 * F);
        d.batch = nb;
        d.c_batch_stride = NL > 1 ? g->w_dil[1] - g->w_dil[0] : 0;
        d.b_dil_growth = p->dil_factor > 0 ? p->dil_factor : 2;
        d.c_tap_cin = F;
        d.beta = 1.f;
        d.split_k = defer_split_impl(rows);
        d.workspace = ws + L.bsl;
        FX_TRY(launch_gemm(d, sd));
        FX_TRY(launch_colsum_batched(dZall + (long long)base * L.rowsF, F, L.rowsF, rows, F, nb, g->b_dil[base],
                                     NL > 1 ? g->b_dil[1] - g->b_dil[0] : 0, 1, ws + L.csb, sd));
      }
      return FX_OK;
    };
    if (fchain) {
      // the fused chain into the per-layer slots: dZ_NL-1 by the 1x1 backward GEMM, then per layer ONE
      // kernel for dH_i (-> dHall[i-1]) and dZ_i-1 (-> dZall[i-1]); the bottom layer's conv backward
      // alone; the weight gradients of every layer follow as the batched side-stream GEMMs below
      if (drop)
        FX_TRY(launch_dropout(dHall + (NL - 1) * L.rowsF, F, rows, F, F, 0, p->dropout,
                              fx_drop_subseed(p->seed, NL - 1), dBall + (NL - 1) * L.rowsF, F, s));
      FX_TRY(pw_dx(dBall + (NL - 1) * L.rowsF, NL - 1, dZall + (NL - 1) * L.rowsF, saved + L.z + (NL - 1) * L.rowsF));
      if (NL > 1) prof_begin(7, s);   // (the chain of NL - 1 back-to-back launches timed as one)
      for (int i = NL - 1; i >= 1; --i) {
        FX_TRY(launch_frl(dZall + i * L.rowsF, F, rows, T, layer_dilation(p, i), -1, q.off, q.nvid,
                          wk1 + (long long)i * 3 * F * F, nullptr, 0, dHall + i * L.rowsF, F,
                          dHall + (i - 1) * L.rowsF, F, wk2 + (long long)(i - 1) * F * F, nullptr, nullptr, 0,
                          saved + L.z + (i - 1) * L.rowsF, F, dZall + (i - 1) * L.rowsF, F, 0.f, 0, s,
                          drop ? p->dropout : 0.f, fx_drop_subseed(p->seed, i - 1),
                          drop ? dBall + (i - 1) * L.rowsF : nullptr, F));
        // (dZ_j, dH_j+1 of every layer j >= i - 1 exist now)
      }
      if (NL > 1)
        prof_end(7, s, (NL - 1) * 2.0 * rows * F * 4.0 * F, (NL - 1) * 4.0 * (4.0 * rows * F + 4.0 * F * F), NL - 1);
    }
    for (int i = fchain ? 0 : NL - 1; i >= 0; --i) {
      const float* zi = saved + L.z + i * L.rowsF;
      const float* gU = dHall + i * L.rowsF;
      float* dZ = dZall + i * L.rowsF;
      if (!fchain) {   // (fused chain: dZ_0 came with dH_1)
        if (drop)
          FX_TRY(launch_dropout(gU, F, rows, F, F, 0, p->dropout, fx_drop_subseed(p->seed, i), dBall + i * L.rowsF,
                                F, s));
        FX_TRY(pw_dx(dBall + i * L.rowsF, i, dZ, zi));
      }
      // the bottom layer's dH is the stack's input gradient: straight into dx when there is no input map
      const bool to_dx = i == 0 && !p->in_map && dx;
      float* dHn = i > 0 ? dHall + (i - 1) * L.rowsF : (to_dx ? dx : Hb[0]);
      fx_gemm_desc d = gemm_desc(rows, F, 3 * F, conv_operand(dZ, F, F, layer_dilation(p, i), -1, q, false),
                                 op_rows(wbp + (long long)i * 3 * F * F, 3 * F), dHn, to_dx ? lddx : F);
      d.resid = gU;
      d.ld_resid = F;
      prof_begin(0, s);
      FX_TRY(launch_gemm(d, s));
      prof_end(0, s, 2.0 * rows * F * 3.0 * F, 4.0 * (3.0 * rows * F + 3.0 * F * F));
    }
    dH = (!p->in_map && dx) ? nullptr : Hb[0];   // (nullptr: already in dx)
    FX_TRY(batched_dw(0, NL));   // every layer's weight gradients, after the chain
  }
  for (int i = NL - 1; !fchain && !defer && i >= 0; --i) {
    const int step = NL - 1 - i;
    const float* zi = saved + L.z + i * L.rowsF;
    const float* gU = dH;
    if (p->layernorm) {
      FX_TRY(launch_layernorm_bwd(dH, F, nullptr, 0, saved + L.xh + i * L.rowsF, F, p->ln_w[i],
                                  saved + L.rs + (long long)i * rows, rows, F, 0, dU, F, g->ln_w[i], g->ln_b[i],
                                  spm, s));
      gU = dU;
    }
    // the 1x1 branch saw dropout: its gradient is gU masked the same way (the residual keeps gU)
    const float* gB = gU;
    if (drop) {
      float* gm = ws + L.buf4;   // (single-stream path: dZ stays in buf2, buf4 is free)
      FX_TRY(launch_dropout(gU, F, rows, F, F, 0, p->dropout, fx_drop_subseed(p->seed, i), gm, F, s));
      gB = gm;
    }
    // pointwise: dW_pw = dB^T z, db_pw = colsum(dB) (side), dZ = (dB . W_pw) * (z > 0) (main)
    FX_TRY(fork(1));
    FX_TRY(linear_dwdb(gB, F, zi, F, rows, F, F, g->w_pw[i], g->b_pw[i], 1, spl, sd));
    float* dZ = ss ? Zb[step & 1] : Zb[0];
    FX_TRY(wait_side(i + 2));   // dZ buffer last read by layer i + 2's conv dW
    FX_TRY(pw_dx(gB, i, dZ, zi));
    // conv: dW (tap-major columns stored straight into (F,F,3)) + db (ones column) (side),
    // dH_i = dU + conv^T(dZ) (main)
    FX_TRY(fork(2));
    FX_TRY(conv_dw(i, dZ));
    FX_TRY(side_done(i));
    {
      float* dHn;
      if (p->layernorm) {
        dHn = (gU == dH) ? dU : dH;   // (LN: single stream) write into the buffer not holding gU
      } else {
        dHn = Hb[(step + 1) % 3];
        FX_TRY(wait_side(i + 2));     // that buffer was gU of layer i + 2
      }
      fx_gemm_desc d = gemm_desc(rows, F, 3 * F, conv_operand(dZ, F, F, layer_dilation(p, i), -1, q, false),
                                 op_rows(wbp + (long long)i * 3 * F * F, 3 * F), dHn, F);
      d.resid = gU;
      d.ld_resid = F;
      prof_begin(0, s);
      FX_TRY(launch_gemm(d, s));
      prof_end(0, s, 2.0 * rows * F * 3.0 * F, 4.0 * (3.0 * rows * F + 3.0 * F * F));
      if (p->layernorm) {
        if (dHn != dH) std::swap(dH, dU);   // dH now holds dH_i
      } else {
        dH = dHn;
      }
    }
  }
  if (p->in_map) {
    if (g->w_in) {
      FX_TRY(fork(0));
      FX_TRY(linear_dwdb(dH, F, x, ldx, rows, p->cin, F, g->w_in, g->b_in, 1, spl, sd));
    }
    if (dx) FX_TRY(linear_dx(dH, F, p->w_in, rows, p->cin, F, dx, lddx, 0, nullptr, 0, spm, s));
  } else if (dx && dH) {
    FX_CHECK_HIP(hipMemcpy2DAsync(dx, lddx * sizeof(float), dH, F * sizeof(float), F * sizeof(float), rows,
                                  hipMemcpyDeviceToDevice, s));
  }
  if (ss && !p->side_defer) {   // join: everything the side stream did is ordered before later work
    FX_CHECK_HIP(hipEventRecord(ss->join, sd));
    FX_CHECK_HIP(hipStreamWaitEvent(s, ss->join, 0));
  }
  return FX_OK;
}

// ---------------------------------------------------------------- MS-TCN++ (MSTCN2)
}  // extern "C"

namespace fx {
namespace {

struct Mstcn2Layout {
  long long rowsF;
  long long f, cat, r, wb1, wb2, total_saved;            // saved: f_0..f_L, cat_i (2F), r_i, dX-packed weights
  long long wf1, wf2, hb0, hb1, du, dcat, spm, spl, bsl, total_ws;
};

Mstcn2Layout mstcn2_layout(const fx_mstcn2_params* p, int rows) {
  Mstcn2Layout L{};
  const long long F = p->F;
  const int NL = p->num_layers;
  L.rowsF = (long long)rows * F;
  L.f = 0;
  L.cat = L.f + (NL + 1) * L.rowsF;
  L.r = L.cat + 2 * NL * L.rowsF;
  const long long wsz = 3 * F * F;
  L.wb1 = L.r + NL * L.rowsF;
  L.wb2 = L.wb1 + NL * wsz;
  L.total_saved = L.wb2 + NL * wsz;
  L.wf1 = 0;
  L.wf2 = L.wf1 + NL * wsz;
  L.hb0 = L.wf2 + NL * wsz;                 // input-gradient chain: dF ping-pong
  L.hb1 = L.hb0 + L.rowsF;
  L.du = L.hb1 + L.rowsF;                   // every layer's dU_i (fusion pre-activation gradient)
  L.dcat = L.du + NL * L.rowsF;             // every layer's dCat_i = [dA_i | dB_i]
  L.spm = L.dcat + 2 * NL * L.rowsF;        // split-K partials: main-stream GEMMs
  long long sp = 0;
  sp = std::max(sp, split_ws(rows, F, p->cout));
  sp = std::max(sp, split_ws(rows, 2 * F, F));
  sp = std::max(sp, split_ws(rows, F, 3 * F));
  if (p->in_map) sp = std::max(sp, split_ws(rows, p->cin, F));
  L.spl = L.spm + sp;                       // ... side stream (out / in map dW)
  long long sl = std::max(dwdb_ws(rows, F, p->cout), p->in_map ? dwdb_ws(rows, p->cin, F) : 0LL);
  L.bsl = L.spl + sl;                       // ... the (batched) layer dW GEMMs
  long long sb = 0;
  for (int nb : {1, std::max(NL, 1)}) {
    sb = std::max(sb, split_ws(F, 2 * F + 1, rows, nb));
    sb = std::max(sb, split_ws(F, 3 * F + 1, rows, nb));
  }
  L.total_ws = L.bsl + sb;
  return L;
}

int mstcn2_dil(const fx_mstcn2_params* p, int e) {   // dil_factor^e
  const int f = p->dil_factor > 0 ? p->dil_factor : 2;
  long long d = 1;
  for (int k = 0; k < e; ++k) d *= f;
  return (int)d;
}

int pack_conv_set(const float* const* w, int NL, int F, float* wf, float* wb, hipStream_t s) {
  PackArgs a{};
  a.F = F;
  const long long wsz = 3LL * F * F;
  for (int l = 0; l < NL; ++l) {
    a.w[l] = w[l];
    a.wf[l] = wf + l * wsz;
    a.wb[l] = wb + l * wsz;
  }
  fx_launch(pack_conv_kernel, dim3(cdiv(F, 32), cdiv(F, 32), NL), dim3(256), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

template <typename V>
bool uniform_stride(V v, int n) {
  for (int i = 0; i < n; ++i)
    if (!v[i]) return false;
  for (int i = 2; i < n; ++i)
    if (v[i] - v[i - 1] != v[1] - v[0]) return false;
  return true;
}

}  // namespace
}  // namespace fx

extern "C" {

long long fx_mstcn2_saved_floats(const fx_mstcn2_params* p, int rows) { return mstcn2_layout(p, rows).total_saved; }
long long fx_mstcn2_workspace_floats(const fx_mstcn2_params* p, int rows) { return mstcn2_layout(p, rows).total_ws; }

int fx_mstcn2_fwd(const fx_mstcn2_params* p, const float* x, long long ldx, int T, int nvid, float* y, long long ldy,
                  float* saved, float* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  FX_REQUIRE(p && p->num_layers >= 0 && p->num_layers <= 32, "mstcn2: 0..32 layers");
  FX_REQUIRE(p->in_map || p->cin == p->F, "mstcn2: in_map=0 needs cin == F");
  FX_REQUIRE(p->dropout >= 0.f && p->dropout < 1.f, "mstcn2: dropout must be in [0, 1)");
  FX_REQUIRE(saved && workspace && y, "mstcn2: bad arguments");
  const Seqs q{T, nvid, p->seq_off};
  FX_TRY(check_seqs(q));
  const int rows = q.rows(), F = p->F, NL = p->num_layers;
  const Mstcn2Layout L = mstcn2_layout(p, rows);
  float* ws = workspace;
  if (NL > 0) {   // forward images into the workspace, dX images into `saved` for the backward
    FX_TRY(pack_conv_set(p->w_d1, NL, F, ws + L.wf1, saved + L.wb1, s));
    FX_TRY(pack_conv_set(p->w_d2, NL, F, ws + L.wf2, saved + L.wb2, s));
  }
  float* f0 = saved + L.f;
  if (p->in_map) {
    FX_TRY(linear_fwd(x, ldx, rows, p->cin, p->w_in, p->b_in, f0, F, F, 0, s));
  } else {
    FX_CHECK_HIP(hipMemcpy2DAsync(f0, F * sizeof(float), x, ldx * sizeof(float), F * sizeof(float), rows,
                                  hipMemcpyDeviceToDevice, s));
  }
  for (int i = 0; i < NL; ++i) {
    const float* fi = saved + L.f + i * L.rowsF;
    float* fn = saved + L.f + (i + 1) * L.rowsF;
    float* cat = saved + L.cat + 2 * i * L.rowsF;
    float* ri = saved + L.r + i * L.rowsF;
    // cat = [conv_d1(f) | conv_d2(f)]: the two dilated convs store into the halves of one buffer
    // (no torch.cat)   (basic.py:276)
    // (one batch-2 launch: batch h takes conv h's dilation, packed weights, bias and output half --
    // at Breakfast's 2048 rows the pair fills the chip with 128x64 tiles where one conv could not)
    {
      fx_gemm_desc d = gemm_desc(rows, F, 3 * F, conv_operand(fi, F, F, mstcn2_dil(p, NL - 1 - i), 1, q, false),
                                 op_rows(ws + L.wf1 + (long long)i * 3 * F * F, 3 * F), cat, 2 * F);
      d.batch = 2;
      d.a_dil_b1 = mstcn2_dil(p, i);
      d.b.batch_stride = L.wf2 - L.wf1;
      d.c_batch_stride = F;
      d.bias = p->b_d1[i];
      d.bias_batch_stride = p->b_d2[i] - p->b_d1[i];
      prof_begin(0, s);
      FX_TRY(launch_gemm(d, s));
      prof_end(0, s, 2.0 * 2.0 * rows * F * 3.0 * F, 4.0 * (3.0 * rows * F + 6.0 * F * F));
    }
    // r = dropout(relu(W_fu . cat + b_fu)) (no dropout on the last layer), f' = f + r  (basic.py:276-280)
    fx_gemm_desc e = gemm_desc(rows, F, 2 * F, op_rows(cat, 2 * F), op_rows(p->w_fu[i], 2 * F), ri, F);
    e.bias = p->b_fu[i];
    e.relu = 2;
    if (i != NL - 1) {
      e.drop_p = p->dropout;
      e.drop_seed = fx_drop_subseed(p->seed, i);
    }
    FX_TRY(launch_gemm(e, s));
    FX_TRY(add2(fi, F, ri, F, rows, F, fn, F, 0, s));
  }
  return linear_fwd(saved + L.f + NL * L.rowsF, F, rows, F, p->w_out, p->b_out, y, ldy, p->cout, 0, s);
}

int fx_mstcn2_bwd(const fx_mstcn2_params* p, const fx_mstcn2_grads* g, const float* x, long long ldx, int T, int nvid,
                  const float* dy, long long lddy, float* dx, long long lddx, const float* saved, float* workspace,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  FX_REQUIRE(p && g && saved && workspace && dy, "mstcn2 bwd: bad arguments");
  const Seqs q{T, nvid, p->seq_off};
  FX_TRY(check_seqs(q));
  const int rows = q.rows(), F = p->F, NL = p->num_layers;
  const Mstcn2Layout L = mstcn2_layout(p, rows);
  float* ws = workspace;
  SideStream* ss = side_stream();
  hipStream_t sd = ss ? ss->s : s;
  auto fork = [&](int e) -> int {
    if (!ss) return FX_OK;
    FX_CHECK_HIP(hipEventRecord(ss->to_side[e], s));
    FX_CHECK_HIP(hipStreamWaitEvent(sd, ss->to_side[e], 0));
    return FX_OK;
  };
  float* spm = ws + L.spm;
  float* spl = ws + L.spl;
  const float* fL = saved + L.f + NL * L.rowsF;
  FX_TRY(fork(0));
  {
    WsBound wb(spl, L.bsl - L.spl);
    FX_TRY(linear_dwdb(dy, lddy, fL, F, rows, F, p->cout, g->w_out, g->b_out, 1, spl, sd));
  }
  WsBound wbm(spm, L.spl - L.spm);
  float* Hb[2] = {ws + L.hb0, ws + L.hb1};
  float* gF = Hb[0];
  FX_TRY(linear_dx(dy, lddy, p->w_out, rows, F, p->cout, gF, F, 0, nullptr, 0, spm, s));
  for (int i = NL - 1; i >= 0; --i) {
    const float* ri = saved + L.r + i * L.rowsF;
    float* dU = ws + L.du + i * L.rowsF;
    float* dCat = ws + L.dcat + 2 * i * L.rowsF;
    // dU = dropout_i(gF) * (r_i > 0)   (r_i is stored after the dropout: zero where dropped)
    if (i != NL - 1 && p->dropout > 0.f) {
      FX_TRY(launch_dropout(gF, F, rows, F, F, 0, p->dropout, fx_drop_subseed(p->seed, i), dU, F, s));
      FX_TRY(relu_bwd(dU, F, ri, F, rows, F, dU, F, s));
    } else {
      FX_TRY(relu_bwd(gF, F, ri, F, rows, F, dU, F, s));
    }
    // dCat = dU . W_fu   (rows x 2F)
    FX_TRY(launch_gemm(gemm_desc(rows, 2 * F, F, op_rows(dU, F), op_cols(p->w_fu[i], 2 * F), dCat, 2 * F), s));
    // dF_i = gF + conv_d1^T(dA) + conv_d2^T(dB)
    float* dFn = Hb[(NL - i) & 1];
    for (int h = 0; h < 2; ++h) {
      const int dil = h == 0 ? mstcn2_dil(p, NL - 1 - i) : mstcn2_dil(p, i);
      fx_gemm_desc d = gemm_desc(rows, F, 3 * F, conv_operand(dCat + h * F, 2 * F, F, dil, -1, q, false),
                                 op_rows(saved + (h == 0 ? L.wb1 : L.wb2) + (long long)i * 3 * F * F, 3 * F), dFn, F);
      if (h == 0) {
        d.resid = gF;
        d.ld_resid = F;
      } else {
        d.beta = 1.f;
      }
      prof_begin(0, s);
      FX_TRY(launch_gemm(d, s));
      prof_end(0, s, 2.0 * rows * F * 3.0 * F, 4.0 * (3.0 * rows * F + 3.0 * F * F));
    }
    gF = dFn;
  }
  // weight gradients of every layer, after the chain (side stream): batched over the layers when the
  // gradient buffers are uniformly strided (views of one flat buffer), else one launch per layer
  FX_TRY(fork(1));
  if (NL > 0) {
    WsBound wbb(ws + L.bsl, L.total_ws - L.bsl);
    const bool uni = uniform_stride(g->w_fu, NL) && uniform_stride(g->b_fu, NL) && uniform_stride(g->w_d1, NL) &&
                     uniform_stride(g->b_d1, NL) && uniform_stride(g->w_d2, NL) && uniform_stride(g->b_d2, NL);
    const int growth = p->dil_factor > 0 ? p->dil_factor : 2;
    auto st = [&](float* const* v) -> long long { return NL > 1 ? v[1] - v[0] : 0; };
    const int nb = uni ? NL : 1;
    for (int i0 = 0; i0 < NL; i0 += nb) {
      {   // fusion 1x1: dW_fu,i += dU_i^T cat_i, db_fu,i += colsum(dU_i)
        fx_operand a = op_cols(ws + L.du + i0 * L.rowsF, F);
        a.batch_stride = L.rowsF;
        fx_operand b = op_cols(saved + L.cat + 2 * i0 * L.rowsF, 2 * F);
        b.batch_stride = 2 * L.rowsF;
        b.ones_col = 2 * F + 1;
        fx_gemm_desc d = gemm_desc(F, 2 * F + 1, rows, a, b, g->w_fu[i0], 2 * F);
        d.batch = nb;
        d.c_batch_stride = st(g->w_fu);
        d.c_last_col = g->b_fu[i0];
        d.c_last_batch_stride = st(g->b_fu);
        d.beta = 1.f;
        d.split_k = pick_split(F, 2 * F + 1, rows, nb);
        d.workspace = ws + L.bsl;
        FX_TRY(launch_gemm(d, sd));
      }
      for (int h = 0; h < 2; ++h) {
        // dilated conv h: dW_i += dC_h,i^T taps(f_i), db_i += colsum(dC_h,i); conv_d2's dilation grows with
        // the layer (batch b = layer i0 + b), conv_d1's shrinks: its batch b is layer NL-1-b (negative strides)
        const int il = (h == 0 && uni) ? NL - 1 : i0;
        const long long dir = (h == 0 && uni) ? -1 : 1;
        const int dil = h == 0 ? mstcn2_dil(p, NL - 1 - il) : mstcn2_dil(p, il);
        float* const* gw = h == 0 ? g->w_d1 : g->w_d2;
        float* const* gb = h == 0 ? g->b_d1 : g->b_d2;
        FX_TRY(per_video(q, [&](int r0, int nr, const Seqs& qv) -> int {
          fx_operand a = op_cols(ws + L.dcat + 2 * il * L.rowsF + (long long)r0 * 2 * F + h * F, 2 * F);
          a.batch_stride = dir * 2 * L.rowsF;
          fx_operand b = conv_operand(saved + L.f + il * L.rowsF + (long long)r0 * F, F, F, dil, 1, qv, true);
          b.batch_stride = dir * L.rowsF;
          b.ones_col = 3 * F + 1;
          fx_gemm_desc d = gemm_desc(F, 3 * F + 1, nr, a, b, gw[il], 3 * F);
          d.batch = nb;
          d.c_batch_stride = dir * st(gw);
          d.c_last_col = gb[il];
          d.c_last_batch_stride = dir * st(gb);
          d.b_dil_growth = nb > 1 ? growth : 0;
          d.c_tap_cin = F;
          d.beta = 1.f;
          d.split_k = pick_split(F, 3 * F + 1, nr, nb);
          d.workspace = ws + L.bsl;
          return launch_gemm(d, sd);
        }));
      }
    }
  }
  if (p->in_map) {
    if (g->w_in) {
      FX_TRY(fork(2));
      WsBound wb(spl, L.bsl - L.spl);
      FX_TRY(linear_dwdb(gF, F, x, ldx, rows, p->cin, F, g->w_in, g->b_in, 1, spl, sd));
    }
    if (dx) FX_TRY(linear_dx(gF, F, p->w_in, rows, p->cin, F, dx, lddx, 0, nullptr, 0, spm, s));
  } else if (dx) {
    FX_CHECK_HIP(hipMemcpy2DAsync(dx, lddx * sizeof(float), gF, F * sizeof(float), F * sizeof(float), rows,
                                  hipMemcpyDeviceToDevice, s));
  }
  if (ss && !p->side_defer) {
    FX_CHECK_HIP(hipEventRecord(ss->join, sd));
    FX_CHECK_HIP(hipStreamWaitEvent(s, ss->join, 0));
  }
  return FX_OK;
}

}  // extern "C"

namespace fx {
hipStream_t side_fork(hipStream_t s, int e) {
  SideStream* ss = side_stream();
  if (!ss) return s;
  if (hipEventRecord(ss->to_side[e], s) != hipSuccess || hipStreamWaitEvent(ss->s, ss->to_side[e], 0) != hipSuccess)
    return s;
  return ss->s;
}

int side_join_into(hipStream_t s) {
  SideStream* ss = side_stream();
  if (!ss) return FX_OK;
  FX_CHECK_HIP(hipEventRecord(ss->join, ss->s));
  FX_CHECK_HIP(hipStreamWaitEvent(s, ss->join, 0));
  return FX_OK;
}

hipStream_t aux_fork(hipStream_t s) {
  SideStream* ss = side_stream();
  if (!ss || !knobs().aux_stream) return s;   // FX_AUX_STREAM=0: everything on the caller's stream (A/B)
  if (hipEventRecord(ss->aux_fork, s) != hipSuccess || hipStreamWaitEvent(ss->aux, ss->aux_fork, 0) != hipSuccess)
    return s;
  return ss->aux;
}

int aux_join_into(hipStream_t s, hipStream_t a) {
  SideStream* ss = side_stream();
  if (!ss || a == s) return FX_OK;
  FX_CHECK_HIP(hipEventRecord(ss->aux_done, ss->aux));
  FX_CHECK_HIP(hipStreamWaitEvent(s, ss->aux_done, 0));
  return FX_OK;
}

int defer_split(int rows) { return defer_split_impl(rows); }
}  // namespace fx

extern "C" {

void* fx_side_stream(void) {
  SideStream* ss = side_stream();
  return ss ? (void*)ss->s : nullptr;
}

int fx_side_join(void* stream) {
  SideStream* ss = side_stream();
  FX_REQUIRE(ss, "side stream unavailable");
  FX_CHECK_HIP(hipEventRecord(ss->join, ss->s));
  FX_CHECK_HIP(hipStreamWaitEvent((hipStream_t)stream, ss->join, 0));
  return FX_OK;
}

// ---------------------------------------------------------------- row ops
int fx_layernorm_fwd(const float* x, long long ldx, const float* r, long long ldr, const float* w, const float* b,
                     float eps, int rows, int cols, int relu, float* y, long long ldy, float* xhat, long long ldxh,
                     float* rstd, void* stream) {
  return launch_layernorm_fwd(x, ldx, r, ldr, w, b, eps, rows, cols, relu, y, ldy, nullptr, rstd, xhat, ldxh,
                              (hipStream_t)stream);
}

long long fx_layernorm_bwd_workspace_floats(int rows, int cols) { return layernorm_bwd_ws_floats(rows, cols); }

int fx_layernorm_bwd(const float* dy, long long lddy, const float* y, long long ldy, const float* xhat,
                     long long ldxh, const float* w, const float* rstd, int rows, int cols, int relu, float* dx,
                     long long lddx, float* dw, float* db, float* workspace, void* stream) {
  return launch_layernorm_bwd(dy, lddy, y, ldy, xhat, ldxh, w, rstd, rows, cols, relu, dx, lddx, dw, db, workspace,
                              (hipStream_t)stream);
}

int fx_softmax_rows(const float* logits, long long ldl, int rows, int cols, float scale, float* probs,
                    long long ldp, void* stream) {
  return launch_softmax_rows(logits, ldl, rows, cols, scale, probs, ldp, (hipStream_t)stream);
}

int fx_softmax_rows_bwd(const float* probs, long long ldp, const float* dprobs, long long lddp,
                        const float* dlogit_extra, long long lde, int rows, int cols, float scale, float* dlogit,
                        long long ldd, void* stream) {
  return launch_softmax_rows_bwd(probs, ldp, dprobs, lddp, dlogit_extra, lde, rows, cols, scale, dlogit, ldd,
                                 (hipStream_t)stream);
}

int fx_process_feature_fwd(const float* x, long long ldx, int rows, int cols, int n, float* out, long long ldo,
                           float* clogit, long long ldc, void* stream) {
  return launch_pf_fwd(x, ldx, rows, cols, n, out, ldo, clogit, ldc, (hipStream_t)stream);
}

int fx_process_feature_bwd(const float* out, long long ldo, const float* dout, long long lddo, const float* dclogit,
                           long long lddc, int rows, int cols, int n, float* dx, long long lddx, void* stream) {
  return launch_pf_bwd(out, ldo, dout, lddo, dclogit, lddc, rows, cols, n, dx, lddx, (hipStream_t)stream);
}

int fx_l2norm_fwd(const float* x, long long ldx, int rows, int cols, float* y, long long ldy, float* norm,
                  void* stream) {
  return launch_l2n_fwd(x, ldx, rows, cols, y, ldy, norm, (hipStream_t)stream);
}

int fx_l2norm_bwd(const float* y, long long ldy, const float* norm, const float* dy, long long lddy, int rows,
                  int cols, float* dx, long long lddx, void* stream) {
  return launch_l2n_bwd(y, ldy, norm, dy, lddy, rows, cols, dx, lddx, (hipStream_t)stream);
}

int fx_relu_bwd(const float* dy, long long lddy, const float* y, long long ldy, int rows, int cols, float* dz,
                long long lddz, void* stream) {
  return relu_bwd(dy, lddy, y, ldy, rows, cols, dz, lddz, (hipStream_t)stream);
}

int fx_add(const float* a, long long lda, const float* b, long long ldb, int rows, int cols, float* out,
           long long ldo, int accumulate, void* stream) {
  return add2(a, lda, b, ldb, rows, cols, out, ldo, accumulate, (hipStream_t)stream);
}

// ---------------------------------------------------------------- MHA core
long long fx_mha_core_workspace_floats(int Lq, int Lk, int E, int nhead) {
  const int hd = E / std::max(nhead, 1);
  long long ws = 2LL * nhead * Lq * Lk;   // dropped probabilities, dS
  long long sp = 0;
  sp = std::max(sp, split_ws(Lq, hd, Lk, nhead));
  sp = std::max(sp, split_ws(Lk, hd, Lq, nhead));
  sp = std::max(sp, split_ws(Lq, Lk, hd, nhead));
  return ws + 2 * sp;
}

int fx_mha_core_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                    int Lq, int Lk, int E, int nhead, float drop_p, unsigned long long seed, float* probs, float* o,
                    long long ldo, float* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  FX_REQUIRE(nhead > 0 && E % nhead == 0, "mha: E must be divisible by nhead");
  FX_REQUIRE(drop_p == 0.f || workspace, "mha: dropout needs the workspace");
  const int hd = E / nhead;
  const float scale = 1.0f / std::sqrt((float)hd);
  const long long nLL = (long long)nhead * Lq * Lk;
  float* spl = workspace ? workspace + 2 * nLL : nullptr;
  WsBound wb(spl, workspace ? fx_mha_core_workspace_floats(Lq, Lk, E, nhead) - 2 * nLL : 0);
  // S_h = (Q_h K_h^T) * scale  -> probs buffer, then row softmax in place
  fx_gemm_desc d = gemm_desc(Lq, Lk, hd, op_rows(q, ldq), op_rows(k, ldk), probs, Lk);
  d.batch = nhead;
  d.a.batch_stride = hd;
  d.b.batch_stride = hd;
  d.c_batch_stride = (long long)Lq * Lk;
  d.alpha = scale;
  FX_TRY(launch_gemm(d, s));
  FX_TRY(launch_softmax_rows(probs, Lk, nhead * Lq, Lk, 1.f, probs, Lk, s));
  // attention dropout (nn.MultiheadAttention dropout=attn_dropout): O = dropout(P) V, mask index
  // (h Lq + i) Lk + j
  const float* pv = probs;
  if (drop_p > 0.f) {
    FX_TRY(launch_dropout(probs, Lk, nhead * Lq, Lk, Lk, 0, drop_p, seed, workspace, Lk, s));
    pv = workspace;
  }
  // O_h = P_h V_h
  fx_gemm_desc e = gemm_desc(Lq, hd, Lk, op_rows(pv, Lk), op_cols(v, ldv), o, ldo);
  e.batch = nhead;
  e.a.batch_stride = (long long)Lq * Lk;
  e.b.batch_stride = hd;
  e.c_batch_stride = hd;
  e.split_k = workspace ? pick_split(Lq, hd, Lk, nhead) : 1;
  e.workspace = spl;
  return launch_gemm(e, s);
}

int fx_mha_core_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                    const float* probs, const float* dout, long long lddo, int Lq, int Lk, int E, int nhead,
                    float drop_p, unsigned long long seed, float* dq, long long lddq, float* dk, long long lddk,
                    float* dv, long long lddv, float* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  FX_REQUIRE(nhead > 0 && E % nhead == 0, "mha: E must be divisible by nhead");
  const int hd = E / nhead;
  const float scale = 1.0f / std::sqrt((float)hd);
  const long long nLL = (long long)nhead * Lq * Lk;
  float* pd = workspace;
  float* dS = workspace + nLL;
  float* spl = workspace + 2 * nLL;
  WsBound wb(spl, fx_mha_core_workspace_floats(Lq, Lk, E, nhead) - 2 * nLL);
  // dP_h = dO_h V_h^T   (through the dropout: the same mask and scale)
  fx_gemm_desc d = gemm_desc(Lq, Lk, hd, op_rows(dout, lddo), op_rows(v, ldv), dS, Lk);
  d.batch = nhead;
  d.a.batch_stride = hd;
  d.b.batch_stride = hd;
  d.c_batch_stride = (long long)Lq * Lk;
  FX_TRY(launch_gemm(d, s));
  const float* pv = probs;
  if (drop_p > 0.f) {
    FX_TRY(launch_dropout(dS, Lk, nhead * Lq, Lk, Lk, 0, drop_p, seed, dS, Lk, s));
    FX_TRY(launch_dropout(probs, Lk, nhead * Lq, Lk, Lk, 0, drop_p, seed, pd, Lk, s));
    pv = pd;
  }
  // dS = softmax_bwd(P, dP)
  FX_TRY(launch_softmax_rows_bwd(probs, Lk, dS, Lk, nullptr, 0, nhead * Lq, Lk, 1.f, dS, Lk, s));
  // dQ_h = scale * dS_h K_h
  if (dq) {
    fx_gemm_desc e = gemm_desc(Lq, hd, Lk, op_rows(dS, Lk), op_cols(k, ldk), dq, lddq);
    e.batch = nhead;
    e.a.batch_stride = (long long)Lq * Lk;
    e.b.batch_stride = hd;
    e.c_batch_stride = hd;
    e.alpha = scale;
    e.split_k = pick_split(Lq, hd, Lk, nhead);
    e.workspace = spl;
    FX_TRY(launch_gemm(e, s));
  }
  // dK_h = scale * dS_h^T Q_h
  if (dk) {
    fx_gemm_desc e = gemm_desc(Lk, hd, Lq, op_cols(dS, Lk), op_cols(q, ldq), dk, lddk);
    e.batch = nhead;
    e.a.batch_stride = (long long)Lq * Lk;
    e.b.batch_stride = hd;
    e.c_batch_stride = hd;
    e.alpha = scale;
    e.split_k = pick_split(Lk, hd, Lq, nhead);
    e.workspace = spl;
    FX_TRY(launch_gemm(e, s));
  }
  // dV_h = dropout(P_h)^T dO_h
  if (dv) {
    fx_gemm_desc e = gemm_desc(Lk, hd, Lq, op_cols(pv, Lk), op_cols(dout, lddo), dv, lddv);
    e.batch = nhead;
    e.a.batch_stride = (long long)Lq * Lk;
    e.b.batch_stride = hd;
    e.c_batch_stride = hd;
    e.split_k = pick_split(Lk, hd, Lq, nhead);
    e.workspace = spl;
    FX_TRY(launch_gemm(e, s));
  }
  return FX_OK;
}

// ---------------------------------------------------------------- MHA over T (fused)
long long fx_mha_t_workspace_floats(int nvid, int Lq, int T, int hd, int nhead) {
  return tattn_ws_floats(nvid, Lq, T, hd, nhead);
}

int fx_mha_t_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv, int nvid,
                 int Lq, int T, int hd, int nhead, float scale, float* o, long long ldo, float* lse, float* workspace,
                 void* stream) {
  return launch_tattn_fwd(q, ldq, k, ldk, v, ldv, nvid, Lq, T, hd, nhead, scale, o, ldo, lse, workspace,
                          (hipStream_t)stream);
}

int fx_mha_t_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                 const float* o, long long ldo, const float* dout, long long lddo, const float* lse, int nvid, int Lq,
                 int T, int hd, int nhead, float scale, float* dq, long long lddq, float* dk, long long lddk, float* dv,
                 long long lddv, float* workspace, void* stream) {
  return launch_tattn_bwd(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, nvid, Lq, T, hd, nhead, scale, dq, lddq, dk,
                          lddk, dv, lddv, workspace, (hipStream_t)stream);
}

// ---------------------------------------------------------------- X2Y_map
// Single-head cross attention of basic.py:349-389 (kq_pos=True), nvid videos stacked by rows:
// video v owns X rows [x_off[v], x_off[v+1]) and Y rows [y_off[v], y_off[v+1]) (host prefix arrays,
// NULL for one video); projections run over all rows at once, the attention core per video.
// logit / attn hold each video's (ny_v x nx_v) block, packed in video order.
// saved: xin (Nx*xdim, X+Xpos when Xpos), yin (Ny*ydim), xk, xv (Nx*Hd), yq, feat (Ny*Hd)
}  // extern "C"
namespace {
constexpr int GMAX_GROUP = 4;   // members of one grouped direct-GEMM launch (gemm_f32.hip GMAX)
struct X2YLayout {
  long long xin, yin, xk, xv, yq, feat, total;
};
X2YLayout x2y_layout(int Nx, int xdim, int Ny, int ydim, int Hd) {
  X2YLayout L{};
  L.xin = 0;
  L.yin = L.xin + al64((long long)Nx * xdim);
  L.xk = L.yin + al64((long long)Ny * ydim);
  L.xv = L.xk + al64((long long)Nx * Hd);
  L.yq = L.xv + al64((long long)Nx * Hd);
  L.feat = L.yq + al64((long long)Ny * Hd);
  L.total = L.feat + al64((long long)Ny * Hd);
  return L;
}
struct VidRows {
  int n;
  std::vector<int> x, y;        // prefix offsets (n + 1)
  std::vector<long long> a;     // attention block offsets (n + 1)
};
VidRows vid_rows(int Nx, int Ny, int nvid, const int* x_off, const int* y_off) {
  VidRows v;
  v.n = std::max(nvid, 1);
  if (v.n == 1 || !x_off || !y_off) {
    v.n = 1;
    v.x = {0, Nx};
    v.y = {0, Ny};
  } else {
    v.x.assign(x_off, x_off + v.n + 1);
    v.y.assign(y_off, y_off + v.n + 1);
  }
  v.a.assign(v.n + 1, 0);
  for (int i = 0; i < v.n; ++i)
    v.a[i + 1] = v.a[i] + (long long)(v.y[i + 1] - v.y[i]) * (v.x[i + 1] - v.x[i]);
  return v;
}
long long x2y_split_ws1(int Nx, int xdim, int Ny, int ydim, int Hd, int outdim) {
  long long sp = 0;
  sp = std::max(sp, split_ws(Ny, Nx, Hd));             // logits
  sp = std::max(sp, split_ws(Ny, Hd, Nx));             // feat, dyq
  sp = std::max(sp, split_ws(Nx, Hd, Ny));             // dxv, dxk
  sp = std::max(sp, split_ws(Ny, ydim + Hd, outdim));  // dcat
  sp = std::max(sp, dwdb_ws(Ny, ydim, outdim));        // dW_y pieces (+ bias column)
  sp = std::max(sp, dwdb_ws(Ny, Hd, outdim));
  sp = std::max(sp, dwdb_ws(Nx, xdim, Hd));            // dW_k / dW_v
  sp = std::max(sp, dwdb_ws(Ny, ydim, Hd));            // dW_q
  sp = std::max(sp, split_ws(Nx, xdim, Hd));           // dX
  sp = std::max(sp, split_ws(Ny, ydim, Hd));           // dY
  return sp;
}
long long x2y_split_ws(const VidRows& v, int xdim, int ydim, int Hd, int outdim) {
  long long sp = x2y_split_ws1(v.x[v.n], xdim, v.y[v.n], ydim, Hd, outdim);
  if (Hd % 32 == 0) sp = std::max(sp, x2y_a2f_dw_ws_floats(v.n, Hd));   // (the a2f dW kernel's partials)
  for (int i = 0; i < v.n; ++i)
    sp = std::max(sp, x2y_split_ws1(v.x[i + 1] - v.x[i], xdim, v.y[i + 1] - v.y[i], ydim, Hd, outdim));
  return sp;
}
}  // namespace
extern "C" {

long long fx_x2y_saved_floats(int Nx, int xdim, int Ny, int ydim, int Hd) {
  return x2y_layout(Nx, xdim, Ny, ydim, Hd).total;
}

// [dcat][dL][dxv][dxk][dyq][dXk][dYq][split-K][colsum][catd: dropped cat[Y, feat] (dropout only)]
// split-K slabs of the weight-gradient GEMMs on the side stream (their own region: the main stream's
// GEMMs keep using the x2y split region meanwhile)
static long long x2y_side_ws(int Nx, int xdim, int Ny, int ydim, int Hd, int outdim) {
  auto one = [](int rows, int M, int N) {
    const int sp = std::max(pick_split(M, N, rows), defer_split(rows));
    return sp > 1 ? (long long)sp * M * N : 0LL;
  };
  // without dropout dW_y is two GEMMs ([Y | 1] and feat), each narrower than the concatenation and so
  // possibly split more ways (fewer tiles): a 1724-row ragged batch split the [Y | 1] piece 7 ways
  // where the concatenation takes 3
  long long w = std::max(one(Ny, outdim, ydim + Hd + 1), one(Nx, Hd, xdim + 1));
  w = std::max(w, std::max(one(Ny, outdim, ydim + 1), one(Ny, outdim, Hd + 1)));
  return std::max(w, one(Ny, Hd, ydim + 1));
}

static long long x2y_ws_nocatd(int Nx, int xdim, int Ny, int ydim, int Hd, int outdim, const VidRows& v) {
  // dcat, dL, dxv, dxk, dyq, dXk, dYq (fx_x2y_bwd), each region 64-float aligned
  long long w = al64((long long)Ny * (ydim + Hd)) + al64(v.a[v.n]) + 2 * al64((long long)Nx * Hd) +
                al64((long long)Ny * Hd) + al64((long long)Nx * xdim) + al64((long long)Ny * ydim);
  return w + al64(x2y_split_ws(v, xdim, ydim, Hd, outdim)) +
         al64(colsum_workspace_floats(std::max(Nx, Ny), std::max(Hd, outdim)));
}

long long fx_x2y_workspace_floats(int Nx, int xdim, int Ny, int ydim, int Hd, int outdim, int nvid,
                                  const int* x_off, const int* y_off) {
  const VidRows v = vid_rows(Nx, Ny, nvid, x_off, y_off);
  return x2y_ws_nocatd(Nx, xdim, Ny, ydim, Hd, outdim, v) + al64((long long)Ny * (ydim + Hd)) +
         x2y_side_ws(Nx, xdim, Ny, ydim, Hd, outdim) + x2y_f2a_ws_floats(v.n, v.x.data(), Hd);
}

// catd = dropout(cat[Y, feat]) (basic.py:382), mask index r (ydim + Hd) + c
static int x2y_drop_cat(const float* Y, long long ldy, const float* feat, int Ny, int ydim, int Hd, float p,
                        unsigned long long seed, float* catd, hipStream_t s) {
  const int cw = ydim + Hd;
  FX_TRY(launch_dropout(Y, ldy, Ny, ydim, cw, 0, p, seed, catd, cw, s));
  return launch_dropout(feat, Hd, Ny, Hd, cw, ydim, p, seed, catd + ydim, cw, s);
}

int fx_x2y_fwd(const float* X, long long ldx, int Nx, int xdim, const float* Xpos, long long ldxp, int xpos_cols,
               const float* Y, long long ldy, int Ny, int ydim, const float* Ypos, long long ldyp, int ypos_cols,
               const float* wk, const float* bk, const float* wv, const float* bv, const float* wq, const float* bq,
               const float* wy, const float* by, int Hd, int outdim, int nvid, const int* x_off, const int* y_off,
               float drop_p, unsigned long long seed, float* out, long long ldo, float* logit, float* attn,
               float* saved, float* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const VidRows V = vid_rows(Nx, Ny, nvid, x_off, y_off);
  FX_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "x2y: dropout must be in [0, 1)");
  FX_REQUIRE(V.x[V.n] == Nx && V.y[V.n] == Ny, "x2y: offsets must end at Nx / Ny");
  const X2YLayout L = x2y_layout(Nx, xdim, Ny, ydim, Hd);
  WsBound wb(workspace, x2y_split_ws(V, xdim, ydim, Hd, outdim));
  float* xk = saved + L.xk;
  float* xv = saved + L.xv;
  float* yq = saved + L.yq;
  float* feat = saved + L.feat;
  // keep X+Xpos / Y+Ypos for the weight gradients (basic.py:357-369); the position covers the first
  // *pos_cols channels (one launch either way)
  const float* xin = X;
  long long ldxin = ldx;
  if (Xpos) {
    FX_TRY(add2(X, ldx, Xpos, ldxp, Nx, xdim, saved + L.xin, xdim, 0, s, xpos_cols));
    xin = saved + L.xin;
    ldxin = xdim;
  }
  const float* yin = Y;
  long long ldyin = ldy;
  if (Ypos) {
    FX_TRY(add2(Y, ldy, Ypos, ldyp, Ny, ydim, saved + L.yin, ydim, 0, s, ypos_cols));
    yin = saved + L.yin;
    ldyin = ydim;
  }
  prof_begin(10, s);
  FX_TRY(linear_fwd(xin, ldxin, Nx, xdim, wk, bk, xk, Hd, Hd, 0, s));
  FX_TRY(linear_fwd(X, ldx, Nx, xdim, wv, bv, xv, Hd, Hd, 0, s));
  FX_TRY(linear_fwd(yin, ldyin, Ny, ydim, wq, bq, yq, Hd, Hd, 0, s));
  // algorithmic: the input rows, weights and outputs of the three products once
  prof_end(10, s, 2.0 * Hd * (2.0 * Nx * xdim + (double)Ny * ydim),
           4.0 * (2.0 * Nx * xdim + (double)Ny * ydim + Hd * (2.0 * xdim + ydim) + Hd * (2.0 * Nx + Ny)), 3);
  const float scale = 1.0f / std::sqrt((float)Hd);
  // a short key side (the a2f map: <= 64 action tokens per video): the whole core in one launch
  const bool al16 =
      ((reinterpret_cast<uintptr_t>(yq) | reinterpret_cast<uintptr_t>(xk) | reinterpret_cast<uintptr_t>(xv)) & 15) == 0;
  // algorithmic bytes of the attention core (bench roofline_attention): the query / key / value rows, the
  // logit and probability tiles, the attended features
  const double na = (double)V.a[V.n];
  const double core_bytes = 4.0 * ((double)Ny * Hd + 2.0 * Nx * Hd + 2.0 * na + (double)Ny * Hd);
  // fx_prof kinds 3 / 5 for frame-level calls, 11 / 13 for segment-level ones (bench.py reports them apart)
  const int kseg = std::max(Nx, Ny) >= 1024 ? 0 : 8;
  if (knobs().x2y_fused && x2y_a2f_fusable(V.n, V.x.data(), Hd) && al16) {
    prof_begin(3 + kseg, s);
    FX_TRY(launch_x2y_a2f_fwd(yq, xk, xv, Hd, scale, V.n, V.y.data(), V.x.data(), V.a.data(), logit, attn, feat, s));
    prof_end(3 + kseg, s, 4.0 * na * Hd, core_bytes);
  } else if (knobs().x2y_fused && x2y_f2a_fusable(V.n, V.x.data(), V.y.data(), Hd) && al16) {
    // the f2a map (frames -> tokens): per-chunk partials after every other region of the workspace
    float* f2a_ws = workspace + x2y_ws_nocatd(Nx, xdim, Ny, ydim, Hd, outdim, V) + al64((long long)Ny * (ydim + Hd)) +
                    x2y_side_ws(Nx, xdim, Ny, ydim, Hd, outdim);
    prof_begin(5 + kseg, s);
    FX_TRY(launch_x2y_f2a_fwd(yq, xk, xv, Hd, scale, V.n, V.y.data(), V.x.data(), V.a.data(), logit, attn, feat,
                              f2a_ws, s));
    prof_end(5 + kseg, s, 4.0 * na * Hd, core_bytes);
  } else
  // per video: logits = scale yq . xk^T, attn = softmax(logits), feat = attn . xv  (the GEMMs of up to
  // two videos in one grouped launch each)
  for (int v0 = 0; v0 < V.n; v0 += 2) {
    fx_gemm_desc g1[2], g2[2];
    int n1 = 0, n2 = 0;
    for (int v = v0; v < std::min(V.n, v0 + 2); ++v) {
      const int nx = V.x[v + 1] - V.x[v], ny = V.y[v + 1] - V.y[v];
      if (nx == 0 || ny == 0) continue;
      fx_gemm_desc d = gemm_desc(ny, nx, Hd, op_rows(yq + (long long)V.y[v] * Hd, Hd),
                                 op_rows(xk + (long long)V.x[v] * Hd, Hd), logit + V.a[v], nx);
      d.alpha = scale;
      d.split_k = pick_split(ny, nx, Hd);
      d.workspace = workspace;
      g1[n1++] = d;
      d = gemm_desc(ny, Hd, nx, op_rows(attn + V.a[v], nx), op_cols(xv + (long long)V.x[v] * Hd, Hd),
                    feat + (long long)V.y[v] * Hd, Hd);
      d.split_k = pick_split(ny, Hd, nx);
      d.workspace = workspace;
      g2[n2++] = d;
    }
    FX_TRY(launch_gemm_group(g1, n1, s));
    for (int v = v0; v < std::min(V.n, v0 + 2); ++v) {
      const int nx = V.x[v + 1] - V.x[v], ny = V.y[v + 1] - V.y[v];
      if (nx == 0 || ny == 0) continue;
      FX_TRY(launch_softmax_rows(logit + V.a[v], nx, ny, nx, 1.f, attn + V.a[v], nx, s));
    }
    FX_TRY(launch_gemm_group(g2, n2, s));
  }
  // Y_W(cat[Y, feat]) with the concatenation folded into the A-operand loader; with dropout the
  // dropped concatenation is materialised (training only)
  fx_operand a = op_rows(Y, ldy);
  a.ptr1 = feat;
  a.ld1 = Hd;
  a.k_split = ydim;
  if (drop_p > 0.f) {
    float* catd = workspace + x2y_ws_nocatd(Nx, xdim, Ny, ydim, Hd, outdim, V);
    FX_TRY(x2y_drop_cat(Y, ldy, feat, Ny, ydim, Hd, drop_p, seed, catd, s));
    a = op_rows(catd, ydim + Hd);
  }
  fx_gemm_desc d = gemm_desc(Ny, outdim, ydim + Hd, a, op_rows(wy, ydim + Hd), out, ldo);
  d.bias = by;
  return launch_gemm(d, s);
}

int fx_x2y_bwd(const float* X, long long ldx, int Nx, int xdim, int xpos_cols, const float* Y, long long ldy, int Ny,
               int ydim, int ypos_cols, const float* wk, const float* wv, const float* wq, const float* wy, int Hd,
               int outdim, int nvid, const int* x_off, const int* y_off, float drop_p, unsigned long long seed,
               const float* attn, const float* saved,
               const float* dout, long long lddo, const float* dlogit, const float* dattn, float* dX, float* dXpos,
               float* dY, float* dYpos, float* dwk, float* dbk, float* dwv, float* dbv, float* dwq, float* dbq,
               float* dwy, float* dby, int has_xpos, int has_ypos, float* workspace, int side_defer, int32_t* status,
               void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const VidRows V = vid_rows(Nx, Ny, nvid, x_off, y_off);
  FX_REQUIRE(V.x[V.n] == Nx && V.y[V.n] == Ny, "x2y: offsets must end at Nx / Ny");
  const X2YLayout L = x2y_layout(Nx, xdim, Ny, ydim, Hd);
  const float* xk = saved + L.xk;
  const float* xv = saved + L.xv;
  const float* yq = saved + L.yq;
  const float* feat = saved + L.feat;
  const float* xin = has_xpos ? saved + L.xin : X;
  const long long ldxin = has_xpos ? xdim : ldx;
  const float* yin = has_ypos ? saved + L.yin : Y;
  const long long ldyin = has_ypos ? ydim : ldy;
  const int cw = ydim + Hd;
  float* dcat = workspace;
  float* dL = dcat + al64((long long)Ny * cw);
  float* dxv = dL + al64(V.a[V.n]);
  float* dxk = dxv + al64((long long)Nx * Hd);
  float* dyq = dxk + al64((long long)Nx * Hd);
  float* dXk = dyq + al64((long long)Ny * Hd);
  float* dYq = dXk + al64((long long)Nx * xdim);
  float* spl = dYq + al64((long long)Ny * ydim);
  WsBound wb(spl, x2y_split_ws(V, xdim, ydim, Hd, outdim));
  const float scale = 1.0f / std::sqrt((float)Hd);
  // Y_W: dcat = dout . Wy, dWy = dout^T [Y, feat], dby  (dropout: the dropped concatenation and
  // the same mask on dcat)
  FX_TRY(linear_dx(dout, lddo, wy, Ny, cw, outdim, dcat, cw, 0, nullptr, 0, spl, s));
  const float* catd = nullptr;
  if (drop_p > 0.f) {
    float* cd = workspace + x2y_ws_nocatd(Nx, xdim, Ny, ydim, Hd, outdim, V);
    FX_TRY(x2y_drop_cat(Y, ldy, feat, Ny, ydim, Hd, drop_p, seed, cd, s));
    FX_TRY(launch_dropout(dcat, cw, Ny, cw, cw, 0, drop_p, seed, dcat, cw, s));
    catd = cd;
  }
  // a short key side (the a2f map): dP, the softmax backward and dyq in one launch for every video; the
  // products that reduce over the query rows (dxv = attn^T dfeat, dxk = scale dlogit^T yq) stay
  // split-K GEMMs around it
  // the fused cores do float4 loads of the saved xk / xv / yq rows and of dcat: the same 16-B test as
  // the forward's (X2YLayout offsets Nx*xdim + Ny*ydim (+k*Nx*Hd) need not be multiples of 4 floats)
  const bool al16 = ((reinterpret_cast<uintptr_t>(xk) | reinterpret_cast<uintptr_t>(xv) |
                      reinterpret_cast<uintptr_t>(yq) | reinterpret_cast<uintptr_t>(dcat + ydim)) & 15) == 0;
  const bool fused = knobs().x2y_fused && x2y_a2f_fusable(V.n, V.x.data(), Hd) && (cw & 3) == 0 && al16;
  // algorithmic bytes of the backward core: dfeat, xv, xk, yq, attn (+ dattn / dlogit in), dlogit, dxv,
  // dxk, dyq out
  const double na = (double)V.a[V.n];
  const double core_bytes = 4.0 * (2.0 * Ny * Hd + 4.0 * Nx * Hd + 4.0 * na + (double)Ny * Hd);
  // the fused f2a core (bracketed as fx_prof kind 6 only when it runs: the per-video GEMM fallback below
  // is not the kernel whose algorithmic bytes kind 6 reports)
  const int f2a_mode = knobs().x2y_f2a_bwd;
  const bool f2a_fused = !fused && knobs().x2y_fused &&
                         (f2a_mode == 1 || (f2a_mode == 2 && x2y_f2a_chunks(V.n, V.x.data()) >= 64)) &&
                         x2y_f2a_fusable(V.n, V.x.data(), V.y.data(), Hd) && (cw & 3) == 0 && al16;
  const int kseg = std::max(Nx, Ny) >= 1024 ? 0 : 8;   // (fx_prof: frame-level 4 / 6, segment-level 12 / 14)
  if (fused) prof_begin(4 + kseg, s);
  else if (f2a_fused) prof_begin(6 + kseg, s);
  if (fused) {
    FX_TRY(launch_x2y_a2f_bwd(dcat + ydim, cw, xv, xk, attn, dattn, dlogit, Hd, scale, V.n, V.y.data(), V.x.data(),
                              V.a.data(), dL, dyq, s));
    // dxv = attn^T dfeat and dxk = scale dlogit^T yq: one launch over every video (x2y_a2f_dw_kernel), or
    // (FX_X2Y_A2F_DW=0) grouped split-K GEMMs of up to two videos per launch
    if (knobs().x2y_a2f_dw && x2y_a2f_dw_ok(V.n, V.y.data())) {
      FX_TRY(launch_x2y_a2f_dw(attn, dL, dcat + ydim, cw, yq, Hd, scale, V.n, V.y.data(), V.x.data(), V.a.data(), dxv,
                               dxk, spl, s));
    } else
    for (int v0 = 0; v0 < V.n; v0 += GMAX_GROUP / 2) {
      fx_gemm_desc g2[GMAX_GROUP];
      int n2 = 0;
      for (int v = v0; v < std::min(V.n, v0 + GMAX_GROUP / 2); ++v) {
        const int nx = V.x[v + 1] - V.x[v], ny = V.y[v + 1] - V.y[v];
        if (nx == 0 || ny == 0) continue;
        const long long xr = (long long)V.x[v] * Hd, yr = (long long)V.y[v] * Hd;
        fx_gemm_desc d = gemm_desc(nx, Hd, ny, op_cols(attn + V.a[v], nx),
                                   op_cols(dcat + (long long)V.y[v] * cw + ydim, cw), dxv + xr, Hd);
        d.split_k = pick_split(nx, Hd, ny);
        d.workspace = spl;
        g2[n2++] = d;
        d = gemm_desc(nx, Hd, ny, op_cols(dL + V.a[v], nx), op_cols(yq + yr, Hd), dxk + xr, Hd);
        d.alpha = scale;
        d.split_k = pick_split(nx, Hd, ny);
        d.workspace = spl;
        g2[n2++] = d;
      }
      FX_TRY(launch_gemm_group(g2, n2, s));
    }
  } else if (f2a_fused) {
    // the f2a map: dP / dxv, then dlogit / dxk / dyq partials per 64-key chunk, then the ordered dyq merge
    float* f2a_ws = workspace + x2y_ws_nocatd(Nx, xdim, Ny, ydim, Hd, outdim, V) + al64((long long)Ny * cw) +
                    x2y_side_ws(Nx, xdim, Ny, ydim, Hd, outdim);
    FX_TRY(launch_x2y_f2a_bwd(dcat + ydim, cw, xv, xk, yq, attn, dattn, dlogit, Hd, scale, V.n, V.y.data(), V.x.data(),
                              V.a.data(), dL, dxv, dxk, dyq, f2a_ws, reinterpret_cast<unsigned*>(status), s));
  } else
  // per video: dP = dfeat . xv^T (+ dattn), dxv = attn^T . dfeat  (independent: one grouped launch
  // for up to two videos), softmax backward, then dyq = dlogit . xk, dxk = dlogit^T . yq (grouped)
  for (int v0 = 0; v0 < V.n; v0 += 2) {
    fx_gemm_desc g1[4], g2[4];
    int n1 = 0, n2 = 0;
    for (int v = v0; v < std::min(V.n, v0 + 2); ++v) {
      const int nx = V.x[v + 1] - V.x[v], ny = V.y[v + 1] - V.y[v];
      if (nx == 0 || ny == 0) continue;
      const float* dfeat = dcat + (long long)V.y[v] * cw + ydim;
      const float* at = attn + V.a[v];
      float* dl = dL + V.a[v];
      const long long xr = (long long)V.x[v] * Hd, yr = (long long)V.y[v] * Hd;
      fx_gemm_desc d = gemm_desc(ny, nx, Hd, op_rows(dfeat, cw), op_rows(xv + xr, Hd), dl, nx);
      d.resid = dattn ? dattn + V.a[v] : nullptr;
      d.ld_resid = nx;
      d.split_k = pick_split(ny, nx, Hd);
      d.workspace = spl;
      g1[n1++] = d;
      d = gemm_desc(nx, Hd, ny, op_cols(at, nx), op_cols(dfeat, cw), dxv + xr, Hd);
      d.split_k = pick_split(nx, Hd, ny);
      d.workspace = spl;
      g1[n1++] = d;
      d = gemm_desc(ny, Hd, nx, op_rows(dl, nx), op_cols(xk + xr, Hd), dyq + yr, Hd);
      d.alpha = scale;
      d.split_k = pick_split(ny, Hd, nx);
      d.workspace = spl;
      g2[n2++] = d;
      d = gemm_desc(nx, Hd, ny, op_cols(dl, nx), op_cols(yq + yr, Hd), dxk + xr, Hd);
      d.alpha = scale;
      d.split_k = pick_split(nx, Hd, ny);
      d.workspace = spl;
      g2[n2++] = d;
    }
    FX_TRY(launch_gemm_group(g1, n1, s));
    // dlogit = softmax_bwd(attn, dP) + dlogit_direct   (in place)
    for (int v = v0; v < std::min(V.n, v0 + 2); ++v) {
      const int nx = V.x[v + 1] - V.x[v], ny = V.y[v + 1] - V.y[v];
      if (nx == 0 || ny == 0) continue;
      float* dl = dL + V.a[v];
      FX_TRY(launch_softmax_rows_bwd(attn + V.a[v], nx, dl, nx, dlogit ? dlogit + V.a[v] : nullptr, nx, ny, nx, 1.f,
                                     dl, nx, s));
    }
    FX_TRY(launch_gemm_group(g2, n2, s));
  }
  if (fused) prof_end(4 + kseg, s, 8.0 * na * Hd, core_bytes);
  else if (f2a_fused) prof_end(6 + kseg, s, 8.0 * na * Hd, core_bytes);
  // weight gradients (Y_W; projections X_K, X_V, Y_Q): nothing below needs them -> side stream, each
  // frame-level GEMM split defer_split(rows) ways into its own slab region
  {
    hipStream_t sd = side_fork(s, 1);
    float* sps = workspace + x2y_ws_nocatd(Nx, xdim, Ny, ydim, Hd, outdim, V) + al64((long long)Ny * cw);
    WsBound wbs(sps, x2y_side_ws(Nx, xdim, Ny, ydim, Hd, outdim));
    auto dw = [&](const float* dy, long long lddy, const float* x, long long ldx_, int rows, int K, int N, float* w,
                  float* b, long long ldw) -> int {
      fx_gemm_desc d = desc_linear_dwdb(dy, lddy, x, ldx_, rows, K, N, w, b, 1, sps, ldw);
      if (sd != s) d.split_k = std::max(d.split_k, defer_split(rows));
      return launch_gemm(d, sd);
    };
    if (catd) {
      FX_TRY(dw(dout, lddo, catd, cw, Ny, cw, outdim, dwy, dby, cw));
    } else {
      FX_TRY(dw(dout, lddo, Y, ldy, Ny, ydim, outdim, dwy, dby, cw));
      FX_TRY(dw(dout, lddo, feat, Hd, Ny, Hd, outdim, dwy + ydim, nullptr, cw));
    }
    FX_TRY(dw(dxk, Hd, xin, ldxin, Nx, xdim, Hd, dwk, dbk, -1));
    FX_TRY(dw(dxv, Hd, X, ldx, Nx, xdim, Hd, dwv, dbv, -1));
    FX_TRY(dw(dyq, Hd, yin, ldyin, Ny, ydim, Hd, dwq, dbq, -1));
    if (sd != s && !side_defer) FX_TRY(side_join_into(s));
  }
  if (dX || dXpos) {
    FX_TRY(linear_dx(dxk, Hd, wk, Nx, xdim, Hd, dXk, xdim, 0, nullptr, 0, spl, s));
    if (dXpos) FX_TRY(add2(dXk, xdim, nullptr, 0, Nx, xpos_cols, dXpos, xpos_cols, (has_xpos >> 1) & 1, s));
    if (dX) {
      fx_gemm_desc d = gemm_desc(Nx, xdim, Hd, op_rows(dxv, Hd), op_cols(wv, xdim), dX, xdim);
      d.resid = dXk;
      d.ld_resid = xdim;
      d.split_k = pick_split(Nx, xdim, Hd);
      d.workspace = spl;
      FX_TRY(launch_gemm(d, s));
    }
  }
  if (dY || dYpos) {
    FX_TRY(linear_dx(dyq, Hd, wq, Ny, ydim, Hd, dYq, ydim, 0, nullptr, 0, spl, s));
    if (dYpos) FX_TRY(add2(dYq, ydim, nullptr, 0, Ny, ypos_cols, dYpos, ypos_cols, (has_ypos >> 1) & 1, s));
    if (dY) FX_TRY(add2(dYq, ydim, dcat, cw, Ny, ydim, dY, ydim, 0, s));
  }
  return FX_OK;
}

// ---------------------------------------------------------------- bidirectional GRU
long long fx_gru_saved_floats(int S, int Hh) { return 10LL * S * Hh; }

static long long gru_split_ws(int S, int In, int Hh) {
  long long sp = std::max(dwdb_ws(S, In, 3 * Hh), dwdb_ws(S, Hh, 3 * Hh));
  return std::max(sp, split_ws(S, In, 3 * Hh));
}

// fwd: [sync area][gi (S, 6Hh)];  bwd: [dgi (S, 6Hh)][dgh 2 x (S, 3Hh)][split-K][colsum][sync area]
long long fx_gru_workspace_floats(int S, int nseq, int In, int Hh) {
  const long long H3 = 3LL * Hh;
  long long fwd = gru_sync_floats(Hh, nseq) + S * 2 * H3;
  long long sp = gru_split_ws(S, In, Hh);
  long long bwd = S * 2 * H3 + 2 * S * H3 + sp + colsum_workspace_floats(S, 3 * Hh) + gru_sync_floats(Hh, nseq);
  return std::max(fwd, bwd);
}

static std::vector<int> seq_offsets(int S, int nseq, const int* seq_off) {
  if (nseq <= 1 || !seq_off) return {0, S};
  return std::vector<int>(seq_off, seq_off + nseq + 1);
}

int fx_gru_bidir_fwd(const float* x, long long ldx, int S, int nseq, const int* seq_off, int In, int Hh,
                     const float* w_ih_f, const float* w_hh_f, const float* b_ih_f, const float* b_hh_f,
                     const float* w_ih_r, const float* w_hh_r, const float* b_ih_r, const float* b_hh_r, float* out,
                     long long ldo, int relu_out, float* saved, float* workspace, int32_t* status, int spin_max,
                     void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int H3 = 3 * Hh;
  const std::vector<int> off = seq_offsets(S, nseq, seq_off);
  const int nq = (int)off.size() - 1;
  FX_REQUIRE(off.back() == S && off.front() == 0, "gru: sequence offsets must span [0, S]");
  float* gi = workspace + gru_sync_floats(Hh, nq);
  // input projections of every step, both directions: gi[:, d*3Hh:(d+1)*3Hh] = x W_ih_d^T + b_ih_d
  FX_TRY(linear_fwd(x, ldx, S, In, w_ih_f, b_ih_f, gi, 2 * H3, H3, 0, s));
  FX_TRY(linear_fwd(x, ldx, S, In, w_ih_r, b_ih_r, gi + H3, 2 * H3, H3, 0, s));
  const float* whh[2] = {w_hh_f, w_hh_r};
  const float* bhh[2] = {b_hh_f, b_hh_r};
  return launch_gru_fwd(gi, 2 * H3, nq, off.data(), Hh, whh, bhh, out, ldo, relu_out, saved, workspace,
                        (unsigned*)status, spin_max, s);
}

int fx_gru_bidir_bwd(const float* x, long long ldx, int S, int nseq, const int* seq_off, int In, int Hh,
                     const float* w_ih_f, const float* w_hh_f, const float* w_ih_r, const float* w_hh_r,
                     const float* saved, const float* dout, long long lddo, const float* relu_y, long long ldy,
                     float* dx, long long lddx, float* dw_ih_f,
                     float* dw_hh_f, float* db_ih_f, float* db_hh_f, float* dw_ih_r, float* dw_hh_r, float* db_ih_r,
                     float* db_hh_r, float* workspace, int32_t* status, int spin_max, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int H3 = 3 * Hh;
  const std::vector<int> off = seq_offsets(S, nseq, seq_off);
  const int nq = (int)off.size() - 1;
  FX_REQUIRE(off.back() == S && off.front() == 0, "gru: sequence offsets must span [0, S]");
  float* dgi = workspace;                          // (S, 6Hh)
  float* dgh = dgi + (long long)S * 2 * H3;        // 2 x (S, 3Hh)
  float* spl = dgh + 2LL * S * H3;
  float* csw = spl + gru_split_ws(S, In, Hh);
  WsBound wb(spl, gru_split_ws(S, In, Hh));
  float* sync_ws = csw + colsum_workspace_floats(S, 3 * Hh);
  const float* whh[2] = {w_hh_f, w_hh_r};
  FX_TRY(launch_gru_bwd(dout, lddo, relu_y, ldy, nq, off.data(), Hh, whh, saved, dgi, 2 * H3, dgh, sync_ws,
                        (unsigned*)status, spin_max, s));
  const float* wih[2] = {w_ih_f, w_ih_r};
  float* dwih[2] = {dw_ih_f, dw_ih_r};
  float* dwhh[2] = {dw_hh_f, dw_hh_r};
  float* dbih[2] = {db_ih_f, db_ih_r};
  float* dbhh[2] = {db_hh_f, db_hh_r};
  for (int d = 0; d < 2; ++d) {
    const float* gi_d = dgi + d * H3;
    const float* gh_d = dgh + (long long)d * S * H3;
    const float* hp_d = saved + (long long)d * S * Hh;
    if (dwih[d]) FX_TRY(linear_dwdb(gi_d, 2 * H3, x, ldx, S, In, H3, dwih[d], dbih[d], 1, spl, s));
    else if (dbih[d]) FX_TRY(launch_colsum(gi_d, 2 * H3, S, H3, dbih[d], 1, csw, s));
    if (dwhh[d]) FX_TRY(linear_dwdb(gh_d, H3, hp_d, Hh, S, Hh, H3, dwhh[d], dbhh[d], 1, spl, s));
    else if (dbhh[d]) FX_TRY(launch_colsum(gh_d, H3, S, H3, dbhh[d], 1, csw, s));
    if (dx) FX_TRY(linear_dx(gi_d, 2 * H3, wih[d], S, In, H3, dx, lddx, d, nullptr, 0, spl, s));
  }
  return FX_OK;
}

// ---------------------------------------------------------------- segments
int fx_segments_from_probs(const float* x, long long ldx, int col0, int ncls, int T, int nvid, const int* row_off,
                           int32_t* pred, int32_t* seg_id, int32_t* seg_start, int32_t* seg_end, int32_t* num_seg,
                           void* stream) {
  return launch_segments(x, ldx, col0, ncls, T, nvid, row_off, pred, seg_id, seg_start, seg_end, num_seg,
                         (hipStream_t)stream);
}

int fx_segments_globalize(int nvid, int T, const int* row_off, const int32_t* num_seg_host, const int32_t* seg_id,
                          const int32_t* seg_start, const int32_t* seg_end, int32_t* gseg_id, int32_t* gstart,
                          int32_t* gend, void* stream) {
  FX_REQUIRE(nvid >= 1 && (T > 0 || row_off) && num_seg_host, "segments_globalize: bad arguments");
  return launch_seg_globalize(nvid, T, row_off, num_seg_host, seg_id, seg_start, seg_end, gseg_id, gstart, gend,
                              (hipStream_t)stream);
}

int fx_seg_mean_fwd(const float* x, long long ldx, const int32_t* seg_start, const int32_t* seg_end, int S, int cols,
                    float* y, long long ldy, void* stream) {
  return launch_seg_reduce(x, ldx, seg_start, seg_end, S, cols, 1, y, ldy, 0, (hipStream_t)stream);
}

int fx_seg_mean_bwd(const float* dy, long long lddy, const int32_t* seg_id, const int32_t* seg_start,
                    const int32_t* seg_end, int T, int cols, float* dx, long long lddx, int accumulate, void* stream) {
  return launch_seg_mean_bwd(dy, lddy, seg_id, seg_start, seg_end, T, cols, dx, lddx, accumulate, (hipStream_t)stream);
}

int fx_seg_sum_rows(const float* dx, long long lddx, const int32_t* seg_start, const int32_t* seg_end, int S, int cols,
                    float* dy, long long lddy, int accumulate, void* stream) {
  return launch_seg_reduce(dx, lddx, seg_start, seg_end, S, cols, 0, dy, lddy, accumulate, (hipStream_t)stream);
}

// ---------------------------------------------------------------- profiling
int fx_prof_enable(int kind, int max_events) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  FX_REQUIRE(kind >= 0 && kind < kProfKinds && max_events >= 0, "prof: kind out of range");
  ProfState& p = g_prof[kind];
  prof_reset(p);
  p.ev.resize(2 * (size_t)max_events);
  for (auto& e : p.ev) FX_CHECK_HIP(hipEventCreate(&e));
  // kernel-time pairs for the attention-over-T and X2Y kinds (a few kernels per call); the MFMA-bound kinds
  // (conv GEMM, fused layer chains, projection GEMMs) are timed by their brackets alone: their kernels run
  // back to back inside one C call, and an event pair per kernel would add its own dispatch gap to the chain
  const bool kpairs = (kind >= 1 && kind <= 6) || kind >= 11;
  p.kev.resize(kpairs ? 2 * (size_t)max_events * 4 : 0);
  for (auto& e : p.kev) FX_CHECK_HIP(hipEventCreate(&e));
  p.flops.assign(max_events, 0.0);
  p.bytes.assign(max_events, 0.0);
  p.launches.assign(max_events, 0);
  p.max_events = max_events;
  return FX_OK;
}

int fx_prof_collect(int kind, double* total_ms, double* total_flops, double* total_bytes, int* count) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  FX_REQUIRE(kind >= 0 && kind < kProfKinds && g_prof[kind].max_events > 0, "prof: kind not enabled");
  const ProfState& p = g_prof[kind];
  double ms = 0, fl = 0, by = 0;
  int n = 0;
  for (int i = 0; i < p.used; ++i) {
    FX_CHECK_HIP(hipEventSynchronize(p.ev[2 * i + 1]));
    float t = 0.f;
    FX_CHECK_HIP(hipEventElapsedTime(&t, p.ev[2 * i], p.ev[2 * i + 1]));
    ms += t;
    fl += p.flops[i];
    by += p.bytes[i];
    n += p.launches[i];
  }
  *total_ms = ms;
  *total_flops = fl;
  *total_bytes = by;
  *count = n;
  return FX_OK;
}

int fx_prof_collect_kernels(int kind, double* kernel_ms, int* kernels, int* untimed) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  FX_REQUIRE(kind >= 0 && kind < kProfKinds && g_prof[kind].max_events > 0, "prof: kind not enabled");
  const ProfState& p = g_prof[kind];
  double ms = 0;
  for (int i = 0; i < p.kused; ++i) {
    FX_CHECK_HIP(hipEventSynchronize(p.kev[2 * i + 1]));
    float t = 0.f;
    FX_CHECK_HIP(hipEventElapsedTime(&t, p.kev[2 * i], p.kev[2 * i + 1]));
    ms += t;
  }
  *kernel_ms = ms;
  *kernels = p.kused;
  *untimed = p.kdropped;
  return FX_OK;
}

void fx_prof_disable(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& p : g_prof) prof_reset(p);
  g_prof_open = -1;
}

int fx_debug_set_spin(int which, int polls) {
  FX_REQUIRE(which == 0 || which == 1, "fx_debug_set_spin: which is 0 (token kernel) or 1 (X2Y f2a backward)");
  g_spin_override[which].store(polls > 0 ? polls : -1, std::memory_order_relaxed);
  return FX_OK;
}

}  // extern "C"
