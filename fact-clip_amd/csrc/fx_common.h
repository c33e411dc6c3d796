// Shared definitions for the factmx HIP library (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/factmx.h"

namespace fx {

// thread-local last error message (fx_last_error)
void set_error(const std::string& msg);

#define FX_CHECK_HIP(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      ::fx::set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                      __FILE__ + ":" + std::to_string(__LINE__));                 \
      return FX_ERR_HIP;                                                          \
    }                                                                             \
  } while (0)

#define FX_REQUIRE(cond, msg)                 \
  do {                                        \
    if (!(cond)) {                            \
      ::fx::set_error(std::string(msg));      \
      return FX_ERR_SHAPE;                    \
    }                                         \
  } while (0)

#define FX_TRY(expr)                 \
  do {                               \
    int _s = (expr);                 \
    if (_s != FX_OK) return _s;      \
  } while (0)

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
// workspace / saved-buffer region sizes rounded up to 64 floats: every region then starts 256-B aligned
// (the GEMM's FAST loaders need 16-B aligned operands; a region after R = 75 token rows of a scalar
// per row would otherwise leave everything behind it misaligned)
inline long long al64(long long n) { return (n + 63) & ~63LL; }

// ------------------------------------------------------------------------
// GEMM (internal C++ view of fx_gemm_desc; see include/factmx.h)
// ------------------------------------------------------------------------
int launch_gemm(const fx_gemm_desc& d, hipStream_t s);
// independent GEMMs (disjoint outputs, at most one split-K workspace user) in one launch when all take
// the direct (small-shape) kernel, else launched one by one in order
int launch_gemm_group(const fx_gemm_desc* d, int n, hipStream_t s);

// Bound on the split-K slabs of the GEMMs issued while one of these is alive (thread-local, nests):
// launch_gemm refuses a split whose slabs would leave [base, base + floats) -- a too-small
// workspace reservation then fails loudly instead of overrunning the caller's buffer.
struct WsBound {
  WsBound(const float* base, long long floats);
  ~WsBound();
  const float* prev_lo;
  const float* prev_hi;
};
// The library's side stream (one per device; FX_SIDE_STREAM=0: none).  side_fork: the side stream
// (after making it wait for everything enqueued on s so far), or s itself when there is none;
// side_join_into: s waits for everything enqueued on the side stream.
hipStream_t side_fork(hipStream_t s, int event);
int side_join_into(hipStream_t s);
// aux_fork: the helper stream (after waiting for everything enqueued on s), or s when there is none;
// aux_join_into(s, a): s waits for what was enqueued on a since (no-op when a == s)
hipStream_t aux_fork(hipStream_t s);
int aux_join_into(hipStream_t s, hipStream_t a);
// split-K factor for weight-gradient GEMMs deferred to the side stream over `rows` rows (keeps each
// workgroup's share of K short, so the main stream's kernels find free CUs)
int defer_split(int rows);
// workspace floats needed by a split-K descriptor
long long gemm_workspace_floats(const fx_gemm_desc& d);

// helpers building common descriptors --------------------------------------
fx_operand op_rows(const float* p, long long ld);        // (r,k) at p[r*ld+k]
fx_operand op_cols(const float* p, long long ld);        // (r,k) at p[k*ld+r]
fx_gemm_desc gemm_desc(int M, int N, int K, fx_operand a, fx_operand b, float* c, long long ldc);

// column sums: out[n] (+)= sum_m X[m*ld + n]   (bias gradients)
int launch_colsum_batched(const float* x, long long ld, long long x_bs, int M, int N, int nb, float* out,
                          long long out_bs, int accumulate, float* ws, hipStream_t s);
int launch_colsum(const float* x, long long ld, int M, int N, float* out, int accumulate,
                  float* ws, hipStream_t s);

// Arrival counters for in-launch "last block merges" reductions (split-K GEMMs, split-T attention):
// one zeroed pool of kArrivalCounters words per (device, stream); the last arriver of every
// counter re-arms it to 0, so launches on one stream can reuse the pool.
constexpr long long kArrivalCounters = 1 << 16;
unsigned* arrival_counters(hipStream_t s);

// ------------------------------------------------------------------------
// Dropout mask (counter-based, regenerated in backward): element idx of a dropout site with seed
// `seed` is kept iff fx_drop_bits(seed, idx) >= fx_drop_thresh(p); kept values are scaled by
// 1 / (1 - p) as nn.Dropout does.  splitmix64 of (seed + (idx + 1) * golden ratio).
__host__ __device__ inline unsigned fx_drop_bits(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (unsigned)(z >> 32);
}
inline unsigned fx_drop_thresh(float p) {
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (unsigned)t;
}
// seed of sub-site i of a site (MS-TCN layer i, ...)
inline unsigned long long fx_drop_subseed(unsigned long long seed, int i) {
  return seed + 0xD1B54A32D192ED03ull * (unsigned long long)(i + 1);
}
// y[r, c] = x[r, c] * keep(seed, r * idx_ld + idx_col0 + c) / (1 - p)   (y may alias x)
int launch_dropout(const float* x, long long ldx, int rows, int cols, long long idx_ld, long long idx_col0, float p,
                   unsigned long long seed, float* y, long long ldy, hipStream_t s);

// A/B switches of the default paths (FX_GEMM_PATH, FX_GEMM_W8, FX_GEMM_WIDE, FX_GEMM_XCDPLANES, FX_GEMM_GROUP,
// FX_SIDE_STREAM, FX_MSTCN_DEFER, the fused-kernel switches below): read from the environment ONCE, at the
// library's first use, into this
// table (std::call_once); no entry point reads the environment itself.  Defaults are the tuned paths.
struct Knobs {
  int gemm_path = 0;        // 1 tiled, 2 direct (0: the planner's choice)
  bool gemm_w8 = true;      // 8-wave 128x64 tiles
  int gemm_wide = -1;       // 0 / 1 force the 128x64 tiles off / on (-1: the planner's choice)
  bool gemm_xcd_planes = true;
  bool gemm_persist = true;  // FX_GEMM_PERSIST=0: one workgroup per wide8 tile (A/B)
  bool gemm_group_m = true;  // FX_GEMM_GROUPM=0: no grouped tile order for large-B GEMMs (A/B)
  bool gemm_row_perm = true;  // FX_GEMM_ROWPERM=0: dilated-conv row tiles in plain order on the XCDs (A/B)
  bool frl_pair = true;        // FX_FRL_PAIR=0: the fused MS-TCN layer synchronises per 32-deep stage (A/B)
  int frl_min_fill = 80;        // FX_FRL_MIN_FILL: fused MS-TCN layer only when its row tiles cover this % of the CUs (shipped yaml, 219 tiles: 80 vs 100 -> 54.5-54.8 vs 55.1-55.2 ms)
  bool aux_stream = true;       // FX_AUX_STREAM=0: the decoder's query-position gradient on the caller's stream
  bool x2y_a2f_dw = true;        // FX_X2Y_A2F_DW=0: the a2f backward's dxv / dxk as grouped split-K GEMMs (A/B)
  bool tattn_fold = true;        // FX_TATTN_FOLD=0: the register-resident kernels' merge as a second launch (A/B)
  bool tattn_rr = true;          // FX_TATTN_RR=0: the LDS-staged attention-over-T kernels for head dim 32 too (A/B)
  bool gru_poll2 = true;        // FX_GRU_POLL2=0: one granule poll in flight per lane (A/B)
  int gru_store_wave = 2;        // FX_GRU_STORE_WAVE: GRU forward table stores -- 0 by wave 0's gate threads, 1 staged for a fifth wave, 2 gate threads on the fifth wave (A/B)
  int frl_xcd = 2;             // FX_FRL_XCD: fused MS-TCN layer row tiles on the XCDs -- 0 round robin,
                              // 1 contiguous runs, 2 runs that follow the conv taps (A/B)
  bool gemm_group = true;
  bool gemm_ktail = true;    // FX_GEMM_KTAIL=0: column-major operands with a K tail take the generic kernel (A/B)
  bool dec_tok = true;       // FX_DEC_TOK=0: the decoders' token rows as separate launches instead of the persistent
                             // token kernel (tokdec.hip) (A/B, and the fallback the tests compare with)
  int tok_spin = 0;          // FX_TOK_SPIN: grid-barrier polls before a token-kernel workgroup gives up (0: ~1 s)
  bool side_stream = true;
  bool mstcn_defer = true;
  bool x2y_fused = true;    // FX_X2Y_FUSED=0: the X2Y attention core as grouped GEMM + softmax launches
  bool x2y_f2a_one = true;  // FX_X2Y_F2A_ONE=0: the fused f2a backward as two launches (dP pass, dlogit pass)
  int x2y_f2a_bwd = 2;      // FX_X2Y_F2A_BWD: the fused f2a backward core (one workgroup per 64-key chunk) 1 always,
                            // 0 never (grouped GEMMs), 2 when the call has >= 64 chunks: at 8192 frames 145 vs
                            // ~180 us for the grouped GEMMs; with a few hundred segments (3-4 chunks) 80 vs ~56 us
};
const Knobs& knobs();

// event-based timing hooks around launches of one kernel class (bench roofline): prof_begin / prof_end
// bracket a call (HIP events on the stream: kernels + any host-issue gap between them), and every kernel
// launched through fx_launch while a bracket is open on this thread also gets its OWN event pair through
// hipExtLaunchKernel, whose timestamps are the kernel's execution (the rocprofv3 kernel-trace duration)
void prof_begin(int kind, hipStream_t s);
void prof_end(int kind, hipStream_t s, double flops, double bytes, int launches = 1);
extern thread_local int g_prof_open;   // kind of the bracket open on this thread, -1: none
bool prof_kernel_events(hipStream_t s, hipEvent_t* e0, hipEvent_t* e1);

// Every kernel launch of the library: hipLaunchKernelGGL, or hipExtLaunchKernelGGL with a kernel-time
// event pair inside an open profiling bracket (bench.py's sampled step only)
template <typename... Args, typename F = void (*)(Args...)>
inline void fx_launch(F kernel, const dim3& grid, const dim3& block, std::uint32_t shm, hipStream_t s, Args... args) {
  hipEvent_t e0, e1;
  if (g_prof_open >= 0 && prof_kernel_events(s, &e0, &e1))
    hipExtLaunchKernelGGL(kernel, grid, block, shm, s, e0, e1, 0u, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, shm, s, args...);
}

// Grid-barrier spin bounds of the persistent kernels (polls before a workgroup gives up and sets its
// status bit): the FX_TOK_SPIN knob, or a value set at run time by fx_debug_set_spin (timeout tests)
unsigned tok_spin_max();
unsigned x2y_spin_max();
// Workgroups of `kernel` (block threads, dynamic LDS bytes) that can be resident on the device at once:
// the occupancy calculator's blocks per CU x the CU count (the bound of a grid-barrier launch's grid)
int coresident_blocks(const void* kernel, int threads, size_t lds);

}  // namespace fx
