// Shared definitions for the factmx HIP library (gfx950 / MI355X only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
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

// ------------------------------------------------------------------------
// GEMM (internal C++ view of fx_gemm_desc; see include/factmx.h)
// ------------------------------------------------------------------------
int launch_gemm(const fx_gemm_desc& d, hipStream_t s);

// Bound on the split-K slabs of the GEMMs issued while one of these is alive (thread-local, nests):
// launch_gemm refuses a split whose slabs would leave [base, base + floats) -- a too-small
// workspace reservation then fails loudly instead of overrunning the caller's buffer.
struct WsBound {
  WsBound(const float* base, long long floats);
  ~WsBound();
  const float* prev_lo;
  const float* prev_hi;
};
// workspace floats needed by a split-K descriptor
long long gemm_workspace_floats(const fx_gemm_desc& d);

// helpers building common descriptors --------------------------------------
fx_operand op_rows(const float* p, long long ld);        // (r,k) at p[r*ld+k]
fx_operand op_cols(const float* p, long long ld);        // (r,k) at p[k*ld+r]
fx_gemm_desc gemm_desc(int M, int N, int K, fx_operand a, fx_operand b, float* c, long long ldc);

// column sums: out[n] (+)= sum_m X[m*ld + n]   (bias gradients)
int launch_colsum(const float* x, long long ld, int M, int N, float* out, int accumulate,
                  float* ws, hipStream_t s);

// Arrival counters for in-launch "last block merges" reductions (split-K GEMMs, split-T attention):
// one zeroed pool of kArrivalCounters words per (device, stream); the last arriver of every
// counter re-arms it to 0, so launches on one stream can reuse the pool.
constexpr long long kArrivalCounters = 1 << 16;
unsigned* arrival_counters(hipStream_t s);

// event-based timing hooks around launches of one kernel class (bench roofline)
void prof_begin(int kind, hipStream_t s);
void prof_end(int kind, hipStream_t s, double flops, double bytes);

}  // namespace fx
