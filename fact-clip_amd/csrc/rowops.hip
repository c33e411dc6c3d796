// Row-wise kernels: LayerNorm (+residual, +ReLU), softmax, process_feature,
// L2 normalisation, and their backwards.  One wave64 per row for rows up to
// 1024 channels (values held in registers, 16 per lane max); a 256-thread
// workgroup per row (global re-reads, L2 resident) for longer rows such as
// attention over T frames.  All reductions are wave shuffles + LDS.
#include <algorithm>

#include "fx_common.h"
#include "ops.h"

namespace fx {
namespace {

constexpr int MAXPL = 16;  // values per lane in the wave-per-row path (cols <= 1024)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- LayerNorm
// y2 (nullable) = y + pos: the decoders' "LayerNorm output + query position" operand written beside y
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* x, long long ldx, const float* r,
                                                     long long ldr, const float* w, const float* b,
                                                     float eps, int rows, int cols, int relu, float* y,
                                                     long long ldy, float* mean_out, float* rstd_out,
                                                     float* xhat, long long ldxh, const float* pos, long long ldp,
                                                     float* y2, long long ldy2) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[MAXPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    v[i] = 0.f;
    if (c < cols) {
      v[i] = x[(long long)row * ldx + c] + (r ? r[(long long)row * ldr + c] : 0.f);
      s += v[i];
    }
  }
  const float mu = wave_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    if (c < cols) {
      const float d = v[i] - mu;
      q += d * d;
    }
  }
  const float rs = rsqrtf(wave_sum(q) / cols + eps);
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    if (c < cols) {
      const float h = (v[i] - mu) * rs;
      if (xhat) xhat[(long long)row * ldxh + c] = h;
      float o = h * w[c] + b[c];
      if (relu) o = fmaxf(o, 0.f);
      y[(long long)row * ldy + c] = o;
      if (y2) y2[(long long)row * ldy2 + c] = o + pos[(long long)row * ldp + c];
    }
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mu;
    if (rstd_out) rstd_out[row] = rs;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy_eff * w
// per-block partial dw/db sums over the block's rows -> ws[blk][2*cols]
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* dy, long long lddy, const float* y,
                                                     long long ldy, const float* xhat, long long ldxh,
                                                     const float* w, const float* rstd, int rows,
                                                     int cols, int relu, float* dx, long long lddx,
                                                     float* ws) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pw[MAXPL], pb[MAXPL];
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) pw[i] = pb[i] = 0.f;
  for (int row = blockIdx.x * 4 + wv; row < rows; row += gridDim.x * 4) {
    float g[MAXPL], h[MAXPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXPL; ++i) {
      const int c = i * 64 + lane;
      g[i] = h[i] = 0.f;
      if (c < cols) {
        float d = dy[(long long)row * lddy + c];
        if (relu && !(y[(long long)row * ldy + c] > 0.f)) d = 0.f;
        h[i] = xhat[(long long)row * ldxh + c];
        pw[i] += d * h[i];
        pb[i] += d;
        g[i] = d * w[c];
        s1 += g[i];
        s2 += g[i] * h[i];
      }
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
    const float rs = rstd[row];
#pragma unroll
    for (int i = 0; i < MAXPL; ++i) {
      const int c = i * 64 + lane;
      if (c < cols) dx[(long long)row * lddx + c] = rs * (g[i] - s1 - h[i] * s2);
    }
  }
  if (!ws) return;
  __shared__ float red[4][2][64];
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    if (i * 64 >= cols) break;
    red[wv][0][lane] = pw[i];
    red[wv][1][lane] = pb[i];
    __syncthreads();
    if (wv == 0) {
      const int c = i * 64 + lane;
      if (c < cols) {
        ws[(long long)blockIdx.x * 2 * cols + c] = red[0][0][lane] + red[1][0][lane] + red[2][0][lane] + red[3][0][lane];
        ws[(long long)blockIdx.x * 2 * cols + cols + c] =
            red[0][1][lane] + red[1][1][lane] + red[2][1][lane] + red[3][1][lane];
      }
    }
    __syncthreads();
  }
}

// token-sized LayerNorm backward (rows <= 64, cols <= 256): ONE 1024-thread block; each of the 16
// waves owns rows w, w+16, w+32, w+48 and issues the loads of all of them up front (one memory
// round trip instead of one per row), writes dx, and keeps per-column partial sums of the weight /
// bias gradients that are reduced in LDS and accumulated (+=) in the same launch.
constexpr int SMALL_RPW = 4;   // rows per wave
constexpr int SMALL_CPL = 4;   // columns per lane (cols <= 256)
__global__ __launch_bounds__(1024) void ln_bwd_small_kernel(const float* dy, long long lddy, const float* y,
                                                            long long ldy, const float* xhat, long long ldxh,
                                                            const float* w, const float* rstd, int rows, int cols,
                                                            int relu, float* dx, long long lddx, float* dw,
                                                            float* db) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ float red[16][2][64];
  float d[SMALL_RPW][SMALL_CPL], h[SMALL_RPW][SMALL_CPL], wc[SMALL_CPL];
#pragma unroll
  for (int i = 0; i < SMALL_CPL; ++i) {
    const int c = i * 64 + lane;
    wc[i] = c < cols ? w[c] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < SMALL_RPW; ++q) {
    const int row = wv + 16 * q;
#pragma unroll
    for (int i = 0; i < SMALL_CPL; ++i) {
      const int c = i * 64 + lane;
      const bool ok = row < rows && c < cols;
      float g = ok ? dy[(long long)row * lddy + c] : 0.f;
      if (relu && ok && !(y[(long long)row * ldy + c] > 0.f)) g = 0.f;
      d[q][i] = g;
      h[q][i] = ok ? xhat[(long long)row * ldxh + c] : 0.f;
    }
  }
  float pw[SMALL_CPL], pb[SMALL_CPL];
#pragma unroll
  for (int i = 0; i < SMALL_CPL; ++i) pw[i] = pb[i] = 0.f;
#pragma unroll
  for (int q = 0; q < SMALL_RPW; ++q) {
    const int row = wv + 16 * q;
    float s1 = 0.f, s2 = 0.f, g[SMALL_CPL];
#pragma unroll
    for (int i = 0; i < SMALL_CPL; ++i) {
      pw[i] += d[q][i] * h[q][i];
      pb[i] += d[q][i];
      g[i] = d[q][i] * wc[i];
      s1 += g[i];
      s2 += g[i] * h[q][i];
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
    if (row < rows) {
      const float rs = rstd[row];
#pragma unroll
      for (int i = 0; i < SMALL_CPL; ++i) {
        const int c = i * 64 + lane;
        if (c < cols) dx[(long long)row * lddx + c] = rs * (g[i] - s1 - h[q][i] * s2);
      }
    }
  }
  if (!dw && !db) return;
#pragma unroll
  for (int i = 0; i < SMALL_CPL; ++i) {
    if (i * 64 >= cols) break;
    red[wv][0][lane] = pw[i];
    red[wv][1][lane] = pb[i];
    __syncthreads();
    const int c = i * 64 + lane;
    if (wv == 0 && c < cols) {
      float a = 0.f, b = 0.f;
      for (int k = 0; k < 16; ++k) {
        a += red[k][0][lane];
        b += red[k][1][lane];
      }
      if (dw) dw[c] += a;
      if (db) db[c] += b;
    }
    __syncthreads();
  }
}

// dw/db partials of the nblk row blocks -> +=: 32 columns x 8 interleaved partial groups per block
// (fixed order: deterministic), so the serial chain per thread is nblk / 8 loads instead of nblk
__global__ __launch_bounds__(256) void ln_bwd_reduce(const float* ws, int nblk, int cols, float* dw, float* db) {
  const int cl = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float a = 0.f, b = 0.f;
  if (c < cols)
    for (int k = q; k < nblk; k += 8) {
      a += ws[(long long)k * 2 * cols + c];
      b += ws[(long long)k * 2 * cols + cols + c];
    }
  __shared__ float ra[8][32], rb[8][32];
  ra[q][cl] = a;
  rb[q][cl] = b;
  __syncthreads();
  if (q == 0 && c < cols) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa += ra[j][cl];
      sb += rb[j][cl];
    }
    if (dw) dw[c] += sa;
    if (db) db[c] += sb;
  }
}

// ---------------------------------------------------------------- softmax
// wave per row (cols <= 1024)
__global__ __launch_bounds__(256) void softmax_wave_kernel(const float* x, long long ldx, int rows, int cols,
                                                           float scale, float* p, long long ldp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float v[MAXPL];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    v[i] = -INFINITY;
    if (c < cols) {
      v[i] = scale * x[(long long)row * ldx + c];
      m = fmaxf(m, v[i]);
    }
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    if (c < cols) {
      v[i] = __expf(v[i] - m);
      s += v[i];
    }
  }
  const float inv = 1.f / wave_sum(s);
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    if (c < cols) p[(long long)row * ldp + c] = v[i] * inv;
  }
}

__device__ __forceinline__ float block_reduce(float v, bool is_max, float* sh) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

// block per row (long rows)
__global__ __launch_bounds__(256) void softmax_block_kernel(const float* x, long long ldx, int rows, int cols,
                                                            float scale, float* p, long long ldp) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const float* xr = x + (long long)row * ldx;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < cols; c += 256) m = fmaxf(m, scale * xr[c]);
  m = block_reduce(m, true, sh);
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += 256) s += __expf(scale * xr[c] - m);
  s = block_reduce(s, false, sh);
  const float inv = 1.f / s;
  float* pr = p + (long long)row * ldp;
  for (int c = threadIdx.x; c < cols; c += 256) pr[c] = __expf(scale * xr[c] - m) * inv;
}

// dlogit = scale * p * (dp - sum(dp * p)) + extra
__global__ __launch_bounds__(256) void softmax_bwd_block_kernel(const float* p, long long ldp, const float* dp,
                                                                long long lddp, const float* extra,
                                                                long long lde, int cols, float scale,
                                                                float* dl, long long ldd) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const float* pr = p + (long long)row * ldp;
  const float* dr = dp + (long long)row * lddp;
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += 256) s += pr[c] * dr[c];
  s = block_reduce(s, false, sh);
  float* out = dl + (long long)row * ldd;
  for (int c = threadIdx.x; c < cols; c += 256) {
    float v = scale * pr[c] * (dr[c] - s);
    if (extra) v += extra[(long long)row * lde + c];
    out[c] = v;
  }
}

__global__ __launch_bounds__(256) void softmax_bwd_wave_kernel(const float* p, long long ldp, const float* dp,
                                                               long long lddp, const float* extra,
                                                               long long lde, int rows, int cols,
                                                               float scale, float* dl, long long ldd) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float pv[MAXPL], dv[MAXPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    pv[i] = dv[i] = 0.f;
    if (c < cols) {
      pv[i] = p[(long long)row * ldp + c];
      dv[i] = dp[(long long)row * lddp + c];
      s += pv[i] * dv[i];
    }
  }
  s = wave_sum(s);
#pragma unroll
  for (int i = 0; i < MAXPL; ++i) {
    const int c = i * 64 + lane;
    if (c < cols) {
      float v = scale * pv[i] * (dv[i] - s);
      if (extra) v += extra[(long long)row * lde + c];
      dl[(long long)row * ldd + c] = v;
    }
  }
}

// ---------------------------------------------------------------- process_feature
__global__ __launch_bounds__(256) void pf_fwd_kernel(const float* x, long long ldx, int rows, int cols, int n,
                                                     float* out, long long ldo, float* clogit, long long ldc) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long long)row * ldx;
  float* orow = out + (long long)row * ldo;
  const int f = cols - n;
  for (int c = lane; c < f; c += 64) orow[c] = xr[c];
  float m = -INFINITY;
  for (int c = lane; c < n; c += 64) m = fmaxf(m, xr[f + c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < n; c += 64) s += __expf(xr[f + c] - m);
  const float inv = 1.f / wave_sum(s);
  for (int c = lane; c < n; c += 64) orow[f + c] = __expf(xr[f + c] - m) * inv;
  if (clogit)
    for (int c = lane; c < n; c += 64) clogit[(long long)row * ldc + c] = xr[f + c];
}

__global__ __launch_bounds__(256) void pf_bwd_kernel(const float* out, long long ldo, const float* dout,
                                                     long long lddo, const float* dcl, long long lddc,
                                                     int rows, int cols, int n, float* dx, long long lddx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int f = cols - n;
  const float* orow = out + (long long)row * ldo;
  const float* drow = dout + (long long)row * lddo;
  float* xrow = dx + (long long)row * lddx;
  for (int c = lane; c < f; c += 64) xrow[c] = drow[c];
  float s = 0.f;
  for (int c = lane; c < n; c += 64) s += orow[f + c] * drow[f + c];
  s = wave_sum(s);
  for (int c = lane; c < n; c += 64) {
    float v = orow[f + c] * (drow[f + c] - s);
    if (dcl) v += dcl[(long long)row * lddc + c];
    xrow[f + c] = v;
  }
}

// ---------------------------------------------------------------- L2 normalise
__global__ __launch_bounds__(256) void l2n_fwd_kernel(const float* x, long long ldx, int rows, int cols, float* y,
                                                      long long ldy, float* nrm) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float v = x[(long long)row * ldx + c];
    s += v * v;
  }
  const float n = fmaxf(sqrtf(wave_sum(s)), 1e-12f);
  const float inv = 1.f / n;
  for (int c = lane; c < cols; c += 64) y[(long long)row * ldy + c] = x[(long long)row * ldx + c] * inv;
  if (lane == 0) nrm[row] = n;
}

// y = x / max(|x|, eps):  dx = (dy - y * <dy, y>) / n   (n > eps; else dx = dy / eps)
__global__ __launch_bounds__(256) void l2n_bwd_kernel(const float* y, long long ldy, const float* nrm,
                                                      const float* dy, long long lddy, int rows, int cols,
                                                      float* dx, long long lddx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float n = nrm[row];
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) s += y[(long long)row * ldy + c] * dy[(long long)row * lddy + c];
  s = wave_sum(s);
  const bool clamped = !(n > 1e-12f);
  const float inv = 1.f / n;
  for (int c = lane; c < cols; c += 64) {
    const float g = dy[(long long)row * lddy + c];
    dx[(long long)row * lddx + c] = clamped ? g * inv : (g - y[(long long)row * ldy + c] * s) * inv;
  }
}

}  // namespace

int launch_layernorm_fwd_pos(const float* x, long long ldx, const float* r, long long ldr, const float* w,
                             const float* b, float eps, int rows, int cols, int relu, float* y, long long ldy,
                             float* mean, float* rstd, float* xhat, long long ldxh, const float* pos, long long ldp,
                             float* y2, long long ldy2, hipStream_t s) {
  FX_REQUIRE(cols > 0 && cols <= 64 * MAXPL, "layernorm: cols must be in (0, 1024]");
  FX_REQUIRE(!y2 || pos, "layernorm: y + pos needs pos");
  if (rows == 0) return FX_OK;
  fx_launch(ln_fwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, r, ldr, w, b, eps, rows, cols,
                     relu, y, ldy, mean, rstd, xhat, ldxh, pos, ldp, y2, ldy2);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_layernorm_fwd(const float* x, long long ldx, const float* r, long long ldr, const float* w,
                         const float* b, float eps, int rows, int cols, int relu, float* y, long long ldy,
                         float* mean, float* rstd, float* xhat, long long ldxh, hipStream_t s) {
  return launch_layernorm_fwd_pos(x, ldx, r, ldr, w, b, eps, rows, cols, relu, y, ldy, mean, rstd, xhat, ldxh,
                                  nullptr, 0, nullptr, 0, s);
}

constexpr int LN_GRAD_MAXJOB = 48;
struct LnGradBatch {
  LnGradJob job[LN_GRAD_MAXJOB];
  int n, rows, cols;
  long long lddy, ldxh;
};

// one thread per (job, column): the rows summed in order, loads unrolled 8 deep
__global__ __launch_bounds__(256) void ln_param_grad_kernel(LnGradBatch b) {
  const int j = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (j >= b.n || c >= b.cols) return;
  const LnGradJob& J = b.job[j];
  float sw = 0.f, sb = 0.f;
  int r = 0;
  for (; r + 8 <= b.rows; r += 8) {
    float d[8], h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      d[i] = J.dy[(long long)(r + i) * b.lddy + c];
      h[i] = J.xhat[(long long)(r + i) * b.ldxh + c];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sw += d[i] * h[i];
      sb += d[i];
    }
  }
  for (; r < b.rows; ++r) {
    const float d = J.dy[(long long)r * b.lddy + c];
    sw += d * J.xhat[(long long)r * b.ldxh + c];
    sb += d;
  }
  if (J.dw) J.dw[c] += sw;
  if (J.db) J.db[c] += sb;
}

// frame-level rows: up to 1024 blocks of 4 waves (a wave's rows run one after another, each a load
// round trip + two wave reductions: 256 blocks left 8 rows per wave at 8192 rows, 58 us)
constexpr int LN_BWD_MAXBLK = 1024;

int launch_ln_param_grads(const LnGradJob* jobs, int n, int rows, int cols, long long lddy, long long ldxh,
                          hipStream_t s) {
  for (int j0 = 0; j0 < n; j0 += LN_GRAD_MAXJOB) {
    LnGradBatch b{};
    b.n = std::min(LN_GRAD_MAXJOB, n - j0);
    for (int j = 0; j < b.n; ++j) b.job[j] = jobs[j0 + j];
    b.rows = rows;
    b.cols = cols;
    b.lddy = lddy;
    b.ldxh = ldxh;
    fx_launch(ln_param_grad_kernel, dim3(cdiv(cols, 256), b.n), dim3(256), 0, s, b);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

long long layernorm_bwd_ws_floats(int rows, int cols) {
  const int nblk = std::min(cdiv(rows, 4), LN_BWD_MAXBLK);
  return (long long)nblk * 2 * cols;
}

int launch_layernorm_bwd(const float* dy, long long lddy, const float* y, long long ldy, const float* xhat,
                         long long ldxh, const float* w, const float* rstd, int rows, int cols, int relu,
                         float* dx, long long lddx, float* dw, float* db, float* ws, hipStream_t s) {
  FX_REQUIRE(cols > 0 && cols <= 64 * MAXPL, "layernorm: cols must be in (0, 1024]");
  if (rows == 0) return FX_OK;
  if (rows <= 16 * SMALL_RPW && cols <= 64 * SMALL_CPL) {
    fx_launch(ln_bwd_small_kernel, dim3(1), dim3(1024), 0, s, dy, lddy, y, ldy, xhat, ldxh, w, rstd, rows,
                       cols, relu, dx, lddx, dw, db);
    FX_CHECK_HIP(hipGetLastError());
    return FX_OK;
  }
  const int nblk = std::min(cdiv(rows, 4), LN_BWD_MAXBLK);
  const bool want = dw || db;
  FX_REQUIRE(!want || ws, "layernorm bwd: workspace required for dw/db");
  fx_launch(ln_bwd_kernel, dim3(nblk), dim3(256), 0, s, dy, lddy, y, ldy, xhat, ldxh, w, rstd, rows,
                     cols, relu, dx, lddx, want ? ws : nullptr);
  if (want) fx_launch(ln_bwd_reduce, dim3(cdiv(cols, 32)), dim3(256), 0, s, ws, nblk, cols, dw, db);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

__global__ __launch_bounds__(256) void dropout_kernel(const float* x, long long ldx, int rows, int cols,
                                                     long long idx_ld, long long idx_col0, unsigned thr, float scale,
                                                     unsigned long long seed, float* y, long long ldy) {
  const long long total = (long long)rows * cols;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int r = (int)(e / cols), c = (int)(e - (long long)r * cols);
    const float v = x[(long long)r * ldx + c];
    const bool keep = fx_drop_bits(seed, (unsigned long long)((long long)r * idx_ld + idx_col0 + c)) >= thr;
    y[(long long)r * ldy + c] = keep ? v * scale : 0.f;
  }
}

int launch_dropout(const float* x, long long ldx, int rows, int cols, long long idx_ld, long long idx_col0, float p,
                   unsigned long long seed, float* y, long long ldy, hipStream_t s) {
  FX_REQUIRE(p >= 0.f && p < 1.f, "dropout: p must be in [0, 1)");
  if ((long long)rows * cols == 0) return FX_OK;
  const int blocks = (int)std::min<long long>(cdiv((long long)rows * cols, 256), 4096);
  fx_launch(dropout_kernel, dim3(blocks), dim3(256), 0, s, x, ldx, rows, cols, idx_ld, idx_col0,
                     p > 0.f ? std::max(fx_drop_thresh(p), 1u) : 0u, 1.f / (1.f - p), seed, y, ldy);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_softmax_rows(const float* x, long long ldx, int rows, int cols, float scale, float* p, long long ldp,
                        hipStream_t s) {
  if (rows == 0 || cols == 0) return FX_OK;
  if (cols <= 64 * MAXPL)
    fx_launch(softmax_wave_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, rows, cols, scale, p, ldp);
  else
    fx_launch(softmax_block_kernel, dim3(rows), dim3(256), 0, s, x, ldx, rows, cols, scale, p, ldp);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_softmax_rows_bwd(const float* p, long long ldp, const float* dp, long long lddp, const float* extra,
                            long long lde, int rows, int cols, float scale, float* dl, long long ldd,
                            hipStream_t s) {
  if (rows == 0 || cols == 0) return FX_OK;
  if (cols <= 64 * MAXPL)
    fx_launch(softmax_bwd_wave_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, p, ldp, dp, lddp, extra, lde,
                       rows, cols, scale, dl, ldd);
  else
    fx_launch(softmax_bwd_block_kernel, dim3(rows), dim3(256), 0, s, p, ldp, dp, lddp, extra, lde, cols,
                       scale, dl, ldd);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_pf_fwd(const float* x, long long ldx, int rows, int cols, int n, float* out, long long ldo,
                  float* clogit, long long ldc, hipStream_t s) {
  FX_REQUIRE(n > 0 && n <= cols, "process_feature: need 0 < n <= cols");
  if (rows == 0) return FX_OK;
  fx_launch(pf_fwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, rows, cols, n, out, ldo, clogit, ldc);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_pf_bwd(const float* out, long long ldo, const float* dout, long long lddo, const float* dcl,
                  long long lddc, int rows, int cols, int n, float* dx, long long lddx, hipStream_t s) {
  FX_REQUIRE(n > 0 && n <= cols, "process_feature: need 0 < n <= cols");
  if (rows == 0) return FX_OK;
  fx_launch(pf_bwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, out, ldo, dout, lddo, dcl, lddc, rows,
                     cols, n, dx, lddx);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_l2n_fwd(const float* x, long long ldx, int rows, int cols, float* y, long long ldy, float* nrm,
                   hipStream_t s) {
  if (rows == 0) return FX_OK;
  fx_launch(l2n_fwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, rows, cols, y, ldy, nrm);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_l2n_bwd(const float* y, long long ldy, const float* nrm, const float* dy, long long lddy, int rows,
                   int cols, float* dx, long long lddx, hipStream_t s) {
  if (rows == 0) return FX_OK;
  fx_launch(l2n_bwd_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, y, ldy, nrm, dy, lddy, rows, cols, dx,
                     lddx);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
