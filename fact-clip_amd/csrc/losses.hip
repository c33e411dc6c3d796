// Fused FACT loss terms (fact_clip/models/loss.py), forward + backward each in one or two launches
// instead of the reference's ~10 ATen ops per term (and as many autograd nodes back).
//
// class_loss  (frame_loss loss.py:246-258, frame_loss_tdu 260-277, smooth_loss 8-18 on the same
//              logits): logits X (R x C), row r's target either a hard label y_r (one-hot) or a soft
//              row Z[r, :] (the segment "zoom" of the one-hots), class weights w:
//                ce = sum_r sum_c -Z[r,c] w[c] log_softmax(X)[r,c] / denom
//                sm = mean_{r < R-1, c} clamp((lp[r+1,c] - lp[r,c])^2, 0, 16)      (optional)
// attn_loss   (cross_attn_loss loss.py:209-222, cross_attn_loss_tdu 224-244, smooth_loss on the
//              attention logits): logits L (R x Q) given by strides (so a transposed view costs
//              nothing), the K matched token columns a_i with target columns Z[:, s_i] and weights
//              sw_i, log_softmax over the K selected columns of a row (axis 1) or over the rows of
//              a selected column (axis 0):
//                xe = sum_{r,i} -Z[r, s_i] sw_i lp[r, i] / denom
//                sm = smooth_loss over all Q columns (row log_softmax over Q, diff over rows)  (optional)
// Forward: per-row (and per-column) partial sums in a fixed grid, then one block adds them in a fixed
// order (deterministic); the row / column log-sum-exps are kept for the backward, which writes the
// whole logit gradient in one row-parallel pass.
#include <cmath>

#include "fx_common.h"

namespace fx {
namespace {

constexpr int LT = 256;       // threads per block (4 waves, one row per wave at a time)
constexpr int NBLK = 128;     // row blocks of the forward partial sums

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

struct Mat {
  const float* p;
  long long sr, sc;   // element (r, c) at p[r*sr + c*sc]
  __device__ __forceinline__ float at(int r, int c) const { return p[(long long)r * sr + (long long)c * sc]; }
};

// log-sum-exp of row r over columns c < n (one wave)
__device__ __forceinline__ float row_lse(const Mat& x, int r, int n, int lane) {
  float m = -INFINITY;
  for (int c = lane; c < n; c += 64) m = fmaxf(m, x.at(r, c));
  m = wmax(m);
  float s = 0.f;
  for (int c = lane; c < n; c += 64) s += __expf(x.at(r, c) - m);
  return m + __logf(wsum(s));
}

// ------------------------------------------------------------------ class loss
struct ClassArgs {
  Mat x;              // (R, C)
  int R, C;
  const long long* y; // hard labels (nullable)
  const float* z;     // soft targets (R, C) dense (nullable)
  const float* w;     // class weights (C)
  float* lse;         // (R) saved
  float* part;        // (NBLK, 2) partials
  int smooth;
};

__global__ __launch_bounds__(LT) void class_loss_fwd_kernel(ClassArgs a) {
  __shared__ float red[2][LT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float ce = 0.f, sm = 0.f;
  for (int r = blockIdx.x * (LT / 64) + wv; r < a.R; r += gridDim.x * (LT / 64)) {
    const float l0 = row_lse(a.x, r, a.C, lane);
    if (lane == 0) a.lse[r] = l0;
    if (a.y) {
      if (lane == 0) {
        const int c = (int)a.y[r];
        ce += a.w[c] * (l0 - a.x.at(r, c));
      }
    } else {
      float t = 0.f;
      for (int c = lane; c < a.C; c += 64) t += a.z[(long long)r * a.C + c] * a.w[c] * (l0 - a.x.at(r, c));
      ce += t;
    }
    if (a.smooth && r + 1 < a.R) {
      const float l1 = row_lse(a.x, r + 1, a.C, lane);
      float t = 0.f;
      for (int c = lane; c < a.C; c += 64) {
        const float d = (a.x.at(r + 1, c) - l1) - (a.x.at(r, c) - l0);
        t += fminf(d * d, 16.f);
      }
      sm += t;
    }
  }
  ce = wsum(ce);
  sm = wsum(sm);
  if (lane == 0) {
    red[0][wv] = ce;
    red[1][wv] = sm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float c0 = 0.f, s0 = 0.f;
    for (int i = 0; i < LT / 64; ++i) {
      c0 += red[0][i];
      s0 += red[1][i];
    }
    a.part[2 * blockIdx.x] = c0;
    a.part[2 * blockIdx.x + 1] = s0;
  }
}

// out[0] = c0 * sum(part[2i]) + c1 * sum(part[2i+1])   (fixed order; c1 == 0 drops the smooth term)
__global__ __launch_bounds__(64) void finish_kernel(const float* part, int n, float c0, float c1, float* out) {
  const int lane = threadIdx.x;
  float a = 0.f, b = 0.f;
  for (int i = lane; i < n; i += 64) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  a = wsum(a);
  b = wsum(b);
  if (lane == 0) out[0] = c1 != 0.f ? c0 * a + c1 * b : c0 * a;
}

struct ClassBwdArgs {
  Mat x;
  int R, C;
  const long long* y;
  const float* z;
  const float* w;
  const float* lse;
  const float* gout;  // upstream gradient of the scalar (device)
  float c_ce, c_sm;   // coefficient / denom, coefficient / count
  float* dx;          // (R, C) dense
  int smooth;
};

__global__ __launch_bounds__(LT) void class_loss_bwd_kernel(ClassBwdArgs a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float g_ce = a.gout[0] * a.c_ce, g_sm = a.gout[0] * a.c_sm;
  for (int r = blockIdx.x * (LT / 64) + wv; r < a.R; r += gridDim.x * (LT / 64)) {
    const float l0 = a.lse[r];
    const float lm = (a.smooth && r > 0) ? a.lse[r - 1] : 0.f;
    const float lp1 = (a.smooth && r + 1 < a.R) ? a.lse[r + 1] : 0.f;
    // soft-target row weight sum (hard: w[y_r])
    float zw = 0.f;
    if (a.y) {
      zw = a.w[(int)a.y[r]];
    } else {
      for (int c = lane; c < a.C; c += 64) zw += a.z[(long long)r * a.C + c] * a.w[c];
      zw = wsum(zw);
    }
    const int yr = a.y ? (int)a.y[r] : -1;
    // g_lp[c] of the smooth term (through the clamp), then through log_softmax
    float gsum = 0.f;
    for (int c = lane; c < a.C; c += 64) {
      float g = 0.f;
      if (a.smooth) {
        const float lpc = a.x.at(r, c) - l0;
        if (r > 0) {
          const float d = lpc - (a.x.at(r - 1, c) - lm);
          if (d * d <= 16.f) g += 2.f * d;
        }
        if (r + 1 < a.R) {
          const float d = (a.x.at(r + 1, c) - lp1) - lpc;
          if (d * d <= 16.f) g -= 2.f * d;
        }
        g *= g_sm;
      }
      gsum += g;
    }
    gsum = wsum(gsum);
    for (int c = lane; c < a.C; c += 64) {
      const float p = __expf(a.x.at(r, c) - l0);
      float g = 0.f;
      if (a.smooth) {
        const float lpc = a.x.at(r, c) - l0;
        if (r > 0) {
          const float d = lpc - (a.x.at(r - 1, c) - lm);
          if (d * d <= 16.f) g += 2.f * d;
        }
        if (r + 1 < a.R) {
          const float d = (a.x.at(r + 1, c) - lp1) - lpc;
          if (d * d <= 16.f) g -= 2.f * d;
        }
        g *= g_sm;
      }
      const float tz = a.y ? (c == yr ? a.w[c] : 0.f) : a.z[(long long)r * a.C + c] * a.w[c];
      a.dx[(long long)r * a.C + c] = (g - p * gsum) + g_ce * (zw * p - tz);
    }
  }
}

// ------------------------------------------------------------------ attention loss
constexpr int MAXK = 64;   // matched columns
struct AttnArgs {
  Mat L;              // (R, Q)
  int R, Q, K, axis, smooth;
  const float* z;     // (R, S) dense targets
  int S;
  int a[MAXK], s[MAXK];
  float sw[MAXK];
  float* lse_sel;     // axis 1: (R) lse over the selected columns; axis 0: (K) lse over rows
  float* lse_full;    // (R) lse over all Q (smooth)
  float* colz;        // axis 0: (K) sum_r Z[r, s_i] sw_i
  float* part;        // (NBLK, 2)
};

__global__ __launch_bounds__(LT) void attn_loss_fwd_kernel(AttnArgs a) {
  __shared__ float red[2][LT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float xe = 0.f, sm = 0.f;
  const int gw = blockIdx.x * (LT / 64) + wv, nw = gridDim.x * (LT / 64);
  if (a.axis == 1) {
    for (int r = gw; r < a.R; r += nw) {
      // lse over the K selected columns (lane i < K holds column a_i)
      const float v = lane < a.K ? a.L.at(r, a.a[lane]) : -INFINITY;
      const float m = wmax(v);
      const float l = m + __logf(wsum(lane < a.K ? __expf(v - m) : 0.f));
      if (lane == 0) a.lse_sel[r] = l;
      xe += lane < a.K ? -(v - l) * a.z[(long long)r * a.S + a.s[lane]] * a.sw[lane] : 0.f;
    }
  } else {
    // one wave per selected column: lse over the rows
    for (int i = gw; i < a.K; i += nw) {
      const int q = a.a[i];
      float m = -INFINITY;
      for (int r = lane; r < a.R; r += 64) m = fmaxf(m, a.L.at(r, q));
      m = wmax(m);
      float s = 0.f, zs = 0.f, zl = 0.f;
      for (int r = lane; r < a.R; r += 64) {
        const float x = a.L.at(r, q);
        const float zz = a.z[(long long)r * a.S + a.s[i]];
        s += __expf(x - m);
        zs += zz;
        zl += zz * x;
      }
      const float l = m + __logf(wsum(s));
      zs = wsum(zs);
      zl = wsum(zl);
      if (lane == 0) {
        a.lse_sel[i] = l;
        a.colz[i] = zs * a.sw[i];
        xe += -(zl - zs * l) * a.sw[i];
      }
    }
  }
  if (a.smooth) {
    for (int r = gw; r < a.R; r += nw) {
      const float l0 = row_lse(a.L, r, a.Q, lane);
      if (lane == 0) a.lse_full[r] = l0;
      if (r + 1 < a.R) {
        const float l1 = row_lse(a.L, r + 1, a.Q, lane);
        float t = 0.f;
        for (int c = lane; c < a.Q; c += 64) {
          const float d = (a.L.at(r + 1, c) - l1) - (a.L.at(r, c) - l0);
          t += fminf(d * d, 16.f);
        }
        sm += t;
      }
    }
  }
  xe = wsum(xe);
  sm = wsum(sm);
  if (lane == 0) {
    red[0][wv] = xe;
    red[1][wv] = sm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float c0 = 0.f, s0 = 0.f;
    for (int i = 0; i < LT / 64; ++i) {
      c0 += red[0][i];
      s0 += red[1][i];
    }
    a.part[2 * blockIdx.x] = c0;
    a.part[2 * blockIdx.x + 1] = s0;
  }
}

struct AttnBwdArgs {
  Mat L;
  int R, Q, K, axis, smooth;
  const float* z;
  int S;
  int a[MAXK], s[MAXK];
  float sw[MAXK];
  const float* lse_sel;
  const float* lse_full;
  const float* colz;
  const float* gout;  // upstream gradient of the scalar (device)
  float c_xe, c_sm;   // coefficient / denom, coefficient / count
  float* dL;          // written with strides (dsr, dsc)
  long long dsr, dsc;
};

__global__ __launch_bounds__(LT) void attn_loss_bwd_kernel(AttnBwdArgs a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float g_xe = a.gout[0] * a.c_xe, g_sm = a.gout[0] * a.c_sm;
  for (int r = blockIdx.x * (LT / 64) + wv; r < a.R; r += gridDim.x * (LT / 64)) {
    const float l0 = a.smooth ? a.lse_full[r] : 0.f;
    const float lm = (a.smooth && r > 0) ? a.lse_full[r - 1] : 0.f;
    const float lp1 = (a.smooth && r + 1 < a.R) ? a.lse_full[r + 1] : 0.f;
    float gsum = 0.f;
    if (a.smooth)
      for (int c = lane; c < a.Q; c += 64) {
        float g = 0.f;
        const float lpc = a.L.at(r, c) - l0;
        if (r > 0) {
          const float d = lpc - (a.L.at(r - 1, c) - lm);
          if (d * d <= 16.f) g += 2.f * d;
        }
        if (r + 1 < a.R) {
          const float d = (a.L.at(r + 1, c) - lp1) - lpc;
          if (d * d <= 16.f) g -= 2.f * d;
        }
        gsum += g * g_sm;
      }
    gsum = wsum(gsum);
    // axis 1: row weight sum of the selected targets
    float zrow = 0.f;
    if (a.axis == 1) zrow = wsum(lane < a.K ? a.z[(long long)r * a.S + a.s[lane]] * a.sw[lane] : 0.f);
    for (int c = lane; c < a.Q; c += 64) {
      float g = 0.f;
      if (a.smooth) {
        const float lpc = a.L.at(r, c) - l0;
        if (r > 0) {
          const float d = lpc - (a.L.at(r - 1, c) - lm);
          if (d * d <= 16.f) g += 2.f * d;
        }
        if (r + 1 < a.R) {
          const float d = (a.L.at(r + 1, c) - lp1) - lpc;
          if (d * d <= 16.f) g -= 2.f * d;
        }
        g = g * g_sm - __expf(lpc) * gsum;
      }
      for (int i = 0; i < a.K; ++i) {
        if (a.a[i] != c) continue;
        const float x = a.L.at(r, c);
        const float zz = a.z[(long long)r * a.S + a.s[i]] * a.sw[i];
        if (a.axis == 1) g += g_xe * (__expf(x - a.lse_sel[r]) * zrow - zz);
        else g += g_xe * (__expf(x - a.lse_sel[i]) * a.colz[i] - zz);
      }
      a.dL[(long long)r * a.dsr + (long long)c * a.dsc] = g;
    }
  }
}

int grid_rows(int R) { return std::max(1, std::min(NBLK, cdiv(R, LT / 64))); }

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

long long fx_loss_workspace_floats(void) { return 2LL * NBLK; }

int fx_class_loss_fwd(const float* x, long long sr, long long sc, int R, int C, const long long* y, const float* z,
                      const float* w, float c_ce, float c_sm, float* lse, float* out, float* workspace,
                      void* stream) {
  FX_REQUIRE(R > 0 && C > 0 && x && w && lse && out && workspace && (y || z), "class_loss: bad arguments");
  const int smooth = c_sm != 0.f;
  hipStream_t s = (hipStream_t)stream;
  ClassArgs a{};
  a.x = Mat{x, sr, sc};
  a.R = R;
  a.C = C;
  a.y = y;
  a.z = z;
  a.w = w;
  a.lse = lse;
  a.part = workspace;
  a.smooth = smooth;
  const int nb = grid_rows(R);
  fx_launch(class_loss_fwd_kernel, dim3(nb), dim3(LT), 0, s, a);
  fx_launch(finish_kernel, dim3(1), dim3(64), 0, s, workspace, nb, c_ce, c_sm, out);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_class_loss_bwd(const float* x, long long sr, long long sc, int R, int C, const long long* y, const float* z,
                      const float* w, const float* lse, float c_ce, float c_sm, const float* gout, float* dx,
                      void* stream) {
  FX_REQUIRE(R > 0 && C > 0 && x && w && lse && dx && gout && (y || z), "class_loss_bwd: bad arguments");
  const int smooth = c_sm != 0.f;
  ClassBwdArgs a{};
  a.x = Mat{x, sr, sc};
  a.R = R;
  a.C = C;
  a.y = y;
  a.z = z;
  a.w = w;
  a.lse = lse;
  a.gout = gout;
  a.c_ce = c_ce;
  a.c_sm = c_sm;
  a.dx = dx;
  a.smooth = smooth;
  fx_launch(class_loss_bwd_kernel, dim3(grid_rows(R)), dim3(LT), 0, (hipStream_t)stream, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_attn_loss_fwd(const float* L, long long sr, long long sc, int R, int Q, int K, const int* a_idx,
                     const int* s_idx, const float* sweight, const float* z, int S, int axis, float c_xe,
                     float c_sm, float* lse_sel, float* lse_full, float* colz, float* out, float* workspace,
                     void* stream) {
  const int smooth = c_sm != 0.f;
  FX_REQUIRE(R > 0 && Q > 0 && K >= 0 && K <= MAXK && Q <= 4096 && (axis == 0 || axis == 1),
             "attn_loss: bad sizes (K <= 64 matched columns)");
  FX_REQUIRE(L && z && out && workspace && lse_sel && (!smooth || lse_full) && (axis == 1 || colz),
             "attn_loss: null buffer");
  hipStream_t s = (hipStream_t)stream;
  AttnArgs a{};
  a.L = Mat{L, sr, sc};
  a.R = R;
  a.Q = Q;
  a.K = K;
  a.axis = axis;
  a.smooth = smooth;
  a.z = z;
  a.S = S;
  for (int i = 0; i < K; ++i) {
    FX_REQUIRE(a_idx[i] >= 0 && a_idx[i] < Q && s_idx[i] >= 0 && s_idx[i] < S, "attn_loss: match index range");
    a.a[i] = a_idx[i];
    a.s[i] = s_idx[i];
    a.sw[i] = sweight[i];
  }
  a.lse_sel = lse_sel;
  a.lse_full = lse_full;
  a.colz = colz;
  a.part = workspace;
  const int nb = grid_rows(std::max(R, K));
  fx_launch(attn_loss_fwd_kernel, dim3(nb), dim3(LT), 0, s, a);
  fx_launch(finish_kernel, dim3(1), dim3(64), 0, s, workspace, nb, c_xe, c_sm, out);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_attn_loss_bwd(const float* L, long long sr, long long sc, int R, int Q, int K, const int* a_idx,
                     const int* s_idx, const float* sweight, const float* z, int S, int axis, const float* lse_sel,
                     const float* lse_full, const float* colz, float c_xe, float c_sm, const float* gout, float* dL,
                     long long dsr, long long dsc, void* stream) {
  const int smooth = c_sm != 0.f;
  FX_REQUIRE(R > 0 && Q > 0 && K >= 0 && K <= MAXK, "attn_loss_bwd: bad sizes");
  AttnBwdArgs a{};
  a.L = Mat{L, sr, sc};
  a.R = R;
  a.Q = Q;
  a.K = K;
  a.axis = axis;
  a.smooth = smooth;
  a.z = z;
  a.S = S;
  for (int i = 0; i < K; ++i) {
    a.a[i] = a_idx[i];
    a.s[i] = s_idx[i];
    a.sw[i] = sweight[i];
  }
  a.lse_sel = lse_sel;
  a.lse_full = lse_full;
  a.colz = colz;
  a.gout = gout;
  a.c_xe = c_xe;
  a.c_sm = c_sm;
  a.dL = dL;
  a.dsr = dsr;
  a.dsc = dsc;
  fx_launch(attn_loss_bwd_kernel, dim3(grid_rows(R)), dim3(LT), 0, (hipStream_t)stream, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // extern "C"
