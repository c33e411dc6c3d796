// The loss phase of FACT / FACT_CLIP for a whole batch of videos in a handful of launches
// (fact_clip/models/loss.py, blocks.py:677-786 _loss_one_video, blocks.py:788-887 eval_with_clip).
//
// The reference builds the loss of every video from ~150 ATen ops (one-hot matrices, index_add
// "zooms" of them onto the TDU segments, F.cross_entropy, the InfoNCE log-softmaxes, numpy soft-IoU
// for the matching) with a Python loop around them; round 1 here still had ~300 small launches with
// host work between them.  Here:
//   fx_match_cost     one launch: every video's Hungarian cost -pc P[:, transcript] - a2fc softIoU.
//                     The soft IoU needs no one-hot matrix: ground-truth segments are frame intervals,
//                     overlap[a,s] = sum of a's attention over segment s and union = len_s + colsum_a -
//                     overlap[a,s] (attention <= 1, so min(attn + 1, 1) = 1 inside the segment).
//   fx_loss_terms_fwd every CE / smooth / cross-attention / InfoNCE term of every block of every video
//                     from ONE device-resident term table: the InfoNCE similarity GEMMs, then ONE launch
//                     of every term over (row blocks x terms), one fixed-order finish (InfoNCE column
//                     log-softmax merged from per-block partials) and one combine into the batch loss and
//                     the per-video values.  Soft targets (the TDU "zoom" of the one-hot labels,
//                     loss.py:226-231, 266-269) are frame-interval overlaps between TDU segments and
//                     ground-truth segments, computed in the kernels.
//   fx_loss_terms_bwd the gradient of every term's logits: class, attention, InfoNCE launches (+ GEMM).
//   fx_eval_pred      one launch: every video's per-frame prediction (eval_with_clip / Block._eval).
#include <algorithm>
#include <cmath>

#include "fx_common.h"
#include "ops.h"

namespace fx {
namespace {

constexpr int VT = 256;        // threads per block (4 waves, one row at a time per wave)

__device__ __forceinline__ float vsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float vmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float at(const fx_loss_term& t, int r, int c) {
  return t.x[(long long)r * t.sr + (long long)c * t.sc];
}

__device__ __forceinline__ float row_lse_t(const fx_loss_term& t, int r, int n, int lane) {
  float m = -INFINITY;
  for (int c = lane; c < n; c += 64) m = fmaxf(m, at(t, r, c));
  m = vmax(m);
  float s = 0.f;
  for (int c = lane; c < n; c += 64) s += __expf(at(t, r, c) - m);
  return m + __logf(vsum(s));
}

// row r's frame interval
__device__ __forceinline__ void row_iv(const fx_loss_term& t, int r, int& a, int& b) {
  if (t.rs) {
    a = t.rs[r];
    b = t.re[r];
  } else {
    a = b = r;
  }
}

__device__ __forceinline__ float overlap(int a0, int a1, int b0, int b1) {
  const int lo = max(a0, b0), hi = min(a1, b1);
  return hi >= lo ? (float)(hi - lo + 1) : 0.f;
}

// first ground-truth segment whose end >= f (segments sorted, contiguous)
__device__ __forceinline__ int first_gt(const fx_loss_term& t, int f) {
  int lo = 0, hi = t.G;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (t.ge[m] < f) lo = m + 1;
    else hi = m;
  }
  return lo;
}

// gradient of the smooth term w.r.t. log_softmax(x)[r, c] (through the clamp), unscaled
__device__ __forceinline__ float smooth_g(const fx_loss_term& t, int r, int c, float l0, float lm, float lp1, int R) {
  float g = 0.f;
  const float lpc = at(t, r, c) - l0;
  if (r > 0) {
    const float d = lpc - (at(t, r - 1, c) - lm);
    if (d * d <= 16.f) g += 2.f * d;
  }
  if (r + 1 < R) {
    const float d = (at(t, r + 1, c) - lp1) - lpc;
    if (d * d <= 16.f) g -= 2.f * d;
  }
  return g;
}

// ------------------------------------------------------------------ class terms (frame / seg / token CE + smooth)
// rows [r0, r1) of one wave: the next row's lse is carried into the following iteration
__device__ void class_fwd(const fx_loss_term& t, int lane, int r0, int r1, float& ce, float& sm) {
  float l0 = r0 < r1 ? row_lse_t(t, r0, t.C, lane) : 0.f;
  for (int r = r0; r < r1; ++r) {
    if (lane == 0) t.lse[r] = l0;
    if (t.y) {
      if (lane == 0) {
        const int c = t.y[r];
        if (c >= 0) ce += t.w[c] * (l0 - at(t, r, c));
      }
    } else if (t.G > 0) {
      // soft target: class distribution of the row's frame interval over the ground-truth segments
      int f0, f1;
      row_iv(t, r, f0, f1);
      const float inv = 1.f / (float)(f1 - f0 + 1);
      float acc = 0.f;
      for (int j = first_gt(t, f0) + lane; j < t.G && t.gs[j] <= f1; j += 64) {
        const int c = t.gl[j];
        acc += overlap(f0, f1, t.gs[j], t.ge[j]) * inv * t.w[c] * (l0 - at(t, r, c));
      }
      ce += acc;
    }
    float l1 = 0.f;
    if (r + 1 < t.R && (t.c_sm != 0.f || r + 1 < r1)) l1 = row_lse_t(t, r + 1, t.C, lane);
    if (t.c_sm != 0.f && r + 1 < t.R) {
      float s = 0.f;
      for (int c = lane; c < t.C; c += 64) {
        const float d = (at(t, r + 1, c) - l1) - (at(t, r, c) - l0);
        s += fminf(d * d, 16.f);
      }
      sm += s;
    }
    l0 = l1;
  }
}

__device__ void class_bwd(const fx_loss_term& t, float* tzrow, int lane, int r0, int r1, float gout) {
  const float g_ce = gout * t.c_ce, g_sm = gout * t.c_sm;
  const bool smooth = t.c_sm != 0.f;
  for (int r = r0; r < r1; ++r) {
    const float l0 = t.lse[r];
    const float lm = (smooth && r > 0) ? t.lse[r - 1] : 0.f;
    const float lp1 = (smooth && r + 1 < t.R) ? t.lse[r + 1] : 0.f;
    // target weights of the row: tz[c] (LDS row of this wave) and their sum zw
    for (int c = lane; c < t.C; c += 64) tzrow[c] = 0.f;
    float zw = 0.f;
    if (t.y) {
      const int yc = t.y[r];
      if (yc >= 0) {
        zw = t.w[yc];
        if (lane == 0) tzrow[yc] = zw;
      }
    } else if (t.G > 0) {
      int f0, f1;
      row_iv(t, r, f0, f1);
      const float inv = 1.f / (float)(f1 - f0 + 1);
      if (lane == 0)   // few segments per row: one lane, fixed order
        for (int j = first_gt(t, f0); j < t.G && t.gs[j] <= f1; ++j) {
          const int c = t.gl[j];
          const float v = overlap(f0, f1, t.gs[j], t.ge[j]) * inv * t.w[c];
          tzrow[c] += v;
          zw += v;
        }
      zw = __shfl(zw, 0, 64);
    }
    __builtin_amdgcn_wave_barrier();
    float gsum = 0.f;
    if (smooth)
      for (int c = lane; c < t.C; c += 64) gsum += smooth_g(t, r, c, l0, lm, lp1, t.R) * g_sm;
    gsum = vsum(gsum);
    for (int c = lane; c < t.C; c += 64) {
      const float p = __expf(at(t, r, c) - l0);
      const float g = smooth ? smooth_g(t, r, c, l0, lm, lp1, t.R) * g_sm : 0.f;
      t.dx[(long long)r * t.dsr + (long long)c * t.dsc] = (g - p * gsum) + g_ce * (zw * p - tzrow[c]);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------ attention terms (cross_attn_loss(_tdu) + smooth)
__device__ __forceinline__ float attn_target(const fx_loss_term& t, int r, int i) {
  int f0, f1;
  row_iv(t, r, f0, f1);
  return overlap(f0, f1, t.kgs[i], t.kge[i]) / (float)(f1 - f0 + 1);
}

__device__ void attn_fwd(const fx_loss_term& t, int lane, int gw, int r0, int r1, float& xe, float& sm) {
  if (t.axis == 1) {   // log_softmax over the K matched columns of each row (K may exceed a wave)
    for (int r = r0; r < r1; ++r) {
      float m = -INFINITY;
      for (int i = lane; i < t.K; i += 64) m = fmaxf(m, at(t, r, t.ka[i]));
      m = vmax(m);
      float se = 0.f;
      for (int i = lane; i < t.K; i += 64) se += __expf(at(t, r, t.ka[i]) - m);
      const float l = m + __logf(vsum(se));
      if (lane == 0) t.lse[r] = l;
      for (int i = lane; i < t.K; i += 64) xe += -(at(t, r, t.ka[i]) - l) * attn_target(t, r, i) * t.ksw[i];
    }
  } else if (gw < t.K) {   // one wave per matched column: log_softmax over the rows
    const int i = gw, q = t.ka[i];
    float m = -INFINITY;
    for (int r = lane; r < t.R; r += 64) m = fmaxf(m, at(t, r, q));
    m = vmax(m);
    float s = 0.f, zs = 0.f, zl = 0.f;
    for (int r = lane; r < t.R; r += 64) {
      const float x = at(t, r, q);
      const float zz = attn_target(t, r, i);
      s += __expf(x - m);
      zs += zz;
      zl += zz * x;
    }
    const float l = m + __logf(vsum(s));
    zs = vsum(zs);
    zl = vsum(zl);
    if (lane == 0) {
      t.lse2[t.R + i] = l;              // per-column lse after the R row slots
      t.colz[i] = zs * t.ksw[i];
      xe += -(zl - zs * l) * t.ksw[i];
    }
  }
  if (t.c_sm != 0.f) {
    float l0 = r0 < r1 ? row_lse_t(t, r0, t.C, lane) : 0.f;
    for (int r = r0; r < r1; ++r) {
      if (lane == 0) t.lse2[r] = l0;
      if (r + 1 < t.R) {
        const float l1 = row_lse_t(t, r + 1, t.C, lane);
        float s = 0.f;
        for (int c = lane; c < t.C; c += 64) {
          const float d = (at(t, r + 1, c) - l1) - (at(t, r, c) - l0);
          s += fminf(d * d, 16.f);
        }
        sm += s;
        l0 = l1;
      }
    }
  }
}

// InfoNCE, rows [r0, r1) of one wave: row lse and CE of the valid frames
__device__ void infonce_rows(const fx_loss_term& t, int lane, int r0, int r1, float& v2t, float& nval) {
  for (int r = r0; r < r1; ++r) {
    const int y = t.y[r];
    const float l = row_lse_t(t, r, t.C, lane);
    if (lane == 0) {
      t.lse[r] = l;
      if (y >= 0) {
        v2t += l - at(t, r, y);
        nval += 1.f;
      }
    }
  }
}

// InfoNCE column partials over the block's rows [b0, b1): per column online (max, sum exp) over the
// valid frames, their count and the sum of the frames labelled with the column's class
__device__ void infonce_cols(const fx_loss_term& t, int b0, int b1, float* cp) {
  for (int c = threadIdx.x; c < t.C; c += VT) {
    float m = -INFINITY, s = 0.f, cnt = 0.f, sx = 0.f;
    for (int r = b0; r < b1; ++r) {
      const int y = t.y[r];
      if (y < 0) continue;
      const float x = at(t, r, c);
      if (x > m) {
        s = s * __expf(m - x) + 1.f;
        m = x;
      } else {
        s += __expf(x - m);
      }
      if (y == c) {
        cnt += 1.f;
        sx += x;
      }
    }
    reinterpret_cast<float4*>(cp)[(long long)blockIdx.x * t.C + c] = make_float4(m, s, cnt, sx);
  }
}

__device__ void attn_bwd(const fx_loss_term& t, int lane, int r0, int r1, float gout) {
  const float g_xe = gout * t.c_ce, g_sm = gout * t.c_sm;
  const bool smooth = t.c_sm != 0.f;
  for (int r = r0; r < r1; ++r) {
    const float l0 = smooth ? t.lse2[r] : 0.f;
    const float lm = (smooth && r > 0) ? t.lse2[r - 1] : 0.f;
    const float lp1 = (smooth && r + 1 < t.R) ? t.lse2[r + 1] : 0.f;
    float gsum = 0.f;
    if (smooth)
      for (int c = lane; c < t.C; c += 64) gsum += smooth_g(t, r, c, l0, lm, lp1, t.R) * g_sm;
    gsum = vsum(gsum);
    float zrow = 0.f;
    if (t.axis == 1) {
      for (int i = lane; i < t.K; i += 64) zrow += attn_target(t, r, i) * t.ksw[i];
      zrow = vsum(zrow);
    }
    for (int c = lane; c < t.C; c += 64) {
      float g = 0.f;
      if (smooth) g = smooth_g(t, r, c, l0, lm, lp1, t.R) * g_sm - __expf(at(t, r, c) - l0) * gsum;
      for (int i = 0; i < t.K; ++i) {
        if (t.ka[i] != c) continue;
        const float x = at(t, r, c);
        const float zz = attn_target(t, r, i) * t.ksw[i];
        if (t.axis == 1) g += g_xe * (__expf(x - t.lse[r]) * zrow - zz);
        else g += g_xe * (__expf(x - t.lse2[t.R + i]) * t.colz[i] - zz);
      }
      t.dx[(long long)r * t.dsr + (long long)c * t.dsc] = g;
    }
  }
}

// ------------------------------------------------------------------ term kernels (grid: row blocks x terms)
// block b of a term owns the contiguous rows [b * rpb, (b + 1) * rpb), each wave a quarter of them
__device__ __forceinline__ void wave_rows(int R, int wv, int& r0, int& r1, int& b0, int& b1) {
  const int rpw = (R + gridDim.x * (VT / 64) - 1) / (gridDim.x * (VT / 64));
  b0 = min(R, (int)blockIdx.x * (VT / 64) * rpw);
  b1 = min(R, b0 + (VT / 64) * rpw);
  r0 = min(R, b0 + wv * rpw);
  r1 = min(R, r0 + rpw);
}

__global__ __launch_bounds__(VT) void terms_fwd_kernel(const fx_loss_term* terms, float* part) {
  __shared__ float red[2][VT / 64];
  const fx_loss_term& t = terms[blockIdx.y];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int gw = blockIdx.x * (VT / 64) + wv;
  int r0, r1, b0, b1;
  wave_rows(t.R, wv, r0, r1, b0, b1);
  float a = 0.f, b = 0.f;
  if (t.kind == FX_TERM_CLASS) class_fwd(t, lane, r0, r1, a, b);
  else if (t.kind == FX_TERM_ATTN) attn_fwd(t, lane, gw, r0, r1, a, b);
  else {
    infonce_rows(t, lane, r0, r1, a, b);
    infonce_cols(t, b0, b1, t.colz + ((t.C + 4) & ~3));
  }
  a = vsum(a);
  b = vsum(b);
  if (lane == 0) {
    red[0][wv] = a;
    red[1][wv] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f;
    for (int i = 0; i < VT / 64; ++i) {
      s0 += red[0][i];
      s1 += red[1][i];
    }
    part[(t.slot * (long long)gridDim.x + blockIdx.x) * 2] = s0;
    part[(t.slot * (long long)gridDim.x + blockIdx.x) * 2 + 1] = s1;
  }
}

__global__ __launch_bounds__(VT) void terms_bwd_kernel(const fx_loss_term* terms, const float* gterm, int kind) {
  extern __shared__ float tz[];   // [4 waves][maxC] target rows of the class terms
  const fx_loss_term& t = terms[blockIdx.y];
  if (t.kind != kind) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int r0, r1, b0, b1;
  wave_rows(t.R, wv, r0, r1, b0, b1);
  if (kind == FX_TERM_CLASS) class_bwd(t, tz + wv * t.C, lane, r0, r1, gterm[blockIdx.y]);
  else attn_bwd(t, lane, r0, r1, gterm[blockIdx.y]);
}

// gterm[i] = sum_o gout[o] coef[o, i]   (upstream gradient of each term)
__global__ __launch_bounds__(64) void combine_bwd_kernel(const float* gout, const float* coef, int nterms, int nout,
                                                         float* gterm) {
  for (int i = blockIdx.x * 64 + threadIdx.x; i < nterms; i += gridDim.x * 64) {
    float s = 0.f;
    for (int o = 0; o < nout; ++o) s += gout[o] * coef[(long long)o * nterms + i];
    gterm[i] = s;
  }
}

// term value = c_ce * sum(part0) + c_sm * sum(part1), blocks in fixed order.  InfoNCE (loss.py:280-341):
// x = sim (R frames x C classes), y = class per frame (-1: masked); the column partials of the row
// blocks merge into the column lse (lse2), the class counts (colz, colz[C] = valid frames) and
//   value = c_ce * ( v2t / n_valid + (1/C) sum_c -(sum_{y_t = c} sim[t, c] - count_c lse_c) / max(count_c, 1) )
constexpr int FT = 1024;   // finish: one wave per InfoNCE column group
__global__ __launch_bounds__(FT) void terms_finish_kernel(const fx_loss_term* terms, const float* part, int nb,
                                                          float* vals) {
  __shared__ float red[FT / 64];
  const int i = blockIdx.x;
  const fx_loss_term& t = terms[i];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float a = 0.f, b = 0.f;
  if (wv == 0) {
    for (int k = lane; k < nb; k += 64) {
      a += part[((long long)t.slot * nb + k) * 2];
      b += part[((long long)t.slot * nb + k) * 2 + 1];
    }
    a = vsum(a);
    b = vsum(b);
  }
  if (t.kind != FX_TERM_INFONCE) {
    if (threadIdx.x == 0) vals[i] = t.c_sm != 0.f ? t.c_ce * a + t.c_sm * b : t.c_ce * a;
    return;
  }
  if (wv == 0 && lane == 0) red[0] = a, red[1] = b;   // (slots reused below after a barrier)
  __syncthreads();
  a = red[0];
  b = red[1];
  __syncthreads();
  // one wave per column, lanes over the row-block partials (float4 {max, sum exp, count, sum x})
  const float4* cp = reinterpret_cast<const float4*>(t.colz + ((t.C + 4) & ~3));
  float t2v = 0.f;
  for (int c = wv; c < t.C; c += FT / 64) {
    float m = -INFINITY, cnt = 0.f, sx = 0.f, s = 0.f;
    for (int k = lane; k < nb; k += 64) {
      const float4 o = cp[(long long)k * t.C + c];
      if (o.y > 0.f) {
        const float mn = fmaxf(m, o.x);
        s = s * __expf(m - mn) + o.y * __expf(o.x - mn);
        m = mn;
      }
      cnt += o.z;
      sx += o.w;
    }
    const float M = vmax(m);
    s = vsum(m == -INFINITY ? 0.f : s * __expf(m - M));
    cnt = vsum(cnt);
    sx = vsum(sx);
    const float l = M + __logf(s);
    if (lane == 0) {
      t.lse2[c] = l;
      t.colz[c] = cnt;
      t2v += cnt > 0.f ? -(sx - cnt * l) / cnt : 0.f;
    }
  }
  if (lane == 0) red[wv] = t2v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tt = 0.f;
    for (int k = 0; k < FT / 64; ++k) tt += red[k];
    t.colz[t.C] = b;
    vals[i] = b > 0.f ? t.c_ce * (a / b + tt / (float)t.C) : 0.f;
  }
}

// dsim[t, c] = g c_ce ( (p_row - [c == y_t]) / n_valid + (has_c p_col[t, c] - [c == y_t] / count_c) / C ) for
// valid frames, 0 for masked ones; written into dx (R x C), then the caller's GEMM takes it to demb
__global__ __launch_bounds__(VT) void infonce_bwd_kernel(const fx_loss_term* terms, const float* gterm) {
  const fx_loss_term& t = terms[blockIdx.y];
  if (t.kind != FX_TERM_INFONCE) return;
  const float n = t.colz[t.C];
  const float g = gterm[blockIdx.y] * t.c_ce;
  const float inv_n = n > 0.f ? 1.f / n : 0.f, inv_c = 1.f / (float)t.C;
  const long long total = (long long)t.R * t.C;
  for (long long e = (long long)blockIdx.x * VT + threadIdx.x; e < total; e += (long long)gridDim.x * VT) {
    const int r = (int)(e / t.C), c = (int)(e - (long long)r * t.C);
    const int y = t.y[r];
    float v = 0.f;
    if (y >= 0 && n > 0.f) {
      const float x = at(t, r, c);
      const float cnt = t.colz[c];
      const float pr = __expf(x - t.lse[r]);
      const float pc = cnt > 0.f ? __expf(x - t.lse2[c]) : 0.f;
      const float d = c == y ? 1.f : 0.f;
      v = g * ((pr - d) * inv_n + (pc - (cnt > 0.f ? d / cnt : 0.f)) * inv_c);
    }
    t.dx[(long long)r * t.dsr + (long long)c * t.dsc] = v;
  }
}

// out[o] = sum_i coef[o * nterms + i] vals[i]   (fixed order)
__global__ __launch_bounds__(64) void combine_kernel(const float* vals, const float* coef, int nterms, int nout,
                                                     float* out) {
  const int o = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  for (int i = lane; i < nterms; i += 64) s += coef[(long long)o * nterms + i] * vals[i];
  s = vsum(s);
  if (lane == 0 && o < nout) out[o] = s;
}

// ------------------------------------------------------------------ matching cost (loss.py:108-153, 91-106)
// frame t's attention to token a: frame-level att[t*lda + a] or segment-level att[seg_id[t]*lda + a]
__device__ __forceinline__ float frame_attn(const fx_video_attn& v, int t, int a) {
  const int row = v.seg_id ? v.seg_id[t] : t;
  return v.attn[(long long)row * v.lda + a];
}

__global__ __launch_bounds__(VT) void match_cost_kernel(const fx_video_attn* vids, float pc, float a2fc, int Gmax,
                                                        float* cost) {
  extern __shared__ float sm[];   // [C1] prob row, then [Gmax] overlaps
  const int a = blockIdx.x, vi = blockIdx.y;
  const fx_video_attn& v = vids[vi];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* prob = sm;
  float* ov = sm + v.C1;
  if (a >= v.Q) return;
  if (wv == 0) {
    const float* row = v.clogit + (long long)a * v.ldc;
    float m = -INFINITY;
    for (int c = lane; c < v.C1; c += 64) m = fmaxf(m, row[c]);
    m = vmax(m);
    float s = 0.f;
    for (int c = lane; c < v.C1; c += 64) s += __expf(row[c] - m);
    s = vsum(s);
    for (int c = lane; c < v.C1; c += 64) prob[c] = __expf(row[c] - m) / s;
  }
  for (int sg = wv; sg < v.G; sg += VT / 64) {
    float acc = 0.f;
    for (int t = v.gs[sg] + lane; t <= v.ge[sg]; t += 64) acc += frame_attn(v, t, a);
    acc = vsum(acc);
    if (lane == 0) ov[sg] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float col = 0.f;
    for (int sg = 0; sg < v.G; ++sg) col += ov[sg];
    ov[v.G] = col;
  }
  __syncthreads();
  const float col = ov[v.G];
  for (int sg = threadIdx.x; sg < Gmax; sg += VT) {
    float c = 0.f;
    if (sg < v.G) {
      const float len = (float)(v.ge[sg] - v.gs[sg] + 1);
      const float den = col - ov[sg] + len;
      const float iou = den != 0.f ? ov[sg] / den : 0.f;
      c = -pc * prob[v.gl[sg]] - a2fc * iou;
    }
    cost[((long long)vi * v.Q + a) * Gmax + sg] = c;
  }
}

// ------------------------------------------------------------------ per-frame prediction (blocks.py:243-261, 854-887)
// fprob = softmax(flogit[t]) (frame classifier or CLIP similarity); if any token predicts a non-null
// class: pred = argmax((1 - w) qtk_prob[best token of t] + w fprob), best token = first argmax of t's
// attention over the non-null tokens; else pred = argmax(fprob).  (first maximum everywhere, as torch)
__global__ __launch_bounds__(VT) void eval_pred_kernel(const fx_video_attn* vids, float w, int32_t* pred) {
  extern __shared__ float sm[];   // [Q][C] token class probs, [Q] is_token flags
  const fx_video_attn& v = vids[blockIdx.y];
  const int C = v.C1 - 1, Q = v.Q;
  float* qp = sm;
  float* ist = sm + Q * C;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int a = wv; a < Q; a += VT / 64) {
    const float* row = v.clogit + (long long)a * v.ldc;
    // argmax over all C1 logits (first max) and softmax over the first C
    float bm = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < v.C1; c += 64) {
      const float x = row[c];
      if (x > bm) {
        bm = x;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(bm, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (om > bm || (om == bm && oi < bi)) {
        bm = om;
        bi = oi;
      }
    }
    float m = -INFINITY;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, row[c]);
    m = vmax(m);
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(row[c] - m);
    s = vsum(s);
    for (int c = lane; c < C; c += 64) qp[a * C + c] = __expf(row[c] - m) / s;
    if (lane == 0) ist[a] = bi != C ? 1.f : 0.f;
  }
  __syncthreads();
  const int t = blockIdx.x * VT + threadIdx.x;
  if (t >= v.T) return;
  bool any = false;
  int best = -1;
  float ba = -INFINITY;
  for (int a = 0; a < Q; ++a) {
    if (ist[a] == 0.f) continue;
    any = true;
    const float x = frame_attn(v, t, a);
    if (best < 0 || x > ba) {
      ba = x;
      best = a;
    }
  }
  const float* fl = v.flogit + (long long)t * v.ldf;
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, fl[c]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += __expf(fl[c] - m);
  const float inv = 1.f / s;
  float bv = -INFINITY;
  int bc = 0;
  for (int c = 0; c < C; ++c) {
    const float fp = __expf(fl[c] - m) * inv;
    const float p = any ? (1.f - w) * qp[best * C + c] + w * fp : fp;
    if (p > bv) {
      bv = p;
      bc = c;
    }
  }
  pred[v.pred_off + t] = bc;
}

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

long long fx_loss_terms_workspace_floats(int nterms) {
  return 2LL * FX_LOSS_NB * std::max(nterms, 1) + std::max(nterms, 1);
}

int fx_loss_terms_fwd(const fx_loss_term* terms_host, const fx_loss_term* terms_dev, int nterms, const float* coef_dev,
                      int nout, float* out, float* workspace, void* stream) {
  FX_REQUIRE(terms_host && terms_dev && nterms > 0 && coef_dev && out && workspace, "loss_terms: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int nb = FX_LOSS_NB;
  float* part = workspace;
  float* vals = workspace + 2LL * nb * nterms;
  for (int i = 0; i < nterms; ++i) {
    const fx_loss_term& t = terms_host[i];
    FX_REQUIRE(t.kind >= 0 && t.kind <= 2, "loss_terms: unknown term kind");
    FX_REQUIRE(t.R > 0 && t.C > 0 && t.x && t.lse, "loss_terms: empty term");
    FX_REQUIRE(t.kind != FX_TERM_ATTN || (t.K >= 0 && t.K <= FX_LOSS_MAXK && t.lse2 && t.colz &&
                                          (t.K == 0 || (t.ka && t.kgs && t.kge && t.ksw))),
               "loss_terms: attention term needs K <= FX_LOSS_MAXK matched columns, their tables and scratch");
    FX_REQUIRE(t.kind != FX_TERM_CLASS || t.w, "loss_terms: class term needs weights");
    FX_REQUIRE(t.kind != FX_TERM_INFONCE || (t.y && t.lse2 && t.colz && t.emb && t.text && t.dx && t.sc == 1 &&
                                             t.dsc == 1 && t.D > 0),
               "loss_terms: InfoNCE term needs labels, embeddings, text and scratch");
    FX_REQUIRE(t.slot == i, "loss_terms: term slot must equal its index");
    if (t.kind == FX_TERM_INFONCE) {   // similarity GEMM first: sim = emb . text^T / temp
      fx_gemm_desc d = gemm_desc(t.R, t.C, t.D, op_rows(t.emb, t.ld_emb), op_rows(t.text, t.D),
                                 const_cast<float*>(t.x), t.sr);
      d.alpha = t.inv_temp;
      FX_TRY(launch_gemm(d, s));
    }
  }
  fx_launch(terms_fwd_kernel, dim3(nb, nterms), dim3(VT), 0, s, terms_dev, part);
  FX_CHECK_HIP(hipGetLastError());
  fx_launch(terms_finish_kernel, dim3(nterms), dim3(FT), 0, s, terms_dev, part, nb, vals);
  FX_CHECK_HIP(hipGetLastError());
  fx_launch(combine_kernel, dim3(nout), dim3(64), 0, s, vals, coef_dev, nterms, nout, out);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_loss_terms_bwd(const fx_loss_term* terms_host, const fx_loss_term* terms_dev, int nterms, const float* coef,
                      int nout, const float* gout, float* workspace, void* stream) {
  FX_REQUIRE(terms_host && terms_dev && nterms > 0 && coef && gout && workspace, "loss_terms_bwd: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  float* gterm = workspace;
  fx_launch(combine_bwd_kernel, dim3(cdiv(nterms, 64)), dim3(64), 0, s, gout, coef, nterms, nout, gterm);
  FX_CHECK_HIP(hipGetLastError());
  int maxC = 1;
  bool has[3] = {false, false, false};
  for (int i = 0; i < nterms; ++i) {
    const fx_loss_term& t = terms_host[i];
    FX_REQUIRE(t.dx, "loss_terms_bwd: term without a gradient buffer");
    has[t.kind] = true;
    if (t.kind == FX_TERM_CLASS) maxC = std::max(maxC, t.C);
  }
  if (has[FX_TERM_CLASS]) {
    fx_launch(terms_bwd_kernel, dim3(FX_LOSS_NB, nterms), dim3(VT), sizeof(float) * 4 * maxC, s, terms_dev, gterm,
                       (int)FX_TERM_CLASS);
    FX_CHECK_HIP(hipGetLastError());
  }
  if (has[FX_TERM_ATTN]) {
    fx_launch(terms_bwd_kernel, dim3(FX_LOSS_NB, nterms), dim3(VT), 0, s, terms_dev, gterm, (int)FX_TERM_ATTN);
    FX_CHECK_HIP(hipGetLastError());
  }
  if (has[FX_TERM_INFONCE]) {
    fx_launch(infonce_bwd_kernel, dim3(256, nterms), dim3(VT), 0, s, terms_dev, gterm);
    FX_CHECK_HIP(hipGetLastError());
    for (int i = 0; i < nterms; ++i) {   // demb = dsim . text / temp
      const fx_loss_term& t = terms_host[i];
      if (t.kind != FX_TERM_INFONCE) continue;
      FX_REQUIRE(t.demb, "loss_terms_bwd: InfoNCE term without an embedding gradient buffer");
      fx_gemm_desc d = gemm_desc(t.R, t.D, t.C, op_rows(t.dx, t.dsr), op_cols(t.text, t.D), t.demb, t.ld_demb);
      d.alpha = t.inv_temp;
      FX_TRY(launch_gemm(d, s));
    }
  }
  return FX_OK;
}

int fx_match_cost(const fx_video_attn* vids_host, const fx_video_attn* vids_dev, int nvid, float pc, float a2fc,
                  int Gmax, float* cost, void* stream) {
  FX_REQUIRE(vids_host && vids_dev && nvid > 0 && Gmax > 0 && cost, "match_cost: bad arguments");
  int Q = 0, C1 = 0;
  for (int i = 0; i < nvid; ++i) {
    FX_REQUIRE(vids_host[i].G <= Gmax && vids_host[i].G >= 1, "match_cost: segment count");
    Q = std::max(Q, vids_host[i].Q);
    C1 = std::max(C1, vids_host[i].C1);
  }
  fx_launch(match_cost_kernel, dim3(Q, nvid), dim3(VT), sizeof(float) * (C1 + Gmax + 1), (hipStream_t)stream,
                     vids_dev, pc, a2fc, Gmax, cost);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_eval_pred(const fx_video_attn* vids_host, const fx_video_attn* vids_dev, int nvid, float mwt, int32_t* pred,
                 void* stream) {
  FX_REQUIRE(vids_host && vids_dev && nvid > 0 && pred, "eval_pred: bad arguments");
  int T = 0, QC = 0;
  for (int i = 0; i < nvid; ++i) {
    const fx_video_attn& v = vids_host[i];
    FX_REQUIRE(v.flogit && v.C1 >= 2 && v.Q >= 1, "eval_pred: video without logits");
    T = std::max(T, v.T);
    QC = std::max(QC, v.Q * v.C1);
  }
  FX_REQUIRE((size_t)QC * sizeof(float) <= 60 * 1024, "eval_pred: too many token x class probabilities");
  fx_launch(eval_pred_kernel, dim3(cdiv(T, VT), nvid), dim3(VT), sizeof(float) * QC, (hipStream_t)stream,
                     vids_dev, mwt, pred);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // extern "C"
