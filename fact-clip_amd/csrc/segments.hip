// Temporal down/up-sampling on device (UpdateBlockTDU.temporal_downsample,
// blocks.py:417-437; TemporalDownsampleUpsample, basic.py:595-651;
// parse_label, utils/utils.py:25-48).
//
// The reference copies the argmax to the host, run-length-encodes it in numpy
// and copies index tensors back.  Here: argmax (many workgroups) -> one
// 1024-thread workgroup does the boundary scan and writes seg_id / starts /
// ends / S; the host reads S once (the reference also synchronises here).
// Segment pooling is a deterministic, frame-ordered sum per segment.
#include <algorithm>

#include "fx_common.h"

namespace fx {
namespace {

__global__ __launch_bounds__(256) void argmax_rows_kernel(const float* x, long long ldx, int col0, int ncls, int T,
                                                          int32_t* pred) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const float* xr = x + (long long)t * ldx + col0;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = lane; c < ncls; c += 64) {
    const float v = xr[c];
    if (v > best) {  // lanes visit increasing c: keeps the first max per lane
      best = v;
      bi = c;
    }
  }
  // reduce (max value, then smallest index) across the wave == torch first-max argmax
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > best || (ov == best && oi < bi)) {
      best = ov;
      bi = oi;
    }
  }
  if (lane == 0) pred[t] = (bi == 0x7fffffff) ? 0 : bi;
}

constexpr int SCAN_THREADS = 1024;

constexpr int MAXV = 32;
struct RowOff {
  int off[MAXV + 1];   // video v of the launch owns rows [off[v], off[v+1])
};

__global__ __launch_bounds__(SCAN_THREADS) void boundary_scan_kernel(const int32_t* pred, RowOff ro, int32_t* seg_id,
                                                                     int32_t* seg_start, int32_t* seg_end,
                                                                     int32_t* num_seg) {
  // one block per video: its rows, video-local segment numbering and frame indices
  const long long vo = ro.off[blockIdx.x];
  const int T = ro.off[blockIdx.x + 1] - ro.off[blockIdx.x];
  pred += vo;
  seg_id += vo;
  seg_start += vo;
  seg_end += vo;
  num_seg += blockIdx.x;
  __shared__ int32_t sums[SCAN_THREADS];
  const int tid = threadIdx.x;
  const int per = (T + SCAN_THREADS - 1) / SCAN_THREADS;
  const int b = tid * per, e = min(T, b + per);
  int cnt = 0;
  for (int t = b; t < e; ++t) cnt += (t == 0 || pred[t] != pred[t - 1]) ? 1 : 0;
  sums[tid] = cnt;
  __syncthreads();
  // Hillis-Steele inclusive scan over 1024 partial counts
  for (int off = 1; off < SCAN_THREADS; off <<= 1) {
    const int v = tid >= off ? sums[tid - off] : 0;
    __syncthreads();
    sums[tid] += v;
    __syncthreads();
  }
  int sid = sums[tid] - cnt - 1;  // segment index before this chunk's first frame
  for (int t = b; t < e; ++t) {
    if (t == 0 || pred[t] != pred[t - 1]) {
      ++sid;
      seg_start[sid] = t;
      if (sid > 0) seg_end[sid - 1] = t - 1;
    }
    seg_id[t] = sid;
  }
  if (tid == SCAN_THREADS - 1) {
    const int S = sums[tid];
    num_seg[0] = S;
    if (S > 0) seg_end[S - 1] = T - 1;
  }
}

// y[s, c] = (sum_{t=start..end} x[t, c]) * (mean ? 1/len : 1)  (+ y if accumulate)
// One workgroup per (segment, 64 channels): 16 waves stride over the segment's frames
// (4 independent loads in flight per lane), then a fixed-order LDS combine (deterministic).
constexpr int SEG_WAVES = 16;
__global__ __launch_bounds__(64 * SEG_WAVES) void seg_reduce_kernel(const float* x, long long ldx, const int32_t* st,
                                                                    const int32_t* en, int S, int cols, int mean,
                                                                    float* y, long long ldy, int accumulate) {
  __shared__ float part[SEG_WAVES][64];
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const int a = st[s], b = en[s];
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  if (c < cols) {
    const float* xp = x + c;
    int t = a + wv;
    for (; t + 3 * SEG_WAVES <= b; t += 4 * SEG_WAVES) {
      acc0 += xp[(long long)t * ldx];
      acc1 += xp[(long long)(t + SEG_WAVES) * ldx];
      acc2 += xp[(long long)(t + 2 * SEG_WAVES) * ldx];
      acc3 += xp[(long long)(t + 3 * SEG_WAVES) * ldx];
    }
    for (; t <= b; t += SEG_WAVES) acc0 += xp[(long long)t * ldx];
  }
  part[wv][lane] = (acc0 + acc1) + (acc2 + acc3);
  __syncthreads();
  if (wv == 0 && c < cols) {
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < SEG_WAVES; ++w) tot += part[w][lane];
    if (mean) tot = tot / (float)(b - a + 1);
    float* yp = y + (long long)s * ldy + c;
    *yp = accumulate ? *yp + tot : tot;
  }
}

// dx[t, c] (+)= dy[seg_id[t], c] / len
__global__ __launch_bounds__(256) void seg_mean_bwd_kernel(const float* dy, long long lddy, const int32_t* sid,
                                                           const int32_t* st, const int32_t* en, int T, int cols,
                                                           float* dx, long long lddx, int accumulate) {
  const int t = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (t >= T || c >= cols) return;
  const int s = sid[t];
  const float v = dy[(long long)s * lddy + c] / (float)(en[s] - st[s] + 1);
  float* p = dx + (long long)t * lddx + c;
  *p = accumulate ? *p + v : v;
}

struct GlobalizeArgs {
  const int32_t* seg_id;  // (nvid*T) video-local ids
  int32_t* gseg_id;       // (nvid*T) global ids
  const int32_t* st;      // (nvid*T) local tables
  const int32_t* en;
  int32_t* gst;           // (sum S) global frame rows
  int32_t* gen;
  int nv;
  int soff[MAXV + 1];     // segment prefix offsets of this chunk's videos
  int roff[MAXV + 1];     // frame-row offsets of this chunk's videos
};

__global__ __launch_bounds__(256) void seg_globalize_kernel(GlobalizeArgs a) {
  const int v = blockIdx.y;
  const int S = a.soff[v + 1] - a.soff[v];
  const long long base = a.roff[v];
  const int T = a.roff[v + 1] - a.roff[v];
  for (int t = blockIdx.x * 256 + threadIdx.x; t < T; t += gridDim.x * 256) {
    a.gseg_id[base + t] = a.seg_id[base + t] + a.soff[v];
    if (t < S) {
      a.gst[a.soff[v] + t] = a.st[base + t] + (int)base;
      a.gen[a.soff[v] + t] = a.en[base + t] + (int)base;
    }
  }
}

}  // namespace

static int row_of(int T, const int* row_off, int v) { return row_off ? row_off[v] : v * T; }

int launch_seg_globalize(int nvid, int T, const int* row_off, const int32_t* num_seg_host, const int32_t* seg_id,
                         const int32_t* st, const int32_t* en, int32_t* gseg_id, int32_t* gst, int32_t* gen,
                         hipStream_t s) {
  int off = 0;
  for (int c0 = 0; c0 < nvid; c0 += MAXV) {
    GlobalizeArgs a{};
    a.seg_id = seg_id;
    a.gseg_id = gseg_id;
    a.st = st;
    a.en = en;
    a.gst = gst;
    a.gen = gen;
    a.nv = std::min(MAXV, nvid - c0);
    int tmax = 1;
    for (int v = 0; v <= a.nv; ++v) {
      a.roff[v] = row_of(T, row_off, c0 + v);
      if (v > 0) tmax = std::max(tmax, a.roff[v] - a.roff[v - 1]);
    }
    for (int v = 0; v < a.nv; ++v) {
      a.soff[v] = off;
      off += num_seg_host[c0 + v];
    }
    a.soff[a.nv] = off;
    fx_launch(seg_globalize_kernel, dim3(std::max(1, std::min(cdiv(tmax, 256), 64)), a.nv), dim3(256), 0, s,
                       a);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

int launch_segments(const float* x, long long ldx, int col0, int ncls, int T, int nvid, const int* row_off,
                    int32_t* pred, int32_t* seg_id, int32_t* seg_start, int32_t* seg_end, int32_t* num_seg,
                    hipStream_t s) {
  FX_REQUIRE(ncls > 0 && nvid >= 1 && (row_off || T > 0), "segments: need T > 0 (or row offsets) and ncls > 0");
  const int rows = row_of(T, row_off, nvid);
  for (int v = 0; v < nvid; ++v) FX_REQUIRE(row_of(T, row_off, v + 1) > row_of(T, row_off, v), "segments: empty video");
  fx_launch(argmax_rows_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, x, ldx, col0, ncls, rows, pred);
  for (int c0 = 0; c0 < nvid; c0 += MAXV) {
    RowOff ro{};
    const int nv = std::min(MAXV, nvid - c0);
    for (int v = 0; v <= nv; ++v) ro.off[v] = row_of(T, row_off, c0 + v);
    fx_launch(boundary_scan_kernel, dim3(nv), dim3(SCAN_THREADS), 0, s, pred, ro, seg_id, seg_start, seg_end,
                       num_seg + c0);
  }
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_seg_reduce(const float* x, long long ldx, const int32_t* st, const int32_t* en, int S, int cols, int mean,
                      float* y, long long ldy, int accumulate, hipStream_t s) {
  if (S == 0 || cols == 0) return FX_OK;
  fx_launch(seg_reduce_kernel, dim3(S, cdiv(cols, 64)), dim3(64 * SEG_WAVES), 0, s, x, ldx, st, en, S, cols,
                     mean, y, ldy, accumulate);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_seg_mean_bwd(const float* dy, long long lddy, const int32_t* sid, const int32_t* st, const int32_t* en,
                        int T, int cols, float* dx, long long lddx, int accumulate, hipStream_t s) {
  if (T == 0 || cols == 0) return FX_OK;
  fx_launch(seg_mean_bwd_kernel, dim3(T, cdiv(cols, 256)), dim3(256), 0, s, dy, lddy, sid, st, en, T, cols,
                     dx, lddx, accumulate);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
