// X2Y attention core for a SHORT key side (X2Y_map.forward, basic.py:349-389, with X = the action
// tokens: the a2f map of UpdateBlock / UpdateBlockTDU, blocks.py:343-367 and 449-485):
//
//   logit = scale * yq . xk^T      (ny x nx, one video: nx <= 64 keys, ny up to T query rows)
//   attn  = softmax_x(logit)
//   feat  = attn . xv              (ny x Hd)
//
// as ONE launch over every video, instead of a grouped logit GEMM, a softmax launch per video and a
// grouped feat GEMM.  A workgroup (8 waves) owns 32 query rows of one video:
//   1. logits: the 32 x nx tile (<= 2 key blocks of 32) on v_mfma_f32_32x32x2_f32, the Hd-deep sum
//      split over the 8 waves (Hd / 8 each; a lane feeds 16 consecutive k of a 32-deep chunk, float4
//      loads straight from L2 -- the k order inside the sum is free as long as A and B agree), the
//      8 partial tiles summed through LDS in wave order (deterministic);
//   2. the row softmax over the nx keys in LDS; logit and attn written (the losses read both);
//   3. feat = attn . xv: 16 column tiles of 32 over Hd = 512, two per wave, K = nx from the LDS
//      probabilities (A) and xv columns (B, 32 lanes read 32 consecutive floats of one key row).
// Algorithmic bytes per 32-row workgroup: yq rows 32 Hd + feat rows 32 Hd (+ logit / attn 2 x 32 nx)
// floats; xk / xv (2 nx Hd floats per video) are L2-resident and shared by every workgroup of the video.
#include "fx_common.h"
#include "ops.h"

#include <algorithm>

namespace fx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int XR = 32;            // query rows per workgroup
constexpr int XT = 512;           // threads (8 waves)
constexpr int XMAXK = 64;         // keys per video
constexpr int LS = XMAXK + 1;     // LDS row stride of the logit / probability tile
constexpr int FX_X2Y_MAXV = 16;   // videos per launch

struct A2fArgs {
  const float* q;       // query-side rows, (Ny, Hd) ld ldq: forward yq, backward dfeat
  long long ldq;
  const float* kmat;    // (Nx, Hd) phase-1 keys: forward xk, backward xv
  const float* vmat;    // (Nx, Hd) phase-3 values: forward xv, backward xk
  const float* attn_in; // backward: the forward's attn (per video (ny_v, nx_v) at aoff[v])
  const float* add_p;   // backward: dattn, added to dP (nullable)
  const float* add_l;   // backward: the direct dlogit, added to the softmax backward (nullable)
  float* out_l;         // forward: logit; backward: dlogit
  float* out_p;         // forward: attn
  float* out_rows;      // (Ny, Hd): forward feat, backward dyq
  int Hd, nvid;
  float scale1, scale3; // forward: logit scale, 1; backward: 1, the logit scale (dyq = scale dlogit . xk)
  int yoff[FX_X2Y_MAXV + 1], xoff[FX_X2Y_MAXV + 1];
  long long aoff[FX_X2Y_MAXV + 1];
  int wg_off[FX_X2Y_MAXV + 1];    // first workgroup of each video
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// MODE 0: forward (logit, attn, feat); MODE 1: input-gradient side of the backward
//   dP = dfeat . xv^T (+ dattn);  dlogit = attn (dP - sum_x attn dP) (+ direct dlogit);  dyq = scale dlogit . xk
// (the weight-side products dxv = attn^T dfeat and dxk = scale dlogit^T yq reduce over the query rows and
// stay split-K GEMMs)
template <int MODE>
__global__ __launch_bounds__(XT) void x2y_a2f_kernel(A2fArgs a) {
  __shared__ float red[8][2][16][64];       // per-wave partial tiles (acc register r, lane)
  __shared__ float P[XR][LS];               // phase-1 tile, then probabilities / dlogit
  __shared__ float rs0[XR], rs1[XR];        // forward: row max, row sum; backward: row sum of attn dP
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  // video of this workgroup (constant indices only: the argument block stays in SGPRs)
  int v = 0;
#pragma unroll
  for (int i = 1; i < FX_X2Y_MAXV; ++i)
    if (i < a.nvid && (int)blockIdx.x >= a.wg_off[i]) v = i;
  int y0 = 0, ny = 0, x0 = 0, nx = 0, wg0 = 0;
  long long ao = 0;
#pragma unroll
  for (int i = 0; i < FX_X2Y_MAXV; ++i)
    if (i == v) {
      y0 = a.yoff[i];
      ny = a.yoff[i + 1] - a.yoff[i];
      x0 = a.xoff[i];
      nx = a.xoff[i + 1] - a.xoff[i];
      ao = a.aoff[i];
      wg0 = a.wg_off[i];
    }
  const int r0 = ((int)blockIdx.x - wg0) * XR;     // first query row (video-local)
  const int Hd = a.Hd;
  const int nkb = nx > 32 ? 2 : 1;
  const int rows = min(XR, ny - r0);

  // ---- 1. T = q . kmat^T over Hd: wave w sums k in [w Hd/8, (w+1) Hd/8) ----
  f32x16 acc[2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[c][i] = 0.f;
  {
    const int kw = Hd >> 3;
    const float* pa = a.q + (long long)(y0 + min(r0 + li, ny - 1)) * a.ldq;
    const bool aok = li < rows;
    for (int k0 = w * kw; k0 < (w + 1) * kw; k0 += 32) {
      const int kk = k0 + 16 * lh;
      float av[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 t = ld4(pa + kk + 4 * q);
        av[4 * q] = aok ? t.x : 0.f;
        av[4 * q + 1] = aok ? t.y : 0.f;
        av[4 * q + 2] = aok ? t.z : 0.f;
        av[4 * q + 3] = aok ? t.w : 0.f;
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (c < nkb) {
          const int key = c * 32 + li;
          const bool bok = key < nx;
          const float* pb = a.kmat + (long long)(x0 + min(key, nx - 1)) * Hd + kk;
          float bv[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 t = ld4(pb + 4 * q);
            bv[4 * q] = bok ? t.x : 0.f;
            bv[4 * q + 1] = bok ? t.y : 0.f;
            bv[4 * q + 2] = bok ? t.z : 0.f;
            bv[4 * q + 3] = bok ? t.w : 0.f;
          }
#pragma unroll
          for (int s = 0; s < 16; ++s) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc[c], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][c][r][lane] = acc[c][r];
  __syncthreads();
  for (int e = tid; e < 2 * 16 * 64; e += XT) {
    const int c = e >> 10, r = (e >> 6) & 15, l = e & 63;
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) sum += red[q][c][r][l];
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = c * 32 + (l & 31);
    float t = a.scale1 * sum;
    if (MODE == 1 && a.add_p && row < rows && col < nx) t += a.add_p[ao + (long long)(r0 + row) * nx + col];
    P[row][col] = t;
  }
  __syncthreads();

  // ---- 2. per row over the nx keys: 16 threads per row (row tid >> 4, columns (tid & 15) + 16 j) ----
  {
    const int row = tid >> 4, c0 = tid & 15;
    const bool rok = row < rows;
    if (MODE == 0) {
      float m = -3.0e38f;
#pragma unroll
      for (int j = 0; j < XMAXK / 16; ++j) {
        const int col = c0 + 16 * j;
        if (col < nx) m = fmaxf(m, P[row][col]);
      }
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 16));
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < XMAXK / 16; ++j) {
        const int col = c0 + 16 * j;
        if (col < nx) sum += __expf(P[row][col] - m);
      }
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 16);
      if (c0 == 0) {
        rs0[row] = m;
        rs1[row] = sum;
      }
    } else {
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < XMAXK / 16; ++j) {
        const int col = c0 + 16 * j;
        if (col < nx && rok) sum += a.attn_in[ao + (long long)(r0 + row) * nx + col] * P[row][col];
      }
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 16);
      if (c0 == 0) rs1[row] = sum;
    }
  }
  __syncthreads();
  for (int e = tid; e < XR * XMAXK; e += XT) {
    const int row = e / XMAXK, col = e - row * XMAXK;
    float p = 0.f;
    if (col < nx && row < rows) {
      const long long o = ao + (long long)(r0 + row) * nx + col;
      const float t = P[row][col];
      if (MODE == 0) {
        p = __expf(t - rs0[row]) / rs1[row];
        a.out_l[o] = t;
        a.out_p[o] = p;
      } else {
        p = a.attn_in[o] * (t - rs1[row]);
        if (a.add_l) p += a.add_l[o];
        a.out_l[o] = p;
      }
    }
    P[row][col] = p;   // (each element is read and rewritten by the same thread)
  }
  __syncthreads();

  // ---- 3. out rows = scale3 P . vmat: column tiles n0 = 32 (2 w + t), t = 0, 1 ----
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n0 = 32 * (2 * w + t);
    if (n0 >= Hd) continue;
    f32x16 f;
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = 0.f;
    for (int k0 = 0; k0 < nx; k0 += 32) {
      float bv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int key = k0 + 16 * lh + s;
        const float x = a.vmat[(long long)(x0 + min(key, nx - 1)) * Hd + n0 + li];
        bv[s] = key < nx ? x : 0.f;
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) f = __builtin_amdgcn_mfma_f32_32x32x2f32(P[li][k0 + 16 * lh + s], bv[s], f, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (row < rows) a.out_rows[(long long)(y0 + r0 + row) * Hd + n0 + li] = a.scale3 * f[r];
    }
  }
}

int launch_a2f(A2fArgs& a, int mode, const int* yoff, const int* xoff, const long long* aoff, hipStream_t s) {
  int wg = 0;
  for (int v = 0; v <= a.nvid; ++v) {
    a.yoff[v] = yoff[v];
    a.xoff[v] = xoff[v];
    a.aoff[v] = aoff[v];
    a.wg_off[v] = wg;
    if (v < a.nvid) {
      const int ny = yoff[v + 1] - yoff[v], nx = xoff[v + 1] - xoff[v];
      // an empty key side leaves no workgroup: softmax over nothing has no rows to write
      if (nx > 0) wg += (ny + XR - 1) / XR;
    }
  }
  for (int v = a.nvid + 1; v <= FX_X2Y_MAXV; ++v) a.wg_off[v] = wg;
  if (wg == 0) return FX_OK;
  if (mode == 0)
    fx_launch(x2y_a2f_kernel<0>, dim3(wg), dim3(XT), 0, s, a);
  else
    fx_launch(x2y_a2f_kernel<1>, dim3(wg), dim3(XT), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

// ---------------------------------------------------------------- long key side (the f2a map)
// X = frames (nx up to T keys), Y = the action tokens (ny <= 64 queries per video), Hd = 512:
//   chunk kernel, one workgroup per 64 keys of a video: S = scale yq . xk_chunk^T (ny x 64, the Hd-deep
//   sum split over the waves), logit written, chunk row max m_c and sum l_c = sum exp(S - m_c), the
//   partial F_c = exp(S - m_c) . xv_chunk (ny x Hd) to a workspace slab;
//   merge kernel, one workgroup per (video, query row): M = max_c m_c, L = sum_c l_c e^(m_c - M),
//   feat = sum_c e^(m_c - M) F_c / L in chunk order (deterministic), attn = exp(logit - M) / L.
// Algorithmic bytes per video: xk, xv (2 nx Hd floats) + logit / attn (2 ny nx) + feat; the slabs add
// 2 ny Hd floats per 64 keys (write + read), 1/32 of the key bytes at ny = 32.
constexpr int FC = 64;             // keys per chunk
constexpr int FMAXQ = 64;          // queries per video

struct F2aArgs {
  const float* yq;      // (Ny, Hd)
  const float* xk;      // (Nx, Hd)
  const float* xv;      // (Nx, Hd)
  float* logit;         // per video (ny_v, nx_v) at aoff[v]
  float* attn;
  float* feat;          // (Ny, Hd)
  float* part;          // (chunks, FMAXQ, Hd) partial F_c
  float* stats;         // (chunks, FMAXQ, 2): m_c, l_c
  int Hd, nvid;
  float scale;
  int yoff[FX_X2Y_MAXV + 1], xoff[FX_X2Y_MAXV + 1];
  long long aoff[FX_X2Y_MAXV + 1];
  int ch_off[FX_X2Y_MAXV + 1];    // first chunk of each video
};

__device__ __forceinline__ void f2a_video(const F2aArgs& a, int v, int& y0, int& ny, int& x0, int& nx, long long& ao,
                                          int& c0) {
#pragma unroll
  for (int i = 0; i < FX_X2Y_MAXV; ++i)
    if (i == v) {
      y0 = a.yoff[i];
      ny = a.yoff[i + 1] - a.yoff[i];
      x0 = a.xoff[i];
      nx = a.xoff[i + 1] - a.xoff[i];
      ao = a.aoff[i];
      c0 = a.ch_off[i];
    }
}

__global__ __launch_bounds__(XT) void x2y_f2a_chunk_kernel(F2aArgs a) {
  __shared__ float red[8][16][64];
  __shared__ float S[FMAXQ][FC + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  int v = 0;
#pragma unroll
  for (int i = 1; i < FX_X2Y_MAXV; ++i)
    if (i < a.nvid && (int)blockIdx.x >= a.ch_off[i]) v = i;
  int y0 = 0, ny = 0, x0 = 0, nx = 0, c0 = 0;
  long long ao = 0;
  f2a_video(a, v, y0, ny, x0, nx, ao, c0);
  const int chunk = blockIdx.x;
  const int k0c = ((int)blockIdx.x - c0) * FC;          // first key of the chunk (video-local)
  const int keys = min(FC, nx - k0c);
  const int Hd = a.Hd;
  const int nrb = ny > 32 ? 2 : 1;                      // 32-row query blocks
  const int nblk = 2 * nrb;                             // output blocks (query block, key block)
  const int wpb = 8 / nblk;                             // waves per block (4 or 2)
  const int blk = w % nblk, kpart = w / nblk;
  const int rb = blk >> 1, cb = blk & 1;

  // ---- 1. S block (rb, cb) partial over k in [kpart Hd/wpb, +Hd/wpb) ----
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  {
    const int q = rb * 32 + li, key = k0c + cb * 32 + li;
    const bool aok = q < ny, bok = cb * 32 + li < keys;
    const float* pa = a.yq + (long long)(y0 + min(q, ny - 1)) * Hd;
    const float* pb = a.xk + (long long)(x0 + min(key, nx - 1)) * Hd;
    const int kw = Hd / wpb;
    for (int k0 = kpart * kw; k0 < (kpart + 1) * kw; k0 += 32) {
      const int kk = k0 + 16 * lh;
      float av[16], bv[16];
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const float4 ta = ld4(pa + kk + 4 * qd), tb = ld4(pb + kk + 4 * qd);
        av[4 * qd] = aok ? ta.x : 0.f;
        av[4 * qd + 1] = aok ? ta.y : 0.f;
        av[4 * qd + 2] = aok ? ta.z : 0.f;
        av[4 * qd + 3] = aok ? ta.w : 0.f;
        bv[4 * qd] = bok ? tb.x : 0.f;
        bv[4 * qd + 1] = bok ? tb.y : 0.f;
        bv[4 * qd + 2] = bok ? tb.z : 0.f;
        bv[4 * qd + 3] = bok ? tb.w : 0.f;
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s2], bv[s2], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][r][lane] = acc[r];
  __syncthreads();
  for (int e = tid; e < nblk * 1024; e += XT) {
    const int b = e >> 10, r = (e >> 6) & 15, l = e & 63;
    float sum = 0.f;
    for (int p = 0; p < wpb; ++p) sum += red[p * nblk + b][r][l];
    const int row = (b >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = (b & 1) * 32 + (l & 31);
    S[row][col] = a.scale * sum;
  }
  __syncthreads();

  // ---- 2. logit out; chunk row max / sum; S <- exp(S - m) (0 outside the chunk's keys) ----
  {
    // 8 threads per query row (64 rows), 8 keys each
    const int row = tid >> 3, c8 = tid & 7;
    float m = -3.0e38f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c8 + 8 * j;
      if (col < keys) m = fmaxf(m, S[row][col]);
    }
#pragma unroll
    for (int o = 4; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 8));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c8 + 8 * j;
      const float t = S[row][col];
      if (row < ny && col < keys) a.logit[ao + (long long)row * nx + k0c + col] = t;
      const float e = col < keys ? __expf(t - m) : 0.f;
      sum += e;
      S[row][col] = e;   // (read and rewritten by the same thread)
    }
#pragma unroll
    for (int o = 4; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 8);
    if (c8 == 0 && row < ny) {
      a.stats[((long long)chunk * FMAXQ + row) * 2] = m;
      a.stats[((long long)chunk * FMAXQ + row) * 2 + 1] = sum;
    }
  }
  __syncthreads();

  // ---- 3. F_c = S . xv_chunk: (nrb x Hd/32) output tiles over the 8 waves, K = 64 keys ----
  const int ntile = nrb * (Hd >> 5);
  for (int t = w; t < ntile; t += 8) {
    const int tr = t / (Hd >> 5), n0 = (t - tr * (Hd >> 5)) * 32;
    f32x16 f;
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = 0.f;
#pragma unroll
    for (int kc = 0; kc < FC; kc += 32) {
      float bv[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int key = kc + 16 * lh + s2;
        const float x = a.xv[(long long)(x0 + min(k0c + key, nx - 1)) * Hd + n0 + li];
        bv[s2] = key < keys ? x : 0.f;
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        f = __builtin_amdgcn_mfma_f32_32x32x2f32(S[tr * 32 + li][kc + 16 * lh + s2], bv[s2], f, 0, 0, 0);
    }
    float* dst = a.part + (long long)chunk * FMAXQ * Hd;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = tr * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (row < ny) dst[(long long)row * Hd + n0 + li] = f[r];
    }
  }
}

// one workgroup per (video, query row)
__global__ __launch_bounds__(XT) void x2y_f2a_merge_kernel(F2aArgs a) {
  __shared__ float wgt[1024];
  __shared__ float ML[2];
  const int tid = threadIdx.x;
  const int v = blockIdx.y, row = blockIdx.x;
  int y0 = 0, ny = 0, x0 = 0, nx = 0, c0 = 0;
  long long ao = 0;
  f2a_video(a, v, y0, ny, x0, nx, ao, c0);
  if (row >= ny || nx == 0) return;
  const int nch = (nx + FC - 1) / FC;
  if (tid < 64) {
    // M and L over the video's chunks, one wave, fixed order per lane then a fixed shuffle tree
    float m = -3.0e38f;
    for (int c = tid; c < nch; c += 64) m = fmaxf(m, a.stats[((long long)(c0 + c) * FMAXQ + row) * 2]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float l = 0.f;
    for (int c = tid; c < nch; c += 64) {
      const float* st = a.stats + ((long long)(c0 + c) * FMAXQ + row) * 2;
      l += st[1] * __expf(st[0] - m);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) l += __shfl_xor(l, o, 64);
    if (tid == 0) {
      ML[0] = m;
      ML[1] = l;
    }
  }
  __syncthreads();
  const float M = ML[0], invL = 1.f / ML[1];
  for (int c = tid; c < nch; c += XT) wgt[c] = __expf(a.stats[((long long)(c0 + c) * FMAXQ + row) * 2] - M) * invL;
  __syncthreads();
  for (int n = tid; n < a.Hd; n += XT) {
    float acc = 0.f;
    for (int c = 0; c < nch; ++c) acc += wgt[c] * a.part[((long long)(c0 + c) * FMAXQ + row) * a.Hd + n];
    a.feat[(long long)(y0 + row) * a.Hd + n] = acc;
  }
  const long long o = ao + (long long)row * nx;
  for (int x = tid; x < nx; x += XT) a.attn[o + x] = __expf(a.logit[o + x] - M) * invL;
}

// ---------------------------------------------------------------- long key side, backward
// Input-gradient side of the f2a core (frames = keys, tokens = queries), per 64-key chunk:
//   pass 1: dP = dfeat . xv_c^T (+ dattn) -> dL (temporarily), the chunk's share of rowdot = sum_x attn dP,
//           dxv_c = attn_c^T . dfeat (complete: a key row belongs to one chunk);
//   pass 2: rowdot = sum of the video's chunk shares (fixed order), dlogit = attn (dP - rowdot) (+ direct
//           dlogit) -> dL, dxk_c = scale dlogit_c^T . yq (complete), dyq partial = scale dlogit_c . xk_c;
//   merge:  dyq = sum_c partial (chunk order).
struct F2aBwdArgs {
  const float* dfeat;   // (Ny, Hd) rows, ld ldf
  long long ldf;
  const float* attn;    // per video (ny_v, nx_v) at aoff[v]
  const float* dattn;   // nullable, same layout
  const float* dl_in;   // nullable, same layout
  const float* xv;      // (Nx, Hd)
  const float* xk;
  const float* yq;      // (Ny, Hd)
  float* dL;            // per video (ny_v, nx_v) at aoff[v]
  float* dxv;           // (Nx, Hd)
  float* dxk;
  float* dyq;           // (Ny, Hd)
  float* part;          // (chunks, FMAXQ, Hd)
  float* stats;         // (chunks, FMAXQ, 2)
  unsigned* bar;        // one-launch form: {arrivals, ..., exits at +32} of the stream's counter pool
  unsigned* status;     // caller's status word (nullable): FX_STATUS_X2Y_TIMEOUT when the barrier gives up
  unsigned spin_max;    // barrier polls before a workgroup gives up
  int Hd, nvid;
  float scale;
  int yoff[FX_X2Y_MAXV + 1], xoff[FX_X2Y_MAXV + 1];
  long long aoff[FX_X2Y_MAXV + 1];
  int ch_off[FX_X2Y_MAXV + 1];
};

// write-through (sc1) buffer access for the one-launch form's hand-off of the row-dot partials
__device__ __forceinline__ __amdgpu_buffer_rsrc_t f2a_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// Grid barrier of the one-launch form (every workgroup co-resident: the grid is capped by the occupancy
// calculator on the host): each workgroup's write-through stores acknowledged (vmcnt 0) before its arrival;
// every workgroup counts its exit, timed out or not, and the last one re-arms the slot.  Bounded spin: a
// workgroup that gives up ORs FX_STATUS_X2Y_TIMEOUT into the caller's status word (read back with the step's
// status, which fails the step and makes FusedAdam skip its update) and goes on -- never a hang
__device__ __forceinline__ void f2a_grid_sync(unsigned* bar, unsigned* status, unsigned spin_max) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned G = gridDim.x;
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned n = 0;
    bool late = false;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G) {
      if (++n >= spin_max) {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (late && status)
      __hip_atomic_fetch_or(status, (unsigned)FX_STATUS_X2Y_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned prev = __hip_atomic_fetch_add(bar + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == G - 1) {   // every workgroup is past the barrier
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void f2ab_video(const F2aBwdArgs& a, int v, int& y0, int& ny, int& x0, int& nx, long long& ao,
                                           int& c0) {
#pragma unroll
  for (int i = 0; i < FX_X2Y_MAXV; ++i)
    if (i == v) {
      y0 = a.yoff[i];
      ny = a.yoff[i + 1] - a.yoff[i];
      x0 = a.xoff[i];
      nx = a.xoff[i + 1] - a.xoff[i];
      ao = a.aoff[i];
      c0 = a.ch_off[i];
    }
}

// out[x][n] = mul sum_y L[y][x] Bm[y][n] for the chunk's keys x (rows of out), y < ny (K), n < Hd:
// (2 key tiles x Hd/32 column tiles) over the 8 waves, A = L^T from LDS, B = Bm columns (global)
__device__ __forceinline__ void keys_out(const float (*L)[FC + 1], const float* Bm, long long ldb, int ny, int keys,
                                         int Hd, float mul, float* out, int w, int li, int lh) {
  const int nct = Hd >> 5;
  for (int t = w; t < 2 * nct; t += 8) {
    const int rt = t / nct, n0 = (t - rt * nct) * 32;
    f32x16 f;
#pragma unroll
    for (int i = 0; i < 16; ++i) f[i] = 0.f;
    for (int k0 = 0; k0 < ny; k0 += 32) {
      float bv[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int y = k0 + 16 * lh + s2;
        const float x = Bm[(long long)min(y, ny - 1) * ldb + n0 + li];
        bv[s2] = y < ny ? x : 0.f;
      }
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int y = k0 + 16 * lh + s2;
        f = __builtin_amdgcn_mfma_f32_32x32x2f32(y < FMAXQ ? L[min(y, FMAXQ - 1)][rt * 32 + li] : 0.f, bv[s2], f, 0, 0,
                                                 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (row < keys) out[(long long)row * Hd + n0 + li] = mul * f[r];
    }
  }
}

// PASS 1: dP, its row-dot partials, dxv; PASS 2: dlogit, dxk, the dyq partials (reading dP back);
// PASS 3: both in one launch, dP kept in LDS, a grid barrier for the row dots in between
template <int PASS>
__global__ __launch_bounds__(XT) void x2y_f2a_bwd_kernel(F2aBwdArgs a) {
  __shared__ float red[8][16][64];
  __shared__ float S[FMAXQ][FC + 1];    // dP, then dlogit (rows = queries, cols = the chunk's keys)
  __shared__ float Pa[FMAXQ][FC + 1];   // attn of the chunk
  __shared__ float rdot[FMAXQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  int v = 0;
#pragma unroll
  for (int i = 1; i < FX_X2Y_MAXV; ++i)
    if (i < a.nvid && (int)blockIdx.x >= a.ch_off[i]) v = i;
  int y0 = 0, ny = 0, x0 = 0, nx = 0, c0 = 0;
  long long ao = 0;
  f2ab_video(a, v, y0, ny, x0, nx, ao, c0);
  const int chunk = blockIdx.x;
  const int k0c = ((int)blockIdx.x - c0) * FC;
  const int keys = min(FC, nx - k0c);
  const int Hd = a.Hd;
  // the chunk's attn (and in pass 2 its dP) into LDS, zero outside (queries < ny, keys < keys)
  for (int e = tid; e < FMAXQ * FC; e += XT) {
    const int y = e / FC, x = e - y * FC;
    const bool ok = y < ny && x < keys;
    const long long o = ao + (long long)y * nx + k0c + x;
    Pa[y][x] = ok ? a.attn[o] : 0.f;
    if (PASS == 2) S[y][x] = ok ? a.dL[o] : 0.f;
  }
  if (PASS == 2 && tid < FMAXQ) {
    const int nch = (nx + FC - 1) / FC;
    float sum = 0.f;
    if (tid < ny)
      for (int c = 0; c < nch; ++c) sum += a.stats[((long long)(c0 + c) * FMAXQ + tid) * 2];
    rdot[tid] = sum;
  }
  __syncthreads();

  if (PASS != 2) {
    // ---- dP = dfeat . xv_c^T (+ dattn): blocks (query block rb, key block cb), waves split Hd ----
    const int nrb = ny > 32 ? 2 : 1, nblk = 2 * nrb, wpb = 8 / nblk;
    const int blk = w % nblk, kpart = w / nblk, rb = blk >> 1, cb = blk & 1;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    {
      const int q = rb * 32 + li, key = k0c + cb * 32 + li;
      const bool aok = q < ny, bok = cb * 32 + li < keys;
      const float* pa = a.dfeat + (long long)(y0 + min(q, ny - 1)) * a.ldf;
      const float* pb = a.xv + (long long)(x0 + min(key, nx - 1)) * Hd;
      const int kw = Hd / wpb;
      for (int k0 = kpart * kw; k0 < (kpart + 1) * kw; k0 += 32) {
        const int kk = k0 + 16 * lh;
        float av[16], bv[16];
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const float4 ta = ld4(pa + kk + 4 * qd), tb = ld4(pb + kk + 4 * qd);
          av[4 * qd] = aok ? ta.x : 0.f;
          av[4 * qd + 1] = aok ? ta.y : 0.f;
          av[4 * qd + 2] = aok ? ta.z : 0.f;
          av[4 * qd + 3] = aok ? ta.w : 0.f;
          bv[4 * qd] = bok ? tb.x : 0.f;
          bv[4 * qd + 1] = bok ? tb.y : 0.f;
          bv[4 * qd + 2] = bok ? tb.z : 0.f;
          bv[4 * qd + 3] = bok ? tb.w : 0.f;
        }
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s2], bv[s2], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][r][lane] = acc[r];
    __syncthreads();
    for (int e = tid; e < nblk * 1024; e += XT) {
      const int b = e >> 10, r = (e >> 6) & 15, l = e & 63;
      float sum = 0.f;
      for (int p = 0; p < wpb; ++p) sum += red[p * nblk + b][r][l];
      const int row = (b >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = (b & 1) * 32 + (l & 31);
      if (a.dattn && row < ny && col < keys) sum += a.dattn[ao + (long long)row * nx + k0c + col];
      S[row][col] = sum;
    }
    __syncthreads();
    // dP out (pass 2 reads it back), the chunk's share of rowdot
    {
      const int row = tid >> 3, c8 = tid & 7;
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = c8 + 8 * j;
        if (row < ny && col < keys) {
          if (PASS == 1) a.dL[ao + (long long)row * nx + k0c + col] = S[row][col];
          part += Pa[row][col] * S[row][col];
        }
      }
#pragma unroll
      for (int o = 4; o >= 1; o >>= 1) part += __shfl_xor(part, o, 8);
      if (c8 == 0 && row < ny) {
        const long long si = ((long long)chunk * FMAXQ + row) * 2;
        if (PASS == 3) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(part), f2a_rsrc(a.stats), (int)(si * 4), 0, 16);
        else a.stats[si] = part;
      }
    }
    // dxv_c = attn_c^T . dfeat
    keys_out(Pa, a.dfeat + (long long)y0 * a.ldf, a.ldf, ny, keys, Hd, 1.f, a.dxv + (long long)(x0 + k0c) * Hd, w, li,
             lh);
  }
  if (PASS == 3) {
    // every chunk's row-dot partial written through: the row sums of this video's chunks
    f2a_grid_sync(a.bar, a.status, a.spin_max);
    if (tid < FMAXQ) {
      const int nch = (nx + FC - 1) / FC;
      float sum = 0.f;
      if (tid < ny)
        for (int c = 0; c < nch; ++c)
          sum += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              f2a_rsrc(a.stats), (int)(((long long)(c0 + c) * FMAXQ + tid) * 2 * 4), 0, 16));
      rdot[tid] = sum;
    }
    __syncthreads();
  }
  if (PASS != 1) {
    // ---- dlogit = attn (dP - rowdot) (+ direct) -> dL and LDS ----
    for (int e = tid; e < FMAXQ * FC; e += XT) {
      const int y = e / FC, x = e - y * FC;
      float d = 0.f;
      if (y < ny && x < keys) {
        const long long o = ao + (long long)y * nx + k0c + x;
        d = Pa[y][x] * (S[y][x] - rdot[y]);
        if (a.dl_in) d += a.dl_in[o];
        a.dL[o] = d;
      }
      S[y][x] = d;   // (read and rewritten by the same thread)
    }
    __syncthreads();
    // dxk_c = scale dlogit_c^T . yq
    keys_out(S, a.yq + (long long)y0 * Hd, Hd, ny, keys, Hd, a.scale, a.dxk + (long long)(x0 + k0c) * Hd, w, li, lh);
    // partial dyq_c = scale dlogit_c . xk_c: (query blocks x Hd/32) tiles, K = the chunk's keys
    const int nrb = ny > 32 ? 2 : 1;
    const int nct = Hd >> 5;
    for (int t = w; t < nrb * nct; t += 8) {
      const int tr = t / nct, n0 = (t - tr * nct) * 32;
      f32x16 f;
#pragma unroll
      for (int i = 0; i < 16; ++i) f[i] = 0.f;
#pragma unroll
      for (int kc = 0; kc < FC; kc += 32) {
        float bv[16];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) {
          const int key = kc + 16 * lh + s2;
          const float x = a.xk[(long long)(x0 + min(k0c + key, nx - 1)) * Hd + n0 + li];
          bv[s2] = key < keys ? x : 0.f;
        }
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          f = __builtin_amdgcn_mfma_f32_32x32x2f32(S[tr * 32 + li][kc + 16 * lh + s2], bv[s2], f, 0, 0, 0);
      }
      float* dst = a.part + (long long)chunk * FMAXQ * Hd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = tr * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < ny) dst[(long long)row * Hd + n0 + li] = a.scale * f[r];
      }
    }
  }
}

// dyq = sum of the chunk partials in chunk order, one workgroup per (query row, video)
__global__ __launch_bounds__(XT) void x2y_f2a_bwd_merge_kernel(F2aBwdArgs a) {
  const int v = blockIdx.y, row = blockIdx.x;
  int y0 = 0, ny = 0, x0 = 0, nx = 0, c0 = 0;
  long long ao = 0;
  f2ab_video(a, v, y0, ny, x0, nx, ao, c0);
  if (row >= ny) return;
  const int nch = (nx + FC - 1) / FC;
  for (int n = threadIdx.x; n < a.Hd; n += XT) {
    float acc = 0.f;
    for (int c = 0; c < nch; ++c) acc += a.part[((long long)(c0 + c) * FMAXQ + row) * a.Hd + n];
    a.dyq[(long long)(y0 + row) * a.Hd + n] = acc;
  }
}

}  // namespace

bool x2y_a2f_fusable(int nvid, const int* xoff, int Hd) {
  if (nvid < 1 || nvid > FX_X2Y_MAXV || Hd % 256 != 0 || Hd > XT) return false;
  for (int v = 0; v < nvid; ++v)
    if (xoff[v + 1] - xoff[v] > XMAXK) return false;
  return true;
}

int launch_x2y_a2f_fwd(const float* yq, const float* xk, const float* xv, int Hd, float scale, int nvid,
                       const int* yoff, const int* xoff, const long long* aoff, float* logit, float* attn,
                       float* feat, hipStream_t s) {
  FX_REQUIRE(x2y_a2f_fusable(nvid, xoff, Hd), "x2y a2f core: <= 64 keys per video, Hd % 256 == 0, <= 16 videos");
  A2fArgs a{};
  a.q = yq;
  a.ldq = Hd;
  a.kmat = xk;
  a.vmat = xv;
  a.out_l = logit;
  a.out_p = attn;
  a.out_rows = feat;
  a.Hd = Hd;
  a.nvid = nvid;
  a.scale1 = scale;
  a.scale3 = 1.f;
  return launch_a2f(a, 0, yoff, xoff, aoff, s);
}

int launch_x2y_a2f_bwd(const float* dfeat, long long ldf, const float* xv, const float* xk, const float* attn,
                       const float* dattn, const float* dlogit_in, int Hd, float scale, int nvid, const int* yoff,
                       const int* xoff, const long long* aoff, float* dlogit, float* dyq, hipStream_t s) {
  FX_REQUIRE(x2y_a2f_fusable(nvid, xoff, Hd), "x2y a2f core: <= 64 keys per video, Hd % 256 == 0, <= 16 videos");
  FX_REQUIRE(ldf % 4 == 0 && (reinterpret_cast<uintptr_t>(dfeat) & 15) == 0, "x2y a2f bwd: dfeat rows must be 16-B aligned");
  A2fArgs a{};
  a.q = dfeat;
  a.ldq = ldf;
  a.kmat = xv;
  a.vmat = xk;
  a.attn_in = attn;
  a.add_p = dattn;
  a.add_l = dlogit_in;
  a.out_l = dlogit;
  a.out_rows = dyq;
  a.Hd = Hd;
  a.nvid = nvid;
  a.scale1 = 1.f;
  a.scale3 = scale;
  return launch_a2f(a, 1, yoff, xoff, aoff, s);
}

// ---------------------------------------------------------------- a2f weight-side products
// dxv = attn^T dfeat and dxk = scale dlogit^T yq of every video (the products of the a2f backward that
// reduce over the query rows) in ONE launch, instead of grouped split-K GEMMs + their reduce launches:
// grid (row chunk, 32-column block of Hd, video x {dxv, dxk}); a workgroup's 4 waves each take a quarter
// of the chunk's rows (sub-chunks of 32: the P values of a row as the A operand with the key as the row
// index -- lane li reads P[r][li], 32 lanes one 128-B row slice --, the B rows likewise), summed through
// LDS in wave order; the chunks of a (video, matrix, column block) are summed in chunk order by the last
// workgroup to finish one (write-through hand-off: partials stored sc1 and acknowledged before the
// arrival, read back sc1 by the last arriver, which re-arms the counter) -- deterministic.
constexpr int DWT = 256;          // threads
constexpr int DW_MAXC = 8;        // row chunks per video
struct A2fDwArgs {
  const float* attn;              // per video (ny x nx) at aoff[v]
  const float* dl;                // dlogit, same layout
  const float* dfeat;             // (Ny, Hd) rows, ld ldf
  long long ldf;
  const float* yq;                // (Ny, Hd) rows, ld Hd
  float* dxv;                     // (Nx, Hd) rows
  float* dxk;
  float scale;
  int Hd, nvid, nchunk, crows;    // chunks per video (grid x), rows per chunk (a multiple of 128)
  float* ws;                      // partials [vid][mat][col block][chunk][64 x][32 d]
  unsigned* cnt;                  // arrival counters [vid][mat][col block]
  int yoff[FX_X2Y_MAXV + 1], xoff[FX_X2Y_MAXV + 1];
  long long aoff[FX_X2Y_MAXV + 1];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dw_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

__global__ __launch_bounds__(DWT) void x2y_a2f_dw_kernel(A2fDwArgs a) {
  __shared__ float red[4][2][16][64];
  __shared__ int last;
  const int c = blockIdx.x, cb = blockIdx.y, vid = blockIdx.z >> 1, mat = blockIdx.z & 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  int y0 = 0, ny = 0, x0 = 0, nx = 0;
  long long ao = 0;
#pragma unroll
  for (int i = 0; i < FX_X2Y_MAXV; ++i)
    if (i == vid) {
      y0 = a.yoff[i];
      ny = a.yoff[i + 1] - a.yoff[i];
      x0 = a.xoff[i];
      nx = a.xoff[i + 1] - a.xoff[i];
      ao = a.aoff[i];
    }
  if (nx <= 0 || ny <= 0) return;                     // (uniform: the whole workgroup)
  const int nch = (ny + a.crows - 1) / a.crows;       // this video's chunks
  if (c >= nch) return;
  const float* P = (mat == 0 ? a.attn : a.dl) + ao;   // (ny x nx)
  const float* B = mat == 0 ? a.dfeat : a.yq;
  const long long ldb = mat == 0 ? a.ldf : a.Hd;
  const int d0 = cb * 32;
  const int nxt = nx > 32 ? 2 : 1;
  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  // this wave's rows: [c crows + w crows/4, + crows/4) in sub-chunks of 32 (lane half lh: rows 16 lh ..
  // + 15): the P values of a row as the A operand with the key as the row index (lane li reads P[r][li],
  // 32 lanes one 128-B row slice), the B rows likewise.  (Staging the chunk through LDS first, and a
  // register double buffer over the sub-chunks, both measured slower.)
  const int wr0 = c * a.crows + w * (a.crows >> 2), wr1 = min(ny, wr0 + (a.crows >> 2));
  for (int r0 = wr0; r0 < wr1; r0 += 32) {
    float pv[2][16], bv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int r = r0 + 16 * lh + s, rc = min(r, ny - 1);
      bv[s] = B[(long long)(y0 + rc) * ldb + d0 + li];
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (t < nxt) pv[t][s] = P[(long long)rc * nx + min(32 * t + li, nx - 1)];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool rok = r0 + 16 * lh + s < wr1;
      const float b = rok ? bv[s] : 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
        if (t < nxt) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(32 * t + li < nx ? pv[t][s] : 0.f, b, acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][t][r][lane] = acc[t][r];
  __syncthreads();
  // the workgroup's tile (64 x, 32 d) summed over the waves in order; thread -> 8 elements (t, r, lane)
  const float mul = mat == 0 ? 1.f : a.scale;
  float* out = mat == 0 ? a.dxv : a.dxk;
  const long long grp = ((long long)vid * 2 + mat) * gridDim.y + cb;
  float* part = a.ws + (grp * a.nchunk + c) * 2048;
  const bool direct = nch == 1 || a.cnt == nullptr;
  float v8[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + i * DWT, t = e >> 10, r = (e >> 6) & 15, l = e & 63;
    v8[i] = (red[0][t][r][l] + red[1][t][r][l]) + (red[2][t][r][l] + red[3][t][r][l]);
    const int x = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), d = d0 + (l & 31);
    if (direct) {
      if (x < nx && t < nxt) out[(long long)(x0 + x) * a.Hd + d] = v8[i] * mul;
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v8[i]), dw_rsrc(part), e * 4, 0, 16);
    }
  }
  if (direct) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's partial stores acknowledged
  __syncthreads();
  if (tid == 0) {
    unsigned* cp = a.cnt + grp;
    const unsigned prev = __hip_atomic_fetch_add(cp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (unsigned)nch - 1;
    if (last) __hip_atomic_store(cp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  const float* pbase = a.ws + grp * a.nchunk * 2048;
  float x8[DW_MAXC][8];
#pragma unroll
  for (int q = 0; q < DW_MAXC; ++q)
#pragma unroll
    for (int i = 0; i < 8; ++i)
      x8[q][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          dw_rsrc(pbase), ((long long)min(q, nch - 1) * 2048 + tid + i * DWT) * 4, 0, 16));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = tid + i * DWT, t = e >> 10, r = (e >> 6) & 15, l = e & 63;
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < DW_MAXC; ++q)
      if (q < nch) sum += x8[q][i];
    const int x = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), d = d0 + (l & 31);
    if (x < nx && t < nxt) out[(long long)(x0 + x) * a.Hd + d] = sum * mul;
  }
}

bool x2y_a2f_dw_ok(int nvid, const int* yoff) {
  (void)yoff;   // (any row count: the chunks grow with the video)
  return nvid >= 1 && nvid <= FX_X2Y_MAXV;
}
long long x2y_a2f_dw_ws_floats(int nvid, int Hd) { return (long long)nvid * 2 * (Hd / 32) * DW_MAXC * 2048; }

int launch_x2y_a2f_dw(const float* attn, const float* dl, const float* dfeat, long long ldf, const float* yq, int Hd,
                      float scale, int nvid, const int* yoff, const int* xoff, const long long* aoff, float* dxv,
                      float* dxk, float* ws, hipStream_t s) {
  FX_REQUIRE(nvid >= 1 && nvid <= FX_X2Y_MAXV && Hd % 32 == 0, "x2y a2f dW: <= 16 videos, Hd % 32 == 0");
  A2fDwArgs a{};
  a.attn = attn;
  a.dl = dl;
  a.dfeat = dfeat;
  a.ldf = ldf;
  a.yq = yq;
  a.dxv = dxv;
  a.dxk = dxk;
  a.scale = scale;
  a.Hd = Hd;
  a.nvid = nvid;
  int nymax = 0;
  for (int v = 0; v <= nvid; ++v) {
    a.yoff[v] = yoff[v];
    a.xoff[v] = xoff[v];
    a.aoff[v] = aoff[v];
    if (v < nvid) {
      FX_REQUIRE(xoff[v + 1] - xoff[v] <= 64, "x2y a2f dW: <= 64 keys per video");
      nymax = std::max(nymax, yoff[v + 1] - yoff[v]);
    }
  }
  if (nymax == 0) return FX_OK;
  // about one workgroup per CU: chunks of a multiple of 128 rows (32 per wave), at most DW_MAXC per video
  const int ncb = Hd / 32;
  const long long groups = (long long)nvid * 2 * ncb;
  int nchunk = (int)std::max<long long>(1, std::min<long long>(DW_MAXC, (256 + groups - 1) / groups));
  int crows = (nymax + nchunk - 1) / nchunk;
  crows = (crows + 127) / 128 * 128;
  nchunk = (nymax + crows - 1) / crows;
  a.nchunk = nchunk;
  a.crows = crows;
  a.ws = ws;
  a.cnt = (nchunk > 1 && groups <= kArrivalCounters) ? arrival_counters(s) : nullptr;
  FX_REQUIRE(nchunk == 1 || (a.cnt && ws), "x2y a2f dW: workspace / counters required");
  fx_launch(x2y_a2f_dw_kernel, dim3(nchunk, ncb, 2 * nvid), dim3(DWT), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

bool x2y_f2a_fusable(int nvid, const int* xoff, const int* yoff, int Hd) {
  if (nvid < 1 || nvid > FX_X2Y_MAXV || Hd % 256 != 0 || Hd > XT) return false;
  long long nch = 0;
  for (int v = 0; v < nvid; ++v) {
    const int nxv = xoff[v + 1] - xoff[v];
    if (yoff[v + 1] - yoff[v] > FMAXQ) return false;
    nch += (nxv + FC - 1) / FC;
    if ((nxv + FC - 1) / FC > 1024) return false;     // merge weights in LDS
  }
  return nch > 0;
}

long long x2y_f2a_chunks(int nvid, const int* xoff) {
  long long nch = 0;
  for (int v = 0; v < nvid; ++v) nch += (xoff[v + 1] - xoff[v] + FC - 1) / FC;
  return nch;
}

long long x2y_f2a_ws_floats(int nvid, const int* xoff, int Hd) {
  long long nch = 0;
  for (int v = 0; v < nvid; ++v) nch += (xoff[v + 1] - xoff[v] + FC - 1) / FC;
  return nch * FMAXQ * ((long long)Hd + 2);
}

int launch_x2y_f2a_fwd(const float* yq, const float* xk, const float* xv, int Hd, float scale, int nvid,
                       const int* yoff, const int* xoff, const long long* aoff, float* logit, float* attn,
                       float* feat, float* ws, hipStream_t s) {
  FX_REQUIRE(x2y_f2a_fusable(nvid, xoff, yoff, Hd), "x2y f2a core: <= 64 queries per video, Hd % 256 == 0");
  F2aArgs a{};
  a.yq = yq;
  a.xk = xk;
  a.xv = xv;
  a.logit = logit;
  a.attn = attn;
  a.feat = feat;
  a.Hd = Hd;
  a.nvid = nvid;
  a.scale = scale;
  int nch = 0, maxq = 0;
  for (int v = 0; v <= nvid; ++v) {
    a.yoff[v] = yoff[v];
    a.xoff[v] = xoff[v];
    a.aoff[v] = aoff[v];
    a.ch_off[v] = nch;
    if (v < nvid) {
      nch += (xoff[v + 1] - xoff[v] + FC - 1) / FC;
      maxq = std::max(maxq, yoff[v + 1] - yoff[v]);
    }
  }
  for (int v = nvid + 1; v <= FX_X2Y_MAXV; ++v) a.ch_off[v] = nch;
  a.part = ws;
  a.stats = ws + (long long)nch * FMAXQ * Hd;
  if (nch == 0 || maxq == 0) return FX_OK;
  fx_launch(x2y_f2a_chunk_kernel, dim3(nch), dim3(XT), 0, s, a);
  fx_launch(x2y_f2a_merge_kernel, dim3(maxq, nvid), dim3(XT), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_x2y_f2a_bwd(const float* dfeat, long long ldf, const float* xv, const float* xk, const float* yq,
                       const float* attn, const float* dattn, const float* dlogit_in, int Hd, float scale, int nvid,
                       const int* yoff, const int* xoff, const long long* aoff, float* dlogit, float* dxv, float* dxk,
                       float* dyq, float* ws, unsigned* status, hipStream_t s) {
  FX_REQUIRE(x2y_f2a_fusable(nvid, xoff, yoff, Hd), "x2y f2a core: <= 64 queries per video, Hd % 256 == 0");
  FX_REQUIRE(ldf % 4 == 0 && (reinterpret_cast<uintptr_t>(dfeat) & 15) == 0, "x2y f2a bwd: dfeat rows must be 16-B aligned");
  F2aBwdArgs a{};
  a.dfeat = dfeat;
  a.ldf = ldf;
  a.attn = attn;
  a.dattn = dattn;
  a.dl_in = dlogit_in;
  a.xv = xv;
  a.xk = xk;
  a.yq = yq;
  a.dL = dlogit;
  a.dxv = dxv;
  a.dxk = dxk;
  a.dyq = dyq;
  a.Hd = Hd;
  a.nvid = nvid;
  a.scale = scale;
  int nch = 0, maxq = 0;
  for (int v = 0; v <= nvid; ++v) {
    a.yoff[v] = yoff[v];
    a.xoff[v] = xoff[v];
    a.aoff[v] = aoff[v];
    a.ch_off[v] = nch;
    if (v < nvid) {
      nch += (xoff[v + 1] - xoff[v] + FC - 1) / FC;
      maxq = std::max(maxq, yoff[v + 1] - yoff[v]);
    }
  }
  for (int v = nvid + 1; v <= FX_X2Y_MAXV; ++v) a.ch_off[v] = nch;
  a.part = ws;
  a.stats = ws + (long long)nch * FMAXQ * Hd;
  if (nch == 0 || maxq == 0) return FX_OK;
  // one launch when every chunk's workgroup can be resident at once (the grid barrier waits for all of
  // them): the occupancy calculator's bound for this kernel on this device (CU count x workgroups per CU);
  // FX_X2Y_F2A_ONE=0 keeps the two launches (A/B)
  a.status = status;
  a.spin_max = x2y_spin_max();
  const int resident = coresident_blocks((const void*)x2y_f2a_bwd_kernel<3>, XT, 0);
  a.bar = (knobs().x2y_f2a_one && nch <= resident) ? arrival_counters(s) : nullptr;
  if (a.bar) {
    fx_launch(x2y_f2a_bwd_kernel<3>, dim3(nch), dim3(XT), 0, s, a);
  } else {
    fx_launch(x2y_f2a_bwd_kernel<1>, dim3(nch), dim3(XT), 0, s, a);
    fx_launch(x2y_f2a_bwd_kernel<2>, dim3(nch), dim3(XT), 0, s, a);
  }
  fx_launch(x2y_f2a_bwd_merge_kernel, dim3(maxq, nvid), dim3(XT), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
