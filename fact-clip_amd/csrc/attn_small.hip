// Fused multi-head attention for token-sized problems (Lq, Lk, head_dim <= 64): the
// nn.MultiheadAttention core of SALayer / SCALayer's self-attention over the Q = Nact action
// tokens (basic.py:442, 500).  One workgroup per head holds Q_h, K_h, V_h, P_h in LDS, so the
// whole forward (S = scale * Q K^T, row softmax, O = P V) or backward (dP = dO V^T,
// dS = P * (dP - rowsum(P * dP)), dQ = scale dS K, dK = scale dS^T Q, dV = P^T dO) is ONE launch
// instead of three batched GEMMs + a softmax (+ split-K reduces).  At 32 x 32 x 32 per head the
// work is ~100 k FMAs per workgroup: latency-bound, so plain fp32 FMAs from LDS (exact f32
// products like the reference CPU path), no MFMA tiling.
#include <algorithm>
#include <cmath>

#include "fx_common.h"
#include "ops.h"

namespace fx {
namespace {

constexpr int SM = 64;        // max Lq, Lk, head_dim
constexpr int SP = SM + 1;    // padded LDS row stride (no bank conflicts on column walks)
// 1024 threads: each output element is one thread's serial FMA chain (fixed order, so the result does
// not depend on NT); at Breakfast's 60 tokens x head dim 64 a 256-thread block left each thread ~15
// elements of 64-deep chains (bwd 72 us per launch over only heads x videos = 32 workgroups)
constexpr int NT = 1024;

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

// keep-scale of probability (head h, query i, key j) of video vid: 1/(1-p) or 0 -- the attention-over-T
// kernels' mask (attn_t.hip drop_keep) with global query row vid*Lq+i and key row vid*Lk+j
__device__ __forceinline__ float keep_scale(unsigned long long seed, unsigned thr, float p, int vid, int nvid, int nh,
                                            int h, int Lq, int Lk, int i, int j) {
  const unsigned long long qg = (unsigned long long)vid * Lq + i, kg = (unsigned long long)vid * Lk + j;
  const unsigned long long idx = (qg * nh + h) * ((unsigned long long)nvid * Lk) + kg;
  return fx_drop_bits(seed, idx) >= thr ? 1.f / (1.f - p) : 0.f;
}

__device__ __forceinline__ void load_tile(float (*dst)[SP], const float* src, long long ld, int rows, int cols) {
  for (int e = threadIdx.x; e < rows * cols; e += NT) {
    const int r = e / cols, c = e - r * cols;
    dst[r][c] = src[(long long)r * ld + c];
  }
}

__global__ __launch_bounds__(NT) void mha_small_fwd_kernel(const float* q, long long ldq, const float* k,
                                                           long long ldk, const float* v, long long ldv, int Lq,
                                                           int Lk, int hd, float scale, float* probs, float* o,
                                                           long long ldo, float drop_p, unsigned thr,
                                                           unsigned long long seed) {
  __shared__ float Qs[SM][SP], Ks[SM][SP], Vs[SM][SP], Ps[SM][SP];
  const int h = blockIdx.x, vid = blockIdx.y;   // head, video (rows vid*Lq.. of q/o, vid*Lk.. of k/v)
  q += (long long)vid * Lq * ldq;
  k += (long long)vid * Lk * ldk;
  v += (long long)vid * Lk * ldv;
  o += (long long)vid * Lq * ldo;
  probs += (long long)vid * gridDim.x * Lq * Lk;
  load_tile(Qs, q + h * hd, ldq, Lq, hd);
  load_tile(Ks, k + h * hd, ldk, Lk, hd);
  load_tile(Vs, v + h * hd, ldv, Lk, hd);
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * Lk; e += NT) {
    const int i = e / Lk, j = e - i * Lk;
    float acc = 0.f;
    for (int d = 0; d < hd; ++d) acc += Qs[i][d] * Ks[j][d];
    Ps[i][j] = acc * scale;
  }
  __syncthreads();
  // row softmax: one wave per row
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < Lq; i += NT / 64) {
    const float x = lane < Lk ? Ps[i][lane] : -INFINITY;
    const float m = wmax(x);
    const float ex = lane < Lk ? __expf(x - m) : 0.f;
    const float p = ex / wsum(ex);
    if (lane < Lk) {
      probs[((long long)h * Lq + i) * Lk + lane] = p;   // saved before dropout (backward recomputes the mask)
      Ps[i][lane] = drop_p > 0.f ? p * keep_scale(seed, thr, drop_p, vid, gridDim.y, gridDim.x, h, Lq, Lk, i, lane) : p;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Lq * hd; e += NT) {
    const int i = e / hd, d = e - i * hd;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc += Ps[i][j] * Vs[j][d];
    o[(long long)i * ldo + h * hd + d] = acc;
  }
}

__global__ __launch_bounds__(NT) void mha_small_bwd_kernel(const float* q, long long ldq, const float* k,
                                                           long long ldk, const float* v, long long ldv,
                                                           const float* probs, const float* dout, long long lddo,
                                                           int Lq, int Lk, int hd, float scale, float* dq,
                                                           long long lddq, float* dk, long long lddk, float* dv,
                                                           long long lddv, float drop_p, unsigned thr,
                                                           unsigned long long seed) {
  __shared__ float Qs[SM][SP], Ks[SM][SP], Vs[SM][SP], Ps[SM][SP], Ds[SM][SP], Gs[SM][SP];
  __shared__ float Ms[SM][SP];   // dropout keep-scales (training only)
  const int h = blockIdx.x, vid = blockIdx.y;
  q += (long long)vid * Lq * ldq;
  k += (long long)vid * Lk * ldk;
  v += (long long)vid * Lk * ldv;
  probs += (long long)vid * gridDim.x * Lq * Lk;
  dout += (long long)vid * Lq * lddo;
  if (dq) dq += (long long)vid * Lq * lddq;
  if (dk) dk += (long long)vid * Lk * lddk;
  if (dv) dv += (long long)vid * Lk * lddv;
  load_tile(Qs, q + h * hd, ldq, Lq, hd);
  load_tile(Ks, k + h * hd, ldk, Lk, hd);
  load_tile(Vs, v + h * hd, ldv, Lk, hd);
  load_tile(Ps, probs + (long long)h * Lq * Lk, Lk, Lq, Lk);
  load_tile(Ds, dout + h * hd, lddo, Lq, hd);   // dO_h
  const bool drop = drop_p > 0.f;
  if (drop)
    for (int e = threadIdx.x; e < Lq * Lk; e += NT) {
      const int i = e / Lk, j = e - i * Lk;
      Ms[i][j] = keep_scale(seed, thr, drop_p, vid, gridDim.y, gridDim.x, h, Lq, Lk, i, j);
    }
  __syncthreads();
  // dP = dO V^T  -> Gs
  for (int e = threadIdx.x; e < Lq * Lk; e += NT) {
    const int i = e / Lk, j = e - i * Lk;
    float acc = 0.f;
    for (int d = 0; d < hd; ++d) acc += Ds[i][d] * Vs[j][d];
    Gs[i][j] = drop ? acc * Ms[i][j] : acc;   // gradient of the un-dropped P
  }
  __syncthreads();
  // dV = P_d^T dO with P_d the dropped probabilities (uses Ps, Ds before they are overwritten)
  if (dv)
    for (int e = threadIdx.x; e < Lk * hd; e += NT) {
      const int j = e / hd, d = e - j * hd;
      float acc = 0.f;
      if (drop)
        for (int i = 0; i < Lq; ++i) acc += Ps[i][j] * Ms[i][j] * Ds[i][d];
      else
        for (int i = 0; i < Lq; ++i) acc += Ps[i][j] * Ds[i][d];
      dv[(long long)j * lddv + h * hd + d] = acc;
    }
  // dS = P * (dP - rowsum(P dP)), one wave per row, in place in Gs
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < Lq; i += NT / 64) {
    const float p = lane < Lk ? Ps[i][lane] : 0.f;
    const float g = lane < Lk ? Gs[i][lane] : 0.f;
    const float r = wsum(p * g);
    if (lane < Lk) Gs[i][lane] = p * (g - r);
  }
  __syncthreads();
  if (dq)
    for (int e = threadIdx.x; e < Lq * hd; e += NT) {
      const int i = e / hd, d = e - i * hd;
      float acc = 0.f;
      for (int j = 0; j < Lk; ++j) acc += Gs[i][j] * Ks[j][d];
      dq[(long long)i * lddq + h * hd + d] = acc * scale;
    }
  if (dk)
    for (int e = threadIdx.x; e < Lk * hd; e += NT) {
      const int j = e / hd, d = e - j * hd;
      float acc = 0.f;
      for (int i = 0; i < Lq; ++i) acc += Gs[i][j] * Qs[i][d];
      dk[(long long)j * lddk + h * hd + d] = acc * scale;
    }
}

}  // namespace

int launch_mha_small_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                         int Lq, int Lk, int hd, int nhead, float scale, float* probs, float* o, long long ldo,
                         hipStream_t s, int nvid, float drop_p, unsigned long long seed) {
  FX_REQUIRE(Lq > 0 && Lk > 0 && hd > 0 && Lq <= SM && Lk <= SM && hd <= SM && nhead > 0,
             "mha_small: Lq, Lk, head_dim must be in [1, 64]");
  FX_REQUIRE(nvid >= 1, "mha_small: nvid >= 1");
  FX_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "mha_small: dropout p in [0, 1)");
  const unsigned thr = drop_p > 0.f ? std::max(fx_drop_thresh(drop_p), 1u) : 0u;
  fx_launch(mha_small_fwd_kernel, dim3(nhead, nvid), dim3(NT), 0, s, q, ldq, k, ldk, v, ldv, Lq, Lk, hd, scale,
                     probs, o, ldo, drop_p, thr, seed);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_mha_small_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                         const float* probs, const float* dout, long long lddo, int Lq, int Lk, int hd, int nhead,
                         float scale, float* dq, long long lddq, float* dk, long long lddk, float* dv, long long lddv,
                         hipStream_t s, int nvid, float drop_p, unsigned long long seed) {
  FX_REQUIRE(Lq > 0 && Lk > 0 && hd > 0 && Lq <= SM && Lk <= SM && hd <= SM && nhead > 0,
             "mha_small: Lq, Lk, head_dim must be in [1, 64]");
  FX_REQUIRE(nvid >= 1, "mha_small: nvid >= 1");
  FX_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "mha_small: dropout p in [0, 1)");
  const unsigned thr = drop_p > 0.f ? std::max(fx_drop_thresh(drop_p), 1u) : 0u;
  fx_launch(mha_small_bwd_kernel, dim3(nhead, nvid), dim3(NT), 0, s, q, ldq, k, ldk, v, ldv, probs, dout, lddo,
                     Lq, Lk, hd, scale, dq, lddq, dk, lddk, dv, lddv, drop_p, thr, seed);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
