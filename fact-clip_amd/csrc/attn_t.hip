// Multi-head attention of a few queries over T frames, fused (SCALayer cross-attention,
// basic.py:508-516: nn.MultiheadAttention with Q = Nact action tokens, K/V = T frames, 8 heads).
//
// The reference runs it as ATen bmm -> softmax -> (dropout) -> bmm and keeps the (h, Q, T)
// probabilities for backward; round 1 here was the same three GEMM/softmax launches (+ a split-K
// reduce) per video.  Here ONE launch covers every video and head, flash-decoding style:
//   grid = (T-chunk c, head h, video v); a workgroup stages q_h (Q x hd), K_c and V_c (Tc x hd) in
//   LDS, computes S = q K_c^T (MFMA 32x32x2 f32), its row max m_c / sum l_c, and O_c = exp(S - m_c) V_c;
//   the partials go to a workspace and a second, small launch (tattn_merge_kernel, one workgroup per
//   (video, head)) merges them in chunk order -- deterministic -- into o = sum_c e^(m_c - M) O_c / L
//   and lse = M + log L.  (An in-launch last-arriver merge behind an arrival counter measured slower:
//   the agent-scope release / acquire hand-off costs more than the second launch)
//   Only lse (Q floats per head) is kept for backward, not the probabilities.
// Backward recomputes P = exp(S - lse) per chunk: dV_c = P^T dO, dP = dO V_c^T, dS = P (dP - D)
// with D = rowsum(dO o), dK_c = scale dS^T q (K/V rows of a chunk belong to ONE workgroup: written,
// not accumulated), and dq = scale sum_c dS_c K_c through the same ordered merge launch.
// HBM bytes per frame and layer: K and V rows read once (2 hd h x 4 B per frame forward; backward
// also writes dK, dV).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <string>

#include "fx_common.h"
#include "ops.h"

namespace fx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int AT = 256;   // threads per workgroup (4 waves)

// Diagnostic builds (-DFX_STAMPS, libfactmx_stamps.so) stamp s_memtime at fixed points of every
// workgroup into a buffer set by fx_dbg_tattn_stamps(); the shipped library compiles them away.
#ifdef FX_STAMPS
__device__ long long* g_tattn_stamps;
#define TSTAMP(slot)                                                                                       \
  do {                                                                                                   \
    if (g_tattn_stamps && threadIdx.x == 0) {                                                            \
      const long long _b = ((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;      \
      g_tattn_stamps[_b * 8 + (slot)] = __builtin_amdgcn_s_memtime();                                    \
    }                                                                                                    \
  } while (0)
#else
#define TSTAMP(slot) \
  do {               \
  } while (0)
#endif

// acc (32x32) += A (32 x K) . B (K x 32), operands in LDS.
//   A element (r, k) = ATR ? a[k*lda + r] : a[r*lda + k]
//   B element (k, c) = BTR ? b[c*ldb + k] : b[k*ldb + c]
// K even; lane half hh takes k in [hh*K/2, hh*K/2 + K/2) -- any k order works as long as A and B agree.
// Strides are odd (row length + 1) so the 32 lanes of a half hit 32 different banks.
template <bool ATR, bool BTR>
__device__ __forceinline__ void mm32(const float* a, int lda, const float* b, int ldb, int K, f32x16& acc, int lane) {
  // K % 8 == 0 (every caller).  Software-pipelined: the LDS reads of the next 4 k-steps are issued
  // before the MFMAs of the current 4.
  const int li = lane & 31, kh = (lane >> 5) * (K >> 1);
  float av[4], bv[4];
  auto ld4 = [&](int j0, float* x, float* y) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kh + j0 + j;
      x[j] = ATR ? a[k * lda + li] : a[li * lda + k];
      y[j] = BTR ? b[li * ldb + k] : b[k * ldb + li];
    }
  };
  ld4(0, av, bv);
  for (int j0 = 0; j0 < (K >> 1); j0 += 4) {
    float an[4], bn[4];
    if (j0 + 4 < (K >> 1)) ld4(j0 + 4, an, bn);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bv[j], acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      av[j] = an[j];
      bv[j] = bn[j];
    }
  }
}

// The same product with A row-major (k contiguous per row) read as ds_read_b128: a lane half's k range is
// contiguous, so one 16-B read feeds 4 MFMAs.  B: BTR -> also contiguous k (b128); else b[k*ldb + c] (b32).
// lda (and ldb for BTR) = row length + 4: 16-B aligned rows, conflict-free b128 lane groups.
template <bool BTR>
__device__ __forceinline__ void mm32v(const float* a, int lda, const float* b, int ldb, int K, f32x16& acc, int lane) {
  const int li = lane & 31, kh = (lane >> 5) * (K >> 1);
  const float* pa = a + li * lda + kh;
  const float* pb = BTR ? b + li * ldb + kh : b + kh * ldb + li;
  auto ldb4 = [&](int j0) {
    if (BTR) return *reinterpret_cast<const float4*>(pb + j0);
    return make_float4(pb[j0 * ldb], pb[(j0 + 1) * ldb], pb[(j0 + 2) * ldb], pb[(j0 + 3) * ldb]);
  };
  float4 av = *reinterpret_cast<const float4*>(pa), bv = ldb4(0);
  for (int j0 = 0; j0 < (K >> 1); j0 += 4) {
    float4 an = av, bn = bv;
    if (j0 + 4 < (K >> 1)) {
      an = *reinterpret_cast<const float4*>(pa + j0 + 4);
      bn = ldb4(j0 + 4);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc, 0, 0, 0);
    av = an;
    bv = bn;
  }
}

__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 0.f;
}

// accumulator element r of a lane: row (r&3) + 8 (r>>2) + 4 (lane>>5), column lane&31
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

constexpr int MAXV = 32;  // videos per launch (per-video key row offsets live in the kernel arguments)

struct TAttnArgs {
  const float* q; long long ldq;
  const float* k; long long ldk;
  const float* v; long long ldv;
  const float* o; long long ldo;        // bwd: forward output
  const float* dout; long long lddo;    // bwd
  float* out; long long ld_out;         // fwd: o;  bwd: dq
  float* dk; long long lddk;            // bwd
  float* dv; long long lddv;            // bwd
  float* lse;                           // (nvid, h, qs): fwd writes, bwd reads
  float* ws;                            // partials
  int Qv, hd, nh, Qp, Hp, Tc, nsplit;   // Qv: queries of this block; nsplit: max chunks over the videos
  int qs, q0;                           // query rows per video (q / o / lse stride), first query of the block
  int acc_kv;                           // bwd: dK / dV += (later query blocks of the same keys)
  float scale;
  int vec;                              // 16-B loads of every q / k / v / o / dout row slice
  float drop_p;                         // attention-probability dropout (training), counter-based mask
  unsigned drop_thr;
  unsigned long long drop_seed;
  long long ktot;                       // key rows over all videos (mask index stride)
  unsigned* cnt;                        // register-resident kernels: arrival counters per (video, head) for the
                                        // in-launch merge (null: partials for tattn_merge_kernel)
  int koff[MAXV + 1];                   // key / value rows of video v: [koff[v], koff[v+1])
};

// keep-scale of probability (global query row qg, head h, global key row kg): 1/(1-p) or 0
__device__ __forceinline__ float drop_keep(const TAttnArgs& a, long long qg, int h, long long kg) {
  const unsigned long long idx = ((unsigned long long)qg * a.nh + h) * (unsigned long long)a.ktot + kg;
  return fx_drop_bits(a.drop_seed, idx) >= a.drop_thr ? 1.f / (1.f - a.drop_p) : 0.f;
}

// Strips of row-major sources staged into LDS images (row stride ld, zero outside the `nvalid` rows and
// `hd` columns).  Every load of a workgroup's strips is issued before the first LDS store (a store
// behind its own load would serialise the strips on the memory latency): float4 loads when every row
// slice is 16-B aligned, up to NV float4 per thread and strip.
template <int NV>
struct Strip {
  float4 v[NV];
  __device__ __forceinline__ void load(int rows, int cols, const float* src, long long lds_, int nvalid, int hd,
                                       int tid) {
    const int c4 = cols >> 2, total = rows * c4;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + i * AT;
      const int r = e / c4, c = (e - r * c4) * 4;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < total && r < nvalid && c < hd) x = *reinterpret_cast<const float4*>(src + (long long)r * lds_ + c);
      v[i] = x;
    }
  }
  __device__ __forceinline__ void store(float* img, int ld, int rows, int cols, int tid) const {
    const int c4 = cols >> 2, total = rows * c4;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + i * AT;
      if (e < total) {
        const int r = e / c4, c = (e - r * c4) * 4;
        float* d = img + r * ld + c;
        d[0] = v[i].x;
        d[1] = v[i].y;
        d[2] = v[i].z;
        d[3] = v[i].w;
      }
    }
  }
};
constexpr int NVQ = 4;    // q / o / dout strips: <= 64 x 64 floats
constexpr int NVK = 8;    // K / V chunks: <= 8192 floats (the host keeps Tc * Hp within it)

// element-wise fallback for unaligned / odd-width slices
__device__ __forceinline__ void stage_scalar(float* img, int ld, int rows, int cols, const float* src, long long lds_,
                                             int nvalid, int hd, int tid) {
  for (int e = tid; e < rows * cols; e += AT) {
    const int r = e / cols, c = e - r * cols;
    img[r * ld + c] = (r < nvalid && c < hd) ? src[(long long)r * lds_ + c] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------ forward
// grid (chunk, head, video).  nsplit == 1: o and lse directly; else the chunk's partial
// O_c = e^(S - m_c) V_c (Qp x Hp) and its row stats (m_c, l_c) go to the workspace for tattn_merge.
__global__ __launch_bounds__(AT) void tattn_fwd_kernel(TAttnArgs a) {
  extern __shared__ float sm[];
  const int c = blockIdx.x, h = blockIdx.y, vid = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Qp = a.Qp, Hp = a.Hp, Tc = a.Tc, hd = a.hd;
  const int lq = Hp + 4, lk = Hp + 4, ls = Tc + 4;   // 16-B aligned rows (b128 operand reads)
  float* qs = sm;                       // [Qp][lq]
  float* ks = qs + Qp * lq;             // [Tc][lk]
  float* vs = ks + Tc * lk;             // [Tc][lk]
  float* ss = vs + Tc * lk;             // [Qp][ls]
  float* red = ss + Qp * ls;            // [4][1024] wave partials
  float* rowm = red + 4 * 1024;         // [Qp]
  float* rowl = rowm + Qp;              // [Qp]
  const int Tv = a.koff[vid + 1] - a.koff[vid];
  const int t0 = c * Tc, nk = min(Tc, Tv - t0);
  if (nk <= 0) return;                  // a shorter video of a ragged batch has fewer chunks
  const long long qrow = (long long)vid * a.qs + a.q0, krow = (long long)a.koff[vid] + t0;
  const float* qsrc = a.q + qrow * a.ldq + h * hd;
  const float* ksrc = a.k + krow * a.ldk + h * hd;
  const float* vsrc = a.v + krow * a.ldv + h * hd;
  TSTAMP(0);
  if (a.vec) {
    Strip<NVQ> sq;
    Strip<NVK> sk, sv;
    sq.load(Qp, Hp, qsrc, a.ldq, a.Qv, hd, tid);
    sk.load(Tc, Hp, ksrc, a.ldk, nk, hd, tid);
    sv.load(Tc, Hp, vsrc, a.ldv, nk, hd, tid);
    sq.store(qs, lq, Qp, Hp, tid);
    sk.store(ks, lk, Tc, Hp, tid);
    sv.store(vs, lk, Tc, Hp, tid);
  } else {
    stage_scalar(qs, lq, Qp, Hp, qsrc, a.ldq, a.Qv, hd, tid);
    stage_scalar(ks, lk, Tc, Hp, ksrc, a.ldk, nk, hd, tid);
    stage_scalar(vs, lk, Tc, Hp, vsrc, a.ldv, nk, hd, tid);
  }
  __syncthreads();
  TSTAMP(1);
  // S^T tiles (keys x queries) = scale K q^T kept in registers: wave w takes tiles w and w + 4 of the
  // (key tile, query tile) grid -- both in query tile w % nrt -- and a lane holds 16 keys of ONE query
  // column, so the softmax statistics are in-register reductions, one exchange with the other lane
  // half and one pass through LDS across the waves.  Keys past the video: -inf.
  const int nrt = Qp / 32, nct = Tc / 32;
  const int qtw = wave % nrt;
  const int myq = qtw * 32 + (lane & 31);
  f32x16 st[2];
  bool has[2];
  float lm = -INFINITY;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = wave + 4 * u;
    has[u] = t < nrt * nct;
    zero16(st[u]);
    if (has[u]) {
      const int kt = t / nrt;
      mm32v<true>(ks + kt * 32 * lk, lk, qs + qtw * 32 * lq, lq, Hp, st[u], lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + acc_row(r, lane);
        st[u][r] = key < nk ? st[u][r] * a.scale : -INFINITY;
        lm = fmaxf(lm, st[u][r]);
      }
    }
  }
  TSTAMP(2);
  float* wmax = red;              // [4][Qp]: per-wave maxima (-inf where the wave has no keys of a query)
  float* wsum = red + 4 * Qp;     // [4][Qp]: per-wave sums
  lm = fmaxf(lm, __shfl_xor(lm, 32, 64));
  if (lane < Qp) wmax[wave * Qp + lane] = (has[0] && (lane >> 5) == qtw) ? lm : -INFINITY;
  __syncthreads();
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < 4; ++w) M = fmaxf(M, wmax[w * Qp + myq]);
  float ls_ = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!has[u]) continue;
    const int kt = (wave + 4 * u) / nrt;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __expf(st[u][r] - M);
      ls_ += p;                                          // the softmax normaliser sees every key
      const int key = kt * 32 + acc_row(r, lane);
      const float kp = (a.drop_p > 0.f && key < nk) ? drop_keep(a, qrow + myq, h, krow + key) : 1.f;
      ss[myq * ls + key] = p * kp;                       // (dropped) P image [query][key] for P V
    }
  }
  ls_ += __shfl_xor(ls_, 32, 64);
  if (lane < Qp) wsum[wave * Qp + lane] = (has[0] && (lane >> 5) == qtw) ? ls_ : 0.f;
  __syncthreads();
  if (wave < nrt && lane < 32) {
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) L += wsum[w * Qp + myq];
    rowm[myq] = M;
    rowl[myq] = L;
  }
  __syncthreads();
  TSTAMP(3);
  // O_c = P V: nt output tiles, each split over wpt waves along the chunk
  const int nht = Hp / 32, nt = nrt * nht, wpt = 4 / nt;
  const int tile = wave / wpt, part = wave - tile * wpt;
  const int dlen = Tc / wpt, d0 = part * dlen;
  const int rt = tile / nht, ht = tile - rt * nht;
  f32x16 acc;
  zero16(acc);
  mm32v<false>(ss + rt * 32 * ls + d0, ls, vs + d0 * lk + ht * 32, lk, dlen, acc, lane);
  if (wpt > 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave * 1024 + r * 64 + lane] = acc[r];
    __syncthreads();
    if (part == 0)
      for (int q = 1; q < wpt; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += red[(wave + q) * 1024 + r * 64 + lane];
  }
  const long long pid = ((long long)vid * a.nh + h) * a.nsplit + c;   // partial index
  if (part == 0) {
    const int col = ht * 32 + (lane & 31);
    if (a.nsplit == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + acc_row(r, lane);
        if (row < a.Qv && col < hd) a.out[(qrow + row) * a.ld_out + h * hd + col] = acc[r] / rowl[row];
      }
    } else {
      float* po = a.ws + pid * Qp * Hp;
#pragma unroll
      for (int r = 0; r < 16; ++r) po[(rt * 32 + acc_row(r, lane)) * Hp + col] = acc[r];
    }
  }
  if (a.nsplit == 1) {
    for (int r = tid; r < a.Qv; r += AT)
      a.lse[((long long)vid * a.nh + h) * a.qs + a.q0 + r] = rowm[r] + __logf(rowl[r]);
    return;
  }
  float* pm = a.ws + (long long)gridDim.z * a.nh * a.nsplit * Qp * Hp;   // m partials, then l partials
  float* pl = pm + (long long)gridDim.z * a.nh * a.nsplit * Qp;
  for (int r = tid; r < Qp; r += AT) {
    pm[pid * Qp + r] = rowm[r];
    pl[pid * Qp + r] = rowl[r];
  }
  TSTAMP(4);
}

// Ordered merge of the nsplit partials of one (video, head) per workgroup, chunk order fixed
// (deterministic).  Forward (stats != 0): w_s(r) = e^(m_s - M) / L, o = sum_s w_s O_s, lse = M + log L;
// backward: dq = scale * sum_s dq_s.  A thread owns 4 consecutive columns of a row with 16 splits'
// float4 loads in flight.
__device__ void tattn_merge(const TAttnArgs& a, int h, int vid, int nvid, int stats, float mul, float* sm) {
  const int tid = threadIdx.x;
  const int Qp = a.Qp, Hp = a.Hp, hd = a.hd, nsm = a.nsplit;
  const int ns = (a.koff[vid + 1] - a.koff[vid] + a.Tc - 1) / a.Tc;   // this video's chunks
  const long long pbase = ((long long)vid * a.nh + h) * nsm;
  const float* part = a.ws + pbase * Qp * Hp;
  float* w = sm;                         // [ns][Qp] weights
  float* wl = sm + ns * Qp;              // [ns][Qp] l partials
  if (stats) {
    const float* pm = a.ws + (long long)nvid * a.nh * nsm * Qp * Hp + pbase * Qp;
    const float* pl = pm + (long long)nvid * a.nh * nsm * Qp;
    for (int e = tid; e < ns * Qp; e += AT) {
      w[e] = pm[e];
      wl[e] = pl[e];
    }
    __syncthreads();
    for (int r = tid; r < Qp; r += AT) {
      float M = -INFINITY;
      for (int sp = 0; sp < ns; ++sp) M = fmaxf(M, w[sp * Qp + r]);
      float L = 0.f;
      for (int sp = 0; sp < ns; ++sp) L += __expf(w[sp * Qp + r] - M) * wl[sp * Qp + r];
      const float inv = 1.f / L;
      for (int sp = 0; sp < ns; ++sp) w[sp * Qp + r] = __expf(w[sp * Qp + r] - M) * inv;
      if (r < a.Qv) a.lse[((long long)vid * a.nh + h) * a.qs + a.q0 + r] = M + __logf(L);
    }
    __syncthreads();
  }
  float* out = a.out + ((long long)vid * a.qs + a.q0) * a.ld_out + h * hd;
  const int c4 = Hp >> 2;
  for (int e = tid; e < a.Qv * c4; e += AT) {
    const int r = e / c4, col = (e - r * c4) * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s0 = 0; s0 < ns; s0 += 16) {
      float4 x[16];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        x[j] = *reinterpret_cast<const float4*>(part + ((long long)min(s0 + j, ns - 1) * Qp + r) * Hp + col);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (s0 + j < ns) {
          const float ww = stats ? w[(s0 + j) * Qp + r] : 1.f;
          acc.x += ww * x[j].x;
          acc.y += ww * x[j].y;
          acc.z += ww * x[j].z;
          acc.w += ww * x[j].w;
        }
      }
    }
    float* o = out + (long long)r * a.ld_out + col;
    const float v[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (col + j < hd) o[j] = v[j] * mul;
  }
}

__global__ __launch_bounds__(AT) void tattn_merge_kernel(TAttnArgs a, int stats, float mul) {
  extern __shared__ float sm[];
  tattn_merge(a, blockIdx.x, blockIdx.y, gridDim.y, stats, mul, sm);
}

// ------------------------------------------------------------------------------------------ backward
__global__ __launch_bounds__(AT) void tattn_bwd_kernel(TAttnArgs a) {
  extern __shared__ float sm[];
  const int c = blockIdx.x, h = blockIdx.y, vid = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Qp = a.Qp, Hp = a.Hp, Tc = a.Tc, hd = a.hd;
  const int lq = Hp + 4, ls = Tc + 4;   // 16-B aligned rows (b128 operand reads)
  float* qs = sm;                       // [Qp][lq]
  float* dos = qs + Qp * lq;            // [Qp][lq]
  float* ks = dos + Qp * lq;            // [Tc][lq]
  float* vs = ks + Tc * lq;             // [Tc][lq]
  float* ps = vs + Tc * lq;             // [Qp][ls]  P   (o until P is written)
  float* ds = ps + Qp * ls;             // [Qp][ls]  dS
  float* red = ds + Qp * ls;            // [4][1024]
  float* rl = red + 4 * 1024;           // [Qp] lse
  float* rd = rl + Qp;                  // [Qp] D
  const int Tv = a.koff[vid + 1] - a.koff[vid];
  const int t0 = c * Tc, nk = min(Tc, Tv - t0);
  if (nk <= 0) return;
  const long long qrow = (long long)vid * a.qs + a.q0, krow = (long long)a.koff[vid] + t0;
  const float* qsrc = a.q + qrow * a.ldq + h * hd;
  const float* dsrc = a.dout + qrow * a.lddo + h * hd;
  const float* osrc = a.o + qrow * a.ldo + h * hd;
  const float* ksrc = a.k + krow * a.ldk + h * hd;
  const float* vsrc = a.v + krow * a.ldv + h * hd;
  if (tid < Qp) rl[tid] = tid < a.Qv ? a.lse[((long long)vid * a.nh + h) * a.qs + a.q0 + tid] : 0.f;
  if (a.vec) {
    Strip<NVQ> sq, sd, so;
    Strip<NVK> sk, sv;
    sq.load(Qp, Hp, qsrc, a.ldq, a.Qv, hd, tid);
    sd.load(Qp, Hp, dsrc, a.lddo, a.Qv, hd, tid);
    so.load(Qp, Hp, osrc, a.ldo, a.Qv, hd, tid);
    sk.load(Tc, Hp, ksrc, a.ldk, nk, hd, tid);
    sv.load(Tc, Hp, vsrc, a.ldv, nk, hd, tid);
    sq.store(qs, lq, Qp, Hp, tid);
    sd.store(dos, lq, Qp, Hp, tid);
    so.store(ps, lq, Qp, Hp, tid);
    sk.store(ks, lq, Tc, Hp, tid);
    sv.store(vs, lq, Tc, Hp, tid);
  } else {
    stage_scalar(qs, lq, Qp, Hp, qsrc, a.ldq, a.Qv, hd, tid);
    stage_scalar(dos, lq, Qp, Hp, dsrc, a.lddo, a.Qv, hd, tid);
    stage_scalar(ps, lq, Qp, Hp, osrc, a.ldo, a.Qv, hd, tid);
    stage_scalar(ks, lq, Tc, Hp, ksrc, a.ldk, nk, hd, tid);
    stage_scalar(vs, lq, Tc, Hp, vsrc, a.ldv, nk, hd, tid);
  }
  __syncthreads();
  // D_i = sum_d dO_id o_id
  if (tid < Qp) {
    float d = 0.f;
    for (int j = 0; j < Hp; ++j) d += dos[tid * lq + j] * ps[tid * lq + j];
    rd[tid] = d;
  }
  __syncthreads();
  const int nrt = Qp / 32, nct = Tc / 32, nht = Hp / 32;
  // P = exp(scale q K^T - lse) and dS = P (dO V^T - D), tile by tile
  for (int t = wave; t < nrt * nct; t += 4) {
    const int rt = t / nct, ct = t - rt * nct;
    f32x16 s, dp;
    zero16(s);
    zero16(dp);
    mm32v<true>(qs + rt * 32 * lq, lq, ks + ct * 32 * lq, lq, Hp, s, lane);
    mm32v<true>(dos + rt * 32 * lq, lq, vs + ct * 32 * lq, lq, Hp, dp, lane);
    const int col = ct * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rt * 32 + acc_row(r, lane);
      const float p = (col < nk && row < a.Qv) ? __expf(s[r] * a.scale - rl[row]) : 0.f;
      // dropout: P_d = P keep / (1-p) multiplies V; dP = (dO V^T) keep / (1-p); D = rowsum(dO o) still
      const float kp = (a.drop_p > 0.f && p != 0.f) ? drop_keep(a, qrow + row, h, krow + col) : 1.f;
      ps[row * ls + col] = p * kp;
      ds[row * ls + col] = p * (dp[r] * kp - rd[row]);
    }
  }
  __syncthreads();
  // dV_c = P^T dO and dK_c = scale dS^T q  (Tc x Hp each), written straight to their rows
  for (int t = wave; t < 2 * nct * nht; t += 4) {
    const int which = t / (nct * nht), u = t - which * nct * nht;
    const int kt = u / nht, ht = u - kt * nht;
    f32x16 acc;
    zero16(acc);
    if (which == 0)
      mm32<true, false>(ps + kt * 32, ls, dos + ht * 32, lq, Qp, acc, lane);
    else
      mm32<true, false>(ds + kt * 32, ls, qs + ht * 32, lq, Qp, acc, lane);
    const int col = ht * 32 + (lane & 31);
    float* dst = which == 0 ? a.dv : a.dk;
    const long long ld = which == 0 ? a.lddv : a.lddk;
    const float mul = which == 0 ? 1.f : a.scale;
    if (col < hd) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + acc_row(r, lane);
        if (key < nk) {
          float* d = dst + (krow + key) * ld + h * hd + col;
          *d = a.acc_kv ? *d + acc[r] * mul : acc[r] * mul;
        }
      }
    }
  }
  // dq partial = dS K_c  (Qp x Hp), tiles split along the chunk like the forward's O
  const int nt = nrt * nht, wpt = 4 / nt;
  const int tile = wave / wpt, part = wave - tile * wpt;
  const int dlen = Tc / wpt, d0 = part * dlen;
  const int rt = tile / nht, ht = tile - rt * nht;
  f32x16 acc;
  zero16(acc);
  mm32v<false>(ds + rt * 32 * ls + d0, ls, ks + d0 * lq + ht * 32, lq, dlen, acc, lane);
  if (wpt > 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave * 1024 + r * 64 + lane] = acc[r];
    __syncthreads();
    if (part == 0)
      for (int q = 1; q < wpt; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += red[(wave + q) * 1024 + r * 64 + lane];
  }
  if (part == 0) {
    const int col = ht * 32 + (lane & 31);
    if (a.nsplit == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + acc_row(r, lane);
        if (row < a.Qv && col < hd) a.out[(qrow + row) * a.ld_out + h * hd + col] = acc[r] * a.scale;
      }
    } else {
      float* po = a.ws + (((long long)vid * a.nh + h) * a.nsplit + c) * Qp * Hp;
#pragma unroll
      for (int r = 0; r < 16; ++r) po[(rt * 32 + acc_row(r, lane)) * Hp + col] = acc[r];
    }
  }
}

// ------------------------------------------------------------------ register-resident kernels (hd 32)
// For head dim 32 and <= 32 queries per video (the benchmark's SCA decoder: 8 heads of 32, 32 tokens)
// every operand goes straight from memory into MFMA registers, no LDS staging:
//   * S^T (keys x queries) = K q^T: lane (li, lh) feeds K[key li][16 lh .. 16 lh + 15] and
//     q[query li][16 lh ..] as A / B (4 float4 each; the d order inside the sum is free as long as A and
//     B agree);
//   * the S^T accumulators hold, per lane, 16 keys of ONE query (keys acc_row(r)): the softmax statistics
//     are in-register reductions plus one exchange with the other lane half;
//   * O^T (d x queries) = V^T P^T takes the probabilities straight from those accumulators as the B
//     operand, the key of MFMA step j being acc_row(j) -- V[key acc_row(j)][d li] as the A operand (32
//     lanes read one 128-B row slice);
//   * each wave owns 32 KT keys of the chunk; the 4 waves' (m, l, O) are combined through LDS once.
// Backward: S^T and dP^T = V dO^T the same way, dq = dS K with dS^T from the accumulators as the A
// operand; dV = P_d^T dO and dK = scale dS^T q need the probabilities with the key as the ROW index, so
// P_d^T and dS^T go through a wave-private LDS tile (no workgroup barrier).
__device__ __forceinline__ float4 ld4g(const float* p) { return *reinterpret_cast<const float4*>(p); }
// Diagnostic builds only (-DTATTN_STAMPS, tools/tattn_stamps.py): s_memrealtime stamps of thread 0 of every
// workgroup of the last tattn_fwd32_kernel launch (fx_debug_tattn_stamps); never in the shipped library
#ifdef TATTN_STAMPS
__device__ unsigned long long g_ta_st[1024 * 8];
#define TA_ST(k)                                                                                        \
  do {                                                                                                  \
    const int b_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                      \
    if (threadIdx.x == 0 && b_ < 1024) g_ta_st[b_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)
#else
#define TA_ST(k) \
  do {           \
  } while (0)
#endif

// write-through (sc1) accesses of the in-launch merge: L1 bypassed, stores written through (the b32
// buffer forms move the float's bits)
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float ldc1(const float* base, long long idx) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(base), (int)(idx * 4), 0, 16));
}
__device__ __forceinline__ float4 ldc4(const float* base, long long idx) {
  const v4f v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)(idx * 4), 0, 16);
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void stc1(float* base, long long idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(base), (int)(idx * 4), 0, 16);
}
__device__ __forceinline__ void stc4(float* base, long long idx, float4 v) {
  v4f x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(base), (int)(idx * 4), 0, 16);
}
constexpr int FOLD_MAX = 16;   // chunks per video merged inside the launch (more: tattn_merge_kernel)

// The chunk partials of (video, head) merged by the LAST workgroup to finish one (the microarch guide's
// write-through hand-off, valid form 1): every workgroup stored its 32 x 32 partial (and forward: row
// max / sum) with sc1 stores and waited for their acknowledgement before its arrival on the counter; the
// last arriver re-arms the counter and reads the partials with sc1 loads, in chunk order (deterministic,
// the same order as tattn_merge).  Forward (stats): o = sum_s e^(m_s - M) O_s / L, lse = M + log L;
// backward: dq = mul sum_s dq_s.  Returns after the merge (or at once for the other workgroups).
__device__ __forceinline__ void fold_merge(const TAttnArgs& a, int vid, int h, int ns, bool stats, float mul,
                                           long long qrow, float (*wm)[32], float (*wl)[32], int* last) {
  const int tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's partial stores acknowledged
  __syncthreads();
  if (stats) TA_ST(4);
  if (tid == 0) {
    unsigned* c = a.cnt + (long long)vid * a.nh + h;
    const unsigned prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = prev == (unsigned)ns - 1;
    if (*last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (stats) TA_ST(5);
  if (!*last) return;
  const long long pbase = ((long long)vid * a.nh + h) * a.nsplit;
  const float* part = a.ws;
  const float* pm = a.ws + (long long)gridDim.z * a.nh * a.nsplit * 32 * 32;
  const float* pl = pm + (long long)gridDim.z * a.nh * a.nsplit * 32;
  // every load of the merge at once: this thread's (query, 4 consecutive d) slice of every partial as one
  // 16-B load each (query tid / 8, d 4 (tid % 8) ..), and (forward) the row statistics of (partial, query)
  // pairs tid, tid + 256
  const int mq = tid >> 3, md = (tid & 7) * 4;
  float4 x[FOLD_MAX];
#pragma unroll
  for (int sp = 0; sp < FOLD_MAX; ++sp) x[sp] = ldc4(part, (pbase + min(sp, ns - 1)) * 1024 + mq * 32 + md);
  if (stats) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * AT, sp = e >> 5, q = e & 31;
      const float m = ldc1(pm, (pbase + min(sp, ns - 1)) * 32 + q), l = ldc1(pl, (pbase + min(sp, ns - 1)) * 32 + q);
      if (sp < ns) {
        wm[sp][q] = m;
        wl[sp][q] = l;
      }
    }
    __syncthreads();
    if (tid < 32) {
      float M = -INFINITY;
      for (int sp = 0; sp < ns; ++sp) M = fmaxf(M, wm[sp][tid]);
      float L = 0.f;
      for (int sp = 0; sp < ns; ++sp) L += __expf(wm[sp][tid] - M) * wl[sp][tid];
      const float inv = 1.f / L;
      for (int sp = 0; sp < ns; ++sp) wm[sp][tid] = __expf(wm[sp][tid] - M) * inv;
      if (tid < a.Qv) a.lse[((long long)vid * a.nh + h) * a.qs + a.q0 + tid] = M + __logf(L);
    }
    __syncthreads();
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int sp = 0; sp < FOLD_MAX; ++sp)
    if (sp < ns) {
      const float wgt = stats ? wm[sp][mq] : 1.f;
      acc.x += wgt * x[sp].x;
      acc.y += wgt * x[sp].y;
      acc.z += wgt * x[sp].z;
      acc.w += wgt * x[sp].w;
    }
  if (mq < a.Qv) {
    float* o = a.out + (qrow + mq) * a.ld_out + h * 32 + md;
    o[0] = acc.x * mul;
    o[1] = acc.y * mul;
    o[2] = acc.z * mul;
    o[3] = acc.w * mul;
  }
  if (stats) TA_ST(6);
}

template <int KT>
__global__ __launch_bounds__(AT) void tattn_fwd32_kernel(TAttnArgs a) {
  __shared__ float xo[4][32][33];   // per-wave O^T partial [d][query]
  __shared__ float xm[4][32], xl[4][32];
  const int c = blockIdx.x, h = blockIdx.y, vid = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  TA_ST(0);
  const int Tv = a.koff[vid + 1] - a.koff[vid];
  const int t0 = c * a.Tc, nk = min(a.Tc, Tv - t0);
  if (nk <= 0) return;
  const long long qrow = (long long)vid * a.qs + a.q0, krow = (long long)a.koff[vid] + t0;
  const int kw0 = w * 32 * KT;
  // every load first: q and K fragments, V columns
  float4 qf[4], kf[KT][4];
  float vf[KT][16];
  {
    const float* qp = a.q + (qrow + min(li, a.Qv - 1)) * a.ldq + h * 32 + 16 * lh;
#pragma unroll
    for (int q = 0; q < 4; ++q) qf[q] = ld4g(qp + 4 * q);
    // (every K fragment before the first V column: loads complete in issue order, so S = q K^T then waits
    // for K alone and the V columns arrive behind its MFMAs)
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const float* kp = a.k + (krow + min(kw0 + 32 * u + li, nk - 1)) * a.ldk + h * 32 + 16 * lh;
#pragma unroll
      for (int q = 0; q < 4; ++q) kf[u][q] = ld4g(kp + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < KT; ++u) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        vf[u][j] = a.v[(krow + min(kw0 + 32 * u + acc_row(j, lane), nk - 1)) * a.ldv + h * 32 + li];
    }
  }
  f32x16 st[KT];
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    zero16(st[u]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      st[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].x, qf[q].x, st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].y, qf[q].y, st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].z, qf[q].z, st[u], 0, 0, 0);
      st[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].w, qf[q].w, st[u], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kw0 + 32 * u + acc_row(r, lane);
      st[u][r] = key < nk ? st[u][r] * a.scale : -INFINITY;
      mx = fmaxf(mx, st[u][r]);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  TA_ST(1);
  float l = 0.f;
  f32x16 ou[KT];   // one P V accumulator per key tile: independent MFMA chains, summed after
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    zero16(ou[u]);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = mx == -INFINITY ? 0.f : __expf(st[u][r] - mx);   // (a wave past the video's keys)
      l += p;                                                         // the normaliser sees every key
      float kp = 1.f;
      if (a.drop_p > 0.f && p != 0.f) kp = drop_keep(a, qrow + li, h, krow + kw0 + 32 * u + acc_row(r, lane));
      st[u][r] = p * kp;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) ou[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[u][j], st[u][j], ou[u], 0, 0, 0);
  }
  f32x16 o = ou[0];
#pragma unroll
  for (int u = 1; u < KT; ++u) o += ou[u];
  l += __shfl_xor(l, 32, 64);
  if (lane < 32) {
    xm[w][li] = mx;
    xl[w][li] = l;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) xo[w][acc_row(r, lane)][li] = o[r];
  TA_ST(2);
  __syncthreads();
  // the 4 waves' partials, in wave order; thread -> (query q, d) pairs
  const long long pid = ((long long)vid * a.nh + h) * a.nsplit + c;
  float* pm = a.ws + (long long)gridDim.z * a.nh * a.nsplit * 32 * 32;
  float* pl = pm + (long long)gridDim.z * a.nh * a.nsplit * 32;
  const int ns = (Tv + a.Tc - 1) / a.Tc;   // this video's chunks
  const bool fold = a.cnt != nullptr;
  // a one-chunk video writes its rows directly, except when a merge launch follows (no fold, more than
  // one chunk in the launch): that launch merges every video, so every video leaves partials
  const bool direct = ns == 1 && (fold || a.nsplit == 1);
  {   // thread -> (query tid / 8, 4 consecutive d): one 16-B partial store (the merge reads it back the same way)
    const int q = tid >> 3, d0 = (tid & 7) * 4;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, xm[ww][q]);
    float4 O = make_float4(0.f, 0.f, 0.f, 0.f);
    float L = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float f = xm[ww][q] == -INFINITY ? 0.f : __expf(xm[ww][q] - M);
      O.x += f * xo[ww][d0][q];
      O.y += f * xo[ww][d0 + 1][q];
      O.z += f * xo[ww][d0 + 2][q];
      O.w += f * xo[ww][d0 + 3][q];
      L += f * xl[ww][q];
    }
    if (direct) {
      if (q < a.Qv) {
        float* op = a.out + (qrow + q) * a.ld_out + h * 32 + d0;
        op[0] = O.x / L;
        op[1] = O.y / L;
        op[2] = O.z / L;
        op[3] = O.w / L;
        if (d0 == 0) a.lse[((long long)vid * a.nh + h) * a.qs + a.q0 + q] = M + __logf(L);
      }
    } else if (fold) {
      stc4(a.ws, (pid * 32 + q) * 32 + d0, O);
      if (d0 == 0) {
        stc1(pm, pid * 32 + q, M);
        stc1(pl, pid * 32 + q, L);
      }
    } else {
      *reinterpret_cast<float4*>(a.ws + (pid * 32 + q) * 32 + d0) = O;
      if (d0 == 0) {
        pm[pid * 32 + q] = M;
        pl[pid * 32 + q] = L;
      }
    }
  }
  TA_ST(3);
  if (ns > 1 && fold) {
    __shared__ int last;
    // (the wave partial images are free now: the merge's weights reuse them)
    fold_merge(a, vid, h, ns, true, 1.f, qrow, reinterpret_cast<float(*)[32]>(&xo[0][0][0]),
               reinterpret_cast<float(*)[32]>(&xo[2][0][0]), &last);
  }
}

template <int KT>
__global__ __launch_bounds__(AT) void tattn_bwd32_kernel(TAttnArgs a) {
  __shared__ float tp[4][32][33];    // wave-private: P_d^T of the current key tile [key][query]
  __shared__ float tds[4][32][33];   // dS^T [key][query]
  __shared__ float xq[4][32][33];    // per-wave dq partial [query][d]
  const int c = blockIdx.x, h = blockIdx.y, vid = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int Tv = a.koff[vid + 1] - a.koff[vid];
  const int t0 = c * a.Tc, nk = min(a.Tc, Tv - t0);
  if (nk <= 0) return;
  const long long qrow = (long long)vid * a.qs + a.q0, krow = (long long)a.koff[vid] + t0;
  const int kw0 = w * 32 * KT;
  const int Qv = a.Qv;
  // every load first.  Query-side fragments (query li, d 16 lh ..): q, dO, o; query-side columns (query
  // acc_row(j), d li): q, dO (the B operands of dK and dV); key side: K and V fragments (key li, d 16 lh ..)
  // and K columns (key acc_row(j), d li) for dq
  float4 qf[4], df[4], of[4], kf[KT][4], vf[KT][4];
  float qt[16], dt[16], kt[KT][16];
  const int qi = min(li, Qv - 1);
  {
    const float* qp = a.q + (qrow + qi) * a.ldq + h * 32 + 16 * lh;
    const float* dp = a.dout + (qrow + qi) * a.lddo + h * 32 + 16 * lh;
    const float* op = a.o + (qrow + qi) * a.ldo + h * 32 + 16 * lh;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      qf[q] = ld4g(qp + 4 * q);
      df[q] = ld4g(dp + 4 * q);
      of[q] = ld4g(op + 4 * q);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const long long qr = qrow + min(acc_row(j, lane), Qv - 1);
      qt[j] = a.q[qr * a.ldq + h * 32 + li];
      dt[j] = a.dout[qr * a.lddo + h * 32 + li];
    }
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const long long kr = krow + min(kw0 + 32 * u + li, nk - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        kf[u][q] = ld4g(a.k + kr * a.ldk + h * 32 + 16 * lh + 4 * q);
        vf[u][q] = ld4g(a.v + kr * a.ldv + h * 32 + 16 * lh + 4 * q);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j)
        kt[u][j] = a.k[(krow + min(kw0 + 32 * u + acc_row(j, lane), nk - 1)) * a.ldk + h * 32 + li];
    }
  }
  const float lse = li < Qv ? a.lse[((long long)vid * a.nh + h) * a.qs + a.q0 + li] : 0.f;
  // D = rowsum(dO o) of this lane's query
  float D = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) D += (df[q].x * of[q].x + df[q].y * of[q].y) + (df[q].z * of[q].z + df[q].w * of[q].w);
  D += __shfl_xor(D, 32, 64);
  f32x16 dqu[KT];   // one dq accumulator per key tile (independent chains), summed after
#pragma unroll
  for (int u = 0; u < KT; ++u) {
    zero16(dqu[u]);
    f32x16 s, dp;
    zero16(s);
    zero16(dp);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].x, qf[q].x, s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[u][q].x, df[q].x, dp, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].y, qf[q].y, s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[u][q].y, df[q].y, dp, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].z, qf[q].z, s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[u][q].z, df[q].z, dp, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[u][q].w, qf[q].w, s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[u][q].w, df[q].w, dp, 0, 0, 0);
    }
    // P^T, P_d^T, dS^T = P (dP keep - D) (dropout: P_d = P keep multiplied V, dP = (dO V^T) keep)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kl = acc_row(r, lane), key = kw0 + 32 * u + kl;
      const float p = (key < nk && li < Qv) ? __expf(s[r] * a.scale - lse) : 0.f;
      const float kp = (a.drop_p > 0.f && p != 0.f) ? drop_keep(a, qrow + li, h, krow + key) : 1.f;
      const float ds = p * (dp[r] * kp - D);
      tp[w][kl][li] = p * kp;
      tds[w][kl][li] = ds;
      s[r] = ds;
    }
    // dq += dS K: A = dS (query li, key acc_row(j)) from the accumulators, B = K (key acc_row(j), d li)
#pragma unroll
    for (int j = 0; j < 16; ++j) dqu[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(s[j], kt[u][j], dqu[u], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's tile writes are visible to its lanes
    // dV = P_d^T dO and dK = dS^T q over the queries: A = the LDS tile (key li, query acc_row(j))
    f32x16 dv, dk;
    zero16(dv);
    zero16(dk);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int qj = acc_row(j, lane);
      dv = __builtin_amdgcn_mfma_f32_32x32x2f32(tp[w][li][qj], dt[j], dv, 0, 0, 0);
      dk = __builtin_amdgcn_mfma_f32_32x32x2f32(tds[w][li][qj], qt[j], dk, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kw0 + 32 * u + acc_row(r, lane);
      if (key < nk) {
        float* pv = a.dv + (krow + key) * a.lddv + h * 32 + li;
        float* pk = a.dk + (krow + key) * a.lddk + h * 32 + li;
        *pv = a.acc_kv ? *pv + dv[r] : dv[r];
        *pk = a.acc_kv ? *pk + dk[r] * a.scale : dk[r] * a.scale;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // tile reads done before the next tile's writes
  }
  f32x16 dq = dqu[0];
#pragma unroll
  for (int u = 1; u < KT; ++u) dq += dqu[u];
#pragma unroll
  for (int r = 0; r < 16; ++r) xq[w][acc_row(r, lane)][li] = dq[r];
  __syncthreads();
  const long long pid = ((long long)vid * a.nh + h) * a.nsplit + c;
  const int ns = (Tv + a.Tc - 1) / a.Tc;
  const bool fold = a.cnt != nullptr;
  const bool direct = ns == 1 && (fold || a.nsplit == 1);   // (see the forward)
  {   // thread -> (query tid / 8, 4 consecutive d): one 16-B partial store (as the forward)
    const int q = tid >> 3, d0 = (tid & 7) * 4;
    float4 v;
    v.x = (xq[0][q][d0] + xq[1][q][d0]) + (xq[2][q][d0] + xq[3][q][d0]);
    v.y = (xq[0][q][d0 + 1] + xq[1][q][d0 + 1]) + (xq[2][q][d0 + 1] + xq[3][q][d0 + 1]);
    v.z = (xq[0][q][d0 + 2] + xq[1][q][d0 + 2]) + (xq[2][q][d0 + 2] + xq[3][q][d0 + 2]);
    v.w = (xq[0][q][d0 + 3] + xq[1][q][d0 + 3]) + (xq[2][q][d0 + 3] + xq[3][q][d0 + 3]);
    if (direct) {
      if (q < Qv) {
        float* op = a.out + (qrow + q) * a.ld_out + h * 32 + d0;
        op[0] = v.x * a.scale;
        op[1] = v.y * a.scale;
        op[2] = v.z * a.scale;
        op[3] = v.w * a.scale;
      }
    } else if (fold) {
      stc4(a.ws, (pid * 32 + q) * 32 + d0, v);
    } else {
      *reinterpret_cast<float4*>(a.ws + (pid * 32 + q) * 32 + d0) = v;
    }
  }
  if (ns > 1 && fold) {
    __shared__ int last;
    fold_merge(a, vid, h, ns, false, a.scale, qrow, nullptr, nullptr, &last);
  }
}

struct TAttnGeom {
  int Qp, Hp, Tc, nsplit;
  size_t lds;
};

constexpr int QB = 64;    // queries per launch (query blocks of more tokens run as successive launches)

// chunk: the largest power of two in [32, 256] whose LDS images fit (Tc * Hp <= NVK float4 per thread),
// halved while the launch has fewer than ~256 workgroups.  Tv: the longest video's key count.
TAttnGeom tattn_geom(int nvid, int Qv, int Tv, int hd, int nh, bool bwd) {
  TAttnGeom g{};
  g.Qp = std::max(32, (std::min(Qv, QB) + 31) / 32 * 32);
  g.Hp = std::max(32, (hd + 31) / 32 * 32);
  auto lds_b = [&](int Tc) {
    const size_t q = bwd ? 2 : 1, p = bwd ? 2 : 1;
    return sizeof(float) * (q * g.Qp * (g.Hp + 4) + 2 * (size_t)Tc * (g.Hp + 4) + p * g.Qp * (Tc + 4) + 4 * 1024 +
                            2 * g.Qp + 4);
  };
  int Tc = 256;   // the largest key chunk (smaller chunks, more workgroups per CU, measured slower: round 4)
  // (forward: at most 8 score tiles, two per wave, in registers)
  while (Tc > 32 && (lds_b(Tc) > 150 * 1024 || Tc * g.Hp > NVK * 4 * AT || Tc * g.Qp > 8 * 1024)) Tc >>= 1;
  constexpr int kMinWorkgroups = 256;   // one per CU
  while (Tc > 32 && (long long)nvid * nh * ((Tv + Tc - 1) / Tc) < kMinWorkgroups) Tc >>= 1;
  g.Tc = Tc;
  g.nsplit = std::max(1, (Tv + Tc - 1) / Tc);
  g.lds = lds_b(Tc);
  return g;
}

}  // namespace

#ifdef FX_STAMPS
extern "C" int fx_dbg_tattn_stamps(long long* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tattn_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -2;
}
#endif

// the register-resident kernels' chunk: 32 KT keys per wave, KT = 2 (256-key chunks) unless that leaves
// fewer than one workgroup per CU, then KT = 1 (128-key chunks)
static int tattn_rr_tc(int nvid, int Tv, int nh) {
  return (long long)nvid * nh * ((Tv + 255) / 256) >= 256 ? 256 : 128;
}
static bool tattn_rr_ok(int Qv, int hd, bool aligned) { return knobs().tattn_rr && hd == 32 && Qv <= 32 && aligned; }
// the register-resident kernels merge in the launch (fold_merge) when every video has <= FOLD_MAX chunks:
// the stream's arrival counters, one per (video, head); else null (tattn_merge_kernel after the launch)
static unsigned* tattn_fold_counters(int nsplit, int nvid, int nh, hipStream_t s) {
  if (!knobs().tattn_fold || nsplit <= 1 || nsplit > FOLD_MAX || (long long)nvid * nh > kArrivalCounters) return nullptr;
  return arrival_counters(s);
}

long long tattn_ws_floats(int nvid, int Qv, int Tv, int hd, int nh) {
  long long w = 0;
  if (hd == 32 && Qv <= 32) {   // (the register-resident geometry: 32 x 32 partials)
    const long long np = (long long)nvid * nh * ((Tv + tattn_rr_tc(nvid, Tv, nh) - 1) / tattn_rr_tc(nvid, Tv, nh));
    w = np * 32 * 32 + 2 * np * 32;
  }
  for (int bwd = 0; bwd < 2; ++bwd) {
    const TAttnGeom g = tattn_geom(nvid, Qv, Tv, hd, nh, bwd);
    const long long np = (long long)nvid * nh * g.nsplit;
    w = std::max(w, np * g.Qp * g.Hp + 2 * np * g.Qp);
  }
  return w;
}

static size_t merge_lds(const TAttnGeom& g) { return sizeof(float) * 2 * (size_t)g.nsplit * g.Qp; }

static bool a16(const void* p, long long ld) { return p == nullptr || (((uintptr_t)p & 15) == 0 && (ld & 3) == 0); }

// shared argument set-up: key offsets (uniform Tv per video when opt->koff is NULL), dropout
static int tattn_setup(TAttnArgs& a, int nvid, int Qv, int Tv, int hd, int nh, const TAttnOpts* opt, int& Tmax,
                       long long& ktot) {
  static std::once_flag once;
  std::call_once(once, [] {   // dynamic LDS above the 64 KB default (gfx950: 160 KB per workgroup)
    (void)hipFuncSetAttribute((const void*)tattn_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tattn_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tattn_merge_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  FX_REQUIRE(nvid >= 1 && nvid <= MAXV && Qv >= 1 && hd >= 1 && hd <= 64 && nh >= 1,
             "attention over T: 1..32 videos, >= 1 query, head dim <= 64");
  Tmax = 0;
  a.koff[0] = 0;
  for (int v = 0; v < nvid; ++v) {
    const int k0 = opt && opt->koff ? opt->koff[v] : v * Tv, k1 = opt && opt->koff ? opt->koff[v + 1] : (v + 1) * Tv;
    FX_REQUIRE(k1 > k0 && k0 >= 0, "attention over T: every video needs >= 1 key row, offsets increasing");
    a.koff[v] = k0;
    a.koff[v + 1] = k1;
    Tmax = std::max(Tmax, k1 - k0);
  }
  ktot = a.koff[nvid];
  const float p = opt ? opt->drop_p : 0.f;
  FX_REQUIRE(p >= 0.f && p < 1.f, "attention over T: dropout p in [0, 1)");
  a.drop_p = p;
  a.drop_thr = p > 0.f ? std::max(fx_drop_thresh(p), 1u) : 0u;
  a.drop_seed = opt ? opt->drop_seed : 0ull;
  a.ktot = ktot;
  a.hd = hd;
  a.nh = nh;
  a.qs = Qv;
  return FX_OK;
}

int launch_tattn_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                     int nvid, int Qv, int Tv, int hd, int nh, float scale, float* o, long long ldo, float* lse,
                     float* ws, hipStream_t s, const TAttnOpts* opt) {
  TAttnArgs a{};
  int Tmax = 0;
  long long ktot = 0;
  FX_TRY(tattn_setup(a, nvid, Qv, Tv, hd, nh, opt, Tmax, ktot));
  const TAttnGeom g = tattn_geom(nvid, Qv, Tmax, hd, nh, false);
  FX_REQUIRE(ws || g.nsplit == 1, "attention over T: workspace required");
  FX_REQUIRE(g.lds <= 160 * 1024, "attention over T: LDS images too large");
  FX_REQUIRE(merge_lds(g) <= 160 * 1024, "attention over T: too many frames per video for the in-LDS merge");
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv;
  a.out = o; a.ld_out = ldo; a.lse = lse; a.ws = ws;
  a.Qp = g.Qp; a.Hp = g.Hp; a.Tc = g.Tc; a.nsplit = g.nsplit;
  a.scale = scale;
  a.vec = (hd % 4 == 0) && a16(q, ldq) && a16(k, ldk) && a16(v, ldv);
  // algorithmic traffic: K and V rows read once per query block, q read, o and lse written
  const int nqb = (Qv + QB - 1) / QB;
  const double kv = (double)ktot * nh * hd * nqb, qo = (double)nvid * Qv * nh * hd;
  if (tattn_rr_ok(Qv, hd, a.vec)) {
    a.Tc = tattn_rr_tc(nvid, Tmax, nh);
    a.nsplit = (Tmax + a.Tc - 1) / a.Tc;
    a.Qp = a.Hp = 32;
    a.q0 = 0;
    a.Qv = Qv;
    FX_REQUIRE(ws || a.nsplit == 1, "attention over T: workspace required");
    a.cnt = tattn_fold_counters(a.nsplit, nvid, nh, s);
    prof_begin(1, s);
    if (a.Tc == 256) fx_launch(tattn_fwd32_kernel<2>, dim3(a.nsplit, nh, nvid), dim3(AT), 0, s, a);
    else fx_launch(tattn_fwd32_kernel<1>, dim3(a.nsplit, nh, nvid), dim3(AT), 0, s, a);
    FX_CHECK_HIP(hipGetLastError());
    if (a.nsplit > 1 && !a.cnt) {
      fx_launch(tattn_merge_kernel, dim3(nh, nvid), dim3(AT), sizeof(float) * 2 * a.nsplit * 32, s, a, 1,
                         1.f);
      FX_CHECK_HIP(hipGetLastError());
    }
    prof_end(1, s, 4.0 * qo * (double)ktot / nvid, 4.0 * (2.0 * kv + 2.0 * qo + (double)nvid * nh * Qv));
    return FX_OK;
  }
  prof_begin(1, s);
  for (int q0 = 0; q0 < Qv; q0 += QB) {
    a.q0 = q0;
    a.Qv = std::min(QB, Qv - q0);
    fx_launch(tattn_fwd_kernel, dim3(g.nsplit, nh, nvid), dim3(AT), std::max(g.lds, merge_lds(g) + 16), s,
                       a);
    FX_CHECK_HIP(hipGetLastError());
    if (g.nsplit > 1) {
      fx_launch(tattn_merge_kernel, dim3(nh, nvid), dim3(AT), merge_lds(g), s, a, 1, 1.f);
      FX_CHECK_HIP(hipGetLastError());
    }
  }
  prof_end(1, s, 4.0 * qo * (double)ktot / nvid, 4.0 * (2.0 * kv + 2.0 * qo + (double)nvid * nh * Qv));
  return FX_OK;
}

int launch_tattn_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv,
                     const float* o, long long ldo, const float* dout, long long lddo, const float* lse, int nvid,
                     int Qv, int Tv, int hd, int nh, float scale, float* dq, long long lddq, float* dk, long long lddk,
                     float* dv, long long lddv, float* ws, hipStream_t s, const TAttnOpts* opt) {
  TAttnArgs a{};
  int Tmax = 0;
  long long ktot = 0;
  FX_TRY(tattn_setup(a, nvid, Qv, Tv, hd, nh, opt, Tmax, ktot));
  const TAttnGeom g = tattn_geom(nvid, Qv, Tmax, hd, nh, true);
  FX_REQUIRE(ws || g.nsplit == 1, "attention over T: workspace required");
  FX_REQUIRE(g.lds <= 160 * 1024, "attention over T: LDS images too large");
  FX_REQUIRE(dq && dk && dv, "attention over T backward: dq, dk, dv required");
  a.q = q; a.ldq = ldq; a.k = k; a.ldk = ldk; a.v = v; a.ldv = ldv;
  a.o = o; a.ldo = ldo; a.dout = dout; a.lddo = lddo;
  a.out = dq; a.ld_out = lddq; a.dk = dk; a.lddk = lddk; a.dv = dv; a.lddv = lddv;
  a.lse = const_cast<float*>(lse); a.ws = ws;
  a.Qp = g.Qp; a.Hp = g.Hp; a.Tc = g.Tc; a.nsplit = g.nsplit;
  a.scale = scale;
  a.vec = (hd % 4 == 0) && a16(q, ldq) && a16(k, ldk) && a16(v, ldv) && a16(o, ldo) && a16(dout, lddo);
  // algorithmic traffic: K, V read and dK, dV written once per query block; q, o, dout, lse read, dq written.
  // flops: S = qK^T recomputed, dP = dO V^T, dV = P^T dO, dK = dS^T q, dq = dS K
  const int nqb = (Qv + QB - 1) / QB;
  const double kv = (double)ktot * nh * hd * nqb, qo = (double)nvid * Qv * nh * hd;
  if (tattn_rr_ok(Qv, hd, a.vec)) {
    a.Tc = tattn_rr_tc(nvid, Tmax, nh);
    a.nsplit = (Tmax + a.Tc - 1) / a.Tc;
    a.Qp = a.Hp = 32;
    a.q0 = 0;
    a.Qv = Qv;
    a.acc_kv = opt && opt->acc_kv;
    FX_REQUIRE(ws || a.nsplit == 1, "attention over T: workspace required");
    a.cnt = tattn_fold_counters(a.nsplit, nvid, nh, s);
    prof_begin(2, s);
    if (a.Tc == 256) fx_launch(tattn_bwd32_kernel<2>, dim3(a.nsplit, nh, nvid), dim3(AT), 0, s, a);
    else fx_launch(tattn_bwd32_kernel<1>, dim3(a.nsplit, nh, nvid), dim3(AT), 0, s, a);
    FX_CHECK_HIP(hipGetLastError());
    if (a.nsplit > 1 && !a.cnt) {
      fx_launch(tattn_merge_kernel, dim3(nh, nvid), dim3(AT), 0, s, a, 0, scale);
      FX_CHECK_HIP(hipGetLastError());
    }
    prof_end(2, s, 10.0 * qo * (double)ktot / nvid, 4.0 * (4.0 * kv + 4.0 * qo + (double)nvid * nh * Qv));
    return FX_OK;
  }
  prof_begin(2, s);
  // query blocks one after another: a later block ADDS its dK / dV to the earlier blocks' (same key rows)
  for (int q0 = 0; q0 < Qv; q0 += QB) {
    a.q0 = q0;
    a.Qv = std::min(QB, Qv - q0);
    a.acc_kv = (q0 > 0) || (opt && opt->acc_kv);
    fx_launch(tattn_bwd_kernel, dim3(g.nsplit, nh, nvid), dim3(AT), std::max(g.lds, merge_lds(g) + 16), s,
                       a);
    FX_CHECK_HIP(hipGetLastError());
    if (g.nsplit > 1) {
      fx_launch(tattn_merge_kernel, dim3(nh, nvid), dim3(AT), 0, s, a, 0, scale);
      FX_CHECK_HIP(hipGetLastError());
    }
  }
  prof_end(2, s, 10.0 * qo * (double)ktot / nvid, 4.0 * (4.0 * kv + 4.0 * qo + (double)nvid * nh * Qv));
  return FX_OK;
}

}  // namespace fx

#ifdef TATTN_STAMPS
extern "C" int fx_debug_tattn_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(fx::g_ta_st), sizeof(fx::g_ta_st)) == hipSuccess ? 0 : -1;
}
#endif
