// Persistent token-side decoder kernel: every token-row operation of an SCADecoder / SADecoder layer
// between two attention-over-T launches in ONE launch (SCALayer basic.py:494-523, SALayer 429-452,
// SCADecoder 542-557, SADecoder 578-593).
//
// The token rows of a lockstep batch are few (R = videos x Nact, 64 at the benchmark shape) and a
// layer is a chain of small dependent products -- in-projection, self-attention over the tokens, out-
// projection + residual, LayerNorm, query projection, (attention over T), out-projection + residual,
// LayerNorm, FFN, FFN + residual, LayerNorm -- that ran as ~12 launches of 5-10 us each.  Here a
// launch executes a short PROGRAM of phases (TokPhase, by value in the kernel arguments) on a small
// persistent grid; phases are separated by a grid barrier.  A phase is a list of items (32-row x
// 32-column output tiles of a GEMM, or one (video, head) of the self-attention) dealt round robin to
// the workgroups.
//
//   * LayerNorm forward and backward are not phases of their own: a GEMM whose A operand is a
//     LayerNorm output (or the gradient that flows back through one) normalises the 32 rows of its tile
//     while staging them into LDS (row statistics over 8 lanes per row, every workgroup for its own
//     rows), and the items of the first column tiles also write the saved LN outputs (x-hat, 1/std,
//     the output and output + query position) that the residuals and the backward read.
//   * The self-attention in-projection and the attention core of one (video, head) are one item: the
//     head's v, then q / k columns (q = k input = rows + query position) from the staged rows, then S,
//     softmax, P V in LDS with the fixed-order FMA chains of attn_small.hip.
//   * Hand-offs between the phases of a launch use the microarch guide's write-through form (Valid
//     forms, first table row): every store of data a later phase reads is an `sc1` buffer store, every
//     load of such data an `sc1` buffer load (no agent-scope release / acquire fences), every storing
//     wave waits for its stores (vmcnt 0) before its workgroup's single arrival add, and the waiting
//     lane polls the per-launch arrival counter with `sc1` loads.  Weights and tensors written before
//     the launch are read with plain loads.
//   * Every spin is bounded: a workgroup that waits ~1 s sets FX_STATUS_TOK_TIMEOUT in the caller's
//     status word and leaves the program.
// Products use v_mfma_f32_32x32x2f32 (exact f32 products, as the rest of the library), K split over
// the 4 waves of a workgroup and summed in LDS in a fixed order (deterministic).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

#include "fx_common.h"
#include "ops.h"
#include "tokdec.h"

namespace fx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int TT = 256;                 // threads per workgroup (4 waves)
constexpr int HS = 33;                  // self-attention LDS row stride (head dim 32 + 1)

// ------------------------------------------------------------------ write-through (sc1) accesses
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
// (cache-policy operand 16 = sc1 on gfx950: L1 bypassed, stores written through)
__device__ __forceinline__ float4 ldc4(const float* base, long long idx) {
  const v4f v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), (int)(idx * 4), 0, 16);
  return make_float4(v[0], v[1], v[2], v[3]);
}
// (the b32 forms move 32-bit integers: the float's bits, not its value)
__device__ __forceinline__ float ldc1(const float* base, long long idx) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(base), (int)(idx * 4), 0, 16));
}
__device__ __forceinline__ void stc1(float* base, long long idx, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(base), (int)(idx * 4), 0, 16);
}
__device__ __forceinline__ void stc4(float* base, long long idx, float4 v) {
  v4f x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(base), (int)(idx * 4), 0, 16);
}
// plain accesses to tensors written before the launch, as global-memory instructions (the phase fields
// come through LDS, so the compiler cannot tell that their pointers are global and would emit flat ones)
// (through the native vector type: float4's copy constructor would take the operand back to a generic
// reference)
typedef __attribute__((address_space(1))) const v4f gcf4;
typedef __attribute__((address_space(1))) const float gcf1;
typedef __attribute__((address_space(1))) float gf1;
__device__ __forceinline__ float4 ld4(const float* p) {
  const v4f v = *(gcf4*)(p);
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ float ld1(const float* p) { return *(gcf1*)(p); }
__device__ __forceinline__ void st1(float* p, float v) { *(gf1*)(p) = v; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

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
// sum over the 8 lanes of one staged row (consecutive lanes)
__device__ __forceinline__ float rsum8(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}
__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 0.f;
}
__device__ __forceinline__ float keepf(unsigned long long seed, unsigned thr, float scale, unsigned long long idx) {
  return fx_drop_bits(seed, idx) >= thr ? scale : 0.f;
}
// accumulator element r of a lane: row (r & 3) + 8 (r >> 2) + 4 (lane >> 5), column lane & 31
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS accesses, not for its global
// stores (__syncthreads() also waits for every outstanding global store -- with write-through stores,
// their write acknowledgements -- before the barrier; the phases' global hand-offs are ordered by the
// grid barrier's own wait instead)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// diagnostic stamps (FX_TOK_DEBUG): the current phase's 8 LDS slots of this workgroup, or null
__device__ __forceinline__ void tstamp(unsigned long long* st, int k) {
  if (st && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------ grid barrier
// A launch owns one slot {arrivals | exits} (two 128-B lines), zero when it starts: barrier n of the
// launch waits for (n + 1) G arrivals; after the last phase every workgroup adds to `exits` and the last
// one re-arms the slot for the launch that reuses it (slots are dealt round robin per stream).
struct BarState {
  unsigned long long* cnt;
  unsigned long long target;
  unsigned* status;
  unsigned spin_max;
  int G;
};

__device__ __forceinline__ bool grid_sync(BarState& b, int* dead) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this wave has left (sc1: written through)
  __syncthreads();
  b.target += (unsigned long long)b.G;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(b.cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // two polls in flight, half a round trip apart: the last arrival is seen up to half a memory round
    // trip sooner than with one poll at a time
    unsigned long long x0 = __hip_atomic_load(b.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_sleep(4);
    unsigned long long x1 = __hip_atomic_load(b.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned n = 0;
    while (true) {
      if ((long long)(x0 - b.target) >= 0) break;
      x0 = __hip_atomic_load(b.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((long long)(x1 - b.target) >= 0) break;
      x1 = __hip_atomic_load(b.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_sleep(1);
      if (++n > b.spin_max) {
        __hip_atomic_fetch_or(b.status, (unsigned)FX_STATUS_TOK_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *dead = 1;
        break;
      }
    }
  }
  __syncthreads();
  return !*dead;
}

// Every workgroup counts its exit, also one that gave up at a barrier: the count reaches G only once every
// workgroup has left the program, so the re-arm never races a live workgroup, and a launch that timed out
// still leaves its slot zero for the launch that is dealt it next (slots are reused round robin)
__device__ __forceinline__ void grid_exit(BarState& b) {
  if (threadIdx.x == 0) {
    unsigned long long* ex = b.cnt + 16;
    const unsigned long long prev = __hip_atomic_fetch_add(ex, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned long long)b.G - 1) {   // every workgroup is past every barrier of this launch
      __hip_atomic_store(b.cnt, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ex, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------ A row tile staging
// The 32 rows [r0, r0 + 32) of the phase's A operand (rows >= rlim read as zero), transformed by the
// phase's mode, into LDS As[row][k] (row stride as, zero for K <= k < Kp).  Thread (row = tid / 8,
// sub = tid % 8) holds columns 4 sub + 32 i.  Every load the staging needs -- the rows, x-hat, 1/std,
// gamma / beta, the position rows -- is issued before any arithmetic (one memory round trip for a
// LayerNorm row of <= 256 columns; plain rows in groups of 384 columns).
// Write duty: columns [wd, wd + 32) of the LN outputs (wd == TOK_DUTY_ALL: every column; wd < 0: none;
// the row scalars with wd == 0 or all).  addpos: stage A' + apos (the query-position operand).
constexpr int NGL = 8;    // float4 groups per thread of a LayerNorm row (K <= 256)
constexpr int NGP = 12;   // ... of a plain row group (384 columns)
constexpr int DUTY_ALL = -2;

__device__ __forceinline__ bool duty_col(int wd, int k) { return wd == DUTY_ALL || (wd >= 0 && (k >> 5) == (wd >> 5)); }

// keep mask of up to 32 dropout draws idx0 + off(e) (one bit each): the hash in a loop that is not
// unrolled (its 64-bit multiplies are long; unrolled per element they were a large share of the code)
__device__ __forceinline__ unsigned keep_bits(unsigned long long seed, unsigned thr, unsigned long long idx0, int n,
                                              int stride4) {
  unsigned km = 0;
#pragma unroll 1
  for (int e = 0; e < n; ++e)
    km |= (fx_drop_bits(seed, idx0 + (unsigned long long)((e >> 2) * stride4 + (e & 3))) >= thr ? 1u : 0u) << e;
  return km;
}
__device__ __forceinline__ float kbit(unsigned km, int e, float scale) { return (km >> e) & 1u ? scale : 0.f; }

// LayerNorm rows, forward (bwd false: the stored rows are the pre-LN sum) or backward (the stored rows
// are dL/d(LN output); x-hat and 1/std read).  addpos: the staged rows get + apos.
__device__ __forceinline__ void stage_ln(const TokPhase& P, bool bwd, int r0, int rlim, float* As, int as, int wd,
                                         bool addpos) {
  const int tid = threadIdx.x, row = tid >> 3, sub = tid & 7;
  const int m = r0 + row, K = P.K;
  const bool mok = m < rlim;
  const int ng = (K + 31) / 32;
  float4 v[NGL], x[NGL], gw[NGL], pp[NGL];
  // unconditional loads from clamped in-range addresses, zeroed by selects after every load has been
  // issued: no branch around a load, so no wait between them.  x: beta (forward) or x-hat (backward);
  // tensors written before the launch (x-hat, 1/std, gamma, beta, positions) take plain loads
  const int mc = min(m, rlim - 1);
  const float* xs = bwd ? P.ln.xhat + (long long)mc * K : P.ln.b;
  const float* ps = addpos ? P.apos + (long long)mc * P.ldpos : P.ln.w;
#pragma unroll
  for (int i = 0; i < NGL; ++i) {
    const int kc = min(4 * sub + 32 * i, K - 4);
    v[i] = ldc4(P.a, (long long)mc * P.lda + kc);
    x[i] = ld4(xs + kc);
    gw[i] = ld4(P.ln.w + kc);
    pp[i] = ld4(ps + kc);
  }
  const float rsb = bwd ? ld1(P.ln.rstd + mc) : 0.f;
#pragma unroll
  for (int i = 0; i < NGL; ++i) {
    const int k = 4 * sub + 32 * i;
    const bool kok = i < ng && k < K, ok = kok && mok;
    v[i] = ok ? v[i] : zero4();
    x[i] = (bwd ? ok : kok) ? x[i] : zero4();
    gw[i] = kok ? gw[i] : zero4();
    pp[i] = (ok && addpos) ? pp[i] : zero4();
  }
  if (!bwd) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NGL; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float mu = rsum8(s) / K;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NGL; ++i) {
      const int k = 4 * sub + 32 * i;
      const bool kok = i < ng && k < K;
      const float a = v[i].x - mu, b = v[i].y - mu, c = v[i].z - mu, d = v[i].w - mu;
      q += kok ? (a * a + b * b) + (c * c + d * d) : 0.f;
    }
    const float rs = rsqrtf(rsum8(q) / K + P.ln.eps);
#pragma unroll
    for (int i = 0; i < NGL; ++i) {
      const int k = 4 * sub + 32 * i;
      if (i < ng && k < K) {
        const float4 g = gw[i], bb = x[i];
        const float4 hh = make_float4((v[i].x - mu) * rs, (v[i].y - mu) * rs, (v[i].z - mu) * rs, (v[i].w - mu) * rs);
        const float4 y = make_float4(hh.x * g.x + bb.x, hh.y * g.y + bb.y, hh.z * g.z + bb.z, hh.w * g.w + bb.w);
        if (mok && duty_col(wd, k)) {
          const long long o = (long long)m * K + k;
          if (P.ln.xh) stc4(P.ln.xh, o, hh);
          if (P.ln.y) stc4(P.ln.y, o, y);
          if (P.ln.y2) stc4(P.ln.y2, o, add4(y, (addpos && P.ln.pos == P.apos) ? pp[i] : ld4(P.ln.pos + o)));
        }
        v[i] = add4(y, pp[i]);
      }
    }
    if (mok && (wd == 0 || wd == DUTY_ALL) && sub == 0 && P.ln.rs) stc1(P.ln.rs, m, rs);
  } else {
    // dR = rstd (g - mean(g) - xhat mean(g xhat)), g = dT w  (rowops ln_bwd);  dU = dR keep / (1 - p)
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NGL; ++i) {
      const float4 g = gw[i];
      v[i] = make_float4(v[i].x * g.x, v[i].y * g.y, v[i].z * g.z, v[i].w * g.w);
      s1 += (v[i].x + v[i].y) + (v[i].z + v[i].w);
      s2 += (v[i].x * x[i].x + v[i].y * x[i].y) + (v[i].z * x[i].z + v[i].w * x[i].w);
    }
    s1 = rsum8(s1) / K;
    s2 = rsum8(s2) / K;
    const bool drop = P.ln.drop_thr != 0;
    const unsigned km = drop ? keep_bits(P.ln.drop_seed, P.ln.drop_thr, (unsigned long long)m * K + 4 * sub,
                                         4 * min(ng, NGL), 32)
                             : ~0u;
    const float dsc = drop ? P.ln.drop_scale : 1.f;
#pragma unroll
    for (int i = 0; i < NGL; ++i) {
      const int k = 4 * sub + 32 * i;
      if (i < ng && k < K) {
        const float4 hh = x[i];
        float4 d = make_float4(rsb * (v[i].x - s1 - hh.x * s2), rsb * (v[i].y - s1 - hh.y * s2),
                               rsb * (v[i].z - s1 - hh.z * s2), rsb * (v[i].w - s1 - hh.w * s2));
        const long long o = (long long)m * K + k;
        const bool duty = mok && duty_col(wd, k);
        if (duty && P.ln.dr) stc4(P.ln.dr, o, d);
        d = make_float4(d.x * kbit(km, 4 * i, dsc), d.y * kbit(km, 4 * i + 1, dsc), d.z * kbit(km, 4 * i + 2, dsc),
                        d.w * kbit(km, 4 * i + 3, dsc));
        if (duty && P.ln.du) stc4(P.ln.du, o, d);
        v[i] = add4(d, pp[i]);
      }
    }
  }
  if (!As) return;
#pragma unroll
  for (int i = 0; i < NGL; ++i) {
    const int k = 4 * sub + 32 * i;
    if (i * 32 < P.Kp) *reinterpret_cast<float4*>(As + row * as + k) = (mok && k < K) ? v[i] : zero4();
  }
}

__device__ __forceinline__ void stage_plain(const TokPhase& P, int r0, int rlim, float* As, int as, int wd, bool addpos) {
  const int tid = threadIdx.x, row = tid >> 3, sub = tid & 7;
  const int m = r0 + row, K = P.K;
  const bool mok = m < rlim;
  for (int c0 = 0; c0 < P.Kp; c0 += 32 * NGP) {
    float4 v[NGP], pp[NGP];
    const int mc = min(m, rlim - 1);
    const float* qp = addpos ? P.apos : P.a;
    const long long qld = addpos ? P.ldpos : P.lda;
#pragma unroll
    for (int i = 0; i < NGP; ++i) {   // (unconditional loads, clamped; zeroed after: see stage_ln)
      const int kc = min(c0 + 4 * sub + 32 * i, K - 4);
      v[i] = ldc4(P.a, (long long)mc * P.lda + kc);
      pp[i] = ld4(qp + (long long)mc * qld + kc);
    }
#pragma unroll
    for (int i = 0; i < NGP; ++i) {
      const int k = c0 + 4 * sub + 32 * i;
      const bool ok = mok && k < K;
      v[i] = ok ? v[i] : zero4();
      pp[i] = (ok && addpos) ? pp[i] : zero4();
    }
#pragma unroll
    for (int i = 0; i < NGP; ++i) {
      const int k = c0 + 4 * sub + 32 * i;
      if (k >= P.Kp) continue;
      // (a plain row's duty: y2 = A + pos, the first layer's saved query operand)
      if (P.ln.y2 && mok && k < K && duty_col(wd, k)) {
        const long long o = (long long)m * K + k;
        stc4(P.ln.y2, o, add4(v[i], ld4(P.ln.pos + o)));
      }
      if (As) *reinterpret_cast<float4*>(As + row * as + k) = add4(v[i], pp[i]);
    }
  }
}

__device__ __forceinline__ void stage_rows(const TokPhase& P, int r0, int rlim, float* As, int as, int wd, bool addpos) {
  if (P.amode == TOK_A_PLAIN) stage_plain(P, r0, rlim, As, as, wd, addpos);
  else stage_ln(P, P.amode == TOK_A_LNBWD, r0, rlim, As, as, wd, addpos);
}

// ------------------------------------------------------------------ 32 x 32 products
// acc += A[li][k] (LDS, row stride as) B[k][n] over this lane half's half of [k0, k0 + kw) (kw % 8 == 0):
// B = W[n][k] (!BT: a float4 along k per lane) or W[k][n] (BT, the dX products: per k one coalesced 4-B
// load per lane).  B loads go out in groups of NGB float4 (32 registers), all of a group before its
// first product.
constexpr int NGB = 8;
template <bool BT>
__device__ __forceinline__ void load_b(const float* W, long long ldw, int n, bool nok, int K, int kb, int ng,
                                       float4* b) {
  // unconditional loads from clamped addresses (n is clamped by the caller), zeroed after: no branch
  // around a load
#pragma unroll
  for (int g = 0; g < NGB; ++g) {
    const int k = kb + 4 * g, kc = min(k, K - 4);
    if (!BT) {
      b[g] = ld4(W + (long long)n * ldw + kc);
    } else {
      b[g] = make_float4(ld1(W + (long long)kc * ldw + n), ld1(W + (long long)(kc + 1) * ldw + n),
                         ld1(W + (long long)(kc + 2) * ldw + n), ld1(W + (long long)(kc + 3) * ldw + n));
    }
  }
  // no zeroing: a clamped k >= K re-reads an in-range weight that meets a zero A column (As is zero for
  // K <= k < Kp), and a clamped column n >= N is never stored; so nothing here waits for the loads
}

__device__ __forceinline__ void mma_groups(const float* arow, int kb, int ng, const float4* b, f32x16& acc) {
#pragma unroll
  for (int g = 0; g < NGB; ++g) {
    if (g < ng) {
      const float4 a = *reinterpret_cast<const float4*>(arow + kb + 4 * g);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[g].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[g].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[g].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[g].w, acc, 0, 0, 0);
    }
  }
}

// the whole product over this lane half's range [kb, kb + 4 ng): the first group's B loads were issued
// by the caller (b), later groups here
template <bool BT>
__device__ __forceinline__ void mma_range(const float* arow, const float* W, long long ldw, int n, bool nok, int K,
                                          int kb, int ng, float4* b, f32x16& acc) {
  mma_groups(arow, kb, min(ng, NGB), b, acc);
  for (int g0 = NGB; g0 < ng; g0 += NGB) {
    load_b<BT>(W, ldw, n, nok, K, kb + 4 * g0, ng - g0, b);
    mma_groups(arow, kb + 4 * g0, min(ng - g0, NGB), b, acc);
  }
}

// sum the 4 waves' partial tiles (LDS red[4][16][64]) in wave order: thread (wave rq, lane) gets the
// accumulator elements 4 rq .. 4 rq + 3 of `lane`: rows 8 rq + 4 (lane >> 5) + 0..3, column lane & 31
__device__ __forceinline__ void red_store(float* red, const f32x16& acc, int w, int lane) {
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc[r];
}
__device__ __forceinline__ float red_sum(const float* red, int r, int lane) {
  return (red[(0 * 16 + r) * 64 + lane] + red[(1 * 16 + r) * 64 + lane]) +
         (red[(2 * 16 + r) * 64 + lane] + red[(3 * 16 + r) * 64 + lane]);
}

// ------------------------------------------------------------------ GEMM phase
// Per item: the B loads, the epilogue operands (bias, residual, gate of this thread's 4 outputs) and the
// staging loads all go out before the first product, so an item costs about one memory round trip.
__device__ __forceinline__ void gemm_phase(const TokPhase& P, float* lds, int G, unsigned long long* st) {
  const int sit = (int)blockIdx.x + (st && st[7] == 3 ? G : 0);   // diagnostic: FX_TOK_DEBUG=3 stamps the second item
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nrt = (P.M + 31) / 32, nct = (P.N + 31) / 32, nitems = nrt * nct;
  const int as = P.Kp + 4;
  float* As = lds;
  float* red = lds + 32 * as;
  const int kw = P.Kp / 4, kh = kw / 2, ngb = kh / 4;   // each wave's k range; per lane half; float4 groups
  const bool duty = P.amode != TOK_A_PLAIN || P.ln.y2;
  for (int it = blockIdx.x; it < nitems; it += G) {
    lds_sync();   // As / red of the previous item are free: before any load of this item, so the B
                       // loads, the epilogue operands and the staging loads are one round trip
    tstamp(it == sit ? st : nullptr, 4);
    const int rt = it / nct, ct = it - rt * nct;
    const int r0 = rt * 32, n0 = ct * 32;
    const int n = n0 + (lane & 31), nc = min(n, P.N - 1);
    const int kb = w * kw + (lane >> 5) * kh;
    const bool nok = n < P.N;
    float4 b[NGB];
    if (P.btrans) load_b<true>(P.w, P.ldw, nc, nok, P.K, kb, ngb, b);
    else load_b<false>(P.w, P.ldw, nc, nok, P.K, kb, ngb, b);
    tstamp(it == sit ? st : nullptr, 6);
    // this thread's outputs: rows r0 + acc_row(4 w + j, lane), column n; their epilogue operands loaded
    // unconditionally (clamped; stand-ins for absent operands) beside the B loads
    const float* rp = P.resid ? P.resid : P.c;
    const long long rld = P.resid ? P.ldr : P.ldc;
    const float* gp = P.gate ? P.gate : P.c;
    const long long gld = P.gate ? P.ldg : P.ldc;
    float ebias = ld1((P.bias ? P.bias : P.w) + nc), eres[4], egate[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int mc = min(r0 + acc_row(4 * w + j, lane), P.M - 1);
      eres[j] = ldc1(rp, (long long)mc * rld + nc);
      egate[j] = ldc1(gp, (long long)mc * gld + nc);
    }
    tstamp(it == sit ? st : nullptr, 2);
    stage_rows(P, r0, P.M, As, as, duty && n0 < P.K ? n0 : -1, P.apos && n0 < P.apos_ncols);
    tstamp(it == sit ? st : nullptr, 3);
    lds_sync();
    f32x16 acc;
    zero16(acc);
    if (P.btrans) mma_range<true>(As + (lane & 31) * as, P.w, P.ldw, nc, nok, P.K, kb, ngb, b, acc);
    else mma_range<false>(As + (lane & 31) * as, P.w, P.ldw, nc, nok, P.K, kb, ngb, b, acc);
    red_store(red, acc, w, lane);
    tstamp(it == sit ? st : nullptr, 5);
    lds_sync();
    // this thread's 4 rows are consecutive: m0 + j (acc_row(4 w + j, lane))
    const int m0 = r0 + acc_row(4 * w, lane);
    unsigned km = ~0u;
    if (P.drop_thr) {
      km = 0;
#pragma unroll 1
      for (int j = 0; j < 4; ++j)
        km |= (fx_drop_bits(P.drop_seed, (unsigned long long)(m0 + j) * P.N + n) >= P.drop_thr ? 1u : 0u) << j;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * w + j;
      float v = red_sum(red, r, lane);
      const int m = r0 + acc_row(r, lane);
      if (m >= P.M || !nok) continue;
      v = v * P.alpha + (P.bias ? ebias : 0.f);
      if (P.relu == 2) v = fmaxf(v, 0.f);
      if (P.drop_thr) v *= kbit(km, j, P.drop_scale);
      if (P.resid) v += eres[j];
      if (P.gate && !(egate[j] > 0.f)) v = 0.f;
      if (P.relu == 1) v = fmaxf(v, 0.f);
      stc1(P.c, (long long)m * P.ldc + n, v);
    }
    tstamp(it == sit ? st : nullptr, 7);
  }
}

// ------------------------------------------------------------------ LN rows phase (outputs only)
__device__ __forceinline__ void ln_phase(const TokPhase& P, int G) {
  const int nrt = (P.M + 31) / 32;
  for (int it = blockIdx.x; it < nrt; it += G) stage_rows(P, it * 32, P.M, nullptr, 0, DUTY_ALL, false);
}

// LDS 32 x 32 x 32 product on the matrix cores (wave-level): acc += A B, A / B row-major or transposed
template <bool ATR, bool BTR>
__device__ __forceinline__ void mm32s(const float* a, int lda, const float* b, int ldb, f32x16& acc, int lane) {
  const int li = lane & 31, kh = (lane >> 5) * 16;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int k = kh + j;
    const float x = ATR ? a[k * lda + li] : a[li * lda + k];
    const float y = BTR ? b[li * ldb + k] : b[k * ldb + li];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc, 0, 0, 0);
  }
}

// ------------------------------------------------------------------ self-attention forward item
// (video v, head h), Qv <= 32 tokens, head dim 32: stage the video's rows (LN on load, this head's
// columns of the LN outputs written), v_h = x W_v,h^T + b from the staged rows, then (rows + query
// position, added in place: (x + p) computed once, as a staged x + p would be) for q_h and k_h; each
// product K-split over the 4 waves with every B load issued up front; then S = scale q k^T and
// O = P_d V on the matrix cores, the row softmax (probabilities saved before the dropout) in between.
__device__ __forceinline__ void safwd_phase(const TokPhase& P, float* lds, int G, unsigned long long* st) {
  const int sit = (int)blockIdx.x + (st && st[7] == 3 ? G : 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nh = P.nh, Qv = P.Qv, A = P.K, nitems = P.nvid * nh;
  const int as = P.Kp + 4;
  float* As = lds;                                  // [32][as]
  float* red = As + 32 * as;                        // [3][4][16][64]
  float* Qs = red + 3 * 4 * 1024;                   // [32][HS] each
  float* Ks = Qs + 32 * HS;
  float* Vs = Ks + 32 * HS;
  float* Ps = Vs + 32 * HS;
  const int kw = P.Kp / 4, kh = kw / 2, ngb = kh / 4;   // <= 8 groups (A <= 256)
  const int c = lane & 31, kb = w * kw + (lane >> 5) * kh;
  const bool qpos = P.apos != nullptr;
  for (int it = blockIdx.x; it < nitems; it += G) {
    const int v = it / nh, h = it - v * nh;
    const int R0 = v * Qv;
    // every load of the item up front: the head's q / k / v weight fragments and the query-position
    // fragments (rows of this lane, its k range) that q and k add to the staged rows
    // (v weights and the position fragments before the staging, q / k weights after it: registers)
    float4 bq[8], bk[8], bv[8], pq[8];
    const int prow = R0 + min(c, Qv - 1);
    lds_sync();   // LDS of the previous item is free (before this item's loads)
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const long long k = min(kb + 4 * g, A - 4);
      bv[g] = ld4(P.w + (long long)(2 * A + h * 32 + c) * P.ldw + k);
      pq[g] = ld4((qpos ? P.apos + (long long)prow * P.ldpos : P.w) + k);
    }
    const float* bp = P.bias ? P.bias : P.w;
    float bb3[3];
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) bb3[mat] = ld1(bp + mat * A + h * 32 + c);
    tstamp(it == sit ? st : nullptr, 2);
    stage_rows(P, R0, R0 + Qv, As, as, P.amode == TOK_A_PLAIN && !P.ln.y2 ? -1 : h * 32, false);
    tstamp(it == sit ? st : nullptr, 3);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const long long k = min(kb + 4 * g, A - 4);
      bq[g] = ld4(P.w + (long long)(h * 32 + c) * P.ldw + k);
      bk[g] = ld4(P.w + (long long)(A + h * 32 + c) * P.ldw + k);
    }
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const bool ok = g < ngb;
      bq[g] = ok ? bq[g] : zero4();
      bk[g] = ok ? bk[g] : zero4();
      bv[g] = ok ? bv[g] : zero4();
      pq[g] = (ok && qpos && c < Qv) ? pq[g] : zero4();
    }
    lds_sync();
    f32x16 av, aq, ak;
    zero16(av);
    zero16(aq);
    zero16(ak);
    {
      const float* arow = As + c * as + kb;
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        if (g < ngb) {
          const float4 a = *reinterpret_cast<const float4*>(arow + 4 * g);
          const float4 ap = add4(a, pq[g]);   // (rows + query position; zero position rows without one)
          av = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bv[g].x, av, 0, 0, 0);
          aq = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.x, bq[g].x, aq, 0, 0, 0);
          ak = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.x, bk[g].x, ak, 0, 0, 0);
          av = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bv[g].y, av, 0, 0, 0);
          aq = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.y, bq[g].y, aq, 0, 0, 0);
          ak = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.y, bk[g].y, ak, 0, 0, 0);
          av = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bv[g].z, av, 0, 0, 0);
          aq = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.z, bq[g].z, aq, 0, 0, 0);
          ak = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.z, bk[g].z, ak, 0, 0, 0);
          av = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bv[g].w, av, 0, 0, 0);
          aq = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.w, bq[g].w, aq, 0, 0, 0);
          ak = __builtin_amdgcn_mfma_f32_32x32x2f32(ap.w, bk[g].w, ak, 0, 0, 0);
        }
      }
    }
    red_store(red, aq, w, lane);
    red_store(red + 4096, ak, w, lane);
    red_store(red + 8192, av, w, lane);
    tstamp(it == sit ? st : nullptr, 4);
    lds_sync();
#pragma unroll
    for (int mat = 0; mat < 3; ++mat) {
      float* dst = mat == 0 ? Qs : mat == 1 ? Ks : Vs;
      const int n = mat * A + h * 32 + c;
      const float bb = P.bias ? bb3[mat] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * w + j, row = acc_row(r, lane);
        const float x = red_sum(red + mat * 4096, r, lane) + bb;
        dst[row * HS + c] = row < Qv ? x : 0.f;
        if (row < Qv) st1(P.qkv + (long long)(R0 + row) * 3 * A + n, x);   // saved for the backward
      }
    }
    lds_sync();
    if (w == 0) {   // S = scale q k^T
      f32x16 sacc;
      zero16(sacc);
      mm32s<false, true>(Qs, HS, Ks, HS, sacc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) Ps[acc_row(r, lane) * HS + c] = sacc[r] * P.scale;
    }
    lds_sync();
    tstamp(it == sit ? st : nullptr, 5);
    float* probs = P.probs + (long long)v * nh * Qv * Qv;
#pragma unroll 1
    for (int i = w; i < 32; i += 4) {
      const float x = (lane < Qv && i < Qv) ? Ps[i * HS + lane] : -INFINITY;
      const float mx = wmax(x);
      const float ex = lane < Qv ? __expf(x - mx) : 0.f;
      const float p = ex / wsum(ex);
      float pd = 0.f;
      if (lane < Qv && i < Qv) {
        st1(probs + ((long long)h * Qv + i) * Qv + lane, p);   // saved before the dropout (the backward redraws it)
        pd = p;
        if (P.attn_thr) {   // mha_small's mask: index (query_row * nh + h) * (nvid Qv) + key_row
          const unsigned long long qg = (unsigned long long)v * Qv + i, kg = (unsigned long long)v * Qv + lane;
          pd = p * keepf(P.attn_seed, P.attn_thr, P.attn_scale, (qg * nh + h) * ((unsigned long long)P.nvid * Qv) + kg);
        }
      }
      if (lane < 32) Ps[i * HS + lane] = pd;
    }
    lds_sync();
    tstamp(it == sit ? st : nullptr, 6);
    if (w == 0) {   // O = P_d V
      f32x16 o;
      zero16(o);
      mm32s<false, false>(Ps, HS, Vs, HS, o, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = acc_row(r, lane);
        if (i < Qv) stc1(P.c, (long long)(R0 + i) * P.ldc + h * 32 + c, o[r]);
      }
    }
    tstamp(it == sit ? st : nullptr, 7);
  }
}

// ------------------------------------------------------------------ self-attention backward item
// mha_small_bwd_kernel's algebra for one (video, head) on the matrix cores: dP = dO V^T (through the
// dropout mask), dV = P_d^T dO, dS = P (dP - rowsum(P dP)), dq = scale dS K, dk = scale dS^T q
// -> [dq | dk | dv] columns of the head.
__device__ __forceinline__ void mhabwd_phase(const TokPhase& P, float* lds, int G) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nh = P.nh, Qv = P.Qv, A = P.K, nitems = P.nvid * nh;
  float* Qs = lds;
  float* Ks = Qs + 32 * HS;
  float* Vs = Ks + 32 * HS;
  float* Ps = Vs + 32 * HS;   // P, then P_d
  float* Ds = Ps + 32 * HS;   // dO
  float* Gs = Ds + 32 * HS;   // dP (masked), then dS
  float* Ms = Gs + 32 * HS;   // keep-scales
  float* Us = Ms + 32 * HS;   // the un-dropped P
  const bool drop = P.attn_thr != 0;
  const int c = lane & 31;
  for (int it = blockIdx.x; it < nitems; it += G) {
    const int v = it / nh, h = it - v * nh;
    const int R0 = v * Qv;
    const float* probs = P.probs + ((long long)v * nh + h) * Qv * Qv;
    lds_sync();
    {   // the head's q, k, v, dO and P tiles: 4 elements per thread each, every load issued first (clamped)
      float q4[4], k4[4], v4[4], d4[4], p4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + u * TT, i = e >> 5, d = e & 31;
        const int ic = min(i, Qv - 1), dc = min(d, Qv - 1);
        const long long row = (long long)(R0 + ic) * 3 * A + h * 32 + d;
        q4[u] = ld1(P.qkv + row);
        k4[u] = ld1(P.qkv + row + A);
        v4[u] = ld1(P.qkv + row + 2 * A);
        d4[u] = ldc1(P.a, (long long)(R0 + ic) * P.lda + h * 32 + d);   // dO of the head
        p4[u] = ld1(probs + ic * Qv + dc);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + u * TT, i = e >> 5, d = e & 31;
        const bool ok = i < Qv, pk = i < Qv && d < Qv;
        Qs[i * HS + d] = ok ? q4[u] : 0.f;
        Ks[i * HS + d] = ok ? k4[u] : 0.f;
        Vs[i * HS + d] = ok ? v4[u] : 0.f;
        Ds[i * HS + d] = ok ? d4[u] : 0.f;
        Ps[i * HS + d] = pk ? p4[u] : 0.f;
        float kp = 1.f;
        if (drop && pk) {
          const unsigned long long qg = (unsigned long long)v * Qv + i, kg = (unsigned long long)v * Qv + d;
          kp = keepf(P.attn_seed, P.attn_thr, P.attn_scale, (qg * nh + h) * ((unsigned long long)P.nvid * Qv) + kg);
        }
        Ms[i * HS + d] = kp;
      }
    }
    lds_sync();
    if (w == 0) {   // dP = dO V^T (masked)
      f32x16 acc;
      zero16(acc);
      mm32s<false, true>(Ds, HS, Vs, HS, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = acc_row(r, lane);
        Gs[i * HS + c] = acc[r] * Ms[i * HS + c];
      }
    } else if (w == 1) {   // dV = P_d^T dO
      for (int e = lane; e < 32 * 32; e += 64) {
        const int i = e >> 5, j = e & 31;
        Us[i * HS + j] = Ps[i * HS + j];     // the un-dropped P for dS (only this wave touches Ps / Us here)
        Ps[i * HS + j] *= Ms[i * HS + j];
      }
      f32x16 acc;
      zero16(acc);
      mm32s<true, false>(Ps, HS, Ds, HS, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = acc_row(r, lane);
        if (j < Qv) stc1(P.c, (long long)(R0 + j) * P.ldc + 2 * A + h * 32 + c, acc[r]);
      }
    }
    lds_sync();
    // dS = P (dP - rowsum(P dP)) with the un-dropped P (Us: wave 1 turned Ps into P_d)
    for (int i = w; i < 32; i += 4) {
      const float p = lane < 32 ? Us[i * HS + lane] : 0.f;
      const float g = lane < 32 ? Gs[i * HS + lane] : 0.f;
      const float r = wsum(p * g);
      if (lane < 32) Gs[i * HS + lane] = p * (g - r);
    }
    lds_sync();
    if (w < 2) {   // dq = scale dS K ; dk = scale dS^T q
      f32x16 acc;
      zero16(acc);
      if (w == 0) mm32s<false, false>(Gs, HS, Ks, HS, acc, lane);
      else mm32s<true, false>(Gs, HS, Qs, HS, acc, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = acc_row(r, lane);
        if (i < Qv) stc1(P.c, (long long)(R0 + i) * P.ldc + w * A + h * 32 + c, acc[r] * P.scale);
      }
    }
  }
}

__global__ __launch_bounds__(TT) void tok_kernel(TokProgram prog) {
  extern __shared__ float lds[];
  __shared__ int dead;
  if (threadIdx.x == 0) dead = 0;
  __syncthreads();
  BarState b{prog.bar, 0ull, prog.status, prog.spin_max, prog.G};
  // the phases are read in place from the kernel-argument segment (indexing prog.ph with the loop
  // counter would copy the whole program into scratch)
#if defined(__HIP_DEVICE_COMPILE__)
  const TokProgram* pk = (const TokProgram*)(__builtin_amdgcn_kernarg_segment_ptr());
#else
  const TokProgram* pk = &prog;
#endif
  // The phases go to LDS once (vector loads by the whole workgroup, one round trip), and each phase from
  // there into registers, made wave-uniform (readfirstlane).  Read in place, the fields are scalar loads
  // from the argument segment that the compiler re-issues wherever it runs short of scalar registers
  // (rather than spilling them), and those reads are slow: chains of them cost microseconds per item.
  static_assert(sizeof(TokPhase) % 4 == 0, "phase copy by words");
  constexpr int kPW = (int)(sizeof(TokPhase) / 4);
  __shared__ unsigned sph[TOK_MAXPH * kPW];
  {
    const unsigned* src = reinterpret_cast<const unsigned*>(pk->ph);
    for (int i = threadIdx.x; i < prog.nphase * kPW; i += TT) sph[i] = src[i];
  }
  // diagnostic stamps (FX_TOK_DEBUG): kept in LDS (a global store at a phase start would put its
  // write acknowledgement in front of the phase's first wait), written out at the end
  __shared__ unsigned long long tst[TOK_MAXPH * 8];
  if (prog.debug && threadIdx.x < TOK_MAXPH * 8) tst[threadIdx.x] = 0;
  __syncthreads();
  for (int p = 0; p < prog.nphase; ++p) {
    TokPhase P;
    {
      unsigned* dst = reinterpret_cast<unsigned*>(&P);
#pragma unroll
      for (int i = 0; i < kPW; ++i) dst[i] = __builtin_amdgcn_readfirstlane(sph[p * kPW + i]);
    }
    unsigned long long* st = prog.debug ? tst + p * 8 : nullptr;
    if (st && threadIdx.x == 0) st[7] = prog.debug;
    __syncthreads();
    tstamp(st, 0);
    if (P.op == TOK_GEMM) gemm_phase(P, lds, prog.G, st);
    else if (P.op == TOK_SAFWD) safwd_phase(P, lds, prog.G, st);
    else if (P.op == TOK_MHABWD) mhabwd_phase(P, lds, prog.G);
    else if (P.op == TOK_LNROWS) ln_phase(P, prog.G);
    if (prog.debug) {
      __syncthreads();
      tstamp(st, 1);
    }
    if (p + 1 < prog.nphase && !grid_sync(b, &dead)) break;
  }
  if (prog.debug && !dead) {
    __syncthreads();
    if (threadIdx.x < prog.nphase * 8) prog.stamps[blockIdx.x * TOK_MAXPH * 8 + threadIdx.x] = tst[threadIdx.x];
  }
  grid_exit(b);
}

// per (device, stream) pool of barrier slots (zeroed once; every slot re-armed by its own launch's last
// workgroup), dealt round robin
constexpr int kTokSlots = 512;
struct TokPool {
  unsigned long long* mem = nullptr;
  unsigned next = 0;
};

}  // namespace

size_t tok_lds_bytes() {
  const size_t gemm = sizeof(float) * (32 * (TOK_MAXK + 4) + 4 * 1024);
  const size_t sa = sizeof(float) * (32 * (TOK_MAXSA + 4) + 3 * 4 * 1024 + 4 * 32 * HS);
  const size_t bwd = sizeof(float) * (8 * 32 * HS);
  return std::max(gemm, std::max(sa, bwd));
}

int launch_tok(TokProgram& prog, hipStream_t s) {
  FX_REQUIRE(prog.nphase >= 1 && prog.nphase <= TOK_MAXPH && prog.G >= 1 && prog.G <= 256, "tok: bad program");
  // the grid barriers need every workgroup resident at once: cap the grid by the occupancy calculator's
  // bound on this device (one workgroup per CU with this LDS size); the phases loop over their items
  static const int resident = coresident_blocks((const void*)tok_kernel, TT, tok_lds_bytes());
  FX_REQUIRE(resident >= 1, "tok: the token kernel cannot be resident on this device");
  prog.G = std::min(prog.G, resident);
  for (int i = 0; i < prog.nphase; ++i) {
    const TokPhase& P = prog.ph[i];
    FX_REQUIRE(P.K >= 4 && P.K % 4 == 0 && P.Kp % 32 == 0 && P.Kp >= P.K && P.Kp <= TOK_MAXK && P.M >= 1,
               "tok: phase K must be a multiple of 4 within the LDS row tile");
    FX_REQUIRE(P.amode == TOK_A_PLAIN || P.K <= 256, "tok: LayerNorm rows of at most 256 columns");
    if (P.op == TOK_SAFWD || P.op == TOK_MHABWD)
      FX_REQUIRE(P.Qv >= 1 && P.Qv <= 32 && P.nh * 32 == P.K && P.K <= TOK_MAXSA, "tok: attention items need head dim 32, <= 32 tokens");
  }
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, TokPool> pools;
  int dev = 0;
  FX_CHECK_HIP(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lk(mu);
    TokPool& pool = pools[std::make_pair(dev, s)];
    if (!pool.mem) {
      const size_t bytes = (size_t)kTokSlots * 256;   // two 128-B lines per slot
      FX_CHECK_HIP(hipMalloc(&pool.mem, bytes));
      FX_CHECK_HIP(hipMemsetAsync(pool.mem, 0, bytes, s));
    }
    prog.bar = pool.mem + (size_t)(pool.next % kTokSlots) * 32;
    pool.next++;
  }
  static const bool attr = [] {
    return hipFuncSetAttribute((const void*)tok_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)tok_lds_bytes()) == hipSuccess;
  }();
  FX_REQUIRE(attr, "tok: cannot raise the LDS limit");
  prog.debug = std::getenv("FX_TOK_DEBUG") ? std::atoi(std::getenv("FX_TOK_DEBUG")) : 0;
  static unsigned long long* dstamps = nullptr;
  if (prog.debug && !dstamps) FX_CHECK_HIP(hipMalloc(&dstamps, 256 * TOK_MAXPH * 8 * sizeof(unsigned long long)));
  if (dstamps) (void)hipMemsetAsync(dstamps, 0, 256 * TOK_MAXPH * 8 * sizeof(unsigned long long), s);
  prog.stamps = dstamps;
  fx_launch(tok_kernel, dim3(prog.G), dim3(TT), tok_lds_bytes(), s, prog);
  FX_CHECK_HIP(hipGetLastError());
  if (prog.debug) {   // diagnostic: synchronous launch + program summary on stderr
    const hipError_t e = hipStreamSynchronize(s);
    std::fprintf(stderr, "tok: G %d phases %d lds %zu sync %s\n", prog.G, prog.nphase, tok_lds_bytes(), hipGetErrorString(e));
    static unsigned long long h[256 * TOK_MAXPH * 8];
    (void)hipMemcpy(h, dstamps, sizeof(h), hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull;
    for (int g = 0; g < prog.G; ++g) t0 = std::min(t0, h[(g * TOK_MAXPH) * 8]);
    for (int i = 0; i < prog.nphase; ++i) {
      const TokPhase& P = prog.ph[i];
      unsigned long long s0 = ~0ull, s1 = 0, e1 = 0;
      double in[6] = {0, 0, 0, 0, 0, 0};
      for (int g = 0; g < prog.G; ++g) {
        const unsigned long long* q = h + (g * TOK_MAXPH + i) * 8;
        s0 = std::min(s0, q[0]);
        s1 = std::max(s1, q[0]);
        e1 = std::max(e1, q[1]);
        for (int k = 0; k < 6; ++k)
          if (q[2 + k]) in[k] = std::max(in[k], (q[2 + k] - q[0]) / 100.0);
      }
      // (s_memrealtime: 100 MHz)
      std::fprintf(stderr, "  ph %d op %d amode %d M %d N %d K %d: start %.2f..%.2f us, work done %.2f us; first item "
                   "(max over wg, from its phase start) %.2f %.2f %.2f %.2f %.2f %.2f\n", i, P.op,
                   P.amode, P.M, P.N, P.K, (s0 - t0) / 100.0, (s1 - t0) / 100.0, (e1 - t0) / 100.0, in[0], in[1], in[2],
                   in[3], in[4], in[5]);
    }
  }
  return FX_OK;
}

}  // namespace fx
