// f32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32 products,
// k-ordered fma chain; no xf32 on gfx950, so the parity path stays fp32).
//
// One kernel template covers every dense contraction of the FACT frame/action
// branches; the operand loader is specialised at compile time:
//   ROWS      element (r,k) = p[r*ld + k]            Linear/Conv1d(k=1) fwd, B = W
//   ROWS_CONV implicit dilated Conv1d(k=3): row r shifted by the tap of k, zero
//             outside the video (fwd and, with reversed taps, dX)
//   ROWS_GEN  concatenated inputs / row gathers / positional adds (generic)
//   COLS      element (r,k) = p[k*ld + r]            dY^T for dW, W^T for dX
//   COLS_CONV conv input for dW, tap from r; optional all-ones row (bias grad)
// Tile: 64x64 output per 256-thread workgroup (4 waves x 32x32 accumulator,
// 16 f32 per lane), K staged through LDS in 32-deep slices with a register
// prefetch of the next slice (one barrier per slice).  All per-thread address
// arithmetic is hoisted out of the K loop; inside it only pointer increments,
// a tap lookup on uniform values, and two float4 loads per operand remain.
// LDS images are [k][row] with a +1 pad: MFMA operand reads are ds_read_b32 of
// 32 consecutive rows (conflict-free), staging writes at most 2-way.
// Blocks are remapped so that consecutive output tiles share an XCD (L2).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "fx_common.h"

namespace fx {
namespace {

// BK: K depth per LDS stage (one barrier per 32 MFMAs per wave); loaders move it in
// two BKH-deep halves (8 elements per thread each).
constexpr int BM = 64, BN = 64, BK = 64, BKH = 32, NTHREADS = 512, LDSS = 65;
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum Kind { ROWS = 0, ROWS_CONV = 1, ROWS_GEN = 2, COLS = 3, COLS_CONV = 4 };

struct GemmDev {
  int M, N, K;
  fx_operand a, b;
  float* c;
  long long ldc, c_bs;
  float alpha, beta;
  const float* bias;
  const float* resid;
  long long ld_resid, resid_bs;
  const float* gate;
  long long ld_gate;
  int relu, split, kt_per_split, a_vec, b_vec, c_tap_cin;
  float* ws;
  float* c_last;
  int tiles_x, tiles_y;
  long long* stamps;
  unsigned* tile_cnt;   // split-K arrival counters (one per output tile), NULL -> separate reduce kernel
};

// Diagnostic builds (-DFX_STAMPS) record s_memtime / s_memrealtime at fixed points of
// every block; the shipped library compiles the macro to nothing.
#ifdef FX_STAMPS
#define FX_STAMP(g, slot)                                                                          \
  do {                                                                                            \
    if ((g).stamps && (threadIdx.x & 255) == 0) {                                                 \
      const long long _b = (long long)blockIdx.z * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + \
                           blockIdx.x;                                                            \
      (g).stamps[(_b * 2 + (threadIdx.x >> 8)) * 10 + 2 * (slot)] = __builtin_amdgcn_s_memtime();    \
      (g).stamps[(_b * 2 + (threadIdx.x >> 8)) * 10 + 2 * (slot) + 1] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                             \
  } while (0)
#else
#define FX_STAMP(g, slot) \
  do {                    \
  } while (0)
#endif

__device__ __forceinline__ int conv_shift(const fx_operand& o, int tap) {
  return (tap - (o.conv_taps - 1) / 2) * o.conv_dil * o.conv_dir;
}

// ---------------------------------------------------------------- generic element fetch
__device__ __forceinline__ float fetch_rm(const fx_operand& o, const float* p0, int r, int k) {
  if (o.conv_taps) {
    const int j = k / o.conv_cin, c = k - j * o.conv_cin, s = conv_shift(o, j);
    const int t = r % o.seq_len + s;
    if (t < 0 || t >= o.seq_len) return 0.f;
    return p0[(long long)(r + s) * o.ld + c];
  }
  if (o.ptr1 && k >= o.k_split) {
    const int rr = o.rows1 ? o.rows1[r] : r;
    return o.ptr1[(long long)rr * o.ld1 + (k - o.k_split)];
  }
  const int rr = o.rows0 ? o.rows0[r] : r;
  float v = p0[(long long)rr * o.ld + k];
  if (o.pos && k < o.pos_cols) v += o.pos[(long long)r * o.ld_pos + k];
  return v;
}

__device__ __forceinline__ float fetch_cm(const fx_operand& o, const float* p0, int r, int k) {
  if (o.ones_col && r == o.ones_col - 1) return 1.f;
  if (o.conv_taps) {
    const int j = r / o.conv_cin, c = r - j * o.conv_cin, s = conv_shift(o, j);
    const int t = k % o.seq_len + s;
    if (t < 0 || t >= o.seq_len) return 0.f;
    return p0[(long long)(k + s) * o.ld + c];
  }
  return p0[(long long)k * o.ld + r];
}

__device__ __forceinline__ void zero8(float* v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
}

__device__ __forceinline__ void ld8(const float* src, float* v) {
  const float4 x0 = *reinterpret_cast<const float4*>(src);
  const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
  v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
  v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
}

// ---------------------------------------------------------------- loaders
// Each thread owns 8 elements of the 64 x 32 (rows x k) tile:
//   row-major kinds: row = tid/4, k = (tid%4)*8 .. +7
//   col-major kinds: row = (tid%8)*8 .. +7, k = tid/8
// The fast path is chosen per TILE with a wave-uniform condition (whole 64-row
// tile and 32-deep slice in range, 16-B aligned, no ones row) so the prefetch
// loads are straight-line code: divergent bounds branches would make the
// compiler drain vmcnt between the A and B prefetches.  Per-row validity of the
// conv gather is a select, not a branch.  Edge tiles take the generic path.
template <int KIND>
struct Loader {
  const fx_operand* o;
  const float* base;  // operand base incl. batch offset
  int R, K;
  bool tile_fast;     // uniform: rows of this tile all in range, operand vector-loadable
  int r;              // row (row-major) or first row of the 8-chunk (col-major)
  int kk;             // k offset inside the tile
  int rmod;           // r % seq_len (ROWS_CONV)
  int tapc, tap_s;    // COLS_CONV: channel and shift of this thread's rows

  __device__ __forceinline__ void init(const fx_operand& op, const float* p0, int r0, int R_, int K_, bool v, int tid) {
    o = &op;
    base = p0;
    R = R_;
    K = K_;
    tile_fast = v && (r0 + 64 <= R_) && !(op.ones_col && r0 + 64 >= op.ones_col);
    if (KIND <= ROWS_GEN) {
      r = r0 + (tid >> 2);
      kk = (tid & 3) * 8;
      if (KIND == ROWS_CONV) rmod = r % op.seq_len;
    } else {
      r = r0 + (tid & 7) * 8;
      kk = tid >> 3;
      if (KIND == COLS_CONV) {
        const int j = r / op.conv_cin;
        tapc = r - j * op.conv_cin;
        tap_s = conv_shift(op, j);
      }
    }
  }

  __device__ __forceinline__ void load_generic(int k0, float* v) const {
    if (KIND <= ROWS_GEN) {
      const int k = k0 + kk;
      if (r >= R) {
        zero8(v);
        return;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (k + e < K) ? fetch_rm(*o, base, r, k + e) : 0.f;
    } else {
      const int k = k0 + kk;
      if (k >= K) {
        zero8(v);
        return;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (r + e < R) ? fetch_cm(*o, base, r + e, k) : 0.f;
    }
  }

  __device__ __forceinline__ void load(int k0, float* v) const {
    const bool fast = tile_fast && (k0 + BKH <= K);
    if (KIND == ROWS_GEN || !fast) {
      load_generic(k0, v);
      return;
    }
    if (KIND == ROWS) {
      ld8(base + (long long)r * o->ld + k0 + kk, v);
    } else if (KIND == ROWS_CONV) {
      // the 32-deep slice lies in one tap (conv_cin % 32 == 0, checked on the host)
      const int j = k0 / o->conv_cin;
      const int c = k0 - j * o->conv_cin + kk;
      const int s = conv_shift(*o, j);
      const int t = rmod + s;
      const bool ok = t >= 0 && t < o->seq_len;
      ld8(base + (long long)(ok ? r + s : r) * o->ld + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ok ? v[e] : 0.f;
    } else if (KIND == COLS) {
      ld8(base + (long long)(k0 + kk) * o->ld + r, v);
    } else {  // COLS_CONV
      const int k = k0 + kk;
      const int t = k % o->seq_len + tap_s;
      const bool ok = t >= 0 && t < o->seq_len;
      ld8(base + (long long)(ok ? k + tap_s : k) * o->ld + tapc, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ok ? v[e] : 0.f;
    }
  }

  __device__ __forceinline__ void store(float (*s)[LDSS], int tid, const float* v) const {
    if (KIND <= ROWS_GEN) {
      const int rl = tid >> 2;
#pragma unroll
      for (int e = 0; e < 8; ++e) s[kk + e][rl] = v[e];
    } else {
      const int rq = (tid & 7) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) s[kk][rq + e] = v[e];
    }
  }
};

// epilogue: v = alpha*acc (+bias) [relu==2: ReLU here] (+resid) (+beta*C_old) (*gate>0) [relu==1: ReLU]
// c_tap_cin != 0: output column n = tap*c_tap_cin + c is stored at c*3 + tap (Conv1d weight layout)
// c_last != NULL: output column N-1 goes to c_last[m] (fused bias gradient)
__device__ __forceinline__ void epilogue_store(const GemmDev& g, int b, int m, int n, float acc) {
  float v = g.alpha * acc;
  if (g.c_last && n == g.N - 1) {
    float* cp = g.c_last + (long long)b * g.M + m;
    if (g.beta != 0.f) v += g.beta * (*cp);
    *cp = v;
    return;
  }
  if (g.bias) v += g.bias[n];
  if (g.relu == 2) v = fmaxf(v, 0.f);
  if (g.resid) v += g.resid[(long long)b * g.resid_bs + (long long)m * g.ld_resid + n];
  long long col = n;
  if (g.c_tap_cin) {
    const int j = n / g.c_tap_cin;
    col = (long long)(n - j * g.c_tap_cin) * 3 + j;
  }
  float* cp = g.c + (long long)b * g.c_bs + (long long)m * g.ldc + col;
  if (g.beta != 0.f) v += g.beta * (*cp);
  if (g.gate && !(g.gate[(long long)m * g.ld_gate + n] > 0.f)) v = 0.f;
  if (g.relu == 1) v = fmaxf(v, 0.f);
  *cp = v;
}

// split-K without a second launch: each block of a tile writes its partial sums to its
// workspace slab; the last block to arrive (per-tile counter) adds the slabs in slab order
// (deterministic) and runs the epilogue, then re-arms the counter for the next launch.
// Ordering follows the agent-scope hand-off recipe (cdna_hip_programming.md, projection GEMM
// item 2): drain the slab stores, ONE release fence by lane 0 before the ticket, ONE acquire fence
// in the reducer; correct for any placement of a tile's slices over XCDs.  `flag` lives inside the
// kernel's existing LDS array (a separate __shared__ word can de-pipeline the k-loop).
template <int TM, int TN>
__device__ void splitk_finish(const GemmDev& g, int bidx, int m0, int n0, int tile_id, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev =
        __hip_atomic_fetch_add(&g.tile_cnt[tile_id], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)g.split - 1;
    if (last) {
      __hip_atomic_store(&g.tile_cnt[tile_id], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  const long long MN = (long long)g.M * g.N;
  const float* base = g.ws + (long long)bidx * g.split * MN;
  for (int e = threadIdx.x; e < TM * TN; e += blockDim.x) {
    const int m = m0 + e / TN, n = n0 + e % TN;
    if (m >= g.M || n >= g.N) continue;
    const float* p = base + (long long)m * g.N + n;
    float v = 0.f;
    for (int k = 0; k < g.split; ++k) v += p[k * MN];
    epilogue_store(g, bidx, m, n, v);
  }
}

template <int AK, int BKIND>
__global__ __launch_bounds__(NTHREADS) void gemm_f32_kernel(GemmDev g) {
  __shared__ float sA[2][BK][LDSS];
  __shared__ float sB[2][BK][LDSS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 8 waves: waves 0-3 multiply k rows [0,32) of every stage, waves 4-7 rows [32,64), into
  // separate accumulators of the same 32x32 sub-tile -> two independent MFMA chains per SIMD,
  // so one wave's loads / selects / LDS traffic hide under the other wave's MFMAs.
  const int kh = wave >> 2, koff = kh * BKH, ltid = tid & 255;
  const int wq = wave & 3, wm = wq >> 1, wn = wq & 1, li = lane & 31, lh = lane >> 5;
  // XCD-aware remap of (x, y) tiles: consecutive remapped ids share an XCD (L2)
  int tx, ty;
  {
    const int nt = g.tiles_x * g.tiles_y;
    const int id = blockIdx.y * g.tiles_x + blockIdx.x;
    const int q = nt / 8, rr = nt % 8, x8 = id % 8, i8 = id / 8;
    const int nid = (x8 < rr ? x8 * (q + 1) : rr * (q + 1) + (x8 - rr) * q) + i8;
    ty = nid / g.tiles_x;
    tx = nid - ty * g.tiles_x;
  }
  const int n0 = tx * BN, m0 = ty * BM;
  const int z = blockIdx.z, bidx = z / g.split, sk = z - bidx * g.split;
  const int nkt = (g.K + BK - 1) / BK;
  const int kt0 = sk * g.kt_per_split;
  const int kt1 = min(nkt, kt0 + g.kt_per_split);

  Loader<AK> la;
  Loader<BKIND> lb;
  la.init(g.a, g.a.ptr + (long long)bidx * g.a.batch_stride, m0, g.M, g.K, g.a_vec, ltid);
  lb.init(g.b, g.b.ptr + (long long)bidx * g.b.batch_stride, n0, g.N, g.K, g.b_vec, ltid);

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  FX_STAMP(g, 0);

  // Each thread stages one 8-element chunk per operand per stage (its wave group's k half).
  // Global loads run TWO stages ahead in ping-pong register sets (r*0 / r*1, static names:
  // a runtime-indexed register array would spill to scratch), so a stage's loads have two
  // MFMA phases to land before they are written to LDS.
  float ra0[8], rb0[8], ra1[8], rb1[8];
  if (kt0 < kt1) {
    la.load(kt0 * BK + koff, ra0);
    lb.load(kt0 * BK + koff, rb0);
    if (kt0 + 1 < kt1) {
      la.load((kt0 + 1) * BK + koff, ra1);
      lb.load((kt0 + 1) * BK + koff, rb1);
    }
    la.store(sA[0] + koff, ltid, ra0);
    lb.store(sB[0] + koff, ltid, rb0);
  }
  __syncthreads();
  auto stage = [&](int kt, int cur, float* ra_free, float* rb_free, const float* ra_next, const float* rb_next) {
    if (kt + 2 < kt1) {
      la.load((kt + 2) * BK + koff, ra_free);
      lb.load((kt + 2) * BK + koff, rb_free);
    }
    // every fragment read of the half-stage first, so LDS latency overlaps the MFMA chain
    float av[BKH / 2], bv[BKH / 2];
#pragma unroll
    for (int s = 0; s < BKH / 2; ++s) {
      av[s] = sA[cur][koff + 2 * s + lh][wm * 32 + li];
      bv[s] = sB[cur][koff + 2 * s + lh][wn * 32 + li];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < BKH / 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc, 0, 0, 0);
    if (kt + 1 < kt1) {
      la.store(sA[cur ^ 1] + koff, ltid, ra_next);
      lb.store(sB[cur ^ 1] + koff, ltid, rb_next);
    }
    __syncthreads();
  };
  FX_STAMP(g, 1);
  for (int kt = kt0; kt < kt1; kt += 2) {
    stage(kt, 0, ra0, rb0, ra1, rb1);               // set 0 held stage kt (already in LDS): refill it
    if (kt + 1 < kt1) stage(kt + 1, 1, ra1, rb1, ra0, rb0);
  }

  FX_STAMP(g, 2);
  // combine the two k-half accumulators through LDS (fixed order: deterministic)
  {
    float* red = &sA[0][0][0];
    if (kh == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(wq * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (kh == 1 && !(g.split > 1 && g.tile_cnt)) return;
    if (kh == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[(wq * 16 + r) * 64 + lane];
    }
  }

  // C/D layout of the 32x32 f32 accumulator: col = lane&31, row = (r&3)+8*(r>>2)+4*(lane>>5)
  const int col = n0 + wn * 32 + li;
  const int rbase = m0 + wm * 32 + 4 * lh;
  if (g.split > 1) {
    if (kh == 0 && col < g.N) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < g.M) g.ws[(((long long)bidx * g.split + sk) * g.M + row) * g.N + col] = acc[r];
      }
    }
    if (g.tile_cnt)   // flag: last word of sA (the k-half combine above uses the first 16 KB)
      splitk_finish<BM, BN>(g, bidx, m0, n0, (bidx * g.tiles_y + ty) * g.tiles_x + tx,
                            reinterpret_cast<int*>(&sA[1][BK - 1][LDSS - 1]));
    return;
  }
  if (col >= g.N) return;
  if (!g.c_last && !g.c_tap_cin && !g.gate && g.beta == 0.f) {
    // common forward epilogue: every read (bias, residual) is issued before the first store,
    // so the 16 loads overlap instead of queueing behind stores they might alias
    const float bv = g.bias ? g.bias[col] : 0.f;
    float res[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      res[r] = (g.resid && row < g.M) ? g.resid[(long long)bidx * g.resid_bs + (long long)row * g.ld_resid + col]
                                      : 0.f;
    }
    float* cb = g.c + (long long)bidx * g.c_bs + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      float v = g.alpha * acc[r] + bv;
      if (g.relu == 2) v = fmaxf(v, 0.f);
      v += res[r];
      if (g.relu == 1) v = fmaxf(v, 0.f);
      if (row < g.M) cb[(long long)row * g.ldc] = v;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      if (row < g.M) epilogue_store(g, bidx, row, col, acc[r]);
    }
  }
  FX_STAMP(g, 3);
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmDev g) {
  const long long total = (long long)g.M * g.N;
  const int bidx = blockIdx.y;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int sk = 0; sk < g.split; ++sk) s += g.ws[((long long)bidx * g.split + sk) * total + i];
    epilogue_store(g, bidx, (int)(i / g.N), (int)(i % g.N), s);
  }
}

// ---------------------------------------------------------------- direct kernel (small shapes)
// Token-level (M = Nact = 32) projections, per-head attention products and their weight
// gradients are far too small for the 64x64 LDS-tiled kernel: its per-tile cost is latency
// (prologue loads, a 1 us MFMA phase per 64-deep stage, the epilogue), so a handful of tiles
// walking K serially takes 10-30 us.  Here each wave owns one 32x32 output tile over a strided
// set of 32-deep k chunks and loads its MFMA fragments straight from global memory (L2): a lane
// takes 16 CONSECUTIVE k of a chunk (the k order inside an MFMA chain is free as long as A and B
// agree), so row-major operands are float4 loads and column-major ones are coalesced across
// lanes.  The waves of a block split K of the same tile and are summed through LDS in wave
// order; optional cross-block split-K goes through workspace slabs + splitk_finish.
constexpr int DCH = 32, DMAXW = 8;

template <int KIND>
__device__ __forceinline__ void dload(const fx_operand& o, const float* base, int r, int R, int k0, int K, bool vec,
                                      float* v) {
  if (KIND == ROWS) {
    if (vec && r < R && k0 + 16 <= K) {
      const float* p = base + (long long)r * o.ld + k0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(p + 4 * q);
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (r < R && k0 + j < K) ? base[(long long)r * o.ld + k0 + j] : 0.f;
  } else if (KIND == COLS) {
    const bool ones = o.ones_col && r == o.ones_col - 1;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      v[j] = (r < R && k0 + j < K) ? (ones ? 1.f : base[(long long)(k0 + j) * o.ld + r]) : 0.f;
  } else {  // ROWS_GEN
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (r < R && k0 + j < K) ? fetch_rm(o, base, r, k0 + j) : 0.f;
  }
}

__device__ __forceinline__ void direct_finish(const GemmDev& g, int bidx, int sk, int row, int col, float v) {
  if (row >= g.M || col >= g.N) return;
  if (g.split > 1)
    g.ws[(((long long)bidx * g.split + sk) * g.M + row) * g.N + col] = v;
  else
    epilogue_store(g, bidx, row, col, v);
}

template <int AK, int BKd>
__global__ __launch_bounds__(DMAXW * 64) void gemm_direct_kernel(GemmDev g) {
  __shared__ float red[DMAXW * 16 * 64 + 1];   // wave partials + the split-K "last block" flag
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int z = blockIdx.z, bidx = z / g.split, sk = z - bidx * g.split;
  const int nch = (g.K + DCH - 1) / DCH;
  const int c0 = sk * g.kt_per_split, c1 = min(nch, c0 + g.kt_per_split);
  const float* pa = g.a.ptr + (long long)bidx * g.a.batch_stride;
  const float* pb = g.b.ptr + (long long)bidx * g.b.batch_stride;
  const int ra = m0 + li, rb = n0 + li, ko = lh * 16;
  const bool av = g.a_vec, bv = g.b_vec;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float a0[16], b0[16], a1[16], b1[16];
  int c = c0 + w;
  if (c < c1) {
    dload<AK>(g.a, pa, ra, g.M, c * DCH + ko, g.K, av, a0);
    dload<BKd>(g.b, pb, rb, g.N, c * DCH + ko, g.K, bv, b0);
  }
  for (; c < c1; c += 2 * nw) {
    const int cn = c + nw;
    if (cn < c1) {
      dload<AK>(g.a, pa, ra, g.M, cn * DCH + ko, g.K, av, a1);
      dload<BKd>(g.b, pb, rb, g.N, cn * DCH + ko, g.K, bv, b1);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc, 0, 0, 0);
    const int cnn = cn + nw;
    if (cnn < c1) {
      dload<AK>(g.a, pa, ra, g.M, cnn * DCH + ko, g.K, av, a0);
      dload<BKd>(g.b, pb, rb, g.N, cnn * DCH + ko, g.K, bv, b0);
    }
    if (cn < c1) {
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc, 0, 0, 0);
    }
  }

  if (nw > 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
    for (int e = tid; e < 1024; e += nw * 64) {
      const int r = e >> 6, l = e & 63;
      float v = 0.f;
      for (int q = 0; q < nw; ++q) v += red[(q * 16 + r) * 64 + l];
      direct_finish(g, bidx, sk, m0 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), n0 + (l & 31), v);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) direct_finish(g, bidx, sk, m0 + (r & 3) + 8 * (r >> 2) + 4 * lh, n0 + li, acc[r]);
  }
  if (g.split > 1 && g.tile_cnt)
    splitk_finish<32, 32>(g, bidx, m0, n0, (bidx * g.tiles_y + blockIdx.y) * g.tiles_x + blockIdx.x,
                          reinterpret_cast<int*>(&red[DMAXW * 16 * 64]));
}

// bias-gradient column sums, two deterministic stages (used only where no dW GEMM carries them)
constexpr int CS_ROWS = 128;
__global__ __launch_bounds__(256) void colsum_stage1(const float* x, long long ld, int M, int N, float* ws) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * CS_ROWS;
  float s = 0.f;
  if (n < N)
    for (int r = r0 + rg; r < min(M, r0 + CS_ROWS); r += 4) s += x[(long long)r * ld + n];
  __shared__ float red[4][64];
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && n < N) ws[(long long)blockIdx.y * N + n] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                                            red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ __launch_bounds__(256) void colsum_stage2(const float* ws, int nblk, int N, float* out, int acc) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += ws[(long long)b * N + n];
  out[n] = acc ? out[n] + s : s;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

bool operand_vec_ok(const fx_operand& o) {
  if (!aligned16(o.ptr) || (o.ld & 3)) return false;
  if (o.batch_stride & 3) return false;
  if (o.conv_taps && (o.conv_cin & 7)) return false;
  if (!o.trans && o.ptr1 && (!aligned16(o.ptr1) || (o.ld1 & 3) || (o.k_split & 7))) return false;
  return true;
}

int kind_of(const fx_operand& o, bool vec) {
  if (o.trans) return o.conv_taps ? COLS_CONV : COLS;
  if (o.conv_taps) return (vec && o.conv_cin % BKH == 0) ? ROWS_CONV : ROWS_GEN;
  if (o.ptr1 || o.rows0 || o.rows1 || o.pos) return ROWS_GEN;
  return ROWS;
}

template <int AK, int BKd>
void launch_t(dim3 grid, hipStream_t s, const GemmDev& g) {
  hipLaunchKernelGGL((gemm_f32_kernel<AK, BKd>), grid, dim3(NTHREADS), 0, s, g);
}

template <int AK>
int launch_b(int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  switch (bk) {
    case ROWS: launch_t<AK, ROWS>(grid, s, g); return FX_OK;
    case COLS: launch_t<AK, COLS>(grid, s, g); return FX_OK;
    case COLS_CONV: launch_t<AK, COLS_CONV>(grid, s, g); return FX_OK;
    case ROWS_GEN: launch_t<AK, ROWS_GEN>(grid, s, g); return FX_OK;
    default: break;
  }
  set_error("gemm: unsupported B operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_tiled(int ak, int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  switch (ak) {
    case ROWS: return launch_b<ROWS>(bk, grid, s, g);
    case ROWS_CONV: return launch_b<ROWS_CONV>(bk, grid, s, g);
    case ROWS_GEN: return launch_b<ROWS_GEN>(bk, grid, s, g);
    case COLS: return launch_b<COLS>(bk, grid, s, g);
    default: break;
  }
  set_error("gemm: unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

template <int AK>
int launch_direct_b(int bk, dim3 grid, dim3 block, hipStream_t s, const GemmDev& g) {
  switch (bk) {
    case ROWS: hipLaunchKernelGGL((gemm_direct_kernel<AK, ROWS>), grid, block, 0, s, g); return FX_OK;
    case COLS: hipLaunchKernelGGL((gemm_direct_kernel<AK, COLS>), grid, block, 0, s, g); return FX_OK;
    default: break;
  }
  set_error("gemm(direct): unsupported B operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_direct(int ak, int bk, dim3 grid, dim3 block, hipStream_t s, const GemmDev& g) {
  switch (ak) {
    case ROWS: return launch_direct_b<ROWS>(bk, grid, block, s, g);
    case ROWS_GEN: return launch_direct_b<ROWS_GEN>(bk, grid, block, s, g);
    case COLS: return launch_direct_b<COLS>(bk, grid, block, s, g);
    default: break;
  }
  set_error("gemm(direct): unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

// Small problems go to the direct kernel: token-level (M or N <= 32) or shallow K.  (Few-tile
// frame-level dW GEMMs with K = T stay tiled: measured 25 vs 32 us at 256x257x4096.)  Conv-gather operands always take the tiled kernel.
// FX_GEMM_PATH=tiled|direct overrides the choice (diagnostic).
bool use_direct(const fx_gemm_desc& d, int ak, int bk) {
  static const int force = [] {
    const char* p = std::getenv("FX_GEMM_PATH");
    if (!p) return 0;
    return std::string(p) == "tiled" ? 1 : std::string(p) == "direct" ? 2 : 0;
  }();
  const bool ok = (ak == ROWS || ak == ROWS_GEN || ak == COLS) && (bk == ROWS || bk == COLS);
  if (!ok || force == 1) return false;
  if (force == 2) return true;
  return d.M <= 32 || d.N <= 32 || d.K <= 64;
}

// Split-K arrival counters, one pool per (device, stream): zeroed once at allocation and
// re-armed by the last block of every tile, so launches on one stream reuse them safely.
constexpr long long kMaxTileCounters = 1 << 16;
unsigned* tile_counters(hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, unsigned*> pool;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(dev, s);
  auto it = pool.find(key);
  if (it != pool.end()) return it->second;
  unsigned* p = nullptr;
  if (hipMalloc(&p, kMaxTileCounters * sizeof(unsigned)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, kMaxTileCounters * sizeof(unsigned), s) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  pool[key] = p;
  return p;
}

}  // namespace

fx_operand op_rows(const float* p, long long ld) {
  fx_operand o{};
  o.ptr = p;
  o.ld = ld;
  o.conv_dir = 1;
  return o;
}

fx_operand op_cols(const float* p, long long ld) {
  fx_operand o = op_rows(p, ld);
  o.trans = 1;
  return o;
}

fx_gemm_desc gemm_desc(int M, int N, int K, fx_operand a, fx_operand b, float* c, long long ldc) {
  fx_gemm_desc d{};
  d.M = M;
  d.N = N;
  d.K = K;
  d.batch = 1;
  d.a = a;
  d.b = b;
  d.c = c;
  d.ldc = ldc;
  d.alpha = 1.f;
  d.split_k = 1;
  return d;
}

long long gemm_workspace_floats(const fx_gemm_desc& d) {
  if (d.split_k <= 1) return 0;
  return (long long)d.batch * d.split_k * d.M * d.N;
}

int launch_gemm(const fx_gemm_desc& d, hipStream_t s) {
  FX_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0 && d.batch >= 1, "gemm: bad sizes");
  if (d.M == 0 || d.N == 0) return FX_OK;
  FX_REQUIRE(d.a.ptr && d.b.ptr && d.c, "gemm: null operand");
  FX_REQUIRE(!(d.a.conv_taps && d.a.seq_len <= 0) && !(d.b.conv_taps && d.b.seq_len <= 0),
             "gemm: conv operand needs seq_len");
  FX_REQUIRE(!(d.a.conv_taps && d.K != d.a.conv_taps * d.a.conv_cin), "gemm: conv A needs K == taps*cin");
  FX_REQUIRE(!(d.b.conv_taps && d.b.trans && d.N != d.b.conv_taps * d.b.conv_cin + (d.b.ones_col ? 1 : 0)),
             "gemm: conv B needs N == taps*cin (+1 with a ones column)");
  FX_REQUIRE(!(d.a.ones_col && !d.a.trans) && !(d.b.ones_col && !d.b.trans), "gemm: ones_col needs trans==1");
  FX_REQUIRE(!(d.b.conv_taps && !d.b.trans), "gemm: row-major conv B operand is not supported");
  GemmDev g{};
  g.M = d.M;
  g.N = d.N;
  g.K = d.K;
  g.a = d.a;
  g.b = d.b;
  g.c = d.c;
  g.ldc = d.ldc;
  g.c_bs = d.c_batch_stride;
  g.alpha = d.alpha;
  g.beta = d.beta;
  g.bias = d.bias;
  g.resid = d.resid;
  g.ld_resid = d.ld_resid;
  g.resid_bs = d.resid_batch_stride;
  g.gate = d.gate;
  g.ld_gate = d.ld_gate;
  g.relu = d.relu;
  g.c_tap_cin = d.c_tap_cin;
  g.c_last = d.c_last_col;
  g.stamps = d.dbg_stamps;
  g.a_vec = operand_vec_ok(d.a);
  g.b_vec = operand_vec_ok(d.b);
  g.ws = d.workspace;
  const int ak = kind_of(d.a, g.a_vec), bk = kind_of(d.b, g.b_vec);
  const bool direct = use_direct(d, ak, bk);
  const int cap = (d.split_k > 1 && d.workspace) ? d.split_k : 1;   // workspace holds `cap` slabs
  FX_REQUIRE(!(d.split_k > 1 && !d.workspace), "gemm: split-K needs a workspace");
  dim3 grid, block;
  if (direct) {
    const int nch = cdiv(d.K, DCH);
    const long long t32 = (long long)cdiv(d.M, 32) * cdiv(d.N, 32) * d.batch;
    const int nw = std::min(DMAXW, std::max(1, nch / 2));
    int split = 1;
    if (cap > 1) {
      const long long want = std::min<long long>(nch / (2 * nw), cdiv(2048, t32 * nw));
      split = (int)std::max<long long>(1, std::min<long long>(cap, want));
    }
    g.kt_per_split = nch > 0 ? cdiv(nch, split) : 0;
    g.split = g.kt_per_split > 0 ? cdiv(nch, g.kt_per_split) : 1;
    g.tiles_x = cdiv(d.N, 32);
    g.tiles_y = cdiv(d.M, 32);
    grid = dim3(g.tiles_x, g.tiles_y, d.batch * g.split);
    block = dim3(nw * 64);
  } else {
    const int nkt = cdiv(d.K, BK);
    int split = std::min(cap, std::max(nkt, 1));
    g.kt_per_split = nkt > 0 ? cdiv(nkt, split) : 0;
    g.split = g.kt_per_split > 0 ? cdiv(nkt, g.kt_per_split) : 1;
    g.tiles_x = cdiv(d.N, BN);
    g.tiles_y = cdiv(d.M, BM);
    grid = dim3(g.tiles_x, g.tiles_y, d.batch * g.split);
    block = dim3(NTHREADS);
  }
  // in-launch reduction only while the last block's serial slab read stays small (<= 32 KB per
  // tile); bigger ones pay less as a separate reduce launch (conv dW split 5: 78 vs 56 us)
  const long long slab_bytes = (long long)g.split * (direct ? 32 * 32 : BM * BN) * 4;
  if (g.split > 1 && slab_bytes <= 32768 && (long long)g.tiles_x * g.tiles_y * d.batch <= kMaxTileCounters)
    g.tile_cnt = tile_counters(s);
  // FX_GEMM_LOG=<file>: append one line per launch (diagnostic shape census, tools/gemm_census.py)
  static FILE* glog = [] {
    const char* p = std::getenv("FX_GEMM_LOG");
    return p ? std::fopen(p, "a") : nullptr;
  }();
  if (glog)
    std::fprintf(glog, "%d %d %d %d %d %d %d %d %d %d %d\n", d.M, d.N, d.K, d.batch, ak, bk, g.split,
                 d.a.conv_taps, d.b.conv_taps, d.relu, direct ? (int)block.x / 64 : 0);
  int st = direct ? launch_direct(ak, bk, grid, block, s, g) : launch_tiled(ak, bk, grid, s, g);
  if (st != FX_OK) return st;
  FX_CHECK_HIP(hipGetLastError());
  if (g.split > 1 && !g.tile_cnt) {
    const long long total = (long long)d.M * d.N;
    int blocks = (int)std::min<long long>(cdiv(total, 256), 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks, d.batch), dim3(256), 0, s, g);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

int launch_colsum(const float* x, long long ld, int M, int N, float* out, int accumulate, float* ws,
                  hipStream_t s) {
  if (N == 0) return FX_OK;
  if (M == 0) {
    if (!accumulate) FX_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(float) * N, s));
    return FX_OK;
  }
  const int nblk = cdiv(M, CS_ROWS);
  hipLaunchKernelGGL(colsum_stage1, dim3(cdiv(N, 64), nblk), dim3(256), 0, s, x, ld, M, N, ws);
  hipLaunchKernelGGL(colsum_stage2, dim3(cdiv(N, 256)), dim3(256), 0, s, ws, nblk, N, out, accumulate);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

long long colsum_workspace_floats(int M, int N) { return (long long)cdiv(M, CS_ROWS) * N; }

}  // namespace fx
