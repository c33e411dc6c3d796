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
//   COLS_CONVR the same over ragged videos (host row offsets): weight gradients of a ragged batch in
//             one launch, K padded to whole stages (rows past the last video read as zero)
//   COLS_KT   COLS with K not a whole number of 64-deep stages (frame-level weight gradients over a
//             ragged frame count): rows past K read as zero from a clamped address, both operands
//
// Tiled kernel: 64x64 output tile per 256-thread workgroup, one wave per SIMD, each wave a
// 32x32 sub-tile over the block's whole K range (32 MFMAs = 2048 matrix-core cycles per
// 64-deep stage between barriers).  K is staged through a 3-slot LDS ring: stage s+2 is
// written while stage s is multiplied, so the fragments of stage s+1 are already visible
// when a wave reaches the end of stage s and one barrier per stage suffices.  Global loads
// run one more stage ahead in two register sets.  Inside a stage each lane works on 32
// CONSECUTIVE k (lane half h takes k in [32h, 32h+32)): A and B agree on that order, which is
// all an MFMA chain needs, and it lets row-major images be read as ds_read_b128 (4 MFMAs of
// operand per read) and written as ds_write_b128 straight from the float4 global loads.
//   row-major kinds -> LDS image [row][k], stride 68 (16-B rows; b128 reads conflict-free)
//   col-major kinds -> LDS image [k][row], stride 65 (b32 reads conflict-free over 64 lanes)
// Blocks are remapped so that consecutive output tiles share an XCD (L2).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "fx_common.h"

namespace fx {
namespace {

constexpr int BM = 64, BN = 64, BK = 64, NTHREADS = 256;
constexpr int RS = 68;              // [row][k] image stride
constexpr int CS = 65;              // [k][row] image stride
constexpr int IMG = BM * RS;        // floats per operand image (>= BK * CS)
constexpr int NSLOT = 3;            // LDS ring depth
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ROWS_CAT: [src0[rows0[r]] | src1[rows1[r]]] split at k_split (a multiple of the 64-deep stage),
//           either gather optional -- the FAST form of the concatenation / gather operands
constexpr int kMaxSeq = 16;        // ragged videos per conv operand

enum Kind { ROWS = 0, ROWS_CONV = 1, ROWS_GEN = 2, COLS = 3, COLS_CONV = 4, ROWS_CAT = 5, COLS_CONVR = 6, COLS_KT = 7 };

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
  unsigned drop_thr;    // dropout (fx_drop_bits >= drop_thr keeps); 0 = off
  float drop_scale;
  unsigned long long drop_seed;
  long long c_last_bs;  // c_last of batch b at c_last + b * c_last_bs
  int b_dil_growth;     // > 1: B's conv dilation of batch b is conv_dil * growth^b
  int xcd_planes;       // wide8: whole z-planes (batch x split-K slice) per XCD, see block_tile
  int row_perm;         // > 1: dilated-conv A shifting by row_perm row tiles: XCD runs follow the taps, see block_tile
  int group_m;          // > 1: tiles in groups of group_m row tiles, column-major inside a group, see block_tile
  int persist;          // wide8 only, > 0: tiles per launch; a grid of gridDim.x workgroups walks them (see
                        // gemm_f32_wide8_kernel)
  int a_dil_b1;         // > 0: A's conv dilation of batch 1 (two dilated convs of one input in one launch)
  long long bias_bs;    // bias of batch b at bias + b * bias_bs
  int nsoff;            // > 0: the conv operand's videos are ragged: video v owns rows [soff[v], soff[v+1])
  int soff[kMaxSeq + 1];   // (COLS_CONVR: entries past nsoff are INT_MAX)
};

// Position of row r inside its video and the video's length (the conv operand's zero padding):
// uniform videos of seq_len rows, or the ragged offsets soff (nsoff videos; read from the kernel
// arguments, a branch-free count of the video starts at or before r).
typedef int SeqOff[kMaxSeq + 1];

__device__ __forceinline__ void seq_pos(int seq_len, const SeqOff& soff, int nsoff, int r, int& pos, int& len) {
  if (nsoff > 0) {
    // fully unrolled (constant indices: scalar loads from the kernel arguments, no private copy):
    // start = the last offset <= r, end = the first offset > r (offsets increase)
    int start = 0, end = 0x7fffffff;
#pragma unroll
    for (int i = 1; i <= kMaxSeq; ++i) {
      if (i <= nsoff) {
        const int o = soff[i];
        if (o <= r) start = o;
        else end = min(end, o);
      }
    }
    pos = r - start;
    len = end - start;
  } else {
    pos = r % seq_len;
    len = seq_len;
  }
}

// Diagnostic builds (-DFX_STAMPS) record s_memtime / s_memrealtime at fixed points of
// every block; the shipped library compiles the macro to nothing.
#ifdef FX_STAMPS
#define FX_STAMP(g, slot)                                                                          \
  do {                                                                                            \
    if ((g).stamps && threadIdx.x == 0) {                                                         \
      const long long _b = (long long)blockIdx.z * gridDim.x * gridDim.y + blockIdx.y * gridDim.x + \
                           blockIdx.x;                                                            \
      (g).stamps[(_b * 2) * 10 + 2 * (slot)] = __builtin_amdgcn_s_memtime();                       \
      (g).stamps[(_b * 2) * 10 + 2 * (slot) + 1] = __builtin_amdgcn_s_memrealtime();               \
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

// A operand of batch bidx: batch 1 may take its own conv dilation (MS-TCN++'s two dilated convs)
__device__ __forceinline__ fx_operand batch_op_a(const fx_operand& a, int dil_b1, int bidx) {
  fx_operand o = a;
  if (dil_b1 > 0 && bidx == 1) o.conv_dil = dil_b1;
  return o;
}

// B operand of batch bidx: a per-batch conv dilation (dilation stacks: layer b's conv_dil * growth^b)
__device__ __forceinline__ fx_operand batch_op_b(const fx_operand& b, int growth, int bidx) {
  fx_operand o = b;
  if (growth > 1)
    for (int i = 0; i < bidx; ++i) o.conv_dil *= growth;
  return o;
}

// ---------------------------------------------------------------- generic element fetch
__device__ __forceinline__ float fetch_rm(const fx_operand& o, const float* p0, int r, int k, const SeqOff& soff,
                                         int nsoff) {
  if (o.conv_taps) {
    const int j = k / o.conv_cin, c = k - j * o.conv_cin, s = conv_shift(o, j);
    int pos, len;
    seq_pos(o.seq_len, soff, nsoff, r, pos, len);
    const int t = pos + s;
    if (t < 0 || t >= len) return 0.f;
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

// COLS_CONVR: does frame k + s lie in frame k's video?  Branch-free over the 16 offsets (entries past
// the last video are INT_MAX, so frames past the last video -- the K padding -- are never valid).
__device__ __forceinline__ bool seq_same(const SeqOff& soff, int k, int s) {
  int start = 0, end = 0x7fffffff;
#pragma unroll
  for (int i = 1; i <= kMaxSeq; ++i) {
    const int o = soff[i];
    start = o <= k ? o : start;
    end = o > k ? min(end, o) : end;
  }
  const int t = k + s;
  return end != 0x7fffffff && t >= start && t < end;
}

__device__ __forceinline__ float fetch_cm(const fx_operand& o, const float* p0, int r, int k) {
  if (o.ones_col && r == o.ones_col - 1) return 1.f;
  if (o.conv_taps) {   // uniform videos only (ragged weight gradients run per video)
    const int j = r / o.conv_cin, c = r - j * o.conv_cin, s = conv_shift(o, j);
    const int t = k % o.seq_len + s;
    if (t < 0 || t >= o.seq_len) return 0.f;
    return p0[(long long)(k + s) * o.ld + c];
  }
  return p0[(long long)k * o.ld + r];
}

__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 ldg4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ---------------------------------------------------------------- loaders
// A stage is the 64 x 64 (rows x k) tile of one operand; each of the 1024 / NJ threads moves NJ
// float4 of it per stage (NJ = 4: 256-thread blocks, NJ = 2: 512-thread blocks):
//   row-major kinds: rows (tid>>4) + (64/NJ) j, k = (tid&15)*4 .. +3      (j < NJ)
//   col-major kinds: k    (tid>>4) + (64/NJ) j, rows (tid&15)*4 .. +3
// so 16 consecutive threads read one 256-B line.
// FAST (chosen per launch on the host: 16-B aligned operands, K % 64 == 0, no gathers): the
// loads are unconditional straight-line code -- rows past the edge are read from a clamped
// in-range address and replaced by a select (0, or 1 for the virtual ones row) -- so the
// pipelined loop has no bounds branches for the compiler to drain vmcnt at.  !FAST fetches
// element by element with full bounds checks (edge shapes, gathers, concatenations).
// KW = 32 (the split-precision kernel's 32-deep stages, 512 threads, NJ = 1): row-major kinds
// take row tid>>3 and k (tid&7)*4; col-major kinds keep k tid>>4 and rows (tid&15)*4.
template <int KIND, bool FAST, int NJ = 4, int KW = 64>
struct Loader {
  static constexpr int RSTEP = 64 / NJ;   // row (or k) step between a thread's NJ vectors
  static constexpr bool kRowImg = KIND <= ROWS_GEN || KIND == ROWS_CAT;
  fx_operand o;        // by value: the address of a kernel argument would force it to scratch
  const float* base;   // operand base incl. batch offset
  int R, K, r0;
  int ta, tb;          // tid>>4, (tid&15)*4
  int rowc[4];         // row-major: clamped row of j (ROWS_CAT: gathered row of the first source)
  int rowc1[4];        // ROWS_CAT: gathered row of the second source
  int rmod[4];         // ROWS_CONV: position of row j in its video
  int rlen[4];         // ROWS_CONV: that video's length
  SeqOff soff;         // ragged conv videos: a register copy of GemmDev::soff (constant indices only; a
  int nsoff;           // pointer into the kernel arguments would force them into private memory)
  unsigned rok;        // row-major: bit j = row j in range
  int rc;              // col-major: clamped first row of the 4
  unsigned emask, omask;   // col-major: bit e = row rc+e in storage / is the ones row
  int tapc, tap_s;     // COLS_CONV: channel / shift of this thread's 4 rows (one tap: cin % 4 == 0)
  // FAST: per-thread addresses made once, so a stage's load is a uniform offset plus one add per
  // row (the per-row 64-bit multiply-adds otherwise sit in every stage, ahead of its MFMAs)
  const float* prow[4];    // row kinds: row j at k = tb (ROWS_CAT: first source)
  const float* prow1[4];   // ROWS_CAT: row j of the second source at k = tb
  const float* pcol;       // COLS: k = ta, first of the thread's 4 rows

  __device__ __forceinline__ void init(const fx_operand& op, const float* p0, int r0_, int R_, int K_, int tid,
                                       const SeqOff& soff_, int nsoff_) {
    o = op;
    base = p0;
    nsoff = (KIND == ROWS_CONV || KIND == ROWS_GEN || KIND == COLS_CONVR) ? nsoff_ : 0;
    if (KIND == ROWS_GEN || KIND == COLS_CONVR) {   // the generic element fetch (edge shapes) looks rows up per element
#pragma unroll
      for (int i = 0; i <= kMaxSeq; ++i) soff[i] = soff_[i];
    }
    R = R_;
    K = K_;
    r0 = r0_;
    if (KW == 32 && kRowImg) {
      ta = tid >> 3;
      tb = (tid & 7) * 4;
    } else {
      ta = tid >> 4;
      tb = (tid & 15) * 4;
    }
    if (!FAST) return;
    if (kRowImg) {
      rok = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = r0 + ta + RSTEP * j;
        rok |= (r < R ? 1u : 0u) << j;
        rowc[j] = min(r, R - 1);
        if (KIND == ROWS_CONV) seq_pos(op.seq_len, soff_, nsoff_, rowc[j], rmod[j], rlen[j]);
        if (KIND == ROWS_CAT) {
          const int rr = rowc[j];
          rowc1[j] = op.rows1 ? op.rows1[rr] : rr;
          rowc[j] = op.rows0 ? op.rows0[rr] : rr;
        }
        prow[j] = p0 + (long long)rowc[j] * op.ld + tb;
        if (KIND == ROWS_CAT) prow1[j] = op.ptr1 ? op.ptr1 + (long long)rowc1[j] * op.ld1 + tb : prow[j];
      }
    } else {
      // rows that exist in storage: all but a trailing virtual ones row
      const int stored = op.ones_col ? op.ones_col - 1 : R;
      const int r = r0 + tb;
      emask = omask = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        emask |= (r + e < stored ? 1u : 0u) << e;
        omask |= (op.ones_col && r + e == op.ones_col - 1 ? 1u : 0u) << e;
      }
      rc = min(r, ((stored - 1) / 4) * 4);
      pcol = p0 + (long long)ta * op.ld + rc;
      if (KIND == COLS_CONV || KIND == COLS_CONVR) {
        const int j = rc / op.conv_cin;
        tapc = rc - j * op.conv_cin;
        tap_s = conv_shift(op, j);
      }
    }
  }

  // Loads are raw and unconditional; every validity select is applied when the registers are
  // written to LDS (store), a full stage later -- a select right after the load would make the
  // compiler wait for the load there and serialise the prefetch.
  // vm: per-stage validity bits (row-major: bit j = row j valid; COLS_CONV: bit j = time in range)
  __device__ __forceinline__ void load(int k0, float4* v, unsigned& vm) const {
    if (!FAST) {
      load_generic(k0, v);
      vm = 0xFu;
      return;
    }
    if (KIND == ROWS) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) v[j] = ldg4(prow[j] + k0);
      vm = rok;
    } else if (KIND == ROWS_CONV) {
      // the 64-deep stage lies in one tap (conv_cin % 64 == 0, checked on the host): a uniform
      // channel offset and a uniform row shift, taken per row only where the shifted frame exists
      const int tap = k0 / o.conv_cin;
      const int c = k0 - tap * o.conv_cin;
      const int s = conv_shift(o, tap);
      const long long soff = (long long)s * o.ld;
      vm = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int t = rmod[j] + s;
        const bool ok = ((rok >> j) & 1u) && t >= 0 && t < rlen[j];
        vm |= (ok ? 1u : 0u) << j;
        v[j] = ldg4(prow[j] + c + (ok ? soff : 0ll));
      }
    } else if (KIND == ROWS_CAT) {
      // the whole stage reads one source (k_split % 64 == 0): a uniform choice of row addresses
      const bool second = o.ptr1 && k0 >= o.k_split;
      const int kk = second ? k0 - o.k_split : k0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) v[j] = ldg4((second ? prow1[j] : prow[j]) + kk);
      vm = rok;
    } else if (KIND == COLS) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) v[j] = ldg4(pcol + (long long)(k0 + RSTEP * j) * o.ld);
      vm = 0xFu;
    } else if (KIND == COLS_KT) {
      vm = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int k = k0 + ta + RSTEP * j;
        const bool ok = k < K;
        vm |= (ok ? 1u : 0u) << j;
        v[j] = ldg4(pcol + (long long)((ok ? k : K - 1) - ta) * o.ld);
      }
    } else if (KIND == COLS_CONV) {
      vm = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int k = k0 + ta + RSTEP * j;
        const int t = k % o.seq_len + tap_s;   // (uniform videos only: ragged weight gradients run per video)
        const bool ok = t >= 0 && t < o.seq_len;
        vm |= (ok ? 1u : 0u) << j;
        v[j] = ldg4(base + (long long)(ok ? k + tap_s : k) * o.ld + tapc);
      }
    } else if (KIND == COLS_CONVR) {
      vm = 0;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int k = k0 + ta + RSTEP * j;
        const bool ok = seq_same(soff, k, tap_s);
        vm |= (ok ? 1u : 0u) << j;
        v[j] = ldg4(base + (long long)(ok ? k + tap_s : k) * o.ld + tapc);
      }
    }
  }

  __device__ __forceinline__ void load_generic(int k0, float4* v) const {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float e[4];
      if (kRowImg) {
        const int r = r0 + ta + RSTEP * j;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = k0 + tb + q;
          e[q] = (r < R && k < K) ? fetch_rm(o, base, r, k, soff, nsoff) : 0.f;
        }
      } else {
        const int k = k0 + ta + RSTEP * j;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = r0 + tb + q;
          e[q] = (r < R && k < K) ? fetch_cm(o, base, r, k) : 0.f;
        }
      }
      v[j] = make_float4(e[0], e[1], e[2], e[3]);
    }
  }

  __device__ __forceinline__ void store(float* img, const float4* v, unsigned vm) const {
    if (kRowImg) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float4 x = (!FAST || ((vm >> j) & 1u)) ? v[j] : zero4();
        *reinterpret_cast<float4*>(img + (ta + RSTEP * j) * RS + tb) = x;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
        if (FAST) {
          const bool tok = (KIND != COLS_CONV && KIND != COLS_CONVR && KIND != COLS_KT) || ((vm >> j) & 1u);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            // (COLS_KT: rows past K are zero, the ones row included)
            const float one = (((omask >> q) & 1u) && (KIND != COLS_KT || tok)) ? 1.f : 0.f;
            e[q] = (tok && ((emask >> q) & 1u)) ? e[q] : one;
          }
        }
        float* d = img + (ta + RSTEP * j) * CS + tb;
        d[0] = e[0]; d[1] = e[1]; d[2] = e[2]; d[3] = e[3];
      }
    }
  }

  // MFMA operand of steps 4q..4q+3 for lane (i = row in the wave's 32-row half at wr, h = k half)
  __device__ __forceinline__ static float4 frag(const float* img, int wr, int i, int h, int q) {
    if (kRowImg) return *reinterpret_cast<const float4*>(img + (wr + i) * RS + h * 32 + 4 * q);
    const float* p = img + (h * 32 + 4 * q) * CS + wr + i;
    return make_float4(p[0], p[CS], p[2 * CS], p[3 * CS]);
  }
};

// epilogue: v = alpha*acc (+bias) [relu==2: ReLU here] (+resid) (+beta*C_old) (*gate>0) [relu==1: ReLU]
// c_tap_cin != 0: output column n = tap*c_tap_cin + c is stored at c*3 + tap (Conv1d weight layout)
// c_last != NULL: output column N-1 goes to c_last[m] (fused bias gradient)
__device__ __forceinline__ float* epilogue_ptr(const GemmDev& g, int b, int m, int n) {
  if (g.c_last && n == g.N - 1) return g.c_last + (long long)b * g.c_last_bs + m;
  long long col = n;
  if (g.c_tap_cin) {
    const int j = n / g.c_tap_cin;
    col = (long long)(n - j * g.c_tap_cin) * 3 + j;
  }
  return g.c + (long long)b * g.c_bs + (long long)m * g.ldc + col;
}

// `pre`: the caller has already loaded the old C value into `cold` (beta != 0), else it is read here
__device__ __forceinline__ void epilogue_store(const GemmDev& g, int b, int m, int n, float acc, bool pre = false,
                                               float cold = 0.f) {
  float v = g.alpha * acc;
  float* cp = epilogue_ptr(g, b, m, n);
  if (g.c_last && n == g.N - 1) {
    if (g.beta != 0.f) v += g.beta * (pre ? cold : *cp);
    *cp = v;
    return;
  }
  if (g.bias) v += g.bias[(long long)b * g.bias_bs + n];
  if (g.relu == 2) v = fmaxf(v, 0.f);
  if (g.drop_thr) {
    const unsigned long long idx = ((unsigned long long)b * g.M + m) * g.N + n;
    v = fx_drop_bits(g.drop_seed, idx) >= g.drop_thr ? v * g.drop_scale : 0.f;
  }
  if (g.resid) v += g.resid[(long long)b * g.resid_bs + (long long)m * g.ld_resid + n];
  if (g.beta != 0.f) v += g.beta * (pre ? cold : *cp);
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
// One pipelined stage for this wave, as ONE basic block (no branches, so the compiler counts
// outstanding loads exactly), in a fixed order pinned by sched_barrier: first the global loads of
// a later stage into set `rn` (they get two MFMA phases to land), then the 32 MFMAs of the
// current slot with each fragment read issued two groups (8 MFMAs, 512 cycles) ahead of its use,
// and the LDS writes of set `rs` (loaded one stage ago) spread over the middle groups.  Two
// accumulators (even / odd fragment groups) keep two independent chains in the matrix core.
template <bool FAST, int AK, int BKd>
__device__ __forceinline__ void stage_body(const Loader<AK, FAST>& la, const Loader<BKd, FAST>& lb, const float* cur,
                                           float* wslot, int kload, const float4* rs_a, const float4* rs_b,
                                           unsigned ms_a, unsigned ms_b, float4* rn_a, float4* rn_b, unsigned& mn_a,
                                           unsigned& mn_b, int wm, int wn, int li, int lh, f32x16& acc0,
                                           f32x16& acc1) {
  using LA = Loader<AK, FAST>;
  using LB = Loader<BKd, FAST>;
  float4 fa[8], fb[8];
  fa[0] = LA::frag(cur, wm * 32, li, lh, 0);
  fb[0] = LB::frag(cur + IMG, wn * 32, li, lh, 0);
  fa[1] = LA::frag(cur, wm * 32, li, lh, 1);
  fb[1] = LB::frag(cur + IMG, wn * 32, li, lh, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    f32x16& acc = (q & 1) ? acc1 : acc0;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[q].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[q].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[q].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[q].w, acc, 0, 0, 0);
    if (q + 2 < 8) {
      fa[q + 2] = LA::frag(cur, wm * 32, li, lh, q + 2);
      fb[q + 2] = LB::frag(cur + IMG, wn * 32, li, lh, q + 2);
    }
    // the next loads' address work runs beside the first MFMA groups, not ahead of them
    if (q == 0) la.load(kload, rn_a, mn_a);
    if (q == 1) lb.load(kload, rn_b, mn_b);
    if (q == 6) la.store(wslot, rs_a, ms_a);   // late: the loads get ~1.7 stages to land
    if (q == 7) lb.store(wslot + IMG, rs_b, ms_b);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The pipelined K loop over stages [kt0, kt1): a 3-slot LDS ring, loads two stages ahead of
// their LDS write.  Out-of-range prefetches are clamped to the last stage (loaded, never used)
// and stores past the end go to a slot nobody reads again, so every iteration is straight-line.
#define FX_INLINE __attribute__((always_inline))
template <bool FAST, int AK, int BKd>
__device__ __forceinline__ void kloop(const Loader<AK, FAST>& la, const Loader<BKd, FAST>& lb, float* lds, int kt0,
                                      int kt1, int wm, int wn, int li, int lh, f32x16& acc0, f32x16& acc1) {
  const int n = kt1 - kt0;
  if (n <= 0) return;
  const int klast = (kt1 - 1) * BK;
  float4 ra0[4], rb0[4], ra1[4], rb1[4];
  unsigned ma0, mb0, ma1, mb1;
  // prologue: stages 0 and 1 into slots 0 and 1, stage 2 in flight in set 0
  la.load(kt0 * BK, ra0, ma0);
  lb.load(kt0 * BK, rb0, mb0);
  la.load(min((kt0 + 1) * BK, klast), ra1, ma1);
  lb.load(min((kt0 + 1) * BK, klast), rb1, mb1);
  la.store(lds, ra0, ma0);
  lb.store(lds + IMG, rb0, mb0);
  la.store(lds + 2 * IMG, ra1, ma1);
  lb.store(lds + 3 * IMG, rb1, mb1);
  la.load(min((kt0 + 2) * BK, klast), ra0, ma0);
  lb.load(min((kt0 + 2) * BK, klast), rb0, mb0);
  __syncthreads();
  // iteration i multiplies slot i%3, writes stage i+2 (held in set i&1) into slot (i+2)%3,
  // and issues the loads of stage i+3 into set (i+1)&1
  int slot = 0;
  auto iter = [&](int i, const float4* rs_a, const float4* rs_b, unsigned ms_a, unsigned ms_b, float4* rn_a,
                  float4* rn_b, unsigned& mn_a, unsigned& mn_b) FX_INLINE {
    const int ws = slot == 0 ? 2 : slot - 1;   // (slot + 2) % 3
    stage_body<FAST, AK, BKd>(la, lb, lds + slot * 2 * IMG, lds + ws * 2 * IMG, min((kt0 + i + 3) * BK, klast), rs_a,
                              rs_b, ms_a, ms_b, rn_a, rn_b, mn_a, mn_b, wm, wn, li, lh, acc0, acc1);
    __syncthreads();
    slot = slot == 2 ? 0 : slot + 1;
  };
  int i = 0;
  for (; i + 1 < n; i += 2) {
    iter(i, ra0, rb0, ma0, mb0, ra1, rb1, ma1, mb1);
    iter(i + 1, ra1, rb1, ma1, mb1, ra0, rb0, ma0, mb0);
  }
  if (i < n) iter(i, ra0, rb0, ma0, mb0, ra1, rb1, ma1, mb1);
}

// Output tile (tx, ty) and z-plane (batch x split-K slice) of this block.  Workgroups go to the 8 XCDs
// round robin by linear dispatch id.  Default: within each z-plane, runs of consecutive tiles (one
// row band's column tiles) share an XCD and its L2.  xcd_planes (launches whose plane count is a
// multiple of 8, e.g. the batched / split weight-gradient GEMMs, K = 8192 rows): plane p runs whole
// on XCD p % 8, so every tile reading the plane's A rows and B rows hits one L2 instead of all eight
// XCDs fetching them from MALL / HBM.
__device__ __forceinline__ void block_tile_id(const GemmDev& g, int id, int& tx, int& ty);
__device__ __forceinline__ void block_tile(const GemmDev& g, int& tx, int& ty, int& z) {
  const int nt = g.tiles_x * g.tiles_y;
  if (g.xcd_planes) {
    const int L = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    const int x8 = L & 7, sl = L >> 3;
    const int pl = sl / nt, t = sl - pl * nt;
    z = pl * 8 + x8;
    ty = t / g.tiles_x;
    tx = t - ty * g.tiles_x;
    return;
  }
  block_tile_id(g, blockIdx.y * g.tiles_x + blockIdx.x, tx, ty);
  z = blockIdx.z;
}
// the (x, y) tile of linear workgroup id `id` (XCD id % 8): XCD runs, then the group / row-permutation orders
__device__ __forceinline__ void block_tile_id(const GemmDev& g, int id, int& tx, int& ty) {
  const int nt = g.tiles_x * g.tiles_y;
  const int q = nt / 8, rr = nt % 8, x8 = id % 8, i8 = id / 8;
  const int nid = (x8 < rr ? x8 * (q + 1) : rr * (q + 1) + (x8 - rr) * q) + i8;
  ty = nid / g.tiles_x;
  tx = nid - ty * g.tiles_x;
  if (g.group_m > 1) {
    // a large B: in row-major order the 32 tiles an XCD runs at once span one row tile and every column
    // tile, so each row tile re-streams all of B through the XCD's L2.  Groups of group_m row tiles (one
    // XCD run), walked column by column: the tiles in flight share a few B columns and the group's A rows
    // (both L2-resident), so B is fetched about once per XCD
    const int gsz = g.group_m * g.tiles_x, grp = nid / gsz, r = nid - grp * gsz;
    const int rows = min(g.group_m, g.tiles_y - grp * g.group_m);
    ty = grp * g.group_m + r % rows;
    tx = r / rows;
  }
  if (g.row_perm > 1) {
    // a dilated conv whose taps shift by row_perm whole row tiles: the XCD runs walk the row tiles in
    // the order 0, p, 2p, ..., 1, 1 + p, ... so the tiles holding a tile's shifted rows sit next to it in
    // its run (same L2) instead of one or more runs away (HBM / MALL re-reads)
    const int per = g.tiles_y / g.row_perm;
    ty = (ty % per) * g.row_perm + ty / per;
  }
}

template <int AK, int BKIND, bool FAST>
__global__ __launch_bounds__(NTHREADS) void gemm_f32_kernel(GemmDev g) {
  __shared__ float lds[NSLOT * 2 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  // XCD-aware remap of (x, y) tiles: consecutive remapped ids share an XCD (L2)
  int tx, ty, z;
  block_tile(g, tx, ty, z);
  const int n0 = tx * BN, m0 = ty * BM;
  const int bidx = z / g.split, sk = z - bidx * g.split;
  const int nkt = (g.K + BK - 1) / BK;
  const int kt0 = sk * g.kt_per_split;
  const int kt1 = min(nkt, kt0 + g.kt_per_split);

  Loader<AK, FAST> la;
  Loader<BKIND, FAST> lb;
  la.init(batch_op_a(g.a, g.a_dil_b1, bidx), g.a.ptr + (long long)bidx * g.a.batch_stride, m0, g.M, g.K, tid, g.soff, g.nsoff);
  lb.init(batch_op_b(g.b, g.b_dil_growth, bidx), g.b.ptr + (long long)bidx * g.b.batch_stride, n0, g.N, g.K, tid, g.soff, g.nsoff);

  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc0[i] = 0.f;
    acc1[i] = 0.f;
  }
  FX_STAMP(g, 0);
  kloop<FAST, AK, BKIND>(la, lb, lds, kt0, kt1, wm, wn, li, lh, acc0, acc1);
  FX_STAMP(g, 2);
  f32x16 acc = acc0 + acc1;

  // C/D layout of the 32x32 f32 accumulator: col = lane&31, row = (r&3)+8*(r>>2)+4*(lane>>5)
  const int col = n0 + wn * 32 + li;
  const int rbase = m0 + wm * 32 + 4 * lh;
  if (g.split > 1) {
    if (col < g.N) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < g.M) g.ws[(((long long)bidx * g.split + sk) * g.M + row) * g.N + col] = acc[r];
      }
    }
    if (g.tile_cnt)   // flag: the last word of the LDS ring (free after the k loop's final barrier)
      splitk_finish<BM, BN>(g, bidx, m0, n0, (bidx * g.tiles_y + ty) * g.tiles_x + tx,
                            reinterpret_cast<int*>(&lds[NSLOT * 2 * IMG - 1]));
    return;
  }
  if (col >= g.N) return;
  if (!g.c_last && !g.c_tap_cin && !g.gate && g.beta == 0.f && !g.drop_thr) {
    // common forward epilogue: every read (bias, residual) is issued before the first store,
    // so the 16 loads overlap instead of queueing behind stores they might alias
    const float bv = g.bias ? g.bias[(long long)bidx * g.bias_bs + col] : 0.f;
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
  } else if (g.beta != 0.f) {
    // accumulating (dW into param.grad): load the 16 old values before the first store
    float cold[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) cold[r] = *epilogue_ptr(g, bidx, min(rbase + (r & 3) + 8 * (r >> 2), g.M - 1), col);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      if (row < g.M) epilogue_store(g, bidx, row, col, acc[r], true, cold[r]);
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

// ---------------------------------------------------------------- wide tile (128 x 64)
// The 64x64 tile moves 32 KB per 64-deep stage for 0.5 MFLOP: at the f32 MFMA rate that is ~32 B/clk
// per CU, i.e. the XCD L2 bandwidth, so that kernel is L2-bound near 40 % of peak.  Here a block
// owns 128 rows x 64 cols: two 64x64 A stages (the same loaders, rows m0 and m0+64) and one B stage
// per step, 48 KB for 1 MFLOP (1.5x the intensity).  Wave w computes rows 64*(w>>1) .. +63 (two
// 32x32 sub-tiles sharing one B fragment) of columns 32*(w&1) .. +31: per stage 64 MFMAs (4096
// matrix-core cycles) per wave.  LDS: 3-slot ring of [A0 | A1 | B] images = 153 KB, one block
// per CU, one wave per SIMD.  FAST operands only (chosen on the host).
constexpr int WBM = 128;
template <int AK, int BKd>
__device__ __forceinline__ void wide_stage(const Loader<AK, true>& la0, const Loader<AK, true>& la1,
                                           const Loader<BKd, true>& lb, const float* cur, float* wslot, int kload,
                                           const float4* rs0, const float4* rs1, const float4* rsb, unsigned ms0,
                                           unsigned ms1, unsigned msb, float4* rn0, float4* rn1, float4* rnb,
                                           unsigned& mn0, unsigned& mn1, unsigned& mnb, int wm, int wn, int li,
                                           int lh, f32x16& acc0, f32x16& acc1) {
  using LA = Loader<AK, true>;
  using LB = Loader<BKd, true>;
  const float* ia = cur + wm * IMG;
  const float* ib = cur + 2 * IMG;
  float4 f0[8], f1[8], fb[8];
  f0[0] = LA::frag(ia, 0, li, lh, 0);
  f1[0] = LA::frag(ia, 32, li, lh, 0);
  fb[0] = LB::frag(ib, wn * 32, li, lh, 0);
  f0[1] = LA::frag(ia, 0, li, lh, 1);
  f1[1] = LA::frag(ia, 32, li, lh, 1);
  fb[1] = LB::frag(ib, wn * 32, li, lh, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(f0[q].x, fb[q].x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(f1[q].x, fb[q].x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(f0[q].y, fb[q].y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(f1[q].y, fb[q].y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(f0[q].z, fb[q].z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(f1[q].z, fb[q].z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(f0[q].w, fb[q].w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(f1[q].w, fb[q].w, acc1, 0, 0, 0);
    if (q + 2 < 8) {
      f0[q + 2] = LA::frag(ia, 0, li, lh, q + 2);
      f1[q + 2] = LA::frag(ia, 32, li, lh, q + 2);
      fb[q + 2] = LB::frag(ib, wn * 32, li, lh, q + 2);
    }
    // the next loads' address work runs beside the first MFMA groups, not ahead of them
    if (q == 0) la0.load(kload, rn0, mn0);
    if (q == 1) la1.load(kload, rn1, mn1);
    if (q == 2) lb.load(kload, rnb, mnb);
    // the stored set was loaded a whole stage ago; storing it late in this stage gives those loads
    // ~1.7 stages to land (PMC: waits on them were a quarter of the wave cycles when stored early)
    if (q == 5) la0.store(wslot, rs0, ms0);
    if (q == 6) la1.store(wslot + IMG, rs1, ms1);
    if (q == 7) lb.store(wslot + 2 * IMG, rsb, msb);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int AK, int BKd>
__device__ __forceinline__ void wide_kloop(const Loader<AK, true>& la0, const Loader<AK, true>& la1,
                                           const Loader<BKd, true>& lb, float* lds, int kt0, int kt1, int wm, int wn,
                                           int li, int lh, f32x16& acc0, f32x16& acc1) {
  const int n = kt1 - kt0;
  if (n <= 0) return;
  const int klast = (kt1 - 1) * BK;
  constexpr int SLOT = 3 * IMG;
  float4 a0x[4], a1x[4], bx[4], a0y[4], a1y[4], by[4];
  unsigned m0x, m1x, mbx, m0y, m1y, mby;
  la0.load(kt0 * BK, a0x, m0x);
  la1.load(kt0 * BK, a1x, m1x);
  lb.load(kt0 * BK, bx, mbx);
  la0.load(min((kt0 + 1) * BK, klast), a0y, m0y);
  la1.load(min((kt0 + 1) * BK, klast), a1y, m1y);
  lb.load(min((kt0 + 1) * BK, klast), by, mby);
  la0.store(lds, a0x, m0x);
  la1.store(lds + IMG, a1x, m1x);
  lb.store(lds + 2 * IMG, bx, mbx);
  la0.store(lds + SLOT, a0y, m0y);
  la1.store(lds + SLOT + IMG, a1y, m1y);
  lb.store(lds + SLOT + 2 * IMG, by, mby);
  la0.load(min((kt0 + 2) * BK, klast), a0x, m0x);
  la1.load(min((kt0 + 2) * BK, klast), a1x, m1x);
  lb.load(min((kt0 + 2) * BK, klast), bx, mbx);
  __syncthreads();
  int slot = 0;
  auto iter = [&](int i, const float4* s0, const float4* s1, const float4* sb, unsigned q0, unsigned q1, unsigned qb,
                  float4* n0, float4* n1, float4* nb, unsigned& p0, unsigned& p1, unsigned& pb) FX_INLINE {
    const int ws = slot == 0 ? 2 : slot - 1;
    wide_stage<AK, BKd>(la0, la1, lb, lds + slot * SLOT, lds + ws * SLOT, min((kt0 + i + 3) * BK, klast), s0, s1, sb,
                        q0, q1, qb, n0, n1, nb, p0, p1, pb, wm, wn, li, lh, acc0, acc1);
    __syncthreads();
    slot = slot == 2 ? 0 : slot + 1;
  };
  int i = 0;
  for (; i + 1 < n; i += 2) {
    iter(i, a0x, a1x, bx, m0x, m1x, mbx, a0y, a1y, by, m0y, m1y, mby);
    iter(i + 1, a0y, a1y, by, m0y, m1y, mby, a0x, a1x, bx, m0x, m1x, mbx);
  }
  if (i < n) iter(i, a0x, a1x, bx, m0x, m1x, mbx, a0y, a1y, by, m0y, m1y, mby);
}

__device__ __forceinline__ void tile_epilogue(const GemmDev& g, int bidx, int rbase, int col, const f32x16& acc) {
  if (col >= g.N) return;
  if (!g.c_last && !g.c_tap_cin && !g.gate && g.beta == 0.f && !g.drop_thr) {
    const float bv = g.bias ? g.bias[(long long)bidx * g.bias_bs + col] : 0.f;
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
      if (row < g.M) cb[(long long)row * g.ldc] = v;   // (non-temporal stores measured even: round 2)
    }
  } else {   // (a preloaded-C variant here costs the 128x64 kernel 416 B of scratch)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = rbase + (r & 3) + 8 * (r >> 2);
      if (row < g.M) epilogue_store(g, bidx, row, col, acc[r]);
    }
  }
}

template <int AK, int BKIND>
__global__ __launch_bounds__(NTHREADS) void gemm_f32_wide_kernel(GemmDev g) {
  __shared__ float lds[NSLOT * 3 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  int tx, ty, z;
  block_tile(g, tx, ty, z);
  const int n0 = tx * BN, m0 = ty * WBM;
  const int bidx = z / g.split, sk = z - bidx * g.split;
  const int nkt = (g.K + BK - 1) / BK;
  const int kt0 = sk * g.kt_per_split;
  const int kt1 = min(nkt, kt0 + g.kt_per_split);
  Loader<AK, true> la0, la1;
  Loader<BKIND, true> lb;
  const float* pa = g.a.ptr + (long long)bidx * g.a.batch_stride;
  la0.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0, g.M, g.K, tid, g.soff, g.nsoff);
  la1.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0 + BM, g.M, g.K, tid, g.soff, g.nsoff);
  lb.init(batch_op_b(g.b, g.b_dil_growth, bidx), g.b.ptr + (long long)bidx * g.b.batch_stride, n0, g.N, g.K, tid, g.soff, g.nsoff);
  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc0[i] = 0.f;
    acc1[i] = 0.f;
  }
  wide_kloop<AK, BKIND>(la0, la1, lb, lds, kt0, kt1, wm, wn, li, lh, acc0, acc1);
  const int col = n0 + wn * 32 + li;
  const int rb0 = m0 + wm * 64 + 4 * lh, rb1 = rb0 + 32;
  if (g.split > 1) {
    if (col < g.N) {
      float* slab = g.ws + ((long long)bidx * g.split + sk) * g.M * (long long)g.N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row0 = rb0 + (r & 3) + 8 * (r >> 2), row1 = row0 + 32;
        if (row0 < g.M) slab[(long long)row0 * g.N + col] = acc0[r];
        if (row1 < g.M) slab[(long long)row1 * g.N + col] = acc1[r];
      }
    }
    if (g.tile_cnt)
      splitk_finish<WBM, BN>(g, bidx, m0, n0, (bidx * g.tiles_y + ty) * g.tiles_x + tx,
                             reinterpret_cast<int*>(&lds[NSLOT * 3 * IMG - 1]));
    return;
  }
  tile_epilogue(g, bidx, rb0, col, acc0);
  tile_epilogue(g, bidx, rb1, col, acc1);
}

// ---------------------------------------------------------------- wide tile, two waves per SIMD
// The same 128 x 64 tile and LDS ring with 8 waves (512 threads): wave w owns ONE 32x32 sub-tile
// (rows 32 (w>>1) of the 128, columns 32 (w&1)), 32 MFMAs per stage over two accumulators, and
// each thread stages 2 float4 per operand image (Loader NJ = 2).  PMC on the 4-wave kernel: the
// matrix pipe was busy 51 % of the wave cycles, the rest waits (barrier / loads, 24 %) and issue
// of the address / select / LDS work (26 %) that one wave cannot hide behind its own MFMAs; with
// a partner wave on the SIMD, one wave's MFMAs run while the other issues or waits.
constexpr int W8T = 512;
template <int AK, int BKd, int PH>
__device__ __forceinline__ void wide8_stage(const Loader<AK, true, 2>& la0, const Loader<AK, true, 2>& la1,
                                            const Loader<BKd, true, 2>& lb, const float* cur, float* wslot,
                                            int kload, const float4* rs0, const float4* rs1, const float4* rsb,
                                            unsigned ms0, unsigned ms1, unsigned msb, float4* rn0, float4* rn1,
                                            float4* rnb, unsigned& mn0, unsigned& mn1, unsigned& mnb, int ai, int wr,
                                            int wn, int li, int lh, f32x16& acc0, f32x16& acc1) {
  using LA = Loader<AK, true, 2>;
  using LB = Loader<BKd, true, 2>;
  const float* ia = cur + ai * IMG;
  const float* ib = cur + 2 * IMG;
  float4 fa[8], fb[8];
  fa[0] = LA::frag(ia, wr, li, lh, 0);
  fb[0] = LB::frag(ib, wn * 32, li, lh, 0);
  fa[1] = LA::frag(ia, wr, li, lh, 1);
  fb[1] = LB::frag(ib, wn * 32, li, lh, 1);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    f32x16& acc = (q & 1) ? acc1 : acc0;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[q].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[q].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[q].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[q].w, acc, 0, 0, 0);
    if (q + 2 < 8) {
      fa[q + 2] = LA::frag(ia, wr, li, lh, q + 2);
      fb[q + 2] = LB::frag(ib, wn * 32, li, lh, q + 2);
    }
    // staggered halves: waves 0-3 (PH 0) load early and store late in the stage, their SIMD
    // partners 4-7 (PH 1) the other way round, so one wave of each SIMD issues plain MFMA groups
    // while the other does its load / LDS-store work
    if (q == (PH ? 4 : 0)) la0.load(kload, rn0, mn0);
    if (q == (PH ? 5 : 1)) la1.load(kload, rn1, mn1);
    if (q == (PH ? 6 : 2)) lb.load(kload, rnb, mnb);
    if (q == (PH ? 1 : 5)) la0.store(wslot, rs0, ms0);
    if (q == (PH ? 2 : 6)) la1.store(wslot + IMG, rs1, ms1);
    if (q == (PH ? 3 : 7)) lb.store(wslot + 2 * IMG, rsb, msb);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// FX_PREC_F32S on the f32 kernel's LDS ring: the fp32 stage images stay as they are and each wave
// splits its own MFMA operands in registers (row-major A and B images only).  Per 16-deep k chunk q
// a lane takes k in [32 lh + 8 q, +8) of the 64-deep stage (two float4 reads per operand: conflict-
// free on the 68-float rows), splits the 8 values of A and of B into NP bf16x8 pieces and issues the
// NP (NP + 1) / 2 piece products on v_mfma_f32_32x32x16_bf16: 4 LDS reads per 6 MFMAs where
// pre-split images need 6, and 4 instead of 6 LDS bytes written per element.
typedef __bf16 bf16x8r __attribute__((ext_vector_type(8)));

template <int NP>
__device__ __forceinline__ void split8(const float4& lo, const float4& hi, bf16x8r* p) {
  const float e[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)e[j];
    p[0][j] = h;
    if (NP > 1) {
      const float r1 = e[j] - (float)h;
      const __bf16 m = (__bf16)r1;
      p[1][j] = m;
      if (NP > 2) p[2][j] = (__bf16)(r1 - (float)m);
    }
  }
}

template <int NP>
__device__ __forceinline__ void split_products(const bf16x8r* a, const bf16x8r* b, f32x16& acc0, f32x16& acc1) {
  if (NP > 2) {
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc1, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc1, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc1, 0, 0, 0);
  }
  if (NP > 1) {
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc1, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc1, 0, 0, 0);
  }
  acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc0, 0, 0, 0);
}

template <int AK, int BKd, int PH, int NP>
__device__ __forceinline__ void wide8s_stage(const Loader<AK, true, 2>& la0, const Loader<AK, true, 2>& la1,
                                             const Loader<BKd, true, 2>& lb, const float* cur, float* wslot,
                                             int kload, const float4* rs0, const float4* rs1, const float4* rsb,
                                             unsigned ms0, unsigned ms1, unsigned msb, float4* rn0, float4* rn1,
                                             float4* rnb, unsigned& mn0, unsigned& mn1, unsigned& mnb, int ai, int wr,
                                             int wn, int li, int lh, f32x16& acc0, f32x16& acc1) {
  const float* ia = cur + ai * IMG + (wr + li) * RS + 32 * lh;
  const float* ib = cur + 2 * IMG + (wn * 32 + li) * RS + 32 * lh;
  float4 fa[4][2], fb[4][2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    fa[q][0] = *reinterpret_cast<const float4*>(ia + 8 * q);
    fa[q][1] = *reinterpret_cast<const float4*>(ia + 8 * q + 4);
    fb[q][0] = *reinterpret_cast<const float4*>(ib + 8 * q);
    fb[q][1] = *reinterpret_cast<const float4*>(ib + 8 * q + 4);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bf16x8r pa[NP], pb[NP];
    split8<NP>(fa[q][0], fa[q][1], pa);
    split8<NP>(fb[q][0], fb[q][1], pb);
    if (q + 2 < 4) {
      fa[q + 2][0] = *reinterpret_cast<const float4*>(ia + 8 * (q + 2));
      fa[q + 2][1] = *reinterpret_cast<const float4*>(ia + 8 * (q + 2) + 4);
      fb[q + 2][0] = *reinterpret_cast<const float4*>(ib + 8 * (q + 2));
      fb[q + 2][1] = *reinterpret_cast<const float4*>(ib + 8 * (q + 2) + 4);
    }
    split_products<NP>(pa, pb, acc0, acc1);
    // the same staggered load / store placement as the f32 stage (two waves per SIMD)
    if (q == (PH ? 2 : 0)) {
      la0.load(kload, rn0, mn0);
      la1.load(kload, rn1, mn1);
    }
    if (q == (PH ? 3 : 1)) lb.load(kload, rnb, mnb);
    if (q == (PH ? 0 : 2)) {
      la0.store(wslot, rs0, ms0);
      la1.store(wslot + IMG, rs1, ms1);
    }
    if (q == (PH ? 1 : 3)) lb.store(wslot + 2 * IMG, rsb, msb);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int AK, int BKd, int PH, int NP = 0>
__device__ __forceinline__ void wide8_kloop(const Loader<AK, true, 2>& la0, const Loader<AK, true, 2>& la1,
                                            const Loader<BKd, true, 2>& lb, float* lds, int kt0, int kt1, int ai,
                                            int wr, int wn, int li, int lh, f32x16& acc0, f32x16& acc1) {
  const int n = kt1 - kt0;
  if (n <= 0) return;
  const int klast = (kt1 - 1) * BK;
  constexpr int SLOT = 3 * IMG;
  float4 a0x[2], a1x[2], bx[2], a0y[2], a1y[2], by[2];
  unsigned m0x, m1x, mbx, m0y, m1y, mby;
  la0.load(kt0 * BK, a0x, m0x);
  la1.load(kt0 * BK, a1x, m1x);
  lb.load(kt0 * BK, bx, mbx);
  la0.load(min((kt0 + 1) * BK, klast), a0y, m0y);
  la1.load(min((kt0 + 1) * BK, klast), a1y, m1y);
  lb.load(min((kt0 + 1) * BK, klast), by, mby);
  la0.store(lds, a0x, m0x);
  la1.store(lds + IMG, a1x, m1x);
  lb.store(lds + 2 * IMG, bx, mbx);
  la0.store(lds + SLOT, a0y, m0y);
  la1.store(lds + SLOT + IMG, a1y, m1y);
  lb.store(lds + SLOT + 2 * IMG, by, mby);
  la0.load(min((kt0 + 2) * BK, klast), a0x, m0x);
  la1.load(min((kt0 + 2) * BK, klast), a1x, m1x);
  lb.load(min((kt0 + 2) * BK, klast), bx, mbx);
  __syncthreads();
  int slot = 0;
  auto iter = [&](int i, const float4* s0, const float4* s1, const float4* sb, unsigned q0, unsigned q1, unsigned qb,
                  float4* n0, float4* n1, float4* nb, unsigned& p0, unsigned& p1, unsigned& pb) FX_INLINE {
    const int ws = slot == 0 ? 2 : slot - 1;
    if constexpr (NP == 0)
      wide8_stage<AK, BKd, PH>(la0, la1, lb, lds + slot * SLOT, lds + ws * SLOT, min((kt0 + i + 3) * BK, klast), s0,
                               s1, sb, q0, q1, qb, n0, n1, nb, p0, p1, pb, ai, wr, wn, li, lh, acc0, acc1);
    else
      wide8s_stage<AK, BKd, PH, NP>(la0, la1, lb, lds + slot * SLOT, lds + ws * SLOT, min((kt0 + i + 3) * BK, klast),
                                    s0, s1, sb, q0, q1, qb, n0, n1, nb, p0, p1, pb, ai, wr, wn, li, lh, acc0, acc1);
    __syncthreads();   // (a barrier after the next stage's first MFMA group instead measured 3 % slower)
    slot = slot == 2 ? 0 : slot + 1;
  };
  int i = 0;
  for (; i + 1 < n; i += 2) {
    iter(i, a0x, a1x, bx, m0x, m1x, mbx, a0y, a1y, by, m0y, m1y, mby);
    iter(i + 1, a0y, a1y, by, m0y, m1y, mby, a0x, a1x, bx, m0x, m1x, mbx);
  }
  if (i < n) iter(i, a0x, a1x, bx, m0x, m1x, mbx, a0y, a1y, by, m0y, m1y, mby);
}

template <int AK, int BKIND, int NP = 0>
__global__ __launch_bounds__(W8T) void gemm_f32_wide8_kernel(GemmDev g) {
  __shared__ float lds[NSLOT * 3 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  const int ai = wm >> 1, wr = (wm & 1) * 32;   // A image (rows m0 / m0 + 64) and row offset in it
  // persist: gridDim.x (a multiple of 8) workgroups walk the tiles as virtual workgroup ids blockIdx.x +
  // i gridDim.x -- same XCD as the physical one -- saving a dispatch and teardown per tile
  for (int vb = blockIdx.x;; vb += gridDim.x) {
  int tx, ty, z;
  if (g.persist) {
    if (vb >= g.persist) break;
    block_tile_id(g, vb, tx, ty);
    z = 0;
  } else {
    block_tile(g, tx, ty, z);
  }
  const int n0 = tx * BN, m0 = ty * WBM;
  const int bidx = z / g.split, sk = z - bidx * g.split;
  const int nkt = (g.K + BK - 1) / BK;
  const int kt0 = sk * g.kt_per_split;
  const int kt1 = min(nkt, kt0 + g.kt_per_split);
  Loader<AK, true, 2> la0, la1;
  Loader<BKIND, true, 2> lb;
  const float* pa = g.a.ptr + (long long)bidx * g.a.batch_stride;
  la0.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0, g.M, g.K, tid, g.soff, g.nsoff);
  la1.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0 + BM, g.M, g.K, tid, g.soff, g.nsoff);
  lb.init(batch_op_b(g.b, g.b_dil_growth, bidx), g.b.ptr + (long long)bidx * g.b.batch_stride, n0, g.N, g.K, tid, g.soff, g.nsoff);
  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc0[i] = 0.f;
    acc1[i] = 0.f;
  }
  if (wave >= 4)   // the second wave of each SIMD runs the staggered stage schedule
    wide8_kloop<AK, BKIND, 1, NP>(la0, la1, lb, lds, kt0, kt1, ai, wr, wn, li, lh, acc0, acc1);
  else
    wide8_kloop<AK, BKIND, 0, NP>(la0, la1, lb, lds, kt0, kt1, ai, wr, wn, li, lh, acc0, acc1);
  const f32x16 acc = acc0 + acc1;
  const int col = n0 + wn * 32 + li;
  const int rbase = m0 + wm * 32 + 4 * lh;
  if (g.split > 1) {
    if (col < g.N) {
      float* slab = g.ws + ((long long)bidx * g.split + sk) * g.M * (long long)g.N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < g.M) slab[(long long)row * g.N + col] = acc[r];
      }
    }
    if (g.tile_cnt)
      splitk_finish<WBM, BN>(g, bidx, m0, n0, (bidx * g.tiles_y + ty) * g.tiles_x + tx,
                             reinterpret_cast<int*>(&lds[NSLOT * 3 * IMG - 1]));
    return;
  }
  tile_epilogue(g, bidx, rbase, col, acc);
  if (!g.persist) break;
  __syncthreads();   // the next tile's prologue refills the LDS ring
  }
}

// ---------------------------------------------------------------- bf16 arithmetic (FX_PREC_BF16)
// The precision mode's frame-level GEMM: the same 128 x 64 tile, 8 waves and operand loaders as the
// f32 wide8 kernel, fp32 storage and fp32 accumulation, but the products on
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate): each stage's fp32 float4 loads are rounded to
// bf16 (v_cvt_pk_bf16_f32, round to nearest even) when they are written to LDS, so the LDS images
// are half the bytes ([row][k] bf16, 144-B rows: ds_write_b64 in, conflict-free ds_read_b128 out,
// one read = one MFMA operand).  Lane half h of an MFMA takes k in [32h, 32h + 32) of the 64-deep
// stage (8 per instruction), for A and B alike.  With 4 MFMAs per wave per stage the loop is bound
// by operand delivery, not the matrix core, so the ring is deeper than the f32 kernel's: 4 LDS
// slots and 3 register sets, a stage's loads issued 5 stages ahead of its MFMAs and written to LDS
// 2 stages after they were issued.  A row-major (forward and input-gradient GEMMs), B row- or
// column-major (W or W^T); weight gradients (A column-major) stay on the f32 kernels.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int BRS = 72;                 // bf16 row stride of a [row][k] stage image (144 B)
constexpr int BIMG = 64 * BRS;          // bf16 per operand image
constexpr int BSLOT = 3 * BIMG;         // [A0 | A1 | B]
constexpr int BNSL = 4;                 // LDS slots
constexpr int BLAG = 5;                 // stages between a load and the MFMAs that use it

// Row-major kinds: a thread's float4 is 4 consecutive k of one row -> one 8-byte LDS write.
// COLS (B = W stored [k][n], the input-gradient products): the float4 is 4 consecutive rows n at one
// k, written transposed into the [n][k] image as 4 two-byte writes (same bytes, 4x the instructions).
template <int KIND>
__device__ __forceinline__ void store_bf16(const Loader<KIND, true, 2>& L, __bf16* img, const float4* v, unsigned vm) {
  if (Loader<KIND, true, 2>::kRowImg) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float4 x = ((vm >> j) & 1u) ? v[j] : zero4();
      bf16x4 b;
      b[0] = (__bf16)x.x;
      b[1] = (__bf16)x.y;
      b[2] = (__bf16)x.z;
      b[3] = (__bf16)x.w;
      *reinterpret_cast<bf16x4*>(img + (L.ta + 32 * j) * BRS + L.tb) = b;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float one = ((L.omask >> q) & 1u) ? 1.f : 0.f;
        const float x = ((L.emask >> q) & 1u) ? e[q] : one;
        img[(L.tb + q) * BRS + L.ta + 32 * j] = (__bf16)x;
      }
    }
  }
}

__device__ __forceinline__ bf16x8 bfrag(const __bf16* img, int row, int h, int q) {
  return *reinterpret_cast<const bf16x8*>(img + row * BRS + 32 * h + 8 * q);
}

template <int AK, int BKd>
struct BfSet {
  float4 a0[2], a1[2], b[2];
  unsigned m0, m1, mb;
};

template <int AK, int BKd>
__device__ __forceinline__ void bf_load(const Loader<AK, true, 2>& la0, const Loader<AK, true, 2>& la1,
                                        const Loader<BKd, true, 2>& lb, int k0, BfSet<AK, BKd>& r) {
  la0.load(k0, r.a0, r.m0);
  la1.load(k0, r.a1, r.m1);
  lb.load(k0, r.b, r.mb);
}

template <int AK, int BKd>
__device__ __forceinline__ void bf_store(const Loader<AK, true, 2>& la0, const Loader<AK, true, 2>& la1,
                                         const Loader<BKd, true, 2>& lb, __bf16* slot, const BfSet<AK, BKd>& r) {
  store_bf16<AK>(la0, slot, r.a0, r.m0);
  store_bf16<AK>(la1, slot + BIMG, r.a1, r.m1);
  store_bf16<BKd>(lb, slot + 2 * BIMG, r.b, r.mb);
}

template <int AK, int BKd>
__global__ __launch_bounds__(W8T) void gemm_bf16_wide8_kernel(GemmDev g) {
  __shared__ __bf16 lds[BNSL * BSLOT];
  __shared__ int flag[1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  const int ai = wm >> 1, wr = (wm & 1) * 32;
  int tx, ty, z;
  block_tile(g, tx, ty, z);
  const int n0 = tx * BN, m0 = ty * WBM;
  const int bidx = z / g.split, sk = z - bidx * g.split;
  const int nkt = (g.K + BK - 1) / BK;
  const int kt0 = sk * g.kt_per_split;
  const int kt1 = min(nkt, kt0 + g.kt_per_split);
  Loader<AK, true, 2> la0, la1;
  Loader<BKd, true, 2> lb;
  const float* pa = g.a.ptr + (long long)bidx * g.a.batch_stride;
  la0.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0, g.M, g.K, tid, g.soff, g.nsoff);
  la1.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0 + BM, g.M, g.K, tid, g.soff, g.nsoff);
  lb.init(batch_op_b(g.b, g.b_dil_growth, bidx), g.b.ptr + (long long)bidx * g.b.batch_stride, n0, g.N, g.K, tid, g.soff, g.nsoff);
  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc0[i] = 0.f;
    acc1[i] = 0.f;
  }
  const int n = kt1 - kt0;
  if (n > 0) {
    const int klast = (kt1 - 1) * BK;
    auto kof = [&](int i) { return min((kt0 + i) * BK, klast); };
    // prologue: stages 0..2 staged in LDS slots 0..2, stages 3 and 4 in flight (register sets)
    BfSet<AK, BKd> r0, r1, r2;
    bf_load<AK, BKd>(la0, la1, lb, kof(0), r0);
    bf_load<AK, BKd>(la0, la1, lb, kof(1), r1);
    bf_load<AK, BKd>(la0, la1, lb, kof(2), r2);
    bf_store<AK, BKd>(la0, la1, lb, lds, r0);
    bf_load<AK, BKd>(la0, la1, lb, kof(3), r0);
    bf_store<AK, BKd>(la0, la1, lb, lds + BSLOT, r1);
    bf_load<AK, BKd>(la0, la1, lb, kof(4), r1);
    bf_store<AK, BKd>(la0, la1, lb, lds + 2 * BSLOT, r2);
    __syncthreads();
    // stage i: MFMAs on slot i % 4; loads of stage i + 5 into one set; the set loaded at stage i - 2
    // (stage i + 3) written to slot (i + 3) % 4 -- the slot read at stage i - 1, free after the barrier
    auto stage = [&](int i, BfSet<AK, BKd>& ld, const BfSet<AK, BKd>& st) FX_INLINE {
      const __bf16* cur = lds + (i & 3) * BSLOT;
      const __bf16* ia = cur + ai * BIMG;
      const __bf16* ib = cur + 2 * BIMG;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        fa[q] = bfrag(ia, wr + li, lh, q);
        fb[q] = bfrag(ib, wn * 32 + li, lh, q);
      }
      bf_load<AK, BKd>(la0, la1, lb, kof(i + BLAG), ld);
      __builtin_amdgcn_sched_barrier(0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[3], fb[3], acc1, 0, 0, 0);
      bf_store<AK, BKd>(la0, la1, lb, lds + ((i + 3) & 3) * BSLOT, st);
      __syncthreads();
    };
    // register sets rotate with period 3: at stage i, load into set i % 3 ... the set stored is the
    // one loaded two stages earlier, (i + 1) % 3
    int i = 0;
    for (; i + 2 < n; i += 3) {
      stage(i, r2, r0);        // loads stage i+5 -> r2; stores stage i+3 (r0, loaded at i-2)
      stage(i + 1, r0, r1);    // loads i+6 -> r0; stores i+4 (r1)
      stage(i + 2, r1, r2);    // loads i+7 -> r1; stores i+5 (r2)
    }
    if (i < n) stage(i, r2, r0);
    if (i + 1 < n) stage(i + 1, r0, r1);
  }
  const f32x16 acc = acc0 + acc1;
  const int col = n0 + wn * 32 + li;
  const int rbase = m0 + wm * 32 + 4 * lh;
  if (g.split > 1) {
    if (col < g.N) {
      float* slab = g.ws + ((long long)bidx * g.split + sk) * g.M * (long long)g.N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < g.M) slab[(long long)row * g.N + col] = acc[r];
      }
    }
    if (g.tile_cnt) splitk_finish<WBM, BN>(g, bidx, m0, n0, (bidx * g.tiles_y + ty) * g.tiles_x + tx, flag);
    return;
  }
  tile_epilogue(g, bidx, rbase, col, acc);
}

// ---------------------------------------------------------------- fp32 by split bf16 (FX_PREC_F32S)
// fp32 GEMM arithmetic on the bf16 matrix cores: every fp32 operand x is split into NP bf16 pieces
// x = p0 + p1 + p2 (p0 = bf16(x), p1 = bf16(x - p0), p2 = bf16(x - p0 - p1): 8 significant bits each,
// so three pieces carry all 24 bits of an fp32 mantissa) and a.b is summed as the NP (NP + 1) / 2
// piece products of order <= NP - 1 (NP = 3: p0q0 + p0q1 + p1q0 + p0q2 + p2q0 + p1q1; the dropped
// terms are below 3 * 2^-24 |a b|, the size of fp32's own rounding of each product's addition).
// Every piece product is exact in the MFMA's fp32 accumulator.  v_mfma_f32_32x32x16_bf16 runs at 16x
// the f32 MFMA rate, so NP = 3 (6 products) is 2.7x the f32 matrix rate at fp32 accuracy; NP = 2
// (3 products, ~2^-16 relative) exists for measurement only.
// Tile and waves as the f32 wide8 kernel (128 x 64, 8 waves, one 32x32 accumulator pair each), with
// 32-deep stages: a stage's fp32 float4 loads are split when they are written to LDS (each element
// once per tile, not once per reading wave), the images hold the NP pieces of A0 | A1 | B as
// [row][k] bf16 with 80-B rows (conflict-free ds_read_b128: 8 consecutive rows start 20 banks
// apart), 3 LDS slots (138 KB at NP = 3), a stage's loads issued 4 stages ahead in one of 3 register
// sets and written to LDS 2 stages later.  Lane half h of MFMA q takes k in [16q + 8h, +8) for A and
// B alike (the k order inside the sum is free as long as both operands agree).
constexpr int SKW = 32;                 // k per stage
constexpr int SRS = 40;                 // bf16 row stride of a piece image (80 B)
constexpr int SIMG = 64 * SRS;          // bf16 per piece image
typedef __bf16 bf16x8s __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4s __attribute__((ext_vector_type(4)));

template <int NP>
__device__ __forceinline__ void split_pieces(float x, __bf16* p) {
  p[0] = (__bf16)x;
  if (NP > 1) {
    const float r1 = x - (float)p[0];
    p[1] = (__bf16)r1;
    if (NP > 2) p[2] = (__bf16)(r1 - (float)p[1]);
  }
}

// one operand stage (one float4 per thread) into its NP piece images (image p at img + p * SIMG)
template <int KIND, int NP>
__device__ __forceinline__ void store_split(const Loader<KIND, true, 1, SKW>& L, __bf16* img, float4 v, unsigned vm) {
  if (Loader<KIND, true, 1, SKW>::kRowImg) {
    const float4 x = (vm & 1u) ? v : zero4();
    const float e[4] = {x.x, x.y, x.z, x.w};
    bf16x4s b[NP];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __bf16 pc[3];
      split_pieces<NP>(e[q], pc);
#pragma unroll
      for (int p = 0; p < NP; ++p) b[p][q] = pc[p];
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) *reinterpret_cast<bf16x4s*>(img + p * SIMG + L.ta * SRS + L.tb) = b[p];
  } else {
    // COLS (B = W stored [k][n]): 4 consecutive n at one k, written transposed into [n][k]
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float one = ((L.omask >> q) & 1u) ? 1.f : 0.f;
      const float x = ((L.emask >> q) & 1u) ? e[q] : one;
      __bf16 pc[3];
      split_pieces<NP>(x, pc);
#pragma unroll
      for (int p = 0; p < NP; ++p) img[p * SIMG + (L.tb + q) * SRS + L.ta] = pc[p];
    }
  }
}

template <int AK, int BKd>
struct SpSet {
  float4 a0, a1, b;
  unsigned m0, m1, mb;
};

template <int AK, int BKd, int NP>
__global__ __launch_bounds__(W8T) void gemm_split_wide8_kernel(GemmDev g) {
  constexpr int SSLOT = 3 * NP * SIMG;   // [A0 pieces | A1 pieces | B pieces]
  __shared__ __bf16 lds[3 * SSLOT];
  __shared__ int flag[1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  const int ai = wm >> 1, wr = (wm & 1) * 32;
  int tx, ty, z;
  block_tile(g, tx, ty, z);
  const int n0 = tx * BN, m0 = ty * WBM;
  const int bidx = z / g.split, sk = z - bidx * g.split;
  const int nkt = (g.K + SKW - 1) / SKW;
  // kt_per_split counts 64-deep stages (the host's split plan): two 32-deep stages each
  const int kt0 = sk * g.kt_per_split * 2;
  const int kt1 = min(nkt, kt0 + g.kt_per_split * 2);
  Loader<AK, true, 1, SKW> la0, la1;
  Loader<BKd, true, 1, SKW> lb;
  const float* pa = g.a.ptr + (long long)bidx * g.a.batch_stride;
  la0.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0, g.M, g.K, tid, g.soff, g.nsoff);
  la1.init(batch_op_a(g.a, g.a_dil_b1, bidx), pa, m0 + BM, g.M, g.K, tid, g.soff, g.nsoff);
  lb.init(batch_op_b(g.b, g.b_dil_growth, bidx), g.b.ptr + (long long)bidx * g.b.batch_stride, n0, g.N, g.K, tid,
          g.soff, g.nsoff);
  f32x16 acc0, acc1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc0[i] = 0.f;
    acc1[i] = 0.f;
  }
  const int n = kt1 - kt0;
  if (n > 0) {
    const int klast = (kt1 - 1) * SKW;
    auto kof = [&](int i) { return min((kt0 + i) * SKW, klast); };
    auto ld = [&](int i, SpSet<AK, BKd>& r) FX_INLINE {
      la0.load(kof(i), &r.a0, r.m0);
      la1.load(kof(i), &r.a1, r.m1);
      lb.load(kof(i), &r.b, r.mb);
    };
    auto st = [&](__bf16* slot, const SpSet<AK, BKd>& r) FX_INLINE {
      store_split<AK, NP>(la0, slot, r.a0, r.m0);
      store_split<AK, NP>(la1, slot + NP * SIMG, r.a1, r.m1);
      store_split<BKd, NP>(lb, slot + 2 * NP * SIMG, r.b, r.mb);
    };
    // prologue: stages 0, 1 in LDS slots 0, 1; stages 2, 3 in flight (set s % 3 holds stage s)
    SpSet<AK, BKd> r0, r1, r2;
    ld(0, r0);
    ld(1, r1);
    ld(2, r2);
    st(lds, r0);
    ld(3, r0);
    st(lds + SSLOT, r1);
    __syncthreads();
    // stage i: MFMAs on slot i % 3; loads of stage i + 4 into set (i + 1) % 3; stage i + 2 (set
    // (i + 2) % 3, loaded two stages ago) written to slot (i + 2) % 3, read at stage i - 1
    auto stage = [&](int i, SpSet<AK, BKd>& lset, const SpSet<AK, BKd>& sset) FX_INLINE {
      const __bf16* cur = lds + (i % 3) * SSLOT;
      const __bf16* ia = cur + ai * NP * SIMG + (wr + li) * SRS + 8 * lh;
      const __bf16* ib = cur + 2 * NP * SIMG + (wn * 32 + li) * SRS + 8 * lh;
      bf16x8s fa[2][NP], fb[2][NP];
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          fa[q][p] = *reinterpret_cast<const bf16x8s*>(ia + p * SIMG + 16 * q);
          fb[q][p] = *reinterpret_cast<const bf16x8s*>(ib + p * SIMG + 16 * q);
        }
      ld(i + 4, lset);
      __builtin_amdgcn_sched_barrier(0);
      // the split + LDS stores of stage i + 2 (another slot) are issued between the MFMA groups, so
      // they run while the matrix core works on this stage's products
      __bf16* wslot = lds + ((i + 2) % 3) * SSLOT;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (NP > 2) {
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][1], fb[q][1], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][2], fb[q][0], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][0], fb[q][2], acc1, 0, 0, 0);
        }
        if (NP > 1) {
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][1], fb[q][0], acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][0], fb[q][1], acc1, 0, 0, 0);
        }
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[q][0], fb[q][0], acc0, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (q == 0) {
          store_split<AK, NP>(la0, wslot, sset.a0, sset.m0);
          store_split<AK, NP>(la1, wslot + NP * SIMG, sset.a1, sset.m1);
        } else {
          store_split<BKd, NP>(lb, wslot + 2 * NP * SIMG, sset.b, sset.mb);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
    };
    int i = 0;
    for (; i + 2 < n; i += 3) {
      stage(i, r1, r2);
      stage(i + 1, r2, r0);
      stage(i + 2, r0, r1);
    }
    if (i < n) stage(i, r1, r2);
    if (i + 1 < n) stage(i + 1, r2, r0);
  }
  const f32x16 acc = acc0 + acc1;
  const int col = n0 + wn * 32 + li;
  const int rbase = m0 + wm * 32 + 4 * lh;
  if (g.split > 1) {
    if (col < g.N) {
      float* slab = g.ws + ((long long)bidx * g.split + sk) * g.M * (long long)g.N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < g.M) slab[(long long)row * g.N + col] = acc[r];
      }
    }
    if (g.tile_cnt) splitk_finish<WBM, BN>(g, bidx, m0, n0, (bidx * g.tiles_y + ty) * g.tiles_x + tx, flag);
    return;
  }
  tile_epilogue(g, bidx, rbase, col, acc);
}

// Separate split-K reduce: a thread sums 4 consecutive elements (float4 over the slabs when M*N % 4 == 0
// and the workspace is 16-B aligned) with up to 8 slab loads in flight, slabs added in order
// (deterministic); the epilogue runs per element.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmDev g, int vec) {
  const long long total = (long long)g.M * g.N;
  const int bidx = blockIdx.y;
  const float* ws = g.ws + (long long)bidx * g.split * total;
  const long long n4 = (total + 3) >> 2;
  for (long long i4 = (long long)blockIdx.x * blockDim.x + threadIdx.x; i4 < n4; i4 += (long long)gridDim.x * blockDim.x) {
    const long long i = i4 * 4;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (vec) {
      for (int k0 = 0; k0 < g.split; k0 += 8) {
        float4 x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          x[j] = *reinterpret_cast<const float4*>(ws + (long long)min(k0 + j, g.split - 1) * total + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (k0 + j < g.split) {
            s[0] += x[j].x;
            s[1] += x[j].y;
            s[2] += x[j].z;
            s[3] += x[j].w;
          }
        }
      }
    } else {
      for (int e = 0; e < 4; ++e)
        if (i + e < total)
          for (int k = 0; k < g.split; ++k) s[e] += ws[(long long)k * total + i + e];
    }
    int m = (int)(i / g.N), n = (int)(i - (long long)m * g.N);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (i + e < total) epilogue_store(g, bidx, m, n, s[e]);
      if (++n == g.N) {
        n = 0;
        ++m;
      }
    }
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
                                      float* v, const SeqOff& soff, int nsoff) {
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
    // edge chunk: clamped, unconditional loads (all 16 in flight at once), zeroed by select
    const int rc = min(r, R - 1);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float x = base[(long long)rc * o.ld + min(k0 + j, K - 1)];
      v[j] = (r < R && k0 + j < K) ? x : 0.f;
    }
  } else if (KIND == COLS) {
    // clamped, unconditional loads so the compiler issues all 16 before the first wait (the ones
    // column is a virtual operand column: its row index is clamped too and the value replaced)
    const bool ones = o.ones_col && r == o.ones_col - 1;
    const int rc = max(min(r, o.ones_col ? o.ones_col - 2 : R - 1), 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float x = base[(long long)min(k0 + j, K - 1) * o.ld + rc];
      v[j] = (r < R && k0 + j < K) ? (ones ? 1.f : x) : 0.f;
    }
  } else {  // ROWS_GEN
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = (r < R && k0 + j < K) ? fetch_rm(o, base, r, k0 + j, soff, nsoff) : 0.f;
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
__device__ __forceinline__ void direct_body(const GemmDev& g, int bx, int by, int z, float* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int n0 = bx * 32, m0 = by * 32;
  const int bidx = z / g.split, sk = z - bidx * g.split;
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
    dload<AK>(g.a, pa, ra, g.M, c * DCH + ko, g.K, av, a0, g.soff, g.nsoff);
    dload<BKd>(g.b, pb, rb, g.N, c * DCH + ko, g.K, bv, b0, g.soff, g.nsoff);
  }
  for (; c < c1; c += 2 * nw) {
    const int cn = c + nw;
    if (cn < c1) {
      dload<AK>(g.a, pa, ra, g.M, cn * DCH + ko, g.K, av, a1, g.soff, g.nsoff);
      dload<BKd>(g.b, pb, rb, g.N, cn * DCH + ko, g.K, bv, b1, g.soff, g.nsoff);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc, 0, 0, 0);
    const int cnn = cn + nw;
    if (cnn < c1) {
      dload<AK>(g.a, pa, ra, g.M, cnn * DCH + ko, g.K, av, a0, g.soff, g.nsoff);
      dload<BKd>(g.b, pb, rb, g.N, cnn * DCH + ko, g.K, bv, b0, g.soff, g.nsoff);
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
  } else if (g.split > 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) direct_finish(g, bidx, sk, m0 + (r & 3) + 8 * (r >> 2) + 4 * lh, n0 + li, acc[r]);
  } else if (g.beta != 0.f) {
    // accumulate into C (e.g. K = 64 dW GEMMs into param.grad): all 16 old values are loaded
    // before the first store; element by element each store would hold back the next load
    float cold[16];
    const int col = min(n0 + li, g.N - 1);
#pragma unroll
    for (int r = 0; r < 16; ++r) cold[r] = *epilogue_ptr(g, bidx, min(m0 + (r & 3) + 8 * (r >> 2) + 4 * lh, g.M - 1), col);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (row < g.M && n0 + li < g.N) epilogue_store(g, bidx, row, n0 + li, acc[r], true, cold[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) direct_finish(g, bidx, sk, m0 + (r & 3) + 8 * (r >> 2) + 4 * lh, n0 + li, acc[r]);
  }
  if (g.split > 1 && g.tile_cnt)
    splitk_finish<32, 32>(g, bidx, m0, n0, (bidx * g.tiles_y + by) * g.tiles_x + bx,
                          reinterpret_cast<int*>(&red[DMAXW * 16 * 64]));
}

template <int AK, int BKd>
__global__ __launch_bounds__(DMAXW * 64) void gemm_direct_kernel(GemmDev g) {
  __shared__ float red[DMAXW * 16 * 64 + 1];   // wave partials + the split-K "last block" flag
  direct_body<AK, BKd>(g, blockIdx.x, blockIdx.y, blockIdx.z, red);
}

// Several independent small GEMMs in ONE launch (e.g. the dW/db and dX GEMMs of one linear layer, both
// reading the same dY): the flat block index picks the problem (block-uniform), each problem keeps
// its own grid, operand kinds, split and epilogue.  Saves a launch (~2.7 us back to back) per member.
constexpr int GMAX = 4;
struct GemmGroup {
  GemmDev g[GMAX];
  int kinds[GMAX];         // ak * 8 + bk
  int start[GMAX + 1];     // first flat block of each problem
  int n;
};

__device__ __forceinline__ void direct_dispatch(const GemmDev& g, int kinds, int local, float* red) {
  const int txy = g.tiles_x * g.tiles_y;
  const int z = local / txy, r = local - z * txy, by = r / g.tiles_x, bx = r - by * g.tiles_x;
  switch (kinds) {
    case ROWS * 8 + ROWS: direct_body<ROWS, ROWS>(g, bx, by, z, red); break;
    case ROWS * 8 + COLS: direct_body<ROWS, COLS>(g, bx, by, z, red); break;
    case ROWS_GEN * 8 + ROWS: direct_body<ROWS_GEN, ROWS>(g, bx, by, z, red); break;
    case ROWS_GEN * 8 + COLS: direct_body<ROWS_GEN, COLS>(g, bx, by, z, red); break;
    case COLS * 8 + ROWS: direct_body<COLS, ROWS>(g, bx, by, z, red); break;
    case COLS * 8 + COLS: direct_body<COLS, COLS>(g, bx, by, z, red); break;
    default: break;
  }
}

__global__ __launch_bounds__(DMAXW * 64) void gemm_direct_group_kernel(GemmGroup G) {
  __shared__ float red[DMAXW * 16 * 64 + 1];
  const int id = blockIdx.x;
  // constant member indices only (a runtime index into the kernel argument would copy it to scratch)
  if (id < G.start[1]) direct_dispatch(G.g[0], G.kinds[0], id, red);
  else if (id < G.start[2]) direct_dispatch(G.g[1], G.kinds[1], id - G.start[1], red);
  else if (id < G.start[3]) direct_dispatch(G.g[2], G.kinds[2], id - G.start[2], red);
  else direct_dispatch(G.g[3], G.kinds[3], id - G.start[3], red);
}

// bias-gradient column sums, two deterministic stages (used only where no dW GEMM carries them)
constexpr int CS_ROWS = 128;
// batch z: x + z * x_bs, partials at ws + z * nblk * N, out + z * out_bs
__global__ __launch_bounds__(256) void colsum_stage1(const float* x, long long ld, long long x_bs, int M, int N,
                                                     float* ws) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * CS_ROWS;
  x += (long long)blockIdx.z * x_bs;
  ws += (long long)blockIdx.z * gridDim.y * N;
  float s = 0.f;
  if (n < N)
    for (int r = r0 + rg; r < min(M, r0 + CS_ROWS); r += 4) s += x[(long long)r * ld + n];
  __shared__ float red[4][64];
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && n < N) ws[(long long)blockIdx.y * N + n] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                                            red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ __launch_bounds__(256) void colsum_stage2(const float* ws, int nblk, int N, float* out, long long out_bs,
                                                     int acc) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  ws += (long long)blockIdx.y * nblk * N;
  out += (long long)blockIdx.y * out_bs;
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
  if (o.trans) return o.conv_taps ? (o.nseq > 0 ? COLS_CONVR : COLS_CONV) : COLS;
  if (o.conv_taps) return (vec && o.conv_cin % BK == 0) ? ROWS_CONV : ROWS_GEN;   // a stage stays in one tap
  if (o.pos) return ROWS_GEN;
  if (o.ptr1 || o.rows0 || o.rows1) return (vec && (!o.ptr1 || o.k_split % BK == 0)) ? ROWS_CAT : ROWS_GEN;
  return ROWS;
}

template <int AK, int BKd>
void launch_t(dim3 grid, hipStream_t s, const GemmDev& g, bool fast) {
  if (fast)
    fx_launch((gemm_f32_kernel<AK, BKd, true>), grid, dim3(NTHREADS), 0, s, g);
  else
    fx_launch((gemm_f32_kernel<AK, BKd, false>), grid, dim3(NTHREADS), 0, s, g);
}

template <int AK>
int launch_wide_b(int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  switch (bk) {
    case ROWS: fx_launch((gemm_f32_wide_kernel<AK, ROWS>), grid, dim3(NTHREADS), 0, s, g); return FX_OK;
    case COLS: fx_launch((gemm_f32_wide_kernel<AK, COLS>), grid, dim3(NTHREADS), 0, s, g); return FX_OK;
    case COLS_CONV:
      fx_launch((gemm_f32_wide_kernel<AK, COLS_CONV>), grid, dim3(NTHREADS), 0, s, g);
      return FX_OK;
    case COLS_CONVR:
      if constexpr (AK == COLS) {
        fx_launch((gemm_f32_wide_kernel<AK, COLS_CONVR>), grid, dim3(NTHREADS), 0, s, g);
        return FX_OK;
      }
      break;
    case COLS_KT:
      if constexpr (AK == COLS_KT) {
        fx_launch((gemm_f32_wide_kernel<AK, COLS_KT>), grid, dim3(NTHREADS), 0, s, g);
        return FX_OK;
      }
      break;
    default: break;
  }
  set_error("gemm(wide): unsupported B operand kind");
  return FX_ERR_UNSUPPORTED;
}

template <int AK>
int launch_wide8_b(int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  switch (bk) {
    case ROWS: fx_launch((gemm_f32_wide8_kernel<AK, ROWS>), grid, dim3(W8T), 0, s, g); return FX_OK;
    case COLS: fx_launch((gemm_f32_wide8_kernel<AK, COLS>), grid, dim3(W8T), 0, s, g); return FX_OK;
    case COLS_CONV:
      fx_launch((gemm_f32_wide8_kernel<AK, COLS_CONV>), grid, dim3(W8T), 0, s, g);
      return FX_OK;
    case COLS_CONVR:
      if constexpr (AK == COLS) {
        fx_launch((gemm_f32_wide8_kernel<AK, COLS_CONVR>), grid, dim3(W8T), 0, s, g);
        return FX_OK;
      }
      break;
    case COLS_KT:
      if constexpr (AK == COLS_KT) {
        fx_launch((gemm_f32_wide8_kernel<AK, COLS_KT>), grid, dim3(W8T), 0, s, g);
        return FX_OK;
      }
      break;
    default: break;
  }
  set_error("gemm(wide8): unsupported B operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_wide8(int ak, int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  switch (ak) {
    case ROWS: return launch_wide8_b<ROWS>(bk, grid, s, g);
    case ROWS_CONV: return launch_wide8_b<ROWS_CONV>(bk, grid, s, g);
    case ROWS_CAT: return launch_wide8_b<ROWS_CAT>(bk, grid, s, g);
    case COLS: return launch_wide8_b<COLS>(bk, grid, s, g);
    case COLS_KT: return launch_wide8_b<COLS_KT>(bk, grid, s, g);
    default: break;
  }
  set_error("gemm(wide8): unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_wide(int ak, int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  switch (ak) {
    case ROWS: return launch_wide_b<ROWS>(bk, grid, s, g);
    case ROWS_CONV: return launch_wide_b<ROWS_CONV>(bk, grid, s, g);
    case ROWS_CAT: return launch_wide_b<ROWS_CAT>(bk, grid, s, g);
    case COLS: return launch_wide_b<COLS>(bk, grid, s, g);
    case COLS_KT: return launch_wide_b<COLS_KT>(bk, grid, s, g);
    default: break;
  }
  set_error("gemm(wide): unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

template <int AK>
int launch_b(int bk, dim3 grid, hipStream_t s, const GemmDev& g, bool fast) {
  switch (bk) {
    case ROWS: launch_t<AK, ROWS>(grid, s, g, fast); return FX_OK;
    case COLS: launch_t<AK, COLS>(grid, s, g, fast); return FX_OK;
    case COLS_CONV: launch_t<AK, COLS_CONV>(grid, s, g, fast); return FX_OK;
    case COLS_CONVR:   // FAST only (plan_gemm checks): the ragged frame lookup lives in the FAST loader
      if constexpr (AK == COLS) {
        if (!fast) break;
        fx_launch((gemm_f32_kernel<AK, COLS_CONVR, true>), grid, dim3(NTHREADS), 0, s, g);
        return FX_OK;
      }
      break;
    case COLS_KT:   // FAST only (plan_gemm picks it for vectorisable operands)
      if constexpr (AK == COLS_KT) {
        if (!fast) break;
        fx_launch((gemm_f32_kernel<AK, COLS_KT, true>), grid, dim3(NTHREADS), 0, s, g);
        return FX_OK;
      }
      break;
    case ROWS_GEN:
    case ROWS_CAT: launch_t<AK, ROWS_GEN>(grid, s, g, false); return FX_OK;
    default: break;
  }
  set_error("gemm: unsupported B operand kind");
  return FX_ERR_UNSUPPORTED;
}

// FAST loop: both operands 16-B vector-loadable, K a multiple of the 64-deep stage, no gathers
int launch_tiled(int ak, int bk, dim3 grid, hipStream_t s, const GemmDev& g) {
  const bool fast = g.a_vec && g.b_vec && ((g.K % BK) == 0 || ak == COLS_KT) && ak != ROWS_GEN && bk != ROWS_GEN;
  switch (ak) {
    case ROWS: return launch_b<ROWS>(bk, grid, s, g, fast);
    case ROWS_CONV: return launch_b<ROWS_CONV>(bk, grid, s, g, fast);
    case ROWS_GEN: return launch_b<ROWS_GEN>(bk, grid, s, g, false);
    case ROWS_CAT: return launch_b<ROWS_CAT>(bk, grid, s, g, fast);
    case COLS: return launch_b<COLS>(bk, grid, s, g, fast);
    case COLS_KT: return launch_b<COLS_KT>(bk, grid, s, g, fast);
    default: break;
  }
  set_error("gemm: unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

template <int AK>
int launch_direct_b(int bk, dim3 grid, dim3 block, hipStream_t s, const GemmDev& g) {
  switch (bk) {
    case ROWS: fx_launch((gemm_direct_kernel<AK, ROWS>), grid, block, 0, s, g); return FX_OK;
    case COLS: fx_launch((gemm_direct_kernel<AK, COLS>), grid, block, 0, s, g); return FX_OK;
    default: break;
  }
  set_error("gemm(direct): unsupported B operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_direct(int ak, int bk, dim3 grid, dim3 block, hipStream_t s, const GemmDev& g) {
  switch (ak) {
    case ROWS: return launch_direct_b<ROWS>(bk, grid, block, s, g);
    case ROWS_GEN:
    case ROWS_CAT: return launch_direct_b<ROWS_GEN>(bk, grid, block, s, g);
    case COLS: return launch_direct_b<COLS>(bk, grid, block, s, g);
    default: break;
  }
  set_error("gemm(direct): unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

// Small problems go to the direct kernel: token-level (M or N <= 64: the Nact tokens of one or two
// lockstep videos) or shallow K.  (Few-tile frame-level dW GEMMs with K = T stay tiled: measured
// 25 vs 32 us at 256x257x4096.)  Conv-gather operands always take the tiled kernel.
// FX_GEMM_PATH=tiled|direct overrides the choice (diagnostic).
bool use_direct(const fx_gemm_desc& d, int ak, int bk) {
  const int force = knobs().gemm_path;
  // the direct kernel addresses ROWS / COLS operands with 32-bit byte offsets (dload)
  auto fits = [&](const fx_operand& o, int kind, int R) {
    const double k = (double)d.K + 2 * DMAXW * DCH + 64, ld = (double)o.ld;
    const double bytes = kind == ROWS ? ((double)R * ld + k) * 4 : kind == COLS ? (k * ld + R) * 4 : 0;
    return bytes < 4294967296.0;
  };
  const bool ok = d.K > 0 && (ak == ROWS || ak == ROWS_GEN || ak == ROWS_CAT || ak == COLS) && (bk == ROWS || bk == COLS) &&
                  fits(d.a, ak, d.M) && fits(d.b, bk, d.N);
  if (!ok || force == 1) return false;
  if (force == 2) return true;
  // gathered A rows (ROWS_GEN / ROWS_CAT) load element by element in the direct kernel: only the
  // 32-row case pays off there (64 x 256 x 1024 concat: 54 us direct vs 29 us tiled)
  const int lim = (ak == ROWS_GEN || ak == ROWS_CAT) ? 32 : 64;
  // a shallow K that is not a whole number of 64-deep stages would take the generic tiled kernel
  // (InfoNCE dF: 4096 x 512 x 70, 80 us there; Breakfast's token dW over 4 x 60 = 240 token rows,
  // 512 x 513 x 240: 61 us there); one pass of the direct kernel per tile is ~10x faster
  if (d.M <= lim || d.N <= lim || d.K <= 64 || (d.K <= 512 && d.K % 64 != 0)) return true;
  // few output tiles (the TDU blocks' segment-level products: S ~ 50-250 segment rows per launch): the
  // tiled kernel's fixed cost -- a 64-deep stage pipeline filled per block, one 64 x 64 block per ~4 tiles
  // of 32 x 32 -- is most of its time there; the direct kernel runs every 32 x 32 tile's K chunks on
  // their own waves.  Measured (tools/r06_seg_gemm.py, SWEEP=1): 192 x 512 x 512 7.9 vs 16.0 us (tiled,
  // 12.8 with split 4), 1024 x 256 x 512 7.9 vs 16.1, 1024 x 512 x 512 14.0 vs 16.4, 192 x 512 x 2048
  // 19.5 vs 20.2 (split 4); past ~512 tiles the tiled kernel wins (1536 x 512 x 512: 20.1 vs 16.7)
  const long long t32 = (long long)cdiv(d.M, 32) * cdiv(d.N, 32) * d.batch;
  return (ak == ROWS || ak == COLS) && t32 <= 512 && d.K <= 2048;
}

// 128x64 tiles where the launch still has ~3/4 of a block per CU: FAST operands only.
// FX_GEMM_WIDE=0|1 forces the choice among eligible launches (diagnostic).
// 128x64 tiles with 8 waves (two per SIMD) instead of 4; FX_GEMM_W8=0|1 overrides (diagnostic)
bool wide8() {
  return knobs().gemm_w8;
}

bool use_wide(const GemmDev& g, int ak, int bk, int batch) {
  const int force = knobs().gemm_wide;
  const bool fast = g.a_vec && g.b_vec && ((g.K % BK) == 0 || ak == COLS_KT);
  const bool ok = fast && (ak == ROWS || ak == ROWS_CONV || ak == ROWS_CAT || ak == COLS || ak == COLS_KT) &&
                  (bk == ROWS || bk == COLS || bk == COLS_CONV || bk == COLS_CONVR || bk == COLS_KT);
  if (!ok || force == 0) return false;
  if (force == 1) return true;
  return (long long)cdiv(g.M, WBM) * g.tiles_x * batch * g.split >= 192;
}

// Split-K arrival counters, one pool per (device, stream): zeroed once at allocation and
// re-armed by the last block of every tile, so launches on one stream reuse them safely.
constexpr long long kMaxTileCounters = kArrivalCounters;
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

unsigned* arrival_counters(hipStream_t s) { return tile_counters(s); }


thread_local const float* t_ws_lo = nullptr;
thread_local const float* t_ws_hi = nullptr;

WsBound::WsBound(const float* base, long long floats) : prev_lo(t_ws_lo), prev_hi(t_ws_hi) {
  t_ws_lo = base;
  t_ws_hi = base ? base + std::max(floats, 0LL) : nullptr;
}
WsBound::~WsBound() {
  t_ws_lo = prev_lo;
  t_ws_hi = prev_hi;
}

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

namespace {

struct GemmPlan {
  GemmDev g;
  dim3 grid, block;
  int ak, bk;
  bool direct, wide;
};

// Everything launch_gemm decides before launching: operand kinds, kernel, tiles, split, counters.
// tile_cnt_base: first arrival counter this launch may use (problems of one grouped launch get
// disjoint counter ranges).
int plan_gemm(const fx_gemm_desc& d, hipStream_t s, GemmPlan& P, long long tile_cnt_base = 0) {
  FX_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0 && d.batch >= 1, "gemm: bad sizes");
  FX_REQUIRE(d.a.ptr && d.b.ptr && d.c, "gemm: null operand");
  FX_REQUIRE(!(d.a.conv_taps && d.a.seq_len <= 0 && d.a.nseq <= 0) &&
                 !(d.b.conv_taps && d.b.seq_len <= 0 && d.b.nseq <= 0),
             "gemm: conv operand needs seq_len or seq_off");
  FX_REQUIRE(d.a.nseq <= 0 || !d.a.trans, "gemm: ragged conv offsets on a row-major A or a column-major B operand");
  FX_REQUIRE(d.b.nseq <= 0 || (d.b.trans && d.b.conv_taps && d.a.nseq <= 0),
             "gemm: ragged column-major conv B needs a plain A operand");
  FX_REQUIRE(!(d.a.conv_taps && d.K != d.a.conv_taps * d.a.conv_cin), "gemm: conv A needs K == taps*cin");
  FX_REQUIRE(!(d.b.conv_taps && d.b.trans && d.N != d.b.conv_taps * d.b.conv_cin + (d.b.ones_col ? 1 : 0)),
             "gemm: conv B needs N == taps*cin (+1 with a ones column)");
  FX_REQUIRE(!(d.a.ones_col && !d.a.trans) && !(d.b.ones_col && !d.b.trans), "gemm: ones_col needs trans==1");
  FX_REQUIRE(!(d.b.conv_taps && !d.b.trans), "gemm: row-major conv B operand is not supported");
  GemmDev& g = P.g;
  g = GemmDev{};
  g.M = d.M;
  g.N = d.N;
  g.K = d.K;
  g.a = d.a;
  g.b = d.b;
  {   // ragged conv videos: the offsets travel in the kernel arguments
    const fx_operand& o = d.a;
    if (o.nseq > 0) {
      FX_REQUIRE(o.conv_taps && o.seq_off && o.nseq <= kMaxSeq, "gemm: seq_off needs a conv operand, <= 16 videos");
      const int rows = d.M;
      FX_REQUIRE(o.seq_off[0] == 0 && o.seq_off[o.nseq] == rows, "gemm: seq_off must span the operand's rows");
      for (int v = 0; v <= o.nseq; ++v) {
        FX_REQUIRE(v == 0 || o.seq_off[v] > o.seq_off[v - 1], "gemm: seq_off must increase");
        g.soff[v] = o.seq_off[v];
      }
      g.nsoff = o.nseq;
    }
  }
  {   // ragged column-major conv B (weight gradients of a ragged batch, K = frames): K may pad the last
      // video to whole 64-deep stages; those frames read as zero
    const fx_operand& o = d.b;
    if (o.nseq > 0) {
      FX_REQUIRE(o.seq_off && o.nseq <= kMaxSeq && o.seq_off[0] == 0 && o.seq_off[o.nseq] <= d.K,
                 "gemm: ragged B offsets must start at 0 and end within K, <= 16 videos");
      FX_REQUIRE(operand_vec_ok(d.a) && operand_vec_ok(d.b) && d.K % BK == 0,
                 "gemm: ragged B needs 16-B operands and K a multiple of 64 (pad the frames)");
      for (int v = 0; v <= kMaxSeq; ++v) {
        FX_REQUIRE(v == 0 || v > o.nseq || o.seq_off[v] > o.seq_off[v - 1], "gemm: seq_off must increase");
        g.soff[v] = v <= o.nseq ? o.seq_off[v] : 0x7fffffff;
      }
      g.nsoff = o.nseq;
    }
  }
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
  g.c_last_bs = d.c_last_batch_stride ? d.c_last_batch_stride : d.M;
  g.b_dil_growth = d.b_dil_growth;
  g.a_dil_b1 = d.a_dil_b1;
  g.bias_bs = d.bias_batch_stride;
  FX_REQUIRE(d.a_dil_b1 <= 0 || (d.a.conv_taps && !d.a.trans), "gemm: a_dil_b1 needs a row-major conv A");
  FX_REQUIRE(d.b_dil_growth <= 1 || (d.b.conv_taps && d.b.trans), "gemm: b_dil_growth needs a column-major conv B");
  g.stamps = d.dbg_stamps;
  FX_REQUIRE(d.drop_p >= 0.f && d.drop_p < 1.f, "gemm: dropout p must be in [0, 1)");
  FX_REQUIRE(d.drop_p == 0.f || (!d.c_last_col && !d.c_tap_cin && !d.gate && d.beta == 0.f &&
                                 !(d.relu == 1 && d.resid)),
             "gemm: dropout only on plain outputs (before the residual add)");
  g.drop_thr = d.drop_p > 0.f ? std::max(fx_drop_thresh(d.drop_p), 1u) : 0u;
  g.drop_scale = 1.f / (1.f - d.drop_p);
  g.drop_seed = d.drop_seed;
  g.a_vec = operand_vec_ok(d.a);
  g.b_vec = operand_vec_ok(d.b);
  g.ws = d.workspace;
  int ak = kind_of(d.a, g.a_vec), bk = kind_of(d.b, g.b_vec);
  const bool direct = d.b_dil_growth <= 1 && d.a_dil_b1 <= 0 && use_direct(d, ak, bk);   // (the direct kernel: one dilation)
  // weight gradients over a frame count that is not a whole number of 64-deep stages (ragged batches):
  // the K-tail loaders keep them on the FAST tiled / wide kernels instead of the element-wise generic one
  if (!direct && ak == COLS && bk == COLS && g.a_vec && g.b_vec && d.K % BK != 0 && knobs().gemm_ktail) ak = bk = COLS_KT;
  P.ak = ak;
  P.bk = bk;
  bool wide = false;
  const int cap = (d.split_k > 1 && d.workspace) ? d.split_k : 1;   // workspace holds `cap` slabs
  FX_REQUIRE(!(d.split_k > 1 && !d.workspace), "gemm: split-K needs a workspace");
  dim3 grid, block;
  if (direct) {
    const int nch = cdiv(d.K, DCH);
    const long long t32 = (long long)cdiv(d.M, 32) * cdiv(d.N, 32) * d.batch;
    // one 32-deep k chunk per wave, up to 8 waves per tile (two chunks per wave measured slower: round 3)
    const int cpw = 1;
    const int nw = std::min(DMAXW, std::max(1, nch / cpw));
    int split = 1;
    // split K only for launches of few tiles (the token rows): from 64 tiles up the extra slabs and the
    // last arriver's reduction cost more than they spread (102 x 512 x 512: 7.8 us unsplit, 9.7 in 4)
    if (cap > 1 && t32 < 64) {
      const long long want = std::min<long long>(nch / (cpw * nw), cdiv(2048, t32 * nw));
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
    wide = use_wide(g, ak, bk, d.batch);
    g.tiles_y = cdiv(d.M, wide ? WBM : BM);
    grid = dim3(g.tiles_x, g.tiles_y, d.batch * g.split);
    block = dim3(NTHREADS);
  }
  if (g.split > 1 && t_ws_hi && !(g.ws >= t_ws_lo && g.ws + (long long)g.split * d.M * d.N * d.batch <= t_ws_hi))
    std::fprintf(stderr, "factmx: gemm M %d N %d K %d batch %d split %d (cap %d, %s) needs %lld floats at +%lld of a %lld-float reservation\n",
                 d.M, d.N, d.K, d.batch, g.split, cap, direct ? "direct" : "tiled",
                 (long long)g.split * d.M * d.N * d.batch, (long long)(g.ws - t_ws_lo), (long long)(t_ws_hi - t_ws_lo));
  FX_REQUIRE(g.split <= 1 || !t_ws_hi ||
                 (g.ws >= t_ws_lo && g.ws + (long long)g.split * d.M * d.N * d.batch <= t_ws_hi),
             "gemm: split-K slabs would overrun the entry point's workspace reservation");
  // in-launch reduction only while the last block's serial slab read stays small (<= 32 KB per
  // tile); bigger ones pay less as a separate reduce launch (conv dW split 5: 78 vs 56 us)
  const long long slab_bytes = (long long)g.split * (direct ? 32 * 32 : (wide ? WBM : BM) * BN) * 4;
  if (g.split > 1 && slab_bytes <= 32768 &&
      tile_cnt_base + (long long)g.tiles_x * g.tiles_y * d.batch <= kMaxTileCounters) {
    unsigned* pool = tile_counters(s);
    g.tile_cnt = pool ? pool + tile_cnt_base : nullptr;
  }
  // FX_GEMM_XCDPLANES=0: the per-plane tile mapping for every launch (A/B)
  const bool planes_on = knobs().gemm_xcd_planes;
  const long long nz = (long long)d.batch * g.split;
  g.xcd_planes = planes_on && wide && wide8() && nz >= 8 && nz % 8 == 0;
  // FX_GEMM_ROWPERM=0: keep row tiles in order for dilated-conv A operands too (A/B)
  if (knobs().gemm_row_perm && wide && !g.xcd_planes && d.a.conv_taps > 1 && !d.a.trans && d.a_dil_b1 <= 0) {
    const int sh = d.a.conv_dil / WBM;
    if (sh > 1 && g.tiles_y % sh == 0) g.row_perm = sh;
  }
  // FX_GEMM_GROUPM=0: plain row-major tile runs (A/B).  Grouped order when B does not fit an XCD's L2
  // share (> 2 MB) but one XCD run of A rows does (<= 2 MB), plain operands only
  g.group_m = 0;
  if (knobs().gemm_group_m && !g.xcd_planes && g.row_perm <= 1 && d.a.conv_taps <= 1 && d.b.conv_taps <= 1 &&
      g.tiles_y >= 16 && g.tiles_x >= 8) {
    const int gm = g.tiles_y / 8, tm = wide ? WBM : BM;
    const double b_bytes = 4.0 * d.N * d.K, a_run = 4.0 * gm * tm * d.K;
    if (b_bytes > 2.0 * (1 << 20) && a_run <= 2.0 * (1 << 20)) g.group_m = gm;
  }
  g.persist = 0;
  P.grid = grid;
  P.block = block;
  P.direct = direct;
  P.wide = wide;
  return FX_OK;
}

int launch_reduce(const fx_gemm_desc& d, const GemmPlan& P, hipStream_t s) {
  if (P.g.split > 1 && !P.g.tile_cnt) {
    const long long total = (long long)d.M * d.N;
    const int vec = (total % 4) == 0 && ((uintptr_t)P.g.ws & 15) == 0;
    int blocks = (int)std::min<long long>(cdiv(cdiv(total, 4), 256), 2048);
    fx_launch(splitk_reduce_kernel, dim3(blocks, d.batch), dim3(256), 0, s, P.g, vec);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

}  // namespace

// GEMM arithmetic precision per caller stream (fx_set_stream_precision): a few (stream, precision)
// pairs behind a mutex; streams never set run FX_PREC_F32.  Per stream, so two callers with different
// precisions on different streams (or threads) do not interfere.
std::mutex g_prec_mu;
std::vector<std::pair<hipStream_t, int>> g_prec;
std::atomic<int> g_prec_any{0};   // fast path: no stream has an explicit setting
std::atomic<int> g_prec_default{FX_PREC_F32};   // streams without one (fx_set_default_precision)

int stream_precision(hipStream_t s) {
  if (!g_prec_any.load(std::memory_order_acquire)) return g_prec_default.load(std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(g_prec_mu);
  for (const auto& e : g_prec)
    if (e.first == s) return e.second;
  return g_prec_default.load(std::memory_order_relaxed);
}

bool valid_precision(int prec) {
  return prec == FX_PREC_F32 || prec == FX_PREC_BF16 || prec == FX_PREC_F32S || prec == FX_PREC_F32S2;
}

// FX_PREC_BF16 / FX_PREC_F32S / FX_PREC_F32S2: the 128x64-tile launches with row-major A take the
// bf16-arithmetic kernel / the split-bf16 fp32 kernel; everything else (weight gradients: A column-major;
// direct / small tiles) keeps the f32 MFMA kernels
bool rowmajor_wide(const GemmPlan& P) {
  return P.wide && (P.bk == ROWS || P.bk == COLS) && (P.ak == ROWS || P.ak == ROWS_CONV || P.ak == ROWS_CAT);
}
bool bf16_eligible(const GemmPlan& P, hipStream_t s) {
  return rowmajor_wide(P) && stream_precision(s) == FX_PREC_BF16;
}
// the split kernel's 32-deep stages: a conv stage must stay inside one tap, a concatenation stage in
// one source (the host plan checked 64-alignment for the 64-deep kernels already)
int split_pieces_for(const GemmPlan& P, hipStream_t s) {
  if (!rowmajor_wide(P)) return 0;
  const int prec = stream_precision(s);
  return prec == FX_PREC_F32S ? 3 : prec == FX_PREC_F32S2 ? 2 : 0;
}

template <int AK, int NP>
int launch_split_b(const GemmPlan& P, hipStream_t s) {
  // B row-major: the operands split in registers (wide8 kernel); B column-major: the LDS-image split kernel
  if (P.bk == ROWS)
    fx_launch((gemm_f32_wide8_kernel<AK, ROWS, NP>), P.grid, dim3(W8T), 0, s, P.g);
  else
    fx_launch((gemm_split_wide8_kernel<AK, COLS, NP>), P.grid, dim3(W8T), 0, s, P.g);
  return FX_OK;
}

template <int NP>
int launch_split_np(const GemmPlan& P, hipStream_t s) {
  switch (P.ak) {
    case ROWS: return launch_split_b<ROWS, NP>(P, s);
    case ROWS_CONV: return launch_split_b<ROWS_CONV, NP>(P, s);
    case ROWS_CAT: return launch_split_b<ROWS_CAT, NP>(P, s);
    default: break;
  }
  set_error("gemm(split): unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_split(const GemmPlan& P, int np, hipStream_t s) {
  return np == 3 ? launch_split_np<3>(P, s) : launch_split_np<2>(P, s);
}

template <int AK>
int launch_bf16_b(const GemmPlan& P, hipStream_t s) {
  if (P.bk == ROWS)
    fx_launch((gemm_bf16_wide8_kernel<AK, ROWS>), P.grid, dim3(W8T), 0, s, P.g);
  else
    fx_launch((gemm_bf16_wide8_kernel<AK, COLS>), P.grid, dim3(W8T), 0, s, P.g);
  return FX_OK;
}

int launch_bf16(const GemmPlan& P, hipStream_t s) {
  switch (P.ak) {
    case ROWS: return launch_bf16_b<ROWS>(P, s);
    case ROWS_CONV: return launch_bf16_b<ROWS_CONV>(P, s);
    case ROWS_CAT: return launch_bf16_b<ROWS_CAT>(P, s);
    default: break;
  }
  set_error("gemm(bf16): unsupported A operand kind");
  return FX_ERR_UNSUPPORTED;
}

int launch_gemm(const fx_gemm_desc& d, hipStream_t s) {
  FX_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0 && d.batch >= 1, "gemm: bad sizes");
  if (d.M == 0 || d.N == 0) return FX_OK;
  GemmPlan P;
  FX_TRY(plan_gemm(d, s, P));
  const int np = split_pieces_for(P, s);
  // FX_GEMM_PERSIST=0: one workgroup per tile (A/B).  A persistent grid for the f32 wide8 kernel on
  // single, unsplit products with at least two tiles per CU (the kernel loops over virtual workgroups)
  if (knobs().gemm_persist && !np && !bf16_eligible(P, s) && P.wide && wide8() && P.g.split == 1 && d.batch == 1 &&
      !P.g.xcd_planes) {
    const long long nt = (long long)P.g.tiles_x * P.g.tiles_y;
    constexpr int G = 256;   // (a multiple of 8: a virtual workgroup keeps its physical one's XCD)
    if (nt >= 2 * G) {
      P.g.persist = (int)nt;
      P.grid = dim3(G, 1, 1);
    }
  }
  const GemmDev& g = P.g;
#ifdef FX_GEMM_CENSUS
  // diagnostic build only (tools/r06_gemm_census.sh): one line per GEMM kernel launch, in launch order
  std::fprintf(stderr, "GEMM %p %d %d %d %d %d %d %d %d %d %d %d\n", (void*)s, d.M, d.N, d.K, d.batch, P.ak, P.bk,
               P.g.split, P.direct ? 1 : P.wide ? 2 : 0, P.g.persist, d.a.conv_taps, (int)(P.g.split > 1 && !P.g.tile_cnt));
#endif
  int st = np ? launch_split(P, np, s)
         : bf16_eligible(P, s) ? launch_bf16(P, s)
         : P.direct ? launch_direct(P.ak, P.bk, P.grid, P.block, s, g)
                    : (P.wide ? (wide8() ? launch_wide8(P.ak, P.bk, P.grid, s, g) : launch_wide(P.ak, P.bk, P.grid, s, g))
                              : launch_tiled(P.ak, P.bk, P.grid, s, g));
  if (st != FX_OK) return st;
  FX_CHECK_HIP(hipGetLastError());
  return launch_reduce(d, P, s);
}

// Independent GEMMs (no member reads another's output; disjoint outputs and workspaces) in one
// launch when every member takes the direct kernel; otherwise one launch each, in order.
// FX_GEMM_GROUP=0 disables the grouping (diagnostic A/B).
int launch_gemm_group(const fx_gemm_desc* d, int n, hipStream_t s) {
  const bool on = knobs().gemm_group;
  FX_REQUIRE(n >= 0 && n <= GMAX, "gemm group: 0..4 members");
  int live = 0, nsplit = 0;   // members with M, N > 0; of those, split-K members
  bool all_direct = on;
  GemmPlan P[GMAX];
  long long cnt_base = 0;
  for (int i = 0; i < n && all_direct; ++i) {
    FX_REQUIRE(d[i].M >= 0 && d[i].N >= 0 && d[i].K >= 0 && d[i].batch >= 1, "gemm: bad sizes");
    if (d[i].M == 0 || d[i].N == 0) continue;
    FX_TRY(plan_gemm(d[i], s, P[i], cnt_base));
    if (P[i].g.tile_cnt) cnt_base += (long long)P[i].g.tiles_x * P[i].g.tiles_y * d[i].batch;
    all_direct = all_direct && P[i].direct;
    nsplit += P[i].g.split > 1 ? 1 : 0;
    ++live;
  }
  // split members given the same workspace get consecutive slab ranges in it (checked against the
  // entry point's reservation); split members on different workspaces are not grouped
  bool ws_ok = true;
  if (all_direct && nsplit > 1) {
    const float* base = nullptr;
    long long off = 0;
    for (int i = 0; i < n && ws_ok; ++i) {
      if (d[i].M == 0 || d[i].N == 0 || P[i].g.split <= 1) continue;
      if (!base) base = d[i].workspace;
      ws_ok = d[i].workspace == base && t_ws_hi != nullptr;
      P[i].g.ws = d[i].workspace + off;
      off += (long long)P[i].g.split * d[i].M * d[i].N * d[i].batch;
      ws_ok = ws_ok && P[i].g.ws >= t_ws_lo && P[i].g.ws + (long long)P[i].g.split * d[i].M * d[i].N * d[i].batch <= t_ws_hi;
    }
  }
  if (!all_direct || live < 2 || !ws_ok) {
    for (int i = 0; i < n; ++i) FX_TRY(launch_gemm(d[i], s));
    return FX_OK;
  }
  // one launch per distinct block size: a member planned with fewer waves per tile would otherwise run
  // with idle waves in every block (measured: a K = 32 member beside a K = 4096 one, 2x slower)
  bool done[GMAX] = {};
  for (int i0 = 0; i0 < n; ++i0) {
    if (done[i0] || d[i0].M == 0 || d[i0].N == 0) continue;
    const unsigned nw = P[i0].block.x;
    GemmGroup G{};
    int m = 0;
    G.start[0] = 0;
    for (int i = i0; i < n; ++i) {
      if (done[i] || d[i].M == 0 || d[i].N == 0 || P[i].block.x != nw) continue;
      done[i] = true;
      G.g[m] = P[i].g;
      const int ak = P[i].ak == ROWS_CAT ? ROWS_GEN : P[i].ak;
      G.kinds[m] = ak * 8 + P[i].bk;
      G.start[m + 1] = G.start[m] + (int)(P[i].grid.x * P[i].grid.y * P[i].grid.z);
      ++m;
    }
    for (int i = m + 1; i <= GMAX; ++i) G.start[i] = G.start[m];
    G.n = m;
    if (m == 1) {
#ifdef FX_GEMM_CENSUS
      std::fprintf(stderr, "GEMM %p %d %d %d %d %d %d %d 1 0 0 %d\n", (void*)s, d[i0].M, d[i0].N, d[i0].K, d[i0].batch,
                   P[i0].ak, P[i0].bk, P[i0].g.split, (int)(P[i0].g.split > 1 && !P[i0].g.tile_cnt));
#endif
      FX_TRY(P[i0].direct ? launch_direct(P[i0].ak, P[i0].bk, P[i0].grid, P[i0].block, s, P[i0].g) : FX_ERR_UNSUPPORTED);
    } else {
      fx_launch(gemm_direct_group_kernel, dim3(G.start[m]), dim3(nw), 0, s, G);
    }
    FX_CHECK_HIP(hipGetLastError());
  }
  for (int i = 0; i < n; ++i)
    if (d[i].M != 0 && d[i].N != 0) FX_TRY(launch_reduce(d[i], P[i], s));
  return FX_OK;
}

int launch_colsum_batched(const float* x, long long ld, long long x_bs, int M, int N, int nb, float* out,
                          long long out_bs, int accumulate, float* ws, hipStream_t s) {
  if (N == 0 || nb == 0) return FX_OK;
  if (M == 0) {
    if (!accumulate)
      for (int b = 0; b < nb; ++b) FX_CHECK_HIP(hipMemsetAsync(out + (long long)b * out_bs, 0, sizeof(float) * N, s));
    return FX_OK;
  }
  const int nblk = cdiv(M, CS_ROWS);
  fx_launch(colsum_stage1, dim3(cdiv(N, 64), nblk, nb), dim3(256), 0, s, x, ld, x_bs, M, N, ws);
  fx_launch(colsum_stage2, dim3(cdiv(N, 256), nb), dim3(256), 0, s, ws, nblk, N, out, out_bs, accumulate);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_colsum(const float* x, long long ld, int M, int N, float* out, int accumulate, float* ws,
                  hipStream_t s) {
  return launch_colsum_batched(x, ld, 0, M, N, 1, out, 0, accumulate, ws, s);
}

long long colsum_workspace_floats(int M, int N) { return (long long)cdiv(M, CS_ROWS) * N; }

}  // namespace fx

extern "C" {

int fx_set_stream_precision(void* stream, int prec) {
  FX_REQUIRE(prec == FX_PREC_DEFAULT || fx::valid_precision(prec),
             "gemm precision: FX_PREC_DEFAULT, FX_PREC_F32, FX_PREC_BF16, FX_PREC_F32S or FX_PREC_F32S2");
  std::lock_guard<std::mutex> lk(fx::g_prec_mu);
  const hipStream_t s = (hipStream_t)stream;
  auto& v = fx::g_prec;
  for (auto it = v.begin(); it != v.end(); ++it)
    if (it->first == s) {
      v.erase(it);
      break;
    }
  if (prec != FX_PREC_DEFAULT) v.emplace_back(s, prec);
  fx::g_prec_any.store(v.empty() ? 0 : 1, std::memory_order_release);
  return FX_OK;
}

int fx_get_stream_precision(void* stream) { return fx::stream_precision((hipStream_t)stream); }

int fx_stream_precision_explicit(void* stream) {
  std::lock_guard<std::mutex> lk(fx::g_prec_mu);
  for (const auto& e : fx::g_prec)
    if (e.first == (hipStream_t)stream) return e.second;
  return FX_PREC_DEFAULT;
}

int fx_set_default_precision(int prec) {
  FX_REQUIRE(fx::valid_precision(prec), "default gemm precision: FX_PREC_F32, FX_PREC_BF16, FX_PREC_F32S or FX_PREC_F32S2");
  fx::g_prec_default.store(prec, std::memory_order_relaxed);
  return FX_OK;
}

int fx_get_default_precision(void) { return fx::g_prec_default.load(std::memory_order_relaxed); }

}  // extern "C"
