// One MS-TCN dilated residual layer step as ONE kernel: a dilated-conv GEMM (K = 3F) whose
// row-local epilogue feeds a 1x1 GEMM (K = F) on the same rows, the intermediate tile kept in LDS
// (DilatedResidualLayer.forward, basic.py:154-171, and the matching input-gradient chain).
//
//   forward  (layer i):  z    = relu(conv_d(h_i) + b_dil)             -> out1 (saved for backward)
//                        h_i+1 = h_i + dropout(z . W_pw^T + b_pw)      -> out2
//   backward (layers i, i-1 of the dX chain):
//                        dH_i   = gU_i + conv_d^T(dZ_i)               -> out1
//                        dZ_i-1 = (dH_i . W_pw,i-1) * (z_i-1 > 0)     -> out2
//
// A workgroup owns FR = 32 rows and all F = 256 channels (8 waves x 32 columns, one 32x32 f32
// MFMA accumulator each): the full-width row tile is what makes the second GEMM row-local, and
// 8192 rows give 256 workgroups = one per CU.  Both GEMMs stream their weights (conv 256 x 768,
// 1x1 256 x 256; L2-resident, shared by every CU) through a three-slot LDS ring fed by two
// register sets (a stage's global loads are issued four stages, and stored two stages, ahead of
// its use; one stage index runs over both phases); the conv operand is read straight from the
// row-major activations, each 32-deep k stage lying inside one tap (zero outside the video).
// (Loading each wave's weight rows straight into MFMA registers instead -- no LDS for B -- was
// 1.5x slower: 32 rows per lane-group are 32 cache lines per load instruction.)  The 1x1's first
// weight stages are loaded during the conv's last stages, so the two phases run back to back.
// Measured against the two tuned GEMM launches it replaces (conv 128x64 tiles + 1x1), it is about
// even (58 vs 56 us per layer at 8192 rows: every CU streams the whole weight matrix through its
// LDS, 1.5x the LDS write traffic per flop of a 128x64 tile), so the stack uses it only when
// FX_MSTCN_FUSED=1 (diagnostic / A-B); the two-GEMM path stays the default.
#include <cstdlib>

#include "fx_common.h"
#include "ops.h"

namespace fx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int FR = 32;           // rows per workgroup
constexpr int FN = 256;          // channels: N of both GEMMs, K of the second
constexpr int FBK = 32;          // k per stage
constexpr int FT = 512;          // threads: 8 waves x 32 columns
constexpr int AS = FBK + 4;      // LDS row stride of the stage images ([row][k], k contiguous)
constexpr int VS = FN + 4;       // LDS row stride of the phase-1 tile
constexpr int A_IMG = FR * AS;
constexpr int B_IMG = FN * AS;
constexpr int SLOT = A_IMG + B_IMG;
constexpr int NSL = 3;           // LDS ring depth
constexpr int LDS_FLOATS = NSL * SLOT + FR * VS;

struct FrlArgs {
  const float* x;      // phase-1 conv operand rows (M, FN), ld ldx
  long long ldx;
  int dil, dir, T, M;
  const float* w1;     // (FN, 3 FN) row-major: [n][tap * FN + c]
  const float* bias1;  // nullable
  int relu1;
  const float* resid1; // nullable (M, FN) ld ldr1
  long long ldr1;
  float* out1;
  long long ldo1;
  const float* w2;     // (FN, FN) row-major: [n][k]
  const float* bias2;  // nullable
  const float* resid2; // nullable
  long long ldr2;
  const float* gate2;  // nullable: out2 = 0 where gate2 <= 0
  long long ldg2;
  float* out2;
  long long ldo2;
  unsigned drop_thr;   // dropout on (acc2 + bias2) before resid2; 0 = off
  float drop_scale;
  unsigned long long drop_seed;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// One stage's global loads: A (threads 256..511 repeat 0..255: no branch, so the compiler counts
// the outstanding loads exactly), B = 4 float4 per thread.  The zero select of A rows outside
// their video is applied at the LDS store (applying it at the load would wait for the load).
struct Prefetch {
  float4 a, b[4];
  bool a_ok;
};

__device__ __forceinline__ void load_a(const FrlArgs& g, int m0, int st, int tid, Prefetch& p) {
  const int k0 = st * FBK, tap = k0 / FN, c0 = k0 - tap * FN;
  const int ar = (tid & 255) >> 3, k4 = (tid & 7) * 4;
  const int r = m0 + ar;
  const int sh = (tap - 1) * g.dil * g.dir;
  const int t = r % g.T + sh;
  const bool ok = r < g.M && t >= 0 && t < g.T;
  const long long src = ok ? (long long)(r + sh) : 0;   // clamped, unconditional load
  p.a = ld4(g.x + src * g.ldx + c0 + k4);
  p.a_ok = ok;
}

__device__ __forceinline__ void load_b(const float* w, int ldw, int st, int tid, Prefetch& p) {
  const int k0 = st * FBK, k4 = (tid & 7) * 4, n = tid >> 3;
#pragma unroll
  for (int j = 0; j < 4; ++j) p.b[j] = ld4(w + (long long)(n + 64 * j) * ldw + k0 + k4);
}

__device__ __forceinline__ void store_stage(float* slot, int tid, const Prefetch& p, bool with_a) {
  const int k4 = (tid & 7) * 4, n = tid >> 3;
  if (with_a)   // duplicate lanes write equal data
    st4(slot + ((tid & 255) >> 3) * AS + k4, p.a_ok ? p.a : make_float4(0.f, 0.f, 0.f, 0.f));
  float* b = slot + A_IMG;
#pragma unroll
  for (int j = 0; j < 4; ++j) st4(b + (n + 64 * j) * AS + k4, p.b[j]);
}

// 16 MFMAs of one 32-deep stage: A rows from `a` (row stride as), B = this wave's 32 columns; the
// lane pairs A[li][16 lh + s] with B[n][16 lh + s]
__device__ __forceinline__ void mma_stage(const float* a, int as, const float* b, int w, int li, int lh,
                                          f32x16& acc) {
  float4 fa[4], fb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    fa[q] = ld4(a + li * as + lh * 16 + q * 4);
    fb[q] = ld4(b + (w * 32 + li) * AS + lh * 16 + q * 4);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[q].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[q].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[q].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[q].w, acc, 0, 0, 0);
  }
}

__global__ __launch_bounds__(FT) void frl_kernel(FrlArgs g) {
  extern __shared__ float lds[];
  float* V = lds + NSL * SLOT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int m0 = blockIdx.x * FR;
  constexpr int n1 = 3 * FN / FBK, n2 = FN / FBK, nall = n1 + n2;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  // one stage index over both phases: [0, n1) the conv (A + B), [n1, nall) the 1x1 (B; A = the
  // LDS tile V); every loop has constant bounds and is fully unrolled: no stage branches remain
  auto load = [&](int st, Prefetch& p) {
    if (st < n1) {
      load_a(g, m0, st, tid, p);
      load_b(g.w1, 3 * FN, st, tid, p);
    } else if (st < nall) {
      load_b(g.w2, FN, st - n1, tid, p);
    }
  };
  // two register sets: stage st + 2 (loaded two stages ago) is stored into slot (st + 2) % 3 while
  // stage st computes from slot st % 3, then stage st + 4 is loaded into the freed set
  Prefetch pr[2];
  load(0, pr[0]);
  load(1, pr[1]);
  store_stage(lds, tid, pr[0], true);
  store_stage(lds + SLOT, tid, pr[1], 1 < n1);
  load(2, pr[0]);
  load(3, pr[1]);
  __syncthreads();
  // (sched_barrier pins the order: left to itself the scheduler hoists a set's select / LDS stores
  // up to its loads and waits on loads issued a moment earlier)
  auto step = [&](int st, f32x16& ac, const float* a, int as) {
    const float* cur = lds + (st % NSL) * SLOT;
    mma_stage(a ? a : cur, a ? as : AS, cur + A_IMG, w, li, lh, ac);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 2 < nall) store_stage(lds + ((st + 2) % NSL) * SLOT, tid, pr[st & 1], st + 2 < n1);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 4 < nall) load(st + 4, pr[st & 1]);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
#pragma unroll
  for (int st = 0; st < n1; ++st) step(st, acc, nullptr, 0);
  // ---------------- phase-1 epilogue: out1 and the LDS tile V
  {
    const int col = w * 32 + li;
    const float bv = g.bias1 ? g.bias1[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int gr = m0 + row;
      float v = acc[r] + bv;
      if (g.relu1) v = fmaxf(v, 0.f);
      if (g.resid1 && gr < g.M) v += g.resid1[(long long)gr * g.ldr1 + col];
      if (gr < g.M) g.out1[(long long)gr * g.ldo1 + col] = v;
      V[row * VS + col] = v;
      acc[r] = 0.f;
    }
  }
  __syncthreads();
  // ---------------- phase 2: 1x1 GEMM from the LDS tile, K = FN
#pragma unroll
  for (int j = 0; j < n2; ++j) step(n1 + j, acc, V + j * FBK, VS);
  // ---------------- phase-2 epilogue
  const int col = w * 32 + li;
  const float bv = g.bias2 ? g.bias2[col] : 0.f;
  float res[16], gat[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int gr = min(m0 + (r & 3) + 8 * (r >> 2) + 4 * lh, g.M - 1);
    res[r] = g.resid2 ? g.resid2[(long long)gr * g.ldr2 + col] : 0.f;
    gat[r] = g.gate2 ? g.gate2[(long long)gr * g.ldg2 + col] : 1.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int gr = m0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    float v = acc[r] + bv;
    if (g.drop_thr)
      v = fx_drop_bits(g.drop_seed, (unsigned long long)gr * FN + col) >= g.drop_thr ? v * g.drop_scale : 0.f;
    v += res[r];
    if (!(gat[r] > 0.f)) v = 0.f;
    if (gr < g.M) g.out2[(long long)gr * g.ldo2 + col] = v;
  }
}

}  // namespace

bool frl_supported(int F, const void* x, long long ldx, long long ld_other) {
  return F == FN && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ld_other % 4 == 0;
}

int launch_frl(const float* x, long long ldx, int M, int T, int dil, int dir, const float* w1, const float* bias1,
               int relu1, const float* resid1, long long ldr1, float* out1, long long ldo1, const float* w2,
               const float* bias2, const float* resid2, long long ldr2, const float* gate2, long long ldg2, float* out2,
               long long ldo2, float drop_p, unsigned long long drop_seed, hipStream_t s) {
  FX_REQUIRE(M > 0 && T > 0 && dil > 0 && (dir == 1 || dir == -1), "frl: bad shape");
  FX_REQUIRE(frl_supported(FN, x, ldx, ldo1) && ((uintptr_t)w1 & 15) == 0 && ((uintptr_t)w2 & 15) == 0,
             "frl: needs F = 256 and 16-byte aligned rows");
  FX_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "frl: dropout must be in [0, 1)");
  static const bool attr = [] {
    return hipFuncSetAttribute((const void*)frl_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS_FLOATS * (int)sizeof(float)) == hipSuccess;
  }();
  FX_REQUIRE(attr, "frl: cannot raise the LDS limit");
  FrlArgs a{};
  a.x = x;
  a.ldx = ldx;
  a.dil = dil;
  a.dir = dir;
  a.T = T;
  a.M = M;
  a.w1 = w1;
  a.bias1 = bias1;
  a.relu1 = relu1;
  a.resid1 = resid1;
  a.ldr1 = ldr1;
  a.out1 = out1;
  a.ldo1 = ldo1;
  a.w2 = w2;
  a.bias2 = bias2;
  a.resid2 = resid2;
  a.ldr2 = ldr2;
  a.gate2 = gate2;
  a.ldg2 = ldg2;
  a.out2 = out2;
  a.ldo2 = ldo2;
  a.drop_thr = drop_p > 0.f ? std::max(fx_drop_thresh(drop_p), 1u) : 0u;
  a.drop_scale = 1.f / (1.f - drop_p);
  a.drop_seed = drop_seed;
  hipLaunchKernelGGL(frl_kernel, dim3(cdiv(M, FR)), dim3(FT), LDS_FLOATS * sizeof(float), s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
