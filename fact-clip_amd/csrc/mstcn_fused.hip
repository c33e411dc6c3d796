// One MS-TCN dilated residual layer step as ONE kernel: a dilated-conv GEMM (K = 3F) whose
// row-local epilogue feeds a 1x1 GEMM (K = F) on the same rows, the intermediate tile kept in LDS
// (DilatedResidualLayer.forward, basic.py:154-171, and the matching input-gradient chain).
//
//   forward  (layer i):  z    = relu(conv_d(h_i) + b_dil)             -> out1 (saved for backward)
//                        h_i+1 = h_i + dropout(z . W_pw^T + b_pw)      -> out2
//   backward (layers i, i-1 of the dX chain):
//                        dH_i   = gU_i + conv_d^T(dZ_i)               -> out1
//                        dB_i-1 = dropout_i-1(dH_i)                   -> out3 (training dropout only)
//                        dZ_i-1 = (dB_i-1 . W_pw,i-1) * (z_i-1 > 0)   -> out2
// (with dropout the 1x1 branch of layer i-1 saw mask m: its gradient is dH_i masked the same way --
// the phase-1 tile is masked on its way into LDS, the unmasked dH_i goes to out1 for the residual)
//
// A workgroup owns FR = 32 rows and all F = 256 channels (8 waves x 32 columns, one 32x32 f32 MFMA
// accumulator each): the full-width row tile is what makes the second GEMM row-local, and 8192 rows
// give 256 workgroups = one per CU.
//
// Operand paths.  The activation rows of a stage (32 rows x 32 k) are shared by the 8 waves: they go
// through a 3-slot LDS ring (4.6 KB a slot).  The weights are NOT shared inside a workgroup -- wave w
// multiplies only columns 32 w .. 32 w + 31 -- so each wave loads its own weight fragments straight
// into registers, three stages ahead, from a copy of the weight matrix packed once per call in MFMA
// fragment order (launch_pack_frag): the 16 k values a lane needs for one stage sit in 4 float4 that
// 64 consecutive lanes read as one contiguous 1 KB per load instruction.  (The first version of this
// kernel staged the whole weight matrix through every CU's LDS: 1.5x the LDS write traffic per FLOP of
// the 128 x 64 GEMM tile, and about even with the two GEMM launches it replaces; loading the natural
// [n][k] rows directly was slower still, 32 rows = 32 cache lines per load instruction.)
#include <cstdlib>
#include <map>
#include <mutex>

#include "fx_common.h"
#include "ops.h"

namespace fx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int FR = 32;           // rows per workgroup
constexpr int FN = 256;          // channels: N of both GEMMs, K of the second
constexpr int FBK = 32;          // k per stage
constexpr int FT = 512;          // threads: 8 waves x 32 columns
constexpr int AS = FBK + 4;      // LDS row stride of the activation stage images ([row][k], k contiguous)
constexpr int VS = FN + 4;       // LDS row stride of the phase-1 tile
constexpr int A_IMG = FR * AS;
constexpr int NSL = 3;           // activation ring depth
// weight fragments are loaded PD = 3 stages ahead of their use into NB = PD + 1 register sets (kernel
// template parameter; 5 measured no faster)
constexpr int LDS_FLOATS = NSL * A_IMG + FR * VS;
constexpr int LDS_FLOATS_PAIR = 2 * NSL * A_IMG + FR * VS;
constexpr int kMaxSeqF = 16;     // ragged videos per launch

struct FrlArgs {
  const float* x;      // phase-1 conv operand rows (M, FN), ld ldx
  long long ldx;
  int dil, dir, T, M;
  int xcd_runs;        // 1: consecutive row tiles share an XCD (and its L2), see frl_tile
  int row_perm;        // > 1: the conv taps shift by row_perm whole row tiles (dilation / FR)
  int nsoff;           // > 0: ragged videos, video v owns rows [soff[v], soff[v+1])
  int soff[kMaxSeqF + 1];
  const float* w1p;    // packed (launch_pack_frag) conv weights: [n][tap * FN + c], K = 3 FN
  const float* bias1;  // nullable
  int relu1;
  const float* resid1; // nullable (M, FN) ld ldr1
  long long ldr1;
  float* out1;
  long long ldo1;
  const float* w2p;    // packed 1x1 weights: [n][k], K = FN
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
  unsigned vdrop_thr;  // dropout on the phase-1 tile as phase 2 reads it (out1 keeps it unmasked); 0 = off
  float vdrop_scale;
  unsigned long long vdrop_seed;
  float* out3;         // nullable: the masked phase-1 tile (vdrop only)
  long long ldo3;
};

// Diagnostic builds only (-DFRL_STAMPS, tools/frl_stamps.py): s_memrealtime stamps of thread 0 of every
// workgroup at 8 points of the last launch (fx_debug_frl_stamps); never in the shipped library
#ifdef FRL_STAMPS
__device__ unsigned long long g_frl_st[1024 * 8];
#define FRL_ST(k)                                                                                                  \
  do {                                                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_frl_st[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FRL_ST(k) \
  do {            \
  } while (0)
#endif

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// packed weight fragment of stage st, wave w for this lane: 4 float4 (k = 16 lh + 4 q .. + 3)
__device__ __forceinline__ void load_b(const float* wp, int st, int w, int lane, float4* b) {
  const float* base = wp + ((long long)(st * 8 + w) * 4) * 256 + lane * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) b[q] = ld4(base + q * 256);
}

// A fragments of one 32-deep stage from LDS rows `a` (row stride as): lane (li, lh) takes row li, k 16 lh ..
__device__ __forceinline__ void lds_frag(const float* a, int as, int li, int lh, float4* fa) {
#pragma unroll
  for (int q = 0; q < 4; ++q) fa[q] = ld4(a + li * as + lh * 16 + q * 4);
}

// the 16 MFMAs of one stage from fragments already in registers
__device__ __forceinline__ void mma_frag(const float4* fa, const float4* fb, f32x16& acc) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[q].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[q].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[q].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[q].w, acc, 0, 0, 0);
  }
}

// 16 MFMAs of one 32-deep stage: A rows from `a` (row stride as), B = this wave's fragments; the
// lane pairs A[li][16 lh + s] with B[n][16 lh + s]
__device__ __forceinline__ void mma_stage(const float* a, int as, const float4* fb, int li, int lh, f32x16& acc) {
  float4 fa[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) fa[q] = ld4(a + li * as + lh * 16 + q * 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].x, fb[q].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].y, fb[q].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].z, fb[q].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q].w, fb[q].w, acc, 0, 0, 0);
  }
}

// Row tile of this workgroup.  Workgroups go to the 8 XCDs round robin by dispatch id, so in plain
// order a tile's neighbours -- whose rows are its conv halo (dilation < FR) or its shifted taps -- sit
// on other XCDs and every tile fetches its halo / taps through its own L2 again.  xcd_runs: XCD x gets
// a contiguous run of tiles; row_perm p > 1 (taps shift by p whole tiles): the runs walk the tiles
// 0, p, 2p, ..., 1, 1 + p, ... so a tile and its shifted taps share the run (the GEMM's block_tile
// does the same for the dilated-conv GEMMs).
__device__ __forceinline__ int frl_tile(const FrlArgs& g) {
  const int id = blockIdx.x;
  if (!g.xcd_runs) return id;
  const int nt = gridDim.x, q = nt / 8, rr = nt % 8, x8 = id % 8, i8 = id / 8;
  int t = (x8 < rr ? x8 * (q + 1) : rr * (q + 1) + (x8 - rr) * q) + i8;
  if (g.row_perm > 1) {
    const int per = nt / g.row_perm;
    t = (t % per) * g.row_perm + t / per;
  }
  return t;
}

// PAIR: the activation ring holds stage PAIRS -- threads 0..255 stage the even stage of a pair, 256..511
// the odd one, and the workgroup synchronises once per 64 k instead of once per 32 k; the 1x1 phase reads
// the static LDS tile V without any barrier.  !PAIR: one barrier per 32-deep stage in both phases.
template <bool PAIR, int PD>
__global__ __launch_bounds__(FT) void frl_kernel(FrlArgs g) {
  constexpr int NB = PD + 1;
  extern __shared__ float lds[];
  float* V = lds + (PAIR ? 2 : 1) * NSL * A_IMG;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, lh = lane >> 5;
  FRL_ST(0);
  const int m0 = frl_tile(g) * FR;
  constexpr int n1 = 3 * FN / FBK, n2 = FN / FBK, nall = n1 + n2;
  static_assert(n1 % 2 == 0, "stage pairs");
  // this thread's activation row (!PAIR: threads 256..511 repeat 0..255: no branch, the compiler counts
  // the outstanding loads exactly; duplicate lanes store equal data) and its position inside its video
  const int ar = (tid & 255) >> 3, k4 = (tid & 7) * 4, half = PAIR ? tid >> 8 : 0;
  const int r = m0 + ar;
  int rpos, rlen;
  if (g.nsoff > 0) {
    int start = 0, end = 0x7fffffff;
#pragma unroll
    for (int i = 1; i <= kMaxSeqF; ++i) {
      if (i <= g.nsoff) {
        const int o = g.soff[i];
        if (o <= r) start = o;
        else end = min(end, o);
      }
    }
    rpos = r - start;
    rlen = end - start;
  } else {
    rpos = r % g.T;
    rlen = g.T;
  }
  const bool rok = r < g.M;
  const float* xrow = g.x + (long long)min(r, g.M - 1) * g.ldx + k4;
  auto load_a = [&](int st, float4& v, bool& ok) {
    const int k0 = st * FBK, tap = k0 / FN, c0 = k0 - tap * FN;
    const int sh = (tap - 1) * g.dil * g.dir;
    const int t = rpos + sh;
    ok = rok && t >= 0 && t < rlen;
    v = ld4(xrow + (ok ? (long long)sh * g.ldx : 0ll) + c0);   // clamped, unconditional load
  };
  auto store_a = [&](float* slot, const float4& v, bool ok) {
    st4(slot + ar * AS + k4, ok ? v : make_float4(0.f, 0.f, 0.f, 0.f));
  };
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float4 pb[NB][4];                    // weight fragments, register set st % NB
  float4 pa[2];                        // activation rows of stage st + 2 (set st & 1)
  bool pok[2];
  auto load_w = [&](int st) {
    if (st < n1) load_b(g.w1p, st, w, lane, pb[st % NB]);
    else if (st < nall) load_b(g.w2p, st - n1, w, lane, pb[st % NB]);
  };
  // stage st: multiply slot st % 3 (phase 2: the LDS tile V); store the activation rows of stage st + 2
  // (loaded two stages ago) into slot (st + 2) % 3; load stage st + 4's rows and stage st + PD's weights
  auto step = [&](int st, const float* a, int as) {
    const float* cur = lds + (st % NSL) * A_IMG;
    mma_stage(a ? a : cur, a ? as : AS, pb[st % NB], li, lh, acc);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 2 < n1) store_a(lds + ((st + 2) % NSL) * A_IMG, pa[st & 1], pok[st & 1]);
    if (st + 4 < n1) load_a(st + 4, pa[st & 1], pok[st & 1]);
    load_w(st + PD);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
  // epilogue operands (phase-1 residual; phase-2 residual and gate), loaded into registers before the
  // MFMAs they follow so their latency hides behind them
  const int ecol = w * 32 + li;
  float r1[16], res[16], gat[16];
  auto erow = [&](int q) { return min(m0 + (q & 3) + 8 * (q >> 2) + 4 * lh, g.M - 1); };
  auto load_r1 = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) r1[q] = g.resid1 ? g.resid1[(long long)erow(q) * g.ldr1 + ecol] : 0.f;
  };
#pragma unroll
  for (int st = 0; st < PD; ++st) load_w(st);
  if constexpr (PAIR) {
    // pair p of stages (2p, 2p + 1) in ring slot p % NSL; this thread's stage 2p + half
    constexpr int np = n1 / 2;
    auto slot = [&](int p) { return lds + (p % NSL) * 2 * A_IMG; };
    load_a(half, pa[0], pok[0]);
    load_a(2 + half, pa[1], pok[1]);
    store_a(slot(0) + half * A_IMG, pa[0], pok[0]);
    store_a(slot(1) + half * A_IMG, pa[1], pok[1]);
    load_a(4 + half, pa[0], pok[0]);
    FRL_ST(1);
    __syncthreads();
    FRL_ST(2);
    // A fragments of pair p are read from LDS one pair ahead (during pair p - 1's MFMAs): slot p % NSL
    // was written before the barrier that ended pair p - 2, so the read needs no extra barrier, and
    // after each barrier the MFMAs start on fragments already in registers
    float4 fa[2][2][4];   // [pair parity][stage of the pair][q]
    lds_frag(slot(0), AS, li, lh, fa[0][0]);
    lds_frag(slot(0) + A_IMG, AS, li, lh, fa[0][1]);
#pragma unroll
    for (int p = 0; p < np; ++p) {
      if (p + 1 < np) {
        lds_frag(slot(p + 1), AS, li, lh, fa[(p + 1) & 1][0]);
        lds_frag(slot(p + 1) + A_IMG, AS, li, lh, fa[(p + 1) & 1][1]);
      } else {
        load_r1();
      }
      __builtin_amdgcn_sched_barrier(0);
      mma_frag(fa[p & 1][0], pb[(2 * p) % NB], acc);
      __builtin_amdgcn_sched_barrier(0);
      load_w(2 * p + PD);
      __builtin_amdgcn_sched_barrier(0);
      mma_frag(fa[p & 1][1], pb[(2 * p + 1) % NB], acc);
      __builtin_amdgcn_sched_barrier(0);
      // pair p + 2 (loaded during the previous pair) into the slot pair p - 1 used (its fragments were
      // read during pair p - 2); fetch pair p + 3
      if (p + 2 < np) store_a(slot(p + 2) + half * A_IMG, pa[0], pok[0]);
      if (p + 3 < np) load_a(2 * (p + 3) + half, pa[0], pok[0]);
      load_w(2 * p + 1 + PD);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
    }
  } else {
    load_a(0, pa[0], pok[0]);
    load_a(1, pa[1], pok[1]);
    store_a(lds, pa[0], pok[0]);
    store_a(lds + A_IMG, pa[1], pok[1]);
    load_a(2, pa[0], pok[0]);
    load_a(3, pa[1], pok[1]);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < n1; ++st) step(st, nullptr, 0);
  }
  if (!PAIR) load_r1();
  FRL_ST(3);
  // ---------------- phase-1 epilogue: out1 and the LDS tile V
  {
    const int col = ecol;
    const float bv = g.bias1 ? g.bias1[col] : 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = (q & 3) + 8 * (q >> 2) + 4 * lh;
      const int gr = m0 + row;
      float v = acc[q] + bv;
      if (g.relu1) v = fmaxf(v, 0.f);
      v += r1[q];
      if (gr < g.M) g.out1[(long long)gr * g.ldo1 + col] = v;
      if (g.vdrop_thr) {
        v = fx_drop_bits(g.vdrop_seed, (unsigned long long)gr * FN + col) >= g.vdrop_thr ? v * g.vdrop_scale : 0.f;
        if (g.out3 && gr < g.M) g.out3[(long long)gr * g.ldo3 + col] = v;
      }
      V[row * VS + col] = v;
      acc[q] = 0.f;
    }
  }
  auto load_res = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      res[q] = g.resid2 ? g.resid2[(long long)erow(q) * g.ldr2 + ecol] : 0.f;
      gat[q] = g.gate2 ? g.gate2[(long long)erow(q) * g.ldg2 + ecol] : 1.f;
    }
  };
  load_res();
  FRL_ST(4);
  __syncthreads();
  FRL_ST(5);
  // ---------------- phase 2: 1x1 GEMM from the LDS tile, K = FN
  if constexpr (PAIR) {
    float4 fv[2][4];      // V fragments one stage ahead
    lds_frag(V, VS, li, lh, fv[0]);
#pragma unroll
    for (int j = 0; j < n2; ++j) {
      if (j + 1 < n2) lds_frag(V + (j + 1) * FBK, VS, li, lh, fv[(j + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      mma_frag(fv[j & 1], pb[(n1 + j) % NB], acc);
      __builtin_amdgcn_sched_barrier(0);
      load_w(n1 + j + PD);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < n2; ++j) step(n1 + j, V + j * FBK, VS);
  }
  FRL_ST(6);
  // ---------------- phase-2 epilogue
  const int col = ecol;
  const float bv = g.bias2 ? g.bias2[col] : 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int gr = m0 + (q & 3) + 8 * (q >> 2) + 4 * lh;
    float v = acc[q] + bv;
    if (g.drop_thr)
      v = fx_drop_bits(g.drop_seed, (unsigned long long)gr * FN + col) >= g.drop_thr ? v * g.drop_scale : 0.f;
    v += res[q];
    if (!(gat[q] > 0.f)) v = 0.f;
    if (gr < g.M) g.out2[(long long)gr * g.ldo2 + col] = v;
  }
  FRL_ST(7);
}

// Weight matrices [FN][K] (row-major, leading dim ld) -> MFMA fragment order for frl_kernel:
// dst[((st * 8 + w) * 4 + q) * 64 + lane] = float4(src[n = 32 w + lane % 32][32 st + 16 (lane / 32) + 4 q ..])
// Up to FRAG_JOBS matrices per launch, each with its own K and leading dim (a layer stack's conv and 1x1
// weights, forward and backward orientations, in one launch); blocks past a matrix's K stages exit.
struct PackFragArgs {
  const float* src[FRAG_JOBS];
  float* dst[FRAG_JOBS];
  int ld[FRAG_JOBS];
  int K[FRAG_JOBS];
};

__global__ __launch_bounds__(256) void pack_frag_kernel(PackFragArgs a) {
  const int st = blockIdx.x, w = blockIdx.y, m = blockIdx.z;
  if (st * FBK >= a.K[m]) return;
  const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = w * 32 + (lane & 31), k = st * FBK + 16 * (lane >> 5) + 4 * q;
  const float4 v = ld4(a.src[m] + (long long)n * a.ld[m] + k);
  st4(a.dst[m] + ((long long)((st * 8 + w) * 4 + q) * 64 + lane) * 4, v);
}

}  // namespace

#ifdef FRL_STAMPS
extern "C" int fx_debug_frl_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_frl_st), sizeof(g_frl_st)) == hipSuccess ? 0 : -1;
}
#endif

bool frl_fills_device(long long rows) {
  static std::mutex mu;
  static std::map<int, int> cus;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  int n = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cus.find(dev);
    if (it == cus.end()) {
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 256;
      cus[dev] = n;
    } else {
      n = it->second;
    }
  }
  return (rows + FR - 1) / FR >= (long long)n * knobs().frl_min_fill / 100;
}

bool frl_supported(int F, const void* x, long long ldx, long long ld_other) {
  return F == FN && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ld_other % 4 == 0;
}

long long frl_packed_floats(int K) { return (long long)FN * K; }

int launch_pack_frag(const FragJob* jobs, int n, hipStream_t s) {
  FX_REQUIRE(n >= 1 && n <= FRAG_JOBS, "pack_frag: 1..48 matrices per launch");
  PackFragArgs a{};
  int kmax = 0;
  for (int i = 0; i < n; ++i) {
    FX_REQUIRE(jobs[i].K % FBK == 0 && jobs[i].ld % 4 == 0 && jobs[i].ld >= jobs[i].K, "pack_frag: K % 32 == 0");
    a.src[i] = jobs[i].src;
    a.dst[i] = jobs[i].dst;
    a.ld[i] = jobs[i].ld;
    a.K[i] = jobs[i].K;
    kmax = std::max(kmax, jobs[i].K);
  }
  fx_launch(pack_frag_kernel, dim3(kmax / FBK, FN / 32, n), dim3(256), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_frl(const float* x, long long ldx, int M, int T, int dil, int dir, const int* seq_off, int nseq,
               const float* w1p, const float* bias1, int relu1, const float* resid1, long long ldr1, float* out1,
               long long ldo1, const float* w2p, const float* bias2, const float* resid2, long long ldr2,
               const float* gate2, long long ldg2, float* out2, long long ldo2, float drop_p,
               unsigned long long drop_seed, hipStream_t s, float vdrop_p, unsigned long long vdrop_seed, float* out3,
               long long ldo3) {
  FX_REQUIRE(M > 0 && dil > 0 && (dir == 1 || dir == -1), "frl: bad shape");
  FX_REQUIRE(seq_off ? (nseq >= 1 && nseq <= kMaxSeqF && seq_off[0] == 0 && seq_off[nseq] == M) : T > 0,
             "frl: uniform videos of T rows, or ragged offsets spanning [0, M) (<= 16 videos)");
  FX_REQUIRE(frl_supported(FN, x, ldx, ldo1) && ((uintptr_t)w1p & 15) == 0 && ((uintptr_t)w2p & 15) == 0,
             "frl: needs F = 256 and 16-byte aligned rows");
  FX_REQUIRE(drop_p >= 0.f && drop_p < 1.f && vdrop_p >= 0.f && vdrop_p < 1.f, "frl: dropout must be in [0, 1)");
  FX_REQUIRE(!out3 || (vdrop_p > 0.f && ldo3 % 4 == 0), "frl: out3 holds the masked tile of a dropout layer");
  static const bool attr = [] {
    return hipFuncSetAttribute((const void*)frl_kernel<false, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS_FLOATS * (int)sizeof(float)) == hipSuccess &&
           hipFuncSetAttribute((const void*)frl_kernel<true, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS_FLOATS_PAIR * (int)sizeof(float)) == hipSuccess;
  }();
  FX_REQUIRE(attr, "frl: cannot raise the LDS limit");
  FrlArgs a{};
  a.x = x;
  a.ldx = ldx;
  a.dil = dil;
  a.dir = dir;
  a.T = T > 0 ? T : 1;
  a.M = M;
  const int nt = cdiv(M, FR), sh = dil / FR;
  a.xcd_runs = knobs().frl_xcd >= 1 && nt >= 16;
  a.row_perm = (knobs().frl_xcd >= 2 && dil % FR == 0 && sh > 1 && nt % sh == 0) ? sh : 1;
  a.nsoff = seq_off ? nseq : 0;
  if (seq_off)
    for (int v = 0; v <= nseq; ++v) a.soff[v] = seq_off[v];
  a.w1p = w1p;
  a.bias1 = bias1;
  a.relu1 = relu1;
  a.resid1 = resid1;
  a.ldr1 = ldr1;
  a.out1 = out1;
  a.ldo1 = ldo1;
  a.w2p = w2p;
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
  a.vdrop_thr = vdrop_p > 0.f ? std::max(fx_drop_thresh(vdrop_p), 1u) : 0u;
  a.vdrop_scale = 1.f / (1.f - vdrop_p);
  a.vdrop_seed = vdrop_seed;
  a.out3 = out3;
  a.ldo3 = ldo3;
  if (!knobs().frl_pair)
    fx_launch((frl_kernel<false, 3>), dim3(nt), dim3(FT), LDS_FLOATS * sizeof(float), s, a);
  else   // (weight prefetch 5 stages ahead instead of 3 measured no faster, round 6: 15.07 / 14.59 vs 14.85 / 14.53 ms)
    fx_launch((frl_kernel<true, 3>), dim3(nt), dim3(FT), LDS_FLOATS_PAIR * sizeof(float), s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
