// Bidirectional GRU over TDU segments (UpdateBlockTDU.seg_update, blocks.py:401,432:
// nn.GRU(H, H/2, 1, bidirectional=True), gate order r, z, n, h0 = 0).
//
// Input projections for all steps and both directions are one MFMA GEMM
// (gi = x . [W_ih; W_ih_rev]^T + b_ih).  The recurrence is sequential in S, so
// each direction runs in ONE 1024-thread workgroup that keeps h in LDS and
// streams W_hh (3Hh x Hh fp32, L2 resident) once per step:
//   fwd:  gh = W_hh h + b_hh          (thread = gate row, W_hh stored [k][row]: coalesced)
//         r = s(gi_r + gh_r), z = s(gi_z + gh_z), n = tanh(gi_n + r*gh_n), h' = (1-z) n + z h
//   bwd:  dh   = dout_t + dh_rec
//         dn_p = dh (1-z)(1-n^2);  dz_p = dh (h-n) z(1-z);  dr_p = dn_p gh_n r(1-r)
//         dgi  = [dr_p, dz_p, dn_p];  dgh = [dr_p, dz_p, dn_p * r]
//         dh_rec = dh z + W_hh^T dgh  (thread = hidden unit k, W_hh stored [row][k]: coalesced)
// Weight/bias/input gradients are GEMMs over the saved per-step tables.
#include <algorithm>

#include "fx_common.h"

namespace fx {
namespace {

// ---------------------------------------------------------------------------------------------
// The recurrence is sequential in S and W_hh (3Hh x Hh fp32 = 786 KB at Hh = 256) is too large to
// re-stream through ONE CU every step (that version spent 11 us / 35 us per fwd / bwd step).  Here
// each direction is spread over NW = 16 workgroups that keep their slice of W_hh in REGISTERS for
// the whole sequence; per step they exchange only the new hidden state (fwd, Hh floats) or the
// gate gradients (bwd, 3Hh floats) through epoch-tagged 8-byte granules (the data is the flag:
// agent-scope relaxed atomic stores/loads, cdna_hip_programming.md Guideline 16 recipe R2),
// double-buffered by step parity so a workgroup one step ahead never overwrites a slot another is
// still reading.  All 2*NW workgroups are co-resident (32 of 256 CUs); every spin is bounded and
// sets a timeout word, so the grid always drains.
constexpr int NW = 16;          // workgroups per direction
constexpr int GT = 256;         // threads per workgroup
constexpr int MAXU = 16;        // hidden units per workgroup (Hh <= 256)
constexpr int KCH = 64;         // fwd: k-chunk per thread (4 chunks cover Hh <= 256)
constexpr int RCH = 48;         // bwd: gate rows per thread (16 chunks cover 3Hh <= 768)
constexpr unsigned SPIN_MAX = 1u << 20;   // default: ~1 s of polling; a lost peer ends the kernel, never hangs it

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned epoch, float v) {
  __hip_atomic_store((gu64*)g, ((unsigned long long)epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// one wave gathers n granules of `epoch` into LDS dst (bounded spin; on timeout flags *tmo)
__device__ __forceinline__ bool gather_granules(unsigned long long* g, int n, unsigned epoch, float* dst,
                                                unsigned* tmo, unsigned spin_max, int lane) {
  for (int base = 0; base < n; base += 64 * 4) {
    unsigned long long x[4];
    bool done[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) done[q] = base + q * 64 + lane >= n;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!done[q]) {
          x[q] = __hip_atomic_load((gu64*)(g + base + q * 64 + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(x[q] >> 32) == epoch) {
            dst[base + q * 64 + lane] = __uint_as_float((unsigned)x[q]);
            done[q] = true;
          } else {
            ok = false;
          }
        }
      }
      if (__all(ok)) break;
      if (spins > spin_max) {
        if (lane == 0) __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
  return true;
}

constexpr int MAXSEQ = 32;      // sequences per launch (more are launched in chunks)

struct GruDirArgs {
  const float* gi;     // (S, 3Hh) for this direction, ld = ldgi
  long long ldgi;
  const float* whh;    // (3Hh, Hh) natural layout [row][k]
  const float* bhh;    // (3Hh)
  float* out;          // (S, ldo) h_t written at column offset
  long long ldo;
  float* hprev;        // (S, Hh) h_{t-1} per step
  float* gates;        // (S, 4Hh): r, z, n, gh_n
  int Hh, reverse;
};

// sequence sq of the launch owns rows [off[sq], off[sq+1]) of every table; its direction d uses the
// granule slots gran + ((sq * 2 + d) * 2 + slot) * G
struct GruArgs {
  GruDirArgs d[2];
  unsigned long long* gran;
  unsigned* tmo;        // the caller's status word (fx_gru_bidir_*: FX_STATUS_GRU_TIMEOUT on a lost peer)
  unsigned spin_max;
  int off[MAXSEQ + 1];
};

__global__ __launch_bounds__(GT) void gru_fwd_kernel(GruArgs args) {
  const int sq = blockIdx.x / (2 * NW), rem = blockIdx.x - sq * 2 * NW;
  const int dir = rem / NW, j = rem - dir * NW;
  const GruDirArgs& a = args.d[dir];
  const int Hh = a.Hh, tid = threadIdx.x, lane = tid & 63;
  const int r0 = args.off[sq], S = args.off[sq + 1] - r0;
  unsigned long long* gran = args.gran + (long long)(sq * 2 + dir) * 2 * Hh;
  const int U = (Hh + NW - 1) / NW, u0 = j * U;
  __shared__ float h[256];
  __shared__ float gh[3 * MAXU];
  __shared__ int dead;
  if (tid == 0) dead = 0;
  // this thread's slice of W_hh: row o of the workgroup's 3U rows, k-chunk c
  const int o = tid >> 2, c = tid & 3;
  const int g = o / U, ui = o - g * U, unit = u0 + ui;
  const bool act = o < 3 * U && unit < Hh;
  const int row = g * Hh + unit;
  float w[KCH];
#pragma unroll
  for (int i = 0; i < KCH; ++i) {
    const int k = c * KCH + i;
    w[i] = (act && k < Hh) ? a.whh[(long long)row * Hh + k] : 0.f;
  }
  const float bias = act ? a.bhh[row] : 0.f;
  for (int k = tid; k < 256; k += GT) h[k] = 0.f;
  // the input projections of step s are loaded during step s-1 (their latency hides behind the
  // exchange instead of opening every step)
  const bool own = tid < U && u0 + tid < Hh;
  const int uo = u0 + (own ? tid : 0);
  float pr = 0.f, pz = 0.f, pn = 0.f;
  if (own && S > 0) {
    const float* gg = a.gi + (long long)(r0 + (a.reverse ? S - 1 : 0)) * a.ldgi;
    pr = gg[uo];
    pz = gg[Hh + uo];
    pn = gg[2 * Hh + uo];
  }
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int t = r0 + (a.reverse ? S - 1 - s : s);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < KCH; ++i) acc = fmaf(w[i], h[c * KCH + i], acc);
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    if (act && c == 0) gh[o] = acc + bias;
    __syncthreads();
    if (own) {
      const int u = uo;
      const float gr = pr, gz = pz, gn = pn;
      if (s + 1 < S) {
        const float* gg = a.gi + (long long)(r0 + (a.reverse ? S - 2 - s : s + 1)) * a.ldgi;
        pr = gg[u];
        pz = gg[Hh + u];
        pn = gg[2 * Hh + u];
      }
      const float r = sigm(gr + gh[tid]);
      const float z = sigm(gz + gh[U + tid]);
      const float n = tanhf(gn + r * gh[2 * U + tid]);
      const float hp = h[u];
      const float hn = (1.f - z) * n + z * hp;
      a.out[(long long)t * a.ldo + u] = hn;
      a.hprev[(long long)t * Hh + u] = hp;
      float* gs = a.gates + (long long)t * 4 * Hh;
      gs[u] = r;
      gs[Hh + u] = z;
      gs[2 * Hh + u] = n;
      gs[3 * Hh + u] = gh[2 * U + tid];
      put_granule(gran + (long long)(s & 1) * Hh + u, (unsigned)(s + 1), hn);
    }
    __syncthreads();   // every wave is done with the old h
    if (s + 1 < S) {   // the 4 waves gather a quarter of h each (one round trip instead of several)
      const int q = (Hh + 4 * 64 - 1) / (4 * 64) * 64, b0 = (tid >> 6) * q;
      if (b0 < Hh &&
          !gather_granules(gran + (long long)(s & 1) * Hh + b0, min(q, Hh - b0), (unsigned)(s + 1), h + b0, args.tmo,
                           args.spin_max, lane))
        dead = 1;
    }
    __syncthreads();
    if (dead) break;
  }
}

struct GruBwdDirArgs {
  const float* dout;   // (S, lddo) gradient of h_t at column offset
  long long lddo;
  const float* whh;    // (3Hh, Hh) natural layout [row][k]
  const float* hprev;  // (S, Hh)
  const float* gates;  // (S, 4Hh)
  float* dgi;          // (S, 3Hh) ld lddgi
  long long lddgi;
  float* dgh;          // (S, 3Hh)
  int Hh, reverse;
};

struct GruBwdArgs {
  GruBwdDirArgs d[2];
  unsigned long long* gran;
  unsigned* tmo;        // the caller's status word (fx_gru_bidir_*: FX_STATUS_GRU_TIMEOUT on a lost peer)
  unsigned spin_max;
  int off[MAXSEQ + 1];
};

__global__ __launch_bounds__(GT) void gru_bwd_kernel(GruBwdArgs args) {
  const int sq = blockIdx.x / (2 * NW), rem = blockIdx.x - sq * 2 * NW;
  const int dir = rem / NW, j = rem - dir * NW;
  const GruBwdDirArgs& a = args.d[dir];
  const int Hh = a.Hh, H3 = 3 * Hh, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r0 = args.off[sq], S = args.off[sq + 1] - r0;
  unsigned long long* gran = args.gran + (long long)(sq * 2 + dir) * 2 * H3;
  const int U = (Hh + NW - 1) / NW, u0 = j * U;
  __shared__ float dg[768];
  __shared__ float dh[MAXU], dhd[MAXU];
  __shared__ float part[4][MAXU];
  __shared__ int dead;
  if (tid == 0) dead = 0;
  // this thread's slice of W_hh^T: unit i of the workgroup, gate rows [c*RCH, c*RCH + RCH)
  const int i = tid & 15, c = tid >> 4;
  const bool act = i < U && u0 + i < Hh;
  float w[RCH];
#pragma unroll
  for (int r = 0; r < RCH; ++r) {
    const int row = c * RCH + r;
    w[r] = (act && row < H3) ? a.whh[(long long)row * Hh + u0 + i] : 0.f;
  }
  if (tid < MAXU) dh[tid] = 0.f;
  // step s's saved gates, h_{t-1} and output gradient are loaded during step s-1
  const bool own = tid < U && u0 + tid < Hh;
  const int uo = u0 + (own ? tid : 0);
  float nr = 0.f, nz = 0.f, nn = 0.f, ng = 0.f, nh = 0.f, nd = 0.f;
  auto fetch = [&](int t) {
    const float* gs = a.gates + (long long)t * 4 * Hh;
    nr = gs[uo];
    nz = gs[Hh + uo];
    nn = gs[2 * Hh + uo];
    ng = gs[3 * Hh + uo];
    nh = a.hprev[(long long)t * Hh + uo];
    nd = a.dout[(long long)t * a.lddo + uo];
  };
  if (own && S > 0) fetch(r0 + (a.reverse ? 0 : S - 1));
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int t = r0 + (a.reverse ? s : S - 1 - s);   // reverse of the forward visiting order
    unsigned long long* slot = gran + (long long)(s & 1) * H3;
    if (own) {
      const int u = uo;
      const float r = nr, z = nz, n = nn, ghn = ng, hp = nh, dcur = nd;
      if (s + 1 < S) fetch(r0 + (a.reverse ? s + 1 : S - 2 - s));
      const float d = dcur + dh[tid];
      const float dnp = d * (1.f - z) * (1.f - n * n);
      const float dzp = d * (hp - n) * z * (1.f - z);
      const float drp = dnp * ghn * r * (1.f - r);
      float* gi = a.dgi + (long long)t * a.lddgi;
      gi[u] = drp;
      gi[Hh + u] = dzp;
      gi[2 * Hh + u] = dnp;
      float* gg = a.dgh + (long long)t * H3;
      gg[u] = drp;
      gg[Hh + u] = dzp;
      gg[2 * Hh + u] = dnp * r;
      put_granule(slot + u, (unsigned)(s + 1), drp);
      put_granule(slot + Hh + u, (unsigned)(s + 1), dzp);
      put_granule(slot + 2 * Hh + u, (unsigned)(s + 1), dnp * r);
      dhd[tid] = d * z;   // direct path; W^T dgh added below
    }
    if (s + 1 == S) break;   // the last step's recurrent gradient feeds nothing
    {   // the 4 waves gather a quarter of the 3Hh gate gradients each
      const int q = (H3 + 4 * 64 - 1) / (4 * 64) * 64, b0 = wv * q;
      if (b0 < H3 && !gather_granules(slot + b0, min(q, H3 - b0), (unsigned)(s + 1), dg + b0, args.tmo, args.spin_max,
                                           lane))
        dead = 1;
    }
    __syncthreads();
    if (dead) break;
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < RCH; ++r) {
      const int row = c * RCH + r;
      acc = fmaf(w[r], row < H3 ? dg[row] : 0.f, acc);
    }
    acc += __shfl_xor(acc, 16, 64);
    acc += __shfl_xor(acc, 32, 64);
    if (lane < 16) part[wv][lane] = acc;
    __syncthreads();
    if (tid < U) dh[tid] = dhd[tid] + (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
    __syncthreads();
  }
}

}  // namespace

// floats of the per-call sync area for nseq sequences: timeout word (padded to 16 B) +
// per sequence 2 dirs x 2 slots x 3Hh granules (8 B each)
long long gru_sync_floats(int Hh, int nseq) { return 4 + (long long)std::max(nseq, 1) * 2 * 2 * 3 * Hh * 2; }

int launch_gru_fwd(const float* gi, long long ldgi, int nseq, const int* seq_off, int Hh, const float* const whh[2],
                   const float* const bhh[2], float* out, long long ldo, float* saved, float* ws, unsigned* status,
                   int spin_max, hipStream_t s) {
  FX_REQUIRE(Hh > 0 && Hh <= NW * MAXU, "gru: hidden size per direction must be <= 256");
  const int Stot = seq_off[nseq];
  if (Stot == 0) return FX_OK;
  unsigned* tmo = reinterpret_cast<unsigned*>(ws);
  unsigned long long* gran = reinterpret_cast<unsigned long long*>(ws + 4);
  FX_CHECK_HIP(hipMemsetAsync(ws, 0, sizeof(float) * gru_sync_floats(Hh, nseq), s));
  for (int c0 = 0; c0 < nseq; c0 += MAXSEQ) {
    const int nc = std::min(MAXSEQ, nseq - c0);
    GruArgs args{};
    args.tmo = status ? status : tmo;
    args.spin_max = spin_max > 0 ? (unsigned)spin_max : SPIN_MAX;
    args.gran = gran + (long long)c0 * 2 * 2 * 3 * Hh;
    for (int q = 0; q <= nc; ++q) args.off[q] = seq_off[c0 + q];
    for (int d = 0; d < 2; ++d) {
      GruDirArgs& a = args.d[d];
      a.gi = gi + d * 3 * Hh;
      a.ldgi = ldgi;
      a.whh = whh[d];
      a.bhh = bhh[d];
      a.out = out + d * Hh;
      a.ldo = ldo;
      a.hprev = saved + (long long)d * Stot * Hh;
      a.gates = saved + 2LL * Stot * Hh + (long long)d * Stot * 4 * Hh;
      a.Hh = Hh;
      a.reverse = d;
    }
    hipLaunchKernelGGL(gru_fwd_kernel, dim3(nc * 2 * NW), dim3(GT), 0, s, args);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

int launch_gru_bwd(const float* dout, long long lddo, int nseq, const int* seq_off, int Hh, const float* const whh[2],
                   const float* saved, float* dgi, long long lddgi, float* dgh, float* sync_ws, unsigned* status,
                   int spin_max, hipStream_t s) {
  FX_REQUIRE(Hh > 0 && Hh <= NW * MAXU, "gru: hidden size per direction must be <= 256");
  const int Stot = seq_off[nseq];
  if (Stot == 0) return FX_OK;
  const int H3 = 3 * Hh;
  unsigned* tmo = reinterpret_cast<unsigned*>(sync_ws);
  unsigned long long* gran = reinterpret_cast<unsigned long long*>(sync_ws + 4);
  FX_CHECK_HIP(hipMemsetAsync(sync_ws, 0, sizeof(float) * gru_sync_floats(Hh, nseq), s));
  for (int c0 = 0; c0 < nseq; c0 += MAXSEQ) {
    const int nc = std::min(MAXSEQ, nseq - c0);
    GruBwdArgs args{};
    args.tmo = status ? status : tmo;
    args.spin_max = spin_max > 0 ? (unsigned)spin_max : SPIN_MAX;
    args.gran = gran + (long long)c0 * 2 * 2 * H3;
    for (int q = 0; q <= nc; ++q) args.off[q] = seq_off[c0 + q];
    for (int d = 0; d < 2; ++d) {
      GruBwdDirArgs& a = args.d[d];
      a.dout = dout + d * Hh;
      a.lddo = lddo;
      a.whh = whh[d];
      a.hprev = saved + (long long)d * Stot * Hh;
      a.gates = saved + 2LL * Stot * Hh + (long long)d * Stot * 4 * Hh;
      a.dgi = dgi + d * H3;
      a.lddgi = lddgi;
      a.dgh = dgh + (long long)d * Stot * H3;
      a.Hh = Hh;
      a.reverse = d;
    }
    hipLaunchKernelGGL(gru_bwd_kernel, dim3(nc * 2 * NW), dim3(GT), 0, s, args);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

}  // namespace fx
