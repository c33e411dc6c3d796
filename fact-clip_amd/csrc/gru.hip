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
constexpr int GT = 256;         // threads per workgroup (the backward's; the forward adds a store wave)
constexpr int GTF = GT + 64;    // forward: 4 compute waves + 1 wave that writes the per-step tables
constexpr int MAXU = 16;        // hidden units per workgroup (Hh <= 256)
constexpr int KCH = 64;         // fwd: k-chunk per thread (4 chunks cover Hh <= 256)
constexpr unsigned SPIN_MAX = 1u << 20;   // default: ~1 s of polling; a lost peer ends the kernel, never hangs it

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// tanh through one exp (the recurrence's critical path; tanhf's range reduction is several times
// longer): tanh|x| = (1 - e) / (1 + e), e = exp(-2|x|) in (0, 1]; absolute error a few ulp of 1
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) / (1.f + e), x);
}

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned epoch, float v) {
  __hip_atomic_store((gu64*)g, ((unsigned long long)epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// one wave gathers n granules of `epoch` into LDS dst (bounded spin; on timeout flags *tmo)
__device__ __forceinline__ bool gather_granules(unsigned long long* g, int n, unsigned epoch, float* dst,
                                                unsigned* tmo, unsigned spin_max, int lane, bool poll2) {
  if (poll2 && n <= 64) {
    // one granule per lane, two polls in flight, each re-issued right after its check (epochs only move
    // forward while this wave still needs the slot).  Per recurrent step (tools/r04_gru_bench.py, S = 3400,
    // 2 sequences): fwd 1.88 -> 1.70-1.80 us, bwd 2.49 -> 2.20-2.36 us; four polls in flight were slower
    // (the extra L2 / MALL traffic), delaying the second poll by 256-1024 cycles gained nothing
    const bool mine = lane < n;
    gu64* p = (gu64*)(g + (mine ? lane : 0));
    unsigned long long a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long b = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spins = 0;; spins += 2) {
      if (__all(!mine || (unsigned)(a >> 32) == epoch)) {
        if (mine) dst[lane] = __uint_as_float((unsigned)a);
        return true;
      }
      a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all(!mine || (unsigned)(b >> 32) == epoch)) {
        if (mine) dst[lane] = __uint_as_float((unsigned)b);
        return true;
      }
      b = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (spins > spin_max) {
        if (lane == 0) __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
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
  float* out;          // (S, ldo) h_t written at column offset (relu(h_t) with relu_out)
  long long ldo;
  int relu_out;
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
  int poll2;            // two granule polls in flight (FX_GRU_POLL2, default on)
  int store_wave;       // 1: a fifth wave writes the per-step tables (FX_GRU_STORE_WAVE)
  int off[MAXSEQ + 1];
};

__global__ __launch_bounds__(GTF) void gru_fwd_kernel(GruArgs args) {
  // workgroup (sequence * 2 + direction) * NW + j
  const int lb = (int)blockIdx.x;
  const int sq = lb / (2 * NW), rem = lb - sq * 2 * NW;
  const int dir = rem / NW, j = rem - dir * NW;
  const GruDirArgs& a = args.d[dir];
  const int Hh = a.Hh, tid = threadIdx.x, lane = tid & 63;
  const int r0 = args.off[sq], S = args.off[sq + 1] - r0;
  unsigned long long* gran = args.gran + (long long)(sq * 2 + dir) * 2 * Hh;
  const int U = (Hh + NW - 1) / NW, u0 = j * U;
  // Wave wv owns k-chunk wv of the recurrent product: it gathers units [64 wv, 64 wv + 64) of the new
  // state (the other workgroups' granules, and this one's) and multiplies them into its lanes' rows
  // (lane o = row o of the workgroup's 3U gate rows) without waiting for the other waves; ONE barrier
  // per step then joins the four partial sums for the gate threads.  h and the partials are double-
  // buffered by step parity (a wave may run one step ahead of the gate threads, never two: reaching
  // step s + 2 takes step s + 1's barrier).
  __shared__ float h[2][256];
  __shared__ float part[2][4][64];
  // the step's results (h_t, h_t-1, r, z, n, gh_n of the U units) staged for the store wave (wave 4), which
  // writes them to the output / saved tables one step later: vector stores count in the same in-order
  // counter as the granule polls, so the polling waves issue no table stores of their own (the backward,
  // with two barriers per step, measured no gain from the same change and keeps its gate-thread stores)
  __shared__ float stage[2][6][MAXU];
  // lost peer: 1 + the step whose gather gave up.  A step number, not a flag, because with one barrier
  // per step a fast wave may already be in step s + 1's gather while a slow one still reads the word
  // after barrier s: a failure of step s + 1 must not make the slow wave leave at step s (the waves
  // would then run different numbers of barriers)
  __shared__ int dead;
  if (tid == 0) dead = 0;
  const int wv = tid >> 6;
  const int o = lane;
  const int g = o / U, ui = o - g * U, unit = u0 + ui;
  const bool act = o < 3 * U && unit < Hh;
  const int row = g * Hh + unit;
  float w[KCH];
#pragma unroll
  for (int i = 0; i < KCH; ++i) {
    const int k = wv * KCH + i;
    w[i] = (act && k < Hh) ? a.whh[(long long)row * Hh + k] : 0.f;
  }
  for (int k = tid; k < 512; k += blockDim.x) (&h[0][0])[k] = 0.f;
  const bool storer = wv == 4;   // (launched only with args.store_wave)
  auto flush = [&](int s_) {   // store wave: step s_'s staged results
    const int u = lane;
    if (u < U && u0 + u < Hh) {
      const int t_ = r0 + (a.reverse ? S - 1 - s_ : s_);
      const float* st_ = &stage[s_ & 1][0][0];
      const int uu = u0 + u;
      a.out[(long long)t_ * a.ldo + uu] = a.relu_out ? fmaxf(st_[0 * MAXU + u], 0.f) : st_[0 * MAXU + u];
      a.hprev[(long long)t_ * Hh + uu] = st_[1 * MAXU + u];
      float* gs = a.gates + (long long)t_ * 4 * Hh;
      gs[uu] = st_[2 * MAXU + u];
      gs[Hh + uu] = st_[3 * MAXU + u];
      gs[2 * Hh + uu] = st_[4 * MAXU + u];
      gs[3 * Hh + uu] = st_[5 * MAXU + u];
    }
  };
  // the gate threads (wave 0, lanes < U): their three b_hh entries, and the input projections of step s
  // loaded during step s-1 (their latency hides behind the exchange instead of opening every step)
  // (store_wave 2: the gate threads are wave 4's lanes < U -- the polling waves then issue no stores at
  // all, not even the granule's; store_wave 1: wave 0's, their results staged for wave 4)
  const int gl = args.store_wave == 2 ? (wv == 4 ? lane : GTF) : tid;   // gate-thread index
  const bool own = gl < U && u0 + gl < Hh;
  const int uo = u0 + (own ? gl : 0);
  const float br = own ? a.bhh[uo] : 0.f, bz = own ? a.bhh[Hh + uo] : 0.f, bn = own ? a.bhh[2 * Hh + uo] : 0.f;
  float pr = 0.f, pz = 0.f, pn = 0.f;
  if (own && S > 0) {
    const float* gg = a.gi + (long long)(r0 + (a.reverse ? S - 1 : 0)) * a.ldgi;
    pr = gg[uo];
    pz = gg[Hh + uo];
    pn = gg[2 * Hh + uo];
  }
  const int kc0 = wv * KCH, kcn = max(0, min(KCH, Hh - kc0));   // this wave's chunk of the state
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int t = r0 + (a.reverse ? S - 1 - s : s);
    float* hc = h[s & 1];
    if (s > 0 && kcn > 0 && !storer) {   // the state after step s-1: granules of epoch s in slot (s-1) & 1
      if (!gather_granules(gran + (long long)((s - 1) & 1) * Hh + kc0, kcn, (unsigned)s, hc + kc0, args.tmo,
                           args.spin_max, lane, args.poll2 != 0))
        dead = s + 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS writes land before its reads
    }
    if (!storer) {
      // four independent FMA chains over the wave's 64-deep chunk (broadcast LDS reads)
      float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
      const float4* hv = reinterpret_cast<const float4*>(hc + kc0);
#pragma unroll
      for (int i = 0; i < KCH / 4; ++i) {
        const float4 x = hv[i];
        c0 = fmaf(w[4 * i], x.x, c0);
        c1 = fmaf(w[4 * i + 1], x.y, c1);
        c2 = fmaf(w[4 * i + 2], x.z, c2);
        c3 = fmaf(w[4 * i + 3], x.w, c3);
      }
      part[s & 1][wv][o] = (c0 + c1) + (c2 + c3);
    }
    __syncthreads();
    {
      const int ds = dead;
      if (ds != 0 && ds <= s + 1) break;
    }
    if (storer && s > 0 && args.store_wave == 1) flush(s - 1);
    if (own) {
      const int u = uo;
      const float gr = pr, gz = pz, gn = pn;
      if (s + 1 < S) {
        const float* gg = a.gi + (long long)(r0 + (a.reverse ? S - 2 - s : s + 1)) * a.ldgi;
        pr = gg[u];
        pz = gg[Hh + u];
        pn = gg[2 * Hh + u];
      }
      const float (*pp)[64] = part[s & 1];
      const float ghr = (pp[0][gl] + pp[1][gl]) + (pp[2][gl] + pp[3][gl]) + br;
      const float ghz = (pp[0][U + gl] + pp[1][U + gl]) + (pp[2][U + gl] + pp[3][U + gl]) + bz;
      const float ghn = (pp[0][2 * U + gl] + pp[1][2 * U + gl]) + (pp[2][2 * U + gl] + pp[3][2 * U + gl]) + bn;
      const float r = sigm(gr + ghr);
      const float z = sigm(gz + ghz);
      const float n = tanh_fast(gn + r * ghn);
      const float hp = hc[u];
      const float hn = (1.f - z) * n + z * hp;
      if (s + 1 < S) put_granule(gran + (long long)(s & 1) * Hh + u, (unsigned)(s + 1), hn);
      if (args.store_wave == 1) {
        float* st_ = &stage[s & 1][0][0];
        st_[0 * MAXU + tid] = hn;
        st_[1 * MAXU + tid] = hp;
        st_[2 * MAXU + tid] = r;
        st_[3 * MAXU + tid] = z;
        st_[4 * MAXU + tid] = n;
        st_[5 * MAXU + tid] = ghn;
      } else {
        a.out[(long long)t * a.ldo + u] = a.relu_out ? fmaxf(hn, 0.f) : hn;
        a.hprev[(long long)t * Hh + u] = hp;
        float* gs = a.gates + (long long)t * 4 * Hh;
        gs[u] = r;
        gs[Hh + u] = z;
        gs[2 * Hh + u] = n;
        gs[3 * Hh + u] = ghn;
      }
    }
  }
  // the last step's results (every wave leaves the loop together; none after a lost peer)
  __syncthreads();
  if (storer && S > 0 && !dead && args.store_wave == 1) flush(S - 1);
}

struct GruBwdDirArgs {
  const float* dout;   // (S, lddo) gradient of h_t at column offset (of relu(h_t) with relu_y)
  long long lddo;
  const float* relu_y; // nullable: the forward's relu(h_t) output (ld ldy), the ReLU's backward gate
  long long ldy;
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
  int poll2;
  int off[MAXSEQ + 1];
};

// Backward recurrence, row-partitioned like the forward: workgroup j keeps W_hh's rows of its own U
// units (3U rows x Hh, thread k = column k) and turns its units' gate gradients dgh (3U values) into a
// partial dh_rec over ALL Hh units, p_j[k] = sum_{its rows r} W[r][k] dgh[r]; each unit's owner then
// sums the NW partials in source order (deterministic).  Per step a workgroup sends U granules to
// every workgroup and gathers NW x U = Hh of its own -- one granule per lane, the forward's exchange --
// instead of gathering all 3Hh gate gradients (3 per lane).  Granule block of destination d, source j:
// slot + (d * NW + j) * U.
__global__ __launch_bounds__(GT) void gru_bwd_kernel(GruBwdArgs args) {
  const int lb = (int)blockIdx.x;
  const int sq = lb / (2 * NW), rem = lb - sq * 2 * NW;
  const int dir = rem / NW, j = rem - dir * NW;
  const GruBwdDirArgs& a = args.d[dir];
  const int Hh = a.Hh, H3 = 3 * Hh, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r0 = args.off[sq], S = args.off[sq + 1] - r0;
  const int U = (Hh + NW - 1) / NW, u0 = j * U, NG = NW * U;   // NG granules per destination block
  unsigned long long* gran = args.gran + (long long)(sq * 2 + dir) * 2 * NW * NG;
  __shared__ float dgo[3 * MAXU];       // this workgroup's gate gradients of the step (r, z, n*r rows)
  __shared__ float red[NW * MAXU];      // gathered partials: red[src * U + ui]
  __shared__ float dh[MAXU], dhd[MAXU];
  __shared__ int dead;
  if (tid == 0) dead = 0;
  // thread k: column k of the workgroup's 3U rows (row g * Hh + u0 + ui at index g * U + ui)
  const int k = tid;
  const bool kact = k < Hh;
  float w[3 * MAXU];
#pragma unroll
  for (int q = 0; q < 3 * MAXU; ++q) {
    const int g = q / MAXU, ui = q - g * MAXU;
    w[q] = (kact && ui < U && u0 + ui < Hh) ? a.whh[(long long)(g * Hh + u0 + ui) * Hh + k] : 0.f;
  }
  // every k < NW * U puts (zero past Hh), so each workgroup's block is complete whatever Hh % U
  const bool kput = k < NG;
  const int kd = kput ? k / U : 0, kl = kput ? k - kd * U : 0;   // owner workgroup of unit k, its index there
  if (tid < MAXU) dh[tid] = 0.f;
  // step s's saved gates, h_{t-1} and output gradient are loaded during step s-1
  // gate threads: wave 0's lanes < U (a fifth wave holding them, as the forward's tables, measured even:
  // 2.25 vs 2.26 us per recurrent step, round 5)
  const int gl = tid;
  const bool own = gl < U && u0 + gl < Hh;
  const int uo = u0 + (own ? gl : 0);
  float nr = 0.f, nz = 0.f, nn = 0.f, ng = 0.f, nh = 0.f, nd = 0.f;
  auto fetch = [&](int t) {
    const float* gs = a.gates + (long long)t * 4 * Hh;
    nr = gs[uo];
    nz = gs[Hh + uo];
    nn = gs[2 * Hh + uo];
    ng = gs[3 * Hh + uo];
    nh = a.hprev[(long long)t * Hh + uo];
    nd = a.dout[(long long)t * a.lddo + uo];
    if (a.relu_y && !(a.relu_y[(long long)t * a.ldy + uo] > 0.f)) nd = 0.f;
  };
  if (own && S > 0) fetch(r0 + (a.reverse ? 0 : S - 1));
  if (tid < 3 * MAXU) dgo[tid] = 0.f;
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    const int t = r0 + (a.reverse ? s : S - 1 - s);   // reverse of the forward visiting order
    unsigned long long* slot = gran + (long long)(s & 1) * NW * NG;
    if (own) {
      const int u = uo;
      const float r = nr, z = nz, n = nn, ghn = ng, hp = nh, dcur = nd;
      if (s + 1 < S) fetch(r0 + (a.reverse ? s + 1 : S - 2 - s));
      const float d = dcur + dh[gl];
      const float dnp = d * (1.f - z) * (1.f - n * n);
      const float dzp = d * (hp - n) * z * (1.f - z);
      const float drp = dnp * ghn * r * (1.f - r);
      dgo[gl] = drp;
      dgo[U + gl] = dzp;
      dgo[2 * U + gl] = dnp * r;
      float* gi = a.dgi + (long long)t * a.lddgi;
      gi[u] = drp;
      gi[Hh + u] = dzp;
      gi[2 * Hh + u] = dnp;
      float* gg = a.dgh + (long long)t * H3;
      gg[u] = drp;
      gg[Hh + u] = dzp;
      gg[2 * Hh + u] = dnp * r;
      dhd[gl] = d * z;   // direct path; the NW partials of W^T dgh are added below
    }
    if (s + 1 == S) break;   // the last step's recurrent gradient feeds nothing
    __syncthreads();         // dgo of this step visible to every column thread
    if (kput) {
      // p_j[k] over the 3U rows (four independent chains; rows past the real units have zero weights)
      float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
      for (int q = 0; q < 3 * MAXU; q += 4) {
        const int g0 = q / MAXU, i0 = q - g0 * MAXU;   // dgo index g * U + ui
        c0 = fmaf(w[q], dgo[g0 * U + min(i0, U - 1)], c0);
        c1 = fmaf(w[q + 1], dgo[g0 * U + min(i0 + 1, U - 1)], c1);
        c2 = fmaf(w[q + 2], dgo[g0 * U + min(i0 + 2, U - 1)], c2);
        c3 = fmaf(w[q + 3], dgo[g0 * U + min(i0 + 3, U - 1)], c3);
      }
      put_granule(slot + (long long)(kd * NW + j) * U + kl, (unsigned)(s + 1), (c0 + c1) + (c2 + c3));
    }
    {   // this workgroup's destination block: NW sources x U units, one granule per lane
      const int b0 = wv * 64;
      if (b0 < NG && !gather_granules(slot + (long long)j * NG + b0, min(64, NG - b0), (unsigned)(s + 1), red + b0,
                                      args.tmo, args.spin_max, lane, args.poll2 != 0))
        dead = 1;
    }
    __syncthreads();
    if (dead) break;
    if (own) {   // sources in order (deterministic); dh[tid] / dhd[tid] are this thread's own
      float acc = 0.f;
      for (int src = 0; src < NW; ++src) acc += red[src * U + gl];
      dh[gl] = dhd[gl] + acc;
    }
  }
}

}  // namespace

// floats of the per-call sync area for nseq sequences: timeout word (padded to 16 B) +
// per sequence 2 dirs x 2 slots x max(3Hh, NW * NW * U) granules (8 B each: the forward uses Hh of them,
// the backward NW x NW x U)
// workgroups of a launch over nc sequences: 2 nc groups of NW (placing a group on one XCD measured no gain,
// round 5: its granules are agent-scope stores, which a same-XCD reader sees at the cross-XCD rate)
static int gru_grid(int nc) { return 2 * nc * NW; }

long long gru_sync_floats(int Hh, int nseq) {
  const long long U = (Hh + NW - 1) / NW;
  const long long per = std::max<long long>(3LL * Hh, (long long)NW * NW * U);   // granules per slot
  return 4 + (long long)std::max(nseq, 1) * 2 * 2 * per * 2;
}

int launch_gru_fwd(const float* gi, long long ldgi, int nseq, const int* seq_off, int Hh, const float* const whh[2],
                   const float* const bhh[2], float* out, long long ldo, int relu_out, float* saved, float* ws,
                   unsigned* status, int spin_max, hipStream_t s) {
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
    args.store_wave = knobs().gru_store_wave;
    args.poll2 = knobs().gru_poll2;
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
      a.relu_out = relu_out;
      a.hprev = saved + (long long)d * Stot * Hh;
      a.gates = saved + 2LL * Stot * Hh + (long long)d * Stot * 4 * Hh;
      a.Hh = Hh;
      a.reverse = d;
    }
    fx_launch(gru_fwd_kernel, dim3(gru_grid(nc)), dim3(args.store_wave ? GTF : GT), 0, s, args);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

int launch_gru_bwd(const float* dout, long long lddo, const float* relu_y, long long ldy, int nseq, const int* seq_off,
                   int Hh, const float* const whh[2], const float* saved, float* dgi, long long lddgi, float* dgh,
                   float* sync_ws, unsigned* status, int spin_max, hipStream_t s) {
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
    args.poll2 = knobs().gru_poll2;
    args.gran = gran + (long long)c0 * 2 * 2 * NW * NW * ((Hh + NW - 1) / NW);
    for (int q = 0; q <= nc; ++q) args.off[q] = seq_off[c0 + q];
    for (int d = 0; d < 2; ++d) {
      GruBwdDirArgs& a = args.d[d];
      a.dout = dout + d * Hh;
      a.lddo = lddo;
      a.relu_y = relu_y ? relu_y + d * Hh : nullptr;
      a.ldy = ldy;
      a.whh = whh[d];
      a.hprev = saved + (long long)d * Stot * Hh;
      a.gates = saved + 2LL * Stot * Hh + (long long)d * Stot * 4 * Hh;
      a.dgi = dgi + d * H3;
      a.lddgi = lddgi;
      a.dgh = dgh + (long long)d * Stot * H3;
      a.Hh = Hh;
      a.reverse = d;
    }
    fx_launch(gru_bwd_kernel, dim3(gru_grid(nc)), dim3(GT), 0, s, args);
    FX_CHECK_HIP(hipGetLastError());
  }
  return FX_OK;
}

}  // namespace fx
