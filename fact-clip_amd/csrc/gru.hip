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
#include "fx_common.h"

namespace fx {
namespace {

constexpr int GRU_THREADS = 1024;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

struct GruDirArgs {
  const float* gi;     // (S, 3Hh) for this direction, ld = ldgi
  long long ldgi;
  const float* whT;    // (Hh, 3Hh): W_hh transposed, [k][row]
  const float* bhh;    // (3Hh)
  float* out;          // (S, ldo) h_t written at column offset
  long long ldo;
  float* hprev;        // (S, Hh) h_{t-1} per step
  float* gates;        // (S, 4Hh): r, z, n, gh_n
  int S, Hh, reverse;
};

struct GruArgs {
  GruDirArgs d[2];
};

__global__ __launch_bounds__(GRU_THREADS) void gru_fwd_kernel(GruArgs args) {
  const GruDirArgs a = args.d[blockIdx.x];
  extern __shared__ float sm[];
  float* h = sm;                 // Hh
  float* gh = sm + a.Hh;         // 3Hh
  const int tid = threadIdx.x, H3 = 3 * a.Hh;
  for (int j = tid; j < a.Hh; j += GRU_THREADS) h[j] = 0.f;
  __syncthreads();
  for (int s = 0; s < a.S; ++s) {
    const int t = a.reverse ? a.S - 1 - s : s;
    for (int row = tid; row < H3; row += GRU_THREADS) {
      float acc = a.bhh[row];
      const float* w = a.whT + row;
#pragma unroll 8
      for (int k = 0; k < a.Hh; ++k) acc = fmaf(w[(long long)k * H3], h[k], acc);
      gh[row] = acc;
    }
    __syncthreads();
    for (int j = tid; j < a.Hh; j += GRU_THREADS) {
      const float* g = a.gi + (long long)t * a.ldgi;
      const float r = sigm(g[j] + gh[j]);
      const float z = sigm(g[a.Hh + j] + gh[a.Hh + j]);
      const float n = tanhf(g[2 * a.Hh + j] + r * gh[2 * a.Hh + j]);
      const float hp = h[j];
      const float hn = (1.f - z) * n + z * hp;
      a.out[(long long)t * a.ldo + j] = hn;
      a.hprev[(long long)t * a.Hh + j] = hp;
      float* gs = a.gates + (long long)t * 4 * a.Hh;
      gs[j] = r;
      gs[a.Hh + j] = z;
      gs[2 * a.Hh + j] = n;
      gs[3 * a.Hh + j] = gh[2 * a.Hh + j];
      h[j] = hn;
    }
    __syncthreads();
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
  int S, Hh, reverse;
};

struct GruBwdArgs {
  GruBwdDirArgs d[2];
};

__global__ __launch_bounds__(GRU_THREADS) void gru_bwd_kernel(GruBwdArgs args) {
  const GruBwdDirArgs a = args.d[blockIdx.x];
  extern __shared__ float sm[];
  const int Hh = a.Hh, H3 = 3 * Hh;
  float* dh = sm;              // Hh: recurrent gradient into h_{t}
  float* g3 = sm + Hh;         // 3Hh: dgh of the current step
  float* part = g3 + H3;       // 4 x Hh partial sums of W^T dgh
  const int tid = threadIdx.x;
  for (int j = tid; j < Hh; j += GRU_THREADS) dh[j] = 0.f;
  __syncthreads();
  for (int s = 0; s < a.S; ++s) {
    const int t = a.reverse ? s : a.S - 1 - s;   // reverse of the forward visiting order
    const float* gs = a.gates + (long long)t * 4 * Hh;
    for (int j = tid; j < Hh; j += GRU_THREADS) {
      const float r = gs[j], z = gs[Hh + j], n = gs[2 * Hh + j], ghn = gs[3 * Hh + j];
      const float hp = a.hprev[(long long)t * Hh + j];
      const float d = a.dout[(long long)t * a.lddo + j] + dh[j];
      const float dnp = d * (1.f - z) * (1.f - n * n);
      const float dzp = d * (hp - n) * z * (1.f - z);
      const float drp = dnp * ghn * r * (1.f - r);
      float* gi = a.dgi + (long long)t * a.lddgi;
      gi[j] = drp;
      gi[Hh + j] = dzp;
      gi[2 * Hh + j] = dnp;
      float* gg = a.dgh + (long long)t * H3;
      gg[j] = drp;
      gg[Hh + j] = dzp;
      gg[2 * Hh + j] = dnp * r;
      g3[j] = drp;
      g3[Hh + j] = dzp;
      g3[2 * Hh + j] = dnp * r;
      dh[j] = d * z;   // direct path; W^T dgh added below
    }
    __syncthreads();
    // dh_rec[k] += sum_row W[row][k] * g3[row]; rows split over 4 thread groups
    {
      const int q = tid / Hh, k = tid - q * Hh;   // Hh <= 256 -> 4 groups of Hh threads
      if (q < 4 && k < Hh) {
        const int r0 = q * ((H3 + 3) / 4), r1 = min(H3, r0 + (H3 + 3) / 4);
        float acc = 0.f;
        for (int row = r0; row < r1; ++row) acc = fmaf(a.whh[(long long)row * Hh + k], g3[row], acc);
        part[q * Hh + k] = acc;
      }
    }
    __syncthreads();
    for (int j = tid; j < Hh; j += GRU_THREADS) dh[j] += (part[j] + part[Hh + j]) + (part[2 * Hh + j] + part[3 * Hh + j]);
    __syncthreads();
  }
}

__global__ void transpose_kernel(const float* in, int rows, int cols, float* out) {
  // out[c][r] = in[r][c]
  const long long total = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols, c = i % cols;
    out[c * rows + r] = in[i];
  }
}

}  // namespace

int launch_gru_fwd(const float* gi, long long ldgi, int S, int Hh, const float* const whh[2], const float* const bhh[2],
                   float* out, long long ldo, float* saved, float* ws, hipStream_t s) {
  FX_REQUIRE(Hh > 0 && Hh <= 256, "gru: hidden size per direction must be <= 256");
  if (S == 0) return FX_OK;
  const int H3 = 3 * Hh;
  GruArgs args{};
  for (int d = 0; d < 2; ++d) {
    float* whT = ws + (long long)d * H3 * Hh;
    hipLaunchKernelGGL(transpose_kernel, dim3(256), dim3(256), 0, s, whh[d], H3, Hh, whT);
    GruDirArgs& a = args.d[d];
    a.gi = gi + d * H3;
    a.ldgi = ldgi;
    a.whT = whT;
    a.bhh = bhh[d];
    a.out = out + d * Hh;
    a.ldo = ldo;
    a.hprev = saved + (long long)d * S * Hh;
    a.gates = saved + 2LL * S * Hh + (long long)d * S * 4 * Hh;
    a.S = S;
    a.Hh = Hh;
    a.reverse = d;
  }
  const size_t lds = sizeof(float) * 4 * Hh;
  hipLaunchKernelGGL(gru_fwd_kernel, dim3(2), dim3(GRU_THREADS), lds, s, args);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int launch_gru_bwd(const float* dout, long long lddo, int S, int Hh, const float* const whh[2], const float* saved,
                   float* dgi, long long lddgi, float* dgh, hipStream_t s) {
  if (S == 0) return FX_OK;
  const int H3 = 3 * Hh;
  GruBwdArgs args{};
  for (int d = 0; d < 2; ++d) {
    GruBwdDirArgs& a = args.d[d];
    a.dout = dout + d * Hh;
    a.lddo = lddo;
    a.whh = whh[d];
    a.hprev = saved + (long long)d * S * Hh;
    a.gates = saved + 2LL * S * Hh + (long long)d * S * 4 * Hh;
    a.dgi = dgi + d * H3;
    a.lddgi = lddgi;
    a.dgh = dgh + (long long)d * S * H3;
    a.S = S;
    a.Hh = Hh;
    a.reverse = d;
  }
  const size_t lds = sizeof(float) * (Hh + 3 * Hh + 4 * Hh);
  hipLaunchKernelGGL(gru_bwd_kernel, dim3(2), dim3(GRU_THREADS), lds, s, args);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // namespace fx
