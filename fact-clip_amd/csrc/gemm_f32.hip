// f32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32 products,
// k-ordered fma chain; no xf32 on gfx950, so the parity path stays fp32).
//
// One kernel covers every dense contraction of the FACT frame/action branches:
//   * Linear / Conv1d(k=1) forward:        A=x (rows), B=W (rows, = N x K)
//   * implicit dilated Conv1d(k=3):        A = x gathered per tap (conv_taps=3)
//   * dX of both (B = W read K-major, taps reversed for the conv)
//   * dW = dY^T X (A read column-major, split-K over the frame axis)
//   * concatenated inputs (Y_W(cat[Y, feat]), sf_merge) and row gathers
// Tile: 64x64 output per 256-thread workgroup, 4 waves each owning a 32x32
// accumulator (16 f32 AGPR/VGPR per lane), K staged through LDS in 32-deep
// slices with a register prefetch of the next slice (one barrier per slice).
// LDS images are stored [k][row] with a +1 pad: MFMA operand reads are
// ds_read_b32 of 32 consecutive rows (conflict-free), staging writes are at
// most 2-way (free for ds_write_b32 on gfx950).
#include <algorithm>

#include "fx_common.h"

namespace fx {
namespace {

constexpr int BM = 64, BN = 64, BK = 32, NTHREADS = 256, LDSS = 65;
typedef float f32x16 __attribute__((ext_vector_type(16)));

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
};

__device__ __forceinline__ int conv_shift(const fx_operand& o, int tap) {
  return (tap - (o.conv_taps - 1) / 2) * o.conv_dil * o.conv_dir;
}

// element (r,k) of a trans==0 operand; r < R, k < K guaranteed by the caller
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

// element (r,k) of a trans==1 operand
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

// 8 consecutive k of row r (trans==0)
__device__ __forceinline__ void load_rm8(const fx_operand& o, const float* p0, int r, int R, int k,
                                         int K, bool vec, float* v) {
  if (r >= R) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    return;
  }
  if (vec && k + 8 <= K) {
    const float* src;
    bool pos_add = false;
    if (o.conv_taps) {
      const int j = k / o.conv_cin, c = k - j * o.conv_cin, s = conv_shift(o, j);
      const int t = r % o.seq_len + s;
      if (t < 0 || t >= o.seq_len) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
        return;
      }
      src = p0 + (long long)(r + s) * o.ld + c;
    } else if (o.ptr1 && k >= o.k_split) {
      const int rr = o.rows1 ? o.rows1[r] : r;
      src = o.ptr1 + (long long)rr * o.ld1 + (k - o.k_split);
    } else {
      const int rr = o.rows0 ? o.rows0[r] : r;
      src = p0 + (long long)rr * o.ld + k;
      pos_add = o.pos && k < o.pos_cols;
    }
    const float4 x0 = *reinterpret_cast<const float4*>(src);
    const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
    v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    if (pos_add) {
      const float* pp = o.pos + (long long)r * o.ld_pos;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (k + e < o.pos_cols) v[e] += pp[k + e];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (k + e < K) ? fetch_rm(o, p0, r, k + e) : 0.f;
}

// 8 consecutive rows r..r+7 at one k (trans==1)
__device__ __forceinline__ void load_cm8(const fx_operand& o, const float* p0, int r, int R, int k,
                                         int K, bool vec, float* v) {
  if (k >= K) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    return;
  }
  if (vec && r + 8 <= R && !(o.ones_col && r + 8 >= o.ones_col)) {
    const float* src;
    if (o.conv_taps) {
      const int j = r / o.conv_cin, c = r - j * o.conv_cin, s = conv_shift(o, j);
      const int t = k % o.seq_len + s;
      if (t < 0 || t >= o.seq_len) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
        return;
      }
      src = p0 + (long long)(k + s) * o.ld + c;
    } else {
      src = p0 + (long long)k * o.ld + r;
    }
    const float4 x0 = *reinterpret_cast<const float4*>(src);
    const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
    v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    return;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (r + e < R) ? fetch_cm(o, p0, r + e, k) : 0.f;
}

template <bool TR>
__device__ __forceinline__ void load_tile(const fx_operand& o, const float* p0, int r0, int R, int k0,
                                          int K, bool vec, int tid, float* v) {
  if (!TR) load_rm8(o, p0, r0 + (tid >> 2), R, k0 + (tid & 3) * 8, K, vec, v);
  else load_cm8(o, p0, r0 + (tid & 7) * 8, R, k0 + (tid >> 3), K, vec, v);
}

template <bool TR>
__device__ __forceinline__ void store_tile(float (*s)[LDSS], int tid, const float* v) {
  if (!TR) {
    const int r = tid >> 2, kq = (tid & 3) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) s[kq + e][r] = v[e];
  } else {
    const int k = tid >> 3, rq = (tid & 7) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) s[k][rq + e] = v[e];
  }
}

// epilogue: v = alpha*acc (+bias) [relu==2: ReLU here] (+resid) (+beta*C_old) (*gate>0) [relu==1: ReLU]
// c_tap_cin != 0: output column n = tap*c_tap_cin + c is stored at c*3 + tap (Conv1d weight layout)
__device__ __forceinline__ void epilogue_store(const GemmDev& g, int b, int m, int n, float acc) {
  float v = g.alpha * acc;
  if (g.c_last && n == g.N - 1) {   // fused bias-gradient column
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

template <bool ATR, bool BTR>
__global__ __launch_bounds__(NTHREADS) void gemm_f32_kernel(GemmDev g) {
  __shared__ float sA[2][BK][LDSS];
  __shared__ float sB[2][BK][LDSS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int z = blockIdx.z, bidx = z / g.split, sk = z - bidx * g.split;
  const float* pa = g.a.ptr + (long long)bidx * g.a.batch_stride;
  const float* pb = g.b.ptr + (long long)bidx * g.b.batch_stride;
  const int nkt = (g.K + BK - 1) / BK;
  const int kt0 = sk * g.kt_per_split;
  const int kt1 = min(nkt, kt0 + g.kt_per_split);

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  float ra[8], rb[8];
  if (kt0 < kt1) {
    load_tile<ATR>(g.a, pa, m0, g.M, kt0 * BK, g.K, g.a_vec, tid, ra);
    load_tile<BTR>(g.b, pb, n0, g.N, kt0 * BK, g.K, g.b_vec, tid, rb);
    store_tile<ATR>(sA[0], tid, ra);
    store_tile<BTR>(sB[0], tid, rb);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      load_tile<ATR>(g.a, pa, m0, g.M, (kt + 1) * BK, g.K, g.a_vec, tid, ra);
      load_tile<BTR>(g.b, pb, n0, g.N, (kt + 1) * BK, g.K, g.b_vec, tid, rb);
    }
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const float av = sA[cur][2 * s + lh][wm * 32 + li];
      const float bv = sB[cur][2 * s + lh][wn * 32 + li];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    if (more) {
      store_tile<ATR>(sA[cur ^ 1], tid, ra);
      store_tile<BTR>(sB[cur ^ 1], tid, rb);
    }
    __syncthreads();
  }

  // C/D layout of the 32x32 f32 accumulator: col = lane&31, row = (r&3)+8*(r>>2)+4*(lane>>5)
  const int col = n0 + wn * 32 + li;
  if (col >= g.N) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
    if (row >= g.M) continue;
    if (g.split > 1) {
      g.ws[(((long long)bidx * g.split + sk) * g.M + row) * g.N + col] = acc[r];
    } else {
      epilogue_store(g, bidx, row, col, acc[r]);
    }
  }
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

// bias-gradient column sums, two deterministic stages
constexpr int CS_ROWS = 128;
__global__ __launch_bounds__(256) void colsum_stage1(const float* x, long long ld, int M, int N, float* ws) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;  // 4 row groups
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
  g.a_vec = operand_vec_ok(d.a);
  g.b_vec = operand_vec_ok(d.b);
  const int nkt = cdiv(d.K, BK);
  int split = d.split_k > 1 ? d.split_k : 1;
  if (split > nkt) split = nkt > 0 ? nkt : 1;
  g.kt_per_split = nkt > 0 ? cdiv(nkt, split) : 0;
  split = g.kt_per_split > 0 ? cdiv(nkt, g.kt_per_split) : 1;
  g.split = split;
  g.ws = d.workspace;
  if (split > 1) FX_REQUIRE(d.workspace, "gemm: split-K needs a workspace");
  dim3 grid(cdiv(d.N, BN), cdiv(d.M, BM), d.batch * split);
  const int ta = d.a.trans ? 1 : 0, tb = d.b.trans ? 1 : 0;
  if (!ta && !tb) hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(NTHREADS), 0, s, g);
  else if (!ta && tb) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(NTHREADS), 0, s, g);
  else if (ta && !tb) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(NTHREADS), 0, s, g);
  else hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(NTHREADS), 0, s, g);
  FX_CHECK_HIP(hipGetLastError());
  if (split > 1) {
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
