// Train-step tail on flat buffers: gradient 2-norm, clip_grad_norm_ and Adam in two launches.
//
// Replaces scripts/train.py:265-267 (torch.nn.utils.clip_grad_norm_(params, clip_grad_norm) then
// torch.optim.Adam.step()) for a model whose parameters and gradients live in one flat fp32
// buffer each (factmx.optim.FlatParams / factmx.dp.FlatGradReducer).  The reference's foreach
// path issues ~20 multi-tensor launches over 400+ parameter tensors plus per-tensor host work;
// here:
//   1. sumsq_partial_kernel: fixed grid of 1024 blocks, each a deterministic partial sum of g^2
//   2. adam_kernel: every block re-reduces the 1024 partials in the same order (so the norm and
//      clip coefficient are bit-identical everywhere, no third launch, no host sync), scales g by
//      clamp(max_norm / (norm + 1e-6), max=1) (written back: param.grad holds the clipped
//      gradient as after clip_grad_norm_), then the Adam update of torch's _multi_tensor_adam:
//        m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g*g
//        p = p - (lr/bc1) * (m / (sqrt(v)/sqrt(bc2) + eps))
//      with L2 weight decay g += wd*p first when wd != 0 (torch.optim.Adam semantics).
// HBM-bound: 4 B x (g read + g write + p rw + m rw + v rw) = 32 B per parameter (+4 for the norm).
#include <algorithm>
#include <cmath>

#include "fx_common.h"

namespace fx {
namespace {

constexpr int NPART = 1024;
constexpr int TPB = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

__global__ __launch_bounds__(TPB) void sumsq_partial_kernel(const float* __restrict__ g, long long n,
                                                            float* __restrict__ part) {
  __shared__ float red[TPB / 64];
  const long long per = (n + NPART - 1) / NPART;
  const long long b0 = (long long)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  float s = 0.f;
  for (long long i = b0 + threadIdx.x; i < b1; i += TPB) s += g[i] * g[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

struct AdamArgs {
  float* p;
  float* g;
  float* m;
  float* v;
  long long n;
  const float* part;   // NPART partial sums of g^2 (nullable: no clipping)
  float max_norm;
  float lr_bc1;        // lr / (1 - b1^t)
  float bc2_sqrt;      // sqrt(1 - b2^t)
  float b1, b2, eps, wd;
  float* norm_out;     // nullable: total norm written by block 0
  const int* status;   // nullable: the device status word; non-zero (a kernel of the step failed, e.g. a
                       // BiGRU backward timeout) -> the whole update is skipped, p / m / v / g untouched
};

__global__ __launch_bounds__(TPB) void adam_kernel(AdamArgs a) {
  __shared__ float coef_s;
  if (a.status && a.status[0] != 0) return;   // uniform over the grid: every block skips
  float coef = 1.f;
  if (a.part) {
    if (threadIdx.x < 64) {
      // fixed-order reduction of the partials (identical in every block)
      float s = 0.f;
      for (int i = threadIdx.x; i < NPART; i += 64) s += a.part[i];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (threadIdx.x == 0) {
        const float norm = sqrtf(s);
        coef_s = fminf(a.max_norm / (norm + 1e-6f), 1.f);
        if (a.norm_out && blockIdx.x == 0) a.norm_out[0] = norm;
      }
    }
    __syncthreads();
    coef = coef_s;
  }
  const float omb1 = 1.f - a.b1, omb2 = 1.f - a.b2;
  const long long n4 = a.n >> 2;
  const long long stride = (long long)gridDim.x * TPB;
  for (long long i = (long long)blockIdx.x * TPB + threadIdx.x; i < n4; i += stride) {
    float4 g = reinterpret_cast<float4*>(a.g)[i];
    float4 p = reinterpret_cast<float4*>(a.p)[i];
    float4 m = reinterpret_cast<float4*>(a.m)[i];
    float4 v = reinterpret_cast<float4*>(a.v)[i];
    float* gp = &g.x;
    float* pp = &p.x;
    float* mp = &m.x;
    float* vp = &v.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gp[j] * coef;
      gp[j] = gj;
      if (a.wd != 0.f) gj += a.wd * pp[j];
      mp[j] = mp[j] + omb1 * (gj - mp[j]);
      vp[j] = a.b2 * vp[j] + omb2 * gj * gj;
      pp[j] = pp[j] - a.lr_bc1 * (mp[j] / (sqrtf(vp[j]) / a.bc2_sqrt + a.eps));
    }
    if (coef != 1.f) reinterpret_cast<float4*>(a.g)[i] = g;
    reinterpret_cast<float4*>(a.p)[i] = p;
    reinterpret_cast<float4*>(a.m)[i] = m;
    reinterpret_cast<float4*>(a.v)[i] = v;
  }
  // scalar tail (n % 4)
  for (long long i = (n4 << 2) + (long long)blockIdx.x * TPB + threadIdx.x; i < a.n; i += stride) {
    float gj = a.g[i] * coef;
    if (coef != 1.f) a.g[i] = gj;
    if (a.wd != 0.f) gj += a.wd * a.p[i];
    const float mj = a.m[i] + omb1 * (gj - a.m[i]);
    const float vj = a.b2 * a.v[i] + omb2 * gj * gj;
    a.m[i] = mj;
    a.v[i] = vj;
    a.p[i] = a.p[i] - a.lr_bc1 * (mj / (sqrtf(vj) / a.bc2_sqrt + a.eps));
  }
}

__global__ __launch_bounds__(TPB) void norm_final_kernel(const float* part, float* norm_out) {
  if (threadIdx.x >= 64) return;
  float s = 0.f;
  for (int i = threadIdx.x; i < NPART; i += 64) s += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (threadIdx.x == 0) norm_out[0] = sqrtf(s);
}

__global__ __launch_bounds__(TPB) void scale_kernel(float* g, long long n, const float* part, float max_norm) {
  __shared__ float coef_s;
  if (threadIdx.x < 64) {
    float s = 0.f;
    for (int i = threadIdx.x; i < NPART; i += 64) s += part[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (threadIdx.x == 0) coef_s = fminf(max_norm / (sqrtf(s) + 1e-6f), 1.f);
  }
  __syncthreads();
  const float c = coef_s;
  if (c == 1.f) return;
  for (long long i = (long long)blockIdx.x * TPB + threadIdx.x; i < n; i += (long long)gridDim.x * TPB) g[i] *= c;
}

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

long long fx_grad_norm_workspace_floats(void) { return NPART; }

int fx_grad_norm(const float* g, long long n, float* workspace, float* norm_out, void* stream) {
  FX_REQUIRE(n >= 0 && g && workspace, "grad_norm: null buffer");
  hipStream_t s = (hipStream_t)stream;
  fx_launch(sumsq_partial_kernel, dim3(NPART), dim3(TPB), 0, s, g, n, workspace);
  if (norm_out) fx_launch(norm_final_kernel, dim3(1), dim3(TPB), 0, s, workspace, norm_out);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_clip_grad_scale(float* g, long long n, const float* workspace, float max_norm, void* stream) {
  FX_REQUIRE(n >= 0 && g && workspace, "clip_grad_scale: null buffer");
  fx_launch(scale_kernel, dim3(1024), dim3(TPB), 0, (hipStream_t)stream, g, n, workspace, max_norm);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

int fx_adam_step(float* p, float* g, float* m, float* v, long long n, long long step, float lr, float beta1,
                 float beta2, float eps, float weight_decay, float max_norm, float* workspace, float* norm_out,
                 void* stream) {
  return fx_adam_step_checked(p, g, m, v, n, step, lr, beta1, beta2, eps, weight_decay, max_norm, workspace, norm_out,
                              nullptr, stream);
}

int fx_adam_step_checked(float* p, float* g, float* m, float* v, long long n, long long step, float lr, float beta1,
                         float beta2, float eps, float weight_decay, float max_norm, float* workspace, float* norm_out,
                         const int* status, void* stream) {
  FX_REQUIRE(n >= 0 && p && g && m && v, "adam_step: null buffer");
  FX_REQUIRE(step >= 1, "adam_step: step counts from 1");
  FX_REQUIRE(((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
               reinterpret_cast<uintptr_t>(v)) & 15) == 0, "adam_step: buffers must be 16-byte aligned");
  FX_REQUIRE(!(max_norm > 0.f && !workspace), "adam_step: clipping needs the grad-norm workspace");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return FX_OK;
  AdamArgs a{};
  a.p = p; a.g = g; a.m = m; a.v = v; a.n = n;
  a.part = max_norm > 0.f ? workspace : nullptr;
  a.max_norm = max_norm;
  // torch.optim.Adam (foreach): bias corrections in double on the host, applied as f32 scalars
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  a.lr_bc1 = (float)(lr / bc1);
  a.bc2_sqrt = (float)std::sqrt(bc2);
  a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay;
  a.norm_out = norm_out;
  a.status = status;
  if (a.part) fx_launch(sumsq_partial_kernel, dim3(NPART), dim3(TPB), 0, s, g, n, workspace);
  const long long n4 = (n + 3) / 4;
  const int blocks = (int)std::min<long long>((n4 + TPB - 1) / TPB, 2048);
  fx_launch(adam_kernel, dim3(blocks), dim3(TPB), 0, s, a);
  FX_CHECK_HIP(hipGetLastError());
  return FX_OK;
}

}  // extern "C"
