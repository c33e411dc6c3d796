// Diagnostic micro-benchmark: device time per launch of fx_gemm on the FACT shapes, timed with
// HIP events over back-to-back launches (no Python in the loop).  Not part of the product.
//   hipcc --offload-arch=gfx950 -O2 -I include tools/ubench.cpp -Lfact-clip_amd/factmx/_lib -lfactmx -o tools/ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "factmx.h"

__global__ void empty_kernel(float* p) {
  if (p && threadIdx.x == 1023) p[0] = 0.f;
}

static float* dalloc(size_t n, float scale) {
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((float)rand() / RAND_MAX - 0.5f);
  float* d;
  hipMalloc(&d, n * sizeof(float));
  hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
  return d;
}

static fx_operand rows(const float* p, long long ld) {
  fx_operand o{};
  o.ptr = p;
  o.ld = ld;
  o.conv_dir = 1;
  return o;
}
static fx_operand cols(const float* p, long long ld) {
  fx_operand o = rows(p, ld);
  o.trans = 1;
  return o;
}

template <class F>
static double time_us(F fn, int iters = 200) {
  for (int i = 0; i < 10; ++i) fn();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) fn();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3 / iters;
}

static void gemm_case(const char* name, int M, int N, int K, fx_operand a, fx_operand b, float* c, long long ldc,
                      int split = 1, float* ws = nullptr, float beta = 0.f, float* c_last = nullptr) {
  fx_gemm_desc d{};
  d.M = M; d.N = N; d.K = K; d.batch = 1; d.a = a; d.b = b; d.c = c; d.ldc = ldc; d.alpha = 1.f;
  d.split_k = split; d.workspace = ws; d.beta = beta; d.c_last_col = c_last;
  int st = fx_gemm(&d, nullptr);
  if (st) { printf("%s: error %s\n", name, fx_last_error()); return; }
  double us = time_us([&] { fx_gemm(&d, nullptr); });
  printf("%-34s M=%5d N=%5d K=%5d  %8.2f us  %7.2f TF/s\n", name, M, N, K, us, 2.0 * M * N * K / us / 1e6);
}

int main() {
  float* big = dalloc(8192 * 2048, 1.f);
  float* w = dalloc(2048 * 2048, 0.05f);
  float* c = dalloc(8192 * 2048, 0.f);
  float* ws = dalloc(16 * 1024 * 1024, 0.f);
  double e = time_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, 0, nullptr); }, 1000);
  printf("empty kernel (256 WG x 256)            %8.2f us\n", e);
  e = time_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(8), dim3(256), 0, 0, nullptr); }, 1000);
  printf("empty kernel (8 WG x 256)              %8.2f us\n", e);
  // token-level (Q = 32 action tokens)
  gemm_case("tok x.W^T   (rows,rows)", 32, 256, 256, rows(big, 256), rows(w, 256), c, 256);
  gemm_case("tok x.W^T   (rows,rows)", 32, 512, 256, rows(big, 256), rows(w, 256), c, 512);
  gemm_case("tok x.W^T   (rows,rows)", 32, 256, 512, rows(big, 512), rows(w, 512), c, 256);
  gemm_case("tok dy.W    (rows,cols)", 32, 256, 256, rows(big, 256), cols(w, 256), c, 256);
  gemm_case("tok dW dy^T.x (cols,cols)", 256, 256, 32, cols(big, 256), cols(w, 256), c, 256);
  gemm_case("tok dW dy^T.x (cols,cols)", 512, 256, 32, cols(big, 512), cols(w, 256), c, 256);
  {
    fx_operand bo = cols(w, 256);
    bo.ones_col = 257;
    gemm_case("tok dW+db beta1 (cols,cols+1)", 256, 257, 32, cols(big, 256), bo, c, 256, 1, nullptr, 1.f, c + 300000);
  }
  {
    float* xh = dalloc(4096 * 256, 1.f);   // sized for the 4096-row (frames) case
    float* rs = dalloc(4096, 1.f);
    float* lw = dalloc(1024, 1.f);
    float* dw = dalloc(1024, 0.f);
    float* lws = dalloc(1 << 20, 0.f);
    double us = time_us([&] { fx_layernorm_bwd(big, 256, nullptr, 0, xh, 256, lw, rs, 32, 256, 0, c, 256, dw, dw + 256,
                                               lws, nullptr); });
    printf("%-34s rows=32 cols=256           %8.2f us\n", "layernorm bwd (token)", us);
    us = time_us([&] { fx_layernorm_fwd(big, 256, nullptr, 0, lw, lw, 1e-5f, 32, 256, 0, c, 256, xh, 256, rs, nullptr); });
    printf("%-34s rows=32 cols=256           %8.2f us\n", "layernorm fwd (token)", us);
    us = time_us([&] { fx_layernorm_bwd(big, 256, nullptr, 0, xh, 256, lw, rs, 4096, 256, 0, c, 256, dw, dw + 256,
                                        lws, nullptr); });
    printf("%-34s rows=4096 cols=256         %8.2f us\n", "layernorm bwd (frames)", us);
  }
  // frame-level
  gemm_case("frame 1x1   (rows,rows)", 4096, 256, 256, rows(big, 256), rows(w, 256), c, 256);
  gemm_case("frame 1x1   (rows,rows)", 8192, 256, 256, rows(big, 256), rows(w, 256), c, 256);
  gemm_case("frame proj  (rows,rows)", 4096, 256, 512, rows(big, 512), rows(w, 512), c, 256);
  gemm_case("frame in-map(rows,rows)", 4096, 256, 2048, rows(big, 2048), rows(w, 2048), c, 256);
  gemm_case("frame 1x1 dX (rows,cols)", 4096, 256, 256, rows(big, 256), cols(w, 256), c, 256);
  gemm_case("frame dW (cols,cols) split8", 256, 256, 4096, cols(big, 256), cols(w, 256), c, 256, 8, ws);
  gemm_case("attn QK^T (rows,rows)", 32, 4096, 32, rows(big, 256), rows(w, 256), c, 4096);
  gemm_case("attn PV   (rows,cols)", 32, 32, 4096, rows(big, 4096), cols(w, 256), c, 32);
  return 0;
}
