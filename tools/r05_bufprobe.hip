// Round-5 probe: sc1 buffer load / store through __builtin_amdgcn_make_buffer_rsrc, and the kernel-argument
// segment pointer, on the GPU (hipcc --offload-arch=gfx950 tools/r05_bufprobe.hip -o tools/r05_bufprobe).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));
struct Args { const float* a; float* b; int n; int pad[61]; int tail; };
__global__ void k(Args g) {
  auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.a), 0, 0x7fffffff, 0x00020000);
  auto rb = __builtin_amdgcn_make_buffer_rsrc(g.b, 0, 0x7fffffff, 0x00020000);
  const int i = threadIdx.x;
  v4f v = __builtin_amdgcn_raw_buffer_load_b128(ra, i * 16, 0, 16);
  v[0] += 1.f;
  __builtin_amdgcn_raw_buffer_store_b128(v, rb, i * 16, 0, 16);
#if defined(__HIP_DEVICE_COMPILE__)
  const Args* pk = (const Args*)(__builtin_amdgcn_kernarg_segment_ptr());
  if (i == 0) g.b[1000] = (float)pk->tail, g.b[1001] = (float)pk->n;
#endif
}
int main() {
  float *a, *b;
  hipMalloc(&a, 8192); hipMalloc(&b, 8192);
  float h[2048];
  for (int i = 0; i < 2048; ++i) h[i] = i;
  hipMemcpy(a, h, 8192, hipMemcpyHostToDevice);
  hipMemset(b, 0, 8192);
  Args g{}; g.a = a; g.b = b; g.n = 7; g.tail = 1234;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, g);
  hipDeviceSynchronize();
  hipMemcpy(h, b, 8192, hipMemcpyDeviceToHost);
  printf("b[0..7] %g %g %g %g %g %g %g %g  tail %g n %g\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[1000], h[1001]);
  return 0;
}
