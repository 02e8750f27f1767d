// Two-arch (gfx942 + gfx950) HIP library with a compressed offload bundle:
// the stand-in for librccl in tests/test_fatbin.py (toolkit/fatbin.py trims it).
#include <hip/hip_runtime.h>
__global__ void add1(float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += 1.0f;
}
extern "C" int launch_add1(float* x, int n) {
  add1<<<(n + 255) / 256, 256>>>(x, n);
  return (int)hipDeviceSynchronize();
}
extern "C" int answer() { return 42; }
