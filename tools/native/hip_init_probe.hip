// Where a fresh process's HIP start-up goes on this box (tools/hip_init_probe.sh):
// wall-clock of each first call, from main.  One JSON line.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <string>

__global__ void touch(float* p) { p[threadIdx.x] = 1.0f; }

int main() {
  using C = std::chrono::steady_clock;
  auto t0 = C::now();
  auto ms = [&]() { return std::chrono::duration<double, std::milli>(C::now() - t0).count(); };
  std::string out = "{";
  auto mark = [&](const char* k) { out += "\"" + std::string(k) + "\": " + std::to_string(ms()) + ", "; };
  if (hipInit(0) != hipSuccess) return 1;
  mark("hipInit");
  int n = 0;
  (void)hipGetDeviceCount(&n);
  mark("hipGetDeviceCount");
  (void)hipSetDevice(0);
  mark("hipSetDevice");
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  mark("hipGetDeviceProperties");
  (void)hipFree(nullptr);
  mark("hipFree0");
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  mark("hipStreamCreate");
  float* d = nullptr;
  (void)hipMalloc(&d, 64 << 20);
  mark("hipMalloc64M");
  touch<<<1, 64, 0, s>>>(d);
  (void)hipStreamSynchronize(s);
  mark("firstKernel");
  touch<<<1, 64, 0, s>>>(d);
  (void)hipStreamSynchronize(s);
  mark("secondKernel");
  out += "\"devices\": " + std::to_string(n) + "}";
  puts(out.c_str());
  fflush(stdout);
  _exit(0);
}
