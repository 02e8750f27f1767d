// Does freeing a large VRAM buffer delay an HSA queue creation right after it?
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>
#include <thread>
using Clock = std::chrono::steady_clock;
static double ms(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }
#define OK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
static hsa_status_t find_gpu(hsa_agent_t a, void* d) {
  hsa_device_type_t t; hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) { *(hsa_agent_t*)d = a; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}
static double queue_ms(hsa_agent_t gpu) {
  hsa_queue_t* q = nullptr;
  auto t = Clock::now();
  if (hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q) != HSA_STATUS_SUCCESS) return -1;
  double r = ms(t);
  hsa_queue_destroy(q);
  return r;
}
int main(int argc, char** argv) {
  const size_t big = (argc > 1 ? atoll(argv[1]) : 2048) << 20;
  OK(hipSetDevice(0));
  hipStream_t s;
  OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hsa_init();
  hsa_agent_t gpu{0};
  hsa_iterate_agents(find_gpu, &gpu);
  queue_ms(gpu);  // first-queue costs
  for (int round = 0; round < 6; ++round) {
    void* p;
    OK(hipMalloc(&p, big));
    OK(hipMemsetAsync(p, 1, big, s));
    OK(hipStreamSynchronize(s));
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    double idle = queue_ms(gpu);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    auto t = Clock::now();
    OK(hipFree(p));
    double f = ms(t);
    double after = queue_ms(gpu);
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    double later = queue_ms(gpu);
    printf("round %d (%zu MiB): queue create idle %.2f ms | right after hipFree %.2f ms (free %.2f ms) | 100 ms later %.2f ms\n",
           round, big >> 20, idle, after, f, later);
  }
  return 0;
}
