// amdgpu-probe (N1): readiness/startup probe of the amd-driver DaemonSet.
//
// The reference checks the driver by hand: driver pods `2/2 Running`
// (/root/reference/README.md:132-139) and `nvidia-smi` inside the driver
// container (README.md:152).  The MI355X driver container runs this probe as
// its readiness probe and as the `driver-validation` gate: it exits 0 only when
// the amdgpu module is live, /dev/kfd exists, KFD exposes the expected number
// of GPU nodes and each has a render node.  With --json it prints the device
// inventory (the machine-readable counterpart of the nvidia-smi table,
// README.md:157-167).  With --ready-file it writes the validation status file
// other operands wait on.
//
// usage: amdgpu-probe [--root DIR] [--expect N] [--json] [--ready-file PATH]
//                     [--wait SECONDS]

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "amdgpu_topo.h"

static void print_json(const char* root) {
  int n = 0;
  at_enumerate(root, nullptr, 0, &n);
  std::vector<at_gpu_t> g(n > 0 ? n : 0);
  int cnt = 0;
  if (n > 0) at_enumerate(root, g.data(), n, &cnt);
  printf("{\"gpus\": [");
  for (int i = 0; i < cnt; ++i) {
    const at_gpu_t& d = g[i];
    printf("%s{\"kfd_node\": %d, \"gpu_id\": %u, \"arch\": \"%s\", \"cu\": %u, \"xcc\": %u, \"vram_bytes\": %llu, "
           "\"bdf\": \"%s\", \"render_minor\": %u, \"numa_node\": %d, \"xgmi_links\": %u, \"hive_id\": %llu, "
           "\"physical_index\": %d, \"partition_index\": %d, \"compute_partition\": \"%s\", \"memory_partition\": \"%s\"}",
           i ? ", " : "", d.kfd_node, d.gpu_id, d.arch, d.cu_count, d.num_xcc, (unsigned long long)d.vram_bytes, d.bdf,
           d.drm_render_minor, d.numa_node, d.num_xgmi_links, (unsigned long long)d.hive_id, d.physical_index,
           d.partition_index, d.compute_partition, d.memory_partition);
  }
  printf("]}\n");
}

int main(int argc, char** argv) {
  const char* root = "/";
  int expect = 0;
  bool json = false;
  const char* ready_file = nullptr;
  double wait_s = 0;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
    else if (!strcmp(argv[i], "--expect") && i + 1 < argc) expect = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--json")) json = true;
    else if (!strcmp(argv[i], "--ready-file") && i + 1 < argc) ready_file = argv[++i];
    else if (!strcmp(argv[i], "--wait") && i + 1 < argc) wait_s = atof(argv[++i]);
    else {
      fprintf(stderr, "usage: %s [--root DIR] [--expect N] [--json] [--ready-file PATH] [--wait SECONDS]\n", argv[0]);
      return 2;
    }
  }
  char msg[256];
  auto t0 = std::chrono::steady_clock::now();
  int rc;
  for (;;) {
    rc = at_probe(root, expect, msg, sizeof(msg));
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc == AT_OK || el >= wait_s) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
  }
  double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (json) print_json(root);
  fprintf(stderr, "amdgpu-probe: %s (%.3fs)\n", msg, el);
  if (rc == AT_OK && ready_file) {
    FILE* f = fopen(ready_file, "w");
    if (!f) {
      perror("ready-file");
      return 3;
    }
    fprintf(f, "driver-ready %s\n", msg);
    fclose(f);
  }
  return rc == AT_OK ? 0 : 1;
}
