// topo_selftest - drives every entry point of libamdgpu_topo (N3 enumeration
// and links, N1 probe, N4 collector, N6 health watcher) once against a sysfs
// root and prints the result as JSON.  Built with ASan/UBSan by `make
// sanitize` and compared against the ctypes view in
// tests/test_native_sanitize.py.  Without a GPU the N4/N6 calls take their
// "library or device unavailable" paths, which is what the sanitizers check
// there; on the GPU box they run for real.

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "amdgpu_topo.h"

int main(int argc, char** argv) {
  const char* root = argc > 1 ? argv[1] : "/";
  const bool with_smi = argc > 2 && std::string(argv[2]) == "--smi";
  std::vector<at_gpu_t> gpus(256);
  int n = 0;
  int rc = at_enumerate(root, gpus.data(), (int)gpus.size(), &n);
  printf("{\"abi\": %d, \"enumerate_rc\": %d, \"gpus\": [", at_abi_version(), rc);
  for (int i = 0; i < n; ++i)
    printf("%s{\"bdf\": \"%s\", \"arch\": \"%s\", \"cu\": %u, \"xgmi\": %u, \"partition\": \"%s\", \"pidx\": %d}",
           i ? ", " : "", gpus[i].bdf, gpus[i].arch, gpus[i].cu_count, gpus[i].num_xgmi_links,
           gpus[i].compute_partition, gpus[i].partition_index);
  std::vector<at_link_t> links(4096);
  int nl = 0;
  rc = at_links(root, links.data(), (int)links.size(), &nl);
  int xgmi = 0;
  for (int i = 0; i < nl; ++i) xgmi += links[i].type == AT_LINK_XGMI;
  // too-small output buffers must report NOSPC, never overflow
  at_gpu_t one;
  int n1 = 0;
  const int nospc = n > 1 ? at_enumerate(root, &one, 1, &n1) : AT_ERR_NOSPC;
  char msg[96];
  const int probe = at_probe(root, n, msg, sizeof msg);
  printf("], \"links_rc\": %d, \"links\": %d, \"xgmi_links\": %d, \"nospc_rc\": %d, \"probe_rc\": %d", rc, nl, xgmi,
         nospc, probe);
  if (with_smi) {
    const int open_rc = at_smi_open();
    int collected = -1;
    if (open_rc == AT_OK) {
      std::vector<at_metrics_t> m(64);
      int c = 0;
      if (at_smi_collect(m.data(), (int)m.size(), &c) == AT_OK) collected = c;
      at_smi_close();
    }
    const int hs = at_health_start();
    at_event_t ev[16];
    int ne = 0;
    const int hp = at_health_poll(10, ev, 16, &ne);
    at_health_stop();
    printf(", \"smi_open_rc\": %d, \"smi_collected\": %d, \"health_start_rc\": %d, \"health_poll_rc\": %d", open_rc,
           collected, hs, hp);
  }
  printf("}\n");
  return 0;
}
