// N3: MI355X device + topology enumeration from KFD / PCI / DRM sysfs, and the
// N1 driver readiness probe.  See amdgpu_topo.h.
//
// Sources read (all relative to `root`):
//   sys/class/kfd/kfd/topology/nodes/<n>/{properties,gpu_id}
//   sys/class/kfd/kfd/topology/nodes/<n>/mem_banks/<m>/properties
//   sys/class/kfd/kfd/topology/nodes/<n>/{io_links,p2p_links}/<l>/properties
//   sys/bus/pci/devices/<bdf>/{numa_node,current_compute_partition,current_memory_partition}
//   sys/module/amdgpu/initstate, dev/kfd, dev/dri/renderD<minor>

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "amdgpu_topo.h"

namespace {

std::string join(const char* root, const std::string& rel) {
  std::string r = (root && *root) ? root : "/";
  if (r.back() != '/') r += '/';
  return r + rel;
}

// sysfs attributes are small: one open + read(2) + close, no iostreams (a
// CPX node has ~4 K io_link property files; stream set-up dominated the scan)
bool read_file(const std::string& path, std::string* out) {
  const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  out->clear();
  char buf[4096];
  for (;;) {
    const ssize_t n = read(fd, buf, sizeof(buf));
    if (n < 0) {
      close(fd);
      return false;
    }
    if (n == 0) break;
    out->append(buf, (size_t)n);
  }
  close(fd);
  return true;
}

std::string trim(std::string s) {
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.pop_back();
  size_t i = 0;
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
  return s.substr(i);
}

using Props = std::map<std::string, unsigned long long>;

Props read_props(const std::string& path) {
  Props p;
  std::string text;
  if (!read_file(path, &text)) return p;
  // "key value\n" lines; a line whose value does not parse is skipped
  const char* c = text.c_str();
  const char* end = c + text.size();
  while (c < end) {
    const char* eol = static_cast<const char*>(memchr(c, '\n', (size_t)(end - c)));
    if (!eol) eol = end;
    const char* k = c;
    while (k < eol && (*k == ' ' || *k == '\t')) ++k;
    const char* ke = k;
    while (ke < eol && *ke != ' ' && *ke != '\t') ++ke;
    const char* v = ke;
    while (v < eol && (*v == ' ' || *v == '\t')) ++v;
    if (ke > k && v < eol && *v >= '0' && *v <= '9') p[std::string(k, ke)] = strtoull(v, nullptr, 10);
    c = eol + 1;
  }
  return p;
}

unsigned long long get(const Props& p, const char* k, unsigned long long dflt = 0) {
  auto it = p.find(k);
  return it == p.end() ? dflt : it->second;
}

std::vector<int> numeric_entries(const std::string& dir) {
  std::vector<int> out;
  DIR* d = opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    const char* n = e->d_name;
    if (!*n) continue;
    bool num = true;
    for (const char* c = n; *c; ++c) num &= (*c >= '0' && *c <= '9');
    if (num) out.push_back(atoi(n));
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

bool exists(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

void copy_str(char* dst, size_t cap, const std::string& s) {
  size_t n = std::min(cap - 1, s.size());
  memcpy(dst, s.data(), n);
  dst[n] = 0;
}

std::string arch_from_version(unsigned long long v) {
  if (!v) return "";
  unsigned major = v / 10000, minor = (v / 100) % 100, step = v % 100;
  char buf[16];
  snprintf(buf, sizeof(buf), "gfx%u%x%x", major, minor, step);
  return buf;
}

struct KfdNode {
  int node;
  Props props;
  unsigned gpu_id;
};

std::string topo_dir(const char* root) { return join(root, "sys/class/kfd/kfd/topology/nodes"); }

// AMDGPU_VISIBLE_GPUS="0,2,0000:a4:00.0": node-level allow-list (enumeration
// index or PCI BDF), e.g. GPUs reserved for the host or a partial-node job.
bool visible(size_t index, const Props& p) {
  const char* env = getenv("AMDGPU_VISIBLE_GPUS");
  if (!env || !*env) return true;
  const unsigned loc = (unsigned)get(p, "location_id"), dom = (unsigned)get(p, "domain");
  char bdf[32];
  snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", dom & 0xffff, (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 7);
  std::stringstream ss(env);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    tok = trim(tok);
    if (tok.empty()) continue;
    if (tok.find_first_not_of("0123456789") == std::string::npos) {
      if ((size_t)atoi(tok.c_str()) == index) return true;
    } else if (tok == bdf) {
      return true;
    }
  }
  return false;
}

// GPU nodes in KFD order (CPU nodes have simd_count == 0 or gpu_id == 0)
std::vector<KfdNode> gpu_nodes(const char* root) {
  std::vector<KfdNode> out;
  size_t gpu_index = 0;
  const std::string base = topo_dir(root);
  for (int n : numeric_entries(base)) {
    const std::string nd = base + "/" + std::to_string(n);
    KfdNode k;
    k.node = n;
    k.props = read_props(nd + "/properties");
    std::string gid;
    k.gpu_id = read_file(nd + "/gpu_id", &gid) ? (unsigned)strtoul(trim(gid).c_str(), nullptr, 10) : 0;
    if (get(k.props, "simd_count") == 0 || k.gpu_id == 0) continue;
    if (visible(gpu_index++, k.props)) out.push_back(k);
  }
  return out;
}

void fill_gpu(const char* root, const KfdNode& k, at_gpu_t* g) {
  memset(g, 0, sizeof(*g));
  const Props& p = k.props;
  g->kfd_node = k.node;
  g->gpu_id = k.gpu_id;
  g->gfx_target_version = (uint32_t)get(p, "gfx_target_version");
  copy_str(g->arch, sizeof(g->arch), arch_from_version(g->gfx_target_version));
  g->simd_count = (uint32_t)get(p, "simd_count");
  g->simd_per_cu = (uint32_t)get(p, "simd_per_cu", 4);
  g->cu_count = g->simd_per_cu ? g->simd_count / g->simd_per_cu : 0;
  g->num_xcc = (uint32_t)get(p, "num_xcc", 1);
  g->max_waves_per_simd = (uint32_t)get(p, "max_waves_per_simd");
  g->wave_front_size = (uint32_t)get(p, "wave_front_size", 64);
  g->lds_size_kib = (uint32_t)get(p, "lds_size_in_kb");
  g->max_engine_clk_mhz = (uint32_t)get(p, "max_engine_clk_fcompute");
  g->drm_render_minor = (uint32_t)get(p, "drm_render_minor");
  g->domain = (uint32_t)get(p, "domain");
  g->location_id = (uint32_t)get(p, "location_id");
  g->vendor_id = (uint32_t)get(p, "vendor_id");
  g->device_id = (uint32_t)get(p, "device_id");
  g->unique_id = get(p, "unique_id");
  g->hive_id = get(p, "hive_id");
  char bdf[32];
  snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", g->domain & 0xffff, (g->location_id >> 8) & 0xff,
           (g->location_id >> 3) & 0x1f, g->location_id & 7);
  copy_str(g->bdf, sizeof(g->bdf), bdf);

  const std::string nd = topo_dir(root) + "/" + std::to_string(k.node);
  uint64_t vram = 0;
  for (int m : numeric_entries(nd + "/mem_banks")) {
    Props mp = read_props(nd + "/mem_banks/" + std::to_string(m) + "/properties");
    unsigned long long ht = get(mp, "heap_type");
    if (ht == 1 || ht == 2) vram += get(mp, "size_in_bytes");
  }
  if (!vram) vram = get(p, "local_mem_size");
  g->vram_bytes = vram;

  const std::string pci = join(root, std::string("sys/bus/pci/devices/") + bdf);
  std::string s;
  g->numa_node = read_file(pci + "/numa_node", &s) ? atoi(trim(s).c_str()) : -1;
  if (read_file(pci + "/current_compute_partition", &s)) copy_str(g->compute_partition, sizeof(g->compute_partition), trim(s));
  if (read_file(pci + "/current_memory_partition", &s)) copy_str(g->memory_partition, sizeof(g->memory_partition), trim(s));
  g->physical_index = -1;
  g->partition_index = 0;
  g->partition_count = 1;
}

}  // namespace

extern "C" {

AT_API int at_abi_version(void) { return 1; }

AT_API int at_enumerate(const char* root, at_gpu_t* out, int max, int* count) {
  if (!count || max < 0 || (max > 0 && !out)) return AT_ERR_INVAL;
  std::vector<KfdNode> nodes = gpu_nodes(root);
  std::vector<at_gpu_t> gpus(nodes.size());
  for (size_t i = 0; i < nodes.size(); ++i) fill_gpu(root, nodes[i], &gpus[i]);

  // group partitions of one physical GPU (same PCI domain + location)
  std::map<std::pair<uint32_t, uint32_t>, std::vector<size_t>> phys;
  std::vector<std::pair<uint32_t, uint32_t>> order;
  for (size_t i = 0; i < gpus.size(); ++i) {
    auto key = std::make_pair(gpus[i].domain, gpus[i].location_id);
    if (!phys.count(key)) order.push_back(key);
    phys[key].push_back(i);
  }
  for (size_t pi = 0; pi < order.size(); ++pi) {
    auto& members = phys[order[pi]];
    for (size_t j = 0; j < members.size(); ++j) {
      at_gpu_t& g = gpus[members[j]];
      g.physical_index = (int)pi;
      g.partition_index = (int)j;
      g.partition_count = (int)members.size();
    }
  }

  // xGMI link count per GPU node (io_links + p2p_links to other GPU nodes)
  std::map<int, size_t> node_to_idx;
  for (size_t i = 0; i < nodes.size(); ++i) node_to_idx[nodes[i].node] = i;
  for (size_t i = 0; i < nodes.size(); ++i) {
    const std::string nd = topo_dir(root) + "/" + std::to_string(nodes[i].node);
    std::map<int, bool> peers;
    for (const char* sub : {"io_links", "p2p_links"}) {
      for (int l : numeric_entries(nd + "/" + sub)) {
        Props lp = read_props(nd + "/" + sub + "/" + std::to_string(l) + "/properties");
        // count every xGMI peer, including GPU nodes this container cannot
        // read (a 1-GPU slice of an 8-GPU hive still shows 7 xGMI links)
        if (get(lp, "type") == AT_LINK_XGMI && (int)get(lp, "node_to") != nodes[i].node) peers[(int)get(lp, "node_to")] = true;
      }
    }
    gpus[i].num_xgmi_links = (uint32_t)peers.size();
  }

  *count = (int)gpus.size();
  if ((int)gpus.size() > max) {
    if (out) std::copy(gpus.begin(), gpus.begin() + max, out);
    return max == 0 ? AT_OK : AT_ERR_NOSPC;
  }
  std::copy(gpus.begin(), gpus.end(), out);
  return AT_OK;
}

AT_API int at_links(const char* root, at_link_t* out, int max, int* count) {
  if (!count || max < 0 || (max > 0 && !out)) return AT_ERR_INVAL;
  std::vector<KfdNode> nodes = gpu_nodes(root);
  std::map<int, int> node_to_idx;
  for (size_t i = 0; i < nodes.size(); ++i) node_to_idx[nodes[i].node] = (int)i;
  std::map<std::pair<int, int>, at_link_t> links;  // de-duplicate io_links vs p2p_links
  for (size_t i = 0; i < nodes.size(); ++i) {
    const std::string nd = topo_dir(root) + "/" + std::to_string(nodes[i].node);
    for (const char* sub : {"io_links", "p2p_links"}) {
      for (int l : numeric_entries(nd + "/" + sub)) {
        Props lp = read_props(nd + "/" + sub + "/" + std::to_string(l) + "/properties");
        auto it = node_to_idx.find((int)get(lp, "node_to"));
        if (it == node_to_idx.end() || it->second == (int)i) continue;
        at_link_t lk;
        lk.from_gpu = (int)i;
        lk.to_gpu = it->second;
        lk.type = (uint32_t)get(lp, "type");
        lk.weight = (uint32_t)get(lp, "weight");
        lk.min_bandwidth_mbps = (uint32_t)get(lp, "min_bandwidth");
        lk.max_bandwidth_mbps = (uint32_t)get(lp, "max_bandwidth");
        auto key = std::make_pair(lk.from_gpu, lk.to_gpu);
        auto ex = links.find(key);
        // prefer the xGMI description of a pair over a PCIe one
        if (ex == links.end() || (ex->second.type != AT_LINK_XGMI && lk.type == AT_LINK_XGMI)) links[key] = lk;
      }
    }
  }
  *count = (int)links.size();
  int i = 0;
  for (auto& kv : links) {
    if (i >= max) return max == 0 ? AT_OK : AT_ERR_NOSPC;
    out[i++] = kv.second;
  }
  return AT_OK;
}

AT_API int at_probe(const char* root, int expect_gpus, char* msg, int msg_len) {
  auto say = [&](const std::string& s, int rc) {
    if (msg && msg_len > 0) copy_str(msg, (size_t)msg_len, s);
    return rc;
  };
  std::string st;
  if (!read_file(join(root, "sys/module/amdgpu/initstate"), &st) || trim(st) != "live")
    return say("amdgpu kernel module not loaded (sys/module/amdgpu/initstate != live)", AT_ERR_NOENT);
  if (!exists(join(root, "dev/kfd"))) return say("/dev/kfd missing", AT_ERR_NOENT);
  std::vector<KfdNode> nodes = gpu_nodes(root);
  if (nodes.empty()) return say("no GPU nodes in KFD topology", AT_ERR_NOENT);
  if (expect_gpus > 0 && (int)nodes.size() < expect_gpus)
    return say("expected " + std::to_string(expect_gpus) + " GPU nodes, found " + std::to_string(nodes.size()), AT_ERR_NOENT);
  // Exact render minors first; a container runtime may re-number the nodes it
  // passes through (KFD minor 184 shows up as renderD128), so fall back to
  // "at least one render node per GPU node".
  size_t exact = 0;
  for (const KfdNode& k : nodes) {
    const unsigned minor = (unsigned)get(k.props, "drm_render_minor");
    if (exists(join(root, "dev/dri/renderD" + std::to_string(minor)))) ++exact;
  }
  if (exact == nodes.size()) return say("ready: " + std::to_string(nodes.size()) + " GPU node(s)", AT_OK);
  size_t any = 0;
  DIR* d = opendir(join(root, "dev/dri").c_str());
  if (d) {
    while (dirent* e = readdir(d)) any += strncmp(e->d_name, "renderD", 7) == 0;
    closedir(d);
  }
  if (any >= nodes.size())
    return say("ready: " + std::to_string(nodes.size()) + " GPU node(s) (render nodes re-numbered by the runtime)", AT_OK);
  return say("render nodes missing: " + std::to_string(any) + " present for " + std::to_string(nodes.size()) + " GPU node(s)",
             AT_ERR_NOENT);
}

}  // extern "C"
