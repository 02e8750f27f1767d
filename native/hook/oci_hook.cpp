// amdgpu-oci-hook (N2): container-toolkit runtime integration for MI355X.
//
// Reference parity: the container-toolkit DaemonSet "installs the tools a
// container runtime (Docker, containerd) needs to use the GPU"
// (/root/reference/README.md:105,203,210).  Upstream that is
// nvidia-container-runtime + libnvidia-container; here there is NO runtime shim
// (BASELINE.json north star).  Two integration paths, both produced by this
// one binary:
//
//   cdi       Generate a CDI spec (kind amd.com/gpu) from the live KFD/DRM
//             topology: one device per GPU (or per compute partition) with its
//             /dev/dri/renderD<N> node, "all", and common edits (/dev/kfd,
//             optional read-only ROCm runtime mount).  containerd >= 1.7 applies
//             it natively when the device plugin returns CDI device names.
//   apply     Edit an OCI bundle's config.json in place: add /dev/kfd and the
//             requested render nodes to linux.devices, allow them in
//             linux.resources.devices, optionally bind-mount ROCm read-only.
//             Idempotent.  Requested devices come from --devices, or the
//             device plugin's volume-mounts list (/dev/null bind mounts at
//             /var/run/amd-container-devices/<sel>, with
//             --accept-volume-mounts), or the container's AMD_VISIBLE_DEVICES
//             env (set by the device plugin's Allocate; with
//             --envvar-privileged-only only for containers holding
//             CAP_SYS_ADMIN, so an unprivileged pod cannot name GPUs it was
//             not allocated), or the amd.com/gpu.devices annotation.
//   prestart  OCI hook entry point: reads the container state JSON on stdin
//             (ociVersion/id/pid/bundle) and runs `apply` on that bundle.
//
// Device selectors: "all", "none"/"void", or a comma list of indices into the
// enumeration order, PCI BDFs ("0000:a4:00.0") or KFD unique ids ("0x...").

#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../include/amdgpu_topo.h"
#include "json.hpp"

namespace {

const char* kVersion = "amdgpu-oci-hook 0.1.0";

struct Opts {
  std::string root = "/";
  std::string bundle;
  std::string devices;  // empty = from the spec
  std::string output;
  std::string rocm_dir = "/opt/rocm";
  std::string kind = "amd.com/gpu";
  bool mount_rocm = false;
  bool dry_run = false;
  bool partitions = true;
  bool accept_volume_mounts = false;   // device list from /var/run/amd-container-devices/<sel> mounts
  bool envvar_privileged_only = false;  // AMD_VISIBLE_DEVICES only from CAP_SYS_ADMIN containers
};

constexpr const char* kDeviceListDir = "/var/run/amd-container-devices/";

std::string join(const std::string& root, const std::string& rel) {
  std::string r = root.empty() ? "/" : root;
  if (r.back() != '/') r += '/';
  return r + (rel.size() && rel[0] == '/' ? rel.substr(1) : rel);
}

bool read_file(const std::string& p, std::string* out) {
  std::ifstream f(p);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

bool write_atomic(const std::string& p, const std::string& data) {
  const std::string tmp = p + ".tmp." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::trunc);
    if (!f) return false;
    f << data;
    if (!f.good()) return false;
  }
  return rename(tmp.c_str(), p.c_str()) == 0;
}

// "major:minor" from a sysfs dev file, else from stat() of the device path
bool dev_numbers(const Opts& o, const std::string& sysfs_dev, const std::string& dev_path, unsigned* maj, unsigned* min) {
  std::string s;
  if (read_file(join(o.root, sysfs_dev), &s)) {
    unsigned a = 0, b = 0;
    if (sscanf(s.c_str(), "%u:%u", &a, &b) == 2) {
      *maj = a;
      *min = b;
      return true;
    }
  }
  struct stat st;
  if (stat(join(o.root, dev_path).c_str(), &st) == 0 && S_ISCHR(st.st_mode)) {
    *maj = major(st.st_rdev);
    *min = minor(st.st_rdev);
    return true;
  }
  return false;
}

struct DevNode {
  std::string path;
  unsigned major = 0, minor = 0;
};

std::vector<at_gpu_t> enumerate(const Opts& o) {
  int n = 0;
  at_enumerate(o.root.c_str(), nullptr, 0, &n);
  std::vector<at_gpu_t> g(n > 0 ? n : 0);
  int cnt = 0;
  if (n > 0) at_enumerate(o.root.c_str(), g.data(), n, &cnt);
  g.resize(cnt);
  return g;
}

bool kfd_node(const Opts& o, DevNode* d) {
  d->path = "/dev/kfd";
  return dev_numbers(o, "sys/class/kfd/kfd/dev", "/dev/kfd", &d->major, &d->minor);
}

bool render_node(const Opts& o, const at_gpu_t& g, DevNode* d) {
  d->path = "/dev/dri/renderD" + std::to_string(g.drm_render_minor);
  if (dev_numbers(o, "sys/class/drm/renderD" + std::to_string(g.drm_render_minor) + "/dev", d->path, &d->major, &d->minor))
    return true;
  d->major = 226;  // DRM major; render minors are the KFD-reported ones
  d->minor = g.drm_render_minor;
  return true;
}

std::string to_lower(std::string s) {
  for (auto& c : s) c = (char)tolower(c);
  return s;
}

// resolve a selector string into enumeration indices; returns false on an unknown id
bool select(const std::vector<at_gpu_t>& gpus, const std::string& sel, std::vector<int>* out, std::string* err) {
  out->clear();
  std::string s = to_lower(sel);
  if (s.empty() || s == "none" || s == "void") return true;
  if (s == "all") {
    for (size_t i = 0; i < gpus.size(); ++i) out->push_back((int)i);
    return true;
  }
  std::set<int> seen;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    while (!tok.empty() && tok.back() == ' ') tok.pop_back();
    while (!tok.empty() && tok.front() == ' ') tok.erase(tok.begin());
    if (tok.empty()) continue;
    int idx = -1;
    bool numeric = !tok.empty() && tok.find_first_not_of("0123456789") == std::string::npos;
    if (numeric) {
      idx = atoi(tok.c_str());
      if (idx < 0 || idx >= (int)gpus.size()) idx = -1;
    } else {
      for (size_t i = 0; i < gpus.size(); ++i) {
        char uid[32];
        snprintf(uid, sizeof(uid), "0x%llx", (unsigned long long)gpus[i].unique_id);
        if (to_lower(gpus[i].bdf) == tok || uid == tok) {
          idx = (int)i;
          break;
        }
      }
    }
    if (idx < 0) {
      *err = "unknown device '" + tok + "'";
      return false;
    }
    if (seen.insert(idx).second) out->push_back(idx);
  }
  return true;
}

mj::Value node_json_cdi(const DevNode& d) {
  mj::Value v = mj::Value::object();
  v["path"] = d.path;
  v["type"] = "c";
  v["major"] = d.major;
  v["minor"] = d.minor;
  v["permissions"] = "rw";
  return v;
}

int cmd_cdi(const Opts& o) {
  std::vector<at_gpu_t> gpus = enumerate(o);
  DevNode kfd;
  if (!kfd_node(o, &kfd)) {
    fprintf(stderr, "amdgpu-oci-hook: cannot resolve /dev/kfd device numbers\n");
    return 1;
  }
  mj::Value spec = mj::Value::object();
  spec["cdiVersion"] = "0.6.0";
  spec["kind"] = o.kind;
  mj::Value devs = mj::Value::array();
  mj::Value all_nodes = mj::Value::array();
  for (size_t i = 0; i < gpus.size(); ++i) {
    DevNode rn;
    render_node(o, gpus[i], &rn);
    mj::Value d = mj::Value::object();
    d["name"] = std::to_string(i);
    mj::Value edits = mj::Value::object();
    mj::Value nodes = mj::Value::array();
    nodes.push(node_json_cdi(rn));
    edits["deviceNodes"] = nodes;
    mj::Value env = mj::Value::array();
    env.push(std::string("AMD_GPU_BDF_") + std::to_string(i) + "=" + gpus[i].bdf);
    edits["env"] = env;
    d["containerEdits"] = edits;
    devs.push(d);
    all_nodes.push(node_json_cdi(rn));
  }
  mj::Value all = mj::Value::object();
  all["name"] = "all";
  mj::Value all_edits = mj::Value::object();
  all_edits["deviceNodes"] = all_nodes;
  all["containerEdits"] = all_edits;
  devs.push(all);
  spec["devices"] = devs;
  mj::Value common = mj::Value::object();
  mj::Value cnodes = mj::Value::array();
  cnodes.push(node_json_cdi(kfd));
  common["deviceNodes"] = cnodes;
  mj::Value env = mj::Value::array();
  env.push("AMD_GPU_OPERATOR_CDI=1");
  common["env"] = env;
  if (o.mount_rocm) {
    mj::Value mounts = mj::Value::array();
    mj::Value m = mj::Value::object();
    m["hostPath"] = o.rocm_dir;
    m["containerPath"] = o.rocm_dir;
    mj::Value opts = mj::Value::array();
    opts.push("ro");
    opts.push("nosuid");
    opts.push("nodev");
    opts.push("rbind");
    m["options"] = opts;
    mounts.push(m);
    common["mounts"] = mounts;
  }
  spec["containerEdits"] = common;
  const std::string text = spec.dump(2) + "\n";
  if (o.output.empty() || o.output == "-") {
    fputs(text.c_str(), stdout);
    return 0;
  }
  if (o.dry_run) {
    fprintf(stdout, "%s", text.c_str());
    return 0;
  }
  if (!write_atomic(o.output, text)) {
    fprintf(stderr, "amdgpu-oci-hook: cannot write %s: %s\n", o.output.c_str(), strerror(errno));
    return 1;
  }
  return 0;
}

std::string env_lookup(const mj::Value& spec, const std::string& key) {
  const mj::Value* proc = spec.find("process");
  if (!proc) return "";
  const mj::Value* env = proc->find("env");
  if (!env || !env->is_array()) return "";
  std::string val;
  bool found = false;
  for (const mj::Value& e : env->arr()) {
    if (!e.is_string()) continue;
    const std::string& s = e.str();
    if (s.compare(0, key.size() + 1, key + "=") == 0) {
      val = s.substr(key.size() + 1);  // last assignment wins, like execve
      found = true;
    }
  }
  return found ? val : "";
}

// Device selectors the device plugin passed as mounts (volume-mounts list
// strategy): destination /var/run/amd-container-devices/<sel>, one per GPU.
std::string volume_mount_list(const mj::Value& spec) {
  const mj::Value* mounts = spec.find("mounts");
  if (!mounts || !mounts->is_array()) return "";
  const std::string dir = kDeviceListDir;
  std::string out;
  for (const mj::Value& m : mounts->arr()) {
    const mj::Value* d = m.is_object() ? m.find("destination") : nullptr;
    if (!d || !d->is_string() || d->str().compare(0, dir.size(), dir) != 0) continue;
    const std::string sel = d->str().substr(dir.size());
    if (sel.empty() || sel.find('/') != std::string::npos) continue;
    out += (out.empty() ? "" : ",") + sel;
  }
  return out;
}

bool privileged(const mj::Value& spec) {
  const mj::Value* proc = spec.find("process");
  const mj::Value* caps = proc ? proc->find("capabilities") : nullptr;
  const mj::Value* bounding = caps ? caps->find("bounding") : nullptr;
  if (!bounding || !bounding->is_array()) return false;
  for (const mj::Value& c : bounding->arr())
    if (c.is_string() && c.str() == "CAP_SYS_ADMIN") return true;
  return false;
}

void add_device(mj::Value& spec, const DevNode& d) {
  mj::Value& linux_ = spec["linux"];
  mj::Value& devs = linux_["devices"];
  if (devs.is_null()) devs = mj::Value::array();
  bool have = false;
  for (const mj::Value& x : devs.arr()) {
    const mj::Value* p = x.find("path");
    if (p && p->is_string() && p->str() == d.path) have = true;
  }
  if (!have) {
    mj::Value v = mj::Value::object();
    v["path"] = d.path;
    v["type"] = "c";
    v["major"] = d.major;
    v["minor"] = d.minor;
    v["fileMode"] = 438;  // 0666
    v["uid"] = 0;
    v["gid"] = 0;
    devs.push(v);
  }
  mj::Value& res = linux_["resources"];
  mj::Value& rules = res["devices"];
  if (rules.is_null()) rules = mj::Value::array();
  bool allowed = false;
  for (const mj::Value& x : rules.arr()) {
    const mj::Value* a = x.find("allow");
    const mj::Value* ma = x.find("major");
    const mj::Value* mi = x.find("minor");
    if (a && a->is_bool() && a->boolean() && ma && mi && ma->is_number() && mi->is_number() &&
        (unsigned)ma->num() == d.major && (unsigned)mi->num() == d.minor)
      allowed = true;
  }
  if (!allowed) {
    mj::Value r = mj::Value::object();
    r["allow"] = true;
    r["type"] = "c";
    r["major"] = d.major;
    r["minor"] = d.minor;
    r["access"] = "rwm";
    rules.push(r);
  }
}

void add_mount(mj::Value& spec, const std::string& dir) {
  mj::Value& mounts = spec["mounts"];
  if (mounts.is_null()) mounts = mj::Value::array();
  for (const mj::Value& m : mounts.arr()) {
    const mj::Value* d = m.find("destination");
    if (d && d->is_string() && d->str() == dir) return;
  }
  mj::Value m = mj::Value::object();
  m["destination"] = dir;
  m["type"] = "bind";
  m["source"] = dir;
  mj::Value opts = mj::Value::array();
  for (const char* x : {"rbind", "ro", "nosuid", "nodev"}) opts.push(x);
  m["options"] = opts;
  mounts.push(m);
}

void set_env(mj::Value& spec, const std::string& key, const std::string& value) {
  mj::Value& proc = spec["process"];
  mj::Value& env = proc["env"];
  if (env.is_null()) env = mj::Value::array();
  for (mj::Value& e : env.arr())
    if (e.is_string() && e.str().compare(0, key.size() + 1, key + "=") == 0) {
      e = mj::Value(key + "=" + value);
      return;
    }
  env.push(key + "=" + value);
}

int cmd_apply(const Opts& o) {
  if (o.bundle.empty()) {
    fprintf(stderr, "amdgpu-oci-hook: --bundle required\n");
    return 2;
  }
  const std::string cfg_path = o.bundle + "/config.json";
  std::string text;
  if (!read_file(cfg_path, &text)) {
    fprintf(stderr, "amdgpu-oci-hook: cannot read %s\n", cfg_path.c_str());
    return 1;
  }
  mj::Value spec;
  try {
    spec = mj::parse(text);
  } catch (const std::exception& e) {
    fprintf(stderr, "amdgpu-oci-hook: %s: %s\n", cfg_path.c_str(), e.what());
    return 1;
  }
  if (!spec.is_object()) {
    fprintf(stderr, "amdgpu-oci-hook: config.json is not an object\n");
    return 1;
  }
  std::string sel = o.devices;
  if (sel.empty() && o.accept_volume_mounts) sel = volume_mount_list(spec);
  if (sel.empty() && (!o.envvar_privileged_only || privileged(spec))) sel = env_lookup(spec, "AMD_VISIBLE_DEVICES");
  if (sel.empty()) {
    const mj::Value* ann = spec.find("annotations");
    const mj::Value* a = ann ? ann->find("amd.com/gpu.devices") : nullptr;
    if (a && a->is_string()) sel = a->str();
  }
  std::vector<at_gpu_t> gpus = enumerate(o);
  std::vector<int> idx;
  std::string err;
  if (!select(gpus, sel, &idx, &err)) {
    fprintf(stderr, "amdgpu-oci-hook: %s\n", err.c_str());
    return 1;
  }
  if (idx.empty()) {
    if (o.dry_run) printf("{\"devices\": []}\n");
    return 0;  // not a GPU container: leave the spec untouched
  }
  DevNode kfd;
  if (!kfd_node(o, &kfd)) {
    fprintf(stderr, "amdgpu-oci-hook: cannot resolve /dev/kfd\n");
    return 1;
  }
  add_device(spec, kfd);
  std::string injected;
  for (int i : idx) {
    DevNode rn;
    render_node(o, gpus[i], &rn);
    add_device(spec, rn);
    injected += (injected.empty() ? "" : ",") + std::to_string(i);
  }
  if (o.mount_rocm) add_mount(spec, o.rocm_dir);
  set_env(spec, "AMD_VISIBLE_DEVICES", injected);
  spec["annotations"]["amd.com/gpu.injected"] = injected;
  const std::string out = spec.dump(2) + "\n";
  if (o.dry_run) {
    fputs(out.c_str(), stdout);
    return 0;
  }
  if (!write_atomic(cfg_path, out)) {
    fprintf(stderr, "amdgpu-oci-hook: cannot write %s: %s\n", cfg_path.c_str(), strerror(errno));
    return 1;
  }
  return 0;
}

int cmd_prestart(Opts o) {
  std::stringstream ss;
  ss << std::cin.rdbuf();
  mj::Value st;
  try {
    st = mj::parse(ss.str());
  } catch (const std::exception& e) {
    fprintf(stderr, "amdgpu-oci-hook: bad OCI state on stdin: %s\n", e.what());
    return 1;
  }
  const mj::Value* b = st.find("bundle");
  if (!b || !b->is_string()) {
    fprintf(stderr, "amdgpu-oci-hook: OCI state has no bundle\n");
    return 1;
  }
  o.bundle = b->str();
  return cmd_apply(o);
}

void usage() {
  fprintf(stderr,
          "usage: amdgpu-oci-hook {cdi|apply|prestart|--version} [--root DIR] [--bundle DIR] [--devices SEL]\n"
          "                       [--output FILE] [--rocm-dir DIR] [--mount-rocm] [--kind KIND] [--dry-run]\n"
          "                       [--accept-volume-mounts] [--envvar-privileged-only]\n");
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    usage();
    return 2;
  }
  std::string cmd = argv[1];
  if (cmd == "--version" || cmd == "version") {
    puts(kVersion);
    return 0;
  }
  Opts o;
  for (int i = 2; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](std::string* dst) {
      if (i + 1 >= argc) return false;
      *dst = argv[++i];
      return true;
    };
    bool ok = true;
    if (a == "--root") ok = next(&o.root);
    else if (a == "--bundle") ok = next(&o.bundle);
    else if (a == "--devices") ok = next(&o.devices);
    else if (a == "--output") ok = next(&o.output);
    else if (a == "--rocm-dir") ok = next(&o.rocm_dir);
    else if (a == "--kind") ok = next(&o.kind);
    else if (a == "--mount-rocm") o.mount_rocm = true;
    else if (a == "--dry-run") o.dry_run = true;
    else if (a == "--accept-volume-mounts") o.accept_volume_mounts = true;
    else if (a == "--envvar-privileged-only") o.envvar_privileged_only = true;
    else ok = false;
    if (!ok) {
      usage();
      return 2;
    }
  }
  if (cmd == "cdi") return cmd_cdi(o);
  if (cmd == "apply") return cmd_apply(o);
  if (cmd == "prestart") return cmd_prestart(o);
  usage();
  return 2;
}
