// amdgpu-oci-hook (N2): container-toolkit runtime integration for MI355X.
//
// Reference parity: the container-toolkit DaemonSet "installs the tools a
// container runtime (Docker, containerd) needs to use the GPU"
// (/root/reference/README.md:105,203,210).  Upstream that is
// nvidia-container-runtime + libnvidia-container; here there is NO runtime shim
// (BASELINE.json north star).  The runtime integration modes, all in this
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
//             Idempotent.  For tools that prepare a bundle before `create`.
//   precreate hooks.d "precreate" stage (CRI-O, podman): the runtime spec on
//             stdin, the edited spec on stdout - the same edits as `apply`,
//             made before the OCI runtime loads the spec, so they take effect.
//   prestart  hooks.d / config.json "prestart" stage: the runtime has already
//             loaded the spec, so editing config.json would change nothing.
//             Reads the container state (pid, bundle) on stdin, selects the
//             devices from the bundle's (read-only) config.json, then creates
//             the device nodes inside the container (/proc/<pid>/root/dev) and
//             allows them in its cgroup-v1 device controller.  On cgroup v2
//             device access is an eBPF program the runtime attached at create
//             time, which a hook cannot extend: it fails and names precreate /
//             CDI instead of starting a container without its GPUs.
//
// Which devices: --devices, else the device plugin's volume-mounts list
// (/dev/null bind mounts at /var/run/amd-container-devices/<sel>, with
// --accept-volume-mounts), else the container's AMD_VISIBLE_DEVICES env (set
// by the device plugin's Allocate) or the amd.com/gpu.devices annotation.
// With --envvar-privileged-only the env AND the annotation are honoured only
// for containers holding CAP_SYS_ADMIN: runtimes copy pod annotations into the
// container spec, so an unprivileged pod must not name GPUs through either.
//
// Device selectors: "all", "none"/"void", or a comma list of indices into the
// enumeration order, PCI BDFs ("0000:a4:00.0") or KFD unique ids ("0x...").

#include <fcntl.h>
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

const char* kVersion = "amdgpu-oci-hook 0.2.0";

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
  bool envvar_privileged_only = false;  // env / annotation only from CAP_SYS_ADMIN containers
  std::string proc_root = "/proc";      // prestart: /proc/<pid>/{root,cgroup} (tests: a fake tree)
  std::string cgroup_root = "/sys/fs/cgroup";
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

// Devices the container asked for (see the header for the precedence).
std::string requested(const Opts& o, const mj::Value& spec) {
  if (!o.devices.empty()) return o.devices;
  std::string sel;
  if (o.accept_volume_mounts) sel = volume_mount_list(spec);
  if (!sel.empty()) return sel;
  const bool trusted = !o.envvar_privileged_only || privileged(spec);
  if (!trusted) return "";
  sel = env_lookup(spec, "AMD_VISIBLE_DEVICES");
  if (sel.empty()) {
    const mj::Value* ann = spec.find("annotations");
    const mj::Value* a = ann ? ann->find("amd.com/gpu.devices") : nullptr;
    if (a && a->is_string()) sel = a->str();
  }
  return sel;
}

// /dev/kfd plus the selected render nodes; false (with *err) on a bad selector.
bool plan_devices(const Opts& o, const mj::Value& spec, std::vector<DevNode>* nodes, std::string* injected,
                  std::string* err) {
  nodes->clear();
  injected->clear();
  std::vector<at_gpu_t> gpus = enumerate(o);
  std::vector<int> idx;
  if (!select(gpus, requested(o, spec), &idx, err)) return false;
  if (idx.empty()) return true;  // not a GPU container
  DevNode kfd;
  if (!kfd_node(o, &kfd)) {
    *err = "cannot resolve /dev/kfd";
    return false;
  }
  nodes->push_back(kfd);
  for (int i : idx) {
    DevNode rn;
    render_node(o, gpus[i], &rn);
    nodes->push_back(rn);
    *injected += (injected->empty() ? "" : ",") + std::to_string(i);
  }
  return true;
}

// Spec edits shared by `apply` and `precreate`; *changed = false for a non-GPU container.
bool edit_spec(const Opts& o, mj::Value& spec, bool* changed, std::string* err) {
  *changed = false;
  if (!spec.is_object()) {
    *err = "runtime spec is not an object";
    return false;
  }
  std::vector<DevNode> nodes;
  std::string injected;
  if (!plan_devices(o, spec, &nodes, &injected, err)) return false;
  if (nodes.empty()) return true;
  for (const DevNode& d : nodes) add_device(spec, d);
  if (o.mount_rocm) add_mount(spec, o.rocm_dir);
  set_env(spec, "AMD_VISIBLE_DEVICES", injected);
  spec["annotations"]["amd.com/gpu.injected"] = injected;
  *changed = true;
  return true;
}

bool parse_json(const std::string& text, const std::string& what, mj::Value* out) {
  try {
    *out = mj::parse(text);
  } catch (const std::exception& e) {
    fprintf(stderr, "amdgpu-oci-hook: %s: %s\n", what.c_str(), e.what());
    return false;
  }
  return true;
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
  if (!parse_json(text, cfg_path, &spec)) return 1;
  bool changed = false;
  std::string err;
  if (!edit_spec(o, spec, &changed, &err)) {
    fprintf(stderr, "amdgpu-oci-hook: %s\n", err.c_str());
    return 1;
  }
  if (!changed) {
    if (o.dry_run) printf("{\"devices\": []}\n");
    return 0;  // not a GPU container: leave the spec untouched
  }
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

// hooks.d precreate: spec in on stdin, (edited) spec out on stdout - always
// the whole spec, unchanged for a non-GPU container.
int cmd_precreate(const Opts& o) {
  std::stringstream ss;
  ss << std::cin.rdbuf();
  mj::Value spec;
  if (!parse_json(ss.str(), "runtime spec on stdin", &spec)) return 1;
  bool changed = false;
  std::string err;
  if (!edit_spec(o, spec, &changed, &err)) {
    fprintf(stderr, "amdgpu-oci-hook: %s\n", err.c_str());
    return 1;
  }
  const std::string out = spec.dump(2) + "\n";
  if (fwrite(out.data(), 1, out.size(), stdout) != out.size() || fflush(stdout) != 0) {
    fprintf(stderr, "amdgpu-oci-hook: cannot write the spec to stdout\n");
    return 1;
  }
  return 0;
}

// The container's device cgroup from /proc/<pid>/cgroup: "v1:<path>" for a
// cgroup-v1 devices hierarchy, "v2:<path>" for the unified hierarchy.
std::string device_cgroup(const Opts& o, long pid) {
  std::string text;
  if (!read_file(join(o.proc_root, std::to_string(pid) + "/cgroup"), &text)) return "";
  std::stringstream ss(text);
  std::string line, v2;
  while (std::getline(ss, line)) {
    const size_t a = line.find(':'), b = a == std::string::npos ? a : line.find(':', a + 1);
    if (b == std::string::npos) continue;
    const std::string ctrls = line.substr(a + 1, b - a - 1), path = line.substr(b + 1);
    std::stringstream cs(ctrls);
    std::string c;
    while (std::getline(cs, c, ','))
      if (c == "devices") return "v1:" + path;
    if (line.compare(0, 3, "0::") == 0) v2 = "v2:" + path;
  }
  return v2;
}

// Create the character device `rel` (e.g. "/dev/dri/renderD128") inside the
// container whose root directory is `rootfs` (/proc/<pid>/root), as host
// root, without following anything the container controls.  A pod volume or
// image can hold symlinks at /dev, /dev/dri or the node's own name that point
// at host paths (absolute links resolve against the hook's root, the host's):
// every directory component is opened with O_NOFOLLOW relative to the one
// before it, the node is made with mknodat in the final directory, and an
// existing entry is accepted only if it is already that char device.  The
// mode is set through the verified O_PATH descriptor, never by path.
bool make_device_node(const std::string& rootfs, const std::string& rel, unsigned major, unsigned minor,
                      std::string* why) {
  int dfd = open(rootfs.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);  // the magic link itself is followed
  if (dfd < 0) return *why = std::string("open container root: ") + strerror(errno), false;
  std::vector<std::string> parts;
  std::stringstream ss(rel);
  for (std::string p; std::getline(ss, p, '/');)
    if (!p.empty()) parts.push_back(p);
  if (parts.empty()) return close(dfd), *why = "empty device path", false;
  for (size_t i = 0; i + 1 < parts.size(); ++i) {
    const std::string& p = parts[i];
    if (p == "." || p == "..") return close(dfd), *why = "path component " + p, false;
    if (mkdirat(dfd, p.c_str(), 0755) != 0 && errno != EEXIST)
      return *why = "mkdir " + p + ": " + strerror(errno), close(dfd), false;
    const int next = openat(dfd, p.c_str(), O_PATH | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
    const int e = errno;
    close(dfd);
    if (next < 0)
      return *why = p + (e == ELOOP || e == ENOTDIR ? " is a symlink or not a directory: refused"
                                                     : std::string(": ") + strerror(e)), false;
    dfd = next;
  }
  const std::string& leaf = parts.back();
  const dev_t want = makedev(major, minor);
  if (mknodat(dfd, leaf.c_str(), S_IFCHR | 0666, want) != 0 && errno != EEXIST)
    return *why = std::string("mknod: ") + strerror(errno), close(dfd), false;
  const int nfd = openat(dfd, leaf.c_str(), O_PATH | O_NOFOLLOW | O_CLOEXEC);
  close(dfd);
  struct stat st;
  if (nfd < 0 || fstat(nfd, &st) != 0 || !S_ISCHR(st.st_mode) || st.st_rdev != want) {
    if (nfd >= 0) close(nfd);
    return *why = "an existing entry is not char device " + std::to_string(major) + ":" + std::to_string(minor) +
                  ": refused", false;
  }
  // chmod through the descriptor (fchmod does not take O_PATH fds)
  const std::string via = "/proc/self/fd/" + std::to_string(nfd);
  const int rc = chmod(via.c_str(), 0666);
  const int e = errno;
  close(nfd);
  if (rc != 0) return *why = std::string("chmod: ") + strerror(e), false;
  return true;
}

// hooks.d / config.json prestart: act on the created container (see header).
int cmd_prestart(Opts o) {
  std::stringstream ss;
  ss << std::cin.rdbuf();
  mj::Value st;
  if (!parse_json(ss.str(), "OCI state on stdin", &st)) return 1;
  const mj::Value* b = st.find("bundle");
  const mj::Value* p = st.find("pid");
  if (!b || !b->is_string()) {
    fprintf(stderr, "amdgpu-oci-hook: OCI state has no bundle\n");
    return 1;
  }
  if (!p || !p->is_number() || p->num() <= 0) {
    fprintf(stderr, "amdgpu-oci-hook: OCI state has no container pid\n");
    return 1;
  }
  const long pid = (long)p->num();
  std::string text;
  const std::string cfg_path = b->str() + "/config.json";
  mj::Value spec;
  if (!read_file(cfg_path, &text) || !parse_json(text, cfg_path, &spec)) {
    fprintf(stderr, "amdgpu-oci-hook: cannot read %s\n", cfg_path.c_str());
    return 1;
  }
  std::vector<DevNode> nodes;
  std::string injected, err;
  if (!spec.is_object() || !plan_devices(o, spec, &nodes, &injected, &err)) {
    fprintf(stderr, "amdgpu-oci-hook: %s\n", err.empty() ? "config.json is not an object" : err.c_str());
    return 1;
  }
  if (nodes.empty()) {
    if (o.dry_run) printf("{\"devices\": []}\n");
    return 0;
  }
  const std::string cg = device_cgroup(o, pid);
  if (cg.compare(0, 3, "v1:") != 0) {
    fprintf(stderr,
            "amdgpu-oci-hook: container %ld is not in a cgroup-v1 devices hierarchy (%s): a prestart hook cannot grant "
            "device access; install the hook at the precreate stage or use CDI (amd.com/gpu=<id>)\n",
            pid, cg.empty() ? "no cgroup" : cg.c_str());
    return 1;
  }
  const std::string rootfs = join(o.proc_root, std::to_string(pid) + "/root");
  const std::string allow = join(join(o.cgroup_root, "devices"), cg.substr(3)) + "/devices.allow";
  mj::Value plan = mj::Value::object();
  mj::Value mk = mj::Value::array(), rules = mj::Value::array();
  for (const DevNode& d : nodes) {
    mj::Value m = mj::Value::object();
    m["path"] = join(rootfs, d.path);
    m["major"] = d.major;
    m["minor"] = d.minor;
    mk.push(m);
    rules.push("c " + std::to_string(d.major) + ":" + std::to_string(d.minor) + " rwm");
  }
  plan["mknod"] = mk;
  plan["devices.allow"] = allow;
  plan["rules"] = rules;
  plan["injected"] = injected;
  if (o.dry_run) {
    fputs((plan.dump(2) + "\n").c_str(), stdout);
    return 0;
  }
  // cgroup first: a node the container cannot open is useless, and a failed
  // write must not leave half-made device nodes behind
  for (const mj::Value& r : rules.arr()) {
    std::ofstream f(allow, std::ios::app);  // one rule per write(2), as cgroupfs wants
    if (!f || !(f << r.str()) || !f.flush()) {
      fprintf(stderr, "amdgpu-oci-hook: cannot write '%s' to %s: %s\n", r.str().c_str(), allow.c_str(),
              strerror(errno));
      return 1;
    }
  }
  for (const DevNode& d : nodes) {
    std::string why;
    if (!make_device_node(rootfs, d.path, d.major, d.minor, &why)) {
      fprintf(stderr, "amdgpu-oci-hook: %s%s: %s\n", rootfs.c_str(), d.path.c_str(), why.c_str());
      return 1;
    }
  }
  return 0;
}

void usage() {
  fprintf(stderr,
          "usage: amdgpu-oci-hook {cdi|apply|precreate|prestart|--version} [--root DIR] [--bundle DIR]\n"
          "                       [--devices SEL] [--output FILE] [--rocm-dir DIR] [--mount-rocm] [--kind KIND]\n"
          "                       [--dry-run] [--accept-volume-mounts] [--envvar-privileged-only]\n"
          "                       [--proc-root DIR] [--cgroup-root DIR]\n");
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
    else if (a == "--proc-root") ok = next(&o.proc_root);
    else if (a == "--cgroup-root") ok = next(&o.cgroup_root);
    else ok = false;
    if (!ok) {
      usage();
      return 2;
    }
  }
  if (cmd == "cdi") return cmd_cdi(o);
  if (cmd == "apply") return cmd_apply(o);
  if (cmd == "precreate") return cmd_precreate(o);
  if (cmd == "prestart") return cmd_prestart(o);
  usage();
  return 2;
}
