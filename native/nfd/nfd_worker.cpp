// N8: amdgpu-nfd - the node-feature-discovery worker as a native process.
//
// The NFD worker is the first operand of every bring-up: the operator learns
// which nodes have GPUs from its labels, so its start-up is on the
// time-to-Ready critical path of every node (the reference deploys NFD for the
// same reason, /root/reference/README.md:107,209).  As a Python operand it
// spent ~0.1 s in interpreter start and imports before its first sysfs read;
// this binary reaches the API server a few milliseconds after exec.
//
// What it does (the same labels as amdgpu_operator/discovery/labels.py
// nfd_labels, checked against it by tests/test_nfd_native.py):
//
//   feature.node.kubernetes.io/pci-<class4>_<vendor>.present = true  (every PCI function)
//   feature.node.kubernetes.io/pci-1002.present              = true  (AMD display / accelerator)
//   feature.node.kubernetes.io/kernel-loadedmodule.amdgpu    = true  (module live)
//   feature.node.kubernetes.io/kernel-version.full           = <release>
//   feature.node.kubernetes.io/rdma.capable / rdma.available  = true  (RDMA device / ib_uverbs + rdma_ucm)
//
// then GET the Node, and PATCH (merge patch) only what differs: new labels,
// stale ones it owns (pci-*, the amdgpu module label) removed, and the
// nfd.amd.com/scanned annotation the operator waits for.  It rescans every
// --interval seconds until SIGTERM (--oneshot: once).
//
// API access: in a pod, the service-account token and CA
// (KUBERNETES_SERVICE_HOST, HTTPS through OpenSSL, server certificate
// verified); outside, a JSON kubeconfig (KUBECONFIG: server, token,
// certificate-authority[-data], insecure-skip-tls-verify).  Readiness: the
// AMDGPU_READY_FILE protocol of the Python operands (<file>.started at main,
// <file> after the first successful sync).
#include <arpa/inet.h>
#include <dirent.h>
#include <fcntl.h>
#include <netdb.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/utsname.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../hook/json.hpp"

namespace {

const char* kPrefix = "feature.node.kubernetes.io/";
const char* kScannedAnn = "nfd.amd.com/scanned";  // amdgpu_operator/wellknown.py NFD_SCANNED_ANN
const char* kAmdVendor = "1002";
const char* kGpuClasses[] = {"1200", "0380", "0300"};  // processing accelerator, display, VGA

volatile sig_atomic_t g_stop = 0;
int g_wake[2] = {-1, -1};  // self-pipe: SIGTERM ends the interval sleep at once

void on_signal(int) {
  g_stop = 1;
  if (g_wake[1] >= 0) {
    char c = 1;
    ssize_t r = write(g_wake[1], &c, 1);
    (void)r;
  }
}

double now() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void log_line(const char* level, const std::string& msg) {
  std::string esc;
  for (char c : msg) {
    if (c == '"' || c == '\\') esc += '\\';
    esc += (c == '\n') ? ' ' : c;
  }
  fprintf(stderr, "{\"ts\": %.3f, \"level\": \"%s\", \"logger\": \"amdgpu.nfd\", \"msg\": \"%s\"}\n", now(), level,
          esc.c_str());
  fflush(stderr);
}

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

// Kubernetes label value: <= 63 chars of [A-Za-z0-9_.-], alphanumeric at both ends
std::string label_value(const std::string& v) {
  std::string s;
  for (char c : v) s += (isalnum((unsigned char)c) || c == '_' || c == '.' || c == '-') ? c : '-';
  if (s.size() > 63) s.resize(63);
  size_t a = s.find_first_not_of("-_."), b = s.find_last_not_of("-_.");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

std::string join(const std::string& root, const std::string& rel) {
  std::string r = root.empty() ? "/" : root;
  if (r.back() == '/') r.pop_back();
  return r + "/" + rel;
}

std::map<std::string, std::string> scan(const std::string& root) {
  std::map<std::string, std::string> labels;
  const std::string pci = join(root, "sys/bus/pci/devices");
  std::vector<std::string> devs;
  if (DIR* d = opendir(pci.c_str())) {
    while (dirent* e = readdir(d))
      if (e->d_name[0] != '.') devs.push_back(e->d_name);
    closedir(d);
  }
  for (const auto& dev : devs) {
    std::string vendor, cls;
    if (!read_file(pci + "/" + dev + "/vendor", &vendor) || !read_file(pci + "/" + dev + "/class", &cls)) continue;
    vendor = lower(trim(vendor));
    cls = lower(trim(cls));
    if (vendor.rfind("0x", 0) == 0) vendor = vendor.substr(2);
    if (cls.rfind("0x", 0) == 0) cls = cls.substr(2);
    if (vendor.empty() || cls.empty()) continue;
    while (cls.size() < 6) cls = "0" + cls;
    const std::string cls4 = cls.substr(0, 4);
    labels[std::string(kPrefix) + "pci-" + cls4 + "_" + vendor + ".present"] = "true";
    if (vendor == kAmdVendor)
      for (const char* g : kGpuClasses)
        if (cls4 == g) labels[std::string(kPrefix) + "pci-" + kAmdVendor + ".present"] = "true";
  }
  std::string state;
  if (read_file(join(root, "sys/module/amdgpu/initstate"), &state) && trim(state) == "live")
    labels[std::string(kPrefix) + "kernel-loadedmodule.amdgpu"] = "true";
  // NFD's rdma feature: an RDMA device present / the user-space RDMA modules loaded
  if (DIR* d = opendir(join(root, "sys/class/infiniband").c_str())) {
    bool any = false;
    while (dirent* e = readdir(d))
      if (e->d_name[0] != '.') any = true;
    closedir(d);
    if (any) labels[std::string(kPrefix) + "rdma.capable"] = "true";
  }
  struct stat st;
  if (stat(join(root, "sys/module/ib_uverbs").c_str(), &st) == 0 && S_ISDIR(st.st_mode) &&
      stat(join(root, "sys/module/rdma_ucm").c_str(), &st) == 0 && S_ISDIR(st.st_mode))
    labels[std::string(kPrefix) + "rdma.available"] = "true";
  std::string rel;
  if (!read_file(join(root, "proc/sys/kernel/osrelease"), &rel) || trim(rel).empty()) {
    struct utsname u;  // a container shares the node's kernel
    rel = uname(&u) == 0 ? u.release : "";
  }
  rel = label_value(trim(rel));
  if (!rel.empty()) labels[std::string(kPrefix) + "kernel-version.full"] = rel;
  return labels;
}

bool owned(const std::string& key) {
  const std::string p(kPrefix);
  return key.rfind(p + "pci-", 0) == 0 || key == p + "kernel-loadedmodule.amdgpu" || key.rfind(p + "rdma.", 0) == 0;
}

// ---------------------------------------------------------------- API access

struct Endpoint {
  bool tls = false;
  std::string host;
  std::string port;
  std::string token;
  std::string ca_file;
  std::string ca_pem;  // certificate-authority-data, decoded
  bool insecure = false;
};

std::string b64decode(const std::string& in) {
  static const std::string tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  int val = 0, bits = -8;
  for (char c : in) {
    size_t p = tbl.find(c);
    if (p == std::string::npos) continue;
    val = ((val << 6) + (int)p) & 0xffffff;
    bits += 6;
    if (bits >= 0) {
      out += (char)((val >> bits) & 0xff);
      bits -= 8;
    }
  }
  return out;
}

bool parse_server(const std::string& url, Endpoint* ep, std::string* err) {
  std::string rest;
  if (url.rfind("https://", 0) == 0) {
    ep->tls = true;
    rest = url.substr(8);
  } else if (url.rfind("http://", 0) == 0) {
    rest = url.substr(7);
  } else {
    *err = "unsupported server URL " + url;
    return false;
  }
  rest = rest.substr(0, rest.find('/'));
  size_t colon = rest.rfind(':');
  if (!rest.empty() && rest[0] == '[') {  // [v6]:port
    size_t close = rest.find(']');
    ep->host = rest.substr(1, close - 1);
    ep->port = close + 1 < rest.size() && rest[close + 1] == ':' ? rest.substr(close + 2) : "";
  } else if (colon != std::string::npos) {
    ep->host = rest.substr(0, colon);
    ep->port = rest.substr(colon + 1);
  } else {
    ep->host = rest;
  }
  if (ep->port.empty()) ep->port = ep->tls ? "443" : "80";
  return true;
}

const mj::Value* named(const mj::Value& doc, const char* list, const std::string& name, const char* field) {
  const mj::Value* arr = doc.find(list);
  if (!arr || !arr->is_array()) return nullptr;
  for (const auto& e : arr->arr()) {
    const mj::Value* n = e.find("name");
    if (n && n->is_string() && (name.empty() || n->str() == name)) return e.find(field);
  }
  return nullptr;
}

bool endpoint_from_env(Endpoint* ep, std::string* err) {
  const char* kc = getenv("KUBECONFIG");
  const char* host = getenv("KUBERNETES_SERVICE_HOST");
  if (host && *host && !(kc && *kc)) {  // in a pod: the service account
    const char* port = getenv("KUBERNETES_SERVICE_PORT");
    ep->tls = true;
    ep->host = host;
    ep->port = port && *port ? port : "443";
    const std::string sa = "/var/run/secrets/kubernetes.io/serviceaccount/";
    if (!read_file(sa + "token", &ep->token)) {
      *err = "no service-account token at " + sa + "token";
      return false;
    }
    ep->token = trim(ep->token);
    ep->ca_file = sa + "ca.crt";
    return true;
  }
  if (!(kc && *kc)) {
    *err = "neither KUBERNETES_SERVICE_HOST (in a pod) nor KUBECONFIG is set";
    return false;
  }
  std::string text;
  if (!read_file(kc, &text)) {
    *err = std::string("cannot read kubeconfig ") + kc;
    return false;
  }
  mj::Value doc;
  try {
    doc = mj::parse(text);
  } catch (const std::exception& e) {
    *err = std::string("kubeconfig ") + kc + " is not JSON (" + e.what() + "); YAML kubeconfigs: use the Python operand";
    return false;
  }
  std::string ctx_name;
  if (const mj::Value* c = doc.find("current-context"); c && c->is_string()) ctx_name = c->str();
  const mj::Value* ctx = named(doc, "contexts", ctx_name, "context");
  std::string cluster_name, user_name;
  if (ctx) {
    if (const mj::Value* v = ctx->find("cluster"); v && v->is_string()) cluster_name = v->str();
    if (const mj::Value* v = ctx->find("user"); v && v->is_string()) user_name = v->str();
  }
  const mj::Value* cluster = named(doc, "clusters", cluster_name, "cluster");
  const mj::Value* server = cluster ? cluster->find("server") : nullptr;
  if (!server || !server->is_string()) {
    *err = "kubeconfig has no cluster server";
    return false;
  }
  if (!parse_server(server->str(), ep, err)) return false;
  if (const mj::Value* v = cluster->find("certificate-authority"); v && v->is_string()) ep->ca_file = v->str();
  if (const mj::Value* v = cluster->find("certificate-authority-data"); v && v->is_string())
    ep->ca_pem = b64decode(v->str());
  if (const mj::Value* v = cluster->find("insecure-skip-tls-verify"); v && v->is_bool()) ep->insecure = v->boolean();
  if (const mj::Value* user = named(doc, "users", user_name, "user")) {
    if (const mj::Value* v = user->find("token"); v && v->is_string()) ep->token = v->str();
    if (const mj::Value* v = user->find("tokenFile"); v && v->is_string() && read_file(v->str(), &ep->token))
      ep->token = trim(ep->token);
    if (user->find("client-certificate") || user->find("client-certificate-data")) {
      *err = "client-certificate kubeconfig users are not supported by amdgpu-nfd (use a token)";
      return false;
    }
  }
  return true;
}

class Conn {
 public:
  ~Conn() { close(); }

  bool open(const Endpoint& ep, std::string* err) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_socktype = SOCK_STREAM;
    int rc = getaddrinfo(ep.host.c_str(), ep.port.c_str(), &hints, &res);
    if (rc != 0) {
      *err = "resolve " + ep.host + ": " + gai_strerror(rc);
      return false;
    }
    for (addrinfo* a = res; a; a = a->ai_next) {
      fd_ = socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC, a->ai_protocol);
      if (fd_ < 0) continue;
      if (connect(fd_, a->ai_addr, a->ai_addrlen) == 0) break;
      ::close(fd_);
      fd_ = -1;
    }
    freeaddrinfo(res);
    if (fd_ < 0) {
      *err = "connect " + ep.host + ":" + ep.port + ": " + strerror(errno);
      return false;
    }
    timeval tv{10, 0};  // a stuck API server fails the request, the loop retries
    setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    if (!ep.tls) return true;
    ctx_ = SSL_CTX_new(TLS_client_method());
    if (!ctx_) return ssl_fail("SSL_CTX_new", err);
    SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
    if (!ep.insecure) {
      SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
      bool loaded = false;
      if (!ep.ca_file.empty()) loaded = SSL_CTX_load_verify_locations(ctx_, ep.ca_file.c_str(), nullptr) == 1;
      if (!ep.ca_pem.empty()) {
        BIO* bio = BIO_new_mem_buf(ep.ca_pem.data(), (int)ep.ca_pem.size());
        X509_STORE* store = SSL_CTX_get_cert_store(ctx_);
        while (X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr)) {
          loaded |= X509_STORE_add_cert(store, x) == 1;
          X509_free(x);
        }
        BIO_free(bio);
        ERR_clear_error();
      }
      if (!loaded && SSL_CTX_set_default_verify_paths(ctx_) != 1) return ssl_fail("CA certificates", err);
    }
    ssl_ = SSL_new(ctx_);
    SSL_set_fd(ssl_, fd_);
    SSL_set_tlsext_host_name(ssl_, ep.host.c_str());
    if (!ep.insecure) {  // the API server's certificate must name the host we dialled
      X509_VERIFY_PARAM* p = SSL_get0_param(ssl_);
      in6_addr a6;
      in_addr a4;
      if (inet_pton(AF_INET, ep.host.c_str(), &a4) == 1 || inet_pton(AF_INET6, ep.host.c_str(), &a6) == 1)
        X509_VERIFY_PARAM_set1_ip_asc(p, ep.host.c_str());
      else
        X509_VERIFY_PARAM_set1_host(p, ep.host.c_str(), 0);
    }
    if (SSL_connect(ssl_) != 1) return ssl_fail("TLS handshake with " + ep.host, err);
    return true;
  }

  bool send_all(const std::string& s, std::string* err) {
    size_t off = 0;
    while (off < s.size()) {
      int n = ssl_ ? SSL_write(ssl_, s.data() + off, (int)(s.size() - off))
                   : (int)::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
      if (n <= 0) {
        *err = std::string("send: ") + strerror(errno);
        return false;
      }
      off += (size_t)n;
    }
    return true;
  }

  // the whole response (Connection: close): read to EOF
  bool read_all(std::string* out, std::string* err) {
    char buf[16384];
    for (;;) {
      int n = ssl_ ? SSL_read(ssl_, buf, sizeof buf) : (int)::recv(fd_, buf, sizeof buf, 0);
      if (n > 0) {
        out->append(buf, (size_t)n);
        continue;
      }
      if (n == 0) return true;
      if (ssl_) {
        int e = SSL_get_error(ssl_, n);
        if (e == SSL_ERROR_ZERO_RETURN || (e == SSL_ERROR_SYSCALL && errno == 0)) return true;
      }
      *err = std::string("recv: ") + strerror(errno);
      return false;
    }
  }

  void close() {
    if (ssl_) {
      SSL_shutdown(ssl_);
      SSL_free(ssl_);
      ssl_ = nullptr;
    }
    if (ctx_) {
      SSL_CTX_free(ctx_);
      ctx_ = nullptr;
    }
    if (fd_ >= 0) {
      ::close(fd_);
      fd_ = -1;
    }
  }

 private:
  bool ssl_fail(const std::string& what, std::string* err) {
    unsigned long e = ERR_get_error();
    char buf[256];
    ERR_error_string_n(e, buf, sizeof buf);
    *err = what + ": " + (e ? buf : "failed");
    return false;
  }

  int fd_ = -1;
  SSL_CTX* ctx_ = nullptr;
  SSL* ssl_ = nullptr;
};

std::string dechunk(const std::string& body) {
  std::string out;
  size_t i = 0;
  while (i < body.size()) {
    size_t eol = body.find("\r\n", i);
    if (eol == std::string::npos) break;
    size_t n = strtoul(body.substr(i, eol - i).c_str(), nullptr, 16);
    if (n == 0) break;
    out += body.substr(eol + 2, n);
    i = eol + 2 + n + 2;
  }
  return out;
}

bool request(const Endpoint& ep, const char* method, const std::string& path, const std::string& body,
             const char* ctype, int* status, std::string* resp, std::string* err) {
  Conn c;
  if (!c.open(ep, err)) return false;
  std::string req = std::string(method) + " " + path + " HTTP/1.1\r\nHost: " + ep.host + ":" + ep.port +
                    "\r\nUser-Agent: amdgpu-nfd\r\nAccept: application/json\r\nConnection: close\r\n";
  if (!ep.token.empty()) req += "Authorization: Bearer " + ep.token + "\r\n";
  if (ctype) req += std::string("Content-Type: ") + ctype + "\r\n";
  req += "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
  std::string raw;
  if (!c.send_all(req, err) || !c.read_all(&raw, err)) return false;
  size_t hdr_end = raw.find("\r\n\r\n");
  if (raw.compare(0, 5, "HTTP/") != 0 || hdr_end == std::string::npos) {
    *err = "malformed HTTP response";
    return false;
  }
  *status = atoi(raw.c_str() + raw.find(' ') + 1);
  std::string headers = lower(raw.substr(0, hdr_end));
  *resp = raw.substr(hdr_end + 4);
  if (headers.find("transfer-encoding: chunked") != std::string::npos) *resp = dechunk(*resp);
  return true;
}

std::string jstr(const std::string& s) { return mj::Value(s).dump(0); }

// one scan + GET + (merge) PATCH; returns the number of label changes, -1 on error
int sync_once(const Endpoint& ep, const std::string& node, const std::string& root, std::string* err) {
  const auto desired = scan(root);
  int status = 0;
  std::string body;
  const std::string path = "/api/v1/nodes/" + node;
  if (!request(ep, "GET", path, "", nullptr, &status, &body, err)) return -1;
  if (status != 200) {
    *err = "GET " + path + ": HTTP " + std::to_string(status) + " " + body.substr(0, 200);
    return -1;
  }
  mj::Value obj;
  try {
    obj = mj::parse(body);
  } catch (const std::exception& e) {
    *err = std::string("GET node: ") + e.what();
    return -1;
  }
  std::map<std::string, std::string> cur;
  bool scanned = false;
  if (const mj::Value* md = obj.find("metadata")) {
    if (const mj::Value* l = md->find("labels"); l && l->is_object())
      for (const auto& kv : l->items())
        if (kv.second.is_string()) cur[kv.first] = kv.second.str();
    if (const mj::Value* a = md->find("annotations"); a && a->is_object())
      if (const mj::Value* v = a->find(kScannedAnn); v && v->is_string() && v->str() == "true") scanned = true;
  }
  std::string patch;
  int changes = 0;
  for (const auto& kv : desired)
    if (cur.count(kv.first) == 0 || cur[kv.first] != kv.second) {
      patch += (patch.empty() ? "" : ",") + jstr(kv.first) + ":" + jstr(kv.second);
      ++changes;
    }
  for (const auto& kv : cur)
    if (owned(kv.first) && desired.count(kv.first) == 0) {
      patch += (patch.empty() ? "" : ",") + jstr(kv.first) + ":null";
      ++changes;
    }
  if (changes == 0 && scanned) return 0;
  std::string doc = "{\"metadata\":{\"labels\":{" + patch + "}";
  if (!scanned) doc += ",\"annotations\":{" + jstr(kScannedAnn) + ":\"true\"}";
  doc += "}}";
  if (!request(ep, "PATCH", path, doc, "application/merge-patch+json", &status, &body, err)) return -1;
  if (status != 200) {
    *err = "PATCH " + path + ": HTTP " + std::to_string(status) + " " + body.substr(0, 200);
    return -1;
  }
  return changes;
}

void write_atomic(const std::string& path, const std::string& text) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  if (FILE* f = fopen(tmp.c_str(), "w")) {
    fputs(text.c_str(), f);
    fclose(f);
    rename(tmp.c_str(), path.c_str());
  }
}

// sleep up to `s` seconds; false when a signal asked us to stop
bool pause_for(double s) {
  pollfd p{g_wake[0], POLLIN, 0};
  int rc = poll(&p, 1, (int)(s * 1000));
  (void)rc;
  return !g_stop;
}

int usage() {
  fprintf(stderr,
          "usage: amdgpu-nfd [--interval S] [--oneshot] [--host-root DIR] [--node NAME] [--print]\n"
          "  labels this node's PCI / kernel features (NFD); in a pod via the service account,\n"
          "  else through a JSON KUBECONFIG.  --print: labels as JSON on stdout, no API access.\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  const char* ready = getenv("AMDGPU_READY_FILE");
  if (ready && *ready) write_atomic(std::string(ready) + ".started", std::to_string(now()));
  double interval = 60.0;
  bool oneshot = false, print_only = false;
  const char* hr = getenv("HOST_ROOT");
  std::string root = hr && *hr ? hr : (access("/host/sys", F_OK) == 0 ? "/host" : "/");
  std::string node = getenv("NODE_NAME") ? getenv("NODE_NAME") : "";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--interval" && i + 1 < argc) {
      interval = atof(argv[++i]);
    } else if (a == "--oneshot") {
      oneshot = true;
    } else if (a == "--print") {
      print_only = true;
    } else if (a == "--host-root" && i + 1 < argc) {
      root = argv[++i];
    } else if (a == "--node" && i + 1 < argc) {
      node = argv[++i];
    } else {
      return usage();
    }
  }
  if (print_only) {
    std::string out = "{";
    for (const auto& kv : scan(root)) out += (out.size() > 1 ? ", " : "") + jstr(kv.first) + ": " + jstr(kv.second);
    printf("%s}\n", out.c_str());
    return 0;
  }
  if (node.empty()) {
    log_line("error", "NODE_NAME is not set");
    return 2;
  }
  Endpoint ep;
  std::string err;
  if (!endpoint_from_env(&ep, &err)) {
    log_line("error", err);
    return 1;
  }
  if (pipe2(g_wake, O_CLOEXEC) != 0) return 1;
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);

  bool signalled_ready = false;
  double backoff = 0.05;
  while (!g_stop) {
    int n = sync_once(ep, node, root, &err);
    if (n < 0) {
      log_line("warning", "sync failed: " + err);
      if (!pause_for(backoff)) break;
      backoff = backoff * 2 > 5.0 ? 5.0 : backoff * 2;
      continue;
    }
    backoff = 0.05;
    if (n > 0 || !signalled_ready) log_line("info", "node " + node + " labelled (" + std::to_string(n) + " changes)");
    if (!signalled_ready) {
      signalled_ready = true;
      if (ready && *ready) write_atomic(ready, std::to_string(now()));
    }
    if (oneshot || !pause_for(interval)) break;
  }
  return 0;
}
