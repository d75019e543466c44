// amd-container-runtime — OCI runtime shim for the containerd `amd` handler (host-only C++17).
//
// The NVIDIA stack the reference deploys uses nvidia-container-runtime: a runc wrapper that edits
// the OCI spec and a prestart hook (libnvidia-container) that mounts /dev/nvidia* plus driver
// libraries according to NVIDIA_VISIBLE_DEVICES (reference gpu-operator/helmrelease.yaml:17-29;
// RuntimeClass `nvidia` in llm/deployment.yaml:21).  ROCm needs no driver libraries from the host
// (the user-space stack lives in the image), so this shim only does device plumbing, and it takes
// the device list from the ONE source a pod cannot forge: the container annotation
// `amd.com/gpu.render-minors` that kubelet copies from the amd.com/gpu device plugin's Allocate
// response (containerd passes it through `container_annotations = ["amd.com/gpu.*"]`; Kubernetes
// has no user-settable container annotations, and pod annotations are not passed).
//
// On `create`/`run` it edits <bundle>/config.json, then execs the real runc with the unchanged
// argv:
//   * linux.devices: /dev/kfd + /dev/dri/renderD<m> for every allocated minor (major/minor from the
//     host device node); every other /dev/dri node is removed unless the container is privileged;
//   * linux.resources.devices: an explicit `allow c major:minor rwm` rule per node (device cgroup);
//   * annotations without the key → the spec is not touched (CPU pods through the same handler).
// Any inconsistency (unparseable minors, missing host node) fails the create loudly instead of
// starting a container without its GPU.
//
//   amd-container-runtime [runc global flags] create --bundle DIR ID      (containerd)
//   amd-container-runtime --amd-edit-bundle DIR                           (print edited spec, no exec)
//   amd-container-runtime --version
//
// Config: /etc/amd-container-runtime/config.json (override: AMD_CONTAINER_RUNTIME_CONFIG)
//   {"runtime": "/usr/local/bin/runc", "fallback_runtimes": [...], "log": "/var/log/...",
//    "annotation_prefix": "amd.com/gpu"}
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "amdk8s_json.h"

namespace {

using amdk8s::json::Value;

const char* kVersion = "amd-container-runtime 0.1.0 (gfx950 / MI355X)";

struct Config {
  std::string runtime = "/usr/local/bin/runc";
  std::vector<std::string> fallbacks = {"/var/lib/rancher/rke2/bin/runc", "/usr/bin/runc",
                                        "/usr/sbin/runc"};
  std::string log;
  std::string prefix = "amd.com/gpu";
};

std::string g_log_path;

void logf(const char* fmt, const std::string& a = "", const std::string& b = "") {
  if (g_log_path.empty()) return;
  FILE* f = std::fopen(g_log_path.c_str(), "a");
  if (!f) return;
  char ts[32];
  std::time_t now = std::time(nullptr);
  std::strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%SZ", std::gmtime(&now));
  std::fprintf(f, "%s [%d] ", ts, (int)getpid());
  std::fprintf(f, fmt, a.c_str(), b.c_str());
  std::fprintf(f, "\n");
  std::fclose(f);
}

bool read_file(const std::string& p, std::string* out) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

Config load_config() {
  Config c;
  const char* env = std::getenv("AMD_CONTAINER_RUNTIME_CONFIG");
  std::string path = env ? env : "/etc/amd-container-runtime/config.json";
  std::string text;
  if (!read_file(path, &text)) return c;
  try {
    Value v = amdk8s::json::parse(text);
    if (const Value* r = v.get("runtime"); r && r->is_str()) c.runtime = r->s;
    if (const Value* l = v.get("log"); l && l->is_str()) c.log = l->s;
    if (const Value* p = v.get("annotation_prefix"); p && p->is_str()) c.prefix = p->s;
    if (const Value* fb = v.get("fallback_runtimes"); fb && fb->is_arr()) {
      c.fallbacks.clear();
      for (const auto& x : *fb->a)
        if (x.is_str()) c.fallbacks.push_back(x.s);
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "amd-container-runtime: ignoring bad config %s: %s\n", path.c_str(), e.what());
  }
  return c;
}

struct DevNode {
  std::string path;
  long long major = 0, minor = 0;
};

bool stat_dev(const std::string& path, DevNode* d, std::string* err) {
  const char* root = std::getenv("AMD_CONTAINER_RUNTIME_DEV_ROOT");  // tests: fabricated /dev
  const std::string host = std::string(root ? root : "") + path;
  struct stat sb;
  if (stat(host.c_str(), &sb) != 0) {
    *err = host + ": " + std::strerror(errno);
    return false;
  }
  d->path = path;
  if (S_ISCHR(sb.st_mode)) {
    d->major = major(sb.st_rdev);
    d->minor = minor(sb.st_rdev);
    return true;
  }
  // Only a fabricated test tree may use regular files: DRM render nodes are char 226:<minor>; the
  // KFD major is dynamic, 241 is what the MI355X test box reported (gpurun_out/facts/dev_nodes.txt).
  if (root && S_ISREG(sb.st_mode)) {
    if (path == "/dev/kfd") {
      d->major = 241;
      d->minor = 0;
    } else {
      d->major = 226;
      d->minor = std::atoll(path.c_str() + path.rfind('D') + 1);
    }
    return true;
  }
  *err = host + " is not a character device";
  return false;
}

bool parse_minors(const std::string& s, std::vector<long long>* out, std::string* err) {
  std::stringstream ss(s);
  std::string tok;
  std::set<long long> seen;
  while (std::getline(ss, tok, ',')) {
    if (tok.empty()) continue;
    char* end = nullptr;
    long long v = std::strtoll(tok.c_str(), &end, 10);
    if (!end || *end != '\0' || v < 0 || v > 1048575) {
      *err = "bad render minor '" + tok + "'";
      return false;
    }
    if (seen.insert(v).second) out->push_back(v);
  }
  if (out->empty()) {
    *err = "empty render-minor list";
    return false;
  }
  return true;
}

bool is_privileged(const Value& spec) {
  const Value* proc = spec.get("process");
  const Value* caps = proc ? proc->get("capabilities") : nullptr;
  const Value* bounding = caps ? caps->get("bounding") : nullptr;
  if (!bounding || !bounding->is_arr()) return false;
  for (const auto& c : *bounding->a)
    if (c.is_str() && c.s == "CAP_SYS_ADMIN") return true;
  return false;
}

Value device_entry(const DevNode& d) {
  Value e = Value::object();
  e.set("path", Value::string(d.path));
  e.set("type", Value::string("c"));
  e.set("major", Value::number(d.major));
  e.set("minor", Value::number(d.minor));
  e.set("fileMode", Value::number(0666));
  e.set("uid", Value::number(0));
  e.set("gid", Value::number(0));
  return e;
}

Value cgroup_rule(const DevNode& d) {
  Value r = Value::object();
  r.set("allow", Value::boolean(true));
  r.set("type", Value::string("c"));
  r.set("major", Value::number(d.major));
  r.set("minor", Value::number(d.minor));
  r.set("access", Value::string("rwm"));
  return r;
}

// Returns 0 = edited, 1 = error, 2 = nothing to do (no GPU annotation).
int edit_spec(Value& spec, const Config& cfg, std::string* err) {
  const Value* ann = spec.get("annotations");
  const Value* minors_v = ann ? ann->get(cfg.prefix + ".render-minors") : nullptr;
  if (!minors_v) return 2;
  if (!minors_v->is_str()) {
    *err = "annotation " + cfg.prefix + ".render-minors is not a string";
    return 1;
  }
  std::vector<long long> minors;
  if (!parse_minors(minors_v->s, &minors, err)) return 1;
  std::vector<DevNode> nodes;
  DevNode kfd;
  if (!stat_dev("/dev/kfd", &kfd, err)) return 1;
  nodes.push_back(kfd);
  for (long long m : minors) {
    DevNode d;
    if (!stat_dev("/dev/dri/renderD" + std::to_string(m), &d, err)) return 1;
    nodes.push_back(d);
  }
  std::set<std::string> wanted;
  for (const auto& n : nodes) wanted.insert(n.path);

  Value& linux_ = spec.ensure("linux", Value::Obj);
  Value& devices = linux_.ensure("devices", Value::Arr);
  const bool privileged = is_privileged(spec);
  Value kept = Value::array();
  for (const auto& d : *devices.a) {
    const Value* p = d.get("path");
    const std::string path = (p && p->is_str()) ? p->s : "";
    if (wanted.count(path)) continue;  // re-added below with host numbers
    if (!privileged && (path.rfind("/dev/dri/", 0) == 0 || path == "/dev/kfd")) continue;
    kept.a->push_back(d);
  }
  for (const auto& n : nodes) kept.a->push_back(device_entry(n));
  devices = kept;

  Value& res = linux_.ensure("resources", Value::Obj);
  Value& rules = res.ensure("devices", Value::Arr);
  for (const auto& n : nodes) {
    bool present = false;
    for (const auto& r : *rules.a) {
      const Value* a = r.get("allow");
      if (a && a->type == Value::Bool && a->b && r.get("major") && r.get("minor") &&
          r.get("major")->as_int(-1) == n.major && r.get("minor")->as_int(-1) == n.minor) {
        present = true;
        break;
      }
    }
    if (!present) rules.a->push_back(cgroup_rule(n));
  }
  return 0;
}

int edit_bundle(const std::string& bundle, const Config& cfg, std::string* out_json) {
  const std::string path = bundle + "/config.json";
  std::string text;
  if (!read_file(path, &text)) {
    std::fprintf(stderr, "amd-container-runtime: cannot read %s: %s\n", path.c_str(), std::strerror(errno));
    return 1;
  }
  Value spec;
  try {
    spec = amdk8s::json::parse(text);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "amd-container-runtime: %s: %s\n", path.c_str(), e.what());
    return 1;
  }
  std::string err;
  const int rc = edit_spec(spec, cfg, &err);
  if (rc == 1) {
    std::fprintf(stderr, "amd-container-runtime: refusing to create container: %s\n", err.c_str());
    logf("create %s FAILED: %s", bundle, err);
    return 1;
  }
  if (rc == 2) {
    if (out_json) *out_json = text;
    logf("create %s: no %s annotation, spec unchanged", bundle, cfg.prefix);
    return 0;
  }
  const std::string edited = amdk8s::json::dump(spec);
  if (out_json) {
    *out_json = edited;
    return 0;
  }
  struct stat sb;
  const mode_t mode = stat(path.c_str(), &sb) == 0 ? (sb.st_mode & 07777) : 0644;
  const std::string tmp = path + ".amd.tmp";
  int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, mode);
  if (fd < 0 || write(fd, edited.data(), edited.size()) != (ssize_t)edited.size() || fsync(fd) != 0 ||
      close(fd) != 0 || rename(tmp.c_str(), path.c_str()) != 0) {
    std::fprintf(stderr, "amd-container-runtime: cannot write %s: %s\n", path.c_str(), std::strerror(errno));
    unlink(tmp.c_str());
    return 1;
  }
  logf("create %s: injected GPU devices for %s", bundle, spec.get("annotations")->get(cfg.prefix + ".render-minors")->s);
  return 0;
}

// runc global flags that take a value (must be skipped when looking for the subcommand)
bool global_flag_takes_value(const std::string& a) {
  return a == "--root" || a == "--log" || a == "--log-format" || a == "--criu" || a == "--rootless";
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && std::strcmp(argv[1], "--version") == 0) {
    std::printf("%s\n", kVersion);
    return 0;
  }
  Config cfg = load_config();
  g_log_path = cfg.log;
  if (argc >= 3 && std::strcmp(argv[1], "--amd-edit-bundle") == 0) {
    std::string out;
    const int rc = edit_bundle(argv[2], cfg, &out);
    if (rc == 0) std::printf("%s\n", out.c_str());
    return rc;
  }
  // locate the subcommand and, for create/run, the bundle
  int sub = -1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.rfind("--", 0) == 0 || a.rfind("-", 0) == 0) {
      if (a.find('=') == std::string::npos && global_flag_takes_value(a)) ++i;
      continue;
    }
    sub = i;
    break;
  }
  if (sub > 0 && (std::strcmp(argv[sub], "create") == 0 || std::strcmp(argv[sub], "run") == 0)) {
    std::string bundle = ".";
    for (int i = sub + 1; i < argc; ++i) {
      std::string a = argv[i];
      if ((a == "--bundle" || a == "-b") && i + 1 < argc) {
        bundle = argv[i + 1];
        break;
      }
      if (a.rfind("--bundle=", 0) == 0) {
        bundle = a.substr(9);
        break;
      }
    }
    if (edit_bundle(bundle, cfg, nullptr) != 0) return 1;
  }
  std::vector<std::string> candidates = {cfg.runtime};
  candidates.insert(candidates.end(), cfg.fallbacks.begin(), cfg.fallbacks.end());
  std::vector<char*> args(argv, argv + argc);
  args.push_back(nullptr);
  for (const auto& rt : candidates) {
    if (access(rt.c_str(), X_OK) != 0) continue;
    args[0] = const_cast<char*>(rt.c_str());
    execv(rt.c_str(), args.data());
    logf("execv %s failed: %s", rt, std::strerror(errno));
  }
  std::fprintf(stderr, "amd-container-runtime: no executable runtime among %s and fallbacks\n",
               cfg.runtime.c_str());
  return 127;
}
