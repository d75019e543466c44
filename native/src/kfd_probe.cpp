// kfd-probe — amdgpu driver-readiness probe (host-only C++17, no ROCm runtime needed).
//
// The reference's operator builds and loads the NVIDIA kernel module in-cluster and everything
// else waits for it (90 min HelmRelease budget, reference
// cluster-config/apps/gpu-operator/helmrelease.yaml:7; failure mode reference README.md:514-517).
// On MI355X the amdgpu module is inbox/DKMS on the host; the driver DaemonSet only has to prove
// it is up.  This probe is that proof:
//
//   1. the KFD topology lists ≥ --expect-gpus GPU agents (gfx target ≥ --min-gfx, default gfx950)
//   2. /dev/kfd opens read-write
//   3. every GPU agent's /dev/dri/renderD<minor> exists and is a character device
//
// It prints one JSON document (the agents it found) and, with --marker, atomically writes the
// readiness marker that the device plugin and validator init-containers gate on.  --wait polls.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "amdk8s_native.h"

namespace {

struct Options {
  std::string sysfs = "/sys/class/kfd/kfd/topology";
  std::string dev_root = "/dev";
  int expect = 1;
  unsigned min_gfx = 90500;  // gfx950
  int wait_s = 0;
  std::string marker;
  bool quiet = false;
  bool skip_dev_open = false;
};

bool is_chr_or_file(const std::string& p) {
  struct stat sb;
  if (stat(p.c_str(), &sb) != 0) return false;
  return S_ISCHR(sb.st_mode) || S_ISREG(sb.st_mode);  // regular files: fabricated test trees
}

bool check_once(const Options& o, std::string* report, std::string* why) {
  std::vector<amdk8s::KfdNode> nodes;
  std::string err;
  if (!amdk8s::read_kfd_topology(o.sysfs, &nodes, &err)) {
    *why = err;
    return false;
  }
  int gpus = 0;
  bool ok = true;
  std::string js = "[";
  for (const auto& n : nodes) {
    if (!n.is_gpu()) continue;
    const std::string render = o.dev_root + "/dri/renderD" + std::to_string(n.drm_render_minor);
    const bool render_ok = n.drm_render_minor >= 0 && is_chr_or_file(render);
    const bool arch_ok = n.gfx_target_version >= o.min_gfx;
    if (gpus) js += ", ";
    char buf[512];
    std::snprintf(buf, sizeof buf,
                  "{\"node\": %d, \"gpu_id\": %u, \"gfx_target_version\": %u, \"render_minor\": %d, "
                  "\"pci\": \"%s\", \"unique_id\": \"%llu\", \"cu\": %u, \"num_xcc\": %u, "
                  "\"vram_bytes\": %llu, \"xgmi_links\": %u, \"render_ok\": %s, \"arch_ok\": %s}",
                  n.node_id, n.gpu_id, n.gfx_target_version, n.drm_render_minor,
                  n.pci_bdf().c_str(), (unsigned long long)n.unique_id, n.cu_count(), n.num_xcc,
                  (unsigned long long)n.vram_bytes, n.io_links_xgmi, render_ok ? "true" : "false",
                  arch_ok ? "true" : "false");
    js += buf;
    ++gpus;
    if (!render_ok) {
      ok = false;
      *why = "missing render node " + render;
    }
    if (!arch_ok) {
      ok = false;
      *why = "agent " + std::to_string(n.node_id) + " has gfx_target_version " +
             std::to_string(n.gfx_target_version) + " < " + std::to_string(o.min_gfx);
    }
  }
  js += "]";
  if (gpus < o.expect) {
    ok = false;
    *why = "found " + std::to_string(gpus) + " GPU agent(s), expected " + std::to_string(o.expect);
  }
  const std::string kfd = o.dev_root + "/kfd";
  if (!o.skip_dev_open) {
    int fd = open(kfd.c_str(), O_RDWR | O_CLOEXEC);
    if (fd < 0) {
      ok = false;
      *why = kfd + ": " + std::strerror(errno);
    } else {
      close(fd);
    }
  } else if (!is_chr_or_file(kfd)) {
    ok = false;
    *why = "missing " + kfd;
  }
  char head[128];
  std::snprintf(head, sizeof head, "{\"ready\": %s, \"gpus\": %d, \"agents\": ", ok ? "true" : "false",
                gpus);
  *report = std::string(head) + js + ", \"reason\": \"" + amdk8s::json_escape(ok ? "" : *why) + "\"}";
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
      return argv[++i];
    };
    if (a == "--sysfs-root") o.sysfs = next();
    else if (a == "--dev-root") o.dev_root = next();
    else if (a == "--expect-gpus") o.expect = std::atoi(next());
    else if (a == "--min-gfx") o.min_gfx = (unsigned)std::atoi(next());
    else if (a == "--wait") o.wait_s = std::atoi(next());
    else if (a == "--marker") o.marker = next();
    else if (a == "--no-open") o.skip_dev_open = true;
    else if (a == "-q" || a == "--quiet") o.quiet = true;
    else {
      std::printf("usage: kfd-probe [--sysfs-root DIR] [--dev-root DIR] [--expect-gpus N] "
                  "[--min-gfx V] [--wait SEC] [--marker FILE] [--no-open] [-q]\n");
      return a == "-h" || a == "--help" ? 0 : 2;
    }
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(o.wait_s);
  std::string report, why;
  bool ok = false;
  for (;;) {
    ok = check_once(o, &report, &why);
    if (ok || std::chrono::steady_clock::now() >= deadline) break;
    std::this_thread::sleep_for(std::chrono::seconds(2));
  }
  if (!o.quiet) std::printf("%s\n", report.c_str());
  if (!ok) {
    std::fprintf(stderr, "kfd-probe: not ready: %s\n", why.c_str());
    if (!o.marker.empty()) unlink(o.marker.c_str());
    return 1;
  }
  if (!o.marker.empty()) {
    const std::string tmp = o.marker + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "w");
    if (!f || std::fputs(report.c_str(), f) < 0 || std::fclose(f) != 0 ||
        std::rename(tmp.c_str(), o.marker.c_str()) != 0) {
      std::fprintf(stderr, "kfd-probe: cannot write marker %s: %s\n", o.marker.c_str(),
                   std::strerror(errno));
      return 1;
    }
  }
  return 0;
}
