// KFD topology reader shared by kfd-probe and amd-oci-hook (host-only C++17).
//
// The amdgpu kernel driver publishes one directory per HSA agent under
// /sys/class/kfd/kfd/topology/nodes/<id>/ with a `properties` file of "key value" lines, a
// `gpu_id` file (0 for CPU agents), a `name` file, `mem_banks/<b>/properties` and
// `io_links/<l>/properties`.  This is the AMD counterpart of what NVML gives NVIDIA's device
// plugin; the reference only consumes it indirectly through the GPU operator.
// On MI355X in CPX mode one ASIC shows up as 8 nodes (num_xcc = 1 each) sharing `unique_id`.
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "amdk8s_native.h"

namespace amdk8s {
namespace {

bool read_file(const std::string& path, std::string* out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

std::map<std::string, std::string> parse_props(const std::string& text) {
  std::map<std::string, std::string> m;
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    std::string k, v;
    if (ls >> k >> v) m[k] = v;
  }
  return m;
}

uint64_t to_u64(const std::map<std::string, std::string>& m, const char* key, uint64_t def = 0) {
  auto it = m.find(key);
  if (it == m.end()) return def;
  return std::strtoull(it->second.c_str(), nullptr, 10);
}

std::vector<std::string> list_numeric_dirs(const std::string& path) {
  std::vector<std::string> out;
  DIR* d = opendir(path.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n.empty() || n[0] == '.') continue;
    if (n.find_first_not_of("0123456789") != std::string::npos) continue;
    out.push_back(n);
  }
  closedir(d);
  std::sort(out.begin(), out.end(),
            [](const std::string& a, const std::string& b) { return std::stoi(a) < std::stoi(b); });
  return out;
}

std::string trim(std::string s) {
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ' || s.back() == '\r')) s.pop_back();
  size_t i = 0;
  while (i < s.size() && s[i] == ' ') ++i;
  return s.substr(i);
}

}  // namespace

std::string KfdNode::pci_bdf() const {
  // location_id = (bus << 8) | (device << 3) | function
  char buf[32];
  std::snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", domain, (location_id >> 8) & 0xff,
                (location_id >> 3) & 0x1f, location_id & 0x7);
  return buf;
}

bool read_kfd_topology(const std::string& root, std::vector<KfdNode>* nodes, std::string* err) {
  nodes->clear();
  const std::string nodes_dir = root + "/nodes";
  struct stat sb;
  if (stat(nodes_dir.c_str(), &sb) != 0 || !S_ISDIR(sb.st_mode)) {
    if (err) *err = "no KFD topology at " + nodes_dir + " (amdgpu driver not loaded?)";
    return false;
  }
  for (const std::string& id : list_numeric_dirs(nodes_dir)) {
    const std::string nd = nodes_dir + "/" + id;
    std::string text;
    if (!read_file(nd + "/properties", &text)) {
      if (err) *err = "unreadable " + nd + "/properties";
      return false;
    }
    auto p = parse_props(text);
    KfdNode n;
    n.node_id = std::stoi(id);
    std::string g;
    if (read_file(nd + "/gpu_id", &g)) n.gpu_id = (uint32_t)std::strtoul(trim(g).c_str(), nullptr, 10);
    std::string nm;
    if (read_file(nd + "/name", &nm)) n.name = trim(nm);
    n.gfx_target_version = (uint32_t)to_u64(p, "gfx_target_version");
    n.drm_render_minor = (int)to_u64(p, "drm_render_minor", (uint64_t)-1);
    if (p.find("drm_render_minor") == p.end()) n.drm_render_minor = -1;
    n.unique_id = to_u64(p, "unique_id");
    n.location_id = (uint32_t)to_u64(p, "location_id");
    n.domain = (uint32_t)to_u64(p, "domain");
    n.simd_count = (uint32_t)to_u64(p, "simd_count");
    n.array_count = (uint32_t)to_u64(p, "array_count");
    n.num_xcc = (uint32_t)to_u64(p, "num_xcc", n.simd_count ? 1 : 0);
    n.vendor_id = (uint32_t)to_u64(p, "vendor_id");
    n.device_id = (uint32_t)to_u64(p, "device_id");
    n.max_engine_clk_fcompute = (uint32_t)to_u64(p, "max_engine_clk_fcompute");
    for (const std::string& b : list_numeric_dirs(nd + "/mem_banks")) {
      std::string bt;
      if (!read_file(nd + "/mem_banks/" + b + "/properties", &bt)) continue;
      auto bp = parse_props(bt);
      const uint64_t heap = to_u64(bp, "heap_type");
      if (heap == 1 || heap == 2) n.vram_bytes += to_u64(bp, "size_in_bytes");  // FB public/private
    }
    for (const std::string& l : list_numeric_dirs(nd + "/io_links")) {
      std::string lt;
      if (!read_file(nd + "/io_links/" + l + "/properties", &lt)) continue;
      auto lp = parse_props(lt);
      if (to_u64(lp, "type") == 11) ++n.io_links_xgmi;  // CRAT_IOLINK_TYPE_XGMI
    }
    nodes->push_back(n);
  }
  return true;
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o;
}

}  // namespace amdk8s
