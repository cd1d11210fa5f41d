// libamdgpu-topo implementation (see amdgpu_topo.hpp).
#include "amdgpu_topo.hpp"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#include "../common/json.hpp"

namespace amdgpu_topo {
namespace {

std::string join(const std::string& a, const std::string& b) {
  if (a.empty() || a == "/") return b;
  return a + b;
}

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

std::string read_file(const std::string& p) {
  std::ifstream f(p);
  if (!f) return "";
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

std::vector<std::string> list_dir(const std::string& p) {
  std::vector<std::string> out;
  DIR* d = opendir(p.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    out.emplace_back(e->d_name);
  }
  closedir(d);
  return out;
}

bool is_num(const std::string& s) {
  return !s.empty() && std::all_of(s.begin(), s.end(), [](char c) { return isdigit((unsigned char)c); });
}

std::map<std::string, uint64_t> read_props(const std::string& p) {
  std::map<std::string, uint64_t> m;
  std::istringstream in(read_file(p));
  std::string k;
  uint64_t v;
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    if (ls >> k >> v) m[k] = v;
  }
  return m;
}

uint64_t get(const std::map<std::string, uint64_t>& m, const char* k, uint64_t d = 0) {
  auto it = m.find(k);
  return it == m.end() ? d : it->second;
}

// "ue: 3\nce: 10" -> uncorrectable count
long ras_ue(const std::string& text) {
  auto pos = text.find("ue:");
  if (pos == std::string::npos) return 0;
  return std::strtol(text.c_str() + pos + 3, nullptr, 10);
}

}  // namespace

std::string gfx_name(uint32_t v) {
  // gfx_target_version = major*10000 + minor*100 + stepping, printed as gfx<maj><min><step hex>
  const uint32_t maj = v / 10000, min = (v / 100) % 100, step = v % 100;
  char b[32];
  snprintf(b, sizeof b, "gfx%u%u%x", maj, min, step);
  return b;
}

Topology enumerate(const std::string& root_in) {
  Topology t;
  t.root = root_in.empty() ? "/" : root_in;
  const std::string root = root_in == "/" ? "" : root_in;
  const std::string base = join(root, "/sys/class/kfd/kfd/topology/nodes");
  t.kfd_present = exists(base) && exists(join(root, "/dev/kfd"));
  std::vector<int> ids;
  for (auto& n : list_dir(base))
    if (is_num(n)) ids.push_back(std::stoi(n));
  std::sort(ids.begin(), ids.end());
  std::map<int, int> node_to_index;
  for (int id : ids) {
    const std::string nd = base + "/" + std::to_string(id);
    const auto props = read_props(nd + "/properties");
    const uint64_t gpu_id = std::strtoull(read_file(nd + "/gpu_id").c_str(), nullptr, 10);
    if (gpu_id == 0 || get(props, "simd_count") == 0) continue;   // CPU agent
    Gpu g;
    g.index = (int)t.gpus.size();
    g.node_id = id;
    g.gpu_id = (uint32_t)gpu_id;
    g.render_minor = (int)get(props, "drm_render_minor", (uint64_t)-1);
    g.unique_id = get(props, "unique_id");
    g.gfx = gfx_name((uint32_t)get(props, "gfx_target_version"));
    g.vendor_id = (uint32_t)get(props, "vendor_id");
    g.device_id = (uint32_t)get(props, "device_id");
    g.simd_count = (int)get(props, "simd_count");
    g.num_xcc = (int)get(props, "num_xcc", 1);
    g.cu_count = g.simd_count / std::max<uint64_t>(1, get(props, "simd_per_cu", 4));
    g.hive_id = get(props, "hive_id");
    const uint64_t loc = get(props, "location_id"), dom = get(props, "domain");
    char b[32];
    snprintf(b, sizeof b, "%04llx:%02llx:%02llx.%llx", (unsigned long long)dom,
             (unsigned long long)((loc >> 8) & 0xff), (unsigned long long)((loc >> 3) & 0x1f),
             (unsigned long long)(loc & 7));
    g.bdf = b;
    for (auto& mb : list_dir(nd + "/mem_banks")) {
      const auto mp = read_props(nd + "/mem_banks/" + mb + "/properties");
      if (get(mp, "heap_type") <= 1) g.vram_bytes += get(mp, "size_in_bytes");
    }
    const std::string numa = read_file(join(root, "/sys/bus/pci/devices/" + g.bdf + "/numa_node"));
    g.numa_node = numa.empty() ? -1 : std::atoi(numa.c_str());
    if (g.render_minor >= 0) {
      const std::string drm = join(root, "/sys/class/drm/renderD" + std::to_string(g.render_minor) +
                                             "/device/drm");
      for (auto& e : list_dir(drm))
        if (e.rfind("card", 0) == 0 && is_num(e.substr(4))) g.card = std::stoi(e.substr(4));
    }
    // health: device node present and no uncorrectable RAS errors
    if (g.render_minor < 0 || !exists(join(root, "/dev/dri/renderD" + std::to_string(g.render_minor)))) {
      g.healthy = false;
      g.health_reason = "render node missing";
    } else if (g.card >= 0) {
      const std::string ras = join(root, "/sys/class/drm/card" + std::to_string(g.card) + "/device/ras");
      for (auto& f : list_dir(ras)) {
        if (f.size() > 10 && f.compare(f.size() - 10, 10, "_err_count") == 0) {
          const long ue = ras_ue(read_file(ras + "/" + f));
          if (ue > 0) {
            g.healthy = false;
            g.health_reason = f + " ue=" + std::to_string(ue);
          }
        }
      }
    }
    node_to_index[id] = g.index;
    t.gpus.push_back(g);
  }
  // xGMI links and partition grouping
  for (auto& g : t.gpus) {
    const std::string ld = base + "/" + std::to_string(g.node_id) + "/io_links";
    for (auto& l : list_dir(ld)) {
      const auto lp = read_props(ld + "/" + l + "/properties");
      if (get(lp, "type") != 11) continue;             // CRAT io-link type XGMI
      auto it = node_to_index.find((int)get(lp, "node_to"));
      if (it != node_to_index.end() && it->second != g.index) g.xgmi_peers.push_back(it->second);
    }
    std::sort(g.xgmi_peers.begin(), g.xgmi_peers.end());
  }
  std::map<uint64_t, std::vector<int>> by_uid;
  for (auto& g : t.gpus)
    if (g.unique_id) by_uid[g.unique_id].push_back(g.index);
  for (auto& kv : by_uid)
    for (size_t k = 0; k < kv.second.size(); ++k) {
      t.gpus[kv.second[k]].partition = (int)k;
      t.gpus[kv.second[k]].partitions = (int)kv.second.size();
    }
  return t;
}

std::string to_json(const Topology& t, int indent) {
  using kgcjson::Value;
  Value root = Value::object();
  root.set("root", Value::str(t.root));
  root.set("kfd_present", Value::boolean(t.kfd_present));
  Value arr = Value::array();
  for (auto& g : t.gpus) {
    Value o = Value::object();
    o.set("index", Value::integer(g.index));
    o.set("node_id", Value::integer(g.node_id));
    o.set("gpu_id", Value::integer(g.gpu_id));
    o.set("render_minor", Value::integer(g.render_minor));
    o.set("card", Value::integer(g.card));
    o.set("pci_bdf", Value::str(g.bdf));
    char u[32];
    snprintf(u, sizeof u, "0x%016llx", (unsigned long long)g.unique_id);
    o.set("unique_id", Value::str(u));
    o.set("gfx", Value::str(g.gfx));
    o.set("vendor_id", Value::integer(g.vendor_id));
    o.set("device_id", Value::integer(g.device_id));
    o.set("simd_count", Value::integer(g.simd_count));
    o.set("cu_count", Value::integer(g.cu_count));
    o.set("num_xcc", Value::integer(g.num_xcc));
    o.set("vram_bytes", Value::integer((int64_t)g.vram_bytes));
    o.set("numa_node", Value::integer(g.numa_node));
    snprintf(u, sizeof u, "0x%016llx", (unsigned long long)g.hive_id);
    o.set("hive_id", Value::str(u));
    o.set("partition", Value::integer(g.partition));
    o.set("partitions", Value::integer(g.partitions));
    Value peers = Value::array();
    for (int p : g.xgmi_peers) peers.push(Value::integer(p));
    o.set("xgmi_peers", peers);
    o.set("healthy", Value::boolean(g.healthy));
    o.set("health_reason", Value::str(g.health_reason));
    arr.push(o);
  }
  root.set("gpus", arr);
  return kgcjson::dump(root, indent);
}

}  // namespace amdgpu_topo

extern "C" int kgc_topo_json(const char* root, char** out) {
  try {
    const std::string s = amdgpu_topo::to_json(amdgpu_topo::enumerate(root ? root : ""), 0);
    *out = static_cast<char*>(std::malloc(s.size() + 1));
    std::memcpy(*out, s.c_str(), s.size() + 1);
    return 0;
  } catch (...) {
    *out = nullptr;
    return 1;
  }
}

extern "C" void kgc_topo_free(char* p) { std::free(p); }
