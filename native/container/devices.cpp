#include "devices.hpp"

#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <stdexcept>

namespace amdctr {

using kgcjson::Value;

std::string read_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw std::runtime_error("cannot read " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

void write_file_atomic(const std::string& path, const std::string& data) {
  const std::string tmp = path + ".kgc.tmp";
  {
    std::ofstream f(tmp, std::ios::trunc);
    if (!f) throw std::runtime_error("cannot write " + tmp);
    f << data;
  }
  if (::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename failed: " + path);
}

static std::string trim(std::string s) {
  while (!s.empty() && isspace((unsigned char)s.back())) s.pop_back();
  size_t i = 0;
  while (i < s.size() && isspace((unsigned char)s[i])) ++i;
  return s.substr(i);
}

std::string requested_spec(const Value& config) {
  if (const Value* proc = config.get("process"))
    if (const Value* env = proc->get("env"))
      if (env->is_arr())
        for (auto& e : *env->a) {
          const std::string s = e.as_str();
          for (const char* key : {"AMD_VISIBLE_DEVICES=", "KGC_VISIBLE_DEVICES="})
            if (s.rfind(key, 0) == 0) return trim(s.substr(strlen(key)));
        }
  if (const Value* ann = config.get("annotations"))
    if (const Value* v = ann->get("amd.com/gpu.devices")) return trim(v->as_str());
  return "";
}

std::vector<int> select_gpus(const std::string& spec_in, const amdgpu_topo::Topology& topo) {
  std::vector<int> out;
  const std::string spec = trim(spec_in);
  if (spec.empty() || spec == "none" || spec == "void") return out;
  const int n = (int)topo.gpus.size();
  if (spec == "all") {
    for (int i = 0; i < n; ++i) out.push_back(i);
    return out;
  }
  std::stringstream ss(spec);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    tok = trim(tok);
    if (tok.empty()) continue;
    bool found = false;
    const auto dash = tok.find('-');
    if (dash != std::string::npos && dash > 0 && std::all_of(tok.begin(), tok.end(), [](char c) {
          return isdigit((unsigned char)c) || c == '-'; })) {
      const int a = std::stoi(tok.substr(0, dash)), b = std::stoi(tok.substr(dash + 1));
      if (a > b || b >= n) throw std::runtime_error("bad GPU range " + tok);
      for (int i = a; i <= b; ++i) out.push_back(i);
      continue;
    }
    if (std::all_of(tok.begin(), tok.end(), [](char c) { return isdigit((unsigned char)c); })) {
      const int i = std::stoi(tok);
      if (i >= n) throw std::runtime_error("GPU index " + tok + " out of range (" + std::to_string(n) + " GPUs)");
      out.push_back(i);
      continue;
    }
    for (auto& g : topo.gpus) {
      char uid[32];
      snprintf(uid, sizeof uid, "0x%016llx", (unsigned long long)g.unique_id);
      std::string low = tok;
      std::transform(low.begin(), low.end(), low.begin(), ::tolower);
      if (low == uid || low == g.bdf || ("gpu-" + std::string(uid + 2)) == low) {
        out.push_back(g.index);
        found = true;
      }
    }
    if (!found) throw std::runtime_error("unknown GPU '" + tok + "'");
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

static std::map<std::string, std::pair<long, long>> fake_devices(const std::string& root) {
  std::map<std::string, std::pair<long, long>> m;
  std::ifstream f(root + "/dev/.kgc_devices");
  std::string p;
  long ma, mi;
  while (f >> p >> ma >> mi) m[p] = {ma, mi};
  return m;
}

std::vector<DevNode> device_nodes(const std::vector<int>& gpus, const amdgpu_topo::Topology& topo,
                                  const std::string& root, bool with_card) {
  std::vector<std::string> paths;
  if (!gpus.empty()) paths.push_back("/dev/kfd");
  for (int i : gpus) {
    const auto& g = topo.gpus.at(i);
    if (g.render_minor >= 0) paths.push_back("/dev/dri/renderD" + std::to_string(g.render_minor));
    if (with_card && g.card >= 0) paths.push_back("/dev/dri/card" + std::to_string(g.card));
  }
  const std::string r = (root == "/" ? "" : root);
  const auto fake = fake_devices(r.empty() ? "/" : r);
  std::vector<DevNode> out;
  for (auto& p : paths) {
    DevNode d;
    d.path = p;
    auto it = fake.find(p);
    if (it != fake.end()) {
      d.major = it->second.first;
      d.minor = it->second.second;
    } else {
      struct stat st;
      if (::stat((r + p).c_str(), &st) != 0) {
        // the DRM card node is optional for compute (ROCm needs /dev/kfd + renderD): a
        // host or container that exposes only render nodes must still get its GPUs
        if (p.rfind("/dev/dri/card", 0) == 0) continue;
        throw std::runtime_error("device node missing: " + r + p);
      }
      if (!S_ISCHR(st.st_mode)) throw std::runtime_error("not a character device: " + r + p);
      d.major = major(st.st_rdev);
      d.minor = minor(st.st_rdev);
    }
    out.push_back(d);
  }
  return out;
}

long group_gid(const std::string& root, const std::string& name) {
  std::ifstream f((root == "/" ? "" : root) + "/etc/group");
  std::string line;
  while (std::getline(f, line)) {
    std::stringstream ss(line);
    std::string n, x, gid;
    std::getline(ss, n, ':');
    std::getline(ss, x, ':');
    std::getline(ss, gid, ':');
    if (n == name && !gid.empty()) return std::stol(gid);
  }
  return -1;
}

int inject(Value& config, const std::vector<DevNode>& nodes, const std::vector<long>& gids,
           const std::vector<int>& gpus) {
  Value& linux_ = config.at("linux");
  Value& devs = linux_.at("devices");
  if (devs.kind == Value::Null) devs = Value::array();
  std::set<std::string> have;
  for (auto& d : *devs.a) have.insert(d.get("path") ? d.get("path")->as_str() : "");
  int added = 0;
  for (auto& n : nodes) {
    if (have.count(n.path)) continue;
    Value d = Value::object();
    d.set("path", Value::str(n.path));
    d.set("type", Value::str(std::string(1, n.type)));
    d.set("major", Value::integer(n.major));
    d.set("minor", Value::integer(n.minor));
    d.set("fileMode", Value::integer(n.mode));
    d.set("uid", Value::integer(0));
    d.set("gid", Value::integer(0));
    devs.push(d);
    ++added;
  }
  Value& rdev = linux_.at("resources").at("devices");
  if (rdev.kind == Value::Null) rdev = Value::array();
  for (auto& n : nodes) {
    bool dup = false;
    for (auto& r : *rdev.a) {
      const Value* ma = r.get("major");
      const Value* mi = r.get("minor");
      if (ma && mi && ma->as_int() == n.major && mi->as_int() == n.minor &&
          r.get("allow") && r.get("allow")->b)
        dup = true;
    }
    if (dup) continue;
    Value rule = Value::object();
    rule.set("allow", Value::boolean(true));
    rule.set("type", Value::str("c"));
    rule.set("major", Value::integer(n.major));
    rule.set("minor", Value::integer(n.minor));
    rule.set("access", Value::str("rwm"));
    rdev.push(rule);
  }
  Value& user = config.at("process").at("user");
  Value& ag = user.at("additionalGids");
  if (ag.kind == Value::Null) ag = Value::array();
  for (long g : gids) {
    if (g < 0) continue;
    bool dup = false;
    for (auto& x : *ag.a) dup |= x.as_int() == g;
    if (!dup) ag.push(Value::integer(g));
  }
  // normalise the visible-device list to the indices granted
  Value& env = config.at("process").at("env");
  if (env.kind == Value::Null) env = Value::array();
  std::string list;
  for (size_t k = 0; k < gpus.size(); ++k) list += (k ? "," : "") + std::to_string(gpus[k]);
  bool set = false;
  for (auto& e : *env.a)
    if (e.as_str().rfind("AMD_VISIBLE_DEVICES=", 0) == 0) { e = Value::str("AMD_VISIBLE_DEVICES=" + list); set = true; }
  if (!set && !gpus.empty()) env.push(Value::str("AMD_VISIBLE_DEVICES=" + list));
  return added;
}

}  // namespace amdctr
