// amd-container-runtime: OCI runtime shim for CRI-O / podman.
//
// Registered as a CRI-O runtime handler (amd-ctk runtime configure), it is invoked
// exactly like crun/runc.  On `create` / `run` it reads <bundle>/config.json, and if
// the container requested GPUs (env AMD_VISIBLE_DEVICES or annotation
// amd.com/gpu.devices) injects /dev/kfd + /dev/dri/renderD* (+ card*) device nodes,
// the matching device-cgroup allow rules and the render/video supplementary
// groups, rewrites config.json atomically, then execs the low-level runtime with
// the unchanged argv.  Every other verb is a pass-through exec.
//
// This replaces the reference's nvidia-container-runtime handler
// (old_README.md:1340-1344) without the CDI-vs-hook-vs-default-runtime conflict it
// hit: one mechanism, config.json edited before crun reads it.
//
// Shim-only options (removed from argv before exec):
//   --kgc-dry-run            print the edited config.json, do not exec
//   --kgc-root=DIR           sysfs/dev/etc root (tests)
// Environment: AMD_CONTAINER_RUNTIME_LOWLEVEL (default: first of crun, runc in PATH),
//              AMD_CONTAINER_RUNTIME_LOG (default /var/log/amd-container-runtime.log).
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <string>
#include <vector>

#include "devices.hpp"

namespace {

std::string g_log_path;

void logf(const std::string& msg) {
  if (g_log_path.empty()) return;
  std::ofstream f(g_log_path, std::ios::app);
  if (!f) return;
  char ts[32];
  std::time_t t = std::time(nullptr);
  std::strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%S", std::gmtime(&t));
  f << ts << " amd-container-runtime: " << msg << "\n";
}

std::string find_in_path(const std::string& name) {
  const char* p = std::getenv("PATH");
  std::string path = p ? p : "/usr/local/bin:/usr/bin:/bin";
  size_t s = 0;
  while (s <= path.size()) {
    size_t e = path.find(':', s);
    if (e == std::string::npos) e = path.size();
    const std::string cand = path.substr(s, e - s) + "/" + name;
    if (::access(cand.c_str(), X_OK) == 0) return cand;
    s = e + 1;
  }
  return "";
}

// KEY=VALUE lines of the node defaults file written by gpu-crio-setup.sh (CRI-O starts
// runtimes with its own environment, so the detected crun >= 1.21 path lives here).
std::string node_default(const std::string& key) {
  const char* f = std::getenv("AMD_CONTAINER_RUNTIME_DEFAULTS");
  std::ifstream in(f && *f ? f : "/etc/default/amd-container-runtime");
  std::string line;
  while (std::getline(in, line))
    if (line.rfind(key + "=", 0) == 0) return line.substr(key.size() + 1);
  return "";
}

std::string lowlevel_runtime() {
  if (const char* e = std::getenv("AMD_CONTAINER_RUNTIME_LOWLEVEL"))
    if (*e) return e;
  const std::string d = node_default("AMD_CONTAINER_RUNTIME_LOWLEVEL");
  if (!d.empty() && ::access(d.c_str(), X_OK) == 0) return d;
  for (const char* r : {"crun", "runc"}) {
    const std::string p = find_in_path(r);
    if (!p.empty()) return p;
  }
  return "";
}

}  // namespace

int main(int argc, char** argv) {
  const char* lp = std::getenv("AMD_CONTAINER_RUNTIME_LOG");
  g_log_path = lp ? lp : "/var/log/amd-container-runtime.log";
  bool dry = false;
  std::string root = "/";
  std::vector<std::string> args;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--kgc-dry-run")) dry = true;
    else if (!std::strncmp(argv[i], "--kgc-root=", 11)) root = argv[i] + 11;
    else args.emplace_back(argv[i]);
  }
  // locate the verb (first non-option argument that is a known verb) and --bundle
  std::string verb, bundle;
  static const char* verbs[] = {"create", "run", "start", "delete", "kill", "state", "exec",
                                "pause", "resume", "list", "ps", "update", "spec", "features",
                                "checkpoint", "restore", "events"};
  for (size_t i = 0; i < args.size(); ++i) {
    const std::string& a = args[i];
    if ((a == "--bundle" || a == "-b") && i + 1 < args.size()) bundle = args[i + 1];
    else if (a.rfind("--bundle=", 0) == 0) bundle = a.substr(9);
    if (verb.empty())
      for (const char* v : verbs)
        if (a == v) verb = a;
  }
  if (verb == "create" || verb == "run") {
    if (bundle.empty()) bundle = ".";
    const std::string cfg_path = bundle + "/config.json";
    try {
      kgcjson::Value cfg = kgcjson::parse(amdctr::read_file(cfg_path));
      const std::string spec = amdctr::requested_spec(cfg);
      if (!spec.empty()) {
        const auto topo = amdgpu_topo::enumerate(root);
        const auto gpus = amdctr::select_gpus(spec, topo);
        if (!gpus.empty()) {
          const auto nodes = amdctr::device_nodes(gpus, topo, root);
          std::vector<long> gids = {amdctr::group_gid(root, "render"), amdctr::group_gid(root, "video")};
          const int n = amdctr::inject(cfg, nodes, gids, gpus);
          logf("bundle " + bundle + ": GPUs '" + spec + "' -> " + std::to_string(gpus.size()) +
               " GPU(s), " + std::to_string(n) + " device node(s) injected");
          if (!dry) amdctr::write_file_atomic(cfg_path, kgcjson::dump(cfg, 2));
        }
      }
      if (dry) {
        std::printf("%s\n", kgcjson::dump(cfg, 2).c_str());
        return 0;
      }
    } catch (const std::exception& e) {
      logf(std::string("error: ") + e.what());
      std::fprintf(stderr, "amd-container-runtime: %s\n", e.what());
      return 1;
    }
  } else if (dry) {
    std::printf("{}\n");
    return 0;
  }
  const std::string rt = lowlevel_runtime();
  if (rt.empty()) {
    std::fprintf(stderr, "amd-container-runtime: no low-level runtime (crun/runc) found\n");
    return 127;
  }
  std::vector<char*> av;
  av.push_back(const_cast<char*>(rt.c_str()));
  for (auto& a : args) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  ::execv(rt.c_str(), av.data());
  std::perror("amd-container-runtime: execv");
  return 127;
}
