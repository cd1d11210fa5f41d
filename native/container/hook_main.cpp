// amd-container-hook: OCI hook (hooks.d, stage prestart / createRuntime) for
// runtimes started without the amd-container-runtime shim (e.g. plain crun with
// CRI-O hooks_dir, podman).  Reads the OCI state on stdin, loads the bundle's
// config.json and, when the container requested GPUs, creates the missing device
// nodes inside the container rootfs (mknod, mode 0666) and reports what it did.
//
// The rootfs /dev of a container is a tmpfs mounted in the CONTAINER's mount namespace,
// so a node created from the runtime's namespace lands underneath that mount, invisible.
// For prestart / createRuntime the hook therefore enters the mount namespace of the
// container process (state.pid, /proc/<pid>/ns/mnt, setns CLONE_NEWNS) before mknod,
// as libnvidia-container does.  createContainer hooks already run in that namespace.
// In both cases pivot_root has not happened yet, so the nodes go to <rootfs>/dev/....
// Device-cgroup access must still be granted by the runtime (the device plugin's
// DeviceSpecs under Kubernetes, or the shim); the hook never edits cgroups.
//
// Counterpart of the reference's oci-nvidia-hook.json prestart hook
// (gpu-crio-setup.sh:114-126).
//   amd-container-hook prestart [--root DIR] [--proc DIR] [--dry-run]  (state JSON on stdin)
#include <fcntl.h>
#include <sched.h>
#include <sys/stat.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <iterator>
#include <string>

#include "devices.hpp"

static int mkdirs(const std::string& p) {
  for (size_t i = 1; i < p.size(); ++i)
    if (p[i] == '/') { ::mkdir(p.substr(0, i).c_str(), 0755); }
  return ::mkdir(p.c_str(), 0755) == 0 || errno == EEXIST ? 0 : -1;
}

int main(int argc, char** argv) {
  std::string stage = argc > 1 ? argv[1] : "prestart";
  std::string root = "/", proc = "/proc";
  bool dry = false;
  for (int i = 2; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--dry-run")) dry = true;
    else if (!std::strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
    else if (!std::strcmp(argv[i], "--proc") && i + 1 < argc) proc = argv[++i];
  }
  if (stage != "prestart" && stage != "createRuntime" && stage != "createContainer") {
    std::fprintf(stderr, "amd-container-hook: unsupported stage %s\n", stage.c_str());
    return 2;
  }
  try {
    std::string state((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
    kgcjson::Value st = kgcjson::parse(state);
    const std::string bundle = st.get("bundle") ? st.get("bundle")->as_str() : "";
    if (bundle.empty()) throw std::runtime_error("state has no bundle");
    kgcjson::Value cfg = kgcjson::parse(amdctr::read_file(bundle + "/config.json"));
    const std::string spec = amdctr::requested_spec(cfg);
    if (spec.empty()) return 0;                      // not a GPU container
    const auto topo = amdgpu_topo::enumerate(root);
    const auto gpus = amdctr::select_gpus(spec, topo);
    const auto nodes = amdctr::device_nodes(gpus, topo, root);
    std::string rootfs = "rootfs";
    if (const kgcjson::Value* r = cfg.get("root"))
      if (const kgcjson::Value* p = r->get("path")) rootfs = p->as_str();
    if (rootfs[0] != '/') rootfs = bundle + "/" + rootfs;
    // all topology/sysfs reads are done: switch to the container's mount namespace
    const kgcjson::Value* pidv = st.get("pid");
    const long pid = pidv ? (long)pidv->as_int(0) : 0;
    if (stage != "createContainer") {
      if (pid <= 0) throw std::runtime_error("state has no pid: cannot reach the container /dev");
      const std::string ns = proc + "/" + std::to_string(pid) + "/ns/mnt";
      if (dry) {
        std::printf("setns %s\n", ns.c_str());
      } else {
        const int fd = ::open(ns.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) throw std::runtime_error("open " + ns + ": " + std::strerror(errno));
        const int rc = ::setns(fd, CLONE_NEWNS);
        const int err = errno;
        ::close(fd);
        if (rc != 0) throw std::runtime_error("setns " + ns + ": " + std::strerror(err));
      }
    }
    for (auto& n : nodes) {
      const std::string dst = rootfs + n.path;
      struct stat sb;
      if (::stat(dst.c_str(), &sb) == 0) continue;
      if (dry) {
        std::printf("mknod %s c %ld %ld\n", dst.c_str(), n.major, n.minor);
        continue;
      }
      mkdirs(dst.substr(0, dst.rfind('/')));
      if (::mknod(dst.c_str(), S_IFCHR | n.mode, makedev(n.major, n.minor)) != 0)
        throw std::runtime_error("mknod " + dst + ": " + std::strerror(errno));
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "amd-container-hook: %s\n", e.what());
    return 1;
  }
  return 0;
}
