// Shared logic of amd-container-runtime / amd-container-hook / amd-ctk: which
// GPUs a container asked for, which device nodes that means, and how to edit an
// OCI runtime spec (config.json) to grant them.
//
// AMD GPU access inside a container needs only device nodes -- /dev/kfd plus one
// /dev/dri/renderD<minor> (and optionally card<k>) per GPU -- the ROCm user space
// ships in the image.  This is the AMD analog of what libnvidia-container does with
// driver-library mounts, reduced to devices + cgroup + groups.
#pragma once
#include <string>
#include <vector>

#include "../common/json.hpp"
#include "../topo/amdgpu_topo.hpp"

namespace amdctr {

struct DevNode {
  std::string path;      // path inside the container (== host path)
  char type = 'c';
  long major = 0, minor = 0;
  unsigned mode = 0666;
};

// Requested GPUs from the OCI spec: env AMD_VISIBLE_DEVICES (also accepts
// ROCR_VISIBLE_DEVICES-style lists) or the annotation "amd.com/gpu.devices".
// Returns "" when the container asked for nothing.
std::string requested_spec(const kgcjson::Value& config);

// "all" | "none" | "void" | comma list of: index, index range a-b, unique id
// (0x...), PCI BDF.  Throws std::runtime_error on an unknown device.
std::vector<int> select_gpus(const std::string& spec, const amdgpu_topo::Topology& topo);

// Device nodes for the selected GPUs (+ /dev/kfd), stat()ed under `root`.  With a
// fake root, majors/minors come from <root>/dev/.kgc_devices ("path major minor").
std::vector<DevNode> device_nodes(const std::vector<int>& gpus, const amdgpu_topo::Topology& topo,
                                  const std::string& root, bool with_card = true);

// gid of a group from <root>/etc/group, -1 if absent.
long group_gid(const std::string& root, const std::string& name);

// Edit the spec: linux.devices (dedupe by path), linux.resources.devices allow
// rules, process.user.additionalGids (render, video), env AMD_VISIBLE_DEVICES
// normalised to the granted indices.  Returns the number of device nodes added.
int inject(kgcjson::Value& config, const std::vector<DevNode>& nodes,
           const std::vector<long>& gids, const std::vector<int>& gpus);

std::string read_file(const std::string& path);
void write_file_atomic(const std::string& path, const std::string& data);

}  // namespace amdctr
