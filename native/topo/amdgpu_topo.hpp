// libamdgpu-topo: enumerate AMD Instinct GPUs (MI355X / gfx950) from the KFD sysfs
// topology, for the amd.com/gpu device plugin and the container tools.
//
// Sources (all under a configurable root so tests can use a fake tree):
//   /sys/class/kfd/kfd/topology/nodes/<n>/{gpu_id,properties}      GPU agents
//   /sys/class/kfd/kfd/topology/nodes/<n>/mem_banks/<b>/properties   VRAM size
//   /sys/class/kfd/kfd/topology/nodes/<n>/io_links/<l>/properties    xGMI peers (type 11)
//   /sys/class/drm/renderD<minor>/device/drm/card<k>                 card index
//   /sys/bus/pci/devices/<bdf>/numa_node                             NUMA affinity
//   /sys/class/drm/card<k>/device/ras/{umc,gfx,...}_err_count        RAS health (ue > 0)
//   /dev/kfd, /dev/dri/renderD<minor>                                device nodes
// Compute partitions (CPX) appear as separate KFD nodes / render nodes and are
// reported as separate devices sharing a unique_id (partition index in order).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace amdgpu_topo {

struct Gpu {
  int index = 0;            // ordinal among GPU agents (HIP/ROCR device order)
  int node_id = 0;          // KFD topology node
  uint32_t gpu_id = 0;
  int render_minor = -1;    // /dev/dri/renderD<minor>
  int card = -1;            // /dev/dri/card<k>
  std::string bdf;          // PCI domain:bus:dev.fn
  uint64_t unique_id = 0;
  std::string gfx;          // e.g. gfx950
  uint32_t vendor_id = 0, device_id = 0;
  int simd_count = 0, num_xcc = 0, cu_count = 0;
  uint64_t vram_bytes = 0;
  int numa_node = -1;
  uint64_t hive_id = 0;
  int partition = 0;        // index among devices sharing unique_id
  int partitions = 1;
  std::vector<int> xgmi_peers;  // indices of GPUs with a direct xGMI link
  bool healthy = true;
  std::string health_reason;
};

struct Topology {
  std::string root;
  bool kfd_present = false;
  std::vector<Gpu> gpus;
};

Topology enumerate(const std::string& root = "");
std::string to_json(const Topology& t, int indent = 2);
std::string gfx_name(uint32_t gfx_target_version);

}  // namespace amdgpu_topo

extern "C" {
// JSON of the topology under `root` ("" = "/"); *out is malloc'd, free with kgc_topo_free.
int kgc_topo_json(const char* root, char** out);
void kgc_topo_free(char* p);
}
