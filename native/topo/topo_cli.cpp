// amdgpu-topo CLI: print the GPU topology as JSON or a table.
//   amdgpu-topo [--root DIR] [--json | --table]
#include <cstdio>
#include <cstring>
#include <string>

#include "amdgpu_topo.hpp"

int main(int argc, char** argv) {
  std::string root;
  bool table = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
    else if (!std::strncmp(argv[i], "--root=", 7)) root = argv[i] + 7;
    else if (!std::strcmp(argv[i], "--table")) table = true;
    else if (!std::strcmp(argv[i], "--json")) table = false;
    else {
      std::fprintf(stderr, "usage: amdgpu-topo [--root DIR] [--json|--table]\n");
      return 2;
    }
  }
  const auto t = amdgpu_topo::enumerate(root);
  if (!table) {
    std::printf("%s\n", amdgpu_topo::to_json(t).c_str());
    return 0;
  }
  std::printf("%-4s %-6s %-14s %-7s %-8s %-6s %-8s %-5s %s\n", "IDX", "NODE", "PCI", "GFX",
              "RENDER", "CARD", "VRAM_GB", "NUMA", "XGMI_PEERS / HEALTH");
  for (auto& g : t.gpus) {
    std::string peers;
    for (int p : g.xgmi_peers) peers += std::to_string(p) + ",";
    std::printf("%-4d %-6d %-14s %-7s %-8d %-6d %-8.1f %-5d [%s] %s%s\n", g.index, g.node_id,
                g.bdf.c_str(), g.gfx.c_str(), g.render_minor, g.card, g.vram_bytes / 1e9,
                g.numa_node, peers.c_str(), g.healthy ? "ok" : "UNHEALTHY ",
                g.health_reason.c_str());
  }
  return 0;
}
