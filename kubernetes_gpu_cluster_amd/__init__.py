"""MI355X-native Kubernetes GPU-cluster LLM serving stack.

Sub-packages: ``models`` (Llama/Qwen/OPT/Mixtral), ``ops`` (gfx950 HIP kernels +
reference oracles), ``parallel`` (TP/PP/EP over RCCL/xGMI), ``engine`` (paged KV,
continuous batching, hipGraph decode), ``entrypoints`` (OpenAI API), ``router``,
``k8s`` (amd.com/gpu device plugin, values renderer), ``utils``.
"""
__version__ = "0.1.0"
