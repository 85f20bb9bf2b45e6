// Captured-graph repair: memset nodes -> fill-kernel nodes.
//
// On this ROCm stack (HIP runtime of ROCm 7.x, MI355X), a hipMemsetAsync
// captured into a hipGraph is correct on the FIRST replay only: from the
// second replay on, buffers of up to at least 16 KB come out with garbage
// (tools/graph_memset_probe.py: memset(buf, 0) -> buf += 1 gives all-ones on
// replay 1, values like INT_MIN and 5 afterwards; a 4 MB memset stays
// correct).  ATen's multi-block reductions zero their semaphore array with
// exactly such a memset, so a reduction replayed from a graph stops writing
// its output — this is what turned the bf16 Linear-bias gradients of the
// captured NewCRF step non-finite (tools/graph_reduce_probe.py).
//
// mde_graph_replace_memsets() rewrites a captured (not yet instantiated)
// graph: every memset node becomes a kernel node that writes the same 2-D
// byte pattern with vector stores, wired to the same dependencies and
// dependents.  GraphTrainer applies it to every graph it captures.
#include <vector>

#include "common.h"

namespace {

// dst[r * pitch + c * elem ...] = value, r < height, c < width (elements of
// 1, 2 or 4 bytes), grid-stride over the width*height elements.
__global__ void __launch_bounds__(256)
    graph_fill_kernel(char* __restrict__ dst, size_t pitch, unsigned value, unsigned elem,
                      size_t width, size_t height) {
  const size_t n = width * height;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / width, c = i - r * width;
    char* p = dst + r * pitch + c * elem;
    if (elem == 4)
      *reinterpret_cast<unsigned*>(p) = value;
    else if (elem == 2)
      *reinterpret_cast<unsigned short*>(p) = (unsigned short)value;
    else
      *p = (char)value;
  }
}

}  // namespace

extern "C" {

int mde_graph_count_memsets(void* graph, int64_t* count) {
  if (!graph || !count) return MDE_ERR_INVALID_ARG;
  hipGraph_t g = (hipGraph_t)graph;
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  if (e != hipSuccess) return (int)e;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && (e = hipGraphGetNodes(g, nodes.data(), &n)) != hipSuccess) return (int)e;
  int64_t k = 0;
  for (hipGraphNode_t node : nodes) {
    hipGraphNodeType t;
    if ((e = hipGraphNodeGetType(node, &t)) != hipSuccess) return (int)e;
    k += t == hipGraphNodeTypeMemset;
  }
  *count = k;
  return MDE_OK;
}

int mde_graph_node_counts(void* graph, int64_t* counts) {
  if (!graph || !counts) return MDE_ERR_INVALID_ARG;
  hipGraph_t g = (hipGraph_t)graph;
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  if (e != hipSuccess) return (int)e;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && (e = hipGraphGetNodes(g, nodes.data(), &n)) != hipSuccess) return (int)e;
  for (int i = 0; i < 6; ++i) counts[i] = 0;
  counts[0] = (int64_t)n;
  for (hipGraphNode_t node : nodes) {
    hipGraphNodeType t;
    if ((e = hipGraphNodeGetType(node, &t)) != hipSuccess) return (int)e;
    switch (t) {
      case hipGraphNodeTypeKernel: ++counts[1]; break;
      case hipGraphNodeTypeMemcpy: ++counts[2]; break;
      case hipGraphNodeTypeMemset: ++counts[3]; break;
      case hipGraphNodeTypeEventRecord:
      case hipGraphNodeTypeWaitEvent: ++counts[4]; break;
      default: ++counts[5]; break;
    }
  }
  return MDE_OK;
}

int mde_graph_node_types(void* graph, int64_t* counts) {
  if (!graph || !counts) return MDE_ERR_INVALID_ARG;
  hipGraph_t g = (hipGraph_t)graph;
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  if (e != hipSuccess) return (int)e;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && (e = hipGraphGetNodes(g, nodes.data(), &n)) != hipSuccess) return (int)e;
  for (int i = 0; i < 16; ++i) counts[i] = 0;
  for (hipGraphNode_t node : nodes) {
    hipGraphNodeType t;
    if ((e = hipGraphNodeGetType(node, &t)) != hipSuccess) return (int)e;
    ++counts[((unsigned)t < 15u) ? (int)t : 15];
  }
  return MDE_OK;
}

int mde_graph_dot(void* graph, const char* path) {
  if (!graph || !path) return MDE_ERR_INVALID_ARG;
  return (int)hipGraphDebugDotPrint((hipGraph_t)graph, path, hipGraphDebugDotFlagsVerbose);
}

int mde_graph_replace_memsets(void* graph, int64_t* replaced) {
  if (!graph) return MDE_ERR_INVALID_ARG;
  hipGraph_t g = (hipGraph_t)graph;
  size_t n = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &n);
  if (e != hipSuccess) return (int)e;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && (e = hipGraphGetNodes(g, nodes.data(), &n)) != hipSuccess) return (int)e;
  int64_t k = 0;
  for (hipGraphNode_t node : nodes) {
    hipGraphNodeType t;
    if ((e = hipGraphNodeGetType(node, &t)) != hipSuccess) return (int)e;
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams p{};
    if ((e = hipGraphMemsetNodeGetParams(node, &p)) != hipSuccess) return (int)e;
    if (p.elementSize != 1 && p.elementSize != 2 && p.elementSize != 4) return MDE_ERR_UNSUPPORTED;
    size_t nd = 0, ndd = 0;
    if ((e = hipGraphNodeGetDependencies(node, nullptr, &nd)) != hipSuccess) return (int)e;
    std::vector<hipGraphNode_t> deps(nd);
    if (nd && (e = hipGraphNodeGetDependencies(node, deps.data(), &nd)) != hipSuccess) return (int)e;
    if ((e = hipGraphNodeGetDependentNodes(node, nullptr, &ndd)) != hipSuccess) return (int)e;
    std::vector<hipGraphNode_t> outs(ndd);
    if (ndd && (e = hipGraphNodeGetDependentNodes(node, outs.data(), &ndd)) != hipSuccess)
      return (int)e;
    char* dst = (char*)p.dst;
    size_t pitch = p.height > 1 ? p.pitch : p.width * p.elementSize;
    unsigned value = p.value, elem = p.elementSize;
    size_t width = p.width, height = p.height ? p.height : 1;
    void* args[] = {&dst, &pitch, &value, &elem, &width, &height};
    const size_t total = width * height;
    size_t blocks = (total + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    hipKernelNodeParams kp{};
    kp.func = reinterpret_cast<void*>(graph_fill_kernel);
    kp.gridDim = dim3((unsigned)blocks);
    kp.blockDim = dim3(256);
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    hipGraphNode_t fill;
    if ((e = hipGraphAddKernelNode(&fill, g, deps.data(), nd, &kp)) != hipSuccess) return (int)e;
    for (hipGraphNode_t o : outs)
      if ((e = hipGraphAddDependencies(g, &fill, &o, 1)) != hipSuccess) return (int)e;
    if ((e = hipGraphDestroyNode(node)) != hipSuccess) return (int)e;
    ++k;
  }
  if (replaced) *replaced = k;
  return MDE_OK;
}

}  // extern "C"
