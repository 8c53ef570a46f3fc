// gate_chain.hip -- probe: what a chain of gated (immediately returning) kernels costs after a long
// kernel on the same stream, launched one by one vs replayed from a captured HIP graph, at the
// general path's grid sizes and at small grids. Answers whether the transform's device verdict
// (ambrycrc_put.cpp: ~23 gated launches behind *xfail) would gain from a graph.
// Build: hipcc -O3 --offload-arch=gfx950 -o gate_chain tools/probes/gate_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void busy(float* x, int iters) {
  float v = x[blockIdx.x * blockDim.x + threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 1.000001f + 0.5f;
  x[blockIdx.x * blockDim.x + threadIdx.x] = v;
}
__global__ void gated(const unsigned* gate, unsigned* out) {
  if (*gate == 0) return;
  out[blockIdx.x * blockDim.x + threadIdx.x] = 1;
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(r_), __LINE__); exit(1); } } while (0)

int main() {
  const int K = 23, reps = 20;
  float* x; unsigned *gate, *out;
  CK(hipMalloc(&x, 1 << 24)); CK(hipMalloc(&gate, 4)); CK(hipMalloc(&out, 64 << 20));
  CK(hipMemset(x, 0, 1 << 24)); CK(hipMemset(gate, 0, 4));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grids[2] = {1024, 32};
  for (int gi = 0; gi < 2; ++gi) {
    const int grid = grids[gi];
    // busy kernel alone
    float t_busy = 0, t_chain = 0, t_graph = 0;
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(busy, dim3(4096), dim3(1024), 0, s, x, 2000);
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) t_busy += ms;
    }
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(busy, dim3(4096), dim3(1024), 0, s, x, 2000);
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(gated, dim3(grid), dim3(256), 0, s, gate, out);
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) t_chain += ms;
    }
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(gated, dim3(grid), dim3(256), 0, s, gate, out);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < reps + 2; ++r) {
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(busy, dim3(4096), dim3(1024), 0, s, x, 2000);
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) t_graph += ms;
    }
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    printf("{\"grid\": %d, \"kernels\": %d, \"busy_us\": %.1f, \"chain_extra_us\": %.1f, \"graph_extra_us\": %.1f}\n", grid, K,
           1000 * t_busy / reps, 1000 * (t_chain - t_busy) / reps, 1000 * (t_graph - t_busy) / reps);
  }
  return 0;
}
