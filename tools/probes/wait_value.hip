// wait_value.hip -- probe: can the transform's device verdict skip the general path's gated launches?
// Round 6. The default transform enqueues ~22 general-path kernels behind a device
// flag; when the fast path took the batch each returns at once, but their dispatches still cost the
// stream ~2 us each. Here the gated chain goes to a side stream forked after the fast kernel, and the
// main stream waits for a completion word instead (hipStreamWaitValue32 on signal memory): set by the
// fast kernel when it took the batch, by the side chain's last kernel otherwise. Prints, per form, the
// time from the fast kernel's start to the next kernel's end on the main stream (median of 51):
//   chain    the product's form: 22 gated kernels on the main stream
//   side     the chain on a side stream, main waits on the word (the fast path took the batch)
//   side_g   the same with the general path taken (the side chain does work; main waits for it)
//   none     the fast kernel alone (the floor)
//   memset2  none, after two 8-B hipMemsetAsync (the transform's resets of its control words)
//   write2   none, after two hipStreamWriteValue64 of 0 instead
//   memset1  none, after one 16-B hipMemsetAsync
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probes/wait_value tools/probes/wait_value.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(e)                                                                        \
  do {                                                                               \
    hipError_t r_ = (e);                                                             \
    if (r_ != hipSuccess) {                                                          \
      printf("HIP error %s at %d\n", hipGetErrorString(r_), __LINE__);               \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// the "fast path": ~0.1 ms of streaming, then the verdict (xfail) and, when it took the batch, done = 1
__global__ void fast(const float4* __restrict__ in, float4* __restrict__ out, size_t n, const unsigned* want_fail,
                     unsigned* xfail, unsigned* done) {
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t i = i0; i < n; i += (size_t)gridDim.x * blockDim.x) out[i] = in[i];
  if (i0 == 0) {
    const unsigned f = *want_fail;
    *xfail = f;
    if (done && f == 0) __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void gated(const unsigned* gate, unsigned* work) {
  if (*gate == 0) return;
  work[blockIdx.x * blockDim.x + threadIdx.x] += 1;
}

__global__ void signal_done(unsigned* done) {
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void after(unsigned* w) {
  if (threadIdx.x == 0 && blockIdx.x == 0) w[0] += 1;
}

int main() {
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("{\"can_use_stream_wait_value\": %d}\n", can);
  if (!can) return 0;
  const size_t n = (256ull << 20) / 16;  // 256 MiB copied: ~0.1 ms
  float4 *in, *out;
  unsigned *xfail, *want, *work, *done;
  CK(hipMalloc(&in, n * 16));
  CK(hipMalloc(&out, n * 16));
  CK(hipMemset(in, 0, n * 16));
  CK(hipMalloc(&xfail, 4));
  CK(hipMalloc(&want, 4));
  CK(hipMalloc(&work, 1024 * 256 * 4));
  CK(hipMemset(work, 0, 1024 * 256 * 4));
  CK(hipExtMallocWithFlags((void**)&done, 8, hipMallocSignalMemory));  // signal memory: 8 bytes
  hipStream_t s, side;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  hipEvent_t e0, e1, fork;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  const int K = 22;
  const char* names[7] = {"chain", "side", "side_g", "none", "memset2", "write2", "memset1"};
  unsigned long long* ctlw;  // two words to reset, as the transform's ctl and fail
  CK(hipMalloc(&ctlw, 64));
  for (int form = 0; form < 7; ++form) {
    const unsigned wf = form == 2 ? 1u : 0u;
    CK(hipMemcpy(want, &wf, 4, hipMemcpyHostToDevice));
    std::vector<float> t;
    for (int rep = 0; rep < 52; ++rep) {
      CK(hipStreamWriteValue32(s, done, 0, 0));
      CK(hipEventRecord(e0, s));
      if (form == 4) {
        CK(hipMemsetAsync(ctlw, 0, 8, s));
        CK(hipMemsetAsync(ctlw + 4, 0, 8, s));
      } else if (form == 5) {
        CK(hipStreamWriteValue64(s, ctlw, 0, 0));
        CK(hipStreamWriteValue64(s, ctlw + 4, 0, 0));
      } else if (form == 6) {
        CK(hipMemsetAsync(ctlw, 0, 16, s));
      }
      hipLaunchKernelGGL(fast, dim3(1024), dim3(256), 0, s, in, out, n, want, xfail, form == 1 || form == 2 ? done : nullptr);
      if (form == 0) {
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(gated, dim3(1024), dim3(256), 0, s, xfail, work);
      } else if (form == 1 || form == 2) {
        CK(hipEventRecord(fork, s));
        CK(hipStreamWaitEvent(side, fork, 0));
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(gated, dim3(1024), dim3(256), 0, side, xfail, work);
        hipLaunchKernelGGL(signal_done, dim3(1), dim3(64), 0, side, done);
        CK(hipStreamWaitValue32(s, done, 1, hipStreamWaitValueEq, 0xFFFFFFFFu));
      }
      hipLaunchKernelGGL(after, dim3(1), dim3(64), 0, s, work);
      CK(hipEventRecord(e1, s));
      CK(hipGetLastError());
      CK(hipStreamSynchronize(s));
      CK(hipStreamSynchronize(side));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("{\"form\": \"%s\", \"gated_kernels\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"ms_max\": %.4f}\n", names[form],
           form >= 3 ? 0 : K, t[t.size() / 2], t.front(), t.back());
    fflush(stdout);
  }
  return 0;
}
