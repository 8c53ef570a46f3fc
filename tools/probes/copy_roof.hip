// copy_roof.hip -- probe: device-to-device copy bandwidth on this GPU at a given size (argv[1] bytes;
// default the transform's 1.39 GB region -> separate output): hipMemcpyAsync, a grid-stride
// 16-B-per-lane kernel with plain / nontemporal loads and stores at a few unroll depths, and a
// contiguous-share form (each wave copies its own contiguous 1/waves of the buffer, 4 KiB per
// step). Prints JSON lines (GB/s of read + write).
// Build: hipcc -O3 --offload-arch=gfx950 -o copy_roof tools/probes/copy_roof.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// each wave copies [w*per, (w+1)*per) 16 B per lane, U wave-loads in flight
template <int U>
__global__ __launch_bounds__(256) void copy_share(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t waves = (size_t)gridDim.x * (blockDim.x / 64);
  const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const size_t lane = threadIdx.x & 63;
  const size_t lo = n * w / waves, hi = n * (w + 1) / waves;
  size_t i = lo + lane;
  for (; i + 64 * (U - 1) < hi; i += 64 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + i + 64 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], dst + i + 64 * u);
  }
  for (; i < hi; i += 64) dst[i] = src[i];
}

// each wave copies 16 KiB chunks w, w + waves, w + 2 waves, ... (the concurrent accesses of all waves
// stay inside one window of waves x 16 KiB that moves through the buffer)
__global__ __launch_bounds__(256) void copy_window(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  const size_t waves = (size_t)gridDim.x * (blockDim.x / 64);
  const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const size_t lane = threadIdx.x & 63;
  constexpr size_t C = 1024;  // 16-B pieces per chunk
  for (size_t c = w * C; c < n; c += waves * C) {
    u32x4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = c + lane + 64 * u < n ? __builtin_nontemporal_load(src + c + lane + 64 * u) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 16; ++u) if (c + lane + 64 * u < n) __builtin_nontemporal_store(v[u], dst + c + lane + 64 * u);
  }
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(r_), __LINE__); exit(1); } } while (0)

template <int U, bool NTL, bool NTS>
static void run(const char* name, const u32x4* s, u32x4* d, size_t n, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  float best = 1e9, sum = 0;
  const int reps = 10;
  for (int r = 0; r < reps + 2; ++r) {
    CK(hipEventRecord(e0, st));
    hipLaunchKernelGGL((copy_k<U, NTL, NTS>), dim3(grid), dim3(256), 0, st, s, d, n);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2) { sum += ms; if (ms < best) best = ms; }
  }
  const double bytes = 2.0 * n * 16;
  printf("{\"copy\": \"%s\", \"grid\": %d, \"ms_avg\": %.4f, \"GBps_avg\": %.1f, \"GBps_best\": %.1f}\n", name, grid,
         sum / reps, bytes / (sum / reps) / 1e6, bytes / best / 1e6);
}

template <int U>
void run_share(const char* name, const u32x4* s, u32x4* d, size_t n, int grid, hipStream_t st, hipEvent_t e0,
               hipEvent_t e1) {
  float sum = 0, best = 1e30f;
  for (int r = 0; r < 12; ++r) {
    CK(hipEventRecord(e0, st));
    hipLaunchKernelGGL(copy_share<U>, dim3(grid), dim3(256), 0, st, s, d, n);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2) sum += ms, best = ms < best ? ms : best;
  }
  printf("{\"copy\": \"%s\", \"bytes\": %zu, \"grid\": %d, \"ms_avg\": %.4f, \"GBps_avg\": %.1f, \"GBps_best\": %.1f}\n",
         name, n * 16, grid, sum / 10, 2.0 * n * 16 / (sum / 10) / 1e6, 2.0 * n * 16 / best / 1e6);
}

int main(int argc, char** argv) {
  // default: 262,144 x 4 KiB PUT messages (bench_put.py's transform case)
  const size_t bytes = argc > 1 ? (size_t)strtoull(argv[1], nullptr, 10) & ~(size_t)4095 : 1389101056;
  const size_t n = bytes / 16;
  u32x4 *s, *d;
  CK(hipMalloc(&s, bytes)); CK(hipMalloc(&d, bytes));
  const int trials = argc > 2 ? atoi(argv[2]) : 0;
  if (trials > 0) {  // placement trials: each a new destination (earlier ones kept), three copy forms
    CK(hipMemset(s, 1, bytes));
    hipStream_t st; CK(hipStreamCreate(&st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int t = 0; t < trials; ++t) {
      if (t) CK(hipMalloc(&d, bytes));
      CK(hipMemset(d, 0, bytes));
      printf("{\"trial\": %d, \"dst_minus_src\": %lld}\n", t, (long long)((char*)d - (char*)s));
      run<8, true, true>("nt_u8", s, d, n, 2048, st, e0, e1);
      run_share<8>("share_nt_u8", s, d, n, 1024, st, e0, e1);
      {
        float sum = 0, best = 1e30f;
        for (int r = 0; r < 12; ++r) {
          CK(hipEventRecord(e0, st));
          hipLaunchKernelGGL(copy_window, dim3(1024), dim3(256), 0, st, s, d, n);
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms; CK(hipEventElapsedTime(&ms, e0, e1));
          if (r >= 2) sum += ms, best = ms < best ? ms : best;
        }
        printf("{\"copy\": \"window16k\", \"grid\": 1024, \"ms_avg\": %.4f, \"GBps_avg\": %.1f, \"GBps_best\": %.1f}\n",
               sum / 10, 2.0 * n * 16 / (sum / 10) / 1e6, 2.0 * n * 16 / best / 1e6);
      }
      fflush(stdout);
    }
    return 0;
  }
  CK(hipMemset(s, 1, bytes)); CK(hipMemset(d, 0, bytes));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  {
    float sum = 0;
    for (int r = 0; r < 12; ++r) {
      CK(hipEventRecord(e0, st));
      CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) sum += ms;
    }
    printf("{\"copy\": \"hipMemcpyAsync\", \"bytes\": %zu, \"ms_avg\": %.4f, \"GBps_avg\": %.1f}\n", bytes, sum / 10,
           2.0 * bytes / (sum / 10) / 1e6);
  }
  int cu = 256;
  for (int g : {cu * 4, cu * 8, cu * 16}) {
    run<4, false, false>("plain_u4", s, d, n, g, st, e0, e1);
    run<4, true, true>("nt_u4", s, d, n, g, st, e0, e1);
    run<4, true, false>("ntload_u4", s, d, n, g, st, e0, e1);
    run<8, true, true>("nt_u8", s, d, n, g, st, e0, e1);
  }
  for (int g : {cu * 2, cu * 4, cu * 8}) {
    run_share<4>("share_nt_u4", s, d, n, g, st, e0, e1);
    run_share<8>("share_nt_u8", s, d, n, g, st, e0, e1);
  }
  return 0;
}
