// readroof.hip -- standalone HBM read-bandwidth probe for gfx950 (not part of libambrycrc).
// Sweeps workgroup size, loads in flight per lane, cache policy and access order over one
// large device buffer, to find the achievable read roof the CRC sweep is compared to.
//   build: hipcc -O3 --offload-arch=gfx950 -o tools/probes/readroof tools/probes/readroof.hip
//   run:   tools/probes/readroof [GiB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// Contiguous per-wave shares, lane l reading 16 B at 16l of each 1 KiB block, U blocks in flight.
template <int U, bool NT>
__global__ void share_kernel(const uint8_t* __restrict__ base, uint64_t nbytes, uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * gridDim.x + blockIdx.x);
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint64_t nb = nbytes / 1024 / nwaves;
  const u32x4* q = reinterpret_cast<const u32x4*>(base + (uint64_t)wave * nb * 1024) + lane;
  uint32_t x = 0;
  for (uint64_t b = 0; b + U <= nb; b += U) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = ld<NT>(q + (b + u) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
  }
  if (x == 0x12345678u) out[0] = x;
}

// Grid-stride over 1 KiB blocks: wave i reads blocks i, i+W, ... (all waves in one window).
template <int U, bool NT>
__global__ void stride_kernel(const uint8_t* __restrict__ base, uint64_t nbytes, uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * gridDim.x + blockIdx.x);
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint64_t nblk = nbytes / 1024;
  const u32x4* q = reinterpret_cast<const u32x4*>(base) + lane;
  uint32_t x = 0;
  for (uint64_t b = wave; b + (uint64_t)(U - 1) * nwaves < nblk; b += (uint64_t)U * nwaves) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = ld<NT>(q + (b + (uint64_t)u * nwaves) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
  }
  if (x == 0x12345678u) out[0] = x;
}

// Contiguous per-wave shares in 4 KiB super-blocks, lane l reading its own 64-B run
// [64l, 64l + 64) of each super-block as 4 x 16 B (no cross-lane transpose needed to walk it);
// U loads in flight per lane (U/4 super-blocks).
template <int U, bool NT>
__global__ void lanerun_kernel(const uint8_t* __restrict__ base, uint64_t nbytes, uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * gridDim.x + blockIdx.x);
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint64_t nsb = nbytes / 4096 / nwaves;
  const u32x4* q = reinterpret_cast<const u32x4*>(base + (uint64_t)wave * nsb * 4096) + 4 * lane;
  uint32_t x = 0;
  constexpr int S = U / 4;
  for (uint64_t b = 0; b + S <= nsb; b += S) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = ld<NT>(q + (b + u / 4) * 256 + (u & 3));
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= w[u].x ^ w[u].y ^ w[u].z ^ w[u].w;
  }
  if (x == 0x12345678u) out[0] = x;
}

typedef void (*kfn)(const uint8_t*, uint64_t, uint32_t*);

static double run(kfn f, int grid, int block, const uint8_t* d, uint64_t n, uint32_t* o) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, n, o);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, d, n, o);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return (double)n / (best / 1e3) / 1e9;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 32.0;
  const uint64_t n = (uint64_t)(gib * (1ull << 30)) & ~((1ull << 24) - 1);
  uint8_t* d;
  uint32_t* o;
  CHECK(hipMalloc(&d, n));
  CHECK(hipMalloc(&o, 4096));
  CHECK(hipMemset(d, 0x5a, n));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  struct Cfg {
    const char* name;
    kfn f;
    int wgs_per_cu, block;
  } cfgs[] = {
      {"share U8 NT 16w", share_kernel<8, true>, 1, 1024},   {"share U8 T 16w", share_kernel<8, false>, 1, 1024},
      {"share U4 NT 16w", share_kernel<4, true>, 1, 1024},   {"share U16 NT 8w", share_kernel<16, true>, 1, 512},
      {"share U8 NT 32w", share_kernel<8, true>, 2, 1024},   {"share U4 NT 32w", share_kernel<4, true>, 2, 1024},
      {"share U8 NT 8w", share_kernel<8, true>, 1, 512},     {"share U16 NT 16w", share_kernel<16, true>, 1, 1024},
      {"stride U8 NT 16w", stride_kernel<8, true>, 1, 1024}, {"stride U8 T 16w", stride_kernel<8, false>, 1, 1024},
      {"stride U8 NT 32w", stride_kernel<8, true>, 2, 1024}, {"stride U16 NT 8w", stride_kernel<16, true>, 1, 512},
      {"lanerun U4 NT 16w", lanerun_kernel<4, true>, 1, 1024}, {"lanerun U8 NT 16w", lanerun_kernel<8, true>, 1, 1024},
      {"lanerun U16 NT 8w", lanerun_kernel<16, true>, 1, 512},
      {"share U4 NT 16w (again)", share_kernel<4, true>, 1, 1024}, {"share U8 NT 16w (again)", share_kernel<8, true>, 1, 1024},
  };
  for (const Cfg& c : cfgs) {
    const double gbs = run(c.f, cus * c.wgs_per_cu, c.block, d, n, o);
    printf("{\"probe\": \"%s\", \"GiB\": %.1f, \"GBps\": %.1f}\n", c.name, gib, gbs);
    fflush(stdout);
  }
  CHECK(hipFree(d));
  CHECK(hipFree(o));
  return 0;
}
