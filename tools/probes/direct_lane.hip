// direct_lane.hip -- probe: can a region of small messages be verified in ONE read, each lane
// hashing its own message straight from memory (no run sums, no second pass)? m messages of S
// bytes packed back to back (S = 1284 / 2208 / 5280: the 100 B / 1 KiB / 4 KiB-blob PUTs of
// tools/bench_messages.py); lane i computes message i's zlib CRC-32 with 16-B aligned loads, one
// 64-B run prefetched ahead, slice-by-4 tables in LDS (replicated per lane column, as the streaming
// kernels' TabR, or one compact copy), partial words at the ends byte by byte. Variants:
//   xor   the same loads, words XORed (the access pattern's memory rate, no hashing)
//   rep   replicated tables, 1024-thread workgroups (one per CU)
//   cmp   compact tables, 256-thread workgroups (AMBRY-style 2 per CU)
// Prints one JSON line per (S, variant): ms per pass (median of 7), GB/s of region bytes, and the
// CRCs of a few messages checked against a host table CRC. Build:
//   hipcc -O3 --offload-arch=gfx950 -o tools/probes/direct_lane tools/probes/direct_lane.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(e)                                                                       \
  do {                                                                              \
    hipError_t r_ = (e);                                                            \
    if (r_ != hipSuccess) {                                                         \
      printf("HIP error %s at %d\n", hipGetErrorString(r_), __LINE__);              \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// replicated: word (j*256 + b)*32 + col, col = lane & 31 (128 KiB); compact: j*256 + b (4 KiB)
__shared__ uint32_t g_tab[4 * 256 * 32];

template <bool REP>
__device__ __forceinline__ uint32_t tl(uint32_t j, uint32_t b, uint32_t col) {
  return REP ? g_tab[((j << 8) | b) * 32 + col] : g_tab[(j << 8) | b];
}

template <bool REP>
__device__ __forceinline__ uint32_t step4(uint32_t x, uint32_t col) {
  return tl<REP>(3, x & 0xffu, col) ^ tl<REP>(2, (x >> 8) & 0xffu, col) ^ tl<REP>(1, (x >> 16) & 0xffu, col) ^
         tl<REP>(0, x >> 24, col);
}

template <int MODE>  // 0 xor, 1 rep, 2 cmp
__global__ __launch_bounds__(MODE == 2 ? 256 : 1024) void direct_lane(const uint8_t* __restrict__ region, uint64_t m,
                                                                      uint32_t S, const uint32_t* __restrict__ tabs,
                                                                      uint32_t* __restrict__ out) {
  constexpr bool REP = MODE == 1;
  if (MODE != 0) {
    for (uint32_t i = threadIdx.x; i < (REP ? 4u * 256u * 32u : 1024u); i += blockDim.x)
      g_tab[i] = REP ? tabs[i / 32] : tabs[i];
    __syncthreads();
  }
  const uint32_t col = threadIdx.x & 31u;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t pa = i * S, pb = pa + S;
    uint64_t a = pa & ~uint64_t(63);
    u32x4 cur[4], nxt[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(region + a) + q);
    uint32_t c = MODE == 0 ? 0u : 0xFFFFFFFFu;
    for (; a < pb; a += 64) {
      if (a + 64 < pb) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          nxt[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(region + a + 64) + q);
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t w = cur[k >> 2][k & 3];
        const uint64_t wa = a + 4 * k;
        if constexpr (MODE == 0) {
          c ^= w;
        } else if (wa >= pa && wa + 4 <= pb) {
          c = step4<REP>(c ^ w, col);
        } else if (wa + 4 > pa && wa < pb) {
          for (uint32_t b = 0; b < 4; ++b)
            if (wa + b >= pa && wa + b < pb) c = tl<REP>(0, (c ^ (w >> (8 * b))) & 0xffu, col) ^ (c >> 8);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    }
    out[i] = MODE == 0 ? c : ~c;
  }
}

__global__ void fill(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    p[i] = x;
  }
}

static uint32_t host_crc(const uint8_t* p, size_t n, const uint32_t* t0) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = t0[(c ^ p[i]) & 0xffu] ^ (c >> 8);
  return ~c;
}

int main(int argc, char** argv) {
  (void)argc;
  (void)argv;
  // slice-by-4 tables: T0 the byte table, T_j[b] = T_{j-1}[b] advanced by one zero byte
  std::vector<uint32_t> t(1024);
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    t[b] = c;
  }
  for (int j = 1; j < 4; ++j)
    for (uint32_t b = 0; b < 256; ++b) t[256 * j + b] = t[t[256 * (j - 1) + b] & 0xffu] ^ (t[256 * (j - 1) + b] >> 8);
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const size_t region_bytes = 1400ull << 20;
  uint8_t* d_region;
  uint32_t *d_tab, *d_out;
  CK(hipMalloc(&d_region, region_bytes + 4096));
  CK(hipMalloc(&d_tab, 4096));
  CK(hipMalloc(&d_out, sizeof(uint32_t) * (1u << 21)));
  CK(hipMemcpy(d_tab, t.data(), 4096, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(d_region), (region_bytes + 4096) / 4,
                     0x1234567u);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t sizes[3] = {1284, 2208, 5280};
  const uint64_t counts[3] = {1048576, 524288, 262144};
  for (int si = 0; si < 3; ++si) {
    const uint32_t S = sizes[si];
    const uint64_t m = counts[si];
    for (int mode = 0; mode < 3; ++mode) {
      std::vector<float> ms;
      for (int r = 0; r < 9; ++r) {
        CK(hipEventRecord(e0, 0));
        if (mode == 0)
          hipLaunchKernelGGL(direct_lane<0>, dim3(ncu), dim3(1024), 0, 0, d_region, m, S, d_tab, d_out);
        else if (mode == 1)
          hipLaunchKernelGGL(direct_lane<1>, dim3(ncu), dim3(1024), 0, 0, d_region, m, S, d_tab, d_out);
        else
          hipLaunchKernelGGL(direct_lane<2>, dim3(2 * ncu), dim3(256), 0, 0, d_region, m, S, d_tab, d_out);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float x;
        CK(hipEventElapsedTime(&x, e0, e1));
        if (r >= 2) ms.push_back(x);
      }
      std::sort(ms.begin(), ms.end());
      int bad = 0;
      if (mode != 0) {
        std::vector<uint8_t> h(S);
        std::vector<uint32_t> o(m);
        CK(hipMemcpy(o.data(), d_out, sizeof(uint32_t) * m, hipMemcpyDeviceToHost));
        const uint64_t pick[4] = {0, 1, m / 2 + 7, m - 1};
        for (uint64_t q : pick) {
          CK(hipMemcpy(h.data(), d_region + q * S, S, hipMemcpyDeviceToHost));
          if (host_crc(h.data(), S, t.data()) != o[q]) ++bad;
        }
      }
      const double med = ms[ms.size() / 2];
      printf("{\"S\": %u, \"m\": %llu, \"variant\": \"%s\", \"ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f, \"crc_bad\": %d}\n",
             S, (unsigned long long)m, mode == 0 ? "xor" : mode == 1 ? "rep" : "cmp", med, ms[0],
             (double)m * S / (med * 1e-3) / 1e9, bad);
      fflush(stdout);
    }
  }
  return 0;
}
