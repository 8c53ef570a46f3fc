// crc32_kernels.h -- launch interface between the C ABI (ambrycrc.cpp) and the
// gfx950 kernels (crc32_kernels.hip). Internal to libambrycrc.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace ambrycrc {

struct PlanArgs {
  const uint64_t* off;   // [n] byte offsets of chunks from base
  const uint64_t* len;   // [n] chunk lengths
  uint32_t n;
  uint32_t tile_log2;
  uint32_t* tile_start;  // [n+1] exclusive prefix of tiles per chunk; [n] = total
  uint32_t* out;         // [n] zeroed here, XOR-accumulated by the tiles kernel
};

struct TilesArgs {
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* len;
  const uint32_t* crc_in;  // [n] or null: zlib-style running CRC to continue from
  uint32_t n;
  uint32_t tile_log2;
  const uint32_t* tile_start;
  const uint32_t* img;     // LDS image (kLdsBytes) followed by 64 words x^(8*2^k)
  uint32_t* out;
};

hipError_t launch_plan(const PlanArgs& a, hipStream_t s);
hipError_t launch_tiles(const TilesArgs& a, int grid, int variant, hipStream_t s);
hipError_t launch_verify(const uint32_t* crc, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                         uint32_t n, hipStream_t s);
hipError_t launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off, hipStream_t s);

}  // namespace ambrycrc
