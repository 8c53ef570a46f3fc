// crc32_kernels.h -- launch interface between the C ABI (ambrycrc.cpp) and the
// gfx950 kernels (crc32_kernels.hip). Internal to libambrycrc.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace ambrycrc {

struct PlanArgs {
  const uint64_t* off;     // [n] byte offsets of chunks from base
  const uint64_t* len;     // [n] chunk lengths
  const uint32_t* crc_in;  // [n] or null
  uint32_t n;
  uint64_t* byte_start;    // [n+1] exclusive scan of len; [n] = total bytes
  uint64_t* block_sum;     // [ceil(n / kPlanPerBlock)] scratch
  uint32_t* out;           // [n] initialised here, XOR-accumulated by the sweep kernel
  uint64_t small_max;      // chunks with 0 < len <= small_max go to the group kernel (0: none)
  uint64_t* block_small;   // [ceil(n / kPlanPerBlock)] scratch: 4 x 16-bit size-class counts
  uint64_t* small_total;   // [5] number of small chunks; start of size classes 1..3 in small_idx;
                           // [4] the sweep's dynamic share counter (zeroed here)
  uint32_t* small_idx;     // [n] their indices, grouped by size class, ascending within a class
};

constexpr uint32_t kPlanPerBlock = 2048;  // chunks per planning workgroup
constexpr uint64_t kShareQuantum = 1024;  // per-wave byte shares are multiples of this
constexpr uint64_t kMinShare = 16384;     // ... and at least this (see crc32_sweep_kernel)

struct SweepArgs {
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* len;
  const uint32_t* crc_in;  // [n] or null: zlib-style running CRC to continue from
  uint32_t n;
  const uint64_t* byte_start;
  const uint32_t* img;     // LDS image (kLdsBytes) followed by 64 words x^(8*2^k)
  uint32_t* out;
  uint64_t small_max;      // sweep: skip chunks with len <= small_max; group kernel: take them
  const uint64_t* small_total;  // [4] as PlanArgs
  uint64_t* claim;              // = PlanArgs small_total + 4 (dynamic shares, variant 27)
  const uint32_t* small_idx;
  // Message verify (class-sized group phase only, variants 26-29): for every chunk the group
  // phase takes, also read the big-endian 8-B CRC stored right after it (base + off + len)
  // and write exp_fill[chunk] = its low word, or ~crc when the high word is not zero (a
  // forced mismatch: a CRC-32 never has upper bits). Null otherwise.
  uint32_t* exp_fill;
  // Byte-share rounds: a batch of more than `window` bytes is swept in R = ceil(total /
  // window) rounds of nwaves shares each (share i -> wave i % nwaves), so at any time the
  // waves read inside about one window, not across the whole batch. 0 = one round.
  uint64_t window;
};

// Group kernel shapes (mode -> G lanes per chunk, NB blocks of 16G bytes): small_max = 16*G*NB.
// 0 = off, 1 = G16/NB8 (2 KiB), 2 = G16/NB16 (4 KiB), 3 = G32/NB8 (4 KiB), 4 = G16/NB32 (8 KiB),
// 5 = G16/NB64 (16 KiB), 6 = G32/NB32 (16 KiB)
constexpr int kNumGroupModes = 7;
// Batches of fewer chunks than this take the sweep (wave mode) for every chunk: with idle
// waves to spare, 64 lanes per chunk beat a 16-lane group's 4x longer chain on latency.
constexpr size_t kGroupMinChunks = 16384;
constexpr uint64_t group_small_max(int mode) {
  return mode == 1 ? 2048u
         : (mode == 2 || mode == 3) ? 4096u
         : mode == 4 ? 8192u
         : (mode == 5 || mode == 6) ? 16384u
                                    : 0u;
}

// sweep-kernel variants (U = loads in flight per lane, NT = nontemporal, PIPE = rolling prefetch,
// IL = two pieces interleaved, WIN = descriptors fetched 64 per wave-load, else one-ahead scalar
// prefetch): 0 U8/NT/PIPE/IL/WIN (the round-1 base shape), 1 = 0 without WIN, 2 U8/NT/PIPE/WIN, 3 U4/NT/PIPE/WIN,
// 4 U8/PIPE/IL/WIN (temporal loads), 5 U8/NT batch loads, 6 U4/NT/PIPE/IL/WIN, 7 U8 batch (temporal)
// 8 R=2 strided lane runs (U8 loads in flight), 9 R=4 strided runs (U8), 10 R=4 strided (U4),
// 11 R=2 strided (U4), 12 64-B runs by quad transpose of coalesced loads (U8), 13 same (U4)
// 14..19 = 0 plus the group kernel (modes 1..6) for small whole chunks; 20, 21, 22 = 0 with the
// group phase (G16/NB32, G16/NB16, G16/NB64: chunks <= 8, 4, 16 KiB) fused into the sweep launch
// 23 = 13 (quad-transposed 64-B lane runs, U4) with the G16/NB64 group phase fused in
// 24 = 12 (quad-transposed 64-B lane runs, U8) with the G16/NB64 group phase fused in
// (8 waves per CU with 256 VGPRs and U8/U16 prefetch lost 3-14 % to these at 16 waves: the
// 4 waves per SIMD hide the LDS chains better; the TPB template parameter is kept)
// 25 = 23 with the quad transposes' lane selects fused into DPP moves (v_cndmask_b32_dpp)
// 26 = 25 with the group phase sized and balanced per size class (G = 4 for <= 256 B, 8 for
// <= 1 KiB, 16 above; every class spread over all waves)
// (prefetching the group rounds' list entries and descriptors two stages ahead measured no
// gain over 26: the 16 waves per CU already hide that latency)
// (dynamic shares -- share/8 bytes each, the rest claimed from an atomic counter after a
// static first one; the DYN template parameter -- lost 0.6 % on C3, 1.3 % on C4 and 12 % on
// C2: each claim pays a chunk search and a descriptor reload, and the tail it would
// shorten was not there)
// 27 = 26 with 64-B lane runs (quad transpose) in the 16-lane groups of classes 2-3
// 28 = 27 with 64-B lane runs in the 8-lane groups of class 1 (257 B - 1 KiB) too
// (two super-blocks, 8 loads per lane, in flight in the sweep body: -6 % on C3, -4 % on C2
// at the 128-VGPR cap)
// 29 (default) = 28 with s_setprio 3 while a wave issues its super-block loads (+0.2-0.5 %)
// (measured and not kept, DESIGN.md §4: 12 waves per CU, 8-lane groups for 1-16 KiB, temporal
// or prioritised group-phase loads, 128-B cut snapping, group caps of 8, 20 and 64 KiB)
constexpr int kNumVariants = 30;
constexpr int kDiagNoFold = 100;  // diagnostic timing build, selectable via ambrycrc_set_variant only

// Message verify (message_kernels.hip): kMsgSlots CRC jobs per message, slot order
// encryption key, blob properties, update, user metadata, blob.
constexpr int kMsgSlots = 5;

struct MsgArgs {
  const uint8_t* region;
  uint64_t region_len;
  const uint64_t* msg_off;  // [m]
  uint64_t m;
  const uint32_t* img;      // table image (T0 used by the header CRC)
  uint64_t* job_off;        // [5m], slot-major: job k*m + i = slot k of message i
  uint64_t* job_len;        // [5m]
  uint32_t* expected;       // [5m]
  const uint32_t* crc;      // [5m] computed record CRCs
  uint32_t* status;         // [m]
  uint64_t* msg_end;        // [m] or null
  uint64_t inline_max;      // records of 1..inline_max bytes: stored CRC read by the sweep's
                            // group phase (SweepArgs::exp_fill), not by the parse kernel
};

// CRC-trailered records (index segment files, log segment headers, user metadata, ...):
// item i = [off[i], off[i] + len[i]) ends in its own big-endian 8-B CRC.
struct TrailerArgs {
  const uint8_t* base;
  const uint64_t* off;      // [n]
  const uint64_t* len;      // [n] including the 8-B trailer
  uint64_t n;
  uint64_t* job_len;        // [n] = len - 8 (0 when len < 8)
  uint32_t* expected;       // [n] stored CRC (low word); left to the group phase for 1..inline_max
  uint8_t* force;           // [n] 1 = mismatch whatever the CRC (len < 8, or a stored high word)
  const uint32_t* crc;      // [n] computed
  uint8_t* mismatch;        // [n] or null
  uint32_t* count;          // or null
  uint64_t inline_max;
};

hipError_t launch_trailer_parse(const TrailerArgs& a, hipStream_t s);
hipError_t launch_trailer_verify(const TrailerArgs& a, hipStream_t s);

hipError_t launch_msg_parse(const MsgArgs& a, hipStream_t s);
hipError_t launch_msg_reduce(const MsgArgs& a, hipStream_t s);

hipError_t launch_plan(const PlanArgs& a, hipStream_t s);
hipError_t launch_sweep(const SweepArgs& a, int grid, int variant, hipStream_t s);
hipError_t launch_group(const SweepArgs& a, int grid, int mode, hipStream_t s);
hipError_t launch_verify(const uint32_t* crc, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                         uint32_t n, hipStream_t s);
hipError_t launch_readbw(const uint8_t* base, uint64_t nbytes, uint32_t* out, int grid, int variant,
                         hipStream_t s);
hipError_t launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off, hipStream_t s);

}  // namespace ambrycrc
