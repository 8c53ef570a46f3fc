// crc32_kernels.h -- launch interface between the C ABI (ambrycrc.cpp) and the
// gfx950 kernels (crc32_kernels.hip). Internal to libambrycrc.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "../../include/ambrycrc.h"
#include "build_knobs.h"

namespace ambrycrc {

struct PropsFix;  // record_fields.h

struct PlanArgs {
  const uint64_t* off;     // [n] byte offsets of chunks from base
  const uint64_t* len;     // [n] chunk lengths
  const uint32_t* crc_in;  // [n] or null
  uint32_t n;
  uint64_t* byte_start;    // [n+1] exclusive scan of len; [n] = total bytes
  uint64_t* block_sum;     // [ceil(n / kPlanPerBlock)] scratch
  uint32_t* out;           // [n] initialised here, XOR-accumulated by the sweep kernel (small chunks:
                           // stored whole by the group phase, not initialised here)
  uint64_t small_max;      // chunks with 0 < len <= small_max go to the group kernel (0: none)
  uint64_t* block_small;   // [ceil(n / kPlanPerBlock)] scratch: 4 x 16-bit size-class counts
  uint64_t* small_total;   // [5] number of small chunks; start of size classes 1..3 in small_idx;
                           // [4] spare
  uint32_t* small_idx;     // [n] their indices, grouped by size class, ascending within a class
  uint32_t* crc_stage;     // [n] copy of crc_in (null iff crc_in is): read before out[] is written,
                           // so out may alias crc_in; the CRC kernels read this copy
  const uint32_t* gate;    // run only when *gate != 0 (null: always): the transform's fallback pass
};

// chunks per planning workgroup (a multiple of 256, <= 65535 so per-block class counts fit 16 bits)
constexpr uint32_t kPlanPerBlock = AMBRY_PLAN_PER_BLOCK;
static_assert(kPlanPerBlock % 256 == 0 && kPlanPerBlock <= 65535, "plan block size");
constexpr uint64_t kShareQuantum = 1024;  // per-wave byte shares are multiples of this
constexpr uint64_t kMinShare = 16384;     // ... and at least this (see crc32_sweep_kernel)

// Load invariant of every CRC kernel (plan, sweep, group phase, copy-through): the only global
// bytes read through `base` are chunk bytes, [base + off[c], base + off[c] + len[c]) for c < n,
// plus -- with exp_fill -- the 8 stored-CRC bytes after a group-phase chunk. An empty chunk reads
// nothing. So base must be a real device pointer that every chunk's bytes lie at or after (it is
// never dereferenced by itself); the serializer's copy-through passes the lowest of its source
// buffers (PutArgs::src_base), not null.
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
  const uint32_t* small_idx;
  // Message verify (class-sized group phase only, variant 29): for every chunk the group
  // phase takes, also read the big-endian 8-B CRC stored right after it (base + off + len)
  // and write exp_fill[chunk] = its low word, or ~crc when the high word is not zero (a
  // forced mismatch: a CRC-32 never has upper bits). Null otherwise.
  uint32_t* exp_fill;
  // Byte-share rounds: a batch of more than `window` bytes is swept in R = ceil(total /
  // window) rounds of nwaves shares each (share i -> wave i % nwaves), so at any time the
  // waves read inside about one window, not across the whole batch. 0 = one round.
  uint64_t window;
  // Copy-through (launch_sweep_copy only): every byte read for chunk c is also written to
  // copy_dst + copy_off[c] + (its offset in the chunk). The PUT serializer's copy mode uses it so a
  // field is read once for both its copy and its CRC. Null for every other launch.
  uint8_t* copy_dst;
  const uint64_t* copy_off;  // kCopySkip: chunk c is read (CRC'd) but not copied
  // Run only when *gate != 0 (null: always): the transform's general path behind its one-pass
  // fast path (ambrycrc_put.cpp).
  const uint32_t* gate = nullptr;
};
constexpr uint64_t kCopySkip = ~0ull;

// Chunks of 1 B .. kGroupSmallMax go to the group phase (variant 29) in batches of at least
// kGroupMinChunks chunks; smaller batches take the sweep (wave mode) for every chunk: with idle
// waves to spare, 64 lanes per chunk beat a 16-lane group's 4x longer chain on latency.
constexpr size_t kGroupMinChunks = 16384;
constexpr uint64_t kGroupSmallMax = 16384;

// Sweep-kernel variants built into the library (round 1 measured 30 shapes; git history has
// them, DESIGN.md §4 the results):
//   0  (kVariantPieces): lane l owns bytes [16l, 16l+16) of every 1 KiB block, 8 blocks in
//      flight, two pieces interleaved; every chunk in the sweep (no group phase). Fallback.
//   29 (kVariantDefault): 64-B lane runs from coalesced 4 KiB super-blocks (quad transpose by
//      v_cndmask_b32_dpp, one x^(8*4096) fold per 64 B), s_setprio 3 around the loads, plus
//      the class-sized group phase (G = 4 / 8 / 16 lanes for <= 256 B / 1 KiB / 16 KiB) with
//      the stored CRC read inline for message verify (SweepArgs::exp_fill).
// A/B builds only (tools/ab_build.sh, -DAMBRY_AB_PROBE_BUILD; never in the product library):
//   100..102: timing diagnostics that produce wrong CRCs (-DAMBRYCRC_DIAGNOSTICS).
//   32 (kVariantSplit): the group phase as a kernel of its own (tools/probes/group_kernels.hip,
//      -DAMBRY_AB_SPLIT_GROUP: 72.5 KiB LDS image, <= 64 VGPRs, two 1024-thread workgroups = 32
//      waves per CU), then variant 29's sweep kernel without its fused group phase. It lost to 29
//      at every size and occupancy (0.45-0.90x).
constexpr int kVariantPieces = 0;
constexpr int kVariantDefault = 29;
constexpr int kVariantSplit = 32;
constexpr bool variant_supported(int v) {
#ifdef AMBRYCRC_DIAGNOSTICS
  if (v >= 100 && v <= 102) return true;
#endif
#ifdef AMBRY_AB_SPLIT_GROUP
  if (v == kVariantSplit) return true;
#endif
  return v == kVariantPieces || v == kVariantDefault;
}
// variants 29 and 32 read group-phase records' stored CRCs inline
constexpr bool variant_groups(int v) { return v == kVariantDefault || v == kVariantSplit; }
constexpr int kDiagNoFold = 100;  // diagnostic timing build, selectable via ambrycrc_set_variant only

// Region mode of the message verify: the log region is swept once as contiguous
// memory, each 64-B run's raw CRC (zero register, no xor-out) stored (crc32_kernels.hip
// region_runs_kernel), then one thread per message parses it and assembles its record CRCs from
// the runs they cover (message_kernels.hip region_msg_kernel, region_crc.h). Runs are [base + 64k, base + 64k + 64) with
// base = the region's start rounded down to 64 B; only 16-B pieces holding region bytes are read.
// A record of more than region::kLongRuns runs (a multi-MiB blob among small messages) that the
// region kernels leave to region_long_kernel: that kernel splits it into kLongPiece-byte pieces
// over the whole grid, each piece's zlib CRC by one wave from the run sums into slot[piece0 + p];
// the wave that finishes a record's last piece (done counts them) folds its pieces (crc(A||B) =
// crc(A) x^(8|B|) + crc(B): a tree over the lanes by x^(8 kLongPiece 2^k)) and compares.
struct LongRec {
  uint64_t pa;       // base-relative start
  uint64_t msg;      // message index
  uint32_t len, ex;  // record length, stored CRC
  uint32_t bit;      // the status bit of its record slot
  uint32_t piece0;   // its first piece in the list's numbering
  uint32_t pieces;   // 0: not listed (the slots ran out; the caller took the record)
  uint32_t done;     // pieces hashed (region_long_kernel; list_long zeroes it)
};
struct LongList {
  LongRec* rec = nullptr;              // [cap]
  unsigned long long* ctr = nullptr;   // records << 32 | pieces, one atomic (piece0 ascending with the index)
  uint32_t* claim = nullptr;           // (zeroed with ctr; reserved)
  uint32_t cap = 0;                    // records the list holds (more: the caller's own path)
  uint32_t* slot = nullptr;            // [pcap] piece CRCs
  uint32_t pcap = 0;
};
// Records of more pieces than this stay with their caller (the combine: one wave, 64 pieces a round).
constexpr uint32_t kLongMaxPieces = 4096;
// Pieces of 64 KiB (x^(8*65536) is the nibble set record_crc_runs_wave folds its streams by): a
// 4 MiB blob is 64 waves' work.
constexpr uint64_t kLongPiece = 64u << 10;

struct RegionArgs {
  const uint8_t* base;   // region start rounded down to 64 B
  uint64_t reg0;         // region start - base (0..63)
  uint64_t reg_end;      // region end - base
  uint64_t lo16, hi16;   // offsets from base of the first and last 16-B pieces holding region bytes
  uint64_t nsb;          // 4 KiB super-blocks (64 runs each) from base over the region
  uint32_t* rk;          // [kRunPad + nsb * 64 + 256]: run k's raw CRC at rk[kRunPad + k]; then a
                         // 1 KiB spill line for the stores of lanes with no sums to write
  const uint32_t* img;   // the table image (kImgBytes)
  LongList lng;          // two-pass region mode: long records (region_runs_kernel zeroes ctr / claim)
};
// Words ahead of run 0: a run group read before run 0 stays inside rk, and each super-block's 64
// sums (one wave store) fill exactly two 128-B lines (a misaligned window left partial lines,
// which cost pass 1 ~80 us per 1.4 GB region).
constexpr uint64_t kRunPad = 32;
constexpr uint64_t kSuperBlock = 4096;
// Region bytes per message up to which the message verify takes region mode (64-B run sums in
// the workspace: region / 16 bytes) instead of CRC jobs through the batch engine. Region / job
// mode per call (profiles/r03za_messages.jsonl, one box, ~1.3 GB regions): 1.3 KiB per message
// 1.21x, 2.2 KiB 1.35x, 3.2 KiB 1.17x, 4.2 KiB 1.07x, 5.3 KiB 1.02x; 64 KiB blobs stream in job mode.
constexpr uint64_t kRegionMaxPerMessage = 6144;
// Region bytes per message up to which the transform (header V3 out) tries the one-pass fast path
// first. Fast / general path, ms per ~1.2 GB batch, interleaved on one box (profiles/
// r04x_put_xform_fastmax*.jsonl): 9.2 KiB per message 0.631-0.634 / 0.899-0.903, 17.4 KiB
// 0.616-0.619 / 0.624, 33.8 KiB 0.593-0.597 / 0.595; 5.3 KiB 0.693-0.697 / 1.163; 67 KiB (before
// the tail work) 2.07 / 1.96. With the copy form's 8-wave workgroups (r04ax,
// r04aq): 9.2 KiB 0.581 / 0.893, 17.4 KiB 0.563 / 0.629, 33.8 KiB 0.567 / 0.601-0.604, 67 KiB
// 2.00 / 1.975 -- hence 40 KiB. AMBRYCRC_XFORM_FAST_MAX overrides it (A/B; 0 = never).
constexpr uint64_t kXformFastMaxPerMessage = 40960;
inline uint64_t region_nsb(const uint8_t* region, uint64_t len) {
  const uint64_t b = reinterpret_cast<uintptr_t>(region) & ~uint64_t(63);
  return (reinterpret_cast<uintptr_t>(region) + len - b + kSuperBlock - 1) / kSuperBlock;
}
// Run sums (rk), then the one-pass kernels' control words and deferred list (FusedArgs ctl, defer)
// for m messages.
inline size_t region_rk_bytes(const uint8_t* region, uint64_t len) {
  return (size_t)((kRunPad + region_nsb(region, len) * 64 + 256) * 4 + 255) & ~size_t(255);
}
inline size_t region_ws_bytes(const uint8_t* region, uint64_t len, uint64_t m) {
  return region_rk_bytes(region, len) + ((256 + 4 * m + 255) & ~size_t(255));
}
hipError_t launch_region_runs(const RegionArgs& a, int grid, hipStream_t s);

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
  const uint32_t* gate = nullptr;  // parse / reduce kernels run only when *gate != 0 (null: always)
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

// PUT serialization (put_kernels.hip): job k of message i is entry k*m + i (slot-major).
struct PutArgs {
  const ::ambrycrc_put_desc* desc;  // [m]
  uint64_t m;
  uint8_t* out;
  const uint8_t* fields;   // or null: key / encryption key / properties / user metadata already in place
  const uint8_t* blobs;    // or null: blob contents already in place
  uint64_t* cp_src;        // [5m] copy jobs: source address - src_base, destination offset in out, length
  uint64_t* cp_dst;
  uint64_t* cp_len;
  uint64_t* cp_cost;       // [5m] len + kCopyJobCost (0 for an empty job): what the copy balances
  uint64_t* crc_off;       // [5m] CRC jobs in out (length 0: absent encryption-key record)
  uint64_t* crc_len;
  const uint32_t* crc;     // [5m] their CRCs (from the batch kernels)
  uint32_t* crc_in;        // [5m] copy-through: the CRC of each record's prefix, the batch's seed
  uint64_t* msg_len;       // [m] or null
  // Transform only: the CRCs of records 1-4 (encryption key, properties, user metadata, blob)
  // known from the input message ([4m], message-major; see TransformArgs::in_crc). When set,
  // put_layout_kernel hashes the new header itself and writes every trailer, and no CRC pass
  // over the output runs. img: the table image (crc_img.h).
  const uint32_t* in_crc;
  const uint32_t* img;
  // Run only when *gate != 0 (null: always). The transform's fallback pass.
  const uint32_t* gate;
  // Transform only ([m] or null): properties re-encoded at V5 -- the copy job moves the stored
  // payload (stored_len bytes), props_fix_kernel then rewrites it in place (record_fields.h).
  const PropsFix* pfix;
  // Subtracted from every cp_src: 0 for the gather copy (absolute addresses); in copy-through mode the
  // lowest of the source buffers, and the CRC batch's base (SweepArgs load invariant).
  uint64_t src_base;
  // Copy-through mode (copy mode without in_crc): the copy jobs become the CRC batch itself --
  // the sweep reads each field once, writes it to the message and CRCs it, seeded (crc_in) with
  // the CRC of the record's prefix (<= 13 B, hashed by the layout kernel), so the batch's result
  // is the record CRC; the layout kernel writes the header trailer itself. A slot with no source
  // buffer (fields or blobs null) re-reads its bytes in place (src = dst).
  bool copy_through;
  // Copy mode with both source buffers (round 6): messages of at most stream_max bytes are written by
  // put_stream_kernel / put_stream_seal_kernel, and put_layout_kernel gives them no jobs (it writes
  // their header and record prefixes); a longer one sets *big, which gates the job path (plan + sweep,
  // seal). 0: every message through the job path.
  uint32_t stream_max = 0;
  uint32_t* big = nullptr;
  // The streamed messages' job entries are left unwritten by the layout pass (they would be 5 x 40 B
  // of zeros a message that nothing reads unless a long message is present); with clear_short the
  // kernel only zeroes them, launched gated on *big ahead of the job path.
  bool clear_short = false;
};

// Each copy job costs its bytes plus kCopyJobCost: a wave pays about one memory round trip
// (~2 us, ~1.6 KB of its share of HBM bandwidth) per job whatever its size, so balancing bytes
// alone put 22,000 24-B key copies on one wave (a 28 ms kernel for 4 GiB of 64 KiB PUTs).
constexpr uint64_t kCopyJobCost = 2048;

struct CopyArgs {
  const uint64_t* src;      // [n] absolute source addresses
  const uint64_t* dst_off;  // [n] destination offsets from dst
  const uint64_t* len;      // [n]
  const uint64_t* start;    // [n+1] exclusive scan of the job costs (len + kCopyJobCost)
  uint32_t n;
  uint8_t* dst;
  const uint32_t* gate;  // run only when *gate != 0 (null: always)
};

// ValidatingTransformer (message_kernels.hip): stored messages -> put descriptors -> serialization.
struct TransformArgs {
  const uint8_t* region;
  uint64_t region_len;
  const uint64_t* msg_off;        // [m]
  uint64_t m;
  const int16_t* life;            // [m] or null
  int header_version;             // of the output
  ::ambrycrc_put_desc* desc;      // [m] built here (header_version 0: not transformed)
  uint64_t* out_len;              // [m]
  uint64_t* out_off;              // [m] or null
  uint32_t* status;               // [m] in: verify bits; out: + NOT_PUT / BAD_RECORD / NO_ROOM
  uint64_t out_cap;
  // [4m] out: per transformed message, the CRCs its encryption-key, properties, user-metadata
  // and blob records will have in the output. The input verified, so each is the stored trailer
  // of the same bytes, except a Blob_Format_V1/V2 record re-written as V3, whose CRC follows by
  // linearity (crc_img.h). Null: the serializer recomputes them.
  uint32_t* in_crc;
  const uint32_t* img;
  // Speculative pass (transform_spec_*): the output is placed and the verify pass copies the
  // records into it before the CRCs are known. xstatus (nullable) takes the transform's own bits
  // (NOT_PUT / BAD_RECORD / NO_ROOM) instead of status; job_off / copy_off are the verify jobs
  // (5m, slot-major) and their copy destinations; fail is set when a placed message then fails
  // verification, which gates the fallback pass (gate: run only when (*gate != 0) == gate_when).
  uint32_t* xstatus;
  const uint64_t* job_off;
  uint64_t* copy_off;
  uint32_t* fail;
  uint8_t* out;
  const uint32_t* gate;
  int gate_when;
  // transform_merge_kernel only: also skip it when *gate2 == 0 (the fast path took the batch, so the
  // general path, whose bits it merges, never ran). Null: no second gate.
  const uint32_t* gate2;
  // [m] how each transformed message's stored BlobProperties payload becomes its V5 bytes
  // (record_fields.h): written by transform_describe, applied by props_fix_kernel after the
  // payload is copied into place.
  PropsFix* pfix;
};

hipError_t launch_transform_desc(const TransformArgs& a, hipStream_t s);
// msg_parse_kernel fused with transform_desc_kernel (the speculative pass): a and t describe the
// same messages.
hipError_t launch_msg_parse_desc(const MsgArgs& a, const TransformArgs& t, hipStream_t s);
hipError_t launch_transform_place(const TransformArgs& a, const uint64_t* start, hipStream_t s);
hipError_t launch_transform_jobs(const TransformArgs& a, hipStream_t s);
hipError_t launch_transform_finish(const TransformArgs& a, hipStream_t s);
hipError_t launch_transform_merge(const TransformArgs& a, hipStream_t s);
// The side-stream device verdict: *done = seq, at system scope -- unconditionally, or
// (xfail non-null) only when *xfail == 0, i.e. the transform's fast path took the batch.
hipError_t launch_xform_signal(const uint32_t* xfail, uint32_t* done, uint32_t seq, hipStream_t s);
hipError_t launch_props_fix(const TransformArgs& a, hipStream_t s);

// ---- copy-mode serialization of small messages by streaming the output (round 6)
// put_stream_kernel: a wave per message writes the whole message -- header and record heads computed,
// fields and blob gathered from their sources, trailers zero -- in 16-B output pieces (four 1 KiB wave
// loads per 4 KiB super-block of output, stores whole pieces, the two it shares with its neighbours byte
// by byte) and keeps the raw CRC of every 64-B output run (quad transpose + run_crc, as
// region_runs_kernel does) in the message's run slots. put_stream_seal_kernel: a thread per message
// assembles the header and record CRCs from those runs (region::record_crc; the partial runs at record
// ends re-read from the output) and writes the trailers. Messages longer than kStreamPutMax take the
// job path (put_layout_kernel sets *big, which gates it).
constexpr uint64_t kStreamPutMax = 6144;
constexpr uint64_t kStreamPutRuns = 100;  // run slots per message: ceil((63 + 6144) / 64) = 97, to a multiple of 4
struct StreamPutArgs {
  const ::ambrycrc_put_desc* desc;  // [m]
  uint64_t m;
  uint8_t* obase;         // the output pointer rounded down to 64 B
  uint64_t oreg0;         // output pointer - obase
  const uint8_t* fields;
  const uint8_t* blobs;
  uint32_t* rk;           // [kRunPad + m * kStreamPutRuns]: message i's run r at rk[kRunPad + i * kStreamPutRuns + r]
  const uint32_t* img;
};
size_t stream_put_rk_bytes(size_t m);
hipError_t launch_put_stream(const StreamPutArgs& a, int num_cu, hipStream_t s);
hipError_t launch_put_stream_seal(const StreamPutArgs& a, int num_cu, hipStream_t s);

hipError_t launch_put_layout(const PutArgs& a, hipStream_t s);
hipError_t launch_put_seal(const PutArgs& a, hipStream_t s);
hipError_t launch_gather_copy(const CopyArgs& a, int grid, hipStream_t s);

hipError_t launch_trailer_parse(const TrailerArgs& a, hipStream_t s);
hipError_t launch_trailer_verify(const TrailerArgs& a, hipStream_t s);

hipError_t launch_msg_parse(const MsgArgs& a, hipStream_t s);
// Region mode, pass 2: parse, record CRCs from the run sums, status (a.job_* / expected / crc unused).
hipError_t launch_region_msg(const MsgArgs& a, const RegionArgs& g, int num_cu, hipStream_t s);
// Region mode, after pass 2 (or the one-pass tail): the long records of g.lng, split over the whole
// grid, then combined (two kernels; both return at once when there are none).
hipError_t launch_region_long(const MsgArgs& a, const RegionArgs& g, int num_cu, hipStream_t s);
hipError_t launch_msg_reduce(const MsgArgs& a, hipStream_t s);

// Region mode in one pass: region_fused_kernel, one workgroup per CU over a
// contiguous share of 16 KiB groups (4 super-blocks). Its streaming waves hash the share into run
// sums (as region_runs_kernel); its processor waves take the messages whose headers lie in the
// share, 64 at a time, as soon as the share's run sums cover them, while the bytes are still in
// the caches. Messages that run past the share (or start before it) are deferred to
// region_tail_kernel, which also redoes every message when the offsets turn out unsorted (each CU
// finds its messages by binary search). ctl[0]: unsorted flag, ctl[1]: deferred count (zeroed
// before the launch); defer[m]: deferred message indices.
struct FusedArgs {
  MsgArgs a;
  RegionArgs g;
  uint64_t ngroups;  // 16 KiB groups over the region: ceil(nsb / 4)
  uint32_t* ctl;
  uint32_t* defer;
  uint32_t nproc;    // processor waves per workgroup (1..kFusedProcMax); the workgroup's last nproc waves
  // Transform fast path (launch_region_fused with copy): when every message is a clean PUT stored
  // at header V3 with canonical V5 properties and a Blob_Format_V3 record, back to back from
  // msg_off[0], the output is the region from msg_off[0] on with each header's life version and
  // CRC rewritten. The streamers copy every byte they stream to out + (position - msg_off[0]);
  // the processors (and the tail kernel, for the deferred messages) write out_off / out_len /
  // xstatus (0) and each header's new life version and CRC into patch[i], or set *xfail when a
  // message does not qualify -- the transform's general path then runs. region_patch_kernel, the
  // last launch, writes the patches into `out` when *xfail is clear: every byte of `out` is then
  // written by one kernel after the one that wrote it before, in stream order.
  uint8_t* out = nullptr;
  uint64_t out_cap = 0;
  uint64_t* out_off = nullptr;  // nullable
  uint64_t* out_len = nullptr;
  const int16_t* life = nullptr;  // nullable: the stored life versions
  uint32_t* xstatus = nullptr;
  uint32_t* xfail = nullptr;
  uint64_t* patch = nullptr;     // [m] life version | header CRC << 32 (with life only)
  uint32_t* path_out = nullptr;  // nullable: region_patch_kernel writes 1 (fast path took the batch) or 0
};
constexpr uint64_t kGroupBytes = 4 * kSuperBlock;
// A message that starts in a CU's share and ends at most this far past it is finished by that
// share's processors, its records past the share hashed straight from the bytes
// (region::record_crc_direct); one reaching further goes to region_tail_kernel.
constexpr uint64_t kDirectSpan = 65536;
// Waves per workgroup of the one-pass kernel (one workgroup per CU, its LDS): fewer waves than 16
// give each more than 128 VGPRs -- at 16 the processors' parse and record code spilled ~400
// VGPRs to scratch (r04an/ao A/B, ms per call: the copy form at 8 waves 0.663 vs 0.767 at 16 for
// 262,144 4 KiB PUTs; verify at 12 waves 0.377 / 0.367 / 0.532 vs 0.422 / 0.484 / 0.81 for 4 KiB
// / 1 KiB / 100-B blobs).
constexpr int kFusedWavesVerify = AMBRY_FUSED_WAVES_VERIFY, kFusedWavesCopy = AMBRY_FUSED_WAVES_COPY;
static_assert(kFusedWavesVerify >= 4 && kFusedWavesVerify <= 16 && kFusedWavesCopy >= 4 && kFusedWavesCopy <= 16,
              "one-pass workgroups: 4 to 16 waves (16 run-sum buffers in LDS)");
// Processor waves per workgroup (the rest stream): chosen per call from the messages per CU
// (fused_proc_waves, ambrycrc.cpp); AMBRY_FUSED_PROC > 0 or AMBRYCRC_FUSED_PROC fixes it (A/B),
// at most the workgroup's waves less two.
constexpr int kFusedProcMax = 12;
hipError_t launch_region_fused(const FusedArgs& f, int num_cu, hipStream_t s);  // f.out set: the copy form

hipError_t launch_plan(const PlanArgs& a, hipStream_t s);
// grid: workgroups of the persistent sweep; num_cu: the device's CUs (the A/B split group kernel
// sizes its own grid from it)
hipError_t launch_sweep(const SweepArgs& a, int grid, int num_cu, int variant, hipStream_t s);
hipError_t launch_sweep_copy(const SweepArgs& a, int grid, int num_cu, int variant, hipStream_t s);
#ifdef AMBRY_AB_SPLIT_GROUP
// The separate group kernel (tools/probes/group_kernels.hip) on num_cu CUs (it sizes its own grid).
hipError_t launch_group(const SweepArgs& a, int num_cu, hipStream_t s);
#endif
hipError_t launch_verify(const uint32_t* crc, const uint32_t* expected, uint8_t* mismatch, uint32_t* count,
                         uint32_t n, hipStream_t s);
hipError_t launch_readbw(const uint8_t* base, uint64_t nbytes, uint32_t* out, int grid, int variant,
                         hipStream_t s);
hipError_t launch_fill(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off, hipStream_t s);

}  // namespace ambrycrc
