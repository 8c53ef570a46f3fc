// crc32_layout.h -- byte layout of the per-CU LDS image used by the gfx950
// kernels, built once per device on the host (ambrycrc.cpp) and copied into LDS
// by every workgroup of the persistent grid.
//
//  [0, 128 KiB)   SLICE: byte tables T0..T3 of slice-by-4, replicated 32x so that
//                 a ds_read_b32 with 32 random byte indices per lane group is
//                 bank-conflict free. Entry (table j, byte b, lane l) lives at
//                     ((j >> 1) << 16) | (b << 8) | ((j & 1) << 7) | ((l & 31) << 2)
//                 i.e. byte b sits in address bits 8..15, so ONE v_perm_b32
//                 builds the address from the CRC state and a per-lane constant.
//  [128 KiB, ...) NIBBLE tables (16 entries x 8 positions = 512 B per constant,
//                 16 entries span 16 distinct banks -> conflict-free, unreplicated):
//                   FOLD          x^(8*1024)        advance a lane stream one 1 KiB block
//                   TREE[l]       x^(8*16*2^l)      wave combine, l = 0..5
//                   POW[k]        x^(8*2^k)         arbitrary shifts, k = 0..kPowTables-1
#pragma once
#include <stdint.h>

namespace ambrycrc {

constexpr uint32_t kSliceBytes = 128u * 1024u;
constexpr uint32_t kNibBase = kSliceBytes;  // absolute LDS byte address of nibble area
constexpr uint32_t kNibSetBytes = 512u;     // one constant: 8 positions x 16 x 4 B
constexpr uint32_t kFoldOff = 0;            // offsets relative to kNibBase
constexpr uint32_t kTreeOff = kFoldOff + kNibSetBytes;
constexpr uint32_t kTreeLevels = 6;
constexpr uint32_t kPowOff = kTreeOff + kTreeLevels * kNibSetBytes;
constexpr uint32_t kPowTables = 36;  // shifts up to 2^36 - 1 bytes from tables; beyond: slow path
constexpr uint32_t kLdsBytes = kNibBase + kPowOff + kPowTables * kNibSetBytes;
static_assert(kLdsBytes <= 160u * 1024u, "LDS image must fit one CU (160 KiB)");
static_assert(kPowOff + kPowTables * kNibSetBytes < 65536u, "nibble offsets must fit ds_read offset");

// The global image (not staged by the sweep): kLdsBytes of LDS image, 64 words x^(8*2^k), then
// the nibble sets of x^(-8*2^k), k = 0..kInvPowSets-1 (region mode's final un-shift,
// region_crc.h).
constexpr uint32_t kImgInvOff = kLdsBytes + 256u;
constexpr uint32_t kInvPowSets = 6;
// Then region pass 2's words (region_crc.h Aux, staged by region_msg_kernel): H0[lo] (64 words:
// the raw register at a 64-B run's end of 0xFF in bytes [lo, lo + min(64 - lo, 4)), i.e. the
// initial register of a record starting at run offset lo, by linearity), GE[a] = the bytes >= a
// of a word and LT[b] = the bytes < b (a, b = 0..4; 8 words each), then the byte tables of
// x^(8*256): B[256j + b] = (b << 8j) * x^(8*256), j = 0..3, then 16 nibble sets for the final
// un-shift by x^(-8d), d = 0..63, in two multiplies: x^(-8 d0) (d0 = 0..7), then x^(-64 d1).
constexpr uint32_t kImgRegOff = kImgInvOff + kInvPowSets * kNibSetBytes;
constexpr uint32_t kRegH0 = 0, kRegGe = 64, kRegLt = 72, kRegAuxWords = 80;
constexpr uint32_t kRegByteWords = 1024;
constexpr uint32_t kRegUnSets = 16, kRegUnWords = kRegUnSets * (kNibSetBytes / 4);
constexpr uint32_t kRegWords = kRegAuxWords + kRegByteWords + kRegUnWords;
constexpr uint32_t kImgBytes = kImgRegOff + 4u * kRegWords;

constexpr uint32_t kBlockBytes = 1024;  // one wave-wide 16 B/lane load
constexpr uint32_t kWaveLanes = 64;

}  // namespace ambrycrc
