// region_proc.h -- the message processors of region mode: one lane per message,
// a wave per 64 messages. A lane parses its message (msg_parse.h, properties read from memory) and
// assembles each record's CRC from the 64-B run sums (region_crc.h); a record longer than
// kLongRuns runs is taken by the whole wave (record_crc_runs_wave, region_crc.h), so one 4 MiB blob
// in a region of small messages costs the wave ~1,000 folds instead of one lane ~65,000 dependent
// Horner steps.
//
// Used by region_fused_kernel (crc32_kernels.hip), whose processor waves run beside its streaming
// waves and take the messages of their CU's share as the share's run sums complete, and by
// region_tail_kernel, which takes the messages the fused kernel deferred (or all of them when the
// offsets were not sorted) once every run sum exists.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32_gf2.h"
#include "crc_img.h"
#include "msg_parse.h"
#include "region_crc.h"

namespace ambrycrc {
namespace region {


__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}

template <int LVL>
__device__ __forceinline__ uint32_t wave_fold(uint32_t s, uint32_t c, uint32_t lane) {
  const uint32_t sh = gf2_mul(left_partner<LVL>(s), c);
  return (lane & (1u << LVL)) ? (s ^ sh) : s;
}

// ---- the whole wave on one short record straight from the region's bytes (no run sums)
// Used by region_tail_kernel's wave-per-message path: a deferred message's records are hashed by
// the wave from memory in one or two round trips, where one lane walking the run sums needs ~20
// dependent loads per message (69 us of tail per 262,144-message transform). The LDS sets (dn):
// stage_direct_nib (region_crc.h).

// Bytes [sh, sh + 16) of w0 || w1, sh wave-uniform.
__device__ __forceinline__ u32x4 funnel_bytes(const u32x4& w0, const u32x4& w1, uint32_t sh) {
  const uint32_t r = sh & 3u;
  switch (sh >> 2) {
    case 0:
      return u32x4{__builtin_amdgcn_alignbyte(w0.y, w0.x, r), __builtin_amdgcn_alignbyte(w0.z, w0.y, r),
                   __builtin_amdgcn_alignbyte(w0.w, w0.z, r), __builtin_amdgcn_alignbyte(w1.x, w0.w, r)};
    case 1:
      return u32x4{__builtin_amdgcn_alignbyte(w0.z, w0.y, r), __builtin_amdgcn_alignbyte(w0.w, w0.z, r),
                   __builtin_amdgcn_alignbyte(w1.x, w0.w, r), __builtin_amdgcn_alignbyte(w1.y, w1.x, r)};
    case 2:
      return u32x4{__builtin_amdgcn_alignbyte(w0.w, w0.z, r), __builtin_amdgcn_alignbyte(w1.x, w0.w, r),
                   __builtin_amdgcn_alignbyte(w1.y, w1.x, r), __builtin_amdgcn_alignbyte(w1.z, w1.y, r)};
    default:
      return u32x4{__builtin_amdgcn_alignbyte(w1.x, w0.w, r), __builtin_amdgcn_alignbyte(w1.y, w1.x, r),
                   __builtin_amdgcn_alignbyte(w1.z, w1.y, r), __builtin_amdgcn_alignbyte(w1.w, w1.z, r)};
  }
}

// zlib CRC-32 of the len bytes at base-relative pa, by the whole wave (every lane the same pa, len)
// from the region's bytes: 64-B runs aligned to the record's end; in round v lane l takes run
// R - 64(V - v) + l (runs before the record: zero), hashed from zero (bytes before pa zeroed, the
// first four XORed with 0xFF), folded over rounds by x^(8*4096), merged by the x^(8*64*2^k) tree:
// lane 63 ends at pb, so no un-shift. Loads are 16-B aligned blocks inside the region's first and
// last blocks (lo16 / hi16), funnel-shifted by pb mod 16.
__device__ __forceinline__ uint32_t record_crc_direct(const TabC& tc, const uint32_t* __restrict__ nib,
                                                      const uint32_t* __restrict__ dn, const RegionArgs& g,
                                                      uint64_t pa, uint64_t len, uint32_t lane) {
  if (len < 4) return record_crc(tc, nib, g.base, g.rk + kRunPad, pa, len);  // bytes (every lane)
  const int64_t pb = (int64_t)(pa + len);
  const int64_t R = (int64_t)((len + 63) >> 6), V = (R + 63) >> 6;
  const uint32_t sh = (uint32_t)(pb & 15);
  const int64_t lo16 = (int64_t)g.lo16, hi16 = (int64_t)g.hi16;
  const int ni = 4;
  uint32_t acc = 0;
  for (int64_t v = 0; v < V; ++v) {
    const int64_t j = R - 64 * (V - v) + (int64_t)lane;  // run index from the record's first
    uint32_t c = 0;
    if (j >= 0) {
      const int64_t o = pb - 64 * (R - j);  // the run's start (may precede pa)
      u32x4 blk[5];
#pragma unroll
      for (int b = 0; b < 5; ++b) {
        int64_t bo = o - (int64_t)sh + 16 * b;
        bo = bo < lo16 ? lo16 : (bo > hi16 ? hi16 : bo);
        blk[b] = *reinterpret_cast<const u32x4*>(g.base + bo);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u32x4 w = funnel_bytes(blk[q], blk[q + 1], sh);
        const int lo = (int)((int64_t)pa - (o + 16 * q));  // record bytes start at piece offset lo
        if (lo > 0) {
          w.x &= keep_ge(lo);
          w.y &= keep_ge(lo - 4);
          w.z &= keep_ge(lo - 8);
          w.w &= keep_ge(lo - 12);
        }
        if (lo > -4 && lo < 16) {  // zlib's initial register over the record's first four bytes
          w.x ^= keep_ge(lo) & keep_lt(lo + ni);
          w.y ^= keep_ge(lo - 4) & keep_lt(lo + ni - 4);
          w.z ^= keep_ge(lo - 8) & keep_lt(lo + ni - 8);
          w.w ^= keep_ge(lo - 12) & keep_lt(lo + ni - 12);
        }
        c = tc.step4(c ^ w.x);
        c = tc.step4(c ^ w.y);
        c = tc.step4(c ^ w.z);
        c = tc.step4(c ^ w.w);
      }
    }
    acc = nmul(dn, acc, kDirFold) ^ c;
  }
  {
    const uint32_t pt = left_partner<0>(acc);
    if (lane & 1u) acc ^= nmul(dn, pt, 0);
  }
  {
    const uint32_t pt = left_partner<1>(acc);
    if (lane & 2u) acc ^= nmul(dn, pt, 1);
  }
  {
    const uint32_t pt = left_partner<2>(acc);
    if (lane & 4u) acc ^= nmul(dn, pt, 2);
  }
  {
    const uint32_t pt = left_partner<3>(acc);
    if (lane & 8u) acc ^= nmul(dn, pt, 3);
  }
  {
    const uint32_t pt = left_partner<4>(acc);
    if (lane & 16u) acc ^= nmul(dn, pt, 4);
  }
  {
    const uint32_t pt = left_partner<5>(acc);
    if (lane & 32u) acc ^= nmul(dn, pt, 5);
  }
  return ~__builtin_amdgcn_readlane(acc, 63);
}

// ONE message by the whole wave (every lane the same i; the parse repeated in every lane, the same
// loads broadcast): short records by record_crc_direct, long ones (more than kLongRuns runs) by
// record_crc_runs_wave from the run sums.
__device__ __forceinline__ void process_message_direct(const MsgArgs& a, const RegionArgs& g,
                                                       const uint32_t* __restrict__ t, const uint32_t* __restrict__ nib,
                                                       const uint32_t* __restrict__ dn, uint64_t i, uint32_t lane,
                                                       uint32_t& st_ret, uint64_t& end_ret,
                                                       const LongList* lng = nullptr) {
  const uint32_t* rk = g.rk + kRunPad;
  const uint64_t off = a.msg_off[i];
  const bool in_region = off <= a.region_len;
  const uint64_t rem = in_region ? a.region_len - off : 0;
  const uint8_t* p = a.region + (in_region ? off : 0);
  const HeaderWords hw = load_header(p, rem);
  MsgParse r;
  PropsFields pf;
  bool pf_ok = false;
  parse_message<false, false>(off, in_region, rem, p, hw, t, nullptr, 0, r, pf, pf_ok);
  uint32_t status = r.status;
  const TabC tc{t};
#pragma unroll 1
  for (int k = 0; k < kMsgSlots; ++k) {
    uint64_t jo = 0, jl = 0;
    uint32_t ex = 0;
#pragma unroll
    for (int q = 0; q < kMsgSlots; ++q)
      if (q == k) {
        jo = r.jo[q];
        jl = r.jl[q];
        ex = r.ex[q];
      }
    if (jl == 0) continue;
    const uint64_t pa = g.reg0 + jo;
    const int64_t runs = (int64_t)((((pa + jl + 63) & ~uint64_t(63)) - (pa & ~uint64_t(63))) >> 6);
    if (runs > kLongRuns && lng && lng->ctr) {  // a multi-MiB record: the whole grid's, after this kernel
      if (list_long_wave(*lng, pa, jl, ex, i, record_bit(k), lane)) continue;
    }
    const uint32_t c = runs > kLongRuns ? record_crc_runs_wave(tc, nib, dn, g.base, rk, pa, jl, lane)
                                        : record_crc_direct(tc, nib, dn, g, pa, jl, lane);
    if (c != ex) status |= record_bit(k);
  }
  if (lane == 0) {
    a.status[i] = status;
    if (a.msg_end) a.msg_end[i] = r.end ? off + r.end : 0;
  }
  st_ret = status;
  end_ret = r.end;
}

// The message processor of one lane (message i when `have`), all run sums of its records
// available: status and message end written. Long records are collected and done by the wave
// after the per-lane ones, so every lane of the wave must call this (have = false for none).
// t: compact slice-by-4 tables (stage_slice_tables), nib: stage_nib's sets; g.rk's run sums.
// keep(pos, end): called for a parsed message whose records need CRCs (pos: its base-relative
// start, end: its length); false = the lane drops it (deferred: no status written, st_ret ~0).
// wait(need): the whole wave waits until every run up to base-relative `need` exists.
// tr: the table access of the per-lane record CRCs (TabR in the one-pass kernel, TabC elsewhere).
// direct_from (base-relative; ~0: none): a record ending past it has no run sums yet (it runs into
// the next CU's share) and is hashed by the wave straight from the region's bytes
// (record_crc_direct with dn's sets), without waiting -- so the message that straddles a share's
// end is finished by its own share's processor instead of the tail kernel.
// ENDS: the lane's own records' head / tail runs hashed right after the parse (record_ends), the
// rest after the wait (AMBRY_FUSED_ENDS: the copy form's 4 KiB PUTs 617 -> 609 us, the verify
// form's 371 -> 392 at 4 KiB blobs, profiles/r05aq_fused_ends_ab.txt).
template <bool ENDS = false, class Tab, class Keep, class Wait>
__device__ __forceinline__ void process_message(const MsgArgs& a, const RegionArgs& g,
                                                const uint32_t* __restrict__ t, const Tab& tr,
                                                const uint32_t* __restrict__ nib, bool have, uint64_t i,
                                                uint32_t lane, uint32_t& st_ret, uint64_t& end_ret, Keep keep,
                                                Wait wait, const uint32_t* __restrict__ dn,
                                                uint64_t direct_from = ~0ull) {
  const uint32_t* rk = g.rk + kRunPad;
  uint32_t status = 0;
  uint64_t end = 0, off = 0;
  uint64_t jo[kMsgSlots] = {0, 0, 0, 0, 0}, jl[kMsgSlots] = {0, 0, 0, 0, 0};
  uint32_t ex[kMsgSlots] = {0, 0, 0, 0, 0};
  uint32_t longs = 0;  // record slots left to the wave
  if (have) {
    off = a.msg_off[i];
    const bool in_region = off <= a.region_len;
    const uint64_t rem = in_region ? a.region_len - off : 0;
    const uint8_t* p = a.region + (in_region ? off : 0);
    const HeaderWords hw = load_header(p, rem);
    MsgParse r;
    PropsFields pf;
    bool pf_ok = false;
    parse_message<false, false>(off, in_region, rem, p, hw, t, nullptr, 0, r, pf, pf_ok);
    status = r.status;
    end = r.end;
#pragma unroll
    for (int k = 0; k < kMsgSlots; ++k) {
      jo[k] = r.jo[k];
      jl[k] = r.jl[k];
      ex[k] = r.ex[k];
    }
  }
  // records to CRC: the message must end inside what the caller streams, else it is deferred
  bool crcs = false;
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) crcs |= have && jl[k] != 0;
  if (crcs && !keep(g.reg0 + off, end)) {
    have = false;
    crcs = false;
  }
  // Long records are the wave's, one by one, each once the frontier passes its own end (a CU's
  // 4 MiB blobs are verified as the stream passes them, not all after it); then the lanes' own
  // records, once it passes the last of them. Unless enough lanes have a long record that the lanes
  // doing their own in parallel finish first (a lane's chain is runs/4 nibble multiplies deep; the
  // wave's per record ~runs/256 plus ~64 for the tree's gf2 shifts).
  auto runs_of = [&](int k) -> int64_t {
    const uint64_t pa = g.reg0 + jo[k];
    return (int64_t)((((pa + jl[k] + 63) & ~uint64_t(63)) - (pa & ~uint64_t(63))) >> 6);
  };
  int64_t lane_runs = 0;
  uint32_t direct = 0;  // record slots hashed straight from the bytes by the wave
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) {
    if (!have || jl[k] == 0) continue;
    if (g.reg0 + jo[k] + jl[k] > direct_from) {
      direct |= 1u << k;
    } else if (runs_of(k) > kLongRuns) {
      longs |= 1u << k;
      lane_runs += runs_of(k);
    }
  }
  {
    const int64_t per_lane = (int64_t)wave_max_u64((uint64_t)lane_runs) / 4;
    int64_t tot = lane_runs;
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);  // sum over lanes
    const int64_t wave = tot / 256 + 64 * (int64_t)__popcll(__ballot(longs != 0));
    if (per_lane <= wave) longs = 0;  // every record by its lane
  }
  longs |= direct;
  const uint32_t own_long = longs;
  // ENDS: the lane's own records' head / tail runs now, while the parse's lines are in L2
  RecEnds ends[kMsgSlots];
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) {
    ends[k] = RecEnds{0u, 0u};
    if (ENDS && have && jl[k] != 0 && !(own_long & (1u << k)))
      ends[k] = record_ends(tr, nib, g.base, g.reg0 + jo[k], jl[k]);
  }
  for (;;) {
    const uint64_t ball = __ballot(longs != 0);
    if (ball == 0) break;
    const uint32_t owner = (uint32_t)__builtin_ctzll(ball);
    const uint32_t kk = (uint32_t)__builtin_ctz(__shfl(longs, (int)owner));
    uint64_t rjo = 0, rjl = 0;
#pragma unroll
    for (int k = 0; k < kMsgSlots; ++k)
      if ((uint32_t)k == kk) {
        rjo = jo[k];
        rjl = jl[k];
      }
    rjo = __shfl(rjo, (int)owner);
    rjl = __shfl(rjl, (int)owner);
    uint32_t c;
    if (__shfl(direct, (int)owner) & (1u << kk)) {  // (wave-uniform) past the share: from the bytes
      c = record_crc_direct(TabC{t}, nib, dn, g, g.reg0 + rjo, rjl, lane);
    } else {
      wait(g.reg0 + rjo + rjl);
      c = record_crc_runs_wave(TabC{t}, nib, dn, g.base, rk, g.reg0 + rjo, rjl, lane);
    }
    if (lane == owner) {
      uint32_t e = 0;
#pragma unroll
      for (int k = 0; k < kMsgSlots; ++k)
        if ((uint32_t)k == kk) e = ex[k];
      if (c != e) status |= record_bit((int)kk);
      longs &= ~(1u << kk);
    }
  }
  uint64_t need = 0;  // base-relative end of the lane's last own record
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k)
    if (have && jl[k] != 0 && !(own_long & (1u << k)) && g.reg0 + jo[k] + jl[k] > need) need = g.reg0 + jo[k] + jl[k];
  wait(wave_max_u64(need));
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) {
    if (!have || jl[k] == 0 || (own_long & (1u << k))) continue;
    const uint32_t c = ENDS ? record_crc_from_ends(nib, rk, g.reg0 + jo[k], jl[k], ends[k])
                            : record_crc(tr, nib, g.base, rk, g.reg0 + jo[k], jl[k]);
    if (c != ex[k]) status |= record_bit(k);
  }
  if (have) {
    a.status[i] = status;
    if (a.msg_end) a.msg_end[i] = end ? off + end : 0;
  }
  st_ret = have ? status : ~0u;
  end_ret = end;
}


// The transform's fast path for message i (FusedArgs::out; verify status st, end `end`): a clean
// PUT at header V3 with canonical V5 properties and a Blob_Format_V3 record, followed directly by
// message i + 1, transforms to its own bytes with the life version rewritten
// (ValidatingTransformer.java:86-95: PutMessageFormatInputStream over the deserialized fields gives
// back the same records, their CRCs unchanged) -- the streamers copy those bytes to
// out + (offset - msg_off[0]); this records the header's new life version and CRC in patch[i]
// (applied by region_patch_kernel once the copy is complete) and writes the outputs.
// Anything else sets *xfail: the general path then redoes the whole batch.
// In two steps: transform_fast_pre reads the message's shape (header, properties, blob record
// version) and computes the patch -- the one-pass kernel calls it right after the parse, while
// those lines are in L2, instead of after the wait for the run sums -- and transform_fast_post
// decides with the verify status.
struct FastPre {
  bool ok;
  uint64_t patch;
};
__device__ __forceinline__ FastPre transform_fast_pre(const FusedArgs& f, const uint32_t* __restrict__ t, uint64_t i,
                                                      uint64_t end) {
  const MsgArgs& a = f.a;
  const uint64_t off = a.msg_off[i];
  FastPre r{false, 0};
  // not verified yet: every read below stays inside the message's parsed extent
  if (off > a.region_len || a.region_len - off < end || end < 40) return r;
  const uint8_t* p = a.region + off;
  HeaderWords hw = load_header(p, 40);
  if (be16(p) != 3) return r;
  int32_t rel[kMsgSlots];
#pragma unroll
  for (int k = 0; k < kMsgSlots; ++k) rel[k] = (int32_t)be32_w0(hw, 3 + k);
  bool ok = rel[2] == -1 && rel[1] >= 0 && rel[3] >= 0 && rel[4] >= 0 && (int64_t)rel[3] >= (int64_t)rel[1] + 10 &&
            (uint64_t)rel[3] <= end && (uint64_t)rel[4] + 2 <= end;
  if (ok) ok = be16(p + rel[4]) == 3;
  if (ok) {  // properties already canonical VERSION_5 bytes, every string ASCII (record_fields.h)
    const uint32_t stored = (uint32_t)(rel[3] - rel[1] - 10);
    PropsFields pf;
    ok = props_parse<true>(p + rel[1] + 2, stored, &pf) == 0 && pf.ascii && props_fix_of(pf, stored).version == 0;
  }
  if (ok && f.life && f.life[i] < 0) ok = false;  // not a life version a V3 header holds
  if (ok && f.life) {  // the index's life version (MessageInfo.getLifeVersion), header CRC recomputed
    const uint32_t lv = (uint16_t)f.life[i];
    hw.w[0] = (hw.w[0] & 0xFFFFu) | (((lv >> 8) | ((lv & 0xFFu) << 8)) << 16);
    r.patch = (uint64_t)lv | ((uint64_t)header_crc(hw, 32, t) << 32);
  }
  r.ok = ok;
  return r;
}

__device__ __forceinline__ void transform_fast_post(const FusedArgs& f, bool have, uint64_t i, uint32_t st,
                                                    uint64_t end, FastPre pre) {
  if (!have || st == ~0u) return;  // no message, or deferred to the tail kernel
  const MsgArgs& a = f.a;
  const uint64_t off = a.msg_off[i], off0 = a.msg_off[0];
  const bool ok = pre.ok && st == 0 && end != 0 && off >= off0 && off - off0 + end <= f.out_cap &&
                  (i + 1 == a.m || a.msg_off[i + 1] == off + end);
  if (!ok) {
    atomicOr(f.xfail, 1u);
    return;
  }
  // region_patch_kernel writes the patch into `out` after the copy has completed (kernel order, no
  // store-ordering argument between this wave and the waves copying the header's bytes)
  if (f.life) f.patch[i] = pre.patch;
  if (f.out_off) f.out_off[i] = off - off0;
  f.out_len[i] = end;
  f.xstatus[i] = 0;
}

__device__ __forceinline__ void transform_fast(const FusedArgs& f, const uint32_t* __restrict__ t, bool have,
                                               uint64_t i, uint32_t st, uint64_t end) {
  if (!have || st == ~0u) return;
  const FastPre pre = st == 0 && end != 0 ? transform_fast_pre(f, t, i, end) : FastPre{false, 0};
  transform_fast_post(f, have, i, st, end, pre);
}

}  // namespace region
}  // namespace ambrycrc
