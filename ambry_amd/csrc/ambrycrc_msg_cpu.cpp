// ambrycrc_msg_cpu.cpp -- one stored message on the CPU: deserializeBlobAll's checks
// (MessageFormatRecord.java:257-303) and ValidatingTransformer.transform
// (ValidatingTransformer.java:46-104), for the per-message callers (a GET of one blob, a
// replication thread transforming one message) that a device batch does not fit. The
// semantics and status bits are ambrycrc_verify_messages_dev's and
// ambrycrc_transform_messages_dev's (message_kernels.hip); the CRCs run through the CLMUL
// host loop (ambrycrc_update).
#include "../../include/ambrycrc.h"

#include <string.h>

#include "put_layout.h"
#include "record_fields.h"

namespace {

uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }
uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) << 32 | rd32(p + 4); }

constexpr uint32_t kRecordBit[5] = {AMBRYCRC_MSG_ENCKEY_CRC, AMBRYCRC_MSG_PROPS_CRC, AMBRYCRC_MSG_UPDATE_CRC,
                                    AMBRYCRC_MSG_USERMETA_CRC, AMBRYCRC_MSG_BLOB_CRC};

// The record-level reads of each deserializer before its CRC (message_kernels.hip record_check).
uint32_t record_check(int k, const uint8_t* q, uint64_t span) {
  if (span < 10) return AMBRYCRC_MSG_BAD_RECORD;
  const uint32_t v = rd16(q);
  switch (k) {
    case 0:
    case 3: {
      if (v != 1) return AMBRYCRC_MSG_BAD_VERSION;
      if (span < 14) return AMBRYCRC_MSG_BAD_RECORD;
      const int32_t n = (int32_t)rd32(q + 2);
      return n >= 0 && (uint64_t)n + 14 == span ? 0u : AMBRYCRC_MSG_BAD_RECORD;
    }
    case 1:
      return ambrycrc::props_record_check(q, span);
    case 2:
      return ambrycrc::update_record_check(q, span);
    default: {
      if (v < 1 || v > 3) return AMBRYCRC_MSG_BAD_VERSION;
      const uint32_t head = v == 1 ? 10u : v == 2 ? 12u : 13u;
      if (span < head + 8) return AMBRYCRC_MSG_BAD_RECORD;
      const uint32_t type = v == 1 ? 0u : rd16(q + 2);
      const uint64_t size = rd64(q + (v == 1 ? 2 : v == 2 ? 4 : 5));
      return type < 2 && size <= 0x7FFFFFFFull && size + head + 8 == span ? 0u : AMBRYCRC_MSG_BAD_RECORD;
    }
  }
}

struct Parsed {
  uint32_t version, hsize, life;
  int64_t total;
  int32_t rel[5];  // encryption key, properties, update, user metadata, blob; -1 absent
  uint64_t end;    // message end, relative
};

// Header and every record of the message at p (rem bytes available): status bits.
uint32_t verify(const uint8_t* p, uint64_t rem, Parsed* m) {
  m->end = 0;
  if (rem < 2) return AMBRYCRC_MSG_BAD_LAYOUT;
  const int v = (int16_t)rd16(p);
  const uint32_t h = v == 1 ? 34u : v == 2 ? 38u : v == 3 ? 40u : 0u;
  if (h == 0) return AMBRYCRC_MSG_BAD_VERSION;
  if (rem < h) return AMBRYCRC_MSG_BAD_LAYOUT;
  if ((uint64_t)ambrycrc_update(0, p, h - 8) != rd64(p + h - 8)) return AMBRYCRC_MSG_HEADER_CRC;  // verifyHeader
  m->version = (uint32_t)v;
  m->hsize = h;
  m->life = 0;
  if (v == 3) {
    if ((int16_t)rd16(p + 2) < 0) return AMBRYCRC_MSG_BAD_LAYOUT;  // checkHeaderConstraints
    m->life = rd16(p + 2);
    m->total = (int64_t)rd64(p + 4);
    for (int k = 0; k < 5; ++k) m->rel[k] = (int32_t)rd32(p + 12 + 4 * k);
  } else {
    m->total = (int64_t)rd64(p + 2);
    const uint8_t* q = p + 10;
    if (v == 1) {
      m->rel[0] = -1;
      for (int k = 0; k < 4; ++k) m->rel[k + 1] = (int32_t)rd32(q + 4 * k);
    } else {
      for (int k = 0; k < 5; ++k) m->rel[k] = (int32_t)rd32(q + 4 * k);
    }
  }
  const int32_t* rel = m->rel;
  const bool is_put = rel[1] != -1 && rel[2] == -1 && rel[3] != -1 && rel[4] != -1;
  const bool is_upd = rel[2] != -1 && rel[0] == -1 && rel[1] == -1 && rel[3] == -1 && rel[4] == -1;
  if (m->total <= 0 || !(is_put || is_upd)) return AMBRYCRC_MSG_BAD_LAYOUT;
  int64_t prev = -1, first = -1;
  for (int k = 0; k < 5; ++k) {
    if (rel[k] == -1) continue;
    if (rel[k] <= prev || rel[k] < (int32_t)h) return AMBRYCRC_MSG_BAD_LAYOUT;
    if (first < 0) first = rel[k];
    prev = rel[k];
  }
  if ((uint64_t)m->total > rem || (uint64_t)first > rem - (uint64_t)m->total) return AMBRYCRC_MSG_BAD_LAYOUT;
  const uint64_t end = (uint64_t)first + (uint64_t)m->total;
  uint64_t rend[5];
  for (int k = 0; k < 5; ++k) {
    rend[k] = end;
    for (int j = k + 1; j < 5; ++j)
      if (rel[j] != -1) {
        rend[k] = (uint64_t)rel[j];
        break;
      }
    if (rel[k] != -1 && rend[k] < (uint64_t)rel[k] + 8) return AMBRYCRC_MSG_BAD_LAYOUT;
  }
  uint32_t status = 0;
  for (int k = 0; k < 5; ++k) {
    if (rel[k] == -1) continue;
    const uint8_t* q = p + rel[k];
    const uint64_t span = rend[k] - (uint64_t)rel[k];
    if ((uint64_t)ambrycrc_update(0, q, span - 8) != rd64(q + span - 8)) status |= kRecordBit[k];
    status |= record_check(k, q, span);
  }
  m->end = end;
  return status;
}

// ValidatingTransformer.transform of one message, split for the batch: transform_plan verifies the
// message and decides its output (status, length, and how to write it) without writing; transform_emit
// writes it. The batch plans every message, places them by one prefix sum and emits each straight
// into the output, with no scratch copy.
struct XPlan {
  uint64_t len = 0;      // output bytes
  bool fast = false;     // the message's own bytes, life version and header CRC rewritten
  int life = -1;         // fast: the life version to write, as the header's 16 bits (-1: keep the stored one)
  ambrycrc_put_desc d;   // general: the re-serialization
  ambrycrc::PropsFix fx;
};

// have_life: write life_version into the new header as given -- a batch's index value, negatives
// included (MessageInfo.LIFE_VERSION_FROM_FRONTEND is -1; ValidatingTransformer.java:90 writes
// msgInfo.getLifeVersion() unchanged, as the device batch does); otherwise keep the stored one.
uint32_t transform_plan(const uint8_t* region, uint64_t region_len, uint64_t off, bool have_life, int life_version,
                        int header_version, XPlan* x) {
  Parsed m;
  m.end = 0;
  const uint32_t st = off <= region_len ? verify(region + off, region_len - off, &m) : (uint32_t)AMBRYCRC_MSG_BAD_LAYOUT;
  if (st) return st;
  const uint8_t* p = region + off;
  const int32_t enc = m.rel[0], bp = m.rel[1], upd = m.rel[2], um = m.rel[3], blob = m.rel[4];
  if (upd != -1 || bp == -1 || um == -1 || blob == -1) return AMBRYCRC_MSG_NOT_PUT;  // "cannot be anything rather than put record"
  // the deserializers' field reads (deserializeBlobEncryptionKey / Properties / UserMetadata / Blob,
  // MessageFormatRecord.java:1568-1833); verify's record checks already hold for them
  const int64_t first = enc != -1 ? enc : bp;
  const uint32_t bv = rd16(p + blob);
  const uint32_t head = bv == 1 ? 10u : bv == 2 ? 12u : 13u;
  // deserializeBlobProperties, re-serialized at VERSION_5 (record_fields.h; verify parsed it)
  const uint32_t stored = (uint32_t)(um - bp - 2 - 8);
  ambrycrc::PropsFields pf;
  if (ambrycrc::props_parse<true>(p + bp + 2, stored, &pf) != 0) return AMBRYCRC_MSG_BAD_RECORD;
  if (!pf.ascii) return AMBRYCRC_MSG_NOT_ENCODABLE;
  x->fx = ambrycrc::props_fix_of(pf, stored);
  // A V3 message with a V3 blob record and properties already canonical VERSION_5 bytes re-serializes
  // at V3 to its own bytes but for the life version and the header CRC (the GPU fast path's rule,
  // region_proc.h transform_fast): one copy and the 32-byte header's CRC, instead of the layout,
  // copy and every record CRC again.
  if (header_version == 3 && m.version == 3 && bv == 3 && x->fx.version == 0) {
    x->fast = true;
    x->len = m.end;
    x->life = have_life && (uint32_t)(uint16_t)life_version != m.life ? (int)(uint16_t)life_version : -1;
    return 0;
  }
  ambrycrc_put_desc& d = x->d;
  memset(&d, 0, sizeof d);
  const bool keep_enc = enc != -1 && header_version >= 2;
  d.out_off = 0;
  d.key_src = off + m.hsize;
  d.key_len = (uint32_t)(first - m.hsize);
  d.enckey_src = keep_enc ? off + enc + 6 : 0;
  d.enckey_len = keep_enc ? (int32_t)rd32(p + enc + 2) : -1;
  d.props_src = off + bp + 2;
  d.props_len = ambrycrc::props_v5_len(x->fx);
  d.usermeta_src = off + um + 6;
  d.usermeta_len = rd32(p + um + 2);
  d.blob_src = off + blob + head;
  d.blob_len = rd64(p + blob + (bv == 1 ? 2 : bv == 2 ? 4 : 5));
  d.life_version = (int16_t)(have_life ? life_version : (int)m.life);
  d.blob_type = (int16_t)(bv == 1 ? 0u : rd16(p + blob + 2));
  d.compressed = (uint8_t)(bv == 3 && p[blob + 4] == 1 ? 1 : 0);
  d.header_version = (uint8_t)header_version;
  x->len = ambrycrc_put_layout(&d, nullptr);
  return x->len ? 0u : (uint32_t)AMBRYCRC_MSG_BAD_RECORD;
}

// Writes the planned message at out (x.len bytes of room).
int transform_emit(const uint8_t* region, uint64_t off, const XPlan& x, uint8_t* out) {
  if (x.fast) {
    memcpy(out, region + off, x.len);
    if (x.life >= 0) {
      ambrycrc::put_be16(out + 2, (uint32_t)x.life);
      ambrycrc::put_be64(out + 32, (uint64_t)ambrycrc_update(0, out, 32));
    }
    return AMBRYCRC_OK;
  }
  // the stored payload is copied (props_len bytes from props_src: the appendix's share of them comes
  // from the user-metadata record that follows, inside the message), then rewritten as V5 and its
  // record CRC recomputed
  const int rc = ambrycrc_serialize_put_host(&x.d, region, region, out, x.len, nullptr);
  if (rc) return rc;
  if (x.fx.version) {
    uint64_t fo[5];
    ambrycrc_put_layout(&x.d, fo);
    uint8_t* rec = out + fo[2] - 2;
    ambrycrc::props_apply_fix(rec + 2, x.fx);
    ambrycrc::put_be64(rec + 2 + x.d.props_len, (uint64_t)ambrycrc_update(0, rec, 2ull + x.d.props_len));
  }
  return AMBRYCRC_OK;
}

}  // namespace

extern "C" {

int ambrycrc_verify_message_cpu(const uint8_t* region, uint64_t region_len, uint64_t off, uint32_t* status,
                                uint64_t* msg_end) {
  if (!region || !status) return AMBRYCRC_EINVAL;
  Parsed m;
  *status = off <= region_len ? verify(region + off, region_len - off, &m) : (uint32_t)AMBRYCRC_MSG_BAD_LAYOUT;
  if (msg_end) *msg_end = off <= region_len && m.end ? off + m.end : 0;
  return AMBRYCRC_OK;
}

int ambrycrc_transform_message_cpu(const uint8_t* region, uint64_t region_len, uint64_t off, int life_version,
                                   int header_version, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                                   uint32_t* status) {
  if (!region || !out_len || !status || header_version < 1 || header_version > 3 || life_version > 32767)
    return AMBRYCRC_EINVAL;
  *out_len = 0;
  XPlan x;
  *status = transform_plan(region, region_len, off, life_version >= 0, life_version, header_version, &x);
  if (*status) return AMBRYCRC_OK;
  if (!out || x.len > out_cap) {
    *status = AMBRYCRC_MSG_NO_ROOM;
    return AMBRYCRC_OK;
  }
  const int rc = transform_emit(region, off, x, out);
  if (rc) return rc;
  *out_len = x.len;
  return AMBRYCRC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- CPU batch forms
// The host entries' CPU leg (ambrycrc_set_host_policy; DESIGN.md §5 "host-resident dispatch"):
// ambrycrc_verify_messages_host / _transform_messages_host over messages in host memory, split
// across `threads` CPU threads by region bytes, each message through the single-message loops
// above. Same outputs as the device batch.
#include <algorithm>
#include <atomic>
#include <thread>
#include <memory>
#include <new>
#include <vector>

#include "ambrycrc_ctx.h"

namespace ambrycrc {
namespace detail {

namespace {
// fn(a, b) over contiguous index ranges of [0, m) holding about equal sums of weight(i).
template <class W, class F>
void split_run(size_t m, int threads, W weight, F fn) {
  threads = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), m));
  if (threads == 1) {
    fn((size_t)0, m);
    return;
  }
  std::vector<uint64_t> pre(m + 1, 0);
  for (size_t i = 0; i < m; ++i) pre[i + 1] = pre[i] + weight(i) + 64;  // + a per-message cost
  std::vector<size_t> cut(threads + 1, m);
  cut[0] = 0;
  for (int t = 1; t < threads; ++t)
    cut[t] = (size_t)(std::lower_bound(pre.begin(), pre.end(), pre[m] * (uint64_t)t / (uint64_t)threads) - pre.begin());
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) {
    if (cut[t] >= cut[t + 1]) continue;
    try {
      th.emplace_back(fn, cut[t], cut[t + 1]);
    } catch (...) {  // no thread (the C ABI does not throw): the part runs here
      fn(cut[t], cut[t + 1]);
    }
  }
  fn(cut[0], cut[1]);
  for (auto& x : th) x.join();
}

uint64_t extent_of(const uint8_t* region, uint64_t region_len, uint64_t off) {
  return off >= region_len ? 0 : message_extent_of(region + off, region_len - off);
}
}  // namespace

int verify_messages_cpu(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                        uint32_t* status, uint64_t* msg_end, int threads) {
  std::atomic<int> rc{AMBRYCRC_OK};  // written by any worker
  split_run(m, threads, [&](size_t i) { return extent_of(region, region_len, msg_off[i]); },
            [&](size_t a, size_t b) {
              for (size_t i = a; i < b; ++i) {
                uint64_t e = 0;
                if (ambrycrc_verify_message_cpu(region, region_len, msg_off[i], &status[i], &e) != AMBRYCRC_OK)
                  rc.store(AMBRYCRC_EINVAL);
                if (msg_end) msg_end[i] = e;
              }
            });
  return rc.load();
}

int transform_messages_cpu(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                           const int16_t* life_version, int header_version, uint8_t* out, uint64_t out_cap,
                           uint64_t* out_off, uint64_t* out_len, uint32_t* status, int threads) {
  // every message planned in parallel (verified, its output length known), placed in message order
  // as the device batch packs it (NO_ROOM once the running sum passes out_cap), then emitted in
  // parallel straight into `out` (round 5's first form transformed into a scratch copy of the region
  // and packed it after: two more passes over the bytes and a fresh allocation's page faults)
  std::vector<XPlan> plan(m);
  split_run(m, threads, [&](size_t i) { return extent_of(region, region_len, msg_off[i]); }, [&](size_t a, size_t b) {
    for (size_t i = a; i < b; ++i)
      status[i] = transform_plan(region, region_len, msg_off[i], life_version != nullptr,
                                 life_version ? life_version[i] : 0, header_version, &plan[i]);
  });
  std::vector<uint64_t> pos(m, ~0ull);  // output position, ~0: not placed
  uint64_t vpos = 0;
  for (size_t i = 0; i < m; ++i) {
    if (status[i] == 0 && plan[i].len) {
      if (vpos + plan[i].len <= out_cap)
        pos[i] = vpos;
      else
        status[i] = AMBRYCRC_MSG_NO_ROOM;
      vpos += plan[i].len;
    }
    if (out_off) out_off[i] = pos[i];
    out_len[i] = pos[i] == ~0ull ? 0 : plan[i].len;
  }
  std::atomic<int> rc{AMBRYCRC_OK};  // written by any worker
  split_run(m, threads, [&](size_t i) { return pos[i] == ~0ull ? 0 : plan[i].len; }, [&](size_t a, size_t b) {
    for (size_t i = a; i < b; ++i)
      if (pos[i] != ~0ull && transform_emit(region, msg_off[i], plan[i], out + pos[i]) != AMBRYCRC_OK)
        rc.store(AMBRYCRC_EINVAL);
  });
  return rc.load();
}

}  // namespace detail
}  // namespace ambrycrc
