// ambrycrc_put.cpp -- write side of the message path: lay out PUT messages
// and fill every CRC trailer, on the CPU for one message (ambrycrc_serialize_put_host) and on the
// GPU for a batch (ambrycrc_serialize_puts_dev). Layout: put_layout.h.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/ambrycrc.h"
#include "ambrycrc_ctx.h"
#include "crc32_kernels.h"
#include "put_layout.h"
#include "record_fields.h"

using namespace ambrycrc;
using namespace ambrycrc::detail;

namespace {

// Workspace of a device batch of m messages: copy jobs (src, dst, len, cost) and CRC jobs (off, len,
// crc, crc_in) of 5 per message, then one batch workspace shared by the copy plan and the CRC batch
// (both run on the same stream, one after the other).
size_t put_jobs_bytes(size_t m) {
  const size_t j = (size_t)kPutSlots * m;
  return (j * (4 * sizeof(uint64_t) + 2 * sizeof(uint64_t) + 2 * sizeof(uint32_t)) + 255) & ~size_t(255);
}

// The job path's workspace (copy and CRC jobs, the batch workspace, the streamed form's `big` word);
// ambrycrc_serialize_puts_workspace_bytes adds the streamed form's run slots after it (the transform,
// which never streams, uses this much).
size_t put_core_bytes(size_t m) { return put_jobs_bytes(m) + ws_need((size_t)kPutSlots * m) + 256; }

// A transform's own workspace: descriptors, the scan's per-message output, in_crc (4 per message),
// the speculative pass's xstatus, its fail flag, the verify jobs' copy destinations (5 per message)
// and the properties re-encodings (one PropsFix per message).
size_t transform_head_bytes(size_t m) {
  return (m * (sizeof(ambrycrc_put_desc) + 6 * sizeof(uint32_t)) + 8 + 15) & ~size_t(15);
}
size_t transform_own_bytes(size_t m) {
  return (transform_head_bytes(m) + (size_t)kPutSlots * m * sizeof(uint64_t) + m * sizeof(PropsFix) + 255) &
         ~size_t(255);
}

}  // namespace

namespace ambrycrc {
namespace detail {

int enqueue_serialize(DevCtx* c, const ::ambrycrc_put_desc* d_desc, size_t m, const uint8_t* d_fields,
                      const uint8_t* d_blobs, uint8_t* d_out, uint64_t* d_msg_len, void* d_ws, hipStream_t stream,
                      const uint32_t* d_in_crc, bool layout_only, const uint32_t* gate, const PropsFix* pfix,
                      bool stream_ok) {
  const size_t j = (size_t)kPutSlots * m;
  uint8_t* w = static_cast<uint8_t*>(d_ws);
  PutArgs a;
  a.desc = d_desc;
  a.m = m;
  a.out = d_out;
  a.fields = d_fields;
  a.blobs = d_blobs;
  a.cp_src = reinterpret_cast<uint64_t*>(w);
  a.cp_dst = a.cp_src + j;
  a.cp_len = a.cp_dst + j;
  a.cp_cost = a.cp_len + j;
  a.crc_off = a.cp_cost + j;
  a.crc_len = a.crc_off + j;
  uint32_t* crc = reinterpret_cast<uint32_t*>(a.crc_len + j);
  a.crc = crc;
  a.crc_in = crc + j;
  a.msg_len = d_msg_len;
  a.in_crc = d_in_crc;
  a.img = c->d_img;
  a.copy_through = (d_fields || d_blobs) && !d_in_crc;
  a.gate = gate;
  a.src_base = 0;
  if (a.copy_through) {  // every source lies in fields, blobs or (a slot in place) the output
    uintptr_t lo = UINTPTR_MAX;
    if (d_fields) lo = std::min(lo, (uintptr_t)d_fields);
    if (d_blobs) lo = std::min(lo, (uintptr_t)d_blobs);
    if (!d_fields || !d_blobs) lo = std::min(lo, (uintptr_t)d_out);
    a.src_base = (uint64_t)lo & ~uint64_t(255);  // offsets keep their addresses' alignment
  }
  a.pfix = pfix;
  void* batch_ws = w + put_jobs_bytes(m);
  // Copy mode with both sources (round 6): messages of at most stream_put_max bytes are
  // streamed -- put_stream_kernel writes each whole and keeps its output runs' CRCs, put_stream_seal_kernel
  // writes its trailers -- and the layout kernel gives them no jobs; a longer one sets `big`, which gates
  // the job path below (CRC batch and seal) on the device.
  const bool streamed = stream_ok && a.copy_through && d_fields && d_blobs && !gate && !pfix && c->stream_put_max;
  StreamPutArgs sa;
  if (streamed) {
    a.stream_max = (uint32_t)c->stream_put_max;
    a.big = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(batch_ws) + ws_need(j));
    if (hipMemsetAsync(a.big, 0, sizeof(uint32_t), stream) != hipSuccess) return AMBRYCRC_EHIP;
    sa.desc = d_desc;
    sa.m = m;
    sa.obase = d_out - (reinterpret_cast<uintptr_t>(d_out) & 63u);
    sa.oreg0 = reinterpret_cast<uintptr_t>(d_out) & 63u;
    sa.fields = d_fields;
    sa.blobs = d_blobs;
    sa.rk = reinterpret_cast<uint32_t*>(w + put_core_bytes(m));
    sa.img = c->d_img;
  }
  if (launch_put_layout(a, stream) != hipSuccess) return AMBRYCRC_EHIP;
  if (layout_only) return AMBRYCRC_OK;
  if (streamed) {
    if (launch_put_stream(sa, c->num_cu, stream) != hipSuccess || launch_put_stream_seal(sa, c->num_cu, stream) != hipSuccess)
      return AMBRYCRC_EHIP;
    a.gate = a.big;  // the job path: only when a message was too long to stream
    PutArgs z = a;   // ... whose first step empties the streamed messages' job entries
    z.clear_short = true;
    if (launch_put_layout(z, stream) != hipSuccess) return AMBRYCRC_EHIP;
  }
  if (a.copy_through) {
    // one pass over the fields: the copy-through sweep reads each from its source, writes it into
    // the message and CRCs it (job k*m+i = slot k of message i, as the CRC jobs)
    const int rc = enqueue_batch(c, reinterpret_cast<const uint8_t*>((uintptr_t)a.src_base), a.cp_src, a.cp_len,
                                 a.crc_in, crc, j, batch_ws, stream, nullptr, d_out, a.cp_dst, a.gate);
    if (rc) return rc;
    return hip_err(launch_put_seal(a, stream));
  }
  if (d_fields || d_blobs) {
    // cost offsets of the copy jobs: the plan kernel's exclusive scan (no small-chunk classes);
    // its per-chunk output initialisation lands in `crc`, overwritten by the CRC batch below
    PlanArgs p;
    p.gate = gate;  // the transform's fallback pass: only when a placed message failed
    p.off = a.cp_dst;
    p.len = a.cp_cost;
    p.crc_in = nullptr;
    p.n = (uint32_t)j;
    p.byte_start = static_cast<uint64_t*>(batch_ws);
    const size_t blocks = (j + kPlanPerBlock - 1) / kPlanPerBlock;
    p.block_sum = p.byte_start + j + 1;
    p.block_small = p.block_sum + blocks;
    p.small_total = p.block_small + blocks;
    p.small_idx = reinterpret_cast<uint32_t*>(p.small_total + 5);
    p.crc_stage = nullptr;
    p.out = crc;
    p.small_max = 0;
    if (launch_plan(p, stream) != hipSuccess) return AMBRYCRC_EHIP;
    CopyArgs ca;
    ca.src = a.cp_src;
    ca.dst_off = a.cp_dst;
    ca.len = a.cp_len;
    ca.start = p.byte_start;
    ca.n = (uint32_t)j;
    ca.dst = d_out;
    ca.gate = gate;
    if (launch_gather_copy(ca, c->num_cu * 8, stream) != hipSuccess) return AMBRYCRC_EHIP;
  }
  if (d_in_crc) return AMBRYCRC_OK;  // the layout kernel wrote every trailer
  const int rc = enqueue_batch(c, d_out, a.crc_off, a.crc_len, nullptr, crc, j, batch_ws, stream);
  if (rc) return rc;
  return hip_err(launch_put_seal(a, stream));
}

}  // namespace detail
}  // namespace ambrycrc

extern "C" {

uint64_t ambrycrc_put_layout(const ambrycrc_put_desc* d, uint64_t* offsets) {
  if (!d) return 0;
  PutLayout L;
  if (!put_layout(*d, L)) return 0;
  if (offsets) put_field_offsets(*d, L, offsets);
  return L.length;
}

int ambrycrc_serialize_put_host(const ambrycrc_put_desc* d, const uint8_t* fields, const uint8_t* blobs, uint8_t* out,
                                uint64_t out_cap, uint32_t* crcs) {
  if (!d || !out) return AMBRYCRC_EINVAL;
  PutLayout L;
  if (!put_layout(*d, L)) return AMBRYCRC_EINVAL;
  if (d->out_off > out_cap || L.length > out_cap - d->out_off) return AMBRYCRC_EINVAL;
  uint8_t* m = out + d->out_off;
  uint64_t fo[5];
  put_field_offsets(*d, L, fo);
  const uint64_t src[5] = {d->key_src, d->enckey_src, d->props_src, d->usermeta_src, d->blob_src};
  const uint64_t len[5] = {d->key_len, L.enc_rec ? (uint64_t)d->enckey_len : 0, d->props_len, d->usermeta_len,
                           d->blob_len};
  for (int k = 0; k < 5; ++k) {
    const uint8_t* base = k == 4 ? blobs : fields;
    if (base && len[k]) memmove(m + fo[k], base + src[k], len[k]);
  }
  put_write_fixed(*d, L, m);
  for (uint32_t k = 0; k < kPutSlots; ++k) {
    uint64_t off, ln;
    bool present;
    put_crc_job(L, k, &off, &ln, &present);
    const uint32_t c = present ? ambrycrc_update(0, m + off, ln) : 0u;
    if (present) put_be64(m + off + ln, (uint64_t)c);
    if (crcs) crcs[k] = c;
  }
  return AMBRYCRC_OK;
}

size_t ambrycrc_serialize_puts_workspace_bytes(size_t m) { return put_core_bytes(m) + stream_put_rk_bytes(m); }

int ambrycrc_serialize_puts_dev(const ambrycrc_put_desc* d_desc, size_t m, const uint8_t* d_fields,
                                const uint8_t* d_blobs, uint8_t* d_out, uint64_t* d_msg_len, void* d_ws,
                                size_t ws_bytes, hipStream_t stream) {
  if (m == 0) return AMBRYCRC_OK;
  if (!d_desc || !d_out || (size_t)kPutSlots * m >= (1ull << 31)) return AMBRYCRC_EINVAL;
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  WsLease lease;
  const int rc = lease.acquire(c, stream, &d_ws, ws_bytes, ambrycrc_serialize_puts_workspace_bytes(m));
  if (rc) return rc;
  return enqueue_serialize(c, d_desc, m, d_fields, d_blobs, d_out, d_msg_len, d_ws, stream, nullptr, false, nullptr,
                           nullptr, true);
}

size_t ambrycrc_transform_workspace_bytes(size_t m) {
  return transform_own_bytes(m) + ws_need(m) + std::max(ambrycrc_messages_workspace_bytes(m), put_core_bytes(m));
}

namespace {
// The one-pass fast path keeps its run sums, control words and deferred list where the general
// path's verify / serializer workspace goes (it runs first, on the same stream).
size_t transform_fast_bytes(const uint8_t* d_region, uint64_t region_len, size_t m) {
  return region_ws_bytes(d_region, region_len, m);
}
}  // namespace

namespace {
// The side-stream verdict's entry for caller stream s (c->xs_mu held): its own, else a new one, else the
// least recently used re-keyed to s (DevCtx::XformSide). Null when one cannot be made.
DevCtx::XformSide* xform_side_for(DevCtx* c, hipStream_t s) {
  DevCtx::XformSide* x = nullptr;
  for (DevCtx::XformSide* e : c->xs_list)
    if (e->stream == s) x = e;
  if (!x && c->xs_list.size() < kMaxStreamWs) {
    auto* n = new DevCtx::XformSide();
    bool ok = hipStreamCreateWithFlags(&n->side, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&n->d_gates), 16 * DevCtx::kXformSlots) == hipSuccess &&
              hipExtMallocWithFlags(reinterpret_cast<void**>(&n->d_done), 8, hipMallocSignalMemory) == hipSuccess &&
              hipEventCreateWithFlags(&n->fork, hipEventDisableTiming) == hipSuccess;
    for (uint32_t k = 0; ok && k < DevCtx::kXformSlots; ++k)
      ok = hipEventCreateWithFlags(&n->ev[k], hipEventDisableTiming) == hipSuccess;
    // the signal starts at 0 (seq 0 is never waited for); both words are set before any stream uses them
    ok = ok && hipMemset(n->d_done, 0, 8) == hipSuccess && hipMemset(n->d_gates, 0, 16 * DevCtx::kXformSlots) == hipSuccess;
    if (!ok) {
      if (n->side) (void)hipStreamDestroy(n->side);
      if (n->d_gates) (void)hipFree(n->d_gates);
      if (n->d_done) (void)hipFree(n->d_done);
      if (n->fork) (void)hipEventDestroy(n->fork);
      for (hipEvent_t e : n->ev)
        if (e) (void)hipEventDestroy(e);
      delete n;
      return nullptr;
    }
    c->xs_list.push_back(n);
    x = n;
  }
  if (!x) {
    x = c->xs_list[0];
    for (DevCtx::XformSide* e : c->xs_list)
      if (e->tick < x->tick) x = e;
  }
  x->stream = s;
  x->tick = ++c->xs_tick;
  return x;
}
}  // namespace

uint64_t ambrycrc_transform_out_bound(uint64_t region_len, size_t m) {
  static_assert(AMBRYCRC_TRANSFORM_GROWTH_MAX == (40 - 34) + kPropsAppendixMax + (13 - 10), "growth bound");
  const uint64_t g = (uint64_t)AMBRYCRC_TRANSFORM_GROWTH_MAX;
  if ((uint64_t)m > (UINT64_MAX - region_len) / g) return UINT64_MAX;
  return region_len + (uint64_t)m * g;
}

int ambrycrc_transform_messages_dev(const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off, size_t m,
                                    const int16_t* d_life_version, int header_version, uint8_t* d_out,
                                    uint64_t out_cap, uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_status,
                                    void* d_ws, size_t ws_bytes, hipStream_t stream) {
  if (m == 0) return AMBRYCRC_OK;
  if (!d_region || !d_msg_off || !d_out || !d_out_len || !d_status || header_version < 1 || header_version > 3 ||
      (size_t)kPutSlots * m >= (1ull << 31))
    return AMBRYCRC_EINVAL;
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  // Fast path (FusedArgs::out): header V3 out, region mode on, a region to sweep, and workspace room
  // for the run sums (the library's own workspace is sized for them; a caller's as given).
  const size_t base_need = ambrycrc_transform_workspace_bytes(m);
  const size_t fast_need = transform_own_bytes(m) + ws_need(m) + transform_fast_bytes(d_region, region_len, m);
  const bool want_fast = header_version == 3 && c->region_mode != 0 && region_len > 0 &&
                         region_len <= c->xform_fast_max * (uint64_t)m;
  const size_t need = want_fast && !d_ws ? std::max(base_need, fast_need) : base_need;
  WsLease lease;
  int rc = lease.acquire(c, stream, &d_ws, ws_bytes, need);
  if (rc) return rc;
  const bool fast = want_fast && (ws_bytes ? ws_bytes : need) >= fast_need;
  // workspace: desc[m] | scan scratch (uint32 per message) | in_crc[4m] | xstatus[m] | fail |
  //            copy_off[5m] | pfix[m] | plan workspace for the m lengths | the verify pipeline's, then the
  //            serializer's (one after the other on the stream)
  uint8_t* w = static_cast<uint8_t*>(d_ws);
  TransformArgs t;
  memset(&t, 0, sizeof t);
  t.region = d_region;
  t.region_len = region_len;
  t.msg_off = d_msg_off;
  t.m = m;
  t.life = d_life_version;
  t.header_version = header_version;
  t.desc = reinterpret_cast<ambrycrc_put_desc*>(w);
  t.out_len = d_out_len;
  t.out_off = d_out_off;
  t.status = d_status;
  t.out_cap = out_cap;
  uint32_t* scan_out = reinterpret_cast<uint32_t*>(w + m * sizeof(ambrycrc_put_desc));
  t.in_crc = scan_out + m;
  uint32_t* xstatus = t.in_crc + 4 * m;
  uint32_t* fail = xstatus + m;
  uint64_t* copy_off = reinterpret_cast<uint64_t*>(w + transform_head_bytes(m));
  t.pfix = reinterpret_cast<PropsFix*>(copy_off + (size_t)kPutSlots * m);
  t.img = c->d_img;
  t.out = d_out;
  t.fail = fail;
  uint8_t* plan_ws = w + transform_own_bytes(m);
  void* shared = plan_ws + ws_need(m);
  // packed output offsets: the plan kernel's exclusive scan of the output lengths
  PlanArgs p;
  p.gate = nullptr;
  p.off = d_msg_off;
  p.len = d_out_len;
  p.crc_in = nullptr;
  p.n = (uint32_t)m;
  p.byte_start = reinterpret_cast<uint64_t*>(plan_ws);
  const size_t blocks = (m + kPlanPerBlock - 1) / kPlanPerBlock;
  p.block_sum = p.byte_start + m + 1;
  p.block_small = p.block_sum + blocks;
  p.small_total = p.block_small + blocks;
  p.small_idx = reinterpret_cast<uint32_t*>(p.small_total + 5);
  p.crc_stage = nullptr;
  p.out = scan_out;
  p.small_max = 0;

  // Speculative pass (two HBM passes: the verify reads every record once and writes the ones the
  // output keeps into place). The descriptors and the packed placement come from the parse alone,
  // before the CRCs are known; the verify's CRC batch is the copy-through kernel. A message that
  // then fails verification sets `fail`, and the fallback pass below rebuilds the output exactly as
  // the three-pass form did (verify bits first, then the transform's own, then the placement).
  const uint32_t* general = nullptr;  // the general path's gate (null: it always runs)
  std::unique_lock<std::mutex> xs_lock;  // held from the side entry's choice to the caller's wait
  DevCtx::XformSide* xs = nullptr;
  uint32_t xs_seq = 0, xs_slot = 0;
  hipStream_t main_stream = stream;
  if (fast) {
    // One pass (region_fused_kernel's copy form, then region_tail_kernel): verify every message
    // while copying the region into the output; when every message qualifies the headers are
    // patched, xfail stays 0, and the call returns without the general path below.
    FusedArgs f;
    f.a.region = d_region;
    f.a.region_len = region_len;
    f.a.msg_off = d_msg_off;
    f.a.m = m;
    f.a.img = c->d_img;
    f.a.status = d_status;
    f.a.msg_end = nullptr;
    f.a.inline_max = 0;
    const uintptr_t rp = reinterpret_cast<uintptr_t>(d_region);
    f.g.base = d_region - (rp & 63u);
    f.g.reg0 = rp & 63u;
    f.g.reg_end = f.g.reg0 + region_len;
    f.g.lo16 = f.g.reg0 & ~uint64_t(15);
    f.g.hi16 = (f.g.reg_end - 1) & ~uint64_t(15);
    f.g.nsb = region_nsb(d_region, region_len);
    f.g.rk = reinterpret_cast<uint32_t*>(shared);
    f.g.img = c->d_img;
    f.ngroups = (f.g.nsb + 3) / 4;
    f.ctl = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(shared) + region_rk_bytes(d_region, region_len));
    f.defer = f.ctl + 64;
    f.nproc = fused_proc_waves(c, m, true);
    f.out = d_out;
    f.out_cap = out_cap;
    f.out_off = d_out_off;
    f.out_len = d_out_len;
    f.life = d_life_version;
    f.xstatus = xstatus;
    // xfail beside `fail`, outside the shared workspace: the general path's kernels reuse `shared`
    // (ctl included) and read their device gate, *xfail, at every launch
    f.xfail = fail + 1;
    f.patch = copy_off;  // (the general path's, unused until then)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cap) != hipSuccess) return AMBRYCRC_EHIP;
    const int slot = c->xform_host_verdict && cap == hipStreamCaptureStatusNone ? c->take_host_word() : -1;
    if (slot < 0 && c->xform_side && cap == hipStreamCaptureStatusNone) {
      // Device verdict on a side stream: this call's gates in ring slot k, reused
      // only once the side chain that last read them has completed.
      xs_lock = std::unique_lock<std::mutex>(c->xs_mu);
      xs = xform_side_for(c, stream);
      if (xs) {
        if (xs->seq >= 0xFFFFFFF0u) {  // before the target wraps: drain both streams, restart at 0
          if (hipStreamSynchronize(xs->side) != hipSuccess || hipStreamSynchronize(stream) != hipSuccess ||
              hipMemset(xs->d_done, 0, 8) != hipSuccess)
            return AMBRYCRC_EHIP;
          xs->seq = 0;
        }
        xs_seq = ++xs->seq;
        xs_slot = xs_seq % DevCtx::kXformSlots;
        if (hipEventQuery(xs->ev[xs_slot]) == hipErrorNotReady &&
            hipStreamWaitEvent(stream, xs->ev[xs_slot], 0) != hipSuccess)
          return AMBRYCRC_EHIP;
        fail = xs->d_gates + 4 * xs_slot;
        f.xfail = fail + 1;
      }
    }
    if (hipMemsetAsync(f.ctl, 0, 8, stream) != hipSuccess || hipMemsetAsync(fail, 0, 8, stream) != hipSuccess)
      return AMBRYCRC_EHIP;
    f.path_out = slot < 0 ? c->d_path : nullptr;
    if (launch_region_fused(f, c->num_cu, stream) != hipSuccess) {
      if (slot >= 0) c->release_host_word(slot);
      return AMBRYCRC_EHIP;
    }
    if (slot >= 0) {
      // Host verdict (ambrycrc_set_transform_verdict): one synchronization with the stream decides
      // -- the batch is done, or the general path is enqueued -- instead of the ~20 gated launches
      // of the general path's empty dispatches. Blocks the calling thread.
      uint32_t* h_xfail = c->h_words + slot;
      *h_xfail = 1;
      const bool ok = hipMemcpyAsync(h_xfail, f.xfail, sizeof(uint32_t), hipMemcpyDeviceToHost, stream) == hipSuccess &&
                      hipStreamSynchronize(stream) == hipSuccess;
      const uint32_t v = *h_xfail;
      c->release_host_word(slot);
      if (!ok) return AMBRYCRC_EHIP;
      if (v == 0) {
        c->last_xform_path.store(1);
        return AMBRYCRC_OK;
      }
      c->last_xform_path.store(0);
    } else {
      // Device verdict (the default, and always under stream capture): the general path below is
      // enqueued behind *xfail -- every one of its kernels returns at once when the fast path took
      // the batch -- so the call only enqueues work, as every *_dev entry does. With a side stream
      // (xs) that chain runs there, and this stream waits only for the done signal.
      general = f.xfail;
      c->last_xform_path.store(2);
      if (xs) {
        if (launch_xform_signal(f.xfail, xs->d_done, xs_seq, stream) != hipSuccess ||
            hipEventRecord(xs->fork, stream) != hipSuccess || hipStreamWaitEvent(xs->side, xs->fork, 0) != hipSuccess)
          return AMBRYCRC_EHIP;
        main_stream = stream;
        stream = xs->side;
      }
    }
  } else {
    c->last_xform_path.store(0);
  }
  // fail[0] is written only by the general path below; the fast path zeroed it with xfail
  if (!fast && hipMemsetAsync(fail, 0, sizeof(uint32_t), stream) != hipSuccess) return AMBRYCRC_EHIP;
  t.fail = fail;
  p.gate = general;
  t.gate = general;
  t.gate_when = 1;
  MsgStage ms;
  t.xstatus = xstatus;
  t.copy_off = copy_off;
  // the parse kernel describes each message as it parses it (transform_desc_kernel fused)
  rc = enqueue_messages_parse(c, d_region, region_len, d_msg_off, m, d_status, nullptr, shared, stream, &ms, &t,
                              general);
  if (rc) return rc;
  t.job_off = ms.a.job_off;
  if (launch_plan(p, stream) != hipSuccess) return AMBRYCRC_EHIP;
  if (launch_transform_place(t, p.byte_start, stream) != hipSuccess) return AMBRYCRC_EHIP;
  if (launch_transform_jobs(t, stream) != hipSuccess) return AMBRYCRC_EHIP;
  rc = enqueue_messages_check(c, ms, stream, d_out, copy_off);
  if (rc) return rc;
  if (launch_transform_finish(t, stream) != hipSuccess) return AMBRYCRC_EHIP;
  rc = enqueue_serialize(c, t.desc, m, d_region, d_region, d_out, nullptr, shared, stream, t.in_crc, true, general);
  if (rc) return rc;
  if (launch_props_fix(t, stream) != hipSuccess) return AMBRYCRC_EHIP;  // after the copy-through
  t.gate = fail;
  t.gate_when = 0;  // no failure: the final status is the verify's bits, else the transform's own
  t.gate2 = general;  // (and only when the general path ran)
  if (launch_transform_merge(t, stream) != hipSuccess) return AMBRYCRC_EHIP;
  t.gate2 = nullptr;

  // Fallback pass (only when `fail` is set; every kernel checks it): descriptors from the final
  // verify status, packed placement, layout and a gather copy of the fields from the region.
  t.xstatus = nullptr;
  t.gate_when = 1;
  p.gate = fail;
  if (launch_transform_desc(t, stream) != hipSuccess) return AMBRYCRC_EHIP;
  if (launch_plan(p, stream) != hipSuccess) return AMBRYCRC_EHIP;
  if (launch_transform_place(t, p.byte_start, stream) != hipSuccess) return AMBRYCRC_EHIP;
  rc = enqueue_serialize(c, t.desc, m, d_region, d_region, d_out, nullptr, shared, stream, t.in_crc, false, fail,
                         t.pfix);
  if (rc) return rc;
  if (launch_props_fix(t, stream) != hipSuccess) return AMBRYCRC_EHIP;  // after the gather copy (gated as the pass)
  if (xs) {  // the side chain's end: done = seq whatever the verdict; the caller's stream waits for it
    if (launch_xform_signal(nullptr, xs->d_done, xs_seq, stream) != hipSuccess ||
        hipEventRecord(xs->ev[xs_slot], stream) != hipSuccess ||
        hipStreamWaitValue32(main_stream, xs->d_done, xs_seq, hipStreamWaitValueGte, 0xFFFFFFFFu) != hipSuccess)
      return AMBRYCRC_EHIP;
  }
  return AMBRYCRC_OK;
}

}  // extern "C"
