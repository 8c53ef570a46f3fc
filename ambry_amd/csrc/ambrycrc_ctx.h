// ambrycrc_ctx.h -- per-device context of libambrycrc and the internal batch entry the C ABI
// functions share (ambrycrc.cpp, ambrycrc_put.cpp). Internal to the library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/ambrycrc.h"
#include "crc32_kernels.h"

namespace ambrycrc {
namespace detail {

// ------------------------------------------------------------ contexts
constexpr int kMaxDevices = 64;
// Host path: a ring of kSlabs staging slabs per device. Up to kSlabs-1 slabs are in
// flight (H2D copy, kernels, D2H of CRCs on the slab's stream) while the host fills
// the next one; 64 MiB keeps the pipeline's fill and drain short (1.2 ms at PCIe rate).
constexpr int kSlabs = 4;
constexpr size_t kSlabBytes = 64ull << 20;    // host-path staging slab
constexpr size_t kSlabChunks = 1u << 14;      // max chunk pieces per slab

struct EventPair {
  hipEvent_t a, b;
};

struct HostSlab {
  uint8_t* h_data = nullptr;   // pinned
  uint64_t* h_meta = nullptr;  // pinned: off[kSlabChunks], len[kSlabChunks]
  uint32_t* h_out = nullptr;   // pinned
  uint8_t* d_data = nullptr;
  uint64_t* d_meta = nullptr;
  uint32_t* d_out = nullptr;
  void* d_ws = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
};

constexpr size_t kSlabMsgs = 1u << 16;  // messages per host-path staging slab

struct MsgSlab {  // message verify staging per HostSlab, allocated on first use
  uint64_t* h_off = nullptr;   // pinned [kSlabMsgs]: message offsets in the slab
  uint32_t* h_status = nullptr;
  uint64_t* h_end = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_status = nullptr;
  uint64_t* d_end = nullptr;
  void* d_ws = nullptr;
};

// Transform staging per HostSlab (ambrycrc_transform_messages_host), allocated on first use: the
// slab's re-serialized messages (at most ambrycrc_transform_out_bound of its span and count).
constexpr size_t kXformOutBytes = kSlabBytes + (size_t)AMBRYCRC_TRANSFORM_GROWTH_MAX * kSlabMsgs;
struct XformSlab {
  int16_t* h_life = nullptr;  // pinned [kSlabMsgs]
  int16_t* d_life = nullptr;
  uint8_t* h_out = nullptr;   // pinned [kXformOutBytes]
  uint8_t* d_out = nullptr;
  uint64_t* h_olen = nullptr;  // pinned [kSlabMsgs]
  uint64_t* d_olen = nullptr;
  uint64_t* d_ooff = nullptr;
  void* d_ws = nullptr;       // ambrycrc_transform_workspace_bytes(kSlabMsgs)
};

struct DevCtx {
  int device = -1;
  int num_cu = 0;
  int grid = 0;
  // kVariantDefault (29): 64-B lane runs (four coalesced 1 KiB loads per 4 KiB super-block,
  // quad transpose by v_cndmask_b32_dpp, one x^(8*4096) fold per 64 B), s_setprio 3 around
  // the loads; plus, for batches of >= kGroupMinChunks chunks, whole chunks <= 16 KiB in the
  // fused group phase, each size class spread over all waves with a class-sized group
  // (G = 2 / 8 / 16 lanes). Measured against the round-1 alternatives in DESIGN.md §4-5.
  int variant = AMBRY_DEFAULT_VARIANT;  // (A/B builds: -DAMBRY_DEFAULT_VARIANT=...)
  // Message verify of regions of at most kRegionMaxPerMessage bytes per message: region mode
  // (region_runs_kernel + region_msg_kernel) instead of jobs through the batch engine.
  // 2 (default): two passes (region_runs_kernel, then region_msg_kernel: one thread per message),
  // 1: one pass (region_fused_kernel + region_tail_kernel; measured 1.5-14 % slower, DESIGN.md
  // §10.1), 0: off. The transform's fast path is the one-pass kernel's copy form whenever region
  // mode is on and the region holds at most xform_fast_max bytes per message.
  int region_mode = 2;
  uint64_t xform_fast_max = kXformFastMaxPerMessage;
  // Serialize copy mode streams messages of at most this many bytes (put_stream_kernel, DESIGN.md
  // §12.6); AMBRYCRC_STREAM_PUT_MAX at init: 0 = every message through the job path (A/B).
  uint64_t stream_put_max = kStreamPutMax;
  // The form the last message verify on this device took (ambrycrc_last_message_mode).
  std::atomic<int> last_msg_mode{-1};
  // The path the last transform took (ambrycrc_last_transform_path): 1 fast, 0 general, 2 decided
  // on the device (region_patch_kernel wrote 1 or 0 to d_path).
  std::atomic<int> last_xform_path{-1};
  uint32_t* d_path = nullptr;  // (inside the d_img allocation)
  // The transform fast path's verdict read by the host (ambrycrc_set_transform_verdict): off by
  // default -- the general path is then enqueued behind a device gate, and the call never blocks.
  std::atomic<int> xform_host_verdict{0};
  // The device verdict's side stream, one per caller stream: the general path's
  // gated kernels go to `side`, forked after the fast path, and the caller's stream waits on the done
  // signal instead (hipStreamWaitValue32, >= the call's seq) -- which the fast path sets when it took
  // the batch, and the side chain's last kernel sets always. Each call's gates (fail, xfail) sit in a
  // slot of a ring, so a side chain still running its no-ops never reads a later call's verdict; a
  // slot is reused only behind its last chain's event. Entries are never freed before shutdown: the
  // least recently used is re-keyed to a new caller stream (its seq keeps increasing, so a wait still
  // pending on the old stream is met). xform_side = 0 (AMBRYCRC_XFORM_SIDE=0): the inline gated chain.
  static constexpr uint32_t kXformSlots = 32;
  struct XformSide {
    hipStream_t stream = nullptr;  // the caller's
    hipStream_t side = nullptr;    // library-owned, non-blocking
    uint32_t* d_gates = nullptr;   // [4 * kXformSlots]: slot k's fail at 4k, xfail at 4k + 1
    uint32_t* d_done = nullptr;    // the low word of one HSA signal (hipMallocSignalMemory)
    hipEvent_t fork = nullptr;
    hipEvent_t ev[kXformSlots] = {};  // recorded on `side` after the chain that used slot k
    uint32_t seq = 0;                 // the last call's target value
    uint64_t tick = 0;
  };
  int xform_side = 1;
  std::mutex xs_mu;
  std::vector<XformSide*> xs_list;  // at most kMaxStreamWs
  uint64_t xs_tick = 0;
  // Pinned words for one-word device-to-host reads (the host verdict): a call holds slot k (busy[k])
  // from its copy until it has read the word, so no two calls in flight share one; with every slot
  // held the call takes the device-gated form instead.
  static constexpr uint32_t kHostWords = 256;
  uint32_t* h_words = nullptr;
  std::atomic<bool> h_word_busy[kHostWords] = {};
  int take_host_word() {
    for (uint32_t k = 0; k < kHostWords; ++k) {
      bool f = false;
      if (!h_word_busy[k].load(std::memory_order_relaxed) &&
          h_word_busy[k].compare_exchange_strong(f, true, std::memory_order_acquire))
        return (int)k;
    }
    return -1;
  }
  void release_host_word(int k) { h_word_busy[k].store(false, std::memory_order_release); }
  // Host-resident dispatch (ambrycrc_set_host_policy): 0 auto, 1 the GPU, 2 the CPU. Auto sends
  // pageable host bytes to the CPU leg when the CPU threads' CRC rate beats gpu_host_gibps, the
  // GPU host path's rate (PCIe-bound: 51 GiB/s measured, BENCH_r04 host_path; refreshed by every
  // GPU host call of >= 64 MiB). last_host_path: 0 CPU, 1 GPU, -1 none yet.
  std::atomic<int> host_policy{0};
  std::atomic<double> gpu_host_gibps{51.0};
  std::atomic<int> last_host_path{-1};
  // The CPU leg's thread budget on this device (ambrycrc_set_host_cpu_threads; 0: the process's,
  // host_cpu_threads). Auto compares the CPU leg's rate AT this budget with the GPU's.
  std::atomic<int> cpu_threads{0};
  // ambrycrc_batch_host's CPU leg as its calls of >= 64 MiB measured it, per thread budget (EWMA;
  // -1: not yet, the calibration at that budget stands for it); under auto every 16th such pageable
  // call takes the other leg, so both rates stay current.
  static constexpr int kMaxCpuThreads = 256;
  std::atomic<double> cpu_batch_gibps[kMaxCpuThreads + 1];
  DevCtx() {
    for (auto& r : cpu_batch_gibps) r.store(-1.0, std::memory_order_relaxed);
  }
  std::atomic<uint32_t> batch_calls{0};
  // The message entries (kMsgVerify, kMsgTransform) compare their own legs' rates over region
  // bytes, GiB/s: a CPU leg parses and (transform) copies each message, so the CRC rate above does
  // not stand for it. Each leg's rate is refreshed by its calls of >= 64 MiB (EWMA); the CPU legs
  // start from a fraction of the CRC rate (-1 until measured), the GPU legs from round 5's
  // measurements (bench_put --transform-host, 4 KiB PUTs); under auto every 16th large pageable call
  // takes the other leg, so a rate that changes is seen.
  std::atomic<double> msg_gpu_gibps[2] = {{44.0}, {22.0}};
  std::atomic<double> msg_cpu_gibps[2] = {{-1.0}, {-1.0}};
  std::atomic<uint32_t> msg_calls[2] = {{0u}, {0u}};
  // Processor waves of the one-pass kernels (0: per call, fused_proc_waves); AMBRYCRC_FUSED_PROC.
  int fused_proc = AMBRY_FUSED_PROC;
  uint64_t region_max = kRegionMaxPerMessage;  // region bytes per message up to which it applies
  // Sweep rounds of at most this many bytes (SweepArgs::window); 0 = one round.
  uint64_t window = 32ull << 30;
  uint32_t* d_img = nullptr;
  // Default workspaces (d_ws == NULL calls), one per stream: calls on one stream are ordered by
  // it, so they may share a buffer; calls on different streams get different buffers. ws_mu is
  // held from choosing the buffer until the call's work is enqueued, so a concurrent call that
  // grows the same stream's buffer retires the old one only behind that work (an event on the
  // stream; freed once it has completed, or at shutdown).
  struct StreamWs {
    hipStream_t stream;
    void* ptr;
    size_t bytes;
    hipEvent_t last;  // recorded on `stream` after each call's work (WsLease), null before the first
    uint64_t tick;    // last use, for eviction
    bool captured;    // a stream capture (HIP graph) recorded this buffer: never freed before shutdown
  };
  struct RetiredWs {
    void* ptr;
    hipEvent_t done;
  };
  std::mutex ws_mu;
  std::vector<StreamWs> ws_list;  // at most kMaxStreamWs: the least recently used is evicted
  std::vector<RetiredWs> ws_retired;
  std::vector<void*> ws_kept;  // buffers a captured graph may still use, replaced or evicted: freed at shutdown
  uint64_t ws_tick = 0;
  bool timing = false;
  std::vector<EventPair> pending, free_events;
  bool slabs_ready = false;
  HostSlab slab[kSlabs];
  bool msg_slabs_ready = false;
  MsgSlab msg_slab[kSlabs];
  bool xform_slabs_ready = false;
  XformSlab xform_slab[kSlabs];
  std::mutex mu;     // guards the slabs (held across a whole host-path call)
  std::mutex ev_mu;  // guards the timing events (taken inside enqueue_batch, which host-path calls reach with mu held)
};

int hip_err(hipError_t e);
// Host-resident dispatch: the CPU threads the CPU leg of device c uses -- its budget
// (ambrycrc_set_host_cpu_threads), else the process's (the same call with device -1), else
// AMBRYCRC_CPU_THREADS, else half this process's CPU share (host_cpu_share: affinity, cgroup quota,
// OMP_NUM_THREADS), so the server's own network and disk threads keep the other half.
int host_cpu_share();
int host_cpu_threads(const DevCtx* c = nullptr);
// The CPU leg's CRC rate in GiB/s with `threads` threads hashing DRAM-resident bytes at once
// (calibrated once per thread count: ambrycrc_host_calibrate, or the first auto decision needing it).
double host_cpu_gibps(int threads);
// True when a host call over `bytes` of host memory should take the CPU leg (device < 0, the
// CPU policy, or auto with pageable bytes the CPU threads hash faster than the GPU host path).
bool host_take_cpu(DevCtx* c, int device, int pinned, uint64_t bytes);
void host_note_cpu(DevCtx* c, uint64_t bytes, double seconds);
// After a GPU host call over `bytes` that took `seconds`: refresh c->gpu_host_gibps.
void host_note_gpu(DevCtx* c, uint64_t bytes, double seconds);
// The message entries' leg choice and rate tracking (DevCtx::msg_*_gibps).
constexpr int kMsgVerify = 0, kMsgTransform = 1;
bool host_take_cpu_msg(DevCtx* c, int device, int pinned, int op, uint64_t bytes);
void host_note_msg(DevCtx* c, int op, bool cpu, uint64_t bytes, double seconds);
double host_msg_cpu_gibps(const DevCtx* c, int op);
DevCtx* ctx_for(int device);
DevCtx* ctx_current();
// Bytes of batch workspace for n chunks (ambrycrc_workspace_bytes).
size_t ws_need(size_t n);
// Default workspaces kept per device: a caller cycling through many short-lived streams (one per
// request) holds at most this many buffers; the least recently used one is retired behind its
// last call's event and freed once that work has completed.
constexpr size_t kMaxStreamWs = 16;
int stream_ws(DevCtx* c, hipStream_t s, size_t need, void** out, size_t* entry, bool* capturing);
// Largest chunk the group phase takes whole for a batch of n chunks on c's variant (0: none).
uint64_t batch_small_max(const DevCtx* c, size_t n);
// Plan + CRC kernels for n chunks on stream s (ws: >= ws_need(n) bytes). exp_fill, copy_dst,
// copy_off: see SweepArgs (copy_dst set: the copy-through kernel, whatever c's variant).
int enqueue_batch(DevCtx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, const uint32_t* crc_in,
                  uint32_t* out, size_t n, void* ws, hipStream_t s, uint32_t* exp_fill = nullptr,
                  uint8_t* copy_dst = nullptr, const uint64_t* copy_off = nullptr, const uint32_t* gate = nullptr);

// The device message-verify pipeline on `stream`: parse -> plan + sweep -> reduce (job mode), or
// parse, region runs, region jobs -> reduce (region mode: c->region_mode, a region of at most
// kRegionMaxPerMessage bytes per message, and ws_bytes room for its run sums). d_ws holds
// ws_bytes >= ambrycrc_messages_workspace_bytes(m) bytes. d_msg_end may be null.
int enqueue_messages(DevCtx* c, const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off, size_t m,
                     uint32_t* d_status, uint64_t* d_msg_end, void* d_ws, size_t ws_bytes, hipStream_t stream);
// Processor waves per workgroup of the one-pass region kernels for m messages (FusedArgs::nproc).
uint32_t fused_proc_waves(const DevCtx* c, size_t m, bool copy);
// Bytes of the job arrays at the start of a message-verify workspace (the rest: batch / run sums).
size_t msg_jobs_bytes(size_t m);
// The same in two halves: the parse kernel (jobs and their stored CRCs in st->a), then the CRC
// batch and the reduce -- with copy_dst / copy_off, the batch is the copy-through kernel
// (SweepArgs::copy_dst), which the transform uses to copy the records while verifying them.
struct MsgStage {
  MsgArgs a;
  uint32_t* crc;  // a.crc, writable: the batch's output
  void* batch_ws;
  size_t j;
};
int enqueue_messages_parse(DevCtx* c, const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off,
                           size_t m, uint32_t* d_status, uint64_t* d_msg_end, void* d_ws, hipStream_t stream,
                           MsgStage* st, const TransformArgs* desc = nullptr, const uint32_t* gate = nullptr);
int enqueue_messages_check(DevCtx* c, const MsgStage& st, hipStream_t stream, uint8_t* copy_dst = nullptr,
                           const uint64_t* copy_off = nullptr);
// The PUT serialization pipeline (layout -> copy -> plan + CRC -> seal); d_ws holds at least
// ambrycrc_serialize_puts_workspace_bytes(m). d_in_crc (transform): the CRCs of records 1-4,
// 4 per message (PutArgs::in_crc); the layout kernel then writes every trailer and the CRC pass
// over the output is skipped.
// layout_only: the layout kernel alone (the transform's speculative pass, whose fields the
// verify already copied); gate: run the layout and copy kernels only when *gate != 0.
int enqueue_serialize(DevCtx* c, const ::ambrycrc_put_desc* d_desc, size_t m, const uint8_t* d_fields,
                      const uint8_t* d_blobs, uint8_t* d_out, uint64_t* d_msg_len, void* d_ws, hipStream_t stream,
                      const uint32_t* d_in_crc = nullptr, bool layout_only = false, const uint32_t* gate = nullptr,
                      const PropsFix* pfix = nullptr, bool stream_ok = false);

// Bytes from a message's start that its verify may read (the header window, or the whole message
// when the header's sizes fit `rem`).
uint64_t message_extent_of(const uint8_t* p, uint64_t rem);
// The host entries' CPU leg (ambrycrc_msg_cpu.cpp): the batch on `threads` CPU threads, each
// message through ambrycrc_verify_message_cpu / ambrycrc_transform_message_cpu; outputs as the
// device batch's.
int verify_messages_cpu(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                        uint32_t* status, uint64_t* msg_end, int threads);
int transform_messages_cpu(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                           const int16_t* life_version, int header_version, uint8_t* out, uint64_t out_cap,
                           uint64_t* out_off, uint64_t* out_len, uint32_t* status, int threads);

// Holds c->ws_mu for the lifetime of a *_dev call that uses the default workspace (d_ws ==
// NULL); a call with its own workspace takes no lock.
struct WsLease {
  std::unique_lock<std::mutex> lk;
  DevCtx* ctx = nullptr;
  hipStream_t stream = nullptr;
  size_t entry = ~size_t(0);
  bool capturing = false;
  // On return *ws is the caller's buffer (checked against need) or the stream's default one.
  int acquire(DevCtx* c, hipStream_t s, void** ws, size_t ws_bytes, size_t need) {
    if (*ws) return ws_bytes < need ? AMBRYCRC_EINVAL : AMBRYCRC_OK;
    lk = std::unique_lock<std::mutex>(c->ws_mu);
    const int rc = stream_ws(c, s, need, ws, &entry, &capturing);
    if (rc == AMBRYCRC_OK) {
      ctx = c;
      stream = s;
    }
    return rc;
  }
  // The call's work is enqueued: mark the buffer's last use on its stream (still under ws_mu). Not
  // under capture: an event recorded there would belong to the graph, not to its replays.
  ~WsLease() {
    if (!ctx || capturing || entry >= ctx->ws_list.size()) return;
    DevCtx::StreamWs& w = ctx->ws_list[entry];
    if (!w.last && hipEventCreateWithFlags(&w.last, hipEventDisableTiming) != hipSuccess) w.last = nullptr;
    if (w.last) (void)hipEventRecord(w.last, stream);
  }
};

}  // namespace detail
}  // namespace ambrycrc
