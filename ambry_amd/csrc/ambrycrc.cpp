// ambrycrc.cpp -- host side of libambrycrc: C ABI (include/ambrycrc.h),
// per-device contexts, kernel launches, host streaming primitives and the
// pinned-staging host-resident batch path.
#include "../../include/ambrycrc.h"

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>
#if defined(__x86_64__)
#include <emmintrin.h>
#endif

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <new>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "crc32_gf2.h"
#include "crc32_kernels.h"
#include "crc32_layout.h"
#include "ambrycrc_ctx.h"
#include "host_crc.h"

using namespace ambrycrc;
using namespace ambrycrc::detail;

namespace {

// ------------------------------------------------------------ host tables
struct HostTables {
  uint32_t t[8][256];
  uint32_t xpow2[64];
  HostTables() {
    slice_tables(t, 8);
    xpow8_pow2_table(xpow2);
  }
};

const HostTables& host_tables() {
  static const HostTables tables;  // C++11 thread-safe static init
  return tables;
}

uint32_t host_xpow8(uint64_t n) {
  const HostTables& h = host_tables();
  uint32_t r = kOne;
  for (int k = 0; n; ++k, n >>= 1)
    if (n & 1) r = gf2_mul(r, h.xpow2[k]);
  return r;
}

// ------------------------------------------------------------ LDS image
std::vector<uint32_t> build_table_image() {
  const uint32_t words = kImgBytes / 4;
  std::vector<uint32_t> img(words, 0u);
  uint32_t t[4][256];
  slice_tables(t, 4);
  for (uint32_t j = 0; j < 4; ++j)
    for (uint32_t b = 0; b < 256; ++b)
      for (uint32_t l = 0; l < 32; ++l) {
        const uint32_t addr = ((j >> 1) << 16) | (b << 8) | ((j & 1) << 7) | (l << 2);
        img[addr / 4] = t[j][b];
      }
  auto put_nib = [&](uint32_t off, uint32_t c) {
    uint32_t nt[8][16];
    nibble_tables(c, nt);
    for (int n = 0; n < 8; ++n)
      for (int x = 0; x < 16; ++x) img[(kNibBase + off + 64u * n + 4u * x) / 4] = nt[n][x];
  };
  put_nib(kFoldOff, host_xpow8(kBlockBytes));
  for (uint32_t l = 0; l < kTreeLevels; ++l) put_nib(kTreeOff + kNibSetBytes * l, host_xpow8(16ull << l));
  for (uint32_t k = 0; k < kPowTables; ++k) put_nib(kPowOff + kNibSetBytes * k, host_xpow8(1ull << k));
  const HostTables& h = host_tables();
  for (int k = 0; k < 64; ++k) img[kLdsBytes / 4 + k] = h.xpow2[k];
  // x^-1 in the reflected order: u * x = v  <=>  u = v << 1 (bit 31 of v clear), or
  // ((v ^ P) << 1) | 1 (set), since u * x = (u >> 1) ^ (P if bit 0 of u).
  uint32_t inv = kOne;
  for (int i = 0; i < 8; ++i) inv = (inv & 0x80000000u) ? (((inv ^ kPoly) << 1) | 1u) : (inv << 1);  // x^-8
  for (uint32_t k = 0; k < kInvPowSets; ++k) {
    uint32_t nt[8][16];
    nibble_tables(inv, nt);
    for (int n = 0; n < 8; ++n)
      for (int x = 0; x < 16; ++x) img[(kImgInvOff + kNibSetBytes * k + 64u * n + 4u * x) / 4] = nt[n][x];
    inv = gf2_mul(inv, inv);
  }
  // region pass 2's words (crc32_layout.h kImgRegOff)
  uint32_t* reg = img.data() + kImgRegOff / 4;
  for (uint32_t lo = 0; lo < 64; ++lo) {
    const uint32_t ni = 64 - lo < 4 ? 64 - lo : 4;
    uint32_t r = 0;
    for (uint32_t i = 0; i < 64; ++i) r = t[0][(r ^ (i >= lo && i < lo + ni ? 0xFFu : 0u)) & 0xFFu] ^ (r >> 8);
    reg[kRegH0 + lo] = r;
  }
  for (uint32_t a = 0; a <= 4; ++a) {
    reg[kRegGe + a] = a < 4 ? 0xFFFFFFFFu << (8 * a) : 0u;
    reg[kRegLt + a] = a < 4 ? (1u << (8 * a)) - 1u : 0xFFFFFFFFu;
  }
  {
    uint32_t nt[8][16];
    nibble_tables(host_xpow8(256), nt);
    for (uint32_t j = 0; j < 4; ++j)
      for (uint32_t b = 0; b < 256; ++b)
        reg[kRegAuxWords + 256 * j + b] = nt[2 * j][b & 15] ^ nt[2 * j + 1][b >> 4];
  }
  {
    uint32_t inv8 = kOne;  // x^-8
    for (int i = 0; i < 8; ++i) inv8 = (inv8 & 0x80000000u) ? (((inv8 ^ kPoly) << 1) | 1u) : (inv8 << 1);
    uint32_t inv64 = kOne;
    for (int i = 0; i < 8; ++i) inv64 = gf2_mul(inv64, inv8);
    uint32_t u0 = kOne, u1 = kOne;  // x^(-8 d0), x^(-64 d1)
    for (uint32_t d = 0; d < 8; ++d) {
      uint32_t nt[8][16];
      nibble_tables(u0, nt);
      for (int n = 0; n < 8; ++n)
        for (int x = 0; x < 16; ++x) reg[kRegAuxWords + kRegByteWords + 128u * d + 16u * n + x] = nt[n][x];
      nibble_tables(u1, nt);
      for (int n = 0; n < 8; ++n)
        for (int x = 0; x < 16; ++x) reg[kRegAuxWords + kRegByteWords + 128u * (8 + d) + 16u * n + x] = nt[n][x];
      u0 = gf2_mul(u0, inv8);
      u1 = gf2_mul(u1, inv64);
    }
  }
  return img;
}

}  // namespace

namespace ambrycrc {
namespace detail {

std::mutex g_mu;
DevCtx* g_ctx[kMaxDevices] = {nullptr};

int hip_err(hipError_t e) { return e == hipSuccess ? AMBRYCRC_OK : AMBRYCRC_EHIP; }

// ------------------------------------------------------------ staging copy pool
// Pageable host chunks (a Netty direct ByteBuf, a FileChannel read buffer) must be
// memcpy'd into a pinned slab before the DMA engine can move them. One core copies
// ~25 GB/s, half of PCIe Gen5 x16, so the slab fill is split over a few worker
// threads (AMBRYCRC_COPY_THREADS, default 8; 1 disables the pool). Process-wide,
// started on first use; jobs from concurrent callers interleave safely.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool pool;
    return pool;
  }
  int threads() const { return nthreads_; }
  // Runs fn(0..parts-1) across the workers and the calling thread; returns when all are done.
  void run(int parts, const std::function<void(int)>& fn) {
    if (parts <= 1 || workers_.empty()) {
      for (int i = 0; i < parts; ++i) fn(i);
      return;
    }
    Batch b{&fn, parts};
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int i = 1; i < parts; ++i) queue_.push_back({&b, i});
    }
    cv_.notify_all();
    fn(0);
    finish_one(b);
    // help with this batch's remaining parts instead of idling
    for (;;) {
      Job j{nullptr, 0};
      {
        std::lock_guard<std::mutex> g(mu_);
        for (size_t q = 0; q < queue_.size(); ++q)
          if (queue_[q].batch == &b) {
            j = queue_[q];
            queue_.erase(queue_.begin() + q);
            break;
          }
      }
      if (!j.batch) break;
      (*j.batch->fn)(j.part);
      finish_one(b);
    }
    std::unique_lock<std::mutex> lk(b.mu);
    b.cv.wait(lk, [&] { return b.left == 0; });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  struct Batch {
    const std::function<void(int)>* fn;
    int left;
    std::mutex mu;
    std::condition_variable cv;
  };
  struct Job {
    Batch* batch;
    int part;
  };
  CopyPool() {
    int t = 8;
    if (const char* e = getenv("AMBRYCRC_COPY_THREADS")) t = atoi(e);
    nthreads_ = std::max(1, std::min(t, 64));
    try {
      for (int i = 1; i < nthreads_; ++i) workers_.emplace_back([this] { loop(); });
    } catch (...) {  // fewer workers than asked (the C ABI does not throw): the parts queue on those started
    }
    nthreads_ = (int)workers_.size() + 1;
  }
  static void finish_one(Batch& b) {
    std::lock_guard<std::mutex> g(b.mu);
    if (--b.left == 0) b.cv.notify_all();
  }
  void loop() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !queue_.empty(); });
        if (stop_ && queue_.empty()) return;
        j = queue_.front();
        queue_.erase(queue_.begin());
      }
      (*j.batch->fn)(j.part);
      finish_one(*j.batch);
    }
  }
  int nthreads_ = 1;
  std::vector<std::thread> workers_;
  std::vector<Job> queue_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

struct CopyJob {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t n;
};

// Copies the jobs (disjoint destinations) with the pool: the slab's bytes are split into
// `parts` equal ranges, each thread copying its range of every job it overlaps.
void parallel_copy(const std::vector<CopyJob>& jobs, uint64_t total) {
  if (jobs.empty()) return;
  CopyPool& pool = CopyPool::get();
  const int parts = (int)std::min<uint64_t>((uint64_t)pool.threads(), std::max<uint64_t>(1, total >> 20));
  if (parts <= 1) {
    for (const CopyJob& j : jobs) memcpy(j.dst, j.src, j.n);
    return;
  }
  std::vector<uint64_t> start(jobs.size() + 1, 0);
  for (size_t i = 0; i < jobs.size(); ++i) start[i + 1] = start[i] + jobs[i].n;
  pool.run(parts, [&](int p) {
    const uint64_t lo = total * (uint64_t)p / (uint64_t)parts, hi = total * (uint64_t)(p + 1) / (uint64_t)parts;
    size_t i = std::upper_bound(start.begin(), start.end(), lo) - start.begin() - 1;
    for (; i < jobs.size() && start[i] < hi; ++i) {
      const uint64_t a = std::max(lo, start[i]), b = std::min(hi, start[i + 1]);
      if (b > a) memcpy(jobs[i].dst + (a - start[i]), jobs[i].src + (a - start[i]), b - a);
    }
  });
}

DevCtx* ctx_for(int device) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> g(g_mu);
  return g_ctx[device];
}

DevCtx* ctx_current() {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  return ctx_for(dev);
}

// workspace: byte_start[n+1] | block_sum[B] | block_small[B] | small_total[5] (uint64:
//            total, start of size classes 1..3 in small_idx, spare) |
//            small_idx[n] (uint32) | crc_stage[n] (uint32: crc_in as read by the plan),
//            B = ceil(n / kPlanPerBlock)
size_t ws_need(size_t n) {
  const size_t blocks = (n + kPlanPerBlock - 1) / kPlanPerBlock;
  return ((n + 6 + 2 * blocks) * sizeof(uint64_t) + 2 * n * sizeof(uint32_t) + 255) & ~size_t(255);
}

// Frees retired default workspaces whose last user has completed. Caller holds c->ws_mu.
void reap_retired_ws(DevCtx* c) {
  auto& r = c->ws_retired;
  for (size_t i = 0; i < r.size();) {
    if (hipEventQuery(r[i].done) == hipSuccess) {
      (void)hipFree(r[i].ptr);
      (void)hipEventDestroy(r[i].done);
      r[i] = r.back();
      r.pop_back();
    } else {
      ++i;
    }
  }
}

// The default workspace of `stream` with at least `need` bytes. Caller holds c->ws_mu until the
// work that uses it is enqueued on `stream`. A buffer that is too small is retired behind an
// event on the stream (work already queued there may still read it), never freed in place.
// (A destroyed stream's handle may be reused by a new stream; hipStreamDestroy drains the old
// stream's work first, so the buffer is idle by then.)
//
// Under stream capture (a HIP graph) nothing here may query events, synchronize or allocate: a
// capture uses the stream's buffer as an earlier uncaptured call sized it, or gets EINVAL. The graph
// then holds that buffer's address, so the entry is marked captured: when a later call grows it, or
// the entry is evicted, the buffer is kept (c->ws_kept) until shutdown instead of being freed, and
// replays stay valid. Replays share it with later calls on the stream, so they must be ordered with
// them (launched on that stream), as any two calls on one stream are.
int stream_ws(DevCtx* c, hipStream_t s, size_t need, void** out, size_t* entry, bool* capturing_out) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess) return AMBRYCRC_EHIP;
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (capturing_out) *capturing_out = capturing;
  if (!capturing) reap_retired_ws(c);
  DevCtx::StreamWs* w = nullptr;
  for (auto& e : c->ws_list)
    if (e.stream == s) w = &e;
  if (capturing && (!w || w->bytes < need)) return AMBRYCRC_EINVAL;
  if (capturing) {
    w->captured = true;
    *entry = (size_t)(w - c->ws_list.data());
    *out = w->ptr;
    return AMBRYCRC_OK;
  }
  if (!w && c->ws_list.size() >= kMaxStreamWs) {
    // evict the least recently used stream's buffer: retired behind its last call's event
    // (the entry's event moves with it), the entry reused for s
    w = &c->ws_list[0];
    for (auto& e : c->ws_list)
      if (e.tick < w->tick) w = &e;
    if (w->ptr && w->captured) {
      c->ws_kept.push_back(w->ptr);
      if (w->last) (void)hipEventDestroy(w->last);
    } else if (w->ptr) {
      if (w->last) {
        c->ws_retired.push_back({w->ptr, w->last});
      } else {
        (void)hipDeviceSynchronize();  // no event to wait on (its creation failed): drain, then free
        (void)hipFree(w->ptr);
      }
    } else if (w->last) {
      (void)hipEventDestroy(w->last);
    }
    *w = {s, nullptr, 0, nullptr, 0, false};
  }
  if (!w) {
    c->ws_list.push_back({s, nullptr, 0, nullptr, 0, false});
    w = &c->ws_list.back();
  }
  w->tick = ++c->ws_tick;
  *entry = (size_t)(w - c->ws_list.data());
  if (w->bytes >= need) {
    *out = w->ptr;
    return AMBRYCRC_OK;
  }
  if (w->ptr && w->captured) {
    c->ws_kept.push_back(w->ptr);
    w->ptr = nullptr;
    w->captured = false;
  } else if (w->ptr) {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return AMBRYCRC_EHIP;
    if (hipEventRecord(ev, s) != hipSuccess) {
      (void)hipEventDestroy(ev);
      return AMBRYCRC_EHIP;
    }
    c->ws_retired.push_back({w->ptr, ev});
    w->ptr = nullptr;
  }
  const size_t sz = std::max(need, w->bytes * 2);
  w->bytes = 0;
  if (hipMalloc(&w->ptr, sz) != hipSuccess) {
    w->ptr = nullptr;
    return AMBRYCRC_ENOMEM;
  }
  w->bytes = sz;
  *out = w->ptr;
  return AMBRYCRC_OK;
}

// Largest chunk the group phase takes whole for a batch of n chunks on c's variant (0: none).
uint64_t batch_small_max(const DevCtx* c, size_t n) {
  if (n < kGroupMinChunks || !variant_groups(c->variant)) return 0;
  return kGroupSmallMax;
}

// exp_fill: SweepArgs::exp_fill (message verify; honoured by the group phase of variant 29).
// crc_in may equal out (an in-place continuation): the plan copies crc_in into the workspace
// before it initialises out, and the CRC kernels read the copy.
int enqueue_batch(DevCtx* c, const uint8_t* base, const uint64_t* off, const uint64_t* len, const uint32_t* crc_in,
                  uint32_t* out, size_t n, void* ws, hipStream_t s, uint32_t* exp_fill, uint8_t* copy_dst,
                  const uint64_t* copy_off, const uint32_t* gate) {
  if (n == 0) return AMBRYCRC_OK;
  PlanArgs p;
  p.gate = gate;
  p.off = off;
  p.len = len;
  p.crc_in = crc_in;
  p.n = (uint32_t)n;
  p.byte_start = static_cast<uint64_t*>(ws);
  const size_t blocks = (n + kPlanPerBlock - 1) / kPlanPerBlock;
  p.block_sum = p.byte_start + n + 1;
  p.block_small = p.block_sum + blocks;
  p.small_total = p.block_small + blocks;
  p.small_idx = reinterpret_cast<uint32_t*>(p.small_total + 5);
  p.crc_stage = crc_in ? p.small_idx + n : nullptr;
  p.out = out;
  p.small_max = copy_dst ? (n >= kGroupMinChunks ? kGroupSmallMax : 0) : batch_small_max(c, n);
  hipError_t e = launch_plan(p, s);
  if (e != hipSuccess) return AMBRYCRC_EHIP;
  SweepArgs t;
  t.base = base;
  t.off = off;
  t.len = len;
  t.crc_in = p.crc_stage;
  t.n = (uint32_t)n;
  t.byte_start = p.byte_start;
  t.img = c->d_img;
  t.out = out;
  t.small_max = p.small_max;
  t.small_total = p.small_total;
  t.small_idx = p.small_idx;
  t.exp_fill = exp_fill;
  t.window = c->window;
  t.copy_dst = copy_dst;
  t.copy_off = copy_off;
  t.gate = gate;
  if (gate && !copy_dst) return AMBRYCRC_EINVAL;  // only the copy-through sweep checks the gate
  EventPair ev{nullptr, nullptr};
  if (c->timing) {
    std::lock_guard<std::mutex> g(c->ev_mu);
    if (!c->free_events.empty()) {
      ev = c->free_events.back();
      c->free_events.pop_back();
    } else if (hipEventCreate(&ev.a) != hipSuccess || hipEventCreate(&ev.b) != hipSuccess) {
      return AMBRYCRC_EHIP;
    }
    if (hipEventRecord(ev.a, s) != hipSuccess) return AMBRYCRC_EHIP;
  }
  e = copy_dst ? launch_sweep_copy(t, c->grid, c->num_cu, c->variant == kVariantSplit ? kVariantSplit : kVariantDefault, s)
               : launch_sweep(t, c->grid, c->num_cu, c->variant, s);
  if (e != hipSuccess) return AMBRYCRC_EHIP;
  if (c->timing) {
    if (hipEventRecord(ev.b, s) != hipSuccess) return AMBRYCRC_EHIP;
    std::lock_guard<std::mutex> g(c->ev_mu);
    c->pending.push_back(ev);
  }
  return AMBRYCRC_OK;
}

// Device pointers a and b of n uint32 each either coincide or do not overlap (in-place
// continuation d_out == d_crc_in is supported; a shifted overlap is not).
bool same_or_disjoint(const uint32_t* a, const uint32_t* b, size_t n) {
  if (!a || !b || a == b) return true;
  const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
  return x + 4 * n <= y || y + 4 * n <= x;
}

std::atomic<int> g_cpu_threads{0};  // the process's CPU-leg budget (ambrycrc_set_host_cpu_threads(-1, n)); 0: default

int host_cpu_share() {
  static const int share = [] {
    int n = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
    // a cgroup v2 CPU quota ("max 100000" when unlimited): a container's share of a larger machine
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long period = 0;
      if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
        const long long quota = atoll(q);
        if (quota > 0) n = std::min<long long>(n, std::max<long long>(1, (quota + period - 1) / period));
      }
      fclose(f);
    }
    if (const char* v = getenv("OMP_NUM_THREADS")) {
      const int t = atoi(v);
      if (t > 0) n = std::min(n, t);
    }
    return std::min(n, 256);
  }();
  return share;
}

int host_cpu_threads(const DevCtx* c) {
  int t = c ? c->cpu_threads.load(std::memory_order_relaxed) : 0;
  if (t <= 0) t = g_cpu_threads.load(std::memory_order_relaxed);
  if (t > 0) return t;
  if (const char* v = getenv("AMBRYCRC_CPU_THREADS")) {
    const int e = atoi(v);
    if (e > 0) return std::min(e, 256);
  }
  return std::max(1, host_cpu_share() / 2);
}

namespace {
// The calibration for `t` threads: each thread hashes its own slice (16 MiB, 256 MiB in all at most,
// 1 MiB at least) of a buffer the calling thread wrote with nontemporal stores -- so the timed pass
// reads DRAM, not the L3, from the pages one writer placed, as a caller's buffer is. Slices each
// thread wrote itself read 440-679 GiB/s against 172-246 measured on a 2 GiB sample the main thread
// wrote (r05ao, r05aq: 16 threads, their own slices near them and in their CCDs' L3); a single
// thread times threads (round 5's first form): 662 against 262.
double calibrate_cpu(int t) {
  const size_t slice = std::max<size_t>(1u << 20, std::min<size_t>(16u << 20, ((size_t)256 << 20) / (size_t)t)) &
                       ~size_t(4095);
  const size_t total = slice * (size_t)t;
  std::unique_ptr<uint8_t[]> buf(new (std::nothrow) uint8_t[total]);  // not zero-filled: first touch below
  if (!buf) return 1.0;
  // The threads hash their slices once from a common start (all spawned and waiting: spawning
  // inside the timed span read ~half the rate on a 16-CPU box), timed from the start to the last
  // thread's end. (A second pass would read the L3.)
  std::atomic<int> ready{0};
  std::atomic<int> go{0};
  std::atomic<int64_t> last_end{0};
  std::atomic<uint32_t> sink{0};
  std::vector<std::thread> th;
  th.reserve(t);
  {
    uint8_t* p = buf.get();
#if defined(__x86_64__)
    for (size_t i = 0; i < total; i += 16) {  // 16-B aligned (new[] of >= 1 MiB, 4 KiB slices)
      const __m128i v = _mm_set_epi32((int)(i * 131u), (int)(i * 7u), (int)(i ^ 0x5bd1e995u), (int)i);
      _mm_stream_si128(reinterpret_cast<__m128i*>(p + i), v);
    }
    _mm_sfence();
#else
    for (size_t i = 0; i < total; ++i) p[i] = (uint8_t)(i * 131u + 7u);
#endif
  }
  auto body = [&](int k) {
    const uint8_t* p = buf.get() + slice * (size_t)k;
    ready.fetch_add(1);
    while (go.load(std::memory_order_acquire) == 0) std::this_thread::yield();
    sink ^= ambrycrc_update(0, p, slice);
    const int64_t e = std::chrono::steady_clock::now().time_since_epoch().count();
    int64_t cur = last_end.load();
    while (e > cur && !last_end.compare_exchange_weak(cur, e)) {
    }
  };
  try {
    for (int k = 0; k < t; ++k) th.emplace_back(body, k);
  } catch (...) {  // no thread for every slice (the C ABI must not throw): release them, no estimate
    go.store(1, std::memory_order_release);
    for (auto& x : th) x.join();
    return 1.0;
  }
  // (the main thread sleeps while it waits: spinning would take a CPU from the hashing threads)
  while (ready.load() < t) std::this_thread::sleep_for(std::chrono::microseconds(20));
  const int64_t t0 = std::chrono::steady_clock::now().time_since_epoch().count();
  go.store(1, std::memory_order_release);
  for (auto& x : th) x.join();
  const double best = std::chrono::duration<double>(std::chrono::steady_clock::duration(last_end.load() - t0)).count();
  if (!(best > 0)) return 1.0;
  return (double)total / best / (double)(1ull << 30);
}
}  // namespace

double host_cpu_gibps(int threads) {
  static std::mutex mu;
  static std::vector<std::pair<int, double>> cache;  // (threads, GiB/s), one calibration per budget
  threads = std::max(1, std::min(threads, 256));
  std::lock_guard<std::mutex> g(mu);  // one calibration at a time: concurrent ones would share the CPUs
  for (const auto& e : cache)
    if (e.first == threads) return e.second;
  const double r = calibrate_cpu(threads);
  cache.emplace_back(threads, r);
  return r;
}

// The CPU leg's CRC rate on c: as its large calls measured it, else the calibration at c's budget.
double host_batch_cpu_gibps(const DevCtx* c) {
  const int t = host_cpu_threads(c);
  const double r = c ? c->cpu_batch_gibps[std::min(t, DevCtx::kMaxCpuThreads)].load() : -1.0;
  return r >= 0 ? r : host_cpu_gibps(t);
}

bool host_take_cpu(DevCtx* c, int device, int pinned, uint64_t bytes) {
  if (device < 0) return true;
  if (!c || c->host_policy == 1) return false;
  if (c->host_policy == 2) return true;
  if (pinned) return false;
  const bool cpu = host_batch_cpu_gibps(c) > c->gpu_host_gibps.load();
  if (bytes >= (64ull << 20) && c->batch_calls.fetch_add(1) % 16 == 15) return !cpu;  // the other leg's rate
  return cpu;
}

void host_note_cpu(DevCtx* c, uint64_t bytes, double seconds) {
  if (!c || bytes < (64ull << 20) || seconds <= 0) return;
  const double r = (double)bytes / seconds / (double)(1ull << 30);
  std::atomic<double>& a = c->cpu_batch_gibps[std::min(host_cpu_threads(c), DevCtx::kMaxCpuThreads)];
  const double old = a.load();
  a.store(old < 0 ? r : 0.5 * old + 0.5 * r);
}

// The CPU leg of a message entry before it has been measured: verify parses and CRCs each
// message, the transform also copies it out (measured on 16 CPUs, r05ag: verify 86 / 142 GiB/s and
// transform 40 / 60 GiB/s for 4 KiB / 64 KiB PUTs, against a CRC rate of 146-262: ~50 % and ~25 %).
double host_msg_cpu_gibps(const DevCtx* c, int op) {
  const double r = c->msg_cpu_gibps[op].load();
  return r >= 0 ? r
                : host_cpu_gibps(host_cpu_threads(c)) * 0.01 *
                      (op == kMsgVerify ? AMBRY_HOST_VERIFY_CPU_PCT : AMBRY_HOST_XFORM_CPU_PCT);
}

bool host_take_cpu_msg(DevCtx* c, int device, int pinned, int op, uint64_t bytes) {
  if (device < 0) return true;
  if (!c || c->host_policy == 1) return false;
  if (c->host_policy == 2) return true;
  if (pinned) return false;
  const bool cpu = host_msg_cpu_gibps(c, op) > c->msg_gpu_gibps[op].load();
  if (bytes >= (64ull << 20) && c->msg_calls[op].fetch_add(1) % 16 == 15) return !cpu;  // the other leg's rate
  return cpu;
}

void host_note_msg(DevCtx* c, int op, bool cpu, uint64_t bytes, double seconds) {
  if (!c || bytes < (64ull << 20) || seconds <= 0) return;
  const double r = (double)bytes / seconds / (double)(1ull << 30);
  std::atomic<double>& a = cpu ? c->msg_cpu_gibps[op] : c->msg_gpu_gibps[op];
  const double old = a.load();
  a.store(old < 0 ? r : 0.5 * old + 0.5 * r);
}

void host_note_gpu(DevCtx* c, uint64_t bytes, double seconds) {
  if (!c || bytes < (64ull << 20) || seconds <= 0) return;
  const double r = (double)bytes / seconds / (double)(1ull << 30);
  c->gpu_host_gibps.store(0.5 * c->gpu_host_gibps.load() + 0.5 * r);
}

int setup_slabs(DevCtx* c) {
  if (c->slabs_ready) return AMBRYCRC_OK;
  // member by member, skipping what an earlier (failed) attempt already allocated
  auto hhost = [](auto** p, size_t bytes) {
    return *p || hipHostMalloc(reinterpret_cast<void**>(p), bytes, hipHostMallocDefault) == hipSuccess;
  };
  auto hdev = [](auto** p, size_t bytes) { return *p || hipMalloc(reinterpret_cast<void**>(p), bytes) == hipSuccess; };
  for (auto& s : c->slab) {
    if (!hhost(&s.h_data, kSlabBytes) || !hhost(&s.h_meta, 2 * kSlabChunks * sizeof(uint64_t)) ||
        !hhost(&s.h_out, kSlabChunks * sizeof(uint32_t)) || !hdev(&s.d_data, kSlabBytes) ||
        !hdev(&s.d_meta, 2 * kSlabChunks * sizeof(uint64_t)) || !hdev(&s.d_out, kSlabChunks * sizeof(uint32_t)) ||
        !(s.d_ws || hipMalloc(&s.d_ws, ws_need(kSlabChunks)) == hipSuccess))
      return AMBRYCRC_ENOMEM;
    if (!s.stream && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return AMBRYCRC_EHIP;
    if (!s.done && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return AMBRYCRC_EHIP;
  }
  c->slabs_ready = true;
  return AMBRYCRC_OK;
}

void free_ctx(DevCtx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  if (c->d_img) (void)hipFree(c->d_img);
  if (c->h_words) (void)hipHostFree(c->h_words);
  for (auto& w : c->ws_list) {
    if (w.ptr) (void)hipFree(w.ptr);
    if (w.last) (void)hipEventDestroy(w.last);
  }
  for (auto& r : c->ws_retired) {
    (void)hipFree(r.ptr);
    (void)hipEventDestroy(r.done);
  }
  for (void* p : c->ws_kept) (void)hipFree(p);
  for (DevCtx::XformSide* x : c->xs_list) {
    if (x->side) (void)hipStreamDestroy(x->side);
    if (x->d_gates) (void)hipFree(x->d_gates);
    if (x->d_done) (void)hipFree(x->d_done);
    if (x->fork) (void)hipEventDestroy(x->fork);
    for (hipEvent_t e : x->ev)
      if (e) (void)hipEventDestroy(e);
    delete x;
  }
  for (auto& e : c->pending) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  for (auto& e : c->free_events) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  for (auto& ms : c->msg_slab) {  // allocated member by member on first use; free what exists
    if (ms.h_off) (void)hipHostFree(ms.h_off);
    if (ms.h_status) (void)hipHostFree(ms.h_status);
    if (ms.h_end) (void)hipHostFree(ms.h_end);
    if (ms.d_off) (void)hipFree(ms.d_off);
    if (ms.d_status) (void)hipFree(ms.d_status);
    if (ms.d_end) (void)hipFree(ms.d_end);
    if (ms.d_ws) (void)hipFree(ms.d_ws);
  }
  for (auto& x : c->xform_slab) {
    if (x.h_life) (void)hipHostFree(x.h_life);
    if (x.h_out) (void)hipHostFree(x.h_out);
    if (x.h_olen) (void)hipHostFree(x.h_olen);
    if (x.d_life) (void)hipFree(x.d_life);
    if (x.d_out) (void)hipFree(x.d_out);
    if (x.d_olen) (void)hipFree(x.d_olen);
    if (x.d_ooff) (void)hipFree(x.d_ooff);
    if (x.d_ws) (void)hipFree(x.d_ws);
  }
  for (auto& s : c->slab) {  // whatever setup_slabs got to, even if it failed part way
    if (s.h_data) (void)hipHostFree(s.h_data);
    if (s.h_meta) (void)hipHostFree(s.h_meta);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_data) (void)hipFree(s.d_data);
    if (s.d_meta) (void)hipFree(s.d_meta);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.d_ws) (void)hipFree(s.d_ws);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  delete c;
}

}  // namespace detail
}  // namespace ambrycrc

// ================================================================= C ABI
extern "C" {

const char* ambrycrc_strerror(int code) {
  switch (code) {
    case AMBRYCRC_OK: return "ok";
    case AMBRYCRC_EINVAL: return "invalid argument";
    case AMBRYCRC_EHIP: return "HIP runtime error";
    case AMBRYCRC_ENOMEM: return "out of memory";
    case AMBRYCRC_ENOINIT: return "ambrycrc_init() not called for the current device";
    case AMBRYCRC_ENODEV: return "no usable gfx950 device";
    case AMBRYCRC_ECOMM: return "RCCL unavailable or a collective call failed";
    case AMBRYCRC_EPROBE: return "A/B probe build (wrong CRCs) refused: set AMBRYCRC_ALLOW_PROBE=1 to time it";
    default: return "unknown error";
  }
}

const char* ambrycrc_version(void) {
  // "ambrycrc <semver> gfx950", then " ab-probe-build" and " AMBRY_X=v" for every compile-time
  // knob that differs from its product default (build_knobs.h): the product build has neither.
  static const std::string v = [] {
    std::string s = "ambrycrc 0.4.0 gfx950";
    if (AMBRY_IS_PROBE_BUILD) s += " ab-probe-build";
#define AMBRY_KNOB_REPORT(name, def) \
  if ((long)(name) != (long)(def)) s += " " #name "=" + std::to_string((long)(name));
    AMBRY_KNOB_LIST(AMBRY_KNOB_REPORT)
#undef AMBRY_KNOB_REPORT
    return s;
  }();
  return v.c_str();
}

uint32_t ambrycrc_update(uint32_t crc, const void* p, size_t n) {
  if (!p || n == 0) return crc;
  return ~host_update_reg(~crc, static_cast<const uint8_t*>(p), n);
}

const char* ambrycrc_host_impl(void) { return host_impl_name(host_impl()); }

uint32_t ambrycrc_update_iov(uint32_t crc, const void* const* ptrs, const size_t* lens, size_t n) {
  if (!ptrs || !lens) return crc;
  uint32_t reg = ~crc;
  for (size_t i = 0; i < n; ++i)
    if (ptrs[i] && lens[i]) reg = host_update_reg(reg, static_cast<const uint8_t*>(ptrs[i]), lens[i]);
  return ~reg;
}

int ambrycrc_batch_cpu(const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in, uint32_t* out, size_t n,
                       int threads) {
  if (n == 0) return AMBRYCRC_OK;
  if (!ptrs || !lens || !out || threads < 0) return AMBRYCRC_EINVAL;
  for (size_t i = 0; i < n; ++i)
    if (lens[i] && !ptrs[i]) return AMBRYCRC_EINVAL;
  if (threads == 0) {
    cpu_set_t set;
    threads = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
  }
  threads = (int)std::min<size_t>((size_t)std::max(threads, 1), n);
  auto run = [&](size_t a, size_t b) {
    for (size_t i = a; i < b; ++i) {
      const uint32_t c = crc_in ? crc_in[i] : 0u;
      out[i] = lens[i] ? ~host_update_reg(~c, static_cast<const uint8_t*>(ptrs[i]), lens[i]) : c;
    }
  };
  if (threads == 1) {
    run(0, n);
    return AMBRYCRC_OK;
  }
  std::vector<size_t> cut(threads + 1, n);
  const int rc = ambrycrc_shard_by_bytes(lens, n, threads, cut.data());
  if (rc) return rc;
  std::vector<std::thread> th;
  th.reserve(threads - 1);
  for (int t = 1; t < threads; ++t) {
    if (cut[t] >= cut[t + 1]) continue;
    try {
      th.emplace_back(run, cut[t], cut[t + 1]);
    } catch (...) {  // no thread (the C ABI does not throw): the part runs here
      run(cut[t], cut[t + 1]);
    }
  }
  run(cut[0], cut[1]);
  for (auto& t : th) t.join();
  return AMBRYCRC_OK;
}

uint32_t ambrycrc_update_byte(uint32_t crc, int b) {
  const HostTables& h = host_tables();
  uint32_t c = ~crc;
  c = (c >> 8) ^ h.t[0][(c ^ (uint32_t)b) & 0xff];
  return ~c;
}

uint32_t ambrycrc_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return gf2_mul(crc1, host_xpow8(len2)) ^ crc2;
}

uint32_t ambrycrc_zeros(uint32_t crc, uint64_t n) {
  // register' = register * x^(8n); value = ~register.
  return ~gf2_mul(~crc, host_xpow8(n));
}

int ambrycrc_init(int device) {
  if (device < 0 || device >= kMaxDevices) return AMBRYCRC_EINVAL;
  if (AMBRY_IS_PROBE_BUILD) {  // a timing build: its CRCs are wrong by construction
    const char* allow = getenv("AMBRYCRC_ALLOW_PROBE");
    if (!allow || strcmp(allow, "1") != 0) return AMBRYCRC_EPROBE;
  }
  std::lock_guard<std::mutex> g(g_mu);
  if (g_ctx[device]) return AMBRYCRC_OK;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device >= count) return AMBRYCRC_ENODEV;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return AMBRYCRC_EHIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return AMBRYCRC_EHIP;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    (void)hipSetDevice(prev);
    return AMBRYCRC_ENODEV;
  }
  DevCtx* c = new DevCtx();
  c->device = device;
  c->num_cu = prop.multiProcessorCount;
  c->grid = c->num_cu;
  // AMBRYCRC_VARIANT selects a built-in shape for A/B runs; anything else is ignored (a
  // stray value must never change the checksums).
  if (const char* v = getenv("AMBRYCRC_VARIANT")) {
    char* end = nullptr;
    const long x = strtol(v, &end, 10);
    if (end != v && *end == '\0' && x >= 0 && x < 1000 && variant_supported((int)x)) c->variant = (int)x;
  }
  if (const char* v = getenv("AMBRYCRC_REGION")) c->region_mode = strcmp(v, "0") == 0 ? 0 : strcmp(v, "1") == 0 ? 1 : 2;
  if (const char* v = getenv("AMBRYCRC_STREAM_PUT_MAX")) {  // A/B: serialize copy mode's streamed form (0: off)
    char* end = nullptr;
    const unsigned long x = strtoul(v, &end, 10);
    if (end != v && *end == '\0') c->stream_put_max = x < kStreamPutMax ? x : kStreamPutMax;
  }
  if (const char* v = getenv("AMBRYCRC_XFORM_SIDE")) c->xform_side = strcmp(v, "0") == 0 ? 0 : 1;  // A/B: §12.9
  {  // the side-stream verdict needs hipStreamWaitValue32
    int can = 0;
    if (hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device) != hipSuccess || !can)
      c->xform_side = 0;
  }
  if (const char* v = getenv("AMBRYCRC_XFORM_FAST_MAX")) {  // A/B: the transform fast path's cut-off
    char* end = nullptr;
    const unsigned long long x = strtoull(v, &end, 10);
    if (end != v && *end == '\0' && x <= (1ull << 30)) c->xform_fast_max = x;
  }
  if (const char* v = getenv("AMBRYCRC_FUSED_PROC")) {  // A/B: processor waves of the one-pass kernels
    char* end = nullptr;
    const long x = strtol(v, &end, 10);
    if (end != v && *end == '\0' && x >= 0 && x <= kFusedProcMax) c->fused_proc = (int)x;
  }
  if (const char* v = getenv("AMBRYCRC_REGION_MAX_PER_MESSAGE")) {  // A/B: the region-mode cut-off
    char* end = nullptr;
    const unsigned long long x = strtoull(v, &end, 10);
    if (end != v && *end == '\0' && x > 0 && x <= (1ull << 30)) c->region_max = x;
  }
  if (const char* v = getenv("AMBRYCRC_XFORM_HOST_VERDICT")) c->xform_host_verdict = strcmp(v, "1") == 0;
  std::vector<uint32_t> img = build_table_image();
  // the table image, then one 256-B line of device words (d_path)
  const size_t img_bytes = (img.size() * 4 + 255) & ~size_t(255);
  if (hipMalloc(reinterpret_cast<void**>(&c->d_img), img_bytes + 256) != hipSuccess) {
    delete c;
    return AMBRYCRC_ENOMEM;
  }
  c->d_path = c->d_img + img_bytes / 4;
  if (hipMemcpy(c->d_img, img.data(), img.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_path, 0xFF, 256) != hipSuccess) {
    free_ctx(c);
    return AMBRYCRC_EHIP;
  }
  if (hipHostMalloc(reinterpret_cast<void**>(&c->h_words), DevCtx::kHostWords * sizeof(uint32_t),
                    hipHostMallocDefault) != hipSuccess) {
    c->h_words = nullptr;
    free_ctx(c);
    return AMBRYCRC_ENOMEM;
  }
  g_ctx[device] = c;
  (void)hipSetDevice(prev);
  return AMBRYCRC_OK;
}

int ambrycrc_shutdown(void) {
  std::lock_guard<std::mutex> g(g_mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (int d = 0; d < kMaxDevices; ++d) {
    free_ctx(g_ctx[d]);
    g_ctx[d] = nullptr;
  }
  (void)hipSetDevice(prev);
  return AMBRYCRC_OK;
}

size_t ambrycrc_workspace_bytes(size_t n) { return ws_need(n); }

int ambrycrc_batch_dev(const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len, const uint32_t* d_crc_in,
                       uint32_t* d_out, size_t n, void* d_ws, size_t ws_bytes, hipStream_t stream) {
  if (n == 0) return AMBRYCRC_OK;
  if (!d_base || !d_off || !d_len || !d_out || n >= (1ull << 31)) return AMBRYCRC_EINVAL;
  if (!same_or_disjoint(d_crc_in, d_out, n)) return AMBRYCRC_EINVAL;
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  WsLease lease;
  const int rc = lease.acquire(c, stream, &d_ws, ws_bytes, ws_need(n));
  if (rc) return rc;
  return enqueue_batch(c, d_base, d_off, d_len, d_crc_in, d_out, n, d_ws, stream);
}

int ambrycrc_verify_dev(const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len, const uint32_t* d_crc_in,
                        const uint32_t* d_expected, uint32_t* d_out, uint8_t* d_mismatch, uint32_t* d_mismatch_count,
                        size_t n, void* d_ws, size_t ws_bytes, hipStream_t stream) {
  if (n == 0) return AMBRYCRC_OK;
  if (!d_base || !d_off || !d_len || !d_expected || n >= (1ull << 31)) return AMBRYCRC_EINVAL;
  if (!same_or_disjoint(d_crc_in, d_out, n)) return AMBRYCRC_EINVAL;
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  // Without a caller d_out, the CRCs live in the workspace after the batch's own part.
  const size_t extra = d_out ? 0 : ((n * sizeof(uint32_t) + 255) & ~size_t(255));
  WsLease lease;
  int rc = lease.acquire(c, stream, &d_ws, ws_bytes, ws_need(n) + extra);
  if (rc) return rc;
  if (!d_out) d_out = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_ws) + ws_need(n));
  rc = enqueue_batch(c, d_base, d_off, d_len, d_crc_in, d_out, n, d_ws, stream);
  if (rc) return rc;
  return hip_err(launch_verify(d_out, d_expected, d_mismatch, d_mismatch_count, (uint32_t)n, stream));
}

// ambrycrc_batch_host's GPU leg (the dispatcher below picks it or the CPU leg).
static int batch_host_gpu(DevCtx* c, const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in,
                          uint32_t* out, size_t n, int device, int pinned) {
  std::lock_guard<std::mutex> g(c->mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return AMBRYCRC_EHIP;
  int rc = setup_slabs(c);
  if (rc) return rc;

  // Pieces: chunks are cut at slab boundaries; pieces of one chunk are combined on the host.
  struct Piece {
    size_t chunk;
    uint64_t pos, len;
  };
  std::vector<uint32_t> acc(n, 0u);
  for (size_t i = 0; i < n; ++i) acc[i] = crc_in ? crc_in[i] : 0u;

  size_t ci = 0;
  uint64_t cpos = 0;
  int k = 0;  // slabs issued; slab k uses ring entry k % kSlabs
  std::vector<Piece> inflight[kSlabs];
  std::vector<CopyJob> copies;
  auto drain = [&](int which) -> int {
    HostSlab& s = c->slab[which];
    if (inflight[which].empty()) return AMBRYCRC_OK;
    if (hipEventSynchronize(s.done) != hipSuccess) return AMBRYCRC_EHIP;
    for (size_t j = 0; j < inflight[which].size(); ++j) {
      const Piece& p = inflight[which][j];
      acc[p.chunk] = gf2_mul(acc[p.chunk], host_xpow8(p.len)) ^ s.h_out[j];  // combine(acc, piece, len)
    }
    inflight[which].clear();
    return AMBRYCRC_OK;
  };
  while (ci < n) {
    const int w = k % kSlabs;
    rc = drain(w);  // the oldest slab in flight: the one we are about to refill
    if (rc) break;
    HostSlab& s = c->slab[w];
    uint64_t used = 0;
    size_t np = 0;
    copies.clear();
    while (ci < n && np < kSlabChunks) {
      const uint64_t rem = lens[ci] - cpos;
      const uint64_t room = kSlabBytes - used;
      if (rem > 0 && room < 16) break;
      const uint64_t take = std::min(rem, room);
      if (take > 0 && !ptrs[ci]) {
        rc = AMBRYCRC_EINVAL;
        break;
      }
      const uint8_t* src = static_cast<const uint8_t*>(ptrs[ci]) + cpos;
      if (pinned) {
        if (take && hipMemcpyAsync(s.d_data + used, src, take, hipMemcpyHostToDevice, s.stream) != hipSuccess) {
          rc = AMBRYCRC_EHIP;
          break;
        }
      } else if (take) {
        copies.push_back({s.h_data + used, src, take});
      }
      s.h_meta[np] = used;
      s.h_meta[kSlabChunks + np] = take;
      inflight[w].push_back({ci, cpos, take});
      ++np;
      used = (used + take + 15) & ~uint64_t(15);
      cpos += take;
      if (cpos >= lens[ci]) {
        ++ci;
        cpos = 0;
      }
      if (used >= kSlabBytes) break;
    }
    if (rc) break;
    if (!pinned && used) {
      uint64_t bytes = 0;
      for (const CopyJob& j : copies) bytes += j.n;
      parallel_copy(copies, bytes);  // overlaps the DMA of the slabs already issued
      if (hipMemcpyAsync(s.d_data, s.h_data, std::min<uint64_t>(used, kSlabBytes), hipMemcpyHostToDevice,
                         s.stream) != hipSuccess) {
        rc = AMBRYCRC_EHIP;
        break;
      }
    }
    if (hipMemcpyAsync(s.d_meta, s.h_meta, np * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream) !=
            hipSuccess ||
        hipMemcpyAsync(s.d_meta + kSlabChunks, s.h_meta + kSlabChunks, np * sizeof(uint64_t),
                       hipMemcpyHostToDevice, s.stream) != hipSuccess) {
      rc = AMBRYCRC_EHIP;
      break;
    }
    rc = enqueue_batch(c, s.d_data, s.d_meta, s.d_meta + kSlabChunks, nullptr, s.d_out, np, s.d_ws, s.stream);
    if (rc) break;
    if (hipMemcpyAsync(s.h_out, s.d_out, np * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
        hipEventRecord(s.done, s.stream) != hipSuccess) {
      rc = AMBRYCRC_EHIP;
      break;
    }
    ++k;
  }
  // Oldest slab first: pieces of one chunk must combine in order. On error, still wait
  // for everything issued so no DMA targets a slab the next call refills.
  int rc2 = AMBRYCRC_OK;
  for (int d = 0; d < kSlabs; ++d) {
    const int r = drain((k + d) % kSlabs);
    if (!rc2) rc2 = r;
  }
  (void)hipSetDevice(prev);
  if (rc) return rc;
  if (rc2) return rc2;
  for (size_t i = 0; i < n; ++i) out[i] = acc[i];
  return AMBRYCRC_OK;
}

int ambrycrc_batch_multi(const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in, uint32_t* out,
                         size_t n, const int* devices, int ndev, int pinned) {
  if (ndev <= 0 || ndev > kMaxDevices * 8) return AMBRYCRC_EINVAL;
  if (n == 0) return AMBRYCRC_OK;
  if (!ptrs || !lens || !out) return AMBRYCRC_EINVAL;
  std::vector<int> dev(ndev);
  for (int g = 0; g < ndev; ++g) {
    dev[g] = devices ? devices[g] : g;
    if (!ctx_for(dev[g])) return AMBRYCRC_ENOINIT;
  }
  // host-resident dispatch once for the whole batch: the CPU leg when the CPU threads beat every
  // listed GPU's host path together (auto, pageable), else each range on its GPU
  {
    DevCtx* c0 = ctx_for(dev[0]);
    double gpus = 0;
    for (int g = 0; g < ndev; ++g) gpus += ctx_for(dev[g])->gpu_host_gibps.load();
    const int policy = c0->host_policy.load();
    const bool cpu = policy == 2 || (policy == 0 && !pinned && host_batch_cpu_gibps(c0) > gpus);
    c0->last_host_path.store(cpu ? 0 : 1);
    if (cpu) return ambrycrc_batch_cpu(ptrs, lens, crc_in, out, n, host_cpu_threads(c0));
  }
  std::vector<size_t> cut(ndev + 1, n);
  const int src = ambrycrc_shard_by_bytes(lens, n, ndev, cut.data());
  if (src) return src;
  std::vector<int> rc(ndev, AMBRYCRC_OK);
  std::vector<std::thread> th;
  th.reserve(ndev);
  for (int r = 0; r < ndev; ++r) {
    const size_t a = cut[r], b = cut[r + 1];
    if (a >= b) continue;
    auto part = [&, r, a, b] {
      rc[r] = batch_host_gpu(ctx_for(dev[r]), ptrs + a, lens + a, crc_in ? crc_in + a : nullptr, out + a, b - a, dev[r],
                             pinned);
    };
    try {
      th.emplace_back(part);
    } catch (...) {  // no thread (the C ABI does not throw): this device's share runs here
      part();
    }
  }
  for (auto& t : th) t.join();
  for (int r = 0; r < ndev; ++r)
    if (rc[r]) return rc[r];
  return AMBRYCRC_OK;
}

int ambrycrc_put_crcs(const uint8_t* const* fields, const uint64_t* field_len, const uint8_t* const* prefix,
                      const uint64_t* prefix_len, const uint32_t* blob_crc, const uint64_t* blob_len, size_t n,
                      uint32_t* wire_out, uint32_t* record_out) {
  if (n == 0) return AMBRYCRC_OK;
  if (!blob_crc || !blob_len) return AMBRYCRC_EINVAL;
  if (wire_out && (!fields || !field_len)) return AMBRYCRC_EINVAL;
  if (record_out && (!prefix || !prefix_len)) return AMBRYCRC_EINVAL;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t xb = host_xpow8(blob_len[i]);  // shared by both combines
    if (wire_out) wire_out[i] = gf2_mul(ambrycrc_update(0, fields[i], field_len[i]), xb) ^ blob_crc[i];
    if (record_out) record_out[i] = gf2_mul(ambrycrc_update(0, prefix[i], prefix_len[i]), xb) ^ blob_crc[i];
  }
  return AMBRYCRC_OK;
}

int ambrycrc_range_checksums_host(const uint8_t* file, uint64_t file_len, const int64_t* first, const int64_t* second,
                                  size_t n, uint32_t* out, int device) {
  if (n == 0) return AMBRYCRC_OK;
  if (!first || !second || !out || (!file && file_len)) return AMBRYCRC_EINVAL;
  for (size_t i = 0; i < n; ++i)
    if (first[i] < 0 || second[i] < 0 || first[i] > second[i]) return AMBRYCRC_EINVAL;
  std::vector<const void*> ptrs(n);
  std::vector<uint64_t> lens(n);
  for (size_t i = 0; i < n; ++i) {
    const uint64_t a = std::min<uint64_t>((uint64_t)first[i], file_len);
    const uint64_t b = std::min<uint64_t>((uint64_t)second[i], file_len);
    ptrs[i] = file ? file + a : nullptr;
    lens[i] = b - a;
  }
  return ambrycrc_batch_host(ptrs.data(), lens.data(), nullptr, out, n, device, 0);
}

int ambrycrc_set_variant(int device, int variant) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (!variant_supported(variant)) return AMBRYCRC_EINVAL;
  c->variant = variant;
  return AMBRYCRC_OK;
}

long ambrycrc_set_put_stream_max(int device, long bytes) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (bytes < 0 || (uint64_t)bytes > kStreamPutMax) return AMBRYCRC_EINVAL;
  const long prev = (long)c->stream_put_max;
  c->stream_put_max = (uint64_t)bytes;
  return prev;
}

int ambrycrc_set_region_mode(int device, int enable) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (enable < 0 || enable > 2) return AMBRYCRC_EINVAL;
  c->region_mode = enable;
  return AMBRYCRC_OK;
}


int ambrycrc_get_region_mode(int device) {
  DevCtx* c = ctx_for(device);
  return c ? c->region_mode : AMBRYCRC_ENOINIT;
}

int ambrycrc_last_message_mode(int device) {
  DevCtx* c = ctx_for(device);
  return c ? c->last_msg_mode.load() : AMBRYCRC_ENOINIT;
}

int ambrycrc_last_transform_path(int device) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  const int p = c->last_xform_path.load();
  if (p != 2) return p;
  // decided on the device: region_patch_kernel's word, once the device has finished the call
  uint32_t w = ~0u;
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(&w, c->d_path, sizeof w, hipMemcpyDeviceToHost) != hipSuccess) {
    (void)hipSetDevice(prev);
    return AMBRYCRC_EHIP;
  }
  (void)hipSetDevice(prev);
  return w <= 1 ? (int)w : -1;
}

int ambrycrc_set_transform_verdict(int device, int host) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (host != 0 && host != 1) return AMBRYCRC_EINVAL;
  const int prev = c->xform_host_verdict.exchange(host);
  return prev;
}

int ambrycrc_get_variant(int device) {
  DevCtx* c = ctx_for(device);
  return c ? c->variant : AMBRYCRC_ENOINIT;
}

int ambrycrc_set_grid(int device, int workgroups) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (workgroups < 0) return AMBRYCRC_EINVAL;
  c->grid = workgroups ? workgroups : c->num_cu;
  return AMBRYCRC_OK;
}

int ambrycrc_grid_size(int device) {
  DevCtx* c = ctx_for(device);
  return c ? c->grid : 0;
}

int ambrycrc_set_window(int device, uint64_t bytes) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (bytes != 0 && bytes < (1u << 20)) return AMBRYCRC_EINVAL;
  c->window = bytes;
  return AMBRYCRC_OK;
}

int ambrycrc_timing_enable(int device, int enable) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  c->timing = enable != 0;
  return AMBRYCRC_OK;
}

int ambrycrc_timing_collect_each(int device, float* ms_out, int cap, int* launches) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (cap < 0 || (cap > 0 && !ms_out)) return AMBRYCRC_EINVAL;
  std::lock_guard<std::mutex> g(c->ev_mu);
  int cnt = 0;
  for (auto& e : c->pending) {
    if (hipEventSynchronize(e.b) != hipSuccess) return AMBRYCRC_EHIP;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.a, e.b) != hipSuccess) return AMBRYCRC_EHIP;
    if (cnt < cap) ms_out[cnt] = ms;
    ++cnt;
    c->free_events.push_back(e);
  }
  c->pending.clear();
  if (launches) *launches = cnt;
  return AMBRYCRC_OK;
}

int ambrycrc_timing_collect(int device, double* total_ms, int* launches) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  std::vector<float> ms;
  {
    std::lock_guard<std::mutex> g(c->ev_mu);
    ms.resize(c->pending.size() + 4096);  // room for launches recorded meanwhile
  }
  int cnt = 0;
  const int rc = ambrycrc_timing_collect_each(device, ms.data(), (int)ms.size(), &cnt);
  if (rc != AMBRYCRC_OK) return rc;
  double sum = 0;
  cnt = std::min(cnt, (int)ms.size());
  for (int i = 0; i < cnt; ++i) sum += ms[i];
  if (total_ms) *total_ms = sum;
  if (launches) *launches = cnt;
  return AMBRYCRC_OK;
}

int ambrycrc_fill_random_dev(uint8_t* d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off,
                             hipStream_t stream) {
  if (nbytes == 0) return AMBRYCRC_OK;
  if (!d_dst || (reinterpret_cast<uintptr_t>(d_dst) & 15) || (stream_off & 15)) return AMBRYCRC_EINVAL;
  return hip_err(launch_fill(d_dst, nbytes, seed, stream_off, stream));
}

int ambrycrc_debug_readbw_dev(const uint8_t* d_base, uint64_t nbytes, uint32_t* d_out, int variant,
                              hipStream_t stream) {
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  if (!d_base || !d_out) return AMBRYCRC_EINVAL;
  return hip_err(launch_readbw(d_base, nbytes, d_out, c->grid, variant, stream));
}

size_t ambrycrc_messages_workspace_bytes(size_t m) {
  // job arrays, then the batch workspace of job mode or the run sums of region mode (a region of
  // up to kRegionMaxPerMessage bytes per message: region / 16 bytes + two super-blocks' slack)
  const size_t region = m * (kRegionMaxPerMessage / 16) + 2048 + 512 + 4 * m;
  return msg_jobs_bytes(m) + std::max(ws_need((size_t)kMsgSlots * m), region);
}

}  // extern "C"

namespace ambrycrc {
namespace detail {

// The device message pipeline (parse -> plan + sweep -> reduce) on `stream`; d_ws holds
// at least ambrycrc_messages_workspace_bytes(m).
size_t msg_jobs_bytes(size_t m) {
  const size_t j = (size_t)kMsgSlots * m;
  return (j * 2 * sizeof(uint64_t) + j * 2 * sizeof(uint32_t) + j + 255) & ~size_t(255);
}

// A processor wave finishes a 64-message batch in ~20-40 us (a chain of dependent reads under the
// streamers' load), so the processors a CU needs grow with its messages; the rest of its waves
// stream, and too few streamers starve them (a cliff: 3 of 12 at 1 KiB blobs, 0.367 -> 0.438 ms).
// Measured per messages per CU (r04am-ao, r04au; ms per call): verify form (12 waves) 4 KiB blobs
// (1,024 per CU) best at 5 (0.377; 8: 0.410), 3 KiB (1,280) at 6 (0.408; 5: 0.418), 2 KiB (1,536)
// at 6 (0.374; 5: 0.397, 8: 0.387), 1 KiB (2,048) at 8 (0.367), 100 B (4,096) at 9 (0.532; 8:
// 0.575); copy form (8 waves) at 4 from 128 to 1,024 per CU (4 KiB PUTs 0.663; 3: 0.69, 5: 0.78;
// 16 KiB PUTs 0.549, 2: 0.562; 32 KiB 0.563, 2: 0.570; r04ba). Verify below 512 per CU (not swept):
// one processor per 128 messages, at least 2.
uint32_t fused_proc_waves(const DevCtx* c, size_t m, bool copy) {
  const int waves = copy ? kFusedWavesCopy : kFusedWavesVerify;
  const int most = std::min(kFusedProcMax, waves - 2);  // at least two streamers
  if (c->fused_proc > 0) return (uint32_t)std::min(c->fused_proc, most);
  const size_t per_cu = m / (size_t)std::max(1, c->num_cu);
  int p;
  if (copy) p = 4;
  else if (per_cu <= 512) p = (int)std::max<size_t>(2, (per_cu + 127) / 128);
  else p = per_cu <= 1024 ? 5 : per_cu <= 1536 ? 6 : per_cu <= 3072 ? 8 : 9;
  return (uint32_t)std::min(p, most);
}

// The long-record list in the job arrays' space (unused in region mode), `bytes` long: records from
// byte 64 (at most 4,096), then the piece slots.
static void set_long_list(LongList& l, uint8_t* w, size_t bytes) {
  l.rec = reinterpret_cast<LongRec*>(w + 64);
  l.cap = (uint32_t)std::min<size_t>(4096, (bytes - 64) / 2 / sizeof(LongRec));
  const size_t sb = (64 + l.cap * sizeof(LongRec) + 255) & ~size_t(255);
  l.slot = reinterpret_cast<uint32_t*>(w + sb);
  l.pcap = (uint32_t)std::min<size_t>(1u << 30, (bytes - sb) / sizeof(uint32_t));
}

int enqueue_messages(DevCtx* c, const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off, size_t m,
                     uint32_t* d_status, uint64_t* d_msg_end, void* d_ws, size_t ws_bytes, hipStream_t stream) {
  const bool region = c->region_mode && region_len > 0 && region_len <= c->region_max * (uint64_t)m &&
                      msg_jobs_bytes(m) + region_ws_bytes(d_region, region_len, m) <= ws_bytes;
  MsgStage st;
  c->last_msg_mode.store(region ? c->region_mode : 0);
  if (!region) {
    const int rc = enqueue_messages_parse(c, d_region, region_len, d_msg_off, m, d_status, d_msg_end, d_ws, stream, &st);
    return rc ? rc : enqueue_messages_check(c, st, stream);
  }
  // Region mode: pass 1 sweeps the region into 64-B run sums (kept where job mode keeps its batch
  // workspace), pass 2 parses every message and assembles its record CRCs from them.
  st.a.region = d_region;
  st.a.region_len = region_len;
  st.a.msg_off = d_msg_off;
  st.a.m = m;
  st.a.img = c->d_img;
  st.a.status = d_status;
  st.a.msg_end = d_msg_end;
  st.a.inline_max = 0;
  st.batch_ws = static_cast<uint8_t*>(d_ws) + msg_jobs_bytes(m);
  RegionArgs r;
  const uintptr_t rp = reinterpret_cast<uintptr_t>(d_region);
  r.base = d_region - (rp & 63u);
  r.reg0 = rp & 63u;
  r.reg_end = r.reg0 + region_len;
  r.lo16 = r.reg0 & ~uint64_t(15);
  r.hi16 = (r.reg_end - 1) & ~uint64_t(15);
  r.nsb = region_nsb(d_region, region_len);
  r.rk = static_cast<uint32_t*>(st.batch_ws);
  r.img = c->d_img;
  if (c->region_mode == 2) {  // the two-pass form: runs kernel, then one thread per message
    // long records (more than region::kLongRuns runs) listed in the job arrays' space, which
    // region mode does not use: the whole grid takes them after pass 2
    uint8_t* lw = static_cast<uint8_t*>(d_ws);
    r.lng.ctr = reinterpret_cast<unsigned long long*>(lw);
    r.lng.claim = reinterpret_cast<uint32_t*>(lw + 8);
    set_long_list(r.lng, lw, msg_jobs_bytes(m));
    if (launch_region_runs(r, c->grid, stream) != hipSuccess ||
        launch_region_msg(st.a, r, c->num_cu, stream) != hipSuccess)
      return AMBRYCRC_EHIP;
    return hip_err(launch_region_long(st.a, r, c->num_cu, stream));
  }
  FusedArgs f;
  f.a = st.a;
  f.g = r;
  f.ngroups = (r.nsb + 3) / 4;
  f.ctl = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(st.batch_ws) + region_rk_bytes(d_region, region_len));
  f.defer = f.ctl + 64;
  f.nproc = fused_proc_waves(c, m, false);
  // long records: listed by the processors (records in the job arrays' space, as the two-pass
  // form's; the counters in ctl, zeroed with it), taken by region_long_kernel after the tail
  f.g.lng.ctr = reinterpret_cast<unsigned long long*>(f.ctl + 4);
  f.g.lng.claim = f.ctl + 6;
  set_long_list(f.g.lng, static_cast<uint8_t*>(d_ws), msg_jobs_bytes(m));
  if (hipMemsetAsync(f.ctl, 0, 32, stream) != hipSuccess) return AMBRYCRC_EHIP;
  return hip_err(launch_region_fused(f, c->num_cu, stream));
}

int enqueue_messages_parse(DevCtx* c, const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off,
                           size_t m, uint32_t* d_status, uint64_t* d_msg_end, void* d_ws, hipStream_t stream,
                           MsgStage* st, const TransformArgs* desc, const uint32_t* gate) {
  const size_t j = (size_t)kMsgSlots * m;
  uint8_t* w = static_cast<uint8_t*>(d_ws);
  MsgArgs& a = st->a;
  a.gate = gate;
  a.region = d_region;
  a.region_len = region_len;
  a.msg_off = d_msg_off;
  a.m = m;
  a.img = c->d_img;
  a.job_off = reinterpret_cast<uint64_t*>(w);
  a.job_len = a.job_off + j;
  a.expected = reinterpret_cast<uint32_t*>(a.job_len + j);
  uint32_t* crc = a.expected + j;
  a.crc = crc;
  a.status = d_status;
  a.msg_end = d_msg_end;
  // The class-sized group phase (variant 29) reads the stored CRCs of the records it
  // takes whole; the parse kernel reads the rest.
  const bool inline_exp = variant_groups(c->variant);
  a.inline_max = inline_exp ? batch_small_max(c, j) : 0;
  st->batch_ws = w + msg_jobs_bytes(m);
  st->crc = crc;
  st->j = j;
  return hip_err(desc ? launch_msg_parse_desc(a, *desc, stream) : launch_msg_parse(a, stream));
}

int enqueue_messages_check(DevCtx* c, const MsgStage& st, hipStream_t stream, uint8_t* copy_dst,
                           const uint64_t* copy_off) {
  const MsgArgs& a = st.a;
  // copy-through runs the group-phase kernel whatever c's variant, so the stored CRCs of the records
  // it takes are read there exactly when the parse kernel left them to it (inline_max)
  const int rc = enqueue_batch(c, a.region, a.job_off, a.job_len, nullptr, st.crc, st.j, st.batch_ws, stream,
                               a.inline_max ? a.expected : nullptr, copy_dst, copy_off, copy_dst ? a.gate : nullptr);
  if (rc) return rc;
  return hip_err(launch_msg_reduce(a, stream));
}

}  // namespace detail
}  // namespace ambrycrc

namespace {

uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
uint64_t rd_be64(const uint8_t* p) { return ((uint64_t)rd_be32(p) << 32) | rd_be32(p + 4); }

// member by member, skipping what an earlier (failed) attempt already allocated
template <class T>
bool host_alloc(T** p, size_t bytes) {
  return *p || hipHostMalloc(reinterpret_cast<void**>(p), bytes, hipHostMallocDefault) == hipSuccess;
}
template <class T>
bool dev_alloc(T** p, size_t bytes) {
  return *p || hipMalloc(reinterpret_cast<void**>(p), bytes) == hipSuccess;
}

// The message-verify members of the host slabs (caller holds c->mu, c's device current).
int setup_msg_slabs(DevCtx* c) {
  if (c->msg_slabs_ready) return AMBRYCRC_OK;
  for (MsgSlab& ms : c->msg_slab)
    if (!host_alloc(&ms.h_off, kSlabMsgs * sizeof(uint64_t)) || !host_alloc(&ms.h_status, kSlabMsgs * sizeof(uint32_t)) ||
        !host_alloc(&ms.h_end, kSlabMsgs * sizeof(uint64_t)) || !dev_alloc(&ms.d_off, kSlabMsgs * sizeof(uint64_t)) ||
        !dev_alloc(&ms.d_status, kSlabMsgs * sizeof(uint32_t)) || !dev_alloc(&ms.d_end, kSlabMsgs * sizeof(uint64_t)) ||
        !(ms.d_ws || hipMalloc(&ms.d_ws, ambrycrc_messages_workspace_bytes(kSlabMsgs)) == hipSuccess))
      return AMBRYCRC_ENOMEM;
  c->msg_slabs_ready = true;
  return AMBRYCRC_OK;
}

// The transform members (ambrycrc_transform_messages_host), on top of setup_msg_slabs.
int setup_xform_slabs(DevCtx* c) {
  if (c->xform_slabs_ready) return AMBRYCRC_OK;
  for (XformSlab& x : c->xform_slab)
    if (!host_alloc(&x.h_life, kSlabMsgs * sizeof(int16_t)) || !dev_alloc(&x.d_life, kSlabMsgs * sizeof(int16_t)) ||
        !host_alloc(&x.h_out, kXformOutBytes) || !dev_alloc(&x.d_out, kXformOutBytes) ||
        !host_alloc(&x.h_olen, kSlabMsgs * sizeof(uint64_t)) || !dev_alloc(&x.d_olen, kSlabMsgs * sizeof(uint64_t)) ||
        !dev_alloc(&x.d_ooff, kSlabMsgs * sizeof(uint64_t)) ||
        !(x.d_ws || hipMalloc(&x.d_ws, ambrycrc_transform_workspace_bytes(kSlabMsgs)) == hipSuccess))
      return AMBRYCRC_ENOMEM;
  c->xform_slabs_ready = true;
  return AMBRYCRC_OK;
}

// Bytes from a message's start that the device pipeline may read: the 40-B header window,
// and, when the header's sizes fit the region, the whole message [0, first record + total).
// Every early exit of msg_parse_kernel reads the header alone, so a staging copy of this
// extent gives the same status bits as the whole region would.
uint64_t message_extent(const uint8_t* p, uint64_t rem) {
  const uint64_t hdr = std::min<uint64_t>(rem, 40);
  if (rem < 2) return rem;
  const int v = (int16_t)(((uint32_t)p[0] << 8) | p[1]);
  const uint32_t h = v == 1 ? 34u : v == 2 ? 38u : v == 3 ? 40u : 0u;
  if (h == 0 || rem < h) return hdr;
  int64_t total;
  int32_t rel[kMsgSlots];
  if (v == 1) {
    total = (int64_t)rd_be64(p + 2);
    rel[0] = -1;
    for (int k = 0; k < 4; ++k) rel[k + 1] = (int32_t)rd_be32(p + 10 + 4 * k);
  } else if (v == 2) {
    total = (int64_t)rd_be64(p + 2);
    for (int k = 0; k < 5; ++k) rel[k] = (int32_t)rd_be32(p + 10 + 4 * k);
  } else {
    total = (int64_t)rd_be64(p + 4);
    for (int k = 0; k < 5; ++k) rel[k] = (int32_t)rd_be32(p + 12 + 4 * k);
  }
  int64_t first = -1;
  for (int k = 0; k < kMsgSlots; ++k)
    if (rel[k] != -1) {
      first = rel[k];
      break;
    }
  if (total <= 0 || first < 0 || (uint64_t)total > rem || (uint64_t)first > rem - (uint64_t)total) return hdr;
  return std::max<uint64_t>(hdr, (uint64_t)first + (uint64_t)total);
}

}  // namespace

namespace ambrycrc {
namespace detail {
uint64_t message_extent_of(const uint8_t* p, uint64_t rem) { return message_extent(p, rem); }
}  // namespace detail
}  // namespace ambrycrc

extern "C" {

int ambrycrc_verify_messages_dev(const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off, size_t m,
                                 uint32_t* d_status, uint64_t* d_msg_end, void* d_ws, size_t ws_bytes,
                                 hipStream_t stream) {
  if (m == 0) return AMBRYCRC_OK;
  if (!d_region || !d_msg_off || !d_status || (size_t)kMsgSlots * m >= (1ull << 31)) return AMBRYCRC_EINVAL;
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  WsLease lease;
  size_t need = ambrycrc_messages_workspace_bytes(m);
  // The library's own workspace also covers region mode past the default per-message size
  // (AMBRYCRC_REGION_MAX_PER_MESSAGE, for A/B runs); a caller's is used as sized.
  if (!d_ws && c->region_mode && region_len <= c->region_max * (uint64_t)m)
    need = std::max(need, msg_jobs_bytes(m) + region_ws_bytes(d_region, region_len, m));
  const int rc = lease.acquire(c, stream, &d_ws, ws_bytes, need);
  if (rc) return rc;
  return enqueue_messages(c, d_region, region_len, d_msg_off, m, d_status, d_msg_end, d_ws,
                          ws_bytes ? ws_bytes : need, stream);
}

// ambrycrc_verify_messages_host's GPU leg.
static int verify_messages_host_gpu(DevCtx* c, const uint8_t* region, uint64_t region_len, const uint64_t* msg_off,
                                    size_t m, uint32_t* status, uint64_t* msg_end, int device, int pinned) {
  std::lock_guard<std::mutex> g(c->mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return AMBRYCRC_EHIP;
  int rc = setup_slabs(c);
  if (!rc) rc = setup_msg_slabs(c);
  if (rc) {
    (void)hipSetDevice(prev);
    return rc;
  }

  // Messages in offset order; each slab stages one contiguous span [lo, hi) of the region
  // that covers every packed message's extent. A message whose extent exceeds a slab gets
  // a staging buffer of its own.
  std::vector<size_t> order(m);
  for (size_t i = 0; i < m; ++i) order[i] = i;
  if (!std::is_sorted(msg_off, msg_off + m))  // a recovery scan's offsets already are
    std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return msg_off[x] < msg_off[y]; });
  // Message extents: one header read each, scattered over the region (a cache and TLB miss
  // apiece), so they are read by the copy pool's threads in parallel.
  std::vector<uint64_t> ext(m);
  {
    CopyPool& pool = CopyPool::get();
    const int parts = (int)std::min<size_t>((size_t)pool.threads(), std::max<size_t>(1, m / 4096));
    pool.run(parts, [&](int p) {
      for (size_t i = m * (size_t)p / (size_t)parts; i < m * (size_t)(p + 1) / (size_t)parts; ++i)
        ext[i] = msg_off[i] > region_len ? 0 : message_extent(region + msg_off[i], region_len - msg_off[i]);
    });
  }
  auto extent = [&](size_t i) -> uint64_t { return ext[i]; };

  struct Span {
    uint64_t lo;
    std::vector<size_t> msgs;
  };
  Span inflight[kSlabs];
  auto drain = [&](int which) -> int {
    Span& sp = inflight[which];
    if (sp.msgs.empty()) return AMBRYCRC_OK;
    if (hipEventSynchronize(c->slab[which].done) != hipSuccess) return AMBRYCRC_EHIP;
    const MsgSlab& ms = c->msg_slab[which];
    for (size_t q = 0; q < sp.msgs.size(); ++q) {
      status[sp.msgs[q]] = ms.h_status[q];
      if (msg_end) msg_end[sp.msgs[q]] = ms.h_end[q] ? sp.lo + ms.h_end[q] : 0;
    }
    sp.msgs.clear();
    return AMBRYCRC_OK;
  };
  std::vector<CopyJob> copies;
  size_t oi = 0;
  int k = 0;
  while (oi < m && !rc) {
    const size_t first = order[oi];
    const uint64_t lo = std::min(msg_off[first], region_len);
    if (extent(first) > kSlabBytes) {  // oversize: its own device buffer, synchronously
      uint8_t* d_buf = nullptr;
      uint64_t* d_o = nullptr;
      uint32_t* d_s = nullptr;
      uint64_t* d_e = nullptr;
      void* d_w = nullptr;
      const uint64_t zero = 0;
      uint32_t st = 0;
      uint64_t en = 0;
      if (hipMalloc(reinterpret_cast<void**>(&d_buf), ext[first]) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&d_o), 8) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&d_s), 4) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&d_e), 8) != hipSuccess ||
          hipMalloc(&d_w, ambrycrc_messages_workspace_bytes(1)) != hipSuccess) {
        rc = AMBRYCRC_ENOMEM;
      } else if (hipMemcpy(d_buf, region + lo, ext[first], hipMemcpyHostToDevice) != hipSuccess ||
                 hipMemcpy(d_o, &zero, 8, hipMemcpyHostToDevice) != hipSuccess) {
        rc = AMBRYCRC_EHIP;
      } else {
        rc = enqueue_messages(c, d_buf, ext[first], d_o, 1, d_s, d_e, d_w, ambrycrc_messages_workspace_bytes(1), nullptr);
        if (!rc && (hipMemcpy(&st, d_s, 4, hipMemcpyDeviceToHost) != hipSuccess ||
                    hipMemcpy(&en, d_e, 8, hipMemcpyDeviceToHost) != hipSuccess))
          rc = AMBRYCRC_EHIP;
      }
      (void)hipFree(d_buf);
      (void)hipFree(d_o);
      (void)hipFree(d_s);
      (void)hipFree(d_e);
      (void)hipFree(d_w);
      status[first] = st;
      if (msg_end) msg_end[first] = en ? lo + en : 0;
      ++oi;
      continue;
    }
    const int w = k % kSlabs;
    rc = drain(w);
    if (rc) break;
    HostSlab& s = c->slab[w];
    MsgSlab& ms = c->msg_slab[w];
    Span& sp = inflight[w];
    sp.lo = lo;
    uint64_t hi = lo;
    while (oi < m && sp.msgs.size() < kSlabMsgs) {
      const size_t i = order[oi];
      const uint64_t o = std::min(msg_off[i], region_len);
      const uint64_t e = o + extent(i);
      if (ext[i] > kSlabBytes || std::max(hi, e) - lo > kSlabBytes) break;
      hi = std::max(hi, e);
      ms.h_off[sp.msgs.size()] = o - lo;
      sp.msgs.push_back(i);
      ++oi;
    }
    const uint64_t span = hi - lo;
    // an offset past the region end must stay past the slab end (BAD_LAYOUT either way)
    for (size_t q = 0; q < sp.msgs.size(); ++q)
      if (msg_off[sp.msgs[q]] > region_len) ms.h_off[q] = span + 1;
    if (span) {
      if (pinned) {
        if (hipMemcpyAsync(s.d_data, region + lo, span, hipMemcpyHostToDevice, s.stream) != hipSuccess) rc = AMBRYCRC_EHIP;
      } else {
        copies.clear();
        copies.push_back({s.h_data, region + lo, span});
        parallel_copy(copies, span);  // overlaps the DMA of the slabs already issued
        if (hipMemcpyAsync(s.d_data, s.h_data, span, hipMemcpyHostToDevice, s.stream) != hipSuccess) rc = AMBRYCRC_EHIP;
      }
    }
    const size_t nm = sp.msgs.size();
    if (!rc && hipMemcpyAsync(ms.d_off, ms.h_off, nm * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream) != hipSuccess)
      rc = AMBRYCRC_EHIP;
    if (!rc)
      rc = enqueue_messages(c, s.d_data, span, ms.d_off, nm, ms.d_status, ms.d_end, ms.d_ws,
                            ambrycrc_messages_workspace_bytes(kSlabMsgs), s.stream);
    if (!rc && (hipMemcpyAsync(ms.h_status, ms.d_status, nm * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream) !=
                    hipSuccess ||
                hipMemcpyAsync(ms.h_end, ms.d_end, nm * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream) !=
                    hipSuccess ||
                hipEventRecord(s.done, s.stream) != hipSuccess))
      rc = AMBRYCRC_EHIP;
    if (rc) {
      sp.msgs.clear();
      break;
    }
    ++k;
  }
  int rc2 = AMBRYCRC_OK;
  for (int d = 0; d < kSlabs; ++d) {
    const int r = drain((k + d) % kSlabs);
    if (!rc2) rc2 = r;
  }
  (void)hipSetDevice(prev);
  return rc ? rc : rc2;
}

// ambrycrc_transform_messages_host's GPU leg.
static int transform_messages_host_gpu(DevCtx* c, const uint8_t* region, uint64_t region_len, const uint64_t* msg_off,
                                       size_t m, const int16_t* life_version, int header_version, uint8_t* out,
                                       uint64_t out_cap, uint64_t* out_off, uint64_t* out_len, uint32_t* status,
                                       int device, int pinned) {
  std::lock_guard<std::mutex> g(c->mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return AMBRYCRC_EHIP;
  int rc = setup_slabs(c);
  if (!rc) rc = setup_msg_slabs(c);
  if (!rc) rc = setup_xform_slabs(c);
  if (rc) {
    (void)hipSetDevice(prev);
    return rc;
  }
  // Extents as the verify's (message_extent: a transform reads nothing outside them either).
  std::vector<uint64_t> ext(m);
  {
    CopyPool& pool = CopyPool::get();
    const int parts = (int)std::min<size_t>((size_t)pool.threads(), std::max<size_t>(1, m / 4096));
    pool.run(parts, [&](int p) {
      for (size_t i = m * (size_t)p / (size_t)parts; i < m * (size_t)(p + 1) / (size_t)parts; ++i)
        ext[i] = msg_off[i] > region_len ? 0 : message_extent(region + msg_off[i], region_len - msg_off[i]);
    });
  }
  // Packing follows ambrycrc_transform_messages_dev over the whole batch: message i's bytes go at
  // the sum of the transformed lengths of the messages before it, or it gets AMBRYCRC_MSG_NO_ROOM
  // when they would pass out_cap (that sum still grows by its length, as the device's exclusive
  // scan of the lengths does). Slabs hold runs of consecutive messages in index order, each run's
  // span [lo, hi) staged once; the slab's transform packs its messages from 0 in the same order.
  uint64_t vpos = 0;  // the device scan's running start
  auto place = [&](size_t i, uint32_t st, uint64_t len, const uint8_t* bytes, std::vector<CopyJob>* jobs) {
    if (st == 0 && len) {
      if (vpos + len <= out_cap) {
        if (out_off) out_off[i] = vpos;
        out_len[i] = len;
        status[i] = 0;
        if (jobs) jobs->push_back({out + vpos, bytes, len});
        else memcpy(out + vpos, bytes, len);
      } else {
        if (out_off) out_off[i] = ~0ull;
        out_len[i] = 0;
        status[i] = AMBRYCRC_MSG_NO_ROOM;
      }
      vpos += len;
      return;
    }
    if (out_off) out_off[i] = ~0ull;
    out_len[i] = 0;
    status[i] = st;
  };
  struct Run {
    size_t i0 = 0, n = 0;
  };
  Run inflight[kSlabs];
  std::vector<CopyJob> jobs;
  auto drain = [&](int which) -> int {
    Run& r = inflight[which];
    if (!r.n) return AMBRYCRC_OK;
    if (hipEventSynchronize(c->slab[which].done) != hipSuccess) return AMBRYCRC_EHIP;
    const MsgSlab& ms = c->msg_slab[which];
    const XformSlab& x = c->xform_slab[which];
    jobs.clear();
    uint64_t at = 0, bytes = 0;  // the slab's packed output
    for (size_t q = 0; q < r.n; ++q) {
      const uint64_t len = ms.h_status[q] == 0 ? x.h_olen[q] : 0;
      const size_t before = jobs.size();
      place(r.i0 + q, ms.h_status[q], len, x.h_out + at, &jobs);
      if (jobs.size() > before) bytes += len;
      at += len;
    }
    parallel_copy(jobs, bytes);
    r.n = 0;
    return AMBRYCRC_OK;
  };
  // One message too large for a slab: its own device buffers, synchronously.
  auto oversize = [&](size_t i) -> int {
    const uint64_t lo = std::min(msg_off[i], region_len), n = ext[i];
    const uint64_t cap = ambrycrc_transform_out_bound(n, 1);
    uint8_t *d_buf = nullptr, *d_out = nullptr;
    uint64_t *d_o = nullptr, *d_oo = nullptr, *d_ol = nullptr;
    uint32_t* d_s = nullptr;
    int16_t* d_l = nullptr;
    void* d_w = nullptr;
    std::vector<uint8_t> h;
    const uint64_t zero = 0;
    uint32_t st = 0;
    uint64_t len = 0;
    int e = AMBRYCRC_OK;
    if (hipMalloc(reinterpret_cast<void**>(&d_buf), n) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_out), cap) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_o), 8) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_oo), 8) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_ol), 8) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_s), 4) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_l), 2) != hipSuccess ||
        hipMalloc(&d_w, ambrycrc_transform_workspace_bytes(1)) != hipSuccess) {
      e = AMBRYCRC_ENOMEM;
    } else if (hipMemcpy(d_buf, region + lo, n, hipMemcpyHostToDevice) != hipSuccess ||
               hipMemcpy(d_o, &zero, 8, hipMemcpyHostToDevice) != hipSuccess ||
               (life_version && hipMemcpy(d_l, life_version + i, 2, hipMemcpyHostToDevice) != hipSuccess)) {
      e = AMBRYCRC_EHIP;
    } else {
      e = ambrycrc_transform_messages_dev(d_buf, n, d_o, 1, life_version ? d_l : nullptr, header_version, d_out, cap,
                                          d_oo, d_ol, d_s, d_w, ambrycrc_transform_workspace_bytes(1), nullptr);
      if (!e && (hipMemcpy(&st, d_s, 4, hipMemcpyDeviceToHost) != hipSuccess ||
                 hipMemcpy(&len, d_ol, 8, hipMemcpyDeviceToHost) != hipSuccess))
        e = AMBRYCRC_EHIP;
      if (!e && st == 0) {
        h.resize(len);
        if (len && hipMemcpy(h.data(), d_out, len, hipMemcpyDeviceToHost) != hipSuccess) e = AMBRYCRC_EHIP;
      }
    }
    for (void* p : {(void*)d_buf, (void*)d_out, (void*)d_o, (void*)d_oo, (void*)d_ol, (void*)d_s, (void*)d_l, d_w})
      if (p) (void)hipFree(p);
    if (!e) place(i, st, st == 0 ? len : 0, h.data(), nullptr);
    return e;
  };
  size_t i = 0;
  int k = 0;
  while (i < m && !rc) {
    if (ext[i] > kSlabBytes) {
      for (int d = 0; d < kSlabs && !rc; ++d) rc = drain((k + d) % kSlabs);  // keep the output in order
      if (!rc) rc = oversize(i);
      ++i;
      continue;
    }
    const int w = k % kSlabs;
    rc = drain(w);
    if (rc) break;
    HostSlab& s = c->slab[w];
    MsgSlab& ms = c->msg_slab[w];
    XformSlab& x = c->xform_slab[w];
    Run& r = inflight[w];
    r.i0 = i;
    uint64_t lo = std::min(msg_off[i], region_len), hi = lo + ext[i];
    size_t n = 0;
    // A run ends where its span would pass a slab, or where the summed extents of its messages
    // (each output at most its extent + the growth bound) would pass the slab's output buffer:
    // messages that share bytes (duplicate offsets) never meet a cap one call over the whole region
    // would not have.
    uint64_t outs = 0;
    while (i + n < m && n < kSlabMsgs && ext[i + n] <= kSlabBytes) {
      const uint64_t o = std::min(msg_off[i + n], region_len), e = o + ext[i + n];
      const uint64_t nlo = std::min(lo, o), nhi = std::max(hi, e);
      const uint64_t nouts = outs + ext[i + n] + AMBRYCRC_TRANSFORM_GROWTH_MAX;
      if (nhi - nlo > kSlabBytes || (n && nouts > kXformOutBytes)) break;
      lo = nlo;
      hi = nhi;
      outs = nouts;
      ++n;
    }
    const uint64_t span = hi - lo;
    for (size_t q = 0; q < n; ++q) {
      ms.h_off[q] = msg_off[i + q] > region_len ? span + 1 : msg_off[i + q] - lo;
      if (life_version) x.h_life[q] = life_version[i + q];
    }
    if (span) {
      if (pinned) {
        if (hipMemcpyAsync(s.d_data, region + lo, span, hipMemcpyHostToDevice, s.stream) != hipSuccess) rc = AMBRYCRC_EHIP;
      } else {
        jobs.clear();
        jobs.push_back({s.h_data, region + lo, span});
        parallel_copy(jobs, span);  // overlaps the DMA and kernels of the slabs already issued
        if (hipMemcpyAsync(s.d_data, s.h_data, span, hipMemcpyHostToDevice, s.stream) != hipSuccess) rc = AMBRYCRC_EHIP;
      }
    }
    const uint64_t cap = std::min<uint64_t>(kXformOutBytes, std::max(outs, ambrycrc_transform_out_bound(span, n)));
    if (!rc && (hipMemcpyAsync(ms.d_off, ms.h_off, n * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream) != hipSuccess ||
                (life_version &&
                 hipMemcpyAsync(x.d_life, x.h_life, n * sizeof(int16_t), hipMemcpyHostToDevice, s.stream) != hipSuccess)))
      rc = AMBRYCRC_EHIP;
    if (!rc)
      rc = ambrycrc_transform_messages_dev(s.d_data, span, ms.d_off, n, life_version ? x.d_life : nullptr, header_version,
                                           x.d_out, cap, x.d_ooff, x.d_olen, ms.d_status, x.d_ws,
                                           ambrycrc_transform_workspace_bytes(kSlabMsgs), s.stream);
    if (!rc && (hipMemcpyAsync(ms.h_status, ms.d_status, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream) !=
                    hipSuccess ||
                hipMemcpyAsync(x.h_olen, x.d_olen, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
                hipMemcpyAsync(x.h_out, x.d_out, cap, hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
                hipEventRecord(s.done, s.stream) != hipSuccess))
      rc = AMBRYCRC_EHIP;
    if (rc) break;
    r.n = n;
    i += n;
    ++k;
  }
  int rc2 = AMBRYCRC_OK;
  for (int d = 0; d < kSlabs; ++d) {  // oldest first: the output is packed in message order
    const int rr = drain((k + d) % kSlabs);
    if (!rc2) rc2 = rr;
  }
  (void)hipSetDevice(prev);
  return rc ? rc : rc2;
}

// ---- host-resident dispatch: the CPU leg or the GPU leg per call
namespace {
double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
// The context of a host call (device < 0: none, the CPU leg) and its status.
int host_ctx(int device, DevCtx** c) {
  *c = device >= 0 ? ctx_for(device) : nullptr;
  return device >= 0 && !*c ? AMBRYCRC_ENOINIT : AMBRYCRC_OK;
}
}  // namespace

int ambrycrc_batch_host(const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in, uint32_t* out, size_t n,
                        int device, int pinned) {
  if (n == 0) return AMBRYCRC_OK;
  if (!ptrs || !lens || !out) return AMBRYCRC_EINVAL;
  DevCtx* c;
  if (const int rc = host_ctx(device, &c)) return rc;
  uint64_t bytes = 0;
  for (size_t i = 0; i < n; ++i) bytes += lens[i];
  const auto t0 = std::chrono::steady_clock::now();
  if (host_take_cpu(c, device, pinned, bytes)) {
    if (c) c->last_host_path.store(0);
    const int rc = ambrycrc_batch_cpu(ptrs, lens, crc_in, out, n, host_cpu_threads(c));
    if (rc == AMBRYCRC_OK && device >= 0) host_note_cpu(c, bytes, seconds_since(t0));
    return rc;
  }
  c->last_host_path.store(1);
  const int rc = batch_host_gpu(c, ptrs, lens, crc_in, out, n, device, pinned);
  if (rc == AMBRYCRC_OK && !pinned) host_note_gpu(c, bytes, seconds_since(t0));
  return rc;
}

int ambrycrc_verify_messages_host(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                                  uint32_t* status, uint64_t* msg_end, int device, int pinned) {
  if (m == 0) return AMBRYCRC_OK;
  if (!msg_off || !status || (!region && region_len)) return AMBRYCRC_EINVAL;
  DevCtx* c;
  if (const int rc = host_ctx(device, &c)) return rc;
  const bool cpu = host_take_cpu_msg(c, device, pinned, kMsgVerify, region_len);
  if (c) c->last_host_path.store(cpu ? 0 : 1);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = cpu ? verify_messages_cpu(region, region_len, msg_off, m, status, msg_end, host_cpu_threads(c))
                     : verify_messages_host_gpu(c, region, region_len, msg_off, m, status, msg_end, device, pinned);
  if (rc == AMBRYCRC_OK && !pinned && device >= 0) host_note_msg(c, kMsgVerify, cpu, region_len, seconds_since(t0));
  return rc;
}

int ambrycrc_transform_messages_host(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                                     const int16_t* life_version, int header_version, uint8_t* out, uint64_t out_cap,
                                     uint64_t* out_off, uint64_t* out_len, uint32_t* status, int device, int pinned) {
  if (m == 0) return AMBRYCRC_OK;
  if (!msg_off || !out_len || !status || (!region && region_len) || (!out && out_cap) || header_version < 1 ||
      header_version > 3)
    return AMBRYCRC_EINVAL;
  DevCtx* c;
  if (const int rc = host_ctx(device, &c)) return rc;
  const bool cpu = host_take_cpu_msg(c, device, pinned, kMsgTransform, region_len);
  if (c) c->last_host_path.store(cpu ? 0 : 1);
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = cpu ? transform_messages_cpu(region, region_len, msg_off, m, life_version, header_version, out, out_cap,
                                              out_off, out_len, status, host_cpu_threads(c))
                     : transform_messages_host_gpu(c, region, region_len, msg_off, m, life_version, header_version, out,
                                                   out_cap, out_off, out_len, status, device, pinned);
  if (rc == AMBRYCRC_OK && !pinned && device >= 0) host_note_msg(c, kMsgTransform, cpu, region_len, seconds_since(t0));
  return rc;
}

int ambrycrc_set_host_policy(int device, int policy) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (policy < 0 || policy > 2) return AMBRYCRC_EINVAL;
  return c->host_policy.exchange(policy);
}

int ambrycrc_host_rates(int device, double* cpu_gibps, double* gpu_gibps, int* cpu_threads) {
  DevCtx* c = device < 0 ? nullptr : ctx_for(device);
  if (!c && device >= 0) return AMBRYCRC_ENOINIT;
  const double cpu = host_batch_cpu_gibps(c), gpu = c ? c->gpu_host_gibps.load() : 0.0;
  if (cpu_gibps) *cpu_gibps = cpu;
  if (gpu_gibps) *gpu_gibps = gpu;
  if (cpu_threads) *cpu_threads = host_cpu_threads(c);
  return cpu > gpu ? 0 : 1;  // auto's leg for pageable bytes, whatever the policy
}

int ambrycrc_set_host_cpu_threads(int device, int threads) {
  if (threads < 0 || threads > 256) return AMBRYCRC_EINVAL;
  if (device < 0) return g_cpu_threads.exchange(threads);
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  const int prev = c->cpu_threads.exchange(threads);
  if (prev != threads)  // the message legs' measured rates were at the old budget (the batch's are kept per budget)
    for (auto& r : c->msg_cpu_gibps) r.store(-1.0);
  return prev;
}

int ambrycrc_host_calibrate(int device, double* cpu_gibps) {
  DevCtx* c = device < 0 ? nullptr : ctx_for(device);
  if (!c && device >= 0) return AMBRYCRC_ENOINIT;
  const double r = host_cpu_gibps(host_cpu_threads(c));
  if (cpu_gibps) *cpu_gibps = r;
  return AMBRYCRC_OK;
}

int ambrycrc_host_msg_rates(int device, int op, double* cpu_gibps, double* gpu_gibps) {
  DevCtx* c = ctx_for(device);
  if (!c) return AMBRYCRC_ENOINIT;
  if (op != kMsgVerify && op != kMsgTransform) return AMBRYCRC_EINVAL;
  const double cpu = host_msg_cpu_gibps(c, op), gpu = c->msg_gpu_gibps[op].load();
  if (cpu_gibps) *cpu_gibps = cpu;
  if (gpu_gibps) *gpu_gibps = gpu;
  return cpu > gpu ? 0 : 1;
}

int ambrycrc_last_host_path(int device) {
  DevCtx* c = ctx_for(device);
  return c ? c->last_host_path.load() : AMBRYCRC_ENOINIT;
}

size_t ambrycrc_trailed_workspace_bytes(size_t n) {
  const size_t own = (n * (sizeof(uint64_t) + 2 * sizeof(uint32_t) + 1) + 255) & ~size_t(255);
  return own + ws_need(n);
}

int ambrycrc_verify_trailed_dev(const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len,
                                uint8_t* d_mismatch, uint32_t* d_mismatch_count, size_t n, void* d_ws,
                                size_t ws_bytes, hipStream_t stream) {
  if (n == 0) return AMBRYCRC_OK;
  if (!d_base || !d_off || !d_len || n >= (1ull << 31)) return AMBRYCRC_EINVAL;
  DevCtx* c = ctx_current();
  if (!c) return AMBRYCRC_ENOINIT;
  WsLease lease;
  int rc = lease.acquire(c, stream, &d_ws, ws_bytes, ambrycrc_trailed_workspace_bytes(n));
  if (rc) return rc;
  uint8_t* w = static_cast<uint8_t*>(d_ws);
  TrailerArgs a;
  a.base = d_base;
  a.off = d_off;
  a.len = d_len;
  a.n = n;
  a.job_len = reinterpret_cast<uint64_t*>(w);
  a.expected = reinterpret_cast<uint32_t*>(a.job_len + n);
  uint32_t* crc = a.expected + n;
  a.crc = crc;
  a.force = reinterpret_cast<uint8_t*>(crc + n);
  a.mismatch = d_mismatch;
  a.count = d_mismatch_count;
  const bool inline_exp = variant_groups(c->variant);
  a.inline_max = inline_exp ? batch_small_max(c, n) : 0;
  void* batch_ws = w + ((n * (sizeof(uint64_t) + 2 * sizeof(uint32_t) + 1) + 255) & ~size_t(255));
  if (launch_trailer_parse(a, stream) != hipSuccess) return AMBRYCRC_EHIP;
  rc = enqueue_batch(c, d_base, d_off, a.job_len, nullptr, crc, n, batch_ws, stream,
                         a.inline_max ? a.expected : nullptr);
  if (rc) return rc;
  return hip_err(launch_trailer_verify(a, stream));
}

int ambrycrc_verify_trailed_host(const void* const* ptrs, const uint64_t* lens, uint8_t* mismatch, size_t n,
                                 int device, int pinned) {
  if (n == 0) return AMBRYCRC_OK;
  if (!ptrs || !lens || !mismatch) return AMBRYCRC_EINVAL;
  std::vector<uint64_t> body(n);
  for (size_t i = 0; i < n; ++i) body[i] = lens[i] >= 8 ? lens[i] - 8 : 0;
  std::vector<uint32_t> crc(n);
  const int rc = ambrycrc_batch_host(ptrs, body.data(), nullptr, crc.data(), n, device, pinned);
  if (rc) return rc;
  for (size_t i = 0; i < n; ++i)
    mismatch[i] = lens[i] < 8 || rd_be64(static_cast<const uint8_t*>(ptrs[i]) + body[i]) != (uint64_t)crc[i];
  return AMBRYCRC_OK;
}

size_t ambrycrc_chain_messages_host(const uint8_t* region, uint64_t region_len, uint64_t start, uint64_t* offs,
                                    size_t max) {
  if (!region || !offs) return 0;
  auto be16 = [](const uint8_t* p) { return (uint32_t)((p[0] << 8) | p[1]); };
  auto be32 = [](const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  };
  auto be64 = [&](const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); };
  size_t cnt = 0;
  uint64_t off = start;
  while (cnt < max && off < region_len && region_len - off >= 2) {
    const uint8_t* p = region + off;
    const int v = (int16_t)be16(p);
    const uint32_t h = v == 1 ? 34u : v == 2 ? 38u : v == 3 ? 40u : 0u;
    if (h == 0 || region_len - off < h) break;
    if ((uint64_t)ambrycrc_update(0, p, h - 8) != be64(p + h - 8)) break;
    int64_t total;
    int32_t rel[5];
    if (v == 1) {
      total = (int64_t)be64(p + 2);
      rel[0] = -1;
      for (int k = 0; k < 4; ++k) rel[k + 1] = (int32_t)be32(p + 10 + 4 * k);
    } else if (v == 2) {
      total = (int64_t)be64(p + 2);
      for (int k = 0; k < 5; ++k) rel[k] = (int32_t)be32(p + 10 + 4 * k);
    } else {
      total = (int64_t)be64(p + 4);
      for (int k = 0; k < 5; ++k) rel[k] = (int32_t)be32(p + 12 + 4 * k);
    }
    int64_t first = -1;
    for (int k = 0; k < 5; ++k)
      if (rel[k] != -1) {
        first = rel[k];
        break;
      }
    if (total <= 0 || first < (int64_t)h || (uint64_t)total > region_len - off ||
        (uint64_t)first > region_len - off - (uint64_t)total)
      break;
    offs[cnt++] = off;
    off += (uint64_t)first + (uint64_t)total;
  }
  return cnt;
}

long ambrycrc_debug_table_image(uint32_t* out, size_t max_words) {
  std::vector<uint32_t> img = build_table_image();
  if (!out || max_words < img.size()) return AMBRYCRC_EINVAL;
  memcpy(out, img.data(), img.size() * 4);
  return (long)(img.size() * 4);
}

}  // extern "C"
