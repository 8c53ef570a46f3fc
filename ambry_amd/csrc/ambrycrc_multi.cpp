// ambrycrc_multi.cpp -- the multi-GPU batch path of libambrycrc: per-device CRC
// of a byte-balanced shard, then an RCCL all-gather of the 4-byte CRCs over xGMI so every device
// holds the whole batch's results. Two forms behind the C ABI:
//   ambrycrc_batch_dev_multi   one process driving several GPUs (a JVM storage node scanning
//                              many partitions: ReplicaThread.java:1810-1815, BlobStoreRecovery.java:43-110)
//   ambrycrc_batch_dev_gather  one process per GPU; the communicator is built from a unique id
//                              the caller distributes (ncclCommInitRank)
// RCCL (librccl.so.1, /opt/rocm/lib) is loaded on first use with dlopen and called through its
// own handle, so the library loads, and every single-GPU entry works, on hosts without it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/ambrycrc.h"

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      return fn != nullptr;
    };
    x.ok = sym(x.get_unique_id, "ncclGetUniqueId") && sym(x.comm_init_rank, "ncclCommInitRank") &&
           sym(x.comm_init_all, "ncclCommInitAll") && sym(x.comm_destroy, "ncclCommDestroy") &&
           sym(x.all_gather, "ncclAllGather") && sym(x.group_start, "ncclGroupStart") &&
           sym(x.group_end, "ncclGroupEnd");
    return x;
  }();
  return r;
}

// Per-rank segment of the gather buffer: a multiple of 64 CRCs (256 B), so RCCL moves aligned
// blocks; a batch whose shards all have exactly that many chunks is gathered in place in the
// caller's d_gathered, any other goes through a padded scratch buffer and is compacted after.
// The arithmetic is ambrycrc_gather_layout's; the compaction copies are gather_copies' (the host
// executor ambrycrc_gather_compact_host runs the same list, so the CPU multi-rank tests drive it).
constexpr uint64_t kSegAlign = 64;

struct GatherLayout {
  uint64_t width = 0;  // CRCs per rank segment
  bool in_place = false;
  std::vector<uint64_t> start;  // [nranks + 1]: shard r's CRCs end at d_gathered[start[r] .. start[r+1])
};

GatherLayout gather_layout(const uint64_t* counts, int nranks) {
  GatherLayout g;
  uint64_t w = 0;
  for (int r = 0; r < nranks; ++r) w = std::max(w, counts[r]);
  g.width = (w + kSegAlign - 1) / kSegAlign * kSegAlign;
  g.in_place = g.width > 0;
  g.start.assign(nranks + 1, 0);
  for (int r = 0; r < nranks; ++r) {
    g.start[r + 1] = g.start[r] + counts[r];
    g.in_place = g.in_place && counts[r] == g.width;
  }
  return g;
}

// The padded layout's compaction: fn(dst word, src word, words) for each non-empty shard.
template <class Fn>
int gather_copies(const GatherLayout& g, const uint64_t* counts, int nranks, Fn fn) {
  for (int r = 0; r < nranks; ++r)
    if (counts[r]) {
      const int rc = fn(g.start[r], (uint64_t)r * g.width, counts[r]);
      if (rc) return rc;
    }
  return AMBRYCRC_OK;
}

// Padded gather buffers, one per (local device, stream): a batch on another stream never shares
// one with a batch still queued (its kernels, all-gather and compaction run in stream order).
// `done` is recorded after the compaction; a buffer is reused for another stream, or regrown,
// only after it has fired. At most kScratchPerDevice streams keep one (least recent evicted).
struct DevScratch {
  hipStream_t stream = nullptr;
  uint32_t* ptr = nullptr;
  size_t words = 0;
  hipEvent_t done = nullptr;
  uint64_t last_use = 0;
};
constexpr size_t kScratchPerDevice = 8;

}  // namespace

struct ambrycrc_comm {
  std::vector<ncclComm_t> comms;  // one per device driven by this process
  std::vector<int> devices;
  int nranks = 0;
  int rank = 0;  // rank of comms[0] (0 for ambrycrc_comm_init_all)
  std::vector<std::vector<DevScratch>> scratch;  // per local device
  uint64_t uses = 0;
  std::mutex mu;  // one batch enqueues at a time (RCCL group semantics, scratch bookkeeping)
};

namespace {

// The padded buffer of local device i for `stream` (current device: that device). *entry is where
// the caller records the buffer's `done` event after its last use.
int scratch_for(ambrycrc_comm* c, size_t i, hipStream_t stream, size_t words, uint32_t** out, DevScratch** entry) {
  std::vector<DevScratch>& list = c->scratch[i];
  DevScratch* s = nullptr;
  for (DevScratch& x : list)
    if (x.ptr && x.stream == stream) s = &x;
  if (!s && list.size() < kScratchPerDevice) {
    list.emplace_back();
    s = &list.back();
  }
  if (!s) {  // evict the least recently used stream's buffer
    s = &list[0];
    for (DevScratch& x : list)
      if (x.last_use < s->last_use) s = &x;
  }
  if (s->stream != stream || s->words < words) {
    if (s->done && hipEventSynchronize(s->done) != hipSuccess) return AMBRYCRC_EHIP;  // its last gather
    s->stream = stream;
  }
  if (s->words < words) {
    if (s->ptr) (void)hipFree(s->ptr);
    s->ptr = nullptr;
    s->words = 0;
    if (hipMalloc(reinterpret_cast<void**>(&s->ptr), words * sizeof(uint32_t)) != hipSuccess) return AMBRYCRC_ENOMEM;
    s->words = words;
  }
  if (!s->done && hipEventCreateWithFlags(&s->done, hipEventDisableTiming) != hipSuccess) return AMBRYCRC_EHIP;
  s->last_use = ++c->uses;
  *out = s->ptr;
  *entry = s;
  return AMBRYCRC_OK;
}

void free_scratch(std::vector<DevScratch>& list) {
  for (DevScratch& x : list) {
    if (x.ptr) (void)hipFree(x.ptr);
    if (x.done) (void)hipEventDestroy(x.done);
  }
  list.clear();
}

// Enqueues shard i's CRCs into its segment, for every local shard, then one grouped all-gather,
// then (padded layout) the compaction copies. Caller holds c->mu; device restored by the caller.
int enqueue_gather(ambrycrc_comm* c, const ambrycrc_shard* shards, const uint64_t* counts) {
  const int nranks = c->nranks;
  const GatherLayout g = gather_layout(counts, nranks);
  const uint64_t width = g.width;
  if (width == 0) return AMBRYCRC_OK;
  const bool in_place = g.in_place;
  const size_t local = c->comms.size();
  std::vector<uint32_t*> recv(local, nullptr);
  std::vector<DevScratch*> entry(local, nullptr);
  for (size_t i = 0; i < local; ++i) {
    const ambrycrc_shard& s = shards[i];
    const int rank = c->rank + (int)i;
    if (hipSetDevice(s.device) != hipSuccess) return AMBRYCRC_EHIP;
    if (in_place) {
      recv[i] = s.d_gathered;
    } else {
      const int rc = scratch_for(c, i, s.stream, (size_t)width * nranks, &recv[i], &entry[i]);
      if (rc) return rc;
    }
    const int rc = ambrycrc_batch_dev(s.d_base, s.d_off, s.d_len, s.d_crc_in, recv[i] + (size_t)rank * width, s.n,
                                      nullptr, 0, s.stream);
    if (rc) return rc;
  }
  const Rccl& R = rccl();
  if (R.group_start() != ncclSuccess) return AMBRYCRC_ECOMM;
  int rc = AMBRYCRC_OK;
  for (size_t i = 0; i < local && !rc; ++i) {
    uint32_t* seg = recv[i] + (size_t)(c->rank + (int)i) * width;
    if (R.all_gather(seg, recv[i], width, ncclUint32, c->comms[i], shards[i].stream) != ncclSuccess) rc = AMBRYCRC_ECOMM;
  }
  if (R.group_end() != ncclSuccess && !rc) rc = AMBRYCRC_ECOMM;
  if (rc || in_place) return rc;
  for (size_t i = 0; i < local; ++i) {
    if (hipSetDevice(shards[i].device) != hipSuccess) return AMBRYCRC_EHIP;
    const hipStream_t st = shards[i].stream;
    rc = gather_copies(g, counts, nranks, [&](uint64_t dst, uint64_t src, uint64_t words) {
      return hipMemcpyAsync(shards[i].d_gathered + dst, recv[i] + src, words * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                            st) == hipSuccess
                 ? AMBRYCRC_OK
                 : AMBRYCRC_EHIP;
    });
    if (rc) return rc;
    if (hipEventRecord(entry[i]->done, st) != hipSuccess) return AMBRYCRC_EHIP;
  }
  return AMBRYCRC_OK;
}

bool shard_ok(const ambrycrc_shard& s) {
  if (!s.d_gathered) return false;
  return s.n == 0 || (s.d_base && s.d_off && s.d_len);
}

}  // namespace

extern "C" {

int ambrycrc_gather_layout(const uint64_t* counts, int nranks, uint64_t* width, int* in_place, uint64_t* starts) {
  if (nranks <= 0 || !counts) return AMBRYCRC_EINVAL;
  const GatherLayout g = gather_layout(counts, nranks);
  if (width) *width = g.width;
  if (in_place) *in_place = g.in_place ? 1 : 0;
  if (starts) memcpy(starts, g.start.data(), sizeof(uint64_t) * (nranks + 1));
  return AMBRYCRC_OK;
}

int ambrycrc_gather_compact_host(const uint32_t* padded, const uint64_t* counts, int nranks, uint32_t* out) {
  if (nranks <= 0 || !counts || !out || !padded) return AMBRYCRC_EINVAL;
  const GatherLayout g = gather_layout(counts, nranks);
  if (g.in_place) {  // the gather buffer is the result
    if (out != padded) memmove(out, padded, sizeof(uint32_t) * g.start[nranks]);
    return AMBRYCRC_OK;
  }
  return gather_copies(g, counts, nranks, [&](uint64_t dst, uint64_t src, uint64_t words) {
    memmove(out + dst, padded + src, words * sizeof(uint32_t));
    return AMBRYCRC_OK;
  });
}

int ambrycrc_shard_by_bytes(const uint64_t* lens, size_t n, int nshards, size_t* cuts) {
  if (nshards <= 0 || !cuts || (n && !lens)) return AMBRYCRC_EINVAL;
  unsigned __int128 total = 0;
  for (size_t i = 0; i < n; ++i) total += lens[i];
  cuts[0] = 0;
  for (int g = 1; g <= nshards; ++g) cuts[g] = n;
  if (total == 0) {  // all empty: split by count
    for (int g = 1; g < nshards; ++g) cuts[g] = (size_t)((unsigned __int128)n * g / nshards);
    return AMBRYCRC_OK;
  }
  // shard g = the chunks whose start byte s satisfies g/nshards <= s/total < (g+1)/nshards
  unsigned __int128 prefix = 0;
  int g = 1;
  for (size_t i = 0; i < n && g < nshards; ++i) {
    while (g < nshards && prefix * (unsigned)nshards >= total * (unsigned)g) cuts[g++] = i;
    prefix += lens[i];
  }
  return AMBRYCRC_OK;
}

int ambrycrc_unique_id(uint8_t* id) {
  if (!id) return AMBRYCRC_EINVAL;
  const Rccl& R = rccl();
  if (!R.ok) return AMBRYCRC_ECOMM;
  ncclUniqueId u;
  if (R.get_unique_id(&u) != ncclSuccess) return AMBRYCRC_ECOMM;
  memcpy(id, u.internal, AMBRYCRC_UNIQUE_ID_BYTES);
  return AMBRYCRC_OK;
}

int ambrycrc_comm_init_all(const int* devices, int ndev, ambrycrc_comm** out) {
  if (!out || ndev <= 0 || ndev > 64) return AMBRYCRC_EINVAL;
  *out = nullptr;
  const Rccl& R = rccl();
  if (!R.ok) return AMBRYCRC_ECOMM;
  auto* c = new ambrycrc_comm();
  c->devices.resize(ndev);
  for (int i = 0; i < ndev; ++i) c->devices[i] = devices ? devices[i] : i;
  int prev = 0;
  (void)hipGetDevice(&prev);
  c->comms.resize(ndev);
  const ncclResult_t r = R.comm_init_all(c->comms.data(), ndev, c->devices.data());
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) {
    delete c;
    return AMBRYCRC_ECOMM;
  }
  c->nranks = ndev;
  c->rank = 0;
  c->scratch.resize(ndev);
  *out = c;
  return AMBRYCRC_OK;
}

int ambrycrc_comm_init_rank(const uint8_t* id, int nranks, int rank, int device, ambrycrc_comm** out) {
  if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks || device < 0) return AMBRYCRC_EINVAL;
  *out = nullptr;
  const Rccl& R = rccl();
  if (!R.ok) return AMBRYCRC_ECOMM;
  ncclUniqueId u;
  memcpy(u.internal, id, AMBRYCRC_UNIQUE_ID_BYTES);
  int prev = 0;
  (void)hipGetDevice(&prev);
  if (hipSetDevice(device) != hipSuccess) return AMBRYCRC_EHIP;
  auto* c = new ambrycrc_comm();
  c->comms.resize(1);
  const ncclResult_t r = R.comm_init_rank(&c->comms[0], nranks, u, rank);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) {
    delete c;
    return AMBRYCRC_ECOMM;
  }
  c->devices = {device};
  c->nranks = nranks;
  c->rank = rank;
  c->scratch.resize(1);
  *out = c;
  return AMBRYCRC_OK;
}

int ambrycrc_comm_destroy(ambrycrc_comm* c) {
  if (!c) return AMBRYCRC_OK;
  int prev = 0;
  (void)hipGetDevice(&prev);
  const Rccl& R = rccl();
  int rc = AMBRYCRC_OK;
  for (size_t i = 0; i < c->comms.size(); ++i) {
    (void)hipSetDevice(c->devices[i]);
    (void)hipDeviceSynchronize();
    free_scratch(c->scratch[i]);
    if (c->comms[i] && R.comm_destroy(c->comms[i]) != ncclSuccess) rc = AMBRYCRC_ECOMM;
  }
  (void)hipSetDevice(prev);
  delete c;
  return rc;
}

int ambrycrc_comm_size(const ambrycrc_comm* c) { return c ? c->nranks : AMBRYCRC_EINVAL; }

int ambrycrc_batch_dev_multi(ambrycrc_comm* c, const ambrycrc_shard* shards, int nshards) {
  if (!c || !shards || nshards != (int)c->comms.size() || c->rank != 0 || c->nranks != nshards) return AMBRYCRC_EINVAL;
  std::vector<uint64_t> counts(nshards);
  for (int i = 0; i < nshards; ++i) {
    if (!shard_ok(shards[i]) || shards[i].device != c->devices[i] || shards[i].n >= (1ull << 31)) return AMBRYCRC_EINVAL;
    counts[i] = shards[i].n;
  }
  std::lock_guard<std::mutex> g(c->mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  const int rc = enqueue_gather(c, shards, counts.data());
  (void)hipSetDevice(prev);
  return rc;
}

int ambrycrc_batch_dev_gather(ambrycrc_comm* c, const ambrycrc_shard* mine, const uint64_t* counts) {
  if (!c || !mine || !counts || c->comms.size() != 1) return AMBRYCRC_EINVAL;
  if (!shard_ok(*mine) || mine->device != c->devices[0] || counts[c->rank] != mine->n) return AMBRYCRC_EINVAL;
  for (int r = 0; r < c->nranks; ++r)
    if (counts[r] >= (1ull << 31)) return AMBRYCRC_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  int prev = 0;
  (void)hipGetDevice(&prev);
  const int rc = enqueue_gather(c, mine, counts);
  (void)hipSetDevice(prev);
  return rc;
}

}  // extern "C"
