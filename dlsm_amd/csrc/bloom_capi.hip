// dlsm_amd/csrc/bloom_capi.hip -- the C ABI (include/dlsm_bloom.h): contexts,
// device workspace, job set-up, and the host-buffer (staged) call variants.
// Kernels live in bloom_kernels.hip.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <unordered_map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/dlsm_bloom.h"
#include "bloom_internal.h"

using namespace dlsm;

namespace {

int from_hip(hipError_t e) {
  if (e == hipSuccess) return DLSM_OK;
  if (e == hipErrorOutOfMemory) return DLSM_E_NOMEM;
  return DLSM_E_DEVICE;
}

#define DLSM_TRY(expr)                       \
  do {                                       \
    hipError_t _e = (expr);                  \
    if (_e != hipSuccess) return from_hip(_e); \
  } while (0)

#define DLSM_CHECK(expr)         \
  do {                           \
    int _s = (expr);             \
    if (_s != DLSM_OK) return _s; \
  } while (0)

// Growable device buffer (never shrinks; freed with the context).
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;     // elements
  uint64_t gen = 0;   // bumped by every (re)allocation: contents are gone
  int ensure(size_t n) {
    if (n <= cap && p) return DLSM_OK;
    gen++;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
    size_t want = std::max<size_t>(n, 1);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want * sizeof(T));
    if (e != hipSuccess) {
      p = nullptr;
      return from_hip(e);
    }
    cap = want;
    return DLSM_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

uint32_t ceil_div_u32(uint64_t a, uint64_t b) { return static_cast<uint32_t>((a + b - 1) / b); }

}  // namespace

// Pipelined passes (opt-in knobs).  Probe: round r+1's partition runs on a
// helper stream while the context stream runs round r's slice + unpermute,
// over kProbeBufs rotating intermediate buffers.  Build: job group g+1's
// partition overlaps group g's slices the same way.  The context stream's last
// command depends on every helper command, so a call needs no separate join.
// Off by default: measured on MI355X (profiles/r01_v12_*), the overlapped
// kernels each ran ~2x slower (the slice passes fill every wave slot of a CU)
// and every round added ~10 us of launch gaps, a net loss.
constexpr int kProbeBufs = 3;
constexpr int kStageEvents = 4;

// The scheduling options a pooled context starts with; a recycled context gets
// them back (a thread may have changed them, e.g. a builder's BUILD_EXACT).
// Kept inside the context itself: a detached thread that exits after main
// returns still recycles its context safely (no static map to outlive).
struct CtxOpts {
  int path, build_groups;
  uint64_t probe_round;
  int probe_lgc, probe_lgr, build_exact;
  bool probe_serial;
  int probe_multi;
};

struct dlsm_ctx {
  int device = 0;
  CtxOpts opts0{};          // creation options (pooled thread contexts)
  bool opts0_set = false;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;              // helper stream of the pipelined passes
  hipEvent_t ev_fork = nullptr;           // context stream -> helper
  hipEvent_t ev_part[kStageEvents] = {};  // partition of buffer / group b done (helper)
  hipEvent_t ev_free[kStageEvents] = {};  // buffer b consumed (context stream)
  // dlsm_ctx_set_partition_stream: the partition passes run on pstream
  // (typically restricted to a CU subset), the rest on the context stream
  hipStream_t pstream = nullptr;
  uint32_t pcus = 0;                      // CUs the persistent partition grid is sized for (0: all)
  hipEvent_t ev_pfork = nullptr;          // context stream -> pstream
  hipEvent_t ev_pdone = nullptr;          // partition done (pstream -> context stream)
  int path = 0;
  int build_groups = 1;     // job groups of a build (1 = one partition + one slice launch)
  uint64_t probe_round = 0;  // keys per probe round (0 = whole batch)
  int probe_lgc = 13;        // log2 keys per probe partition chunk (12..14; 13 = two 4,096-key units, 512 threads)
  int probe_lgr = 8;         // log2 stacked lines per probe slice (7: 64 KiB, 8: 128 KiB of LDS)
  int build_exact = 0;       // DLSM_OPT_BUILD_EXACT: 0 auto, 1 always count first, 2 never
  bool probe_serial = false;  // DLSM_OPT_PROBE_ROUND_SERIAL: rounds one after another on one stream
  int fault = 0;              // DLSM_OPT_FAULT_INJECT: > 0 -> builds / probes return -fault
  int probe_multi = 1;        // DLSM_OPT_PROBE_MULTI: 1 one pass over a multi-group set, 0 a pass per group
  uint64_t vslice_bytes = 0;  // DLSM_OPT_VERSION_SLICE_BYTES (0: default)
  uint32_t vpass_slices = kVMaxSlices;  // DLSM_OPT_VERSION_PASS_SLICES
  std::atomic<uint64_t> fallbacks{0};  // dlsm_fallback_note: host re-runs of this context's failed calls
  // build workspace
  DevBuf<uint32_t> entries;
  DevBuf<uint16_t> tab;  // chunk-major bucket offsets
  DevBuf<FullJobDev> jobs;
  DevBuf<uint32_t> starts;  // chunk0s | slice0s
  DevBuf<uint32_t> dchunk;  // per-chunk consecutive-distinct counts
  DevBuf<uint32_t> jobL;    // per-job line count (direct path)
  // last uploaded job table (skip the H2D when a caller repeats a batch); the
  // device buffers' allocation generations are part of the key, so a buffer
  // that ensure() reallocated (reserve, a bigger batch) -- even at the same
  // address -- is never taken as filled
  std::vector<FullJobDev> last_jobs;
  std::vector<uint32_t> last_starts;
  uint64_t last_jobs_gen = 0, last_starts_gen = 0;
  DevBuf<LegacyJobDev> ljobs;
  DevBuf<uint64_t> lstarts;
  // LDS-tiled legacy build (util/bloom.cc format)
  DevBuf<LegacyTileJobDev> ltjobs;
  DevBuf<uint32_t> ltstarts;  // chunk0s | slice0s
  DevBuf<uint16_t> lentries;  // u16 bit positions per tile bucket
  DevBuf<uint16_t> ltab;      // chunk-major tile-bucket offsets
  // probe workspace
  DevBuf<uint32_t> hashes;  // grouped probe / sliced version probe: one BloomHash per lookup
  DevBuf<uint32_t> vgl;     // sliced version probe: per sliced level, each lookup's global line
  DevBuf<uint8_t> vabyte;   // sliced version probe: per lookup, the sliced levels' answer bits
  DevBuf<uint32_t> vplan;   // sliced version probe: per-slice unit counters | slice-pass plan
  uint64_t vplan_zeroed = 0;  // vplan's allocation generation whose counters were zeroed
  DevBuf<uint16_t> pos;
  DevBuf<uint8_t> smask;
  // host-API staging
  DevBuf<uint8_t> st_keys;
  DevBuf<uint64_t> st_offs;
  DevBuf<uint8_t> st_out;
  DevBuf<uint64_t> st_len;
  DevBuf<uint8_t> st_filter;
  // crc32c / block sealing
  DevBuf<uint8_t> crc_streams;
  DevBuf<uint32_t> crc_partial;
  DevBuf<uint32_t> crc_tabs;  // fused seal: full_block_crc_tables(crc_tabs_lgr)
  DevBuf<uint32_t> crc_cnt;   // fused seal: per-job slice counters (zero between calls)
  int crc_tabs_lgr = -1;
  uint64_t crc_tabs_gen = 0;
  DevBuf<uint8_t*> crc_outp;
  DevBuf<uint64_t> crc_cap;
  DevBuf<uint32_t> crc_val;
  // internal-key selection / gather: [blk_cnt | blk_bytes | tot(2) | first_bad]
  DevBuf<uint64_t> sel;
  // host-API results: page-locked, device-mapped, so the build kernels store
  // filters and lengths straight to host memory (one synchronisation, no D2H)
  uint8_t* h_out = nullptr;
  uint64_t h_out_cap = 0;
  uint64_t* h_len = nullptr;
  uint64_t h_len_cap = 0;
  // page-locked host staging lent to the context's (single) builder
  void* host_buf = nullptr;
  uint64_t host_cap = 0;
  std::atomic<const void*> host_owner{nullptr};
  // Page-locked sources of the small tables a call builds on the host and
  // uploads asynchronously (job tables, rebased offsets, lengths, crc stream
  // descriptors): a ring of slots, each reused only after the event recorded
  // behind its copy has completed -- a pageable (e.g. stack) source could be
  // gone before a queued copy reads it.
  // The slots are carved from one page-locked block allocated with the
  // context (hipHostMalloc takes a process-wide lock and milliseconds: lazily
  // allocated slots stalled concurrent builder threads' first calls by up to
  // 15 ms); a table larger than a slot gets a buffer of its own.
  static constexpr int kUpSlots = 16;
  static constexpr uint64_t kUpSlotBytes = 16384;
  uint8_t* up_block = nullptr;
  uint8_t* up_buf[kUpSlots] = {};
  uint64_t up_cap[kUpSlots] = {};
  bool up_own[kUpSlots] = {};  // up_buf[i] is a buffer of its own (not in up_block)
  hipEvent_t up_ev[kUpSlots] = {};
  bool up_live[kUpSlots] = {};
  int up_next = 0;
  // How a host-API call waits for its stream (ctx_sync): 0 hipStreamSynchronize,
  // 1 poll an event, yielding the core between polls, 2 a blocking-sync event
  // (DLSM_HOST_SYNC; default 1).  Many builder threads (dLSM runs 28) share
  // the host's cores with the HIP runtime's own threads: a waiter that spins
  // holds a core the other builders' AddKey hashing needs.
  int host_sync = 1;
  hipEvent_t ev_wait = nullptr;      // ctx_sync modes 1 and 2
};

// A stacked image of the filters of one mask byte that share a line count
// and probe count (at most 8): filter f answers in bit f % 8 of byte f / 8.
// A group of 1, 2 or 3-4 filters gets a packed image instead (W = 1, 2 or 4
// bits per bit position, 64 * W bytes per line: 8 / 4 / 2 times the lines per
// LDS slice), so a large single filter -- the biggest file of a level -- still
// fits the sliced path, and small groups walk fewer, longer bucket runs.
struct ProbeGroup {
  uint64_t* stacked = nullptr;  // L * 8 * 2^lgw u64 words
  uint32_t L = 0, magic = 0;
  int k = 0;
  int mask_byte = 0;
  bool first_of_byte = false;  // writes its mask byte; later groups of the byte OR into it
  int lgw = 3;                  // log2 bits per bit position of the image (3: stacked bytes)
  uint32_t slotmap = 0;         // packed images: member m answers in bit (slotmap >> 4m) & 7
};

// One image-width class of a one-pass multi-group probe: the global slices
// [s0, s0 + S) of the groups with image width lgw, walked by one slice launch
// of wgs workgroups (plan: S + 1 workgroup starts at d_mgplan + plan_off).
struct MGClass {
  int lgw = 0, K = 0;  // K: 6 when every group of the class has k = 6, else 0 (run time k)
  uint32_t s0 = 0, S = 0;
  uint32_t plan_off = 0, wgs = 0;
};

struct dlsm_filterset {
  int device = 0;
  int F = 0;
  uint8_t* blob = nullptr;
  uint64_t blob_bytes = 0;
  FilterDev* d_filters = nullptr;
  FilterDev* d_slots = nullptr;  // 8 stacking slots per group
  std::vector<FilterDev> h;
  // sliced probe: one group (<= 8 filters, one L and k: the bench's set) or
  // several (filters of different sizes, > 8 filters); empty = direct only
  // (a filter in the reference's log2_cache_line_size_ == 0 branch)
  std::vector<ProbeGroup> groups;
  uint64_t stacked_bytes = 0;
  // One-pass probe (2..kMGMaxGroups groups, every group sliceable at 128 KiB
  // slices): the groups in slice order (by image width), their slices
  // numbered globally, and one slice launch per width class.
  MGroupDev* d_mg = nullptr;
  uint32_t* d_mgplan = nullptr;
  int mg_n = 0;
  uint32_t mg_slices = 0;
  uint32_t mg_region = 0;  // entries per chunk region (every group's sub-region)
  uint32_t mg_abytes = 0;  // answer bytes per chunk
  uint32_t mg_stage_bytes = 0;  // the partition's largest staging area (LDS)
  std::vector<MGClass> mg_classes;
};

namespace {

// Wait until everything queued on s so far has completed (see host_sync).
hipError_t ctx_sync(dlsm_ctx* ctx, hipStream_t s) {
  if (ctx->host_sync == 0 || !ctx->ev_wait) return hipStreamSynchronize(s);
  hipError_t e = hipEventRecord(ctx->ev_wait, s);
  if (e != hipSuccess) return e;
  if (ctx->host_sync == 2) return hipEventSynchronize(ctx->ev_wait);
  while ((e = hipEventQuery(ctx->ev_wait)) == hipErrorNotReady) sched_yield();
  return e;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int validate_keyset(const dlsm_keyset& k) {
  if (k.n == 0) return DLSM_OK;
  if (!k.bytes) return DLSM_E_ARG;
  if (k.suffix_len > 255) return DLSM_E_ARG;
  // fixed keys must hold the stripped suffix; zero-length user keys are legal
  if (!k.offsets && k.key_len < k.suffix_len) return DLSM_E_ARG;
  return DLSM_OK;
}

KeyDesc to_desc(const dlsm_keyset& k) {
  KeyDesc d;
  d.bytes = k.bytes;
  d.offsets = k.offsets;
  d.n = k.n;
  d.key_len = k.key_len;
  d.suffix = k.suffix_len;
  return d;
}

// The K20 kernels stage keys through LDS with 16-byte loads.
bool is_k20(const dlsm_keyset& k) {
  return k.offsets == nullptr && k.key_len == 20 && k.suffix_len == 0 &&
         (k.n == 0 || aligned(k.bytes, 16));
}

// 28-byte internal keys (20-byte user key + 8-byte trailer) straight from the
// memtable / compaction iterators take the LDS-tiled K28 partition loaders.
bool is_k28(const dlsm_keyset& k) {
  return k.offsets == nullptr && k.key_len == 28 && k.suffix_len == 8 &&
         (k.n == 0 || aligned(k.bytes, 16));
}

// Slice width for the sliced build: the smallest 2^lgR (lgR in [9, 11]) that
// keeps every job at <= kMaxSlices slices, then narrower (down to 2^7 lines,
// 8 KiB) while the batch has fewer than two slice workgroups per CU -- a
// batch of dLSM-sized flush tables (153,846 keys, 3,005 lines) would
// otherwise leave most CUs idle.  Returns -1 if none fits.
#ifndef DLSM_BUILD_MIN_LGR
#define DLSM_BUILD_MIN_LGR 9  // widest-first search starts at 2^9 lines (32 KiB slices)
#endif
int choose_build_lgR(const std::vector<uint32_t>& Ls) {
  auto slices = [&](int lg, uint64_t* total) {
    bool ok = true;
    *total = 0;
    for (uint32_t L : Ls) {
      const uint64_t n = (static_cast<uint64_t>(L) + (1u << lg) - 1) >> lg;
      ok = ok && n <= kMaxSlices;
      *total += std::max<uint64_t>(n, 1);
    }
    return ok;
  };
  uint64_t total = 0, t2 = 0;
  // A/B knob: the slice-workgroup count below which the slices narrow
  // (default two per CU)
  static const uint64_t min_wgs = [] {
    const char* e = getenv("DLSM_BUILD_SLICE_MIN_WGS");
    return e ? strtoull(e, nullptr, 10) : 2ull * kBuildSliceCUs;
  }();
  for (int lg = DLSM_BUILD_MIN_LGR; lg <= 11; lg++) {
    if (!slices(lg, &total)) continue;
    while (lg > 7 && total < min_wgs && slices(lg - 1, &t2)) {
      lg--;
      total = t2;
    }
    return lg;
  }
  return -1;
}

// The helper stream starts behind everything already queued on the context
// stream (the call's inputs).
int fork_aux(dlsm_ctx* ctx) {
  DLSM_TRY(hipEventRecord(ctx->ev_fork, ctx->stream));
  DLSM_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
  return DLSM_OK;
}

// `to` waits for everything queued on `from` so far.
// dlsm_ctx_set_partition_stream: the partition stream starts behind
// everything queued on the context stream (the call's inputs, and the
// previous call's consumers of the workspace it overwrites) ...
int fork_part(dlsm_ctx* ctx) {
  DLSM_TRY(hipEventRecord(ctx->ev_pfork, ctx->stream));
  DLSM_TRY(hipStreamWaitEvent(ctx->pstream, ctx->ev_pfork, 0));
  return DLSM_OK;
}
// ... and the context stream's next pass starts behind the partition.
int join_part(dlsm_ctx* ctx) {
  DLSM_TRY(hipEventRecord(ctx->ev_pdone, ctx->pstream));
  DLSM_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_pdone, 0));
  return DLSM_OK;
}

int hand_over(hipStream_t from, hipStream_t to, hipEvent_t ev) {
  DLSM_TRY(hipEventRecord(ev, from));
  DLSM_TRY(hipStreamWaitEvent(to, ev, 0));
  return DLSM_OK;
}

// FullFilterBlockReader ctor checks (table/full_filter_block.cc:186-252) on the
// filter's 5-byte tail and total length.
int parse_tail(const uint8_t* tail, uint64_t len64, int* k_out, uint32_t* L_out, int* lg_out) {
  if (len64 < 5 || len64 > 0xffffffffull) return DLSM_E_CORRUPT;
  const int k = static_cast<int>(static_cast<int8_t>(tail[0]));
  if (k < 1) return DLSM_E_CORRUPT;  // the reference exit(1)s
  const uint32_t len = static_cast<uint32_t>(len64) - 5;
  const uint32_t L = uint32_t(tail[1]) | (uint32_t(tail[2]) << 8) | (uint32_t(tail[3]) << 16) |
                     (uint32_t(tail[4]) << 24);
  int lg;
  if (L * kCacheLineBytes == len) {
    // common case; L == 0 (empty filter) would make KeyMayMatch divide by 0,
    // and a wrapped product would index past the filter
    if (L == 0 || static_cast<uint64_t>(L) * kCacheLineBytes != len) return DLSM_E_CORRUPT;
    lg = 6;
  } else if (L == 0 || len % L != 0) {
    return DLSM_E_CORRUPT;  // the reference exit(1)s
  } else {
    lg = 0;  // log2_cache_line_size_ keeps its initialiser (full_filter_block.h:85)
  }
  *k_out = k;
  *L_out = L;
  *lg_out = lg;
  return DLSM_OK;
}

// Asynchronous H2D copy of n bytes of a host-built table (any memory, e.g.
// a std::vector about to go out of scope) on stream s: the bytes are copied
// into one of the context's page-locked upload slots first, so the caller's
// buffer may be released as soon as this returns.  A slot is reused only
// after the event behind its previous copy has completed.
int ctx_upload(dlsm_ctx* ctx, void* dst, const void* src, size_t n, hipStream_t s) {
  if (n == 0) return DLSM_OK;
  const int i = ctx->up_next;
  ctx->up_next = (i + 1) % dlsm_ctx::kUpSlots;
  if (ctx->up_live[i]) {
    DLSM_TRY(hipEventSynchronize(ctx->up_ev[i]));
    ctx->up_live[i] = false;
  }
  if (ctx->up_cap[i] < n) {
    if (ctx->up_own[i]) (void)hipHostFree(ctx->up_buf[i]);
    ctx->up_buf[i] = nullptr;
    ctx->up_cap[i] = 0;
    ctx->up_own[i] = false;
    uint64_t c = 2 * dlsm_ctx::kUpSlotBytes;
    while (c < n) c <<= 1;
    DLSM_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->up_buf[i]), c, hipHostMallocDefault));
    ctx->up_cap[i] = c;
    ctx->up_own[i] = true;
  }
  memcpy(ctx->up_buf[i], src, n);
  DLSM_TRY(hipMemcpyAsync(dst, ctx->up_buf[i], n, hipMemcpyHostToDevice, s));
  DLSM_TRY(hipEventRecord(ctx->up_ev[i], s));
  ctx->up_live[i] = true;
  return DLSM_OK;
}

}  // namespace

extern "C" {

const char* dlsm_strerror(int status) {
  switch (status) {
    case DLSM_OK: return "ok";
    case DLSM_E_ARG: return "invalid argument";
    case DLSM_E_CAPACITY: return "output slot too small";
    case DLSM_E_CORRUPT: return "corrupt bloom filter";
    case DLSM_E_DEVICE: return "HIP device error";
    case DLSM_E_NOMEM: return "device out of memory";
    case DLSM_E_BUSY: return "host staging buffer held by another user";
    default: return "unknown status";
  }
}

int dlsm_abi_version(void) { return DLSM_BLOOM_ABI_VERSION; }

uint32_t dlsm_bloom_hash(const void* key, size_t n) {
  return bloom_hash_host(static_cast<const uint8_t*>(key), n);
}

int dlsm_bloom_full_num_probes(int bits_per_key) { return full_num_probes(bits_per_key); }

int dlsm_bloom_full_size(uint64_t n_dedup, int bits_per_key, uint32_t* num_lines,
                         uint64_t* nbytes) {
  uint32_t tb;
  const uint32_t L = full_num_lines(n_dedup, bits_per_key, &tb);
  if (num_lines) *num_lines = L;
  if (nbytes) *nbytes = static_cast<uint64_t>(tb / 8u) + 5u;
  return DLSM_OK;
}

int dlsm_bloom_legacy_size(uint64_t n, int bits_per_key, uint64_t* nbytes) {
  if (nbytes) *nbytes = legacy_bits(n, bits_per_key) / 8 + 1;
  return DLSM_OK;
}

int dlsm_bloom_full_parse(const uint8_t* f, uint64_t len64, int* num_probes, uint32_t* num_lines,
                          int* log2_line) {
  if (!f || len64 < 5) return DLSM_E_CORRUPT;
  int k, lg;
  uint32_t L;
  DLSM_CHECK(parse_tail(f + len64 - 5, len64, &k, &L, &lg));
  if (num_probes) *num_probes = k;
  if (num_lines) *num_lines = L;
  if (log2_line) *log2_line = lg;
  return DLSM_OK;
}

int dlsm_device_count(int* n) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  if (n) *n = c;
  return e == hipSuccess ? DLSM_OK : from_hip(e);
}

}  // extern "C"
namespace {
// Per-thread contexts (dlsm_thread_ctx): owned = handed out here, returned to
// a per-device free list at the thread's exit; bound = the caller's
// (dlsm_thread_ctx_bind), never touched here.  dLSM starts a std::thread per
// subcompaction (db/db_impl.cc:3373-3386): with the free list a new thread
// takes a context a finished one left -- its stream, page-locked blocks,
// events and grown device workspaces -- instead of paying their creation
// (hipHostMalloc takes a process-wide lock) and teardown per compaction.
// The list is never freed: contexts outlive every thread, so a builder that
// outlives its thread still holds a live context, and nothing is destroyed
// during static destruction, after the HIP runtime may be gone.
struct CtxPool {
  std::mutex m;
  std::map<int, std::vector<dlsm_ctx*>> free;  // device -> idle contexts
  uint64_t created = 0, reused = 0;
};
CtxPool& ctx_pool() {
  static CtxPool* p = new CtxPool();  // intentionally leaked (see above)
  return *p;
}
void ctx_pool_put(dlsm_ctx* c);
struct ThreadCtx {
  dlsm_ctx* owned = nullptr;
  dlsm_ctx* bound = nullptr;
  ~ThreadCtx() {
    if (owned) ctx_pool_put(owned);
  }
};
ThreadCtx& thread_ctx_slot() {
  thread_local ThreadCtx t;
  return t;
}
std::atomic<unsigned> g_thread_ctx_next{0};
std::atomic<uint64_t> g_fallbacks{0};  // dlsm_fallback_note, process-wide
}  // namespace
extern "C" {

int dlsm_thread_ctx(dlsm_ctx** out) {
  if (!out) return DLSM_E_ARG;
  ThreadCtx& t = thread_ctx_slot();
  if (t.bound) {
    *out = t.bound;
    return DLSM_OK;
  }
  if (!t.owned) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) {
      *out = nullptr;
      return DLSM_E_DEVICE;
    }
    const int dev = static_cast<int>(g_thread_ctx_next.fetch_add(1) % static_cast<unsigned>(n));
    CtxPool& p = ctx_pool();
    {
      std::lock_guard<std::mutex> lk(p.m);
      auto& v = p.free[dev];
      if (!v.empty()) {
        t.owned = v.back();
        v.pop_back();
        p.reused++;
      }
    }
    if (!t.owned) {
      DLSM_CHECK(dlsm_ctx_create(dev, &t.owned));
      t.owned->opts0 = CtxOpts{t.owned->path,      t.owned->build_groups, t.owned->probe_round,
                               t.owned->probe_lgc, t.owned->probe_lgr,    t.owned->build_exact,
                               t.owned->probe_serial, t.owned->probe_multi};
      t.owned->opts0_set = true;
      std::lock_guard<std::mutex> lk(p.m);
      p.created++;
    }
  }
  *out = t.owned;
  return DLSM_OK;
}

int dlsm_thread_ctx_bind(dlsm_ctx* ctx) {
  thread_ctx_slot().bound = ctx;
  return DLSM_OK;
}

int dlsm_thread_ctx_stats(uint64_t* created, uint64_t* reused, uint64_t* idle) {
  CtxPool& p = ctx_pool();
  std::lock_guard<std::mutex> lk(p.m);
  uint64_t n = 0;
  for (auto& kv : p.free) n += kv.second.size();
  if (created) *created = p.created;
  if (reused) *reused = p.reused;
  if (idle) *idle = n;
  return DLSM_OK;
}

void dlsm_fallback_note(dlsm_ctx* ctx) {
  g_fallbacks.fetch_add(1, std::memory_order_relaxed);
  if (ctx) ctx->fallbacks.fetch_add(1, std::memory_order_relaxed);
}

int dlsm_fallback_stats(const dlsm_ctx* ctx, uint64_t* ctx_count, uint64_t* process_count) {
  if (ctx_count) *ctx_count = ctx ? ctx->fallbacks.load(std::memory_order_relaxed) : 0;
  if (process_count) *process_count = g_fallbacks.load(std::memory_order_relaxed);
  return DLSM_OK;
}

int dlsm_ctx_create(int device, dlsm_ctx** out) {
  if (!out) return DLSM_E_ARG;
  *out = nullptr;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || device < 0 || device >= c) return DLSM_E_DEVICE;
  DeviceGuard g(device);
  dlsm_ctx* ctx = new (std::nothrow) dlsm_ctx();
  if (!ctx) return DLSM_E_NOMEM;
  ctx->device = device;
  hipError_t e = hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_pfork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_pdone, hipEventDisableTiming);
  for (int b = 0; b < kStageEvents && e == hipSuccess; b++) {
    e = hipEventCreateWithFlags(&ctx->ev_part[b], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_free[b], hipEventDisableTiming);
  }
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&ctx->up_block), dlsm_ctx::kUpSlots * dlsm_ctx::kUpSlotBytes,
                      hipHostMallocDefault);
  for (int i = 0; i < dlsm_ctx::kUpSlots && e == hipSuccess; i++) {
    ctx->up_buf[i] = ctx->up_block + i * dlsm_ctx::kUpSlotBytes;
    ctx->up_cap[i] = dlsm_ctx::kUpSlotBytes;
    e = hipEventCreateWithFlags(&ctx->up_ev[i], hipEventDisableTiming);
  }
  if (const char* v = getenv("DLSM_HOST_SYNC")) ctx->host_sync = atoi(v);
  if (e == hipSuccess)
    e = hipEventCreateWithFlags(&ctx->ev_wait, hipEventDisableTiming |
                                                   (ctx->host_sync == 2 ? hipEventBlockingSync : 0u));
  ctx->stream = ctx->own;
  if (e != hipSuccess) {
    dlsm_ctx_destroy(ctx);
    return from_hip(e);
  }
  if (const char* v = getenv("DLSM_PROBE_ROUND_KEYS")) ctx->probe_round = strtoull(v, nullptr, 10);
  if (const char* v = getenv("DLSM_PROBE_CHUNK_LG")) dlsm_ctx_set_option(ctx, DLSM_OPT_PROBE_CHUNK_LG, strtoull(v, nullptr, 10));
  if (const char* v = getenv("DLSM_PROBE_SLICE_LG")) dlsm_ctx_set_option(ctx, DLSM_OPT_PROBE_SLICE_LG, strtoull(v, nullptr, 10));
  if (const char* v = getenv("DLSM_PROBE_SERIAL")) ctx->probe_serial = atoi(v) != 0;
  if (const char* v = getenv("DLSM_PROBE_MULTI")) ctx->probe_multi = atoi(v) != 0;
  *out = ctx;
  return DLSM_OK;
}

int dlsm_ctx_destroy(dlsm_ctx* ctx) {
  if (!ctx) return DLSM_OK;
  DeviceGuard g(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->aux) (void)hipStreamSynchronize(ctx->aux);
  if (ctx->pstream) (void)hipStreamSynchronize(ctx->pstream);
  ctx->entries.release();
  ctx->tab.release();
  ctx->jobs.release();
  ctx->starts.release();
  ctx->dchunk.release();
  ctx->jobL.release();
  ctx->ljobs.release();
  ctx->lstarts.release();
  ctx->ltjobs.release();
  ctx->ltstarts.release();
  ctx->lentries.release();
  ctx->ltab.release();
  ctx->pos.release();
  ctx->hashes.release();
  ctx->vgl.release();
  ctx->vabyte.release();
  ctx->vplan.release();
  ctx->smask.release();
  ctx->sel.release();
  ctx->st_keys.release();
  ctx->st_offs.release();
  ctx->st_out.release();
  ctx->st_len.release();
  ctx->st_filter.release();
  ctx->crc_streams.release();
  ctx->crc_partial.release();
  ctx->crc_tabs.release();
  ctx->crc_cnt.release();
  ctx->crc_outp.release();
  ctx->crc_cap.release();
  ctx->crc_val.release();
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_wait) (void)hipEventDestroy(ctx->ev_wait);
  if (ctx->ev_pfork) (void)hipEventDestroy(ctx->ev_pfork);
  if (ctx->ev_pdone) (void)hipEventDestroy(ctx->ev_pdone);
  for (int b = 0; b < kStageEvents; b++) {
    if (ctx->ev_part[b]) (void)hipEventDestroy(ctx->ev_part[b]);
    if (ctx->ev_free[b]) (void)hipEventDestroy(ctx->ev_free[b]);
  }
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  if (ctx->own) (void)hipStreamDestroy(ctx->own);
  if (ctx->host_buf) (void)hipHostFree(ctx->host_buf);
  if (ctx->h_out) (void)hipHostFree(ctx->h_out);
  if (ctx->h_len) (void)hipHostFree(ctx->h_len);
  for (int i = 0; i < dlsm_ctx::kUpSlots; i++) {
    if (ctx->up_own[i]) (void)hipHostFree(ctx->up_buf[i]);
    if (ctx->up_ev[i]) (void)hipEventDestroy(ctx->up_ev[i]);
  }
  if (ctx->up_block) (void)hipHostFree(ctx->up_block);
  delete ctx;
  return DLSM_OK;
}

}  // extern "C"
namespace {
// A thread's context back to its device's free list: drained, its stream and
// partition stream reset to its own, its scheduling options to their
// creation values, fault injection off.
void ctx_pool_put(dlsm_ctx* c) {
  {
    DeviceGuard g(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->pstream) (void)hipStreamSynchronize(c->pstream);
  }
  c->stream = c->own;
  c->pstream = nullptr;
  c->pcus = 0;
  c->fault = 0;
  c->vslice_bytes = 0;
  c->vpass_slices = kVMaxSlices;
  c->fallbacks.store(0, std::memory_order_relaxed);  // the next thread's count starts at zero
  if (c->opts0_set) {
    const CtxOpts& o = c->opts0;
    c->path = o.path;
    c->build_groups = o.build_groups;
    c->probe_round = o.probe_round;
    c->probe_lgc = o.probe_lgc;
    c->probe_lgr = o.probe_lgr;
    c->build_exact = o.build_exact;
    c->probe_serial = o.probe_serial;
    c->probe_multi = o.probe_multi;
  }
  CtxPool& p = ctx_pool();
  std::lock_guard<std::mutex> lk(p.m);
  p.free[c->device].push_back(c);
}
}  // namespace
extern "C" {

int dlsm_ctx_set_stream(dlsm_ctx* ctx, void* s) {
  if (!ctx) return DLSM_E_ARG;
  ctx->stream = s ? static_cast<hipStream_t>(s) : ctx->own;
  return DLSM_OK;
}

void* dlsm_ctx_stream(dlsm_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int dlsm_ctx_device(const dlsm_ctx* ctx) { return ctx ? ctx->device : -1; }

int dlsm_ctx_set_partition_stream(dlsm_ctx* ctx, void* s, uint32_t cus) {
  if (!ctx) return DLSM_E_ARG;
  ctx->pstream = static_cast<hipStream_t>(s);
  ctx->pcus = s ? cus : 0u;
  return DLSM_OK;
}

int dlsm_stream_create_cu_mask(int device, const uint32_t* mask, uint32_t words, void** out) {
  if (!out || !mask || words == 0) return DLSM_E_ARG;
  *out = nullptr;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || device < 0 || device >= c) return DLSM_E_DEVICE;
  DeviceGuard g(device);
  hipStream_t st = nullptr;
  DLSM_TRY(hipExtStreamCreateWithCUMask(&st, words, mask));  // size in uint32 elements
  *out = st;
  return DLSM_OK;
}

int dlsm_stream_destroy(void* s) {
  if (!s) return DLSM_E_ARG;
  DLSM_TRY(hipStreamDestroy(static_cast<hipStream_t>(s)));
  return DLSM_OK;
}

int dlsm_ctx_sync(dlsm_ctx* ctx) {
  if (!ctx) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  DLSM_TRY(ctx_sync(ctx, ctx->stream));
  return DLSM_OK;
}

int dlsm_ctx_set_path(dlsm_ctx* ctx, int path) {
  if (!ctx || path < 0 || path > 2) return DLSM_E_ARG;
  ctx->path = path;
  return DLSM_OK;
}

int dlsm_ctx_set_option(dlsm_ctx* ctx, int option, uint64_t value) {
  if (!ctx) return DLSM_E_ARG;
  switch (option) {
    case DLSM_OPT_PATH:
      return value > 2 ? DLSM_E_ARG : dlsm_ctx_set_path(ctx, static_cast<int>(value));
    case DLSM_OPT_PROBE_ROUND_KEYS:
      ctx->probe_round = value;
      return DLSM_OK;
    case DLSM_OPT_BUILD_GROUPS:
      if (value > static_cast<uint64_t>(kStageEvents)) return DLSM_E_ARG;
      ctx->build_groups = value ? static_cast<int>(value) : 1;
      return DLSM_OK;
    case DLSM_OPT_PROBE_CHUNK_LG:
      if (value < 12 || value > 14) return DLSM_E_ARG;
      ctx->probe_lgc = static_cast<int>(value);
      return DLSM_OK;
    case DLSM_OPT_PROBE_SLICE_LG:
      if (value < 7 || value > 8) return DLSM_E_ARG;
      ctx->probe_lgr = static_cast<int>(value);
      return DLSM_OK;
    case DLSM_OPT_BUILD_EXACT:
      if (value > 2) return DLSM_E_ARG;
      ctx->build_exact = static_cast<int>(value);
      return DLSM_OK;
    case DLSM_OPT_PROBE_ROUND_SERIAL:
      if (value > 1) return DLSM_E_ARG;
      ctx->probe_serial = value != 0;
      return DLSM_OK;
    case DLSM_OPT_FAULT_INJECT:
      if (value > static_cast<uint64_t>(-DLSM_E_BUSY)) return DLSM_E_ARG;
      ctx->fault = static_cast<int>(value);
      return DLSM_OK;
    case DLSM_OPT_VERSION_SLICE_BYTES:
      ctx->vslice_bytes = value;
      return DLSM_OK;
    case DLSM_OPT_VERSION_PASS_SLICES:
      if (value < 1 || value > kVMaxSlices) return DLSM_E_ARG;
      ctx->vpass_slices = static_cast<uint32_t>(value);
      return DLSM_OK;
    case DLSM_OPT_PROBE_MULTI:
      if (value > 1) return DLSM_E_ARG;
      ctx->probe_multi = static_cast<int>(value);
      return DLSM_OK;
    default:
      return DLSM_E_ARG;
  }
}

int dlsm_ctx_get_option(dlsm_ctx* ctx, int option, uint64_t* value) {
  if (!ctx || !value) return DLSM_E_ARG;
  switch (option) {
    case DLSM_OPT_PATH: *value = static_cast<uint64_t>(ctx->path); return DLSM_OK;
    case DLSM_OPT_PROBE_ROUND_KEYS: *value = ctx->probe_round; return DLSM_OK;
    case DLSM_OPT_BUILD_GROUPS: *value = static_cast<uint64_t>(ctx->build_groups); return DLSM_OK;
    case DLSM_OPT_PROBE_CHUNK_LG: *value = static_cast<uint64_t>(ctx->probe_lgc); return DLSM_OK;
    case DLSM_OPT_PROBE_SLICE_LG: *value = static_cast<uint64_t>(ctx->probe_lgr); return DLSM_OK;
    case DLSM_OPT_BUILD_EXACT: *value = static_cast<uint64_t>(ctx->build_exact); return DLSM_OK;
    case DLSM_OPT_PROBE_ROUND_SERIAL: *value = ctx->probe_serial ? 1u : 0u; return DLSM_OK;
    case DLSM_OPT_FAULT_INJECT: *value = static_cast<uint64_t>(ctx->fault); return DLSM_OK;
    case DLSM_OPT_VERSION_SLICE_BYTES: *value = ctx->vslice_bytes; return DLSM_OK;
    case DLSM_OPT_VERSION_PASS_SLICES: *value = ctx->vpass_slices; return DLSM_OK;
    case DLSM_OPT_PROBE_MULTI: *value = static_cast<uint64_t>(ctx->probe_multi); return DLSM_OK;
    default: return DLSM_E_ARG;
  }
}

int dlsm_ctx_reserve(dlsm_ctx* ctx, uint64_t max_keys, uint32_t max_jobs) {
  if (!ctx) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  // probe intermediates are sized in whole chunks of up to 2^14 keys
  const uint64_t pkeys = (max_keys + 16383u) & ~uint64_t(16383u);
  // probe entries / answers: chunk regions of probe_region(C) per C keys
  uint64_t pregion = 0;
  for (uint32_t C : {4096u, 8192u, 16384u})
    pregion = std::max<uint64_t>(pregion, ((max_keys + C - 1) / C) * probe_region(C));
  const uint64_t bregion = ((max_keys + kBuildChunk - 1) / kBuildChunk + max_jobs) * kBuildRegion;
  DLSM_CHECK(ctx->entries.ensure(std::max({pkeys, pregion, bregion})));
  DLSM_CHECK(ctx->pos.ensure(pkeys));
  DLSM_CHECK(ctx->smask.ensure(pregion));
  const uint64_t chunks = (max_keys + kBuildChunk - 1) / kBuildChunk + max_jobs;
  DLSM_CHECK(ctx->tab.ensure(chunks * (kMaxSlices + 1)));
  DLSM_CHECK(ctx->jobs.ensure(max_jobs));
  DLSM_CHECK(ctx->starts.ensure(2 * (max_jobs + 1)));
  DLSM_CHECK(ctx->dchunk.ensure(chunks));
  DLSM_CHECK(ctx->jobL.ensure(max_jobs));
  return DLSM_OK;
}

int dlsm_ctx_stats(dlsm_ctx* ctx, uint64_t* device_allocs, uint64_t* device_bytes) {
  if (!ctx) return DLSM_E_ARG;
  uint64_t n = 0, b = 0;
  auto add = [&](const auto& buf) {
    n += buf.gen;
    b += buf.cap * sizeof(*buf.p);
  };
  add(ctx->entries); add(ctx->tab); add(ctx->jobs); add(ctx->starts); add(ctx->dchunk);
  add(ctx->jobL); add(ctx->ljobs); add(ctx->lstarts); add(ctx->ltjobs); add(ctx->ltstarts);
  add(ctx->lentries); add(ctx->ltab); add(ctx->pos); add(ctx->smask); add(ctx->hashes);
  add(ctx->vgl); add(ctx->vabyte); add(ctx->vplan);
  add(ctx->st_keys); add(ctx->st_offs); add(ctx->st_out); add(ctx->st_len); add(ctx->st_filter);
  add(ctx->crc_streams); add(ctx->crc_partial); add(ctx->crc_tabs); add(ctx->crc_cnt); add(ctx->crc_outp); add(ctx->crc_cap);
  add(ctx->crc_val); add(ctx->sel);
  if (device_allocs) *device_allocs = n;
  if (device_bytes) *device_bytes = b;
  return DLSM_OK;
}

int dlsm_host_register(void* p, size_t len) {
  if (!p || !len) return DLSM_E_ARG;
  DLSM_TRY(hipHostRegister(p, len, hipHostRegisterDefault));
  return DLSM_OK;
}

int dlsm_host_unregister(void* p) {
  if (!p) return DLSM_E_ARG;
  DLSM_TRY(hipHostUnregister(p));
  return DLSM_OK;
}

int dlsm_ctx_host_buffer_claim(dlsm_ctx* ctx, const void* owner) {
  if (!ctx || !owner) return DLSM_E_ARG;
  const void* cur = nullptr;
  if (ctx->host_owner.compare_exchange_strong(cur, owner) || cur == owner) return DLSM_OK;
  return DLSM_E_BUSY;
}

int dlsm_ctx_host_buffer_release(dlsm_ctx* ctx, const void* owner) {
  if (!ctx || !owner) return DLSM_E_ARG;
  const void* cur = owner;
  return ctx->host_owner.compare_exchange_strong(cur, nullptr) ? DLSM_OK : DLSM_E_ARG;
}

int dlsm_ctx_host_buffer(dlsm_ctx* ctx, uint64_t min_bytes, uint64_t keep_bytes, void** out,
                         uint64_t* cap) {
  if (!ctx || !out || keep_bytes > ctx->host_cap) return DLSM_E_ARG;
  if (min_bytes > ctx->host_cap || !ctx->host_buf) {
    uint64_t c = std::max<uint64_t>(ctx->host_cap ? 2 * ctx->host_cap : (uint64_t(1) << 20), min_bytes);
    void* p = nullptr;
    DLSM_TRY(hipHostMalloc(&p, c, hipHostMallocDefault));
    if (keep_bytes) memcpy(p, ctx->host_buf, keep_bytes);
    if (ctx->host_buf) {
      // the previous buffer may still be the source of a queued copy
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipHostFree(ctx->host_buf);
    }
    ctx->host_buf = p;
    ctx->host_cap = c;
  }
  *out = ctx->host_buf;
  if (cap) *cap = ctx->host_cap;
  return DLSM_OK;
}

// Process-wide pool of page-locked host buffers (key staging of builders
// that cannot borrow their context's buffer): a released buffer is kept and
// handed to the next acquire that fits, so steady-state staging page-locks
// nothing.  Sizes are powers of two >= 1 MiB.  At most kPoolKeepBytes of
// released buffers are kept (a burst of builders does not pin host memory
// for good); a release past that frees the buffer.
}  // extern "C"
namespace {
constexpr uint64_t kPoolKeepBytes = uint64_t(1) << 30;
struct HostPool {
  std::mutex m;
  std::multimap<uint64_t, void*> free_by_size;
  struct Entry {
    uint64_t size;
    bool in_use;
  };
  std::unordered_map<void*, Entry> entry;
  uint64_t free_bytes = 0;
};
HostPool& host_pool() {
  static HostPool p;
  return p;
}
}  // namespace
extern "C" {

int dlsm_host_pool_acquire(uint64_t min_bytes, void** out, uint64_t* cap) {
  if (!out) return DLSM_E_ARG;
  *out = nullptr;
  HostPool& hp = host_pool();
  {
    std::lock_guard<std::mutex> lk(hp.m);
    auto it = hp.free_by_size.lower_bound(min_bytes);
    if (it != hp.free_by_size.end()) {
      *out = it->second;
      if (cap) *cap = it->first;
      hp.free_bytes -= it->first;
      hp.entry[it->second].in_use = true;
      hp.free_by_size.erase(it);
      return DLSM_OK;
    }
  }
  uint64_t c = uint64_t(1) << 20;
  while (c < min_bytes) c <<= 1;
  void* p = nullptr;
  DLSM_TRY(hipHostMalloc(&p, c, hipHostMallocDefault));
  {
    std::lock_guard<std::mutex> lk(hp.m);
    hp.entry[p] = HostPool::Entry{c, true};
  }
  *out = p;
  if (cap) *cap = c;
  return DLSM_OK;
}

// DLSM_E_ARG for a pointer the pool did not hand out, or one already released
// (a double release would give one buffer to two later acquirers).
int dlsm_host_pool_release(void* p) {
  if (!p) return DLSM_OK;
  HostPool& hp = host_pool();
  void* drop = nullptr;
  {
    std::lock_guard<std::mutex> lk(hp.m);
    auto it = hp.entry.find(p);
    if (it == hp.entry.end() || !it->second.in_use) return DLSM_E_ARG;
    if (hp.free_bytes + it->second.size > kPoolKeepBytes) {
      drop = p;
      hp.entry.erase(it);
    } else {
      it->second.in_use = false;
      hp.free_by_size.emplace(it->second.size, p);
      hp.free_bytes += it->second.size;
    }
  }
  if (drop) DLSM_TRY(hipHostFree(drop));
  return DLSM_OK;
}

int dlsm_host_pool_trim(void) {
  HostPool& hp = host_pool();
  std::lock_guard<std::mutex> lk(hp.m);
  for (auto& kv : hp.free_by_size) {
    (void)hipHostFree(kv.second);
    hp.entry.erase(kv.second);
  }
  hp.free_by_size.clear();
  hp.free_bytes = 0;
  return DLSM_OK;
}

int dlsm_host_alloc(size_t len, void** out) {
  if (!out || !len) return DLSM_E_ARG;
  *out = nullptr;
  DLSM_TRY(hipHostMalloc(out, len, hipHostMallocDefault));
  return DLSM_OK;
}

int dlsm_host_free(void* p) {
  if (!p) return DLSM_OK;
  DLSM_TRY(hipHostFree(p));
  return DLSM_OK;
}

// ---------------------------------------------------------------------------
// Full filter build
// ---------------------------------------------------------------------------
namespace {

// Hashed jobs: keys.bytes holds n BloomHash values (u32, 4-byte aligned,
// key_len 4, no offsets) -- what AddKey computed on the host.
bool is_hash_set(const dlsm_keyset& k) {
  return k.offsets == nullptr && k.key_len == 4 && k.suffix_len == 0 && (k.n == 0 || aligned(k.bytes, 4));
}

// seal (dlsm_bloom_full_build_block_dev): on the sliced path the slices also
// compute their crc32c partials and a seal kernel appends the block trailer
// (*sealed = true); the direct path leaves sealing to the caller.
int full_build_dev_impl(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs, int bits_per_key,
                        uint64_t* out_len_dev, bool hashed, bool seal = false, bool* sealed = nullptr) {
  if (sealed) *sealed = false;
  if (!ctx || n_jobs < 0 || (n_jobs > 0 && (!jobs || !out_len_dev))) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  if (n_jobs == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  const int k = full_num_probes(bits_per_key);
  std::vector<uint32_t> Ls(n_jobs);
  bool all_k20 = true, all_k28 = true, sliced_ok = ctx->path != 1;
  for (int j = 0; j < n_jobs; j++) {
    const dlsm_build_job& b = jobs[j];
    DLSM_CHECK(validate_keyset(b.keys));
    if (hashed && !is_hash_set(b.keys)) return DLSM_E_ARG;
    if (!b.out || !aligned(b.out, 16)) return DLSM_E_ARG;
    if (b.keys.n > 0xffffffffull * kBuildChunk) return DLSM_E_ARG;
    Ls[j] = full_num_lines(b.keys.n, bits_per_key, nullptr);
    all_k20 = all_k20 && is_k20(b.keys);
    all_k28 = all_k28 && is_k28(b.keys);
  }
  int lgR = choose_build_lgR(Ls);
  if (lgR < 0) sliced_ok = false;
  if (ctx->path == 2 && !sliced_ok) return DLSM_E_ARG;
  const int mode = hashed ? KM_HASH : (all_k20 ? KM_K20 : (all_k28 ? KM_K28 : KM_GENERIC));
  // Exact line counts (a count pass before the partition) where duplicate
  // user keys are expected to lower L below the speculative n-key count:
  // internal keys (several versions of a user key, suffix_len 8) and the
  // per-key-length batches a TableBuilder adapter hands over.  The
  // device-resident fixed-length user-key batches (one entry per user key)
  // stay speculative: one pass over the keys, with a per-slice re-hash
  // fallback for the rare batch whose duplicates do change L.
  bool any_suffix = false;
  for (int j = 0; j < n_jobs; j++) any_suffix = any_suffix || jobs[j].keys.suffix_len > 0;
  // Hashed jobs always count first: the entries keep no key to re-hash, so
  // the slice pass's fallback for a lowered line count is not available.
  const bool exact = sliced_ok && (hashed || ctx->build_exact == 1 ||
                                   (ctx->build_exact == 0 && (any_suffix || mode == KM_GENERIC)));

  std::vector<FullJobDev> hj(n_jobs);
  std::vector<uint32_t> starts(2 * n_jobs);
  uint64_t entry = 0, tabw = 0;
  uint32_t chunk = 0, slice = 0;
  for (int j = 0; j < n_jobs; j++) {
    const dlsm_build_job& b = jobs[j];
    FullJobDev& d = hj[j];
    d.keys = to_desc(b.keys);
    d.out = b.out;
    d.out_cap = b.out_cap;
    d.out_len = out_len_dev + j;
    d.entry0 = entry;
    d.n_chunks = ceil_div_u32(b.keys.n, kBuildChunk);
    d.chunk0 = chunk;
    d.L_spec = Ls[j];
    d.magic_spec = Ls[j] ? fastmod_magic(Ls[j]) : 0;
    d.n_slices = sliced_ok ? std::max<uint32_t>(1, ceil_div_u32(Ls[j], 1ull << lgR)) : 1;
    d.slice0 = slice;
    d.tab0 = tabw;
    d.k = k;
    d.bpk = bits_per_key;
    d.exact = exact ? 1 : 0;
    d.reserved = 0;
    starts[j] = chunk;
    starts[n_jobs + j] = slice;
    // chunk regions of kBuildRegion entries (buckets padded to 16-byte units)
    entry += static_cast<uint64_t>(d.n_chunks) * kBuildRegion;
    chunk += d.n_chunks;
    slice += d.n_slices;
    tabw += static_cast<uint64_t>(d.n_slices + 1) * d.n_chunks;
  }
  hipStream_t s = ctx->stream;
  const bool same = ctx->last_jobs.size() == hj.size() && ctx->last_starts == starts &&
                    memcmp(ctx->last_jobs.data(), hj.data(), sizeof(FullJobDev) * n_jobs) == 0 &&
                    ctx->jobs.gen == ctx->last_jobs_gen && ctx->starts.gen == ctx->last_starts_gen &&
                    ctx->jobs.cap >= static_cast<size_t>(n_jobs);
  if (!same) {
    ctx->last_jobs.clear();  // until the upload below is queued
    DLSM_CHECK(ctx->jobs.ensure(n_jobs));
    DLSM_CHECK(ctx->starts.ensure(2 * n_jobs));
    DLSM_CHECK(ctx_upload(ctx, ctx->jobs.p, hj.data(), sizeof(FullJobDev) * n_jobs, s));
    DLSM_CHECK(ctx_upload(ctx, ctx->starts.p, starts.data(), sizeof(uint32_t) * 2 * n_jobs, s));
    ctx->last_jobs = hj;
    ctx->last_starts = starts;
    ctx->last_jobs_gen = ctx->jobs.gen;
    ctx->last_starts_gen = ctx->starts.gen;
  }
  DLSM_CHECK(ctx->dchunk.ensure(chunk));
  DLSM_CHECK(ctx->jobL.ensure(n_jobs));
  const uint32_t* chunk0s = ctx->starts.p;
  const uint32_t* slice0s = ctx->starts.p + n_jobs;
  if (sliced_ok) {
    DLSM_CHECK(ctx->entries.ensure(entry));
    DLSM_CHECK(ctx->tab.ensure(tabw));
    uint32_t* crc_part = nullptr;
    if (seal) {
      DLSM_CHECK(ctx->crc_partial.ensure(slice));
      if (ctx->crc_tabs_lgr != lgR || ctx->crc_tabs.gen != ctx->crc_tabs_gen) {
        DLSM_CHECK(ctx->crc_tabs.ensure(kCrcTabWords));
        std::vector<uint32_t> t(kCrcTabWords);
        full_block_crc_tables(lgR, t.data());
        DLSM_CHECK(ctx_upload(ctx, ctx->crc_tabs.p, t.data(), sizeof(uint32_t) * kCrcTabWords, s));
        ctx->crc_tabs_lgr = lgR;
        ctx->crc_tabs_gen = ctx->crc_tabs.gen;
      }
      crc_part = ctx->crc_partial.p;
      if (ctx->crc_cnt.cap < static_cast<size_t>(n_jobs) || !ctx->crc_cnt.p) {
        DLSM_CHECK(ctx->crc_cnt.ensure(n_jobs));
        DLSM_TRY(hipMemsetAsync(ctx->crc_cnt.p, 0, sizeof(uint32_t) * ctx->crc_cnt.cap, s));  // reset by the sealers after
      }
    }
    // Job groups of about equal chunk counts: group g's partition (HBM-bound)
    // runs on the helper stream while the context stream runs group g-1's
    // slices (LDS-bound).
    const int G = std::max(1, std::min(ctx->build_groups, n_jobs));
    std::vector<int> cut(1, 0);
    for (int j = 1; j < n_jobs && static_cast<int>(cut.size()) < G; j++)
      if (static_cast<uint64_t>(starts[j]) * G >= static_cast<uint64_t>(chunk) * cut.size()) cut.push_back(j);
    cut.push_back(n_jobs);
    const int ng = static_cast<int>(cut.size()) - 1;
    auto chunk_at = [&](int j) { return j < n_jobs ? starts[j] : chunk; };
    auto slice_at = [&](int j) { return j < n_jobs ? starts[n_jobs + j] : slice; };
    // partition stream (dlsm_ctx_set_partition_stream, one job group): the
    // count and partition passes there, the slices on the context stream
    const bool split = ctx->pstream && ng == 1;
    hipStream_t ps = split ? ctx->pstream : s;
    if (split) DLSM_CHECK(fork_part(ctx));
    if (exact) DLSM_TRY(launch_full_count(ctx->jobs.p, chunk0s, n_jobs, chunk, ctx->dchunk.p, mode, ps));
    if (ng > 1) DLSM_CHECK(fork_aux(ctx));
    for (int g = 0; g < ng; g++) {
      const uint32_t c0 = chunk_at(cut[g]), s0 = slice_at(cut[g]);
      DLSM_TRY(launch_full_partition(ctx->jobs.p, chunk0s, n_jobs, c0, chunk_at(cut[g + 1]) - c0,
                                     ctx->dchunk.p, ctx->entries.p, ctx->tab.p, lgR, mode, exact,
                                     ng > 1 ? ctx->aux : ps));
      if (split) DLSM_CHECK(join_part(ctx));
      if (ng > 1) DLSM_CHECK(hand_over(ctx->aux, s, ctx->ev_part[g % kStageEvents]));
      DLSM_TRY(launch_full_slices(ctx->jobs.p, slice0s, n_jobs, s0, slice_at(cut[g + 1]) - s0,
                                  ctx->dchunk.p, ctx->entries.p, ctx->tab.p, lgR, s, crc_part,
                                  ctx->crc_tabs.p, ctx->crc_cnt.p));
    }
    if (seal) {
      DLSM_TRY(launch_full_block_seal(ctx->jobs.p, n_jobs, crc_part, ctx->crc_tabs.p, lgR, s));
      if (sealed) *sealed = true;
    }
  } else {
    DLSM_TRY(launch_full_count(ctx->jobs.p, chunk0s, n_jobs, chunk, ctx->dchunk.p, mode, s));
    DLSM_TRY(launch_full_zero(ctx->jobs.p, n_jobs, ctx->dchunk.p, ctx->jobL.p, s));
    DLSM_TRY(launch_full_scatter(ctx->jobs.p, chunk0s, n_jobs, chunk, ctx->jobL.p, mode, s));
  }
  return DLSM_OK;
}

}  // namespace

int dlsm_bloom_full_build_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                              int bits_per_key, uint64_t* out_len_dev) {
  return full_build_dev_impl(ctx, jobs, n_jobs, bits_per_key, out_len_dev, false);
}

int dlsm_bloom_full_build_hashed_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                     int bits_per_key, uint64_t* out_len_dev) {
  return full_build_dev_impl(ctx, jobs, n_jobs, bits_per_key, out_len_dev, true);
}

namespace {

// Stage host keysets into one device buffer; returns per-job device keysets.
// Variable-length sets are copied from offsets[0] and their offsets rebased.
int stage_keys(dlsm_ctx* ctx, const dlsm_keyset* const* sets, int n, std::vector<dlsm_keyset>& dev) {
  hipStream_t s = ctx->stream;
  uint64_t bytes = 0, offs = 0;
  std::vector<uint64_t> bpos(n), opos(n), src0(n), nb(n);
  for (int j = 0; j < n; j++) {
    const dlsm_keyset& k = *sets[j];
    src0[j] = (k.offsets && k.n) ? k.offsets[0] : 0;
    nb[j] = k.n == 0 ? 0 : (k.offsets ? k.offsets[k.n] - k.offsets[0] : k.n * uint64_t(k.key_len));
    bpos[j] = bytes;
    bytes += (nb[j] + 15) & ~uint64_t(15);
    opos[j] = offs;
    if (k.offsets) offs += k.n + 1;
  }
  DLSM_CHECK(ctx->st_keys.ensure(bytes + 16));
  DLSM_CHECK(ctx->st_offs.ensure(offs + 1));
  dev.resize(n);
  for (int j = 0; j < n; j++) {
    const dlsm_keyset& k = *sets[j];
    dlsm_keyset d = k;
    d.bytes = ctx->st_keys.p + bpos[j];
    if (nb[j])
      DLSM_TRY(hipMemcpyAsync(const_cast<uint8_t*>(d.bytes), k.bytes + src0[j], nb[j],
                              hipMemcpyHostToDevice, s));
    if (k.offsets) {
      std::vector<uint64_t> ro(k.n + 1);
      for (uint64_t i = 0; i <= k.n; i++) ro[i] = k.offsets[i] - src0[j];
      d.offsets = ctx->st_offs.p + opos[j];
      DLSM_CHECK(ctx_upload(ctx, const_cast<uint64_t*>(d.offsets), ro.data(), sizeof(uint64_t) * (k.n + 1), s));
    }
    dev[j] = d;
  }
  return DLSM_OK;
}

}  // namespace

namespace {
// Grow a page-locked host array (contents dropped; the context stream is idle
// between host-API calls, so no queued command still uses the old one).
extern "C++" template <typename T>
int host_ensure(T*& p, uint64_t& cap, uint64_t n) {
  if (n <= cap && p) return DLSM_OK;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  const uint64_t want = std::max<uint64_t>(n, 64);
  DLSM_TRY(hipHostMalloc(reinterpret_cast<void**>(&p), want * sizeof(T), hipHostMallocDefault));
  cap = want;
  return DLSM_OK;
}

// The device address of a page-locked host pointer (hipHostMalloc'd, or
// registered: dlsm_host_register), or nullptr for pageable memory.
uint8_t* host_device_view(void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // not HIP memory: clear the error the query left
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  const uintptr_t off = a.hostPointer ? reinterpret_cast<uintptr_t>(p) - reinterpret_cast<uintptr_t>(a.hostPointer) : 0;
  return static_cast<uint8_t*>(a.devicePointer) + off;
}

// Whether full_build_dev_impl takes the sliced path for this batch (the
// same choice it makes: not forced direct, and a slice width that fits).
bool full_build_sliced(const dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs, int bits_per_key) {
  if (ctx->path == 1) return false;
  std::vector<uint32_t> Ls(n_jobs);
  for (int j = 0; j < n_jobs; j++) Ls[j] = full_num_lines(jobs[j].keys.n, bits_per_key, nullptr);
  return choose_build_lgR(Ls) >= 0;
}

// Host keys -> host filters.  The keys go H2D into the context's staging.
// Sliced path: the slice kernels store each filter straight into the
// caller's slot when it is page-locked (16-byte aligned), else into
// page-locked staging copied out after the call, and the lengths into
// page-locked memory -- one stream synchronisation per call and no
// device-to-host copy commands; their stores are plain 16-byte writes.  The
// direct path (forced, or a batch too large to slice) sets bits with global
// atomics, which must not target host memory (that would need PCIe
// AtomicOps): it builds into device staging and copies the filters out.
int full_build_host_impl(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs, int bits_per_key,
                         uint64_t* out_len, bool hashed) {
  if (!ctx || n_jobs < 0 || (n_jobs > 0 && (!jobs || !out_len))) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  if (n_jobs == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  std::vector<const dlsm_keyset*> sets(n_jobs);
  for (int j = 0; j < n_jobs; j++) {
    DLSM_CHECK(validate_keyset(jobs[j].keys));
    if (!jobs[j].out) return DLSM_E_ARG;
    sets[j] = &jobs[j].keys;
  }
  const bool to_host = full_build_sliced(ctx, jobs, n_jobs, bits_per_key);
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets.data(), n_jobs, dk));
  std::vector<dlsm_build_job> dj(n_jobs);
  std::vector<uint8_t*> direct(n_jobs);
  uint64_t obytes = 0;
  std::vector<uint64_t> opos(n_jobs);
  for (int j = 0; j < n_jobs; j++) {
    const uint64_t spec = full_filter_len(jobs[j].keys.n, bits_per_key);
    const uint64_t cap = std::min(spec, jobs[j].out_cap);
    direct[j] = to_host ? host_device_view(jobs[j].out) : nullptr;
    if (direct[j] && !aligned(direct[j], 16)) direct[j] = nullptr;
    opos[j] = obytes;
    if (!direct[j]) obytes += (cap + 255) & ~uint64_t(255);
    dj[j].keys = dk[j];
    dj[j].out_cap = cap;
  }
  hipStream_t s = ctx->stream;
  if (!to_host) {
    DLSM_CHECK(ctx->st_out.ensure(obytes + 256));
    DLSM_CHECK(ctx->st_len.ensure(n_jobs));
    for (int j = 0; j < n_jobs; j++) dj[j].out = ctx->st_out.p + opos[j];
    DLSM_CHECK(full_build_dev_impl(ctx, dj.data(), n_jobs, bits_per_key, ctx->st_len.p, hashed));
    DLSM_TRY(hipMemcpyAsync(out_len, ctx->st_len.p, sizeof(uint64_t) * n_jobs, hipMemcpyDeviceToHost, s));
    DLSM_TRY(ctx_sync(ctx, s));
    int st = DLSM_OK;
    for (int j = 0; j < n_jobs; j++) {
      if (out_len[j] == 0) {
        st = DLSM_E_CAPACITY;
        continue;
      }
      DLSM_TRY(hipMemcpyAsync(jobs[j].out, dj[j].out, out_len[j], hipMemcpyDeviceToHost, s));
    }
    DLSM_TRY(ctx_sync(ctx, s));
    return st;
  }
  DLSM_CHECK(host_ensure(ctx->h_out, ctx->h_out_cap, obytes + 256));
  DLSM_CHECK(host_ensure(ctx->h_len, ctx->h_len_cap, static_cast<uint64_t>(n_jobs)));
  uint8_t* h_out_dev = host_device_view(ctx->h_out);
  uint64_t* h_len_dev = reinterpret_cast<uint64_t*>(host_device_view(ctx->h_len));
  if (!h_out_dev || !h_len_dev) return DLSM_E_DEVICE;
  for (int j = 0; j < n_jobs; j++) dj[j].out = direct[j] ? direct[j] : h_out_dev + opos[j];
  DLSM_CHECK(full_build_dev_impl(ctx, dj.data(), n_jobs, bits_per_key, h_len_dev, hashed));
  DLSM_TRY(ctx_sync(ctx, s));
  int st = DLSM_OK;
  for (int j = 0; j < n_jobs; j++) {
    out_len[j] = ctx->h_len[j];
    if (out_len[j] == 0) {
      st = DLSM_E_CAPACITY;
      continue;
    }
    if (!direct[j]) memcpy(jobs[j].out, ctx->h_out + opos[j], out_len[j]);
  }
  return st;
}
}  // namespace

int dlsm_bloom_full_build(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs, int bits_per_key,
                          uint64_t* out_len) {
  return full_build_host_impl(ctx, jobs, n_jobs, bits_per_key, out_len, false);
}

int dlsm_bloom_full_build_hashed(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs, int bits_per_key,
                                 uint64_t* out_len) {
  return full_build_host_impl(ctx, jobs, n_jobs, bits_per_key, out_len, true);
}

// ---------------------------------------------------------------------------
// Filter blocks (build + crc32c trailer) and crc32c of device buffers
// ---------------------------------------------------------------------------
namespace {
struct Crc32cTable {
  uint32_t t[256];
  Crc32cTable() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0x82f63b78u : (c >> 1);
      t[i] = c;
    }
  }
};
}  // namespace

uint32_t dlsm_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  // function-local static: C++11 thread-safe initialisation (TableBuilders
  // seal blocks from several threads)
  static const Crc32cTable table;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~init_crc;
  for (size_t i = 0; i < n; i++) c = table.t[(c ^ p[i]) & 0xffu] ^ (c >> 8);
  return ~c;
}

uint32_t dlsm_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

namespace {
int run_crc(dlsm_ctx* ctx, const std::vector<std::vector<uint8_t>>& streams, int n, uint64_t max_total,
            uint8_t* const* seal_out_host, const uint64_t* seal_cap_host, uint64_t* seal_len_dev,
            uint32_t* crc_val_dev) {
  hipStream_t s = ctx->stream;
  const size_t ss = crc_stream_size();
  const int max_parts = static_cast<int>(std::max<uint64_t>(1, crc_max_parts(max_total)));
  DLSM_CHECK(ctx->crc_streams.ensure(ss * n));
  DLSM_CHECK(ctx->crc_partial.ensure(static_cast<size_t>(max_parts) * n));
  std::vector<uint8_t> flat(ss * n);
  for (int j = 0; j < n; j++) memcpy(flat.data() + ss * j, streams[j].data(), ss);
  DLSM_CHECK(ctx_upload(ctx, ctx->crc_streams.p, flat.data(), ss * n, s));
  uint8_t* const* seal_out = nullptr;
  const uint64_t* seal_cap = nullptr;
  if (seal_out_host) {
    DLSM_CHECK(ctx->crc_outp.ensure(n));
    DLSM_CHECK(ctx->crc_cap.ensure(n));
    DLSM_CHECK(ctx_upload(ctx, ctx->crc_outp.p, seal_out_host, sizeof(uint8_t*) * n, s));
    DLSM_CHECK(ctx_upload(ctx, ctx->crc_cap.p, seal_cap_host, sizeof(uint64_t) * n, s));
    seal_out = ctx->crc_outp.p;
    seal_cap = ctx->crc_cap.p;
  }
  DLSM_TRY(launch_crc_streams(ctx->crc_streams.p, n, max_parts, ctx->crc_partial.p, seal_out, seal_cap,
                              seal_len_dev, crc_val_dev, s));
  return DLSM_OK;
}
}  // namespace

int dlsm_bloom_full_build_block_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                    int bits_per_key, uint64_t* out_len_dev) {
  if (!ctx || n_jobs < 0 || (n_jobs > 0 && (!jobs || !out_len_dev))) return DLSM_E_ARG;
  if (n_jobs == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  // The filter must leave room for the 5-byte trailer.
  std::vector<dlsm_build_job> fj(jobs, jobs + n_jobs);
  std::vector<uint8_t*> outs(n_jobs);
  std::vector<uint64_t> caps(n_jobs);
  uint64_t max_total = 0;
  for (int j = 0; j < n_jobs; j++) {
    fj[j].out_cap = jobs[j].out_cap >= 5 ? jobs[j].out_cap - 5 : 0;
    outs[j] = jobs[j].out;
    caps[j] = jobs[j].out_cap;
    max_total = std::max(max_total, full_filter_len(jobs[j].keys.n, bits_per_key) + 1);
  }
  // the sliced build seals its own filters (the crc fused into its slice
  // pass); the direct path takes the separate crc passes below
  bool sealed = false;
  DLSM_CHECK(full_build_dev_impl(ctx, fj.data(), n_jobs, bits_per_key, out_len_dev, false, true, &sealed));
  if (sealed) return DLSM_OK;
  std::vector<std::vector<uint8_t>> st(n_jobs, std::vector<uint8_t>(crc_stream_size()));
  for (int j = 0; j < n_jobs; j++) crc_stream_fill(st[j].data(), jobs[j].out, out_len_dev + j, 0, 1);
  return run_crc(ctx, st, n_jobs, max_total, outs.data(), caps.data(), out_len_dev, nullptr);
}

int dlsm_bloom_full_build_block(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                int bits_per_key, uint64_t* out_len) {
  if (!ctx || n_jobs < 0 || (n_jobs > 0 && (!jobs || !out_len))) return DLSM_E_ARG;
  if (n_jobs == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  std::vector<const dlsm_keyset*> sets(n_jobs);
  for (int j = 0; j < n_jobs; j++) {
    DLSM_CHECK(validate_keyset(jobs[j].keys));
    if (!jobs[j].out) return DLSM_E_ARG;
    sets[j] = &jobs[j].keys;
  }
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets.data(), n_jobs, dk));
  std::vector<dlsm_build_job> dj(n_jobs);
  std::vector<uint64_t> opos(n_jobs);
  uint64_t obytes = 0;
  for (int j = 0; j < n_jobs; j++) {
    const uint64_t spec = full_filter_len(jobs[j].keys.n, bits_per_key) + 5;
    const uint64_t cap = std::min(spec, jobs[j].out_cap);
    opos[j] = obytes;
    obytes += (cap + 255) & ~uint64_t(255);
    dj[j].keys = dk[j];
    dj[j].out_cap = cap;
  }
  DLSM_CHECK(ctx->st_out.ensure(obytes + 256));
  DLSM_CHECK(ctx->st_len.ensure(n_jobs));
  for (int j = 0; j < n_jobs; j++) dj[j].out = ctx->st_out.p + opos[j];
  DLSM_CHECK(dlsm_bloom_full_build_block_dev(ctx, dj.data(), n_jobs, bits_per_key, ctx->st_len.p));
  hipStream_t s = ctx->stream;
  DLSM_TRY(hipMemcpyAsync(out_len, ctx->st_len.p, sizeof(uint64_t) * n_jobs, hipMemcpyDeviceToHost, s));
  DLSM_TRY(ctx_sync(ctx, s));
  int st = DLSM_OK;
  for (int j = 0; j < n_jobs; j++) {
    if (out_len[j] == 0) {
      st = DLSM_E_CAPACITY;
      continue;
    }
    DLSM_TRY(hipMemcpyAsync(jobs[j].out, dj[j].out, out_len[j], hipMemcpyDeviceToHost, s));
  }
  DLSM_TRY(ctx_sync(ctx, s));
  return st;
}

int dlsm_crc32c_dev(dlsm_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, int n,
                    uint32_t* crc_out) {
  if (!ctx || n < 0 || (n > 0 && (!bufs || !lens || !crc_out))) return DLSM_E_ARG;
  if (n == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  std::vector<std::vector<uint8_t>> st(n, std::vector<uint8_t>(crc_stream_size()));
  uint64_t max_total = 0;
  for (int j = 0; j < n; j++) {
    if (lens[j] && !bufs[j]) return DLSM_E_ARG;
    crc_stream_fill(st[j].data(), bufs[j], nullptr, lens[j], 0);
    max_total = std::max(max_total, lens[j]);
  }
  DLSM_CHECK(ctx->crc_val.ensure(n));
  DLSM_CHECK(run_crc(ctx, st, n, max_total, nullptr, nullptr, nullptr, ctx->crc_val.p));
  DLSM_TRY(hipMemcpyAsync(crc_out, ctx->crc_val.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, ctx->stream));
  DLSM_TRY(ctx_sync(ctx, ctx->stream));
  return DLSM_OK;
}

// ---------------------------------------------------------------------------
// Internal keys: flush / compaction selection and user-key gather
// ---------------------------------------------------------------------------
int dlsm_internal_keys_select_dev(dlsm_ctx* ctx, const dlsm_keyset* ikeys, int policy,
                                  uint64_t smallest_snapshot, uint8_t* keep_dev, uint64_t* n_kept,
                                  uint64_t* kept_bytes, uint64_t* first_corrupt) {
  if (!ctx || !ikeys || (policy != DLSM_SELECT_FLUSH && policy != DLSM_SELECT_COMPACTION))
    return DLSM_E_ARG;
  dlsm_keyset k = *ikeys;
  k.suffix_len = 0;
  DLSM_CHECK(validate_keyset(k));
  if (ikeys->n > 0 && !keep_dev) return DLSM_E_ARG;
  uint64_t res[4] = {0, 0, ~uint64_t(0), 0};  // n_kept, kept_bytes, first_bad
  if (k.n > 0) {
    DeviceGuard g(ctx->device);
    hipStream_t s = ctx->stream;
    const uint64_t nb = select_blocks(k.n);
    DLSM_CHECK(ctx->sel.ensure(2 * nb + 3));
    uint64_t* bc = ctx->sel.p;
    uint64_t* bb = bc + nb;
    uint64_t* tot = bb + nb;
    uint64_t* bad = tot + 2;
    DLSM_TRY(hipMemsetAsync(bad, 0xff, sizeof(uint64_t), s));
    DLSM_TRY(launch_key_select(to_desc(k), policy, smallest_snapshot, keep_dev, bc, bb,
                               reinterpret_cast<unsigned long long*>(bad), tot, s));
    DLSM_TRY(hipMemcpyAsync(res, tot, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    DLSM_TRY(ctx_sync(ctx, s));
  }
  if (n_kept) *n_kept = res[0];
  if (kept_bytes) *kept_bytes = res[1];
  if (first_corrupt) *first_corrupt = res[2];
  if (policy == DLSM_SELECT_FLUSH && res[2] != ~uint64_t(0)) return DLSM_E_CORRUPT;
  return DLSM_OK;
}

int dlsm_user_keys_gather_dev(dlsm_ctx* ctx, const dlsm_keyset* ikeys, const uint8_t* keep_dev,
                              uint8_t* user_keys_dev, uint64_t* offsets_dev) {
  if (!ctx || !ikeys) return DLSM_E_ARG;
  dlsm_keyset k = *ikeys;
  k.suffix_len = 0;
  DLSM_CHECK(validate_keyset(k));
  if (k.offsets && !offsets_dev) return DLSM_E_ARG;
  if (!k.offsets && k.key_len < DLSM_INTERNAL_KEY_TRAILER) return DLSM_E_ARG;
  if (k.n == 0) {
    if (offsets_dev) DLSM_TRY(hipMemsetAsync(offsets_dev, 0, sizeof(uint64_t), ctx->stream));
    return DLSM_OK;
  }
  if (!keep_dev || !user_keys_dev) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  const uint64_t nb = select_blocks(k.n);
  DLSM_CHECK(ctx->sel.ensure(2 * nb + 3));
  uint64_t* bc = ctx->sel.p;
  uint64_t* bb = bc + nb;
  DLSM_TRY(launch_key_gather(to_desc(k), keep_dev, bc, bb, user_keys_dev,
                             k.offsets ? offsets_dev : nullptr, bb + nb, ctx->stream));
  return DLSM_OK;
}

// ---------------------------------------------------------------------------
// Full filter probe
// ---------------------------------------------------------------------------
}  // extern "C"
namespace {
uint32_t device_cus_of(int dev) {
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  return static_cast<uint32_t>(n);
}

// The one-pass layout of a multi-group set (bloom_internal.h, MGroupDev): the
// groups ordered by image width (one slice launch per width), every group cut
// into full 128 KiB slices (2^(11 - lgw) lines), the slices numbered globally.
// Each width class gets a workgroup plan over the CUs: a slice's share of the
// workgroups is its share of the class's entries -- every lookup has one entry
// per group, so slice s of group j (nl_s of L_j lines) expects nl_s / L_j of
// them (a 3-slice group's slices get ~10x the workgroups of a 30-slice
// group's).  A set that does not fit (a group with more than 256 slices, more
// than kMGMaxSlices in all) keeps the per-group passes.  `s` is synchronised by
// the caller before the host tables go out of scope.
hipError_t mg_layout(dlsm_filterset* fs, hipStream_t s) {
  const int G = static_cast<int>(fs->groups.size());
  std::vector<int> order(G);
  for (int j = 0; j < G; j++) order[j] = j;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return fs->groups[a].lgw < fs->groups[b].lgw; });
  std::vector<MGroupDev> md;
  uint32_t sbase = 0;
  for (int j : order) {
    const ProbeGroup& g = fs->groups[j];
    const uint32_t R = 1u << (11 - g.lgw);
    const uint32_t S = ceil_div_u32(g.L, R);
    if (S < 1 || S > static_cast<uint32_t>(kMaxSlices) || !g.stacked) return hipSuccess;
    MGroupDev d{};
    d.image = reinterpret_cast<const uint8_t*>(g.stacked);
    d.L = g.L;
    d.magic = g.magic;
    d.R = R;
    d.rmagic = fastmod_magic(R);
    d.S = S;
    d.sbase = sbase;
    d.slotmap = g.slotmap;
    d.k = g.k;
    d.lgw = g.lgw;
    d.mask_byte = g.mask_byte;
    md.push_back(d);
    sbase += S;
  }
  if (sbase > kMGMaxSlices) return hipSuccess;
  // every group's fixed sub-regions: entries, answers; its table columns
  const uint32_t C = 1u << mg_chunk_lg(G);
  uint32_t eoff = 0, aoff = 0;
  for (int j = 0; j < G; j++) {
    md[j].tcol = md[j].sbase + static_cast<uint32_t>(j);
    md[j].eoff = eoff;
    md[j].aoff = aoff;
    eoff += mg_sub_entries(C, md[j].S);
    aoff += mg_sub_abytes(C, md[j].S, md[j].lgw);
  }
  if (eoff > 65535u || aoff > 96u * 1024u) return hipSuccess;  // u16 table offsets / the unpermute's LDS
  // the partition's staging LDS: the largest set of mg_set_size groups
  const int P = mg_set_size(mg_chunk_lg(G));
  uint32_t stage = 0;
  for (int j0 = 0; j0 < G; j0 += P) {
    uint32_t st = 0;
    for (int j = j0; j < std::min(G, j0 + P); j++) st += mg_sub_entries(C, md[j].S) * 4u;
    stage = std::max(stage, st);
  }
  if (stage > 64u * 1024u) return hipSuccess;
  const uint32_t budget = device_cus_of(fs->device);
  std::vector<uint32_t> plan;
  std::vector<MGClass> classes;
  for (int j = 0; j < G;) {
    MGClass cl;
    cl.lgw = md[j].lgw;
    cl.s0 = md[j].sbase;
    cl.K = 6;
    std::vector<double> w;  // expected entry share per slice
    int q = j;
    for (; q < G && md[q].lgw == cl.lgw; q++) {
      if (md[q].k != 6) cl.K = 0;
      for (uint32_t t = 0; t < md[q].S; t++) {
        const uint32_t nl = std::min(md[q].R, md[q].L - t * md[q].R);
        w.push_back(static_cast<double>(nl) / md[q].L);
      }
    }
    cl.S = static_cast<uint32_t>(w.size());
    double W = 0;
    for (double x : w) W += x;
    std::vector<uint32_t> parts(cl.S);
    std::vector<std::pair<double, uint32_t>> rem;
    uint32_t used = 0;
    for (uint32_t t = 0; t < cl.S; t++) {
      const double want = budget * w[t] / W;
      parts[t] = std::max<uint32_t>(1u, static_cast<uint32_t>(want));
      used += parts[t];
      rem.push_back({want - parts[t], t});
    }
    std::sort(rem.begin(), rem.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (size_t r = 0; r < rem.size() && used < budget; r++, used++) parts[rem[r].second]++;
    cl.plan_off = static_cast<uint32_t>(plan.size());
    uint32_t acc = 0;
    for (uint32_t t = 0; t < cl.S; t++) {
      plan.push_back(acc);
      acc += parts[t];
    }
    plan.push_back(acc);
    cl.wgs = acc;
    classes.push_back(cl);
    j = q;
  }
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&fs->d_mg), sizeof(MGroupDev) * md.size());
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&fs->d_mgplan), sizeof(uint32_t) * plan.size());
  if (e == hipSuccess) e = hipMemcpy(fs->d_mg, md.data(), sizeof(MGroupDev) * md.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(fs->d_mgplan, plan.data(), sizeof(uint32_t) * plan.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  (void)s;
  fs->mg_n = G;
  fs->mg_slices = sbase;
  fs->mg_region = eoff;
  fs->mg_abytes = aoff;
  fs->mg_stage_bytes = stage;
  fs->mg_classes = classes;
  return hipSuccess;
}
}  // namespace
extern "C" {

int dlsm_filterset_create(dlsm_ctx* ctx, const uint8_t* const* filters, const uint64_t* lens,
                          int n_filters, int filters_are_device, dlsm_filterset** out) {
  if (!ctx || !out || !filters || !lens || n_filters < 1 || n_filters > 64) return DLSM_E_ARG;
  *out = nullptr;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  // Metadata (k, num_lines) from each filter's 5-byte tail.
  std::vector<FilterDev> h(n_filters);
  std::vector<uint64_t> off(n_filters);
  uint64_t blob = 0;
  for (int f = 0; f < n_filters; f++) {
    if (!filters[f] || lens[f] < 5) return DLSM_E_CORRUPT;
    uint8_t tail[5];
    const uint8_t* tp = filters[f] + lens[f] - 5;
    if (filters_are_device) {
      DLSM_TRY(hipMemcpyAsync(tail, tp, 5, hipMemcpyDeviceToHost, s));
      DLSM_TRY(ctx_sync(ctx, s));
    } else {
      memcpy(tail, tp, 5);
    }
    int k, lg;
    uint32_t L;
    DLSM_CHECK(parse_tail(tail, lens[f], &k, &L, &lg));
    h[f].L = L;
    h[f].magic = fastmod_magic(L);
    h[f].k = k;
    h[f].lg = lg;
    off[f] = blob;
    blob += (lens[f] + 255) & ~uint64_t(255);
  }
  dlsm_filterset* fs = new (std::nothrow) dlsm_filterset();
  if (!fs) return DLSM_E_NOMEM;
  fs->device = ctx->device;
  fs->F = n_filters;
  fs->blob_bytes = blob;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&fs->blob), blob);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&fs->d_filters), sizeof(FilterDev) * n_filters);
  if (e != hipSuccess) {
    dlsm_filterset_destroy(fs);
    return from_hip(e);
  }
  for (int f = 0; f < n_filters; f++) {
    e = hipMemcpyAsync(fs->blob + off[f], filters[f], lens[f],
                       filters_are_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s);
    if (e != hipSuccess) break;
    h[f].data = fs->blob + off[f];
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(fs->d_filters, h.data(), sizeof(FilterDev) * n_filters, hipMemcpyHostToDevice, s);
  fs->h = h;
  // Sliced-probe groups: within each mask byte, the filters with one (L, k)
  // share a stacked image.  Every filter must have 64-byte lines (the
  // reader's common case) for the sliced path; otherwise the set is probed
  // directly.
  bool stack = true;
  for (int f = 0; f < n_filters; f++) stack = stack && h[f].lg == 6;
  std::vector<std::vector<int>> members;
  if (stack) {
    for (int b = 0; b * 8 < n_filters; b++) {
      bool first = true;
      std::vector<bool> done(8, false);
      for (int f = 8 * b; f < std::min(n_filters, 8 * b + 8); f++) {
        if (done[f - 8 * b]) continue;
        ProbeGroup g;
        g.L = h[f].L;
        g.magic = h[f].magic;
        g.k = h[f].k;
        g.mask_byte = b;
        g.first_of_byte = first;
        first = false;
        std::vector<int> m;
        for (int q = f; q < std::min(n_filters, 8 * b + 8); q++)
          if (!done[q - 8 * b] && h[q].L == g.L && h[q].k == g.k) {
            done[q - 8 * b] = true;
            m.push_back(q);
          }
        const int nm = static_cast<int>(m.size());
        g.lgw = nm == 1 ? 0 : nm == 2 ? 1 : nm <= 4 ? 2 : 3;
        if (const char* e = getenv("DLSM_PROBE_PACKED"); e && atoi(e) == 0) g.lgw = 3;  // A/B knob
        for (int j = 0; j < nm && g.lgw < 3; j++) g.slotmap |= static_cast<uint32_t>(m[j] % 8) << (4 * j);
        fs->groups.push_back(g);
        members.push_back(m);
      }
    }
  }
  const size_t G = fs->groups.size();
  if (e == hipSuccess && G) {
    std::vector<FilterDev> slots(8 * G, FilterDev{nullptr, 0, 0, 0, 0});
    for (size_t g = 0; g < G; g++)
      for (int f : members[g]) slots[8 * g + (f % 8)] = h[f];
    e = hipMalloc(reinterpret_cast<void**>(&fs->d_slots), sizeof(FilterDev) * slots.size());
    if (e == hipSuccess)
      e = hipMemcpyAsync(fs->d_slots, slots.data(), sizeof(FilterDev) * slots.size(), hipMemcpyHostToDevice, s);
    for (size_t g = 0; g < G && e == hipSuccess; g++) {
      ProbeGroup& grp = fs->groups[g];
      const uint64_t bytes = static_cast<uint64_t>(grp.L) * (64u << grp.lgw);
      e = hipMalloc(reinterpret_cast<void**>(&grp.stacked), bytes);
      if (e == hipSuccess)
        e = grp.lgw == 3 ? launch_stack_filters(fs->d_slots + 8 * g, grp.L, grp.stacked, s)
                         : launch_pack_filters(fs->d_slots + 8 * g, grp.slotmap, grp.lgw, grp.L, grp.stacked, s);
      fs->stacked_bytes += bytes;
    }
  }
  if (e == hipSuccess && G >= 2 && G <= static_cast<size_t>(kMGMaxGroups)) e = mg_layout(fs, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // `slots` (and mg_layout's tables) are pageable host memory
  if (e != hipSuccess) {
    dlsm_filterset_destroy(fs);
    return from_hip(e);
  }
  *out = fs;
  return DLSM_OK;
}

int dlsm_filterset_destroy(dlsm_filterset* fs) {
  if (!fs) return DLSM_OK;
  DeviceGuard g(fs->device);
  for (auto& grp : fs->groups)
    if (grp.stacked) (void)hipFree(grp.stacked);
  if (fs->d_mg) (void)hipFree(fs->d_mg);
  if (fs->d_mgplan) (void)hipFree(fs->d_mgplan);
  if (fs->d_slots) (void)hipFree(fs->d_slots);
  if (fs->d_filters) (void)hipFree(fs->d_filters);
  if (fs->blob) (void)hipFree(fs->blob);
  delete fs;
  return DLSM_OK;
}

int dlsm_filterset_size(const dlsm_filterset* fs, int* n_filters, uint64_t* device_bytes) {
  if (!fs) return DLSM_E_ARG;
  if (n_filters) *n_filters = fs->F;
  if (device_bytes) *device_bytes = fs->blob_bytes + fs->stacked_bytes;
  return DLSM_OK;
}

namespace {

// Slices of a group's image (line count L): the LDS holds up to 2^lgR lines
// (a byte-wide stacked table with more than kMaxSlices slices of 64 KiB moves
// to 128 KiB, one workgroup per CU; packed images always use 128 KiB of
// 2^(11 - lgw) lines).  Balanced: the slice pass runs S x parts workgroups
// with parts = 256 / S0 (slice_parts, S0 = the slice count at full width),
// so the slices are narrowed to R = ceil(L / floor(256 / parts)) lines to fill
// the 256 CUs exactly -- 8 x 1.6 M-key filters (31,251 lines): 128 slices of
// 245 lines x 2 parts = 256 workgroups instead of 123 x 2 = 246.
// ($DLSM_PROBE_BALANCE=0: full-width slices, for A/B.)  Returns S, or 0
// when the group cannot be sliced.
uint32_t group_slices(const dlsm_ctx* ctx, const ProbeGroup& g, int* lgR, uint32_t* R_out) {
  static const bool balance = [] {
    const char* e = getenv("DLSM_PROBE_BALANCE");
    return !(e && atoi(e) == 0);
  }();
  const uint32_t L = g.L;
  if (g.lgw < 3) {
    *lgR = 11 - g.lgw;
  } else {
    *lgR = ctx->probe_lgr;
    if (ceil_div_u32(L, 1u << *lgR) > kMaxSlices && *lgR < 8) *lgR = 8;
  }
  const uint32_t Rmax = 1u << *lgR;
  const uint32_t S0 = ceil_div_u32(L, Rmax);
  if (S0 < 1 || S0 > kMaxSlices) return 0;
  uint32_t R = Rmax;
  const uint32_t per_cu = *lgR == 7 && g.lgw == 3 ? 2u : 1u;  // slice workgroups resident per CU
  const uint32_t slots = kBuildSliceCUs * per_cu;
  if (balance && S0 < slots) {
    const uint32_t parts = std::max(1u, slots / S0);
    const uint32_t S_target = slots / parts;
    R = std::min(Rmax, ceil_div_u32(L, S_target));
  }
  *R_out = R;
  return ceil_div_u32(L, R);
}

// (slice, part) workgroups of the slice pass: about one resident wave of
// workgroups (256 CUs x 2 slices of 64 KiB or 1 of 128 KiB), each part at
// least one chunk per wave (a part's waves split its chunks into equal
// groups).  ($DLSM_SLICE_WGS_PER_CU overrides the 2 / 1 slices per CU,
// $DLSM_SLICE_PARTS the parts: A/B knobs.)
int slice_parts(uint32_t S, uint32_t nC, int lgR) {
  static const uint32_t per_cu_env = [] {
    const char* e = getenv("DLSM_SLICE_WGS_PER_CU");
    return e ? static_cast<uint32_t>(atoi(e)) : 0u;
  }();
  static const int parts_env = [] {  // A/B knob: parts per slice
    const char* e = getenv("DLSM_SLICE_PARTS");
    return e ? atoi(e) : 0;
  }();
  if (parts_env > 0) return parts_env;
  const uint32_t resident = 256u * (per_cu_env ? per_cu_env : (lgR == 7 ? 2u : 1u));
  int parts = static_cast<int>(std::max<uint32_t>(1, (resident + S / 2) / S));
  return std::min<int>(parts, static_cast<int>(std::max<uint32_t>(1, nC / 16)));
}

// A filter set of several groups (filters of different sizes, more than 8
// filters): every lookup is hashed ONCE (hash pass, 4 B per key), then each
// group partitions the hashes by its own line count and probes its stacked
// image, OR-ing its answer bits into the group's mask byte.  A group too large
// to slice is probed directly from the same hashes.
int probe_grouped(dlsm_ctx* ctx, const dlsm_filterset* fs, const KeyDesc& kd, int mode, uint8_t* mask_dev) {
  hipStream_t s = ctx->stream;
  const uint64_t n = kd.n;
  const int lgC = ctx->probe_lgc;
  const uint64_t C = 1ull << lgC;
  const int mb = (fs->F + 7) / 8;
  const uint32_t nC = ceil_div_u32(n, C);
  KeyDesc hk = kd;  // hashed lookups (KM_HASH) are probed as given
  if (mode != KM_HASH) {
    DLSM_CHECK(ctx->hashes.ensure(n));
    DLSM_TRY(launch_probe_hash(kd, ctx->hashes.p, mode, s));
    hk.bytes = reinterpret_cast<const uint8_t*>(ctx->hashes.p);
    hk.offsets = nullptr;
    hk.n = n;
    hk.key_len = 4;
    hk.suffix = 0;
  }
  uint32_t Smax = 0;
  for (const auto& g : fs->groups) {
    int lg;
    uint32_t R;
    Smax = std::max(Smax, group_slices(ctx, g, &lg, &R));
  }
  const uint64_t rstride = static_cast<uint64_t>(nC) * probe_region(static_cast<uint32_t>(C));
  DLSM_CHECK(ctx->entries.ensure(rstride));
  DLSM_CHECK(ctx->pos.ensure(static_cast<uint64_t>(nC) * C));
  DLSM_CHECK(ctx->smask.ensure(rstride));
  DLSM_CHECK(ctx->tab.ensure(static_cast<uint64_t>(Smax + 1) * nC));
  for (size_t gi = 0; gi < fs->groups.size(); gi++) {
    const ProbeGroup& g = fs->groups[gi];
    int lgR;
    uint32_t R;
    const uint32_t S = group_slices(ctx, g, &lgR, &R);
    if (S == 0 || ctx->path == 1) {
      DLSM_TRY(launch_probe_direct_group(fs->d_slots + 8 * gi, hk, mask_dev, mb, g.mask_byte,
                                         g.first_of_byte, s));
      continue;
    }
    DLSM_TRY(launch_probe_partition(hk, g.L, g.magic, R, S, ctx->entries.p, ctx->pos.p, ctx->tab.p,
                                    KM_HASH, lgC, s));
    DLSM_TRY(launch_probe_slices(g.stacked, g.L, g.magic, g.k, lgR, R, g.lgw, g.slotmap, S, nC, ctx->entries.p,
                                 ctx->tab.p, ctx->smask.p, slice_parts(S, nC, lgR), lgC, s));
    DLSM_TRY(launch_probe_unpermute_group(n, ctx->pos.p, ctx->smask.p, mask_dev, mb, g.mask_byte,
                                          g.first_of_byte, lgC, s));
  }
  return DLSM_OK;
}

// A multi-group set in ONE pass (dlsm_filterset::d_mg): one partition that
// reads and hashes each lookup once and buckets it by every group's slice, one
// slice launch per image-width class over all of the class's slices, one
// unpermute that assembles every mask byte.  Per lookup: 20 B key in, G x
// (4 B entry + 2 B position) out; G x 4 B in, G x W/8 B out (W: the group's
// image field, 1..8 bits); G x (2 B + W/8 B) in, the mask bytes out --
// against the per-group passes' hash pass plus G x (4 B hash in + 6 B out,
// 5 B, 3 B + a mask read-modify-write).
int probe_multi(dlsm_ctx* ctx, const dlsm_filterset* fs, const KeyDesc& kd, int mode, uint8_t* mask_dev) {
  hipStream_t s = ctx->stream;
  const uint64_t n = kd.n;
  const int G = fs->mg_n;
  const int lgC = mg_chunk_lg(G);
  const uint64_t C = 1ull << lgC;
  const uint32_t rowlen = fs->mg_slices + static_cast<uint32_t>(G);
  const uint64_t mbytes = (fs->F + 7) / 8;
  // Rounds of probe_round keys (DLSM_OPT_PROBE_ROUND_KEYS), pipelined over
  // two streams as in the one-group path: round r's partition (HBM-bound, on
  // the helper stream) beside round r-1's slice pass (LDS-bound) and
  // unpermute, over kProbeBufs rotating buffer sets.
  uint64_t round = n;
  if (ctx->probe_round && ctx->probe_round < n) round = std::max<uint64_t>(C, (ctx->probe_round / C) * C);
  const uint64_t n_rounds = (n + round - 1) / round;
  const bool pipe = n_rounds > 1 && !ctx->probe_serial;
  const int nbuf = pipe ? kProbeBufs : 1;
  const uint64_t nCmax = (std::min(round, n) + C - 1) >> lgC;
  const uint64_t estride = nCmax * fs->mg_region, astride = nCmax * fs->mg_abytes;
  const uint64_t pstride = nCmax * G * C, tstride = nCmax * rowlen;
  DLSM_CHECK(ctx->entries.ensure(estride * nbuf));
  DLSM_CHECK(ctx->smask.ensure(astride * nbuf));
  DLSM_CHECK(ctx->pos.ensure(pstride * nbuf));
  DLSM_CHECK(ctx->tab.ensure(tstride * nbuf));
  if (pipe) DLSM_CHECK(fork_aux(ctx));
  hipStream_t ps = pipe ? ctx->aux : s;
  for (uint64_t r = 0; r < n_rounds; r++) {
    const uint64_t r0 = r * round;
    const uint64_t nr = std::min(round, n - r0);
    const uint64_t nC = (nr + C - 1) >> lgC;
    const int b = static_cast<int>(r % nbuf);
    uint32_t* ent = ctx->entries.p + b * estride;
    uint8_t* ans = ctx->smask.p + b * astride;
    uint16_t* pos = ctx->pos.p + b * pstride;
    uint16_t* tab = ctx->tab.p + b * tstride;
    KeyDesc kr = kd;
    kr.n = nr;
    if (kd.offsets) kr.offsets = kd.offsets + r0;
    else kr.bytes = kd.bytes + r0 * kd.key_len;
    if (pipe && r >= static_cast<uint64_t>(nbuf)) DLSM_TRY(hipStreamWaitEvent(ps, ctx->ev_free[b], 0));
    DLSM_TRY(launch_probe_mpartition(kr, fs->d_mg, G, rowlen, fs->mg_region, fs->mg_stage_bytes, ent, pos, tab,
                                     mode, ps));
    if (pipe) DLSM_CHECK(hand_over(ps, s, ctx->ev_part[b]));
    for (const MGClass& cl : fs->mg_classes)
      DLSM_TRY(launch_probe_mslices(cl.lgw, cl.K, fs->d_mg, G, cl.s0, cl.S, rowlen, fs->mg_region, fs->mg_abytes,
                                    static_cast<uint32_t>(nC), ent, tab, ans, fs->d_mgplan + cl.plan_off, cl.wgs, s));
    DLSM_TRY(launch_probe_munpermute(nr, fs->d_mg, G, fs->mg_abytes, pos, ans, mask_dev + r0 * mbytes, mbytes, s));
    if (pipe) DLSM_TRY(hipEventRecord(ctx->ev_free[b], s));
  }
  return DLSM_OK;
}

}  // namespace

namespace {
// hashed: the keys are BloomHash values (u32 each, key_len 4), as the host
// computes them in KeyMayMatch (full_filter_block.cc:271).
int full_probe_dev_impl(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* keys, uint8_t* mask_dev,
                        bool hashed) {
  if (!ctx || !fs || !keys) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  if (fs->device != ctx->device) return DLSM_E_ARG;
  DLSM_CHECK(validate_keyset(*keys));
  if (hashed && !is_hash_set(*keys)) return DLSM_E_ARG;
  if (keys->n == 0) return DLSM_OK;
  if (!mask_dev) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  const int mode = hashed ? KM_HASH : is_k20(*keys) ? KM_K20 : (is_k28(*keys) ? KM_K28 : KM_GENERIC);
  const KeyDesc kd = to_desc(*keys);
  const int lgC = ctx->probe_lgc;
  const uint64_t C = 1ull << lgC;
  const bool fits = keys->n <= 0xffffffffull * C;
  // The set's sliceable groups (all of them must be, for the forced sliced path).
  bool all_sliceable = !fs->groups.empty();
  for (const auto& grp : fs->groups) {
    int lg;
    uint32_t R;
    all_sliceable = all_sliceable && group_slices(ctx, grp, &lg, &R) != 0;
  }
  if (ctx->path == 2 && !(all_sliceable && fits)) return DLSM_E_ARG;
  if (fs->groups.empty() || ctx->path == 1 || !fits) {
    DLSM_TRY(launch_probe_direct(fs->d_filters, fs->F, kd, mask_dev, mode, s));
    return DLSM_OK;
  }
  if (fs->mg_n > 0 && ctx->probe_multi && fs->groups.size() > 1 &&
      keys->n <= (0xffffffffull << mg_chunk_lg(fs->mg_n)))
    return probe_multi(ctx, fs, kd, mode, mask_dev);
  if (fs->groups.size() > 1 || !all_sliceable) return probe_grouped(ctx, fs, kd, mode, mask_dev);

  // One group (the bench's set: <= 8 filters of one line count): the keys are
  // hashed inside the partition pass.
  const ProbeGroup& grp = fs->groups[0];
  int lgR;
  uint32_t R;
  const uint32_t S = group_slices(ctx, grp, &lgR, &R);
  // Rounds of probe_round keys, pipelined: round r's partition (helper
  // stream) overlaps round r-1's slice + unpermute (context stream), or
  // serial (DLSM_OPT_PROBE_ROUND_SERIAL).  A round's intermediates (4 B hash +
  // 2 B position + 1 B answer per key) live in one of kProbeBufs rotating
  // buffers, small enough to stay resident in the 256 MiB Infinity Cache
  // while the keys stream past.
  const uint64_t n = keys->n;
  uint64_t round = n;
  if (ctx->probe_round && ctx->probe_round < n)
    round = std::max<uint64_t>(C, (ctx->probe_round / C) * C);
  const uint64_t n_rounds = (n + round - 1) / round;
  const bool pipe = n_rounds > 1 && !ctx->probe_serial;
  const int nbuf = pipe ? kProbeBufs : 1;
  const uint32_t nCmax = ceil_div_u32(std::min(round, n), C);
  const uint64_t kstride = static_cast<uint64_t>(nCmax) * C;  // keys per buffer (16-B aligned)
  const uint64_t rstride = static_cast<uint64_t>(nCmax) * probe_region(static_cast<uint32_t>(C));  // entries / answers
  const uint64_t tstride = static_cast<uint64_t>(S + 1) * nCmax;        // table u16 per buffer
  DLSM_CHECK(ctx->entries.ensure(rstride * nbuf));
  DLSM_CHECK(ctx->pos.ensure(kstride * nbuf));
  DLSM_CHECK(ctx->smask.ensure(rstride * nbuf));
  DLSM_CHECK(ctx->tab.ensure(tstride * nbuf));
  if (pipe) DLSM_CHECK(fork_aux(ctx));
  // dlsm_ctx_set_partition_stream (one round): the partition there, the
  // slice + unpermute passes on the context stream
  const bool split = ctx->pstream && n_rounds == 1;
  if (split) DLSM_CHECK(fork_part(ctx));
  hipStream_t ps = pipe ? ctx->aux : (split ? ctx->pstream : s);
  for (uint64_t r = 0; r < n_rounds; r++) {
    const uint64_t r0 = r * round;
    const uint64_t nr = std::min(round, n - r0);
    const uint32_t nC = ceil_div_u32(nr, C);
    const int b = static_cast<int>(r % nbuf);
    uint32_t* ent = ctx->entries.p + b * rstride;
    uint16_t* pos = ctx->pos.p + b * kstride;
    uint8_t* sm = ctx->smask.p + b * rstride;
    uint16_t* tab = ctx->tab.p + b * tstride;
    KeyDesc kr = kd;
    kr.n = nr;
    if (kd.offsets) kr.offsets = kd.offsets + r0;
    else kr.bytes = kd.bytes + r0 * kd.key_len;
    if (pipe && r >= static_cast<uint64_t>(nbuf)) DLSM_TRY(hipStreamWaitEvent(ps, ctx->ev_free[b], 0));
    DLSM_TRY(launch_probe_partition(kr, grp.L, grp.magic, R, S, ent, pos, tab, mode, lgC, ps,
                                    split ? ctx->pcus : 0u));
    if (pipe) DLSM_CHECK(hand_over(ps, s, ctx->ev_part[b]));
    if (split) DLSM_CHECK(join_part(ctx));
    DLSM_TRY(launch_probe_slices(grp.stacked, grp.L, grp.magic, grp.k, lgR, R, grp.lgw, grp.slotmap, S, nC, ent,
                                 tab, sm, slice_parts(S, nC, lgR), lgC, s));
    DLSM_TRY(launch_probe_unpermute(nr, pos, sm, mask_dev + r0, lgC, s));
    if (pipe) DLSM_TRY(hipEventRecord(ctx->ev_free[b], s));
  }
  return DLSM_OK;
}
}  // namespace

int dlsm_bloom_full_probe_dev(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* keys,
                              uint8_t* mask_dev) {
  return full_probe_dev_impl(ctx, fs, keys, mask_dev, false);
}

int dlsm_bloom_full_probe_hashed_dev(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* hashes,
                                     uint8_t* mask_dev) {
  return full_probe_dev_impl(ctx, fs, hashes, mask_dev, true);
}

int dlsm_bloom_full_probe(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* keys,
                          uint8_t* mask) {
  if (!ctx || !fs || !keys) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  DLSM_CHECK(validate_keyset(*keys));
  if (keys->n == 0) return DLSM_OK;
  if (!mask) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  const dlsm_keyset* sets[1] = {keys};
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets, 1, dk));
  const uint64_t mb = static_cast<uint64_t>((fs->F + 7) / 8) * keys->n;
  DLSM_CHECK(ctx->st_out.ensure(mb));
  DLSM_CHECK(dlsm_bloom_full_probe_dev(ctx, fs, &dk[0], ctx->st_out.p));
  DLSM_TRY(hipMemcpyAsync(mask, ctx->st_out.p, mb, hipMemcpyDeviceToHost, ctx->stream));
  DLSM_TRY(ctx_sync(ctx, ctx->stream));
  return DLSM_OK;
}

// ---------------------------------------------------------------------------
// Legacy block-based filter block (table/filter_block.cc), §8f row 4
// ---------------------------------------------------------------------------
namespace {
constexpr uint64_t kFilterBaseLg = 11;  // filter_block.cc:15-16: a filter every 2 KiB

// FilterBlockBuilder's filter groups for the StartBlock / AddKey sequence of a
// TableBuilder: keys of data block b, then StartBlock(block_end_offset[b])
// (TableBuilder::Flush); GenerateFilter takes every pending key (first loop
// turn) or none (later turns); Finish generates one more if keys are pending.
struct FilterGroups {
  std::vector<uint64_t> begin, end;  // key range per filter (empty allowed)
  std::vector<uint32_t> off;         // filter_offsets_
  uint64_t array_offset = 0;
  uint64_t total = 0;  // block length
};

int filter_groups(const uint64_t* block_key_end, const uint64_t* block_end_offset, int n_blocks,
                  uint64_t n_keys, int bits_per_key, FilterGroups& G) {
  if (n_blocks < 0 || (n_blocks > 0 && (!block_key_end || !block_end_offset))) return DLSM_E_ARG;
  uint64_t pending = 0, prev_end = 0, result = 0;
  auto generate = [&](uint64_t upto) {
    G.off.push_back(static_cast<uint32_t>(result));
    G.begin.push_back(pending);
    G.end.push_back(upto);
    if (upto > pending) result += legacy_bits(upto - pending, bits_per_key) / 8 + 1;  // CreateFilter
    pending = upto;
  };
  for (int b = 0; b < n_blocks; b++) {
    const uint64_t ke = block_key_end[b];
    if (ke < prev_end || ke > n_keys) return DLSM_E_ARG;
    prev_end = ke;
    const uint64_t index = block_end_offset[b] / (uint64_t(1) << kFilterBaseLg);
    if (index < G.off.size()) return DLSM_E_ARG;  // assert(filter_index >= filter_offsets_.size())
    while (index > G.off.size()) generate(ke);     // later turns: no pending keys -> empty
  }
  if (n_keys > pending) generate(n_keys);  // Finish: start_ not empty
  G.array_offset = result;
  G.total = result + 4 * G.off.size() + 4 + 1;
  if (G.array_offset > 0xffffffffull) return DLSM_E_ARG;  // Fixed32 offsets
  return DLSM_OK;
}
}  // namespace

int dlsm_filter_block_size(const uint64_t* block_key_end, const uint64_t* block_end_offset,
                           int n_blocks, uint64_t n_keys, int bits_per_key, uint64_t* nbytes) {
  if (!nbytes) return DLSM_E_ARG;
  FilterGroups G;
  DLSM_CHECK(filter_groups(block_key_end, block_end_offset, n_blocks, n_keys, bits_per_key, G));
  *nbytes = G.total;
  return DLSM_OK;
}

int dlsm_filter_block_build_dev(dlsm_ctx* ctx, const dlsm_keyset* keys, const uint64_t* block_key_end,
                                const uint64_t* block_end_offset, int n_blocks, int bits_per_key,
                                uint8_t* out_dev, uint64_t out_cap, uint64_t* out_len) {
  if (!ctx || !keys || !out_dev) return DLSM_E_ARG;
  DLSM_CHECK(validate_keyset(*keys));
  FilterGroups G;
  DLSM_CHECK(filter_groups(block_key_end, block_end_offset, n_blocks, keys->n, bits_per_key, G));
  if (out_len) *out_len = 0;
  if (G.total > out_cap) return DLSM_E_CAPACITY;
  DeviceGuard g(ctx->device);
  // one legacy CreateFilter job per non-empty group, written in place
  std::vector<dlsm_build_job> jobs;
  for (size_t f = 0; f < G.off.size(); f++) {
    if (G.end[f] == G.begin[f]) continue;
    dlsm_build_job j{};
    j.keys = *keys;
    j.keys.n = G.end[f] - G.begin[f];
    if (keys->offsets) j.keys.offsets = keys->offsets + G.begin[f];
    else j.keys.bytes = keys->bytes + G.begin[f] * keys->key_len;
    j.out = out_dev + G.off[f];
    j.out_cap = legacy_bits(j.keys.n, bits_per_key) / 8 + 1;
    jobs.push_back(j);
  }
  if (!jobs.empty()) {
    DLSM_CHECK(ctx->st_len.ensure(jobs.size()));
    DLSM_CHECK(dlsm_bloom_legacy_build_dev(ctx, jobs.data(), static_cast<int>(jobs.size()), bits_per_key,
                                           ctx->st_len.p));
  }
  // Finish: Fixed32 filter offsets, Fixed32 array offset, kFilterBaseLg
  std::vector<uint8_t> tail(G.total - G.array_offset);
  for (size_t f = 0; f < G.off.size(); f++) memcpy(&tail[4 * f], &G.off[f], 4);  // little-endian
  const uint32_t ao = static_cast<uint32_t>(G.array_offset);
  memcpy(&tail[4 * G.off.size()], &ao, 4);
  tail.back() = static_cast<uint8_t>(kFilterBaseLg);
  DLSM_TRY(hipMemcpyAsync(out_dev + G.array_offset, tail.data(), tail.size(), hipMemcpyHostToDevice,
                          ctx->stream));
  DLSM_TRY(ctx_sync(ctx, ctx->stream));  // `tail` is pageable host memory
  if (out_len) *out_len = G.total;
  return DLSM_OK;
}

int dlsm_filter_block_probe_dev(dlsm_ctx* ctx, const uint8_t* block_dev, uint64_t len,
                                const dlsm_keyset* keys, const uint64_t* block_offsets_dev,
                                uint8_t* out_dev) {
  if (!ctx || !keys) return DLSM_E_ARG;
  DLSM_CHECK(validate_keyset(*keys));
  if (keys->n == 0) return DLSM_OK;
  if (!out_dev || !block_offsets_dev || (len && !block_dev)) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  DLSM_TRY(launch_filter_block_probe(block_dev, len, to_desc(*keys), block_offsets_dev, out_dev, ctx->stream));
  return DLSM_OK;
}

int dlsm_filter_block_build(dlsm_ctx* ctx, const dlsm_keyset* keys, const uint64_t* block_key_end,
                            const uint64_t* block_end_offset, int n_blocks, int bits_per_key,
                            uint8_t* out, uint64_t out_cap, uint64_t* out_len) {
  if (!ctx || !keys || !out) return DLSM_E_ARG;
  DLSM_CHECK(validate_keyset(*keys));
  uint64_t need = 0;
  DLSM_CHECK(dlsm_filter_block_size(block_key_end, block_end_offset, n_blocks, keys->n, bits_per_key, &need));
  if (out_len) *out_len = 0;
  if (need > out_cap) return DLSM_E_CAPACITY;
  DeviceGuard g(ctx->device);
  const dlsm_keyset* sets[1] = {keys};
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets, 1, dk));
  DLSM_CHECK(ctx->st_out.ensure(need));
  uint64_t len = 0;
  DLSM_CHECK(dlsm_filter_block_build_dev(ctx, &dk[0], block_key_end, block_end_offset, n_blocks,
                                         bits_per_key, ctx->st_out.p, need, &len));
  DLSM_TRY(hipMemcpyAsync(out, ctx->st_out.p, len, hipMemcpyDeviceToHost, ctx->stream));
  DLSM_TRY(ctx_sync(ctx, ctx->stream));
  if (out_len) *out_len = len;
  return DLSM_OK;
}

int dlsm_filter_block_probe(dlsm_ctx* ctx, const uint8_t* block, uint64_t len, const dlsm_keyset* keys,
                            const uint64_t* block_offsets, uint8_t* out) {
  if (!ctx || !keys) return DLSM_E_ARG;
  DLSM_CHECK(validate_keyset(*keys));
  if (keys->n == 0) return DLSM_OK;
  if (!out || !block_offsets || (len && !block)) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  const dlsm_keyset* sets[1] = {keys};
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets, 1, dk));
  // staging: [block | offsets | answers]
  const uint64_t bo = (len + 15) & ~uint64_t(15);
  const uint64_t oo = bo + 8 * keys->n;
  DLSM_CHECK(ctx->st_out.ensure(oo + keys->n));
  if (len) DLSM_TRY(hipMemcpyAsync(ctx->st_out.p, block, len, hipMemcpyHostToDevice, s));
  DLSM_TRY(hipMemcpyAsync(ctx->st_out.p + bo, block_offsets, 8 * keys->n, hipMemcpyHostToDevice, s));
  DLSM_CHECK(dlsm_filter_block_probe_dev(ctx, len ? ctx->st_out.p : nullptr, len, &dk[0],
                                         reinterpret_cast<const uint64_t*>(ctx->st_out.p + bo),
                                         ctx->st_out.p + oo));
  DLSM_TRY(hipMemcpyAsync(out, ctx->st_out.p + oo, keys->n, hipMemcpyDeviceToHost, s));
  DLSM_TRY(ctx_sync(ctx, s));
  return DLSM_OK;
}

// ---------------------------------------------------------------------------
// Version: files + filters for the MultiGet-style probe (§8f row 3)
// ---------------------------------------------------------------------------
static_assert(DLSM_NUM_LEVELS == kNumLevels, "config::kNumLevels");

// A level probed by the sliced version probe: its filters' lines back to
// back in one image (`image`, `lines` lines of 64 B, one probe count `k`).
struct VersionLevel {
  int level = 0;
  int k = 0;
  uint32_t lines = 0;
  const uint8_t* image = nullptr;
};

struct dlsm_version {
  int device = 0;
  VersionDev v{};
  int n_files = 0;
  uint8_t* mem = nullptr;  // one allocation: files | key blob | filters (sliced levels: their images)
  std::vector<VersionLevel> sliced;
};

namespace {
// A level >= 1 goes to the sliced probe when its filters hold more than this
// many bytes and every filter of the level has 64-byte lines and one probe
// count.  Default 256 MiB, the Infinity Cache: below it the direct probe's
// line reads (four lanes per line, tasks queued per wave) are served on-die
// and beat a partition / slice / unpermute round per level -- the db_bench
// version (139.5 MB of filters) takes 4.0 ms direct against 5.4 ms with its
// two big levels sliced (profiles/r05_version_probe.txt).
// ($DLSM_VERSION_SLICE_MIN_BYTES overrides; 0 disables the sliced probe.)
// The sliced version probe measured slower than the direct one at both level
// sizes tried (db_bench's 125 MB level 3: 3.76 vs 3.48 ms per 100 M Gets; a
// 1.25 GB level 3: 11.1 vs 5.0 ms; profiles/r05_p_version_large.txt), so no
// level is sliced unless a caller asks ($DLSM_VERSION_SLICE_MIN_BYTES or
// DLSM_OPT_VERSION_SLICE_BYTES: levels whose filters exceed that many bytes).
uint64_t version_slice_min_bytes() {
  static const uint64_t v = [] {
    const char* e = getenv("DLSM_VERSION_SLICE_MIN_BYTES");
    return e ? strtoull(e, nullptr, 10) : uint64_t(0);
  }();
  return v;
}
}  // namespace

int dlsm_version_create(dlsm_ctx* ctx, const dlsm_version_file* files, int n_files,
                        int filters_are_device, dlsm_version** out) {
  if (!ctx || !out || n_files < 0 || (n_files > 0 && !files)) return DLSM_E_ARG;
  *out = nullptr;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  // search order: level 0 newest first (NewestFirst, version_set.cc:268-270),
  // then each level >= 1 in the caller's (key) order
  std::vector<int> order;
  int n_l0 = 0;
  uint32_t begin[kNumLevels] = {}, count[kNumLevels] = {};
  for (int f = 0; f < n_files; f++) {
    const dlsm_version_file& F = files[f];
    if (F.level < 0 || F.level >= kNumLevels) return DLSM_E_ARG;
    if ((F.smallest_len && !F.smallest_user_key) || (F.largest_len && !F.largest_user_key)) return DLSM_E_ARG;
    if (F.smallest_len > 0xffffffffull || F.largest_len > 0xffffffffull) return DLSM_E_ARG;
    if (F.level == 0) n_l0++;
  }
  if (n_l0 > 64 - (kNumLevels - 1)) return DLSM_E_ARG;
  for (int f = 0; f < n_files; f++)
    if (files[f].level == 0) order.push_back(f);
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return files[a].number > files[b].number; });
  for (int lv = 1; lv < kNumLevels; lv++) {
    begin[lv] = static_cast<uint32_t>(order.size());
    for (int f = 0; f < n_files; f++)
      if (files[f].level == lv) order.push_back(f);
    count[lv] = static_cast<uint32_t>(order.size()) - begin[lv];
  }
  // layout: VFileDev[n] | key blob | filters (each 256-B aligned)
  std::vector<VFileDev> h(n_files);
  std::vector<uint8_t> keys;
  std::vector<uint64_t> foff(n_files, 0);
  const uint64_t files_bytes = (sizeof(VFileDev) * n_files + 255) & ~uint64_t(255);
  for (int j = 0; j < n_files; j++) {
    const dlsm_version_file& F = files[order[j]];
    VFileDev& d = h[j];
    d.smallest_off = keys.size();
    d.smallest_len = static_cast<uint32_t>(F.smallest_len);
    keys.insert(keys.end(), F.smallest_user_key, F.smallest_user_key + F.smallest_len);
    d.largest_off = keys.size();
    d.largest_len = static_cast<uint32_t>(F.largest_len);
    keys.insert(keys.end(), F.largest_user_key, F.largest_user_key + F.largest_len);
    d.largest_trailer = F.largest_trailer;
    d.f = FilterDev{};
  }
  // 16-byte big-endian key prefixes (VersionDev::pre_small / pre_large)
  std::vector<ulonglong2> pre(2 * static_cast<size_t>(n_files));
  auto be_prefix = [](const uint8_t* p, uint64_t n) {
    ulonglong2 r{0, 0};
    for (uint64_t i = 0; i < 16 && i < n; i++) {
      if (i < 8) r.x |= static_cast<uint64_t>(p[i]) << (56 - 8 * i);
      else r.y |= static_cast<uint64_t>(p[i]) << (56 - 8 * (i - 8));
    }
    return r;
  };
  for (int j = 0; j < n_files; j++) {
    pre[j] = be_prefix(keys.data() + h[j].smallest_off, h[j].smallest_len);
    pre[n_files + j] = be_prefix(keys.data() + h[j].largest_off, h[j].largest_len);
  }
  const uint64_t pre_bytes = (sizeof(ulonglong2) * pre.size() + 255) & ~uint64_t(255);
  const uint64_t keys_bytes = (keys.size() + 255) & ~uint64_t(255);
  // The interval index (VIntervalDev): the distinct bound prefixes in order,
  // and per open interval between two of them the level-0 files that hold
  // it and each level's FindFile pick.  For a lookup prefix strictly between
  // bnd[j-1] and bnd[j]: a bound with prefix index < j sorts below the lookup,
  // one with index >= j above it.
  auto pre_lt = [](const ulonglong2& a, const ulonglong2& b) { return a.x < b.x || (a.x == b.x && a.y < b.y); };
  std::vector<ulonglong2> bnd(pre);
  std::sort(bnd.begin(), bnd.end(), pre_lt);
  bnd.erase(std::unique(bnd.begin(), bnd.end(),
                        [](const ulonglong2& a, const ulonglong2& b) { return a.x == b.x && a.y == b.y; }),
            bnd.end());
  auto bidx = [&](const ulonglong2& p) {
    return static_cast<uint32_t>(std::lower_bound(bnd.begin(), bnd.end(), p, pre_lt) - bnd.begin());
  };
  std::vector<uint32_t> is(n_files), il(n_files);
  for (int j = 0; j < n_files; j++) {
    is[j] = bidx(pre[j]);
    il[j] = bidx(pre[n_files + j]);
  }
  const uint32_t n_bnd = static_cast<uint32_t>(bnd.size());
  std::vector<VIntervalDev> ivl(n_bnd + 1);
  // FindFile's pick per level as a two-pointer sweep: right(j) = the first
  // file r < count-1 whose largest has prefix index >= j (else count-1); the
  // set of such r only shrinks as j grows, so right(j) never decreases and
  // each level is walked once over all j (O(n_bnd + files), not O(n_bnd x
  // files): a 60,000-file level took seconds per version before).
  uint32_t rgt[kNumLevels] = {};
  for (uint32_t j = 0; j <= n_bnd; j++) {
    VIntervalDev& r = ivl[j];
    r.l0mask = 0;
    r.reserved[0] = r.reserved[1] = r.reserved[2] = 0;
    for (int f = 0; f < n_l0; f++)  // smallest <= lookup <= largest
      if (is[f] < j && il[f] >= j) r.l0mask |= 1ull << f;
    for (int lv = 1; lv < kNumLevels; lv++) {
      r.pick[lv - 1] = 0xffffu;
      if (!count[lv] || begin[lv] + count[lv] > 0xffffu) continue;  // (> 65,535 files: never read)
      // FindFile (version_set.cc:95-118): files [0, count-1) whose largest
      // sorts below the lookup come first; right starts at count-1
      uint32_t& right = rgt[lv];
      while (right < count[lv] - 1 && il[begin[lv] + right] < j) right++;
      if (is[begin[lv] + right] < j) r.pick[lv - 1] = static_cast<uint16_t>(begin[lv] + right);
    }
  }
  const uint64_t bnd_bytes = (sizeof(ulonglong2) * std::max<size_t>(1, bnd.size()) + 255) & ~uint64_t(255);
  const uint64_t ivl_bytes = (sizeof(VIntervalDev) * ivl.size() + 255) & ~uint64_t(255);
  uint64_t total = files_bytes + pre_bytes + keys_bytes + bnd_bytes + ivl_bytes;
  for (int j = 0; j < n_files; j++) {
    const dlsm_version_file& F = files[order[j]];
    if (!F.filter) continue;
    if (F.filter_len < 5) return DLSM_E_CORRUPT;
    uint8_t tail[5];
    if (filters_are_device) {
      DLSM_TRY(hipMemcpyAsync(tail, F.filter + F.filter_len - 5, 5, hipMemcpyDeviceToHost, s));
      DLSM_TRY(ctx_sync(ctx, s));
    } else {
      memcpy(tail, F.filter + F.filter_len - 5, 5);
    }
    int k, lg;
    uint32_t L;
    DLSM_CHECK(parse_tail(tail, F.filter_len, &k, &L, &lg));
    h[j].f.L = L;
    h[j].f.magic = fastmod_magic(L);
    h[j].f.k = k;
    h[j].f.lg = lg;
  }
  // Levels for the sliced probe; their filters' lines are laid out back to
  // back (line0 per file), the other filters one by one, 256-byte aligned.
  std::vector<VersionLevel> sliced;
  int32_t lvl_sliced[kNumLevels];
  std::vector<uint64_t> copy_len(n_files, 0);
  for (int lv = 0; lv < kNumLevels; lv++) lvl_sliced[lv] = -1;
  const uint64_t min_bytes = ctx->vslice_bytes == 0 ? version_slice_min_bytes()
                             : (ctx->vslice_bytes == UINT64_MAX ? 0 : ctx->vslice_bytes);
  for (int lv = 1; lv < kNumLevels && min_bytes; lv++) {
    uint64_t lines = 0;
    int k = 0;
    bool ok = true;
    for (uint32_t j = begin[lv]; j < begin[lv] + count[lv]; j++) {
      if (!files[order[j]].filter) continue;
      ok = ok && h[j].f.lg == 6 && (k == 0 || h[j].f.k == k);
      k = h[j].f.k;
      lines += h[j].f.L;
    }
    if (!ok || lines * 64 <= min_bytes || lines >= kVNoLine) continue;
    lvl_sliced[lv] = static_cast<int32_t>(sliced.size());
    VersionLevel vl;
    vl.level = lv;
    vl.k = k;
    vl.lines = static_cast<uint32_t>(lines);
    sliced.push_back(vl);
  }
  std::vector<uint64_t> image_off(sliced.size(), 0);
  for (size_t q = 0; q < sliced.size(); q++) {
    const int lv = sliced[q].level;
    image_off[q] = total;
    uint32_t line0 = 0;
    for (uint32_t j = begin[lv]; j < begin[lv] + count[lv]; j++) {
      if (!files[order[j]].filter) continue;
      h[j].line0 = line0;
      foff[j] = total + static_cast<uint64_t>(line0) * 64;
      copy_len[j] = static_cast<uint64_t>(h[j].f.L) * 64;  // the lines; the trailer was parsed above
      line0 += h[j].f.L;
    }
    total += (static_cast<uint64_t>(sliced[q].lines) * 64 + 255) & ~uint64_t(255);
  }
  for (int j = 0; j < n_files; j++) {
    const dlsm_version_file& F = files[order[j]];
    if (!F.filter || copy_len[j]) continue;
    foff[j] = total;
    copy_len[j] = F.filter_len;
    total += (F.filter_len + 255) & ~uint64_t(255);
  }
  dlsm_version* ver = new (std::nothrow) dlsm_version();
  if (!ver) return DLSM_E_NOMEM;
  ver->device = ctx->device;
  ver->n_files = n_files;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&ver->mem), std::max<uint64_t>(total, 256));
  for (int j = 0; j < n_files && e == hipSuccess; j++) {
    const dlsm_version_file& F = files[order[j]];
    if (!F.filter) continue;
    h[j].f.data = ver->mem + foff[j];
    e = hipMemcpyAsync(ver->mem + foff[j], F.filter, copy_len[j],
                       filters_are_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s);
  }
  for (size_t q = 0; q < sliced.size(); q++) sliced[q].image = ver->mem + image_off[q];
  ver->sliced = sliced;
  if (e == hipSuccess && n_files)
    e = hipMemcpyAsync(ver->mem, h.data(), sizeof(VFileDev) * n_files, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n_files)
    e = hipMemcpyAsync(ver->mem + files_bytes, pre.data(), sizeof(ulonglong2) * pre.size(),
                       hipMemcpyHostToDevice, s);
  if (e == hipSuccess && !keys.empty())
    e = hipMemcpyAsync(ver->mem + files_bytes + pre_bytes, keys.data(), keys.size(), hipMemcpyHostToDevice, s);
  const uint64_t bnd_off = files_bytes + pre_bytes + keys_bytes;
  if (e == hipSuccess && !bnd.empty())
    e = hipMemcpyAsync(ver->mem + bnd_off, bnd.data(), sizeof(ulonglong2) * bnd.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(ver->mem + bnd_off + bnd_bytes, ivl.data(), sizeof(VIntervalDev) * ivl.size(),
                       hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // pageable sources: finish before returning
  if (e != hipSuccess) {
    dlsm_version_destroy(ver);
    return from_hip(e);
  }
  ver->v.files = reinterpret_cast<const VFileDev*>(ver->mem);
  ver->v.pre_small = reinterpret_cast<const ulonglong2*>(ver->mem + files_bytes);
  ver->v.pre_large = ver->v.pre_small + n_files;
  ver->v.keyblob = ver->mem + files_bytes + pre_bytes;
  ver->v.bnd = reinterpret_cast<const ulonglong2*>(ver->mem + bnd_off);
  ver->v.ivl = reinterpret_cast<const VIntervalDev*>(ver->mem + bnd_off + bnd_bytes);
  ver->v.n_bnd = n_bnd;
  ver->v.k_all = 0;
  {
    int kc = 0;
    bool same = true;
    for (int j = 0; j < n_files; j++) {
      if (!files[order[j]].filter) continue;
      same = same && (kc == 0 || h[j].f.k == kc);
      kc = h[j].f.k;
    }
    ver->v.k_all = same ? kc : 0;
  }
  ver->v.n_l0 = static_cast<uint32_t>(n_l0);
  for (int lv = 0; lv < kNumLevels; lv++) {
    ver->v.lvl_begin[lv] = begin[lv];
    ver->v.lvl_count[lv] = count[lv];
    ver->v.lvl_sliced[lv] = lvl_sliced[lv];
  }
  *out = ver;
  return DLSM_OK;
}

int dlsm_version_destroy(dlsm_version* v) {
  if (!v) return DLSM_OK;
  DeviceGuard g(v->device);
  if (v->mem) (void)hipFree(v->mem);
  delete v;
  return DLSM_OK;
}

int dlsm_version_slots(const dlsm_version* v, int* n_l0, int* n_slots) {
  if (!v) return DLSM_E_ARG;
  if (n_l0) *n_l0 = static_cast<int>(v->v.n_l0);
  if (n_slots) *n_slots = static_cast<int>(v->v.n_l0) + kNumLevels - 1;
  return DLSM_OK;
}

int dlsm_version_probe_dev(dlsm_ctx* ctx, const dlsm_version* v, const dlsm_keyset* keys,
                           uint64_t snapshot, uint64_t* slot_mask_dev, uint32_t* level_file_dev) {
  if (!ctx || !v || !keys) return DLSM_E_ARG;
  if (v->device != ctx->device) return DLSM_E_ARG;
  if (snapshot > ((uint64_t(1) << 56) - 1)) return DLSM_E_ARG;  // kMaxSequenceNumber
  DLSM_CHECK(validate_keyset(*keys));
  if (keys->n == 0) return DLSM_OK;
  if (!slot_mask_dev) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  const KeyDesc kd = to_desc(*keys);
  if (v->sliced.empty() || ctx->path == 1) {
    // every level probed directly: one thread per lookup, filter lines read
    // where they lie (the L2-resident shape)
    VersionDev vd = v->v;
    for (int lv = 0; lv < kNumLevels; lv++) vd.lvl_sliced[lv] = -1;
    DLSM_TRY(launch_version_probe(vd, kd, snapshot, slot_mask_dev, level_file_dev, s));
    return DLSM_OK;
  }
  // Sliced: a route pass (the direct levels answered, each sliced level's
  // global line per lookup), then per sliced level and group of up to
  // kVMaxSlices slices a partition / LDS slice / unpermute round.
  const uint64_t n = keys->n;
  const int J = static_cast<int>(v->sliced.size());
  const uint32_t nC = ceil_div_u32(n, kVChunk);
  const uint64_t span = static_cast<uint64_t>(ctx->vpass_slices) << kVSliceLg;
  struct Pass {
    int j;
    uint32_t g0, S, L;
  };
  std::vector<Pass> passes;
  uint32_t Smax = 1;
  for (int j = 0; j < J; j++)
    for (uint64_t g0 = 0; g0 < v->sliced[j].lines; g0 += span) {
      const uint32_t L = static_cast<uint32_t>(std::min<uint64_t>(v->sliced[j].lines - g0, span));
      const uint32_t S = ceil_div_u32(L, 1u << kVSliceLg);
      passes.push_back(Pass{j, static_cast<uint32_t>(g0), S, L});
      Smax = std::max(Smax, S);
    }
  uint64_t slots = 0;
  for (int j = 0; j < J; j++) slots |= static_cast<uint64_t>(v->v.n_l0 + v->sliced[j].level - 1) << (8 * j);
  DLSM_CHECK(ctx->hashes.ensure(n));
  DLSM_CHECK(ctx->vgl.ensure(static_cast<uint64_t>(J) * n));
  DLSM_CHECK(ctx->entries.ensure(static_cast<uint64_t>(nC) * kVRegion));
  DLSM_CHECK(ctx->smask.ensure(static_cast<uint64_t>(nC) * kVRegion));
  DLSM_CHECK(ctx->pos.ensure(static_cast<uint64_t>(nC) * kVChunk));
  DLSM_CHECK(ctx->tab.ensure(static_cast<uint64_t>(nC) * (Smax + 1)));
  if (passes.size() > 1) DLSM_CHECK(ctx->vabyte.ensure(n));
  DLSM_CHECK(ctx->vplan.ensure(2 * (kVMaxSlices + 1)));
  uint32_t* gcnt = ctx->vplan.p;
  uint32_t* plan = ctx->vplan.p + kVMaxSlices + 1;
  if (ctx->vplan_zeroed != ctx->vplan.gen) {  // the plan kernel re-zeroes the counters after every pass
    DLSM_TRY(hipMemsetAsync(gcnt, 0, sizeof(uint32_t) * (kVMaxSlices + 1), s));
    ctx->vplan_zeroed = ctx->vplan.gen;
  }
  DLSM_TRY(launch_version_route(v->v, kd, snapshot, slot_mask_dev, level_file_dev, ctx->hashes.p, ctx->vgl.p, s));
  for (size_t p = 0; p < passes.size(); p++) {
    const Pass& P = passes[p];
    const VersionLevel& VL = v->sliced[P.j];
    DLSM_TRY(launch_version_partition(ctx->hashes.p, ctx->vgl.p + static_cast<uint64_t>(P.j) * n, n, P.g0, P.S,
                                      ctx->entries.p, ctx->pos.p, ctx->tab.p, gcnt, plan, s));
    DLSM_TRY(launch_version_slices(VL.image + static_cast<uint64_t>(P.g0) * 64, P.L, VL.k, P.S, nC,
                                   ctx->entries.p, ctx->tab.p, ctx->smask.p, plan, s));
    DLSM_TRY(launch_version_unpermute(n, ctx->pos.p, ctx->smask.p, ctx->vabyte.p, slot_mask_dev, P.j, J, slots,
                                      p == 0, p + 1 == passes.size(), s));
  }
  return DLSM_OK;
}

// ---------------------------------------------------------------------------
// Legacy FilterPolicy format (util/bloom.cc)
// ---------------------------------------------------------------------------
namespace {
// Tiles per legacy slice workgroup (log2): 16 (128 KiB of LDS, one workgroup
// per CU) unless the batch then has fewer slices than the chip has CUs.
int choose_legacy_tps_lg(const std::vector<uint32_t>& n_tiles) {
  if (const char* e = getenv("DLSM_LEGACY_TPS_LG")) {
    const int v = atoi(e);
    if (v >= 0 && v <= 4) return v;
  }
  int lg = 4;
  for (; lg > 0; lg--) {
    uint64_t total = 0;
    for (uint32_t t : n_tiles) total += (t + (1u << lg) - 1) >> lg;
    if (total >= kBuildSliceCUs) break;
  }
  return lg;
}
}  // namespace

int dlsm_bloom_legacy_build_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                int bits_per_key, uint64_t* out_len_dev) {
  if (!ctx || n_jobs < 0 || (n_jobs > 0 && (!jobs || !out_len_dev))) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  if (n_jobs == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  const int k = legacy_num_probes(bits_per_key);
  bool all_k20 = true, all_k28 = true;
  bool fits_a = k <= kLegacyKmaxA, fits_b = k <= kLegacyKmaxB;
  uint64_t ws = 0, total = 0;
  std::vector<uint64_t> wpos(n_jobs), lens(n_jobs);
  std::vector<uint32_t> tiles(n_jobs), regions(n_jobs);
  for (int j = 0; j < n_jobs; j++) {
    DLSM_CHECK(validate_keyset(jobs[j].keys));
    if (!jobs[j].out) return DLSM_E_ARG;
    const uint64_t bits = legacy_bits(jobs[j].keys.n, bits_per_key);
    lens[j] = bits / 8 + 1;
    if (lens[j] > jobs[j].out_cap) return DLSM_E_CAPACITY;
    wpos[j] = ws;
    ws += (bits / 8 + 3 + 255) & ~uint64_t(255);
    all_k20 = all_k20 && is_k20(jobs[j].keys);
    all_k28 = all_k28 && is_k28(jobs[j].keys);
    // the LDS-tiled path: positions as u16 inside 2^16-bit tiles, one chunk's
    // region (k positions per key + up to 7 pads per tile) staged in LDS
    const uint64_t nt = (bits + (uint64_t(1) << kLegacyTileLg) - 1) >> kLegacyTileLg;
    const uint64_t reg = (static_cast<uint64_t>(k) * kLegacyChunk + 7 * nt + 7) & ~uint64_t(7);
    tiles[j] = static_cast<uint32_t>(std::min<uint64_t>(nt, 0xffffffffu));
    regions[j] = static_cast<uint32_t>(std::min<uint64_t>(reg, 0xffffffffu));
    const bool ok = bits <= 0xffffffffull && jobs[j].keys.n <= 0x7fffffffull * kLegacyChunk;
    fits_a = fits_a && ok && nt <= kLegacyTilesA && reg <= kLegacyStageA;
    fits_b = fits_b && ok && nt <= kLegacyTilesB && reg <= kLegacyStageB;
  }
  const int mode = all_k20 ? KM_K20 : (all_k28 ? KM_K28 : KM_GENERIC);
  if (ctx->path != 1 && fits_b) {
    const int tps_lg = choose_legacy_tps_lg(tiles);
    std::vector<LegacyTileJobDev> hj(n_jobs);
    std::vector<uint32_t> starts(2 * n_jobs);
    uint64_t entry = 0, tabw = 0;
    uint32_t chunk = 0, slice = 0;
    for (int j = 0; j < n_jobs; j++) {
      LegacyTileJobDev& d = hj[j];
      const uint64_t bits = legacy_bits(jobs[j].keys.n, bits_per_key);
      d.keys = to_desc(jobs[j].keys);
      d.out = jobs[j].out;
      d.out_len = out_len_dev + j;
      d.entry0 = entry;
      d.tab0 = tabw;
      d.bits = static_cast<uint32_t>(bits);
      d.magic = fastmod_magic(d.bits);
      d.n_tiles = tiles[j];
      d.region = regions[j];
      d.n_chunks = ceil_div_u32(jobs[j].keys.n, kLegacyChunk);
      d.chunk0 = chunk;
      d.n_slices = (tiles[j] + (1u << tps_lg) - 1) >> tps_lg;
      d.slice0 = slice;
      d.k = k;
      d.reserved = 0;
      starts[j] = chunk;
      starts[n_jobs + j] = slice;
      entry += static_cast<uint64_t>(d.n_chunks) * d.region;
      tabw += static_cast<uint64_t>(d.n_chunks) * (d.n_tiles + 1);
      chunk += d.n_chunks;
      slice += d.n_slices;
    }
    DLSM_CHECK(ctx->ltjobs.ensure(n_jobs));
    DLSM_CHECK(ctx->ltstarts.ensure(2 * n_jobs));
    DLSM_CHECK(ctx->lentries.ensure(entry + 8));
    DLSM_CHECK(ctx->ltab.ensure(tabw + 1));
    DLSM_CHECK(ctx_upload(ctx, ctx->ltjobs.p, hj.data(), sizeof(LegacyTileJobDev) * n_jobs, s));
    DLSM_CHECK(ctx_upload(ctx, ctx->ltstarts.p, starts.data(), sizeof(uint32_t) * 2 * n_jobs, s));
    DLSM_TRY(launch_legacy_partition(ctx->ltjobs.p, ctx->ltstarts.p, n_jobs, chunk, ctx->lentries.p, ctx->ltab.p,
                                     fits_a ? 0 : 1, mode, s));
    DLSM_TRY(launch_legacy_slices(ctx->ltjobs.p, ctx->ltstarts.p + n_jobs, n_jobs, slice, ctx->lentries.p,
                                  ctx->ltab.p, tps_lg, s));
    return DLSM_OK;
  }
  // path 2 (sliced forced) with a batch the tiled kernels cannot take
  // (k > kLegacyKmaxB, i.e. bits_per_key >= 14, or too many tiles): the
  // direct kernel builds it -- the same bytes
  // Direct path: global atomics into an aligned workspace, then copies to the slots.
  DLSM_CHECK(ctx->st_filter.ensure(ws + 256));
  DLSM_TRY(hipMemsetAsync(ctx->st_filter.p, 0, ws, s));
  for (int j0 = 0; j0 < n_jobs; j0 += 256) {
    const int nj = std::min(256, n_jobs - j0);
    std::vector<LegacyJobDev> hj(nj);
    std::vector<uint64_t> key0s(nj);
    uint64_t tk = 0;
    for (int q = 0; q < nj; q++) {
      const dlsm_build_job& b = jobs[j0 + q];
      LegacyJobDev& d = hj[q];
      d.keys = to_desc(b.keys);
      d.out = ctx->st_filter.p + wpos[j0 + q];
      d.bits = legacy_bits(b.keys.n, bits_per_key);
      d.magic = d.bits <= 0xffffffffull ? fastmod_magic(static_cast<uint32_t>(d.bits)) : 0;
      d.k = k;
      d.key0 = tk;
      key0s[q] = tk;
      tk += b.keys.n;
    }
    total += tk;
    DLSM_CHECK(ctx->ljobs.ensure(nj));
    DLSM_CHECK(ctx->lstarts.ensure(nj));
    DLSM_CHECK(ctx_upload(ctx, ctx->ljobs.p, hj.data(), sizeof(LegacyJobDev) * nj, s));
    DLSM_CHECK(ctx_upload(ctx, ctx->lstarts.p, key0s.data(), sizeof(uint64_t) * nj, s));
    DLSM_TRY(launch_legacy_scatter(ctx->ljobs.p, ctx->lstarts.p, nj, tk, mode == KM_K20 ? KM_K20 : KM_GENERIC, s));
    // the job table is reused by the next group: keep the stream ordered
  }
  for (int j = 0; j < n_jobs; j++) {
    DLSM_TRY(hipMemcpyAsync(jobs[j].out, ctx->st_filter.p + wpos[j], lens[j] - 1,
                            hipMemcpyDeviceToDevice, s));
    DLSM_TRY(hipMemsetAsync(jobs[j].out + lens[j] - 1, static_cast<int>(static_cast<uint8_t>(k)), 1, s));
  }
  DLSM_CHECK(ctx_upload(ctx, out_len_dev, lens.data(), sizeof(uint64_t) * n_jobs, s));
  (void)total;
  return DLSM_OK;
}

int dlsm_bloom_legacy_build(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs, int bits_per_key,
                            uint64_t* out_len) {
  if (!ctx || n_jobs < 0 || (n_jobs > 0 && (!jobs || !out_len))) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  if (n_jobs == 0) return DLSM_OK;
  DeviceGuard g(ctx->device);
  std::vector<const dlsm_keyset*> sets(n_jobs);
  for (int j = 0; j < n_jobs; j++) {
    DLSM_CHECK(validate_keyset(jobs[j].keys));
    if (!jobs[j].out) return DLSM_E_ARG;
    const uint64_t len = legacy_bits(jobs[j].keys.n, bits_per_key) / 8 + 1;
    if (len > jobs[j].out_cap) return DLSM_E_CAPACITY;
    sets[j] = &jobs[j].keys;
  }
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets.data(), n_jobs, dk));
  std::vector<dlsm_build_job> dj(n_jobs);
  std::vector<uint64_t> opos(n_jobs);
  uint64_t ob = 0;
  for (int j = 0; j < n_jobs; j++) {
    const uint64_t len = legacy_bits(jobs[j].keys.n, bits_per_key) / 8 + 1;
    opos[j] = ob;
    ob += (len + 255) & ~uint64_t(255);
    dj[j].keys = dk[j];
    dj[j].out_cap = len;
  }
  DLSM_CHECK(ctx->st_out.ensure(ob + 256));
  DLSM_CHECK(ctx->st_len.ensure(n_jobs));
  for (int j = 0; j < n_jobs; j++) dj[j].out = ctx->st_out.p + opos[j];
  DLSM_CHECK(dlsm_bloom_legacy_build_dev(ctx, dj.data(), n_jobs, bits_per_key, ctx->st_len.p));
  hipStream_t s = ctx->stream;
  for (int j = 0; j < n_jobs; j++) {
    out_len[j] = dj[j].out_cap;
    DLSM_TRY(hipMemcpyAsync(jobs[j].out, dj[j].out, out_len[j], hipMemcpyDeviceToHost, s));
  }
  DLSM_TRY(ctx_sync(ctx, s));
  return DLSM_OK;
}

int dlsm_bloom_legacy_probe_dev(dlsm_ctx* ctx, const uint8_t* filter_dev, uint64_t len,
                                const dlsm_keyset* keys, uint8_t* out_dev) {
  if (!ctx || !keys) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  DLSM_CHECK(validate_keyset(*keys));
  if (keys->n == 0) return DLSM_OK;
  if (!out_dev) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  // util/bloom.cc:57-81: len < 2 -> false; k (signed char -> size_t) > 30 -> true.
  int trivial = 0, k = 0;
  uint64_t bits = 0;
  if (len < 2 || !filter_dev) {
    trivial = 1;
  } else {
    uint8_t kb;
    DLSM_TRY(hipMemcpyAsync(&kb, filter_dev + len - 1, 1, hipMemcpyDeviceToHost, s));
    DLSM_TRY(ctx_sync(ctx, s));
    const int ks = static_cast<int>(static_cast<int8_t>(kb));
    if (ks < 0 || ks > 30) trivial = 2;
    else if (ks == 0) trivial = 2;  // zero probes -> match
    k = ks;
    bits = (len - 1) * 8;
  }
  const uint32_t magic = (bits && bits <= 0xffffffffull) ? fastmod_magic(static_cast<uint32_t>(bits)) : 0;
  const int mode = is_k20(*keys) ? KM_K20 : KM_GENERIC;
  DLSM_TRY(launch_legacy_probe(filter_dev, bits, magic, k, trivial, to_desc(*keys), out_dev, mode, s));
  return DLSM_OK;
}

int dlsm_bloom_legacy_probe(dlsm_ctx* ctx, const uint8_t* filter, uint64_t len,
                            const dlsm_keyset* keys, uint8_t* out) {
  if (!ctx || !keys) return DLSM_E_ARG;
  if (ctx->fault) return -ctx->fault;
  DLSM_CHECK(validate_keyset(*keys));
  if (keys->n == 0) return DLSM_OK;
  if (!out) return DLSM_E_ARG;
  DeviceGuard g(ctx->device);
  hipStream_t s = ctx->stream;
  const dlsm_keyset* sets[1] = {keys};
  std::vector<dlsm_keyset> dk;
  DLSM_CHECK(stage_keys(ctx, sets, 1, dk));
  const uint8_t* fdev = nullptr;
  if (filter && len) {
    DLSM_CHECK(ctx->st_filter.ensure(len));
    DLSM_TRY(hipMemcpyAsync(ctx->st_filter.p, filter, len, hipMemcpyHostToDevice, s));
    fdev = ctx->st_filter.p;
  }
  DLSM_CHECK(ctx->st_out.ensure(keys->n));
  DLSM_CHECK(dlsm_bloom_legacy_probe_dev(ctx, fdev, len, &dk[0], ctx->st_out.p));
  DLSM_TRY(hipMemcpyAsync(out, ctx->st_out.p, keys->n, hipMemcpyDeviceToHost, s));
  DLSM_TRY(ctx_sync(ctx, s));
  return DLSM_OK;
}

}  // extern "C"
