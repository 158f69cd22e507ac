/*
 * dlsm_bloom.h -- C ABI of the MI355X-native SSTable Bloom-filter engine.
 *
 * Drop-in boundary for dLSM's (TimberSaw) filter hot path.  Plain C types
 * only: pointers, sizes, status codes.  No exceptions cross this boundary
 * (the reference builds with -fno-exceptions, CMakeLists.txt:79-81).
 *
 * Reference interfaces replaced (file:line in ruihong123/dLSM):
 *   BloomHash                      include/TimberSaw/filter_policy.h:26-28
 *   FullFilterBlockBuilder         table/full_filter_block.h:33-70,
 *       AddKey/Finish              table/full_filter_block.cc:39-141
 *   FullFilterBlockReader          table/full_filter_block.h:71-94,
 *       ctor / KeyMayMatch         table/full_filter_block.cc:186-284
 *   FilterPolicy / BloomFilterPolicy include/TimberSaw/filter_policy.h:31-71,
 *       CreateFilter/KeyMayMatch   util/bloom.cc:25-81
 * See INTEGRATION.md for the reference-side binding.
 *
 * Output format: byte-identical to the reference on the same inputs.  The
 * reference ORs bits into caller-zeroed RDMA slots (full_filter_block.cc:99-108
 * after table_builder_computeside.cc:38,48); this library writes every byte of
 * the filter (zeros included), so the result equals the reference's on a
 * zeroed slot, which every reference caller guarantees.
 *
 * Memory: functions suffixed _dev take DEVICE pointers (keys, offsets, output
 * slots, masks) and are asynchronous on the context's stream.  Unsuffixed
 * functions take HOST pointers, stage through device memory, and return after
 * the result is in the host buffer (the reference's synchronous call shape).
 */
#ifndef DLSM_BLOOM_H_
#define DLSM_BLOOM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLSM_BLOOM_ABI_VERSION 1

/* Status codes (full_filter_block.cc:192-249 exit(1)s become DLSM_E_CORRUPT). */
#define DLSM_OK 0
#define DLSM_E_ARG (-1)      /* bad argument / unsupported shape */
#define DLSM_E_CAPACITY (-2) /* output slot too small (the reference only asserts, :103) */
#define DLSM_E_CORRUPT (-3)  /* filter metadata the reference rejects or cannot probe */
#define DLSM_E_DEVICE (-4)   /* HIP runtime error */
#define DLSM_E_NOMEM (-5)    /* device allocation failed */
#define DLSM_E_BUSY (-6)     /* the context's host staging buffer is held by another user */

typedef struct dlsm_ctx dlsm_ctx;             /* one device + one stream + workspace */
typedef struct dlsm_filterset dlsm_filterset; /* F parsed full filters resident on a device */

/* A packed key set.  Fixed-length keys: offsets == NULL and every key is
 * key_len bytes at bytes + i*key_len.  Variable-length keys: offsets has n+1
 * entries and key i is bytes[offsets[i], offsets[i+1]).
 *
 * The reference hashes user keys (ExtractUserKey, db/dbformat.h:374-377, as
 * table_builder_computeside.cc:222-224 and InternalFilterPolicy,
 * db/dbformat.cc:93-109, do).  suffix_len = 0: the keys are user keys, hashed
 * as given.  suffix_len = DLSM_INTERNAL_KEY_TRAILER (8): the keys are internal
 * keys (user key || Fixed64(sequence << 8 | type)) straight from a memtable or
 * compaction iterator, and every build / probe hashes ExtractUserKey(key).
 * Fixed-length keys need key_len >= suffix_len; a variable-length key shorter
 * than suffix_len (the reference asserts) hashes as the empty user key. */
#define DLSM_INTERNAL_KEY_TRAILER 8
typedef struct {
  const uint8_t* bytes;
  const uint64_t* offsets;
  uint32_t key_len;
  uint32_t suffix_len;
  uint64_t n;
} dlsm_keyset;

/* One SSTable's filter: its keys in table order and its output slot. */
typedef struct {
  dlsm_keyset keys;
  uint8_t* out;     /* output slot (16-byte aligned for the _dev calls) */
  uint64_t out_cap; /* slot capacity in bytes */
} dlsm_build_job;

/* ---- host-only helpers (no device touched) ------------------------------ */

const char* dlsm_strerror(int status);
int dlsm_abi_version(void);

/* BloomHash(key) = Hash(key, n, 0xbc9f1d34); util/hash.cc:22-62 and
 * include/TimberSaw/filter_policy.h:26-28 (tail bytes sign-extended). */
uint32_t dlsm_bloom_hash(const void* key, size_t n);

/* ChooseNumProbes: util/bloom_impl.h:351-357 (full filter, via
 * full_filter_block.cc:19). */
int dlsm_bloom_full_num_probes(int bits_per_key);

/* CalculateSpace for n_dedup consecutive-distinct hashes:
 * table/full_filter_block.cc:61-92.  nbytes = num_lines*64 + 5. */
int dlsm_bloom_full_size(uint64_t n_dedup, int bits_per_key, uint32_t* num_lines,
                         uint64_t* nbytes);

/* BloomFilterPolicy::CreateFilter output size (bytes + the k byte):
 * util/bloom.cc:27-34,53-54. */
int dlsm_bloom_legacy_size(uint64_t n, int bits_per_key, uint64_t* nbytes);

/* FullFilterBlockReader ctor metadata parse: table/full_filter_block.cc:186-252.
 * Returns DLSM_E_CORRUPT where the reference exit(1)s, and also for filters the
 * reference accepts but cannot probe without undefined behaviour (<= 5 bytes:
 * h % 0).  log2_line is 6 in the common case and 0 in the reference's
 * "len % num_lines == 0" branch (log2_cache_line_size_ left at 0). */
int dlsm_bloom_full_parse(const uint8_t* filter, uint64_t len, int* num_probes,
                          uint32_t* num_lines, int* log2_line);

/* ---- context ------------------------------------------------------------ */

int dlsm_device_count(int* n);
int dlsm_ctx_create(int device, dlsm_ctx** out);
int dlsm_ctx_destroy(dlsm_ctx* ctx);
/* Work on the caller's hipStream_t (e.g. torch.cuda.current_stream()); NULL
 * restores the context's own stream. */
int dlsm_ctx_set_stream(dlsm_ctx* ctx, void* hip_stream);
void* dlsm_ctx_stream(dlsm_ctx* ctx);
/* The calling thread's context: the one bound with dlsm_thread_ctx_bind, else
 * one the library hands out on the thread's first call -- on device (i mod
 * device count) for the i-th thread that asks -- and takes back when the
 * thread exits.  Returned contexts wait in a per-device free list (drained,
 * their stream and scheduling options reset) for the next new thread: dLSM
 * starts a std::thread per subcompaction (db/db_impl.cc:3373-3386), which then
 * reuses a context instead of creating one.  dLSM runs each TableBuilder on
 * one thread (flush / compaction / subcompaction threads,
 * include/TimberSaw/options.h:73-78), so a FullFilterBlockBuilder with the
 * reference's (ibv_mr*, bits_per_key) signature (table/full_filter_block.h:35)
 * takes its context from here. */
int dlsm_thread_ctx(dlsm_ctx** out);
/* Bind a context the caller owns (NULL: unbind) as the calling thread's. */
int dlsm_thread_ctx_bind(dlsm_ctx* ctx);
/* Thread contexts created so far, handed out again from the free list, and
 * idle in the free list now. */
int dlsm_thread_ctx_stats(uint64_t* created, uint64_t* reused, uint64_t* idle);
/* Host fallbacks.  The C++ adapter (dlsm_bloom_adapter.hpp) answers a call
 * the GPU failed (device error, out of memory, injected fault, no device) with
 * the reference's own host loop -- so Finish never emits a 0-byte filter the
 * reference reader would exit on -- and records every such re-run here: on
 * the context (if any) and process-wide.  Parity tests assert both stay 0. */
void dlsm_fallback_note(dlsm_ctx* ctx);
int dlsm_fallback_stats(const dlsm_ctx* ctx, uint64_t* ctx_count, uint64_t* process_count);
/* The device a context runs on (-1 for NULL). */
int dlsm_ctx_device(const dlsm_ctx* ctx);
int dlsm_ctx_sync(dlsm_ctx* ctx);
/* Run the HBM-bound partition passes of sliced builds (one job group) and of
 * single-group probes (one round) on `hip_stream`, and the LDS-bound slice and
 * unpermute passes on the context stream; events order the two, and a call
 * is complete when the context stream is.  `cus` sizes the persistent probe
 * partition grid (the compute units `hip_stream` may use, 0 = all).  With
 * CU-masked streams (dlsm_stream_create_cu_mask) one node's flush builds and
 * Get probes share the GPU: partitions on most CUs, build slices on a few.
 * NULL restores one stream.  Scheduling only: results never depend on it.
 * The stream must outlive the context (dlsm_ctx_destroy synchronises it) or
 * be detached with NULL first. */
int dlsm_ctx_set_partition_stream(dlsm_ctx* ctx, void* hip_stream, uint32_t cus);
/* A hipStream_t restricted to the compute units whose bits are set in
 * mask[0..words) (bit i of word w = CU 32w + i; hipExtStreamCreateWithCUMask). */
int dlsm_stream_create_cu_mask(int device, const uint32_t* mask, uint32_t words, void** out);
int dlsm_stream_destroy(void* hip_stream);
/* Pre-size the device workspace so later calls never allocate (graph capture). */
int dlsm_ctx_reserve(dlsm_ctx* ctx, uint64_t max_keys, uint32_t max_jobs);
/* Workspace statistics: device allocations the context has made so far
 * (every growth of a workspace buffer counts one) and the bytes it holds.
 * After dlsm_ctx_reserve (or one warm-up call of each shape) the count stays
 * put: the hot path does not allocate. */
int dlsm_ctx_stats(dlsm_ctx* ctx, uint64_t* device_allocs, uint64_t* device_bytes);
/* Select kernels: 0 = auto, 1 = direct (global atomics / global probes),
 * 2 = sliced (LDS-tiled).  For A/B measurement; results are identical. */
int dlsm_ctx_set_path(dlsm_ctx* ctx, int path);

/* Scheduling knobs; results never depend on them.
 *   DLSM_OPT_PATH             same as dlsm_ctx_set_path
 *   DLSM_OPT_PROBE_ROUND_KEYS keys per pipelined probe round (default 0 = one
 *                             round, or $DLSM_PROBE_ROUND_KEYS)
 *   DLSM_OPT_BUILD_GROUPS     job groups of a pipelined build (0/1 = one, up to 4)
 *   DLSM_OPT_PROBE_CHUNK_LG   log2 keys per probe partition chunk, 12..14 (default 13,
 *                             or $DLSM_PROBE_CHUNK_LG)
 *   DLSM_OPT_PROBE_SLICE_LG   log2 stacked filter lines per probe LDS slice, 7 (64 KiB)
 *                             or 8 (128 KiB) (default 8, or $DLSM_PROBE_SLICE_LG)
 *   DLSM_OPT_BUILD_EXACT      0 auto (default): count consecutive-distinct hashes in a
 *                             pass of their own before bucketing when the batch has
 *                             internal keys (suffix_len > 0) or per-key lengths (offsets),
 *                             whose duplicate user keys lower the line count; 1 always;
 *                             2 never (one pass; a batch whose duplicates change the line
 *                             count then takes a slower per-slice re-hash fallback)
 *   DLSM_OPT_PROBE_ROUND_SERIAL 1: probe rounds run one after another on the context
 *                             stream (one buffer set) instead of pipelined over two
 *                             streams (default 0, or $DLSM_PROBE_SERIAL)
 *   DLSM_OPT_FAULT_INJECT     test hook: v > 0 makes every build and probe call on the
 *                             context return -v (4 = DLSM_E_DEVICE, 5 = DLSM_E_NOMEM)
 *                             before touching the device; 0 (default) off
 *   DLSM_OPT_VERSION_SLICE_BYTES  EXPERIMENTAL (off by default, kept with its tests):
 *                             dlsm_version_create on this context: a level >= 1 whose
 *                             filters hold more bytes goes to the sliced version probe
 *                             (0: $DLSM_VERSION_SLICE_MIN_BYTES, default never --
 *                             the sliced probe measured slower at 125 MB and 1.25 GB
 *                             levels, no size tried favours it; DESIGN.md §9 item 9
 *                             names the form left to try; UINT64_MAX: never)
 *   DLSM_OPT_VERSION_PASS_SLICES  128 KiB slices per partition pass of the sliced version
 *                             probe, 1..1024 (default 1024; larger levels take several)
 *   DLSM_OPT_PROBE_MULTI      a filter set of several (L, k) groups (a Version's files of
 *                             different sizes): 1 (default, or $DLSM_PROBE_MULTI) one
 *                             partition + slice + unpermute pass over every group, 0 one
 *                             such pass per group
 */
#define DLSM_OPT_PATH 0
#define DLSM_OPT_PROBE_ROUND_KEYS 1
#define DLSM_OPT_BUILD_GROUPS 2
#define DLSM_OPT_PROBE_CHUNK_LG 3
#define DLSM_OPT_PROBE_SLICE_LG 4
#define DLSM_OPT_BUILD_EXACT 5
#define DLSM_OPT_PROBE_ROUND_SERIAL 6
#define DLSM_OPT_FAULT_INJECT 7
#define DLSM_OPT_VERSION_SLICE_BYTES 8
#define DLSM_OPT_VERSION_PASS_SLICES 9
#define DLSM_OPT_PROBE_MULTI 10
int dlsm_ctx_set_option(dlsm_ctx* ctx, int option, uint64_t value);
/* The current value of an option (so a caller can restore it). */
int dlsm_ctx_get_option(dlsm_ctx* ctx, int option, uint64_t* value);

/* Page-lock a host range (e.g. an RDMA-registered FilterChunk slot) so D2H
 * copies land in it directly. */
int dlsm_host_register(void* p, size_t len);
int dlsm_host_unregister(void* p);
/* Page-locked host allocation (the H2D / D2H of the host-memory calls then
 * run as DMA at the link rate). */
int dlsm_host_alloc(size_t len, void** out);
int dlsm_host_free(void* p);
/* A process-wide pool of page-locked host buffers: acquire returns a buffer
 * of at least min_bytes (*cap: its size), reusing a released one when one
 * fits; release returns it to the pool (DLSM_E_ARG for a pointer the pool
 * did not hand out or one already released); trim frees every buffer in the
 * pool.  At most 1 GiB of released buffers is kept: a release past that frees
 * the buffer.  For key staging of builders that share no context. */
int dlsm_host_pool_acquire(uint64_t min_bytes, void** out, uint64_t* cap);
int dlsm_host_pool_release(void* p);
int dlsm_host_pool_trim(void);
/* The context's own page-locked host staging buffer, lent to ONE user at a
 * time (the reference runs one TableBuilder per thread, one context per
 * thread): claim returns DLSM_OK when the buffer is free or already held by
 * `owner`, DLSM_E_BUSY when another owner holds it; release gives it back.
 * dlsm_ctx_host_buffer (for the holder): at least min_bytes; when it has to
 * grow, its first keep_bytes bytes move to the new buffer.  Valid until the
 * next call that grows it or dlsm_ctx_destroy.  Builders created per SSTable
 * reuse it, so key staging allocates nothing after the first table. */
int dlsm_ctx_host_buffer_claim(dlsm_ctx* ctx, const void* owner);
int dlsm_ctx_host_buffer_release(dlsm_ctx* ctx, const void* owner);
int dlsm_ctx_host_buffer(dlsm_ctx* ctx, uint64_t min_bytes, uint64_t keep_bytes, void** out,
                         uint64_t* cap);

/* ---- full filter (SSTable format), build -------------------------------- */

/* Build one full filter per job: FullFilterBlockBuilder(mr, bpk); AddKey(k)
 * for every key in order; Finish().  Device pointers; asynchronous.
 * out_len_dev: device uint64[n_jobs] receiving each filter's length
 * (num_lines*64+5), or 0 when that job's slot was too small. */
int dlsm_bloom_full_build_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                              int bits_per_key, uint64_t* out_len_dev);

/* Same with host keys and host output slots (H2D + build + D2H, synchronous).
 * out_len: host uint64[n_jobs].  Returns DLSM_E_CAPACITY if any slot is too
 * small (its out_len is 0). */
int dlsm_bloom_full_build(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                          int bits_per_key, uint64_t* out_len);

/* The same build from BloomHash values instead of keys: each job's keys is a
 * set of n u32 hashes (key_len 4, offsets NULL, suffix_len 0, 4-byte aligned)
 * in AddKey order -- FullFilterBlockBuilder::hash_entries_
 * (full_filter_block.cc:39-49), which a caller that hashes in AddKey on the
 * host hands over at 4 bytes per key instead of the key bytes.  Consecutive
 * equal hashes are dropped on the GPU exactly like AddKey's check, so the
 * hashes may be given deduplicated or not. */
int dlsm_bloom_full_build_hashed_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                     int bits_per_key, uint64_t* out_len_dev);
int dlsm_bloom_full_build_hashed(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                 int bits_per_key, uint64_t* out_len);

/* ---- concurrent Finish calls gathered into batched builds --------------- */

/* A per-device submission queue for many builder threads (dLSM runs up to 4
 * flush + 12 compaction + 12 subcompaction builders at once,
 * include/TimberSaw/options.h:73-78).  dlsm_batcher_full_build[_hashed] has
 * dlsm_bloom_full_build[_hashed]'s meaning for ONE job (host keys, host slot)
 * and blocks until that filter is in the slot; concurrent calls are gathered
 * into one batched build by `executors` worker threads (each with its own
 * context and stream) that take every queued job, after waiting up to
 * window_us (0: no wait) for at most max_jobs.  The job's key bytes and slot
 * must stay valid until the call returns (page-locked memory: DMA). */
typedef struct dlsm_batcher dlsm_batcher;
int dlsm_batcher_create(int device, int executors, uint32_t window_us, uint32_t max_jobs, dlsm_batcher** out);
int dlsm_batcher_destroy(dlsm_batcher* b);
int dlsm_batcher_full_build(dlsm_batcher* b, const dlsm_build_job* job, int bits_per_key, uint64_t* out_len);
int dlsm_batcher_full_build_hashed(dlsm_batcher* b, const dlsm_build_job* job, int bits_per_key,
                                   uint64_t* out_len);
/* The general form: flags DLSM_BATCH_HASHED (the keys are BloomHash values,
 * as dlsm_batcher_full_build_hashed) | DLSM_BATCH_EXACT (the builder saw
 * repeated keys: the executor counts the line number exactly before
 * bucketing, DLSM_OPT_BUILD_EXACT = 1).  Jobs are batched only with jobs of
 * the same bits_per_key and flags.  A job whose batch fails for another
 * reason than a small slot is re-run alone, so each caller gets its own
 * status. */
#define DLSM_BATCH_HASHED 1
#define DLSM_BATCH_EXACT 2
int dlsm_batcher_submit(dlsm_batcher* b, const dlsm_build_job* job, int bits_per_key, int flags,
                        uint64_t* out_len);
/* Batches run, jobs built, and the largest batch so far. */
int dlsm_batcher_stats(dlsm_batcher* b, uint64_t* batches, uint64_t* jobs, uint64_t* max_batch);

/* FinishFilterBlock (table/table_builder_computeside.cc:389-432): the full
 * filter followed by the 5-byte block trailer [type 0][Fixed32(crc32c::Mask(
 * crc32c(filter || type)))] -- the exact bytes FlushFilter RDMA-writes
 * (:551-567).  out_len = filter length + 5, or 0 if the slot is too small.
 * crc32c on the GPU (util/crc32c.h:17-37 semantics). */
int dlsm_bloom_full_build_block_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                    int bits_per_key, uint64_t* out_len_dev);
int dlsm_bloom_full_build_block(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                int bits_per_key, uint64_t* out_len);

/* crc32c::Value of n device buffers on the GPU (ReadFilterBlock's check,
 * table/format.cc:398-408); crc_out: host uint32[n].  Synchronous. */
int dlsm_crc32c_dev(dlsm_ctx* ctx, const uint8_t* const* bufs, const uint64_t* lens, int n,
                    uint32_t* crc_out);
/* Host helpers: crc32c::Extend and crc32c::Mask (util/crc32c.h:17-31). */
uint32_t dlsm_crc32c_extend(uint32_t init_crc, const void* data, size_t n);
uint32_t dlsm_crc32c_mask(uint32_t crc);

/* ---- internal keys: the flush / compaction loops that feed AddKey -------- */

/* The two compute-node loops that hand keys to TableBuilder::Add (and so to
 * FullFilterBlockBuilder::AddKey through ExtractUserKey):
 *   DLSM_SELECT_FLUSH       FlushJob::BuildTable, db/memtable_list.cc:855-886:
 *                           keep the first entry of each user key; a key that
 *                           ParseInternalKey (db/dbformat.h:451-461) rejects
 *                           aborts the flush (IOError).
 *   DLSM_SELECT_COMPACTION  DBImpl::DoCompactionWork, db/db_impl.cc:3500-3562:
 *                           drop an entry hidden by a newer one of the same user
 *                           key whose sequence <= smallest_snapshot (rule (A));
 *                           corrupt keys are kept and restart the user key. */
#define DLSM_SELECT_FLUSH 0
#define DLSM_SELECT_COMPACTION 1

/* ikeys: internal keys in iterator order (user key || Fixed64(seq<<8|type));
 * its suffix_len is ignored.  keep_dev[i] (device, n bytes) = 1 iff the loop
 * passes key i to Add.  Host outputs (any may be NULL): n_kept, kept_bytes (the
 * kept keys' ExtractUserKey bytes), first_corrupt (index of the first key
 * ParseInternalKey rejects, or UINT64_MAX).  FLUSH returns DLSM_E_CORRUPT when
 * there is one.  Synchronous.
 * The full filter of the kept keys equals the full filter of ALL the keys with
 * suffix_len = 8: every dropped entry repeats the user key of the entry before
 * it, whose hash AddKey's consecutive dedup drops anyway -- so a filter build
 * never has to wait for this selection. */
int dlsm_internal_keys_select_dev(dlsm_ctx* ctx, const dlsm_keyset* ikeys, int policy,
                                  uint64_t smallest_snapshot, uint8_t* keep_dev, uint64_t* n_kept,
                                  uint64_t* kept_bytes, uint64_t* first_corrupt);

/* Pack ExtractUserKey(key) of every key with keep_dev[i] != 0, in order.
 * Fixed-length ikeys (key_len >= 8): user key j at user_keys_dev + j*(key_len-8),
 * offsets_dev unused.  Variable-length ikeys: the bytes back to back and
 * offsets_dev[0..n_kept] (device u64).  Size the outputs from
 * dlsm_internal_keys_select_dev's n_kept / kept_bytes.  Asynchronous. */
int dlsm_user_keys_gather_dev(dlsm_ctx* ctx, const dlsm_keyset* ikeys, const uint8_t* keep_dev,
                              uint8_t* user_keys_dev, uint64_t* offsets_dev);

/* ---- full filter, probe ------------------------------------------------- */

/* Parse + upload F full filters (1 <= F <= 64), FullFilterBlockReader ctor
 * semantics for each.  filters_are_device: the filter pointers are device
 * pointers already resident on ctx's device.  The set keeps its own copy. */
int dlsm_filterset_create(dlsm_ctx* ctx, const uint8_t* const* filters, const uint64_t* lens,
                          int n_filters, int filters_are_device, dlsm_filterset** out);
int dlsm_filterset_destroy(dlsm_filterset* fs);
int dlsm_filterset_size(const dlsm_filterset* fs, int* n_filters, uint64_t* device_bytes);

/* KeyMayMatch of every key against every filter of the set.  mask has
 * n * ceil(F/8) bytes; bit f of key i's bytes = filter f's answer.  Device
 * pointers; asynchronous. */
int dlsm_bloom_full_probe_dev(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* keys,
                              uint8_t* mask_dev);
/* Host keys and host mask, synchronous. */
int dlsm_bloom_full_probe(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* keys,
                          uint8_t* mask);
/* The same probe from BloomHash values: `hashes` is a set of n u32 hashes
 * (key_len 4, offsets NULL, suffix_len 0, 4-byte aligned, device memory) --
 * what KeyMayMatch computes on the host (full_filter_block.cc:271) -- so a
 * caller whose lookups start in host memory moves 4 bytes per key over PCIe
 * instead of the key bytes (dlsm_bloom_hash_batch).  Asynchronous. */
int dlsm_bloom_full_probe_hashed_dev(dlsm_ctx* ctx, const dlsm_filterset* fs, const dlsm_keyset* hashes,
                                     uint8_t* mask_dev);

/* BloomHash (include/TimberSaw/filter_policy.h:26-28) of every key of a host
 * key set (ExtractUserKey when suffix_len > 0) into out[n] (host), on up to
 * `threads` host threads of a process-wide pool (0: all), sixteen 20-byte
 * keys at a time with AVX-512 when the CPU has it.  The host side of the
 * hashed build and probe: the hashes go to dlsm_bloom_full_build_hashed* /
 * dlsm_bloom_full_probe_hashed_dev.  Synchronous; no device is touched. */
int dlsm_bloom_hash_batch(const dlsm_keyset* keys, uint32_t* out, int threads);

/* Streams n host bytes at p (n a multiple of 8) on the same pool and the same
 * NUMA placement dlsm_bloom_hash_batch uses (its threads move to the node
 * holding the bytes), XOR-folding them into *fold: the host's read ceiling
 * for that memory and those cores, which the host-side hashing is measured
 * against.  Synchronous; no device is touched. */
int dlsm_host_read_bytes(const void* p, uint64_t n, int threads, uint64_t* fold);

/* ---- MultiGet-style probe of a version's files ---- */

/* One SSTable of a version: its key range and its full filter.  Mirrors
 * RemoteMemTableMetaData's smallest / largest InternalKeys and number
 * (db/version_edit.h) and the table's FullFilterBlockReader. */
typedef struct {
  const uint8_t* smallest_user_key; /* host memory */
  uint64_t smallest_len;
  const uint8_t* largest_user_key; /* host memory */
  uint64_t largest_len;
  uint64_t largest_trailer; /* DecodeFixed64 of largest's last 8 bytes: seq << 8 | type */
  uint64_t number;          /* file number: level-0 files are searched largest first */
  int32_t level;            /* 0 .. DLSM_NUM_LEVELS-1 */
  int32_t reserved;
  const uint8_t* filter; /* full filter bytes, or NULL: a table without a filter */
  uint64_t filter_len;
} dlsm_version_file;

#define DLSM_NUM_LEVELS 6 /* config::kNumLevels, db/dbformat.h:26 */

typedef struct dlsm_version dlsm_version; /* the files and filters, resident on a device */

/* files: every SSTable of the version; within each level >= 1 in key order
 * (Version::levels_, non-overlapping), level-0 files in any order.  At most
 * 64 - (DLSM_NUM_LEVELS - 1) level-0 files.  filters_are_device: the filter
 * pointers are device pointers on ctx's device (key bounds are host memory
 * either way).  Filters are parsed like FullFilterBlockReader (DLSM_E_CORRUPT
 * where it exit(1)s or cannot probe). */
int dlsm_version_create(dlsm_ctx* ctx, const dlsm_version_file* files, int n_files,
                        int filters_are_device, dlsm_version** out);
int dlsm_version_destroy(dlsm_version* v);
/* Search slots: 0 .. n_l0-1 = level-0 files newest first (largest number
 * first); n_l0 + level - 1 = the one candidate file of level 1..5. */
int dlsm_version_slots(const dlsm_version* v, int* n_l0, int* n_slots);

/* For every lookup key (user keys; suffix_len 8 for internal keys), the files
 * Version::Get would visit -- Version::ForEachOverlapping (db/version_set.cc:
 * 273-321): level-0 files whose [smallest, largest] user-key range holds the
 * key, newest first, then per level the file FindFile (:95-118) picks for
 * LookupKey(key, snapshot) (db/dbformat.cc:111-128) unless the key sorts
 * before its smallest key -- whose filter passes the key (Table::InternalGet,
 * table/table.cc:350-358: FullFilterBlockReader::KeyMayMatch, or always when
 * the table has no filter).  slot_mask_dev[i] (device u64): bit s set for such
 * a file in search slot s; a Get reads the set slots in increasing order and
 * stops at the first that holds the key.  level_file_dev (device u32, n x
 * (DLSM_NUM_LEVELS-1), or NULL): per level the index inside that level of the
 * candidate file, UINT32_MAX when the level has none.  Asynchronous. */
int dlsm_version_probe_dev(dlsm_ctx* ctx, const dlsm_version* v, const dlsm_keyset* keys,
                           uint64_t snapshot, uint64_t* slot_mask_dev, uint32_t* level_file_dev);

/* ---- legacy FilterPolicy format (util/bloom.cc) ------------------------- */

/* CreateFilter(keys, n, dst) per job: writes bytes+1 bytes at out.
 * out_len_dev: device uint64[n_jobs]. */
int dlsm_bloom_legacy_build_dev(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                                int bits_per_key, uint64_t* out_len_dev);
int dlsm_bloom_legacy_build(dlsm_ctx* ctx, const dlsm_build_job* jobs, int n_jobs,
                            int bits_per_key, uint64_t* out_len);

/* KeyMayMatch(key, filter) for every key against one legacy filter; out has one
 * byte (0/1) per key.  filter is a device (``_dev``) or host pointer. */
int dlsm_bloom_legacy_probe_dev(dlsm_ctx* ctx, const uint8_t* filter_dev, uint64_t len,
                                const dlsm_keyset* keys, uint8_t* out_dev);
int dlsm_bloom_legacy_probe(dlsm_ctx* ctx, const uint8_t* filter, uint64_t len,
                            const dlsm_keyset* keys, uint8_t* out);

/* ---- legacy block-based filter block (table/filter_block.cc) ------------ */

/* FilterBlockBuilder (table/filter_block.cc:14-113) over one table, with the
 * legacy BloomFilterPolicy: `keys` in table order; data block b holds keys
 * [block_key_end[b-1], block_key_end[b]) and is followed by
 * StartBlock(block_end_offset[b]) (TableBuilder::Flush).  A filter covers
 * each 2 KiB (kFilterBaseLg = 11) of data-block offsets; keys after the last
 * block end go to Finish's filter.  The block is the filters, Fixed32 offsets,
 * Fixed32 array offset and the byte 11 -- bytes identical to Finish().
 * dlsm_filter_block_size gives its length; build writes it to out_dev
 * (device) and sets *out_len (host).  Synchronous. */
int dlsm_filter_block_size(const uint64_t* block_key_end, const uint64_t* block_end_offset,
                           int n_blocks, uint64_t n_keys, int bits_per_key, uint64_t* nbytes);
int dlsm_filter_block_build_dev(dlsm_ctx* ctx, const dlsm_keyset* keys, const uint64_t* block_key_end,
                                const uint64_t* block_end_offset, int n_blocks, int bits_per_key,
                                uint8_t* out_dev, uint64_t out_cap, uint64_t* out_len);

/* FilterBlockReader::KeyMayMatch(block_offset, key) (filter_block.cc:117-142)
 * for every key against one filter block (device): out_dev[i] = 0/1 for key i
 * in the data block at block_offsets_dev[i] (device u64).  Malformed blocks
 * answer 1 ("errors are treated as potential matches").  Asynchronous. */
int dlsm_filter_block_probe_dev(dlsm_ctx* ctx, const uint8_t* block_dev, uint64_t len,
                                const dlsm_keyset* keys, const uint64_t* block_offsets_dev,
                                uint8_t* out_dev);
/* Host-memory forms of the two calls above (keys, block, offsets, outputs on
 * the host; staged through device memory).  Synchronous. */
int dlsm_filter_block_build(dlsm_ctx* ctx, const dlsm_keyset* keys, const uint64_t* block_key_end,
                            const uint64_t* block_end_offset, int n_blocks, int bits_per_key,
                            uint8_t* out, uint64_t out_cap, uint64_t* out_len);
int dlsm_filter_block_probe(dlsm_ctx* ctx, const uint8_t* block, uint64_t len, const dlsm_keyset* keys,
                            const uint64_t* block_offsets, uint8_t* out);

/* ---- several GPUs from one process -------------------------------------- */

/* One device's share of a flush/compaction round plus a Get batch: its
 * SSTables' build jobs (device pointers) and its shard of the lookups against
 * its own copy of the stacked filter set (SSTables are
 * independent, so nothing crosses devices). */
typedef struct {
  dlsm_ctx* probe_ctx;         /* the device's probe context (its stream) */
  dlsm_ctx* build_ctx;         /* == probe_ctx, or a second context on the same device: the
                                  build then runs on its stream beside the probe */
  const dlsm_build_job* jobs;  /* n_jobs SSTables (device keys, device slots) */
  int n_jobs;
  uint64_t* out_len_dev;       /* device uint64[n_jobs] */
  const dlsm_filterset* fs;    /* NULL: no probe */
  dlsm_keyset keys;            /* device lookup shard */
  uint8_t* mask_dev;
} dlsm_device_work;

/* Run `warmup` untimed then `steps` timed steps (build, then probe) on every
 * entry concurrently, one host thread per entry (dLSM's shape: its builders
 * are threads of one process, db/db_impl.cc:3373-3386).  The timed region
 * starts when every device is idle and ends when every device has drained
 * (host barriers on both sides): wall_seconds is the slowest device's.
 * pass_ms (host float[2 * steps], or NULL): entry 0's build / probe time per
 * step from HIP events on the streams they run on. */
int dlsm_multi_device_run(const dlsm_device_work* work, int n_devices, int bits_per_key, int steps, int warmup,
                          double* wall_seconds, float* pass_ms);
/* The same, with entry 0's passes timed on every event_every-th step only
 * (steps i with i % event_every == event_every - 1); the other steps' pass_ms
 * entries are -1.  A timed event pair at a call boundary leaves the GPU idle
 * for several microseconds, so sampling keeps the timed steps' shape.  When
 * entry 0's build runs on its own stream (build_ctx != probe_ctx), a sampled
 * step runs its two passes one after the other, alone on the device, so
 * pass_ms holds each pass's own time rather than its time beside the other. */
int dlsm_multi_device_run_sampled(const dlsm_device_work* work, int n_devices, int bits_per_key, int steps,
                                  int warmup, int event_every, double* wall_seconds, float* pass_ms);
/* The same, with every entry's passes timed: pass_ms (host float[n_devices *
 * 2 * steps], or NULL) holds entry d's build / probe ms of step i at
 * [d * 2 * steps + 2 * i] / [+ 1] (-1 on the steps not sampled), and
 * device_seconds (host double[n_devices], or NULL) each entry's own time from
 * the start barrier until its device drained -- the slowest is the wall time,
 * the spread the N-GPU job's imbalance. */
int dlsm_multi_device_run_timed(const dlsm_device_work* work, int n_devices, int bits_per_key, int steps,
                                int warmup, int event_every, double* wall_seconds, float* pass_ms,
                                double* device_seconds);

/* ---- measurement helper (not on the filter path) ------------------------ */

/* The box's HBM streaming ceilings for the roofline (bench.py): launch one
 * 16-byte-per-lane streaming kernel on hip_stream over `bytes` (a multiple of
 * 16; 16-byte-aligned buffers).  kind 0: read src (dst receives at most 512
 * u32 of sink writes, normally none); kind 1: copy src -> dst; kind 2: the
 * probe partition's byte shape, reading src and writing 3/10 as many bytes to
 * dst (20 B in, 6 B out per key).  variant bit
 * 0: non-temporal accesses; bit 1: one contiguous range per workgroup (else
 * grid-stride).  blocks: workgroups of 512 threads.  Asynchronous. */
int dlsm_stream_kernel(void* hip_stream, int kind, int variant, const void* src, void* dst, uint64_t bytes,
                       uint32_t blocks);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* DLSM_BLOOM_H_ */
