// dlsm_amd/csrc/bloom_internal.h -- device-side descriptors and the launcher
// interface between the C ABI (bloom_capi.hip) and the kernels
// (bloom_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bloom_math.h"

namespace dlsm {

// Key-load modes: K20 = fixed 20-byte keys at a 16-byte-aligned base (the
// BASELINE shape; staged through LDS with 16-byte loads), GENERIC = any fixed
// length / alignment or offsets (per-thread aligned-dword loads).
// K20: packed 20-B user keys; K28: packed 28-B internal keys hashed as
// ExtractUserKey (suffix 8) -- both 16-B-aligned fixed stride, LDS-tiled in
// the partition passes (other kernels take the K28 keys on the generic path)
// KM_HASH: the "keys" are BloomHash values already (u32 each, from the hash
// pass of a grouped probe): the partition loads them instead of hashing.
enum KeyMode : int { KM_GENERIC = 0, KM_K20 = 1, KM_K28 = 2, KM_HASH = 3 };

struct KeyDesc {
  const uint8_t* bytes;
  const uint64_t* offsets;  // n+1 entries or nullptr
  uint64_t n;
  uint32_t key_len;
  uint32_t suffix;  // bytes dropped from each key's end before hashing (ExtractUserKey: 8)
};

// One full-filter build job as the kernels see it.
struct FullJobDev {
  KeyDesc keys;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* out_len;   // device slot for this job's length
  uint64_t entry0;     // first entry of this job in the entry workspace
  uint64_t tab0;       // first u16 of this job's n_chunks x (n_slices+1) bucket-offset table
  uint32_t chunk0, n_chunks;
  uint32_t slice0, n_slices;
  uint32_t L_spec, magic_spec;  // speculative line count (no duplicates) + fastmod magic
  int32_t k, bpk;
  // 1: a count pass ran first (dchunk holds every chunk's distinct count), so
  // the partition buckets by the true line count, not L_spec -- batches whose
  // duplicates lower L (internal keys with several versions per user key)
  int32_t exact;
  int32_t reserved;
};

// A parsed full filter resident on the device (FullFilterBlockReader state).
struct FilterDev {
  const uint8_t* data;
  uint32_t L, magic;
  int32_t k, lg;
};

// One SSTable of a version (dlsm_version_file) as the version probe sees it.
struct VFileDev {
  uint64_t smallest_off, largest_off;  // user keys inside the version's key blob
  uint32_t smallest_len, largest_len;
  uint64_t largest_trailer;            // seq << 8 | type of the largest internal key
  FilterDev f;                         // f.data == nullptr: the table has no filter
  uint32_t line0;                      // sliced level: the file's first line in the level image
  uint32_t reserved;
};

constexpr int kNumLevels = 6;  // config::kNumLevels (db/dbformat.h:26)

// Sliced version probe (levels whose filters outgrow an XCD's L2): the
// level's filters' lines are stored back to back as one image (line0 per
// file), the route pass writes each lookup's global line in that image, and a
// partition / LDS slice / unpermute round answers all of the level's probes.
constexpr int kVSliceLg = 11;                                  // 2^11 lines (128 KiB) per slice
constexpr uint32_t kVMaxSlices = 1024;                         // slices per partition pass
constexpr int kVChunk = 16384;                                 // lookups per partition chunk
constexpr uint32_t kVRegion = kVChunk + 4u * kVMaxSlices;      // entries per chunk region
constexpr uint32_t kVNoLine = 0xffffffffu;                     // route: no probe in this level
constexpr uint16_t kVNoPos = 0xffffu;                          // partition: no probe in this pass
constexpr uint32_t kVPlanBudget = 512;                         // slice-pass workgroups the entries spread over

// The version's key space cut at every file bound: bnd[0, n_bnd) holds the
// distinct 16-byte prefixes of all files' smallest and largest user keys in
// order, and ivl[j] what Version::Get visits for a lookup whose prefix lies
// strictly between bnd[j-1] and bnd[j] (j = 0: below all, j = n_bnd: above
// all) -- the level-0 files holding it and each level's FindFile pick when
// its smallest key admits the lookup.  Prefixes decide the bytewise order
// whenever they differ, so an open interval's answers are fixed; a lookup
// whose prefix equals a bound takes the full comparison path.
struct VIntervalDev {
  uint64_t l0mask;                  // bit f: level-0 file f (search order) holds the lookup
  uint16_t pick[kNumLevels - 1];    // per level 1..5: the picked file (search order index) or 0xffff
  uint16_t reserved[3];             // (24 B: the wave-queued kernel, the only reader, takes <= 65,535 files)
};
static_assert(sizeof(VIntervalDev) == 24, "interval record layout");

// Files in search order: level-0 newest first, then levels 1.. in key order.
struct VersionDev {
  const VFileDev* files;
  // per file (search order) the first 16 bytes of its smallest / largest user
  // key, zero-padded, as two big-endian u64: comparing them decides the
  // bytewise order unless they are equal (then the full keys are compared)
  const ulonglong2* pre_small;
  const ulonglong2* pre_large;
  const uint8_t* keyblob;
  uint32_t n_l0;
  uint32_t lvl_begin[kNumLevels];
  uint32_t lvl_count[kNumLevels];
  int32_t lvl_sliced[kNumLevels];  // sliced level: its index j among the sliced levels, else -1
  const ulonglong2* bnd;           // interval index (VIntervalDev)
  const VIntervalDev* ivl;
  uint32_t n_bnd;
  int32_t k_all;  // the probe count every filter of the version has, or 0 when they differ
};

// Legacy-format build job.
struct LegacyJobDev {
  KeyDesc keys;
  uint8_t* out;
  uint64_t bits;      // filter bits (multiple of 8)
  uint32_t magic;     // fastmod magic for bits when bits < 2^32
  int32_t k;
  uint64_t key0;      // global index of this job's first key (flattened grid)
};

// Legacy-format build job of the LDS-tiled path (util/bloom.cc:25-55).  The
// filter's bits are cut into tiles of 2^16 bits (8 KiB); the partition pass
// writes every bit position a key sets as a u16 offset inside its tile,
// bucketed by tile inside the key's kLegacyChunk-key chunk (each bucket padded
// to 8 entries = one 16-byte unit with copies of one of its positions: OR-ing
// a bit twice changes nothing), and the slice pass ORs 2^tps_lg tiles in LDS.
struct LegacyTileJobDev {
  KeyDesc keys;
  uint8_t* out;
  uint64_t* out_len;   // device slot for this job's length (bytes + 1)
  uint64_t entry0;     // first u16 of this job's chunk regions
  uint64_t tab0;       // first u16 of this job's n_chunks x (n_tiles+1) bucket-offset table
  uint32_t bits;       // filter bits (multiple of 8, < 2^32)
  uint32_t magic;      // fastmod magic for bits
  uint32_t n_tiles;    // ceil(bits / 2^16)
  uint32_t region;     // u16 entries per chunk region (multiple of 8)
  uint32_t chunk0, n_chunks;
  uint32_t slice0, n_slices;
  int32_t k;
  int32_t reserved;
};
constexpr uint32_t kLegacyTileLg = 16;  // bits per tile: 2^16 (8 KiB of LDS)
#ifndef DLSM_LEGACY_CHUNK
#define DLSM_LEGACY_CHUNK 4096  // keys per legacy partition chunk
#endif
#ifndef DLSM_LEGACY_NT
#define DLSM_LEGACY_NT 512      // threads per legacy partition workgroup
#endif
constexpr int kLegacyChunk = DLSM_LEGACY_CHUNK;
constexpr int kLegacyPartBlock = DLSM_LEGACY_NT;
// Partition variants (static LDS staging of one chunk region of u16 entries:
// k positions per key + up to 7 pads per tile): A: k <= 6, <= 512 tiles;
// B: k <= 8, <= 4 x threads - 1 tiles (the bins one block scan covers: 1,023
// tiles = 64 Mbit at 256 threads).  Larger filters or k take the direct
// (global atomic) path.
constexpr int kLegacyKmaxA = 6, kLegacyKmaxB = 8;
constexpr uint32_t kLegacyTilesA = 512, kLegacyTilesB = 4u * kLegacyPartBlock - 1u;
constexpr uint32_t legacy_region(int k, uint32_t tiles) {
  return (static_cast<uint32_t>(k) * kLegacyChunk + 7u * tiles + 7u) & ~7u;
}
constexpr uint32_t kLegacyStageA = legacy_region(kLegacyKmaxA, kLegacyTilesA);
constexpr uint32_t kLegacyStageB = legacy_region(kLegacyKmaxB, kLegacyTilesB);
constexpr int kLegacySliceBlock = 1024;

constexpr int kBlock = 256;
constexpr int kMaxSlices = 256;     // slice bins per table in one partition pass
constexpr uint32_t kBuildSliceCUs = 256;  // MI355X CUs: the build's slice-count target (choose_build_lgR)
#ifndef DLSM_BUILD_CHUNK
#define DLSM_BUILD_CHUNK 4096
#endif
constexpr int kBuildChunk = DLSM_BUILD_CHUNK;  // keys per partition chunk (build)
// The build partition pads every slice bucket of a chunk to whole 16-byte
// units (pad entries have bit 31 set), so the slice pass loads 4 entries per
// lane per load; each chunk owns a region of kBuildRegion entries (its keys
// plus up to 3 pads per bucket).  r02: build slice 65.7 -> 50.8 us
// (profiles/r02_ab_units_pred.txt).
constexpr uint32_t kBuildRegion = kBuildChunk + 4u * kMaxSlices;
constexpr int kProbeChunkMin = 4096;  // smallest probe partition chunk (lgC 12)
// u32 entries (and answer bytes) per probe chunk region: C keys plus up to 3
// padding entries per slice bucket (buckets are padded to 16-byte units).
constexpr uint32_t probe_region(uint32_t C) { return C + 4u * kMaxSlices; }

// ---- launchers (bloom_kernels.hip) -----------------------------------------
// All return the hipError_t of the launch.  `dchunk` holds one
// consecutive-distinct hash count per build chunk (written by the count /
// partition kernels, summed per job by their consumers, so no per-call memset).
hipError_t launch_full_count(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                             uint32_t total_chunks, uint32_t* dchunk, int mode, hipStream_t s);
hipError_t launch_full_zero(const FullJobDev* jobs, int n_jobs, const uint32_t* dchunk,
                            uint32_t* jobL, hipStream_t s);
hipError_t launch_full_scatter(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                               uint32_t total_chunks, const uint32_t* jobL, int mode, hipStream_t s);
// Partition chunks [chunk_first, +n_chunks) / slices [slice_first, +n_slices)
// of the job table (a contiguous job group of a pipelined build).
// exact: the count pass already filled dchunk; bucket by each job's true line count.
hipError_t launch_full_partition(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                                 uint32_t chunk_first, uint32_t n_chunks, uint32_t* dchunk,
                                 uint32_t* entries, uint16_t* tab, int lgR, int mode, bool exact,
                                 hipStream_t s);
// crc_part (or nullptr): each slice's crc32c register contribution, for
// launch_full_block_seal; crc_tabs: full_block_crc_tables(lgR).
hipError_t launch_full_slices(const FullJobDev* jobs, const uint32_t* slice0s, int n_jobs,
                              uint32_t slice_first, uint32_t n_slices, const uint32_t* dchunk,
                              const uint32_t* entries, const uint16_t* tab, int lgR, hipStream_t s,
                              uint32_t* crc_part = nullptr, const uint32_t* crc_tabs = nullptr,
                              uint32_t* crc_cnt = nullptr);  // per-job counters, zero between calls
// Seal each job's filter as a filter block (after its sliced build with
// crc_part): [filter][type 0][masked crc32c], out_len += 5.
hipError_t launch_full_block_seal(const FullJobDev* jobs, int n_jobs, const uint32_t* crc_part,
                                  const uint32_t* crc_tabs, int lgR, hipStream_t s);
// Host tables for the fused seal at slices of 2^lgR lines (u32): the
// slice-by-4 crc32c tables (1024), per build-slice thread t x^(8 * 2^lgR / 8 *
// (511 - t)) (512), x^(8 * 2^lgR * 64 * m) for m < 256, x^(8 * 64 * m) for
// m <= 2^11.
constexpr size_t kCrcTabWords = 1024 + 512 + 256 + 2049;
void full_block_crc_tables(int lgR, uint32_t* out);

hipError_t launch_probe_direct(const FilterDev* fs, int n_filters, KeyDesc keys, uint8_t* mask,
                               int mode, hipStream_t s);
// Direct probe of one group's 8 slots from precomputed hashes (KM_HASH keys):
// the answer bits OR-ed (or, for the byte's first group, written) into byte
// `byte` of each key's `stride`-byte mask entry.
hipError_t launch_probe_direct_group(const FilterDev* slots, KeyDesc hashes, uint8_t* mask, int stride,
                                     int byte, bool first, hipStream_t s);
// Stacked image of up to 8 filters of one line count: slots[b] (b < 8) is the
// filter whose answer goes to bit b of the answer byte, or has data == nullptr
// (bit b stays 0).
hipError_t launch_stack_filters(const FilterDev* slots, uint32_t L, uint64_t* stacked, hipStream_t s);
// Packed image of a group of at most 2^lgw (< 8) filters of one line count:
// each line holds 512 fields of W = 2^lgw bits (64 * W bytes), field bit m =
// the line's bit of member m, whose slot is (slotmap >> 4m) & 7 (members past
// the group's size, or with data == nullptr, read as 0).
hipError_t launch_pack_filters(const FilterDev* slots, uint32_t slotmap, int lgw, uint32_t L,
                               uint64_t* packed, hipStream_t s);
// BloomHash of every key (u32 per key, coalesced): the grouped probe hashes
// each lookup once and partitions the hashes once per filter group.
hipError_t launch_probe_hash(KeyDesc keys, uint32_t* hashes, int mode, hipStream_t s);
// Unpermute for a filter group of a multi-byte or multi-group set: answer
// byte of key i to mask[i * stride + byte], OR-ed into what is there unless
// `first` (the first group of that mask byte).
hipError_t launch_probe_unpermute_group(uint64_t n_keys, const uint16_t* pos, const uint8_t* smask,
                                        uint8_t* mask, int stride, int byte, bool first, int lgC,
                                        hipStream_t s);
// lgC: log2 keys per probe chunk (12..14); lgR: log2 stacked lines per slice
// (7, 8 for byte-wide stacked images; 11 - lgw for packed ones, lgw < 3).
// R: filter lines per slice (<= 256 for byte images, 2^(11-lgw) for packed).
hipError_t launch_probe_partition(KeyDesc keys, uint32_t L, uint32_t magic, uint32_t R,
                                  uint32_t n_slices, uint32_t* entries, uint16_t* pos,
                                  uint16_t* tab, int mode, int lgC, hipStream_t s,
                                  uint32_t cus = 0);  // CUs the persistent grid is sized for (0: the device's)
// lgw 3: byte-wide stacked image (launch_stack_filters); lgw 0..2: packed
// image (launch_pack_filters) whose member m answers in bit (slotmap >> 4m) & 7.
// lgR: log2 of the LDS capacity in lines; R <= 2^lgR: the slice size in lines.
hipError_t launch_probe_slices(const uint64_t* stacked, uint32_t L, uint32_t magic, int k,
                               int lgR, uint32_t R, int lgw, uint32_t slotmap, uint32_t n_slices, uint32_t n_chunks,
                               const uint32_t* entries, const uint16_t* tab, uint8_t* smask,
                               int parts, int lgC, hipStream_t s);
hipError_t launch_probe_unpermute(uint64_t n_keys, const uint16_t* pos, const uint8_t* smask,
                                  uint8_t* mask, int lgC, hipStream_t s);

// ---- one-pass probe of a multi-group filter set (round 6) -------------------
// A Version's filters differ in line count (flush outputs, size-capped
// compaction outputs, dedup-shifted L), so its filter set splits into groups
// of one (L, k).  The one-pass probe hashes each lookup once in ONE partition
// pass that buckets it by every group's slice; the slice pass walks every
// group's slices (one launch per image width class) and one unpermute ORs
// every group's answer into the key's mask bytes.
// Layout per chunk of C lookups:
//  * entries: a region of `region` u32, group j's bucket runs in its own
//    sub-region [eoff_j, eoff_j + C + 8 S_j) (every bucket padded to 8
//    entries = two 16-byte units; the sub-region's tail is never written);
//  * table: one row of S_tot + G u16 offsets (into the region), group j's
//    S_j + 1 bucket starts at columns [tcol_j, tcol_j + S_j];
//  * positions: pos[(chunk * G + j) * C + i] = key i's entry index inside
//    group j's sub-region;
//  * answers: W_j = 2^lgw_j bits per entry (the image's field: member m in
//    bit m; a byte-wide stacked image's byte, slot-mapped already), group j's
//    at byte aoff_j of the chunk's `abytes`-byte answer area.
struct MGroupDev {
  const uint8_t* image;  // stacked (lgw 3) or packed image, 64 * 2^lgw bytes per line
  uint32_t L, magic;     // line count + fastmod magic
  uint32_t R, rmagic;    // lines per slice (2^(11 - lgw): 128 KiB) + fastdivmod magic
  uint32_t S, sbase;     // slices; the group's first global slice
  uint32_t slotmap;      // packed images: member m answers in bit (slotmap >> 4m) & 7
  int32_t k, lgw, mask_byte;
  uint32_t tcol;         // first table column (sbase + the group's index)
  uint32_t eoff;         // entry sub-region (u32 entries, a multiple of 8)
  uint32_t aoff;         // answer sub-area (bytes, a multiple of 16)
  uint32_t reserved;
};
constexpr int kMGMaxGroups = 16;
constexpr uint32_t kMGMaxSlices = 1024;
constexpr uint32_t kMGPad = 8;  // entries per bucket padding unit (two 16-byte units: whole answer bytes at W = 1)
// Keys per chunk of the one-pass partition (u16 table offsets into the chunk
// region of G * C entries + padding), so larger sets take smaller chunks.
#ifndef DLSM_MG_LG8
#define DLSM_MG_LG8 11  // chunk lg for sets of <= 8 groups (A/B knob; 12: 4,096-key chunks)
#endif
constexpr int mg_chunk_lg(int G) { return G <= 8 ? DLSM_MG_LG8 : 11; }
// Entries of group j's sub-region and bytes of its answer sub-area.
constexpr uint32_t mg_sub_entries(uint32_t C, uint32_t S) { return C + kMGPad * S; }
constexpr uint32_t mg_sub_abytes(uint32_t C, uint32_t S, int lgw) {
  return (((mg_sub_entries(C, S) << lgw) / 8u) + 15u) & ~15u;
}
// stage_bytes: the largest staging area one set of the partition needs
// (the sum of C + 8 S_j entries over the set's groups, x 4 bytes).
hipError_t launch_probe_mpartition(KeyDesc keys, const MGroupDev* groups, int G, uint32_t rowlen,
                                   uint32_t region, uint32_t stage_bytes, uint32_t* entries, uint16_t* pos,
                                   uint16_t* tab, int mode, hipStream_t s);
#ifndef DLSM_MG_P
#define DLSM_MG_P 2     // groups bucketed per phase of the partition (2,048-key chunks)
#endif
constexpr int mg_set_size(int lgC) { return lgC == 11 ? DLSM_MG_P : 2; }
// The slices [s0, s0 + S) of one image-width class (every group with image
// width lgw; K: 6 when every such group has k = 6, else 0 = the group's k),
// workgroups per slice from plan (S + 1 starts, wgs = plan[S]).
hipError_t launch_probe_mslices(int lgw, int K, const MGroupDev* groups, int G, uint32_t s0, uint32_t S,
                                uint32_t rowlen, uint32_t region, uint32_t abytes, uint32_t n_chunks,
                                const uint32_t* entries, const uint16_t* tab, uint8_t* answers,
                                const uint32_t* plan, uint32_t wgs, hipStream_t s);
hipError_t launch_probe_munpermute(uint64_t n_keys, const MGroupDev* groups, int G, uint32_t abytes,
                                   const uint16_t* pos, const uint8_t* answers, uint8_t* mask, int mask_bytes,
                                   hipStream_t s);

hipError_t launch_version_probe(const VersionDev& v, KeyDesc keys, uint64_t snapshot,
                                uint64_t* slot_mask, uint32_t* level_file, hipStream_t s);
// Route pass of the sliced version probe: launch_version_probe's outputs for
// the levels probed directly, plus hv[i] = BloomHash and, for sliced level j,
// gl[j * n + i] = the lookup's global line in the level image (kVNoLine: none).
hipError_t launch_version_route(const VersionDev& v, KeyDesc keys, uint64_t snapshot, uint64_t* slot_mask,
                                uint32_t* level_file, uint32_t* hv, uint32_t* gl, hipStream_t s);
// One partition pass: the lookups whose line g (in gl[0, n)) lies in
// [g0, g0 + S * 2^kVSliceLg) bucketed by slice per kVChunk-lookup chunk
// (entries: chunk regions of kVRegion, tab: chunk-major rows of S+1 u16,
// pos: the bucketed position or kVNoPos).
// gcnt (S u32, zero on entry, zero again on return) collects each slice's
// entry units; plan (S+1 u32) receives the slice pass's workgroup plan.
hipError_t launch_version_partition(const uint32_t* hv, const uint32_t* gl, uint64_t n, uint32_t g0, uint32_t S,
                                    uint32_t* entries, uint16_t* pos, uint16_t* tab, uint32_t* gcnt,
                                    uint32_t* plan, hipStream_t s);
// The slice pass over `image` lines [0, L) of this pass (a 2^kVSliceLg-line
// slice per workgroup, a slice's chunks split over its planned parts, k
// probes per entry): answer bit 0 per entry.
hipError_t launch_version_slices(const uint8_t* image, uint32_t L, int k, uint32_t S, uint32_t n_chunks,
                                 const uint32_t* entries, const uint16_t* tab, uint8_t* smask,
                                 const uint32_t* plan, hipStream_t s);
// Answers back to lookup order: abyte[i] gets bit jbit (written on the first
// pass, OR-ed after); the last pass ORs every sliced level's bit into
// slot_mask[i] at slot (slots >> 8j) & 63.
hipError_t launch_version_unpermute(uint64_t n, const uint16_t* pos, const uint8_t* smask, uint8_t* abyte,
                                    uint64_t* slot_mask, int jbit, int n_sliced, uint64_t slots, bool first,
                                    bool last, hipStream_t s);
hipError_t launch_filter_block_probe(const uint8_t* blk, uint64_t len, KeyDesc keys,
                                     const uint64_t* block_offsets, uint8_t* out, hipStream_t s);
hipError_t launch_legacy_scatter(const LegacyJobDev* jobs, const uint64_t* key0s, int n_jobs,
                                 uint64_t total_keys, int mode, hipStream_t s);
hipError_t launch_legacy_probe(const uint8_t* filter, uint64_t bits, uint32_t magic, int k,
                               int trivial, KeyDesc keys, uint8_t* out, int mode, hipStream_t s);
// LDS-tiled legacy build: variant 0 = A, 1 = B (kLegacy*); tps_lg 0..4 tiles
// per slice workgroup (log2).
hipError_t launch_legacy_partition(const LegacyTileJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                                   uint32_t total_chunks, uint16_t* entries, uint16_t* tab, int variant,
                                   int mode, hipStream_t s);
hipError_t launch_legacy_slices(const LegacyTileJobDev* jobs, const uint32_t* slice0s, int n_jobs,
                                uint32_t total_slices, const uint16_t* entries, const uint16_t* tab, int tps_lg,
                                hipStream_t s);

// key_select.hip: internal-key selection (flush / compaction drop rules) and
// the packing of kept user keys.  Workspace: blk_cnt / blk_bytes hold
// select_blocks(n) u64 each, tot 2 u64, first_bad 1 u64 (preset to ~0).
uint64_t select_blocks(uint64_t n);
hipError_t launch_key_select(KeyDesc kd, int mode, uint64_t snapshot, uint8_t* keep, uint64_t* blk_cnt,
                             uint64_t* blk_bytes, unsigned long long* first_bad, uint64_t* tot,
                             hipStream_t s);
hipError_t launch_key_gather(KeyDesc kd, const uint8_t* keep, uint64_t* blk_cnt, uint64_t* blk_bytes,
                             uint8_t* out, uint64_t* out_offsets, uint64_t* tot, hipStream_t s);

// block_crc.hip: crc32c of device streams, optionally sealing filter blocks.
uint64_t crc_max_parts(uint64_t max_len_plus_extra);
size_t crc_stream_size();
void crc_stream_fill(void* dst, const uint8_t* data, const uint64_t* len_dev, uint64_t len_host,
                     uint32_t extra);
hipError_t launch_crc_streams(const void* streams, int n, int max_parts, uint32_t* partial,
                              uint8_t* const* seal_out, const uint64_t* seal_cap, uint64_t* seal_len,
                              uint32_t* crc_out, hipStream_t s);

}  // namespace dlsm
