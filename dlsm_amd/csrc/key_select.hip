// dlsm_amd/csrc/key_select.hip -- internal-key selection and user-key gather
// on the GPU: the per-key decisions of the two loops
// that feed TableBuilder::Add -- and through it FullFilterBlockBuilder::AddKey
// -- on the compute node, and the packing of the kept user keys.
//
//   FlushJob::BuildTable        db/memtable_list.cc:855-886
//   DBImpl::DoCompactionWork    db/db_impl.cc:3500-3562 (the memory node's
//                               Memory_Node_Keeper::DoCompactionWork repeats it)
//   ParseInternalKey            db/dbformat.h:451-461
//   ExtractUserKey              db/dbformat.h:374-377
//
// Key i's decision depends on key i-1 only, so one pass decides every key:
//   parsed(i)  = len >= 8 and type (low byte of DecodeFixed64(key + len - 8))
//                <= kTypeValue (1); sequence = that Fixed64 >> 8
//   first(i)   = not (parsed(i-1) and parsed(i) and user(i) == user(i-1))
//                (a corrupt key clears has_current_user_key)
//   flush      : keep(i) = first(i); a corrupt key aborts the flush
//                (IOError, builder deleted): DLSM_E_CORRUPT + its index
//   compaction : drop(i) = parsed(i) and not first(i) and seq(i-1) <= snapshot
//                (rule (A)); corrupt keys are kept ("do not hide error keys")
// User keys compare equal iff their bytes are equal (BytewiseComparator; the
// flush loop compares user keys through the InternalKeyComparator, whose
// result is 0 exactly for byte-equal keys of >= 8 bytes).
//
// Gather: an exclusive scan of (kept keys, kept user-key bytes) over blocks
// of 1024 keys (per-block sums, one scan workgroup, then per-block local
// scans) places ExtractUserKey(key) of every kept key in a packed array.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "bloom_internal.h"

namespace dlsm {
namespace {

constexpr int kSelBlock = 256;
constexpr int kSelPer = 4;                       // keys per thread
constexpr int kSelKeys = kSelBlock * kSelPer;   // keys per block

struct IKey {
  const uint8_t* p;
  uint64_t len;
};

__device__ __forceinline__ IKey ikey_at(const KeyDesc& kd, uint64_t i) {
  if (kd.offsets) {
    const uint64_t s = kd.offsets[i];
    return {kd.bytes + s, kd.offsets[i + 1] - s};
  }
  return {kd.bytes + i * kd.key_len, kd.key_len};
}

// ParseInternalKey: false for len < 8 or type > kTypeValue.
__device__ __forceinline__ bool parse_ikey(const IKey& k, uint64_t* seq) {
  if (k.len < 8) return false;
  uint64_t num = 0;
  for (int b = 0; b < 8; b++) num |= static_cast<uint64_t>(k.p[k.len - 8 + b]) << (8 * b);
  *seq = num >> 8;
  return (num & 0xffu) <= 1u;
}

__device__ __forceinline__ bool user_keys_equal(const IKey& a, const IKey& b) {
  if (a.len != b.len) return false;
  const uint64_t n = a.len - 8;
  for (uint64_t j = 0; j < n; j++)
    if (a.p[j] != b.p[j]) return false;
  return true;
}

__device__ __forceinline__ uint8_t decide(const KeyDesc& kd, uint64_t i, int mode,
                                          uint64_t snapshot, bool* corrupt) {
  const IKey k = ikey_at(kd, i);
  uint64_t seq = 0;
  const bool ok = parse_ikey(k, &seq);
  *corrupt = !ok;
  bool first = true;
  uint64_t prev_seq = 0;
  if (ok && i > 0) {
    const IKey q = ikey_at(kd, i - 1);
    if (parse_ikey(q, &prev_seq) && user_keys_equal(k, q)) first = false;
  }
  if (mode == 0) return ok && first;                   // flush
  return !(ok && !first && prev_seq <= snapshot);      // compaction
}

// Pass 1: keep[i], per-block kept count and kept user-key bytes, first corrupt.
__global__ __launch_bounds__(kSelBlock) void select_kernel(KeyDesc kd, int mode, uint64_t snapshot,
                                                           uint8_t* __restrict__ keep,
                                                           uint64_t* __restrict__ blk_cnt,
                                                           uint64_t* __restrict__ blk_bytes,
                                                           unsigned long long* __restrict__ first_bad) {
  __shared__ uint64_t sc[kSelBlock / 64], sb[kSelBlock / 64];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kSelKeys;
  uint64_t cnt = 0, bytes = 0;
#pragma unroll
  for (int r = 0; r < kSelPer; r++) {
    const uint64_t i = base + r * kSelBlock + threadIdx.x;
    if (i >= kd.n) break;
    bool bad = false;
    const uint8_t kp = decide(kd, i, mode, snapshot, &bad);
    keep[i] = kp;
    if (bad) atomicMin(first_bad, static_cast<unsigned long long>(i));
    if (kp) {
      const uint64_t len = ikey_at(kd, i).len;
      cnt++;
      bytes += len >= 8 ? len - 8 : 0;
    }
  }
  for (int d = 32; d > 0; d >>= 1) {
    cnt += __shfl_xor(cnt, d, 64);
    bytes += __shfl_xor(bytes, d, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sc[w] = cnt;
    sb[w] = bytes;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t c = 0, b = 0;
    for (int q = 0; q < kSelBlock / 64; q++) {
      c += sc[q];
      b += sb[q];
    }
    blk_cnt[blockIdx.x] = c;
    blk_bytes[blockIdx.x] = b;
  }
}

// Per-block kept count / bytes from an existing keep[] (the gather's own
// pass, so a gather needs no state from the select call).
__global__ __launch_bounds__(kSelBlock) void count_kernel(KeyDesc kd, const uint8_t* __restrict__ keep,
                                                          uint64_t* __restrict__ blk_cnt,
                                                          uint64_t* __restrict__ blk_bytes) {
  __shared__ uint64_t sc[kSelBlock / 64], sb[kSelBlock / 64];
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kSelKeys;
  uint64_t cnt = 0, bytes = 0;
#pragma unroll
  for (int r = 0; r < kSelPer; r++) {
    const uint64_t i = base + r * kSelBlock + threadIdx.x;
    if (i < kd.n && keep[i]) {
      const uint64_t len = ikey_at(kd, i).len;
      cnt++;
      bytes += len >= 8 ? len - 8 : 0;
    }
  }
  for (int d = 32; d > 0; d >>= 1) {
    cnt += __shfl_xor(cnt, d, 64);
    bytes += __shfl_xor(bytes, d, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sc[w] = cnt;
    sb[w] = bytes;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t c = 0, b = 0;
    for (int q = 0; q < kSelBlock / 64; q++) {
      c += sc[q];
      b += sb[q];
    }
    blk_cnt[blockIdx.x] = c;
    blk_bytes[blockIdx.x] = b;
  }
}

// Pass 2: one workgroup: exclusive scan of the per-block sums (in place),
// totals in tot[0] (kept keys) / tot[1] (kept user-key bytes).
__global__ __launch_bounds__(1024) void block_scan_kernel(uint64_t* __restrict__ cnt,
                                                          uint64_t* __restrict__ bytes, uint64_t nb,
                                                          uint64_t* __restrict__ tot) {
  __shared__ uint64_t wc[16], wb[16];
  __shared__ uint64_t carry_c, carry_b;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) carry_c = carry_b = 0;
  __syncthreads();
  for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
    const uint64_t i = b0 + t;
    const uint64_t c = i < nb ? cnt[i] : 0, y = i < nb ? bytes[i] : 0;
    uint64_t ic = c, iy = y;
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t tc = __shfl_up(ic, d, 64), ty = __shfl_up(iy, d, 64);
      if (lane >= d) {
        ic += tc;
        iy += ty;
      }
    }
    if (lane == 63) {
      wc[w] = ic;
      wb[w] = iy;
    }
    __syncthreads();
    uint64_t oc = carry_c, oy = carry_b, sc = 0, sy = 0;
    for (int q = 0; q < 16; q++) {
      if (q < w) {
        oc += wc[q];
        oy += wb[q];
      }
      sc += wc[q];
      sy += wb[q];
    }
    if (i < nb) {
      cnt[i] = oc + ic - c;
      bytes[i] = oy + iy - y;
    }
    __syncthreads();
    if (t == 0) {
      carry_c += sc;
      carry_b += sy;
    }
    __syncthreads();
  }
  if (t == 0) {
    tot[0] = carry_c;
    tot[1] = carry_b;
  }
}

// Pass 3: per block, local exclusive scan of (keep, user-key bytes) in key
// order, then copy ExtractUserKey(key) of every kept key to its place.
// out_offsets (variable-length output) gets n_kept + 1 entries.
__global__ __launch_bounds__(kSelBlock) void gather_kernel(KeyDesc kd, const uint8_t* __restrict__ keep,
                                                           const uint64_t* __restrict__ blk_cnt,
                                                           const uint64_t* __restrict__ blk_bytes,
                                                           uint8_t* __restrict__ out,
                                                           uint64_t* __restrict__ out_offsets,
                                                           const uint64_t* __restrict__ tot) {
  __shared__ uint64_t wc[kSelBlock / 64], wb[kSelBlock / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kSelKeys;
  // thread t owns keys base + t*kSelPer .. +kSelPer (contiguous, in order)
  uint64_t c = 0, y = 0;
  uint8_t kp[kSelPer];
  uint64_t ul[kSelPer];
#pragma unroll
  for (int r = 0; r < kSelPer; r++) {
    const uint64_t i = base + static_cast<uint64_t>(t) * kSelPer + r;
    kp[r] = i < kd.n ? keep[i] : 0;
    const uint64_t len = i < kd.n ? ikey_at(kd, i).len : 0;
    ul[r] = len >= 8 ? len - 8 : 0;
    if (kp[r]) {
      c++;
      y += ul[r];
    }
  }
  uint64_t ic = c, iy = y;
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t tc = __shfl_up(ic, d, 64), ty = __shfl_up(iy, d, 64);
    if (lane >= d) {
      ic += tc;
      iy += ty;
    }
  }
  if (lane == 63) {
    wc[w] = ic;
    wb[w] = iy;
  }
  __syncthreads();
  uint64_t pc = blk_cnt[blockIdx.x], py = blk_bytes[blockIdx.x];
  for (int q = 0; q < w; q++) {
    pc += wc[q];
    py += wb[q];
  }
  pc += ic - c;
  py += iy - y;
#pragma unroll
  for (int r = 0; r < kSelPer; r++) {
    if (!kp[r]) continue;
    const uint64_t i = base + static_cast<uint64_t>(t) * kSelPer + r;
    const IKey k = ikey_at(kd, i);
    uint8_t* dst = out + (out_offsets ? py : pc * ul[r]);
    for (uint64_t j = 0; j < ul[r]; j++) dst[j] = k.p[j];
    if (out_offsets) out_offsets[pc] = py;
    pc++;
    py += ul[r];
  }
  if (out_offsets && blockIdx.x == gridDim.x - 1 && t == 0) out_offsets[tot[0]] = tot[1];
}

}  // namespace

uint64_t select_blocks(uint64_t n) { return (n + kSelKeys - 1) / kSelKeys; }

hipError_t launch_key_select(KeyDesc kd, int mode, uint64_t snapshot, uint8_t* keep, uint64_t* blk_cnt,
                             uint64_t* blk_bytes, unsigned long long* first_bad, uint64_t* tot,
                             hipStream_t s) {
  const uint64_t nb = select_blocks(kd.n);
  if (nb == 0) return hipSuccess;
  select_kernel<<<static_cast<unsigned>(nb), kSelBlock, 0, s>>>(kd, mode, snapshot, keep, blk_cnt,
                                                               blk_bytes, first_bad);
  block_scan_kernel<<<1, 1024, 0, s>>>(blk_cnt, blk_bytes, nb, tot);
  return hipGetLastError();
}

hipError_t launch_key_gather(KeyDesc kd, const uint8_t* keep, uint64_t* blk_cnt, uint64_t* blk_bytes,
                             uint8_t* out, uint64_t* out_offsets, uint64_t* tot, hipStream_t s) {
  const uint64_t nb = select_blocks(kd.n);
  if (nb == 0) return hipSuccess;
  count_kernel<<<static_cast<unsigned>(nb), kSelBlock, 0, s>>>(kd, keep, blk_cnt, blk_bytes);
  block_scan_kernel<<<1, 1024, 0, s>>>(blk_cnt, blk_bytes, nb, tot);
  gather_kernel<<<static_cast<unsigned>(nb), kSelBlock, 0, s>>>(kd, keep, blk_cnt, blk_bytes, out,
                                                               out_offsets, tot);
  return hipGetLastError();
}

}  // namespace dlsm
