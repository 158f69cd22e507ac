/*
 * oracle/bloom_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker and the
 * CPU baseline).  Nothing under dlsm_amd/ links, loads or calls this file; the
 * product path is the HIP library and fails loudly when it is missing.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * Plain-C restatement of dLSM's (TimberSaw) SSTable Bloom-filter hot path.
 * Every function cites the reference file:line it restates.  Parity is pinned
 * against (a) the reference's own known-answer tests (util/hash_test.cc:23-38),
 * (b) golden fixtures produced by the reference sources compiled in place
 * (oracle/_ref, see oracle/build_ref.sh, tests/golden/make_golden.py) and
 * (c) the survey-time FNV-1a digests of full_filter_block.cc output
 * (SURVEY.md §6.2).
 *
 * The CPU-baseline entry points keep the reference's cost structure: a full
 * filter build hashes every key into a vector (AddKey) and then scatters it
 * (Finish); a probe re-hashes the key for every filter (KeyMayMatch).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_E_ARG (-1)
#define ORC_E_CAPACITY (-2)
#define ORC_E_CORRUPT (-3)

/* port/port_posix.h:301-306 -- x86 value; pinned, it is part of the format. */
#define ORC_CACHE_LINE_SIZE 64u
#define ORC_BLOOM_SEED 0xbc9f1d34u /* include/TimberSaw/filter_policy.h:26-28 */

static inline uint32_t dec32(const uint8_t* p) { /* util/coding.h:130-142 */
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}
static inline void enc32(uint8_t* p, uint32_t v) { /* util/coding.h:184-193 */
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

/* util/hash.cc:22-62 -- MurmurHash1 variant; tail bytes sign-extended. */
uint32_t orc_hash(const uint8_t* data, size_t n, uint32_t seed) {
  const uint32_t m = 0xc6a4a793u;
  uint32_t h = seed ^ (uint32_t)((uint64_t)n * m);
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    h += dec32(data + i);
    h *= m;
    h ^= (h >> 16);
  }
  switch (n - i) {
    case 3:
      h += (uint32_t)(int32_t)(int8_t)data[i + 2] << 16;
      /* fallthrough */
    case 2:
      h += (uint32_t)(int32_t)(int8_t)data[i + 1] << 8;
      /* fallthrough */
    case 1:
      h += (uint32_t)(int32_t)(int8_t)data[i];
      h *= m;
      h ^= (h >> 24);
      break;
    default:
      break;
  }
  return h;
}

/* include/TimberSaw/filter_policy.h:26-28 */
uint32_t orc_bloom_hash(const uint8_t* data, size_t n) {
  return orc_hash(data, n, ORC_BLOOM_SEED);
}

/* util/bloom_impl.h:351-357 LegacyNoLocalityBloomImpl::ChooseNumProbes (full
 * filter, via table/full_filter_block.cc:19). */
int orc_full_num_probes(int bits_per_key) {
  int k = (int)(bits_per_key * 0.69);
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return k;
}

/* util/bloom.cc:16-21 BloomFilterPolicy ctor (size_t cast of the same product). */
int orc_legacy_num_probes(int bits_per_key) {
  double p = bits_per_key * 0.69;
  size_t k = p < 0 ? 0 : (size_t)p;
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return (int)k;
}

/* table/full_filter_block.cc:61-92 GetTotalBitsForLocality + CalculateSpace.
 * All arithmetic in u32 exactly as the reference (int*int product wraps). */
uint32_t orc_full_calc_space(int num_entry, int bits_per_key, uint32_t* total_bits,
                             uint32_t* num_lines) {
  if (num_entry != 0) {
    uint32_t tb = (uint32_t)num_entry * (uint32_t)bits_per_key;
    uint32_t nl = (tb + ORC_CACHE_LINE_SIZE * 8u - 1u) / (ORC_CACHE_LINE_SIZE * 8u);
    if (nl % 2u == 0u) nl++;
    *total_bits = nl * (ORC_CACHE_LINE_SIZE * 8u);
    *num_lines = *total_bits / (ORC_CACHE_LINE_SIZE * 8u);
  } else {
    *total_bits = 0;
    *num_lines = 0;
  }
  return *total_bits / 8u + 5u;
}

/* util/bloom_impl.h:427-443 LegacyLocalityBloomImpl<false>::AddHash with
 * log2_cache_line_bytes = log2(64) = 6 (full_filter_block.cc:50-60). */
static inline void locality_add_hash(uint32_t h, uint32_t num_lines, int num_probes,
                                     uint8_t* data) {
  uint8_t* at = data + ((h % num_lines) << 6);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int i = 0; i < num_probes; ++i) {
    const uint32_t bitpos = h & 511u;
    at[bitpos / 8] |= (uint8_t)(1u << (bitpos % 8));
    h += delta;
  }
}

/* Key accessor for a packed key set: fixed stride when offsets == NULL. */
static inline const uint8_t* key_at(const uint8_t* bytes, const uint64_t* offsets,
                                    uint32_t stride, uint64_t i, size_t* len) {
  if (offsets) {
    *len = (size_t)(offsets[i + 1] - offsets[i]);
    return bytes + offsets[i];
  }
  *len = stride;
  return bytes + (uint64_t)stride * i;
}

/* Consecutive-distinct hash count -- table/full_filter_block.cc:39-49 AddKey
 * (a hash is dropped only when equal to the immediately preceding kept one). */
uint64_t orc_full_dedup_count(const uint8_t* bytes, const uint64_t* offsets,
                              uint32_t stride, uint64_t n) {
  uint64_t cnt = 0;
  uint32_t prev = 0;
  for (uint64_t i = 0; i < n; i++) {
    size_t len;
    const uint8_t* k = key_at(bytes, offsets, stride, i, &len);
    uint32_t h = orc_bloom_hash(k, len);
    if (cnt == 0 || h != prev) {
      cnt++;
      prev = h;
    }
  }
  return cnt;
}

/* Full-filter size for n keys (dedup count) -- full_filter_block.cc:93-96. */
uint64_t orc_full_filter_bytes(uint64_t n_dedup, int bits_per_key, uint32_t* num_lines) {
  uint32_t tb, nl;
  uint32_t sz = orc_full_calc_space((int)(uint32_t)n_dedup, bits_per_key, &tb, &nl);
  if (num_lines) *num_lines = nl;
  return sz;
}

/* FullFilterBlockBuilder: AddKey* then Finish -- table/full_filter_block.cc:39-141.
 * `out` is the caller's slot; like every reference caller
 * (table_builder_computeside.cc:38,48) it is zeroed first.  Returns the filter
 * length (L*64+5) or a negative status. */
int64_t orc_full_build(const uint8_t* bytes, const uint64_t* offsets, uint32_t stride,
                       uint64_t n, int bits_per_key, uint8_t* out, uint64_t out_cap) {
  uint32_t* hashes = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!hashes) return ORC_E_ARG;
  uint64_t cnt = 0;
  for (uint64_t i = 0; i < n; i++) { /* AddKey: hash + consecutive dedup push */
    size_t len;
    const uint8_t* k = key_at(bytes, offsets, stride, i, &len);
    uint32_t h = orc_bloom_hash(k, len);
    if (cnt == 0 || h != hashes[cnt - 1]) hashes[cnt++] = h;
  }
  uint32_t total_bits, num_lines;
  orc_full_calc_space((int)(uint32_t)cnt, bits_per_key, &total_bits, &num_lines);
  uint64_t len = (uint64_t)(total_bits / 8u) + 5u;
  if (len > out_cap) {
    free(hashes);
    return ORC_E_CAPACITY;
  }
  memset(out, 0, (size_t)len);
  int k = orc_full_num_probes(bits_per_key);
  if (total_bits != 0 && num_lines != 0) { /* Finish: scatter */
    for (uint64_t i = 0; i < cnt; i++) locality_add_hash(hashes[i], num_lines, k, out);
  }
  out[total_bits / 8u] = (uint8_t)(int8_t)k;
  enc32(out + total_bits / 8u + 1u, num_lines);
  free(hashes);
  return (int64_t)len;
}

/* FullFilterBlockReader ctor metadata parse -- table/full_filter_block.cc:186-252.
 * Cases where the reference exit(1)s or whose later KeyMayMatch is undefined
 * (len <= 5 -> h % 0 or an out-of-range read) return ORC_E_CORRUPT.  When
 * num_lines*64 != len but len % num_lines == 0 the reference leaves
 * log2_cache_line_size_ at its initialiser 0 (full_filter_block.h:85); we
 * reproduce that. */
int orc_full_reader_parse(const uint8_t* f, uint64_t len_with_meta64, int* num_probes,
                          uint32_t* num_lines, int* log2_line) {
  if (len_with_meta64 < 5 || len_with_meta64 > 0xffffffffull) return ORC_E_CORRUPT;
  uint32_t len_with_meta = (uint32_t)len_with_meta64;
  int k = (int)(int8_t)f[len_with_meta - 5];
  if (k < 1) return ORC_E_CORRUPT;
  uint32_t len = len_with_meta - 5;
  uint32_t L = dec32(f + len_with_meta - 4);
  int lg;
  if (L * ORC_CACHE_LINE_SIZE == len) {
    lg = 6;
    if (L == 0 || (uint64_t)L * ORC_CACHE_LINE_SIZE != len) return ORC_E_CORRUPT;
  } else if (L == 0 || len % L != 0) {
    return ORC_E_CORRUPT;
  } else {
    lg = 0;
  }
  *num_probes = k;
  *num_lines = L;
  *log2_line = lg;
  return ORC_OK;
}

/* FullFilterBlockReader::KeyMayMatch -- table/full_filter_block.cc:269-284 ->
 * util/bloom_impl.h:445-481 (PrepareHashMayMatch + HashMayMatchPrepared). */
static inline int full_hash_may_match(uint32_t h, const uint8_t* data, int k, uint32_t L,
                                      int lg) {
  const uint8_t* at = data + ((h % L) << lg);
  const uint32_t mask = (1u << (lg + 3)) - 1u;
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int i = 0; i < k; ++i) {
    const uint32_t bitpos = h & mask;
    if ((at[bitpos / 8] & (1u << (bitpos % 8))) == 0) return 0;
    h += delta;
  }
  return 1;
}

int orc_full_key_may_match(const uint8_t* filter, uint64_t flen, const uint8_t* key,
                           size_t klen) {
  int k, lg;
  uint32_t L;
  int st = orc_full_reader_parse(filter, flen, &k, &L, &lg);
  if (st) return st;
  return full_hash_may_match(orc_bloom_hash(key, klen), filter, k, L, lg);
}

/* util/bloom.cc:25-55 BloomFilterPolicy::CreateFilter.  The reference ORs into
 * the (un-zeroed, :36-38) region after dst's current size; callers hand it
 * zeroed slots, so this writes a fresh filter: `bytes` data bytes + the k byte. */
uint64_t orc_legacy_filter_bytes(uint64_t n, int bits_per_key) {
  uint64_t bits = n * (uint64_t)(int64_t)bits_per_key;
  if (bits < 64) bits = 64;
  return (bits + 7) / 8 + 1;
}

int64_t orc_legacy_build(const uint8_t* bytes, const uint64_t* offsets, uint32_t stride,
                         uint64_t n, int bits_per_key, uint8_t* out, uint64_t out_cap) {
  uint64_t bits = n * (uint64_t)(int64_t)bits_per_key;
  if (bits < 64) bits = 64;
  uint64_t nbytes = (bits + 7) / 8;
  bits = nbytes * 8;
  if (nbytes + 1 > out_cap) return ORC_E_CAPACITY;
  memset(out, 0, (size_t)nbytes + 1);
  int k = orc_legacy_num_probes(bits_per_key);
  for (uint64_t i = 0; i < n; i++) {
    size_t len;
    const uint8_t* key = key_at(bytes, offsets, stride, i, &len);
    uint32_t h = orc_bloom_hash(key, len);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (int j = 0; j < k; j++) {
      const uint32_t bitpos = (uint32_t)((uint64_t)h % bits);
      out[bitpos / 8] |= (uint8_t)(1u << (bitpos % 8));
      h += delta;
    }
  }
  out[nbytes] = (uint8_t)(int8_t)k;
  return (int64_t)(nbytes + 1);
}

/* util/bloom.cc:57-81 BloomFilterPolicy::KeyMayMatch.  k is read through a
 * (signed) char into size_t, so k byte >= 0x80 is "k > 30" -> match. */
int orc_legacy_key_may_match(const uint8_t* filter, uint64_t len, const uint8_t* key,
                             size_t klen) {
  if (len < 2) return 0;
  const uint64_t bits = (len - 1) * 8;
  const int64_t ks = (int64_t)(int8_t)filter[len - 1];
  if (ks < 0 || ks > 30) return 1;
  uint32_t h = orc_bloom_hash(key, klen);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int64_t j = 0; j < ks; j++) {
    const uint32_t bitpos = (uint32_t)((uint64_t)h % bits);
    if ((filter[bitpos / 8] & (1u << (bitpos % 8))) == 0) return 0;
    h += delta;
  }
  return 1;
}

/* ---------------------------------------------------------------------------
 * Workload generators (benchmarks/db_bench.cc, util/random.h).
 * ------------------------------------------------------------------------- */

/* benchmarks/db_bench.cc:677-711 GenerateKeyFromInt: big-endian v in the first
 * min(key_size, 8) bytes, then '0' padding. */
void orc_dbbench_key(uint64_t v, int key_size, uint8_t* out) {
  int fill = key_size < 8 ? key_size : 8;
  for (int i = 0; i < fill; i++) out[i] = (uint8_t)(v >> ((fill - i - 1) * 8));
  if (key_size > fill) memset(out + fill, '0', (size_t)(key_size - fill));
}

/* Keys v = first + i*step for i < n, packed at stride key_size. */
void orc_gen_keys_arith(uint64_t first, uint64_t step, uint64_t n, int key_size,
                        uint8_t* out) {
  for (uint64_t i = 0; i < n; i++)
    orc_dbbench_key(first + i * step, key_size, out + i * (uint64_t)key_size);
}

/* std::mt19937_64 (the engine behind util/random.h:140-165 Random64), the
 * published MT19937-64 algorithm with the C++ standard's seeding. */
typedef struct {
  uint64_t mt[312];
  int idx;
} orc_mt64;

void orc_mt64_seed(orc_mt64* s, uint64_t seed) {
  s->mt[0] = seed;
  for (int i = 1; i < 312; i++)
    s->mt[i] = 6364136223846793005ull * (s->mt[i - 1] ^ (s->mt[i - 1] >> 62)) + (uint64_t)i;
  s->idx = 312;
}

uint64_t orc_mt64_next(orc_mt64* s) {
  if (s->idx >= 312) {
    for (int i = 0; i < 312; i++) {
      uint64_t x = (s->mt[i] & 0xFFFFFFFF80000000ull) | (s->mt[(i + 1) % 312] & 0x7FFFFFFFull);
      uint64_t xa = x >> 1;
      if (x & 1ull) xa ^= 0xB5026F5AA96619E9ull;
      s->mt[i] = s->mt[(i + 156) % 312] ^ xa;
    }
    s->idx = 0;
  }
  uint64_t y = s->mt[s->idx++];
  y ^= (y >> 29) & 0x5555555555555555ull;
  y ^= (y << 17) & 0x71D67FFFEDA60000ull;
  y ^= (y << 37) & 0xFFF7EEE000000000ull;
  y ^= (y >> 43);
  return y;
}

size_t orc_mt64_state_size(void) { return sizeof(orc_mt64); }

/* Lookup stream of SURVEY.md §8d config 3: v = mt19937_64(seed)() mod modulus. */
void orc_gen_values_mt(uint64_t seed, uint64_t modulus, uint64_t n, uint64_t* out) {
  orc_mt64 s;
  orc_mt64_seed(&s, seed);
  for (uint64_t i = 0; i < n; i++) out[i] = orc_mt64_next(&s) % modulus;
}

void orc_gen_keys_from_values(const uint64_t* v, uint64_t n, int key_size, uint8_t* out) {
  for (uint64_t i = 0; i < n; i++) orc_dbbench_key(v[i], key_size, out + i * (uint64_t)key_size);
}

/* FNV-1a 64 digest used for the survey-time sanity digests. */
uint64_t orc_fnv1a64(const uint8_t* p, uint64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < n; i++) {
    h ^= p[i];
    h *= 1099511628211ull;
  }
  return h;
}

/* ---------------------------------------------------------------------------
 * CPU baseline drivers (reference cost structure, pthreads).
 * ------------------------------------------------------------------------- */

typedef struct {
  const uint8_t* const* keys; /* per table, fixed stride */
  const uint64_t* n;
  uint32_t stride;
  int bits_per_key;
  uint8_t* const* out;
  const uint64_t* out_cap;
  int64_t* out_len;
  int n_tables;
  int tid, nthreads;
} build_job;

static void* build_worker(void* arg) {
  build_job* j = (build_job*)arg;
  for (int t = j->tid; t < j->n_tables; t += j->nthreads)
    j->out_len[t] = orc_full_build(j->keys[t], NULL, j->stride, j->n[t], j->bits_per_key,
                                   j->out[t], j->out_cap[t]);
  return NULL;
}

/* Build n_tables independent full filters, table t on thread t mod nthreads. */
int orc_full_build_many(const uint8_t* const* keys, const uint64_t* n, uint32_t stride,
                        int n_tables, int bits_per_key, uint8_t* const* out,
                        const uint64_t* out_cap, int64_t* out_len, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t th[256];
  build_job jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int i = 0; i < nthreads; i++) {
    build_job b = {keys, n, stride, bits_per_key, out, out_cap, out_len, n_tables, i, nthreads};
    jobs[i] = b;
    if (nthreads == 1) build_worker(&jobs[0]);
    else pthread_create(&th[i], NULL, build_worker, &jobs[i]);
  }
  if (nthreads > 1)
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  return ORC_OK;
}

typedef struct {
  const uint8_t* const* filters;
  const uint64_t* flen;
  int n_filters;
  const uint8_t* keys;
  uint32_t stride;
  uint64_t begin, end;
  uint8_t* mask;
  int status;
} probe_job;

static void* probe_worker(void* arg) {
  probe_job* j = (probe_job*)arg;
  int kf[64], lgf[64];
  uint32_t Lf[64];
  j->status = ORC_OK;
  for (int f = 0; f < j->n_filters; f++) {
    int st = orc_full_reader_parse(j->filters[f], j->flen[f], &kf[f], &Lf[f], &lgf[f]);
    if (st) {
      j->status = st;
      return NULL;
    }
  }
  const int mbytes = (j->n_filters + 7) / 8;
  for (uint64_t i = j->begin; i < j->end; i++) {
    const uint8_t* key = j->keys + i * (uint64_t)j->stride;
    uint8_t* m = j->mask + i * (uint64_t)mbytes;
    memset(m, 0, (size_t)mbytes);
    for (int f = 0; f < j->n_filters; f++) {
      /* re-hash per filter, like Table::InternalGet -> KeyMayMatch */
      uint32_t h = orc_bloom_hash(key, j->stride);
      if (full_hash_may_match(h, j->filters[f], kf[f], Lf[f], lgf[f])) m[f / 8] |= (uint8_t)(1u << (f % 8));
    }
  }
  return NULL;
}

/* Probe n fixed-stride keys against F full filters; mask is n * ceil(F/8)
 * bytes, bit f = filter f's KeyMayMatch. */
int orc_full_probe_many(const uint8_t* const* filters, const uint64_t* flen, int n_filters,
                        const uint8_t* keys, uint32_t stride, uint64_t n, uint8_t* mask,
                        int nthreads) {
  if (n_filters < 1 || n_filters > 64) return ORC_E_ARG;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  probe_job jobs[256];
  for (int i = 0; i < nthreads; i++) {
    probe_job p = {filters, flen, n_filters, keys, stride, n * (uint64_t)i / (uint64_t)nthreads,
                   n * (uint64_t)(i + 1) / (uint64_t)nthreads, mask, 0};
    jobs[i] = p;
    if (nthreads == 1) probe_worker(&jobs[0]);
    else pthread_create(&th[i], NULL, probe_worker, &jobs[i]);
  }
  int st = ORC_OK;
  for (int i = 0; i < nthreads; i++) {
    if (nthreads > 1) pthread_join(th[i], NULL);
    if (jobs[i].status) st = jobs[i].status;
  }
  return st;
}

/* Legacy-format batch probe (one filter), for parity tests. */
int orc_legacy_probe(const uint8_t* filter, uint64_t flen, const uint8_t* bytes,
                     const uint64_t* offsets, uint32_t stride, uint64_t n, uint8_t* out) {
  for (uint64_t i = 0; i < n; i++) {
    size_t len;
    const uint8_t* k = key_at(bytes, offsets, stride, i, &len);
    out[i] = (uint8_t)orc_legacy_key_may_match(filter, flen, k, len);
  }
  return ORC_OK;
}

/* Full-format probe of a variable-length key set against F filters. */
int orc_full_probe_var(const uint8_t* const* filters, const uint64_t* flen, int n_filters,
                       const uint8_t* bytes, const uint64_t* offsets, uint32_t stride,
                       uint64_t n, uint8_t* mask) {
  if (n_filters < 1 || n_filters > 64) return ORC_E_ARG;
  int kf[64], lgf[64];
  uint32_t Lf[64];
  for (int f = 0; f < n_filters; f++) {
    int st = orc_full_reader_parse(filters[f], flen[f], &kf[f], &Lf[f], &lgf[f]);
    if (st) return st;
  }
  const int mbytes = (n_filters + 7) / 8;
  for (uint64_t i = 0; i < n; i++) {
    size_t len;
    const uint8_t* key = key_at(bytes, offsets, stride, i, &len);
    uint8_t* m = mask + i * (uint64_t)mbytes;
    memset(m, 0, (size_t)mbytes);
    uint32_t h = orc_bloom_hash(key, len);
    for (int f = 0; f < n_filters; f++)
      if (full_hash_may_match(h, filters[f], kf[f], Lf[f], lgf[f])) m[f / 8] |= (uint8_t)(1u << (f % 8));
  }
  return ORC_OK;
}

/* ---------------------------------------------------------------------------
 * Filter-block trailer: crc32c (Castagnoli, reflected
 * poly 0x82f63b78) -- util/crc32c.h:17-37 semantics, bitwise table form.
 * ------------------------------------------------------------------------- */
static uint32_t crc_table[256];
static int crc_init_done = 0;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : c >> 1;
    crc_table[i] = c;
  }
  crc_init_done = 1;
}
uint32_t orc_crc32c_extend(uint32_t crc, const uint8_t* p, uint64_t n) {
  if (!crc_init_done) crc_init();
  uint32_t c = ~crc;
  for (uint64_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return ~c;
}
uint32_t orc_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

/* ------------------------------------------------------------------------
 * Internal-key selection: the loops that feed TableBuilder::Add, restated
 * statement by statement (sequential state machine, as the reference runs it).
 *   policy 0 = FlushJob::BuildTable          db/memtable_list.cc:855-886
 *   policy 1 = DBImpl::DoCompactionWork      db/db_impl.cc:3500-3562
 * ParseInternalKey db/dbformat.h:451-461.  keep[i] = 1 iff Add(key i) runs.
 * Returns the number kept; *first_corrupt = index of the first unparsable key
 * or UINT64_MAX.  For the flush the reference stops at that key (IOError,
 * builder deleted): keep[] past it stays 0 and the return value is -1.
 * ------------------------------------------------------------------------ */
static int orc_parse_internal_key(const uint8_t* k, size_t n, uint64_t* seq) {
  if (n < 8) return 0;
  uint64_t num = 0;
  for (int b = 0; b < 8; b++) num |= (uint64_t)k[n - 8 + b] << (8 * b); /* DecodeFixed64 */
  *seq = num >> 8;
  return (num & 0xff) <= 1; /* c <= kTypeValue */
}

int64_t orc_internal_keys_select(const uint8_t* bytes, const uint64_t* offsets, uint32_t stride,
                                 uint64_t n, int policy, uint64_t smallest_snapshot,
                                 uint8_t* keep, uint64_t* first_corrupt) {
  const uint64_t kMaxSequenceNumber = ((uint64_t)1 << 56) - 1; /* db/dbformat.h */
  const uint8_t* cur = NULL; /* current_user_key */
  size_t cur_len = 0;
  int has_current_user_key = 0;
  uint64_t last_sequence_for_key = kMaxSequenceNumber;
  int64_t kept = 0;
  *first_corrupt = UINT64_MAX;
  for (uint64_t i = 0; i < n; i++) keep[i] = 0;
  for (uint64_t i = 0; i < n; i++) {
    size_t len;
    const uint8_t* key = key_at(bytes, offsets, stride, i, &len);
    uint64_t seq = 0;
    int drop = 0;
    if (!orc_parse_internal_key(key, len, &seq)) {
      if (*first_corrupt == UINT64_MAX) *first_corrupt = i;
      has_current_user_key = 0;
      if (policy == 0) return -1; /* flush: "Corrupt key value detected", break */
      last_sequence_for_key = kMaxSequenceNumber;
    } else {
      const size_t ulen = len - 8;
      if (!has_current_user_key || ulen != cur_len || memcmp(key, cur, ulen) != 0) {
        cur = key; /* current_user_key.assign(ikey.user_key) */
        cur_len = ulen;
        has_current_user_key = 1;
        last_sequence_for_key = kMaxSequenceNumber;
      } else if (policy == 0) {
        drop = 1;
      }
      if (policy == 1) {
        if (last_sequence_for_key <= smallest_snapshot) drop = 1; /* (A) */
        last_sequence_for_key = seq;
      }
    }
    if (!drop) {
      keep[i] = 1;
      kept++;
    }
  }
  return kept;
}

/* ------------------------------------------------------------------------
 * Version::ForEachOverlapping + FindFile + Table::InternalGet's filter check,
 * restated (db/version_set.cc:95-118, 268-321; table/table.cc:350-358;
 * db/dbformat.cc:41-57 InternalKeyComparator, :111-128 LookupKey).
 * The layout of orc_version_file matches dlsm_version_file.
 * For each key: out_mask bit s for every file Match() would be called on whose
 * filter passes the key (slot s: level-0 rank newest first, then
 * n_l0 + level - 1); out_level_file[i*5 + level-1] = FindFile's pick inside
 * the level or UINT32_MAX.
 * ------------------------------------------------------------------------ */
typedef struct {
  const uint8_t* smallest;
  uint64_t smallest_len;
  const uint8_t* largest;
  uint64_t largest_len;
  uint64_t largest_trailer;
  uint64_t number;
  int32_t level;
  int32_t reserved;
  const uint8_t* filter;
  uint64_t filter_len;
} orc_version_file;

static int orc_bytewise(const uint8_t* a, size_t an, const uint8_t* b, size_t bn) { /* util/comparator.cc */
  size_t n = an < bn ? an : bn;
  int r = n ? memcmp(a, b, n) : 0;
  if (r == 0) r = an < bn ? -1 : (an > bn ? 1 : 0);
  return r;
}

/* InternalKeyComparator::Compare on (user key, trailer) pairs */
static int orc_icmp(const uint8_t* a, size_t an, uint64_t anum, const uint8_t* b, size_t bn, uint64_t bnum) {
  int r = orc_bytewise(a, an, b, bn);
  if (r == 0) {
    if (anum > bnum) r = -1;
    else if (anum < bnum) r = +1;
  }
  return r;
}

int orc_version_probe(const orc_version_file* files, int n_files, const uint8_t* bytes,
                      const uint64_t* offsets, uint32_t stride, uint32_t suffix, uint64_t n,
                      uint64_t snapshot, uint64_t* out_mask, uint32_t* out_level_file) {
  enum { kNumLevels = 6 };
  int l0[64], n_l0 = 0;
  int* lvl[kNumLevels] = {0};  /* Version::files_[level], any size */
  int nlvl[kNumLevels] = {0};
  for (int level = 1; level < kNumLevels; level++) {
    lvl[level] = (int*)malloc(sizeof(int) * (size_t)(n_files > 0 ? n_files : 1));
    if (!lvl[level]) {
      for (int b = 1; b < level; b++) free(lvl[b]);
      return ORC_E_ARG;
    }
  }
  for (int f = 0; f < n_files; f++) {
    if (files[f].level == 0) {
      if (n_l0 == 64) {
        for (int b = 1; b < kNumLevels; b++) free(lvl[b]);
        return ORC_E_ARG;
      }
      l0[n_l0++] = f;
    } else {
      lvl[files[f].level][nlvl[files[f].level]++] = f;
    }
  }
  /* level-0 slot = rank by number, largest first (NewestFirst) */
  for (int a = 1; a < n_l0; a++)
    for (int b = a; b > 0 && files[l0[b]].number > files[l0[b - 1]].number; b--) {
      int t = l0[b]; l0[b] = l0[b - 1]; l0[b - 1] = t;
    }
  const uint64_t tnum = (snapshot << 8) | 1; /* PackSequenceAndType(s, kValueTypeForSeek) */
  for (uint64_t i = 0; i < n; i++) {
    size_t len;
    const uint8_t* key = key_at(bytes, offsets, stride, i, &len);
    size_t ulen = len > suffix ? len - suffix : 0;
    uint64_t m = 0;
    for (int j = 0; j < n_l0; j++) { /* tmp: overlapping level-0 files, newest first */
      const orc_version_file* F = &files[l0[j]];
      if (orc_bytewise(key, ulen, F->smallest, F->smallest_len) >= 0 &&
          orc_bytewise(key, ulen, F->largest, F->largest_len) <= 0) {
        /* Match -> TableCache::Get -> Table::InternalGet: filter check */
        if (!F->filter || orc_full_key_may_match(F->filter, F->filter_len, key, ulen)) m |= 1ull << j;
      }
    }
    for (int level = 1; level < kNumLevels; level++) {
      uint32_t pick = UINT32_MAX;
      int num_files = nlvl[level];
      if (num_files != 0) {
        /* FindFile: left = 0, right = files.size()-1 */
        uint32_t left = 0, right = (uint32_t)num_files - 1;
        while (left < right) {
          uint32_t mid = (left + right) / 2;
          const orc_version_file* F = &files[lvl[level][mid]];
          if (orc_icmp(F->largest, F->largest_len, F->largest_trailer, key, ulen, tnum) < 0) left = mid + 1;
          else right = mid;
        }
        uint32_t index = right;
        if (index < (uint32_t)num_files) {
          const orc_version_file* F = &files[lvl[level][index]];
          if (orc_bytewise(key, ulen, F->smallest, F->smallest_len) < 0) {
            /* All of "f" is past any data for user_key */
          } else {
            pick = index;
            if (!F->filter || orc_full_key_may_match(F->filter, F->filter_len, key, ulen))
              m |= 1ull << (n_l0 + level - 1);
          }
        }
      }
      if (out_level_file) out_level_file[i * (kNumLevels - 1) + (level - 1)] = pick;
    }
    out_mask[i] = m;
  }
  for (int level = 1; level < kNumLevels; level++) free(lvl[level]);
  return 0;
}

/* ------------------------------------------------------------------------
 * Legacy block-based filter block, restated: FilterBlockBuilder /
 * FilterBlockReader (table/filter_block.cc:14-142) driven the way
 * TableBuilder drives it -- the keys of data block b are AddKey'ed, then
 * StartBlock(block_end_offset[b]) runs (TableBuilder::Flush); keys past the
 * last block end are added before Finish().
 * policy 0 = BloomFilterPolicy(bits_per_key) (util/bloom.cc);
 * policy 1 = TestHashFilter of table/filter_block_test.cc:17-36 (one
 * Fixed32(Hash(key, 1)) per key), so that file's expectations apply verbatim.
 * ------------------------------------------------------------------------ */
typedef struct {
  uint8_t* result; uint64_t size, cap;           /* Slice result */
  uint32_t* offs; uint64_t n_offs, cap_offs;     /* filter_offsets_ */
  uint64_t key_begin, key_end;                   /* start_: pending keys [begin, end) */
  const uint8_t* bytes; const uint64_t* offsets; uint32_t stride;
  int policy, bpk, err;
} orc_fbb;

static void fbb_put32(orc_fbb* b, uint32_t v) {
  if (b->size + 4 > b->cap) { b->err = 1; return; }
  enc32(b->result + b->size, v);
  b->size += 4;
}

static void fbb_generate(orc_fbb* b) { /* GenerateFilter */
  if (b->n_offs == b->cap_offs) { b->err = 1; return; }
  const uint64_t num_keys = b->key_end - b->key_begin;
  b->offs[b->n_offs++] = (uint32_t)b->size; /* both paths push result.size() first */
  if (num_keys == 0) return;                /* fast path */
  if (b->policy == 0) {
    /* CreateFilter on the flattened sub-range (keys re-based like tmp_keys_) */
    const uint64_t need = orc_legacy_filter_bytes(num_keys, b->bpk);
    if (b->size + need > b->cap) { b->err = 1; return; }
    const uint8_t* base = b->offsets ? b->bytes : b->bytes + b->key_begin * b->stride;
    const uint64_t* offs = b->offsets ? b->offsets + b->key_begin : NULL;
    orc_legacy_build(base, offs, b->stride, num_keys, b->bpk, b->result + b->size, need);
    b->size += need;
  } else {
    for (uint64_t i = b->key_begin; i < b->key_end; i++) {
      size_t len;
      const uint8_t* k = key_at(b->bytes, b->offsets, b->stride, i, &len);
      fbb_put32(b, orc_hash(k, len, 1));
    }
  }
  b->key_begin = b->key_end;
}

static void fbb_start_block(orc_fbb* b, uint64_t block_offset) { /* StartBlock */
  const uint64_t filter_index = block_offset / 2048; /* kFilterBase = 1 << 11 */
  if (filter_index < b->n_offs) { b->err = 2; return; } /* assert */
  while (filter_index > b->n_offs && !b->err) fbb_generate(b);
}

int64_t orc_filter_block_build(const uint8_t* bytes, const uint64_t* offsets, uint32_t stride,
                               uint64_t n, const uint64_t* block_key_end,
                               const uint64_t* block_end_offset, int n_blocks, int policy,
                               int bits_per_key, uint8_t* out, uint64_t out_cap) {
  orc_fbb b;
  memset(&b, 0, sizeof(b));
  b.result = out; b.cap = out_cap;
  b.cap_offs = 1 << 22;
  b.offs = (uint32_t*)malloc(sizeof(uint32_t) * b.cap_offs);
  b.bytes = bytes; b.offsets = offsets; b.stride = stride; b.policy = policy; b.bpk = bits_per_key;
  if (!b.offs) return ORC_E_ARG;
  uint64_t next = 0;
  for (int blk = 0; blk < n_blocks && !b.err; blk++) {
    for (; next < block_key_end[blk]; next++) b.key_end = next + 1; /* AddKey */
    fbb_start_block(&b, block_end_offset[blk]);
  }
  for (; next < n; next++) b.key_end = next + 1;
  if (!b.err && b.key_end > b.key_begin) fbb_generate(&b); /* Finish: start_ not empty */
  const uint32_t array_offset = (uint32_t)b.size;
  for (uint64_t i = 0; i < b.n_offs && !b.err; i++) fbb_put32(&b, b.offs[i]);
  fbb_put32(&b, array_offset);
  if (!b.err && b.size + 1 <= b.cap) b.result[b.size++] = 11; /* kFilterBaseLg */
  else b.err = b.err ? b.err : 1;
  free(b.offs);
  if (b.err) return b.err == 2 ? ORC_E_ARG : ORC_E_CAPACITY;
  return (int64_t)b.size;
}

/* FilterBlockReader ctor + KeyMayMatch(block_offset, key). */
int orc_filter_block_key_may_match(const uint8_t* contents, uint64_t n, uint64_t block_offset,
                                   const uint8_t* key, size_t klen, int policy) {
  if (n < 5) return 1; /* data_ == nullptr, num_ == 0 -> "potential match" */
  const uint64_t base_lg = (uint64_t)(int64_t)(int8_t)contents[n - 1];
  const uint32_t last_word = dec32(contents + n - 5);
  if (last_word > n - 5) return 1;
  const uint8_t* data = contents;
  const uint8_t* offset = data + last_word;
  const uint64_t num = (n - 5 - last_word) / 4;
  const uint64_t index = block_offset >> (base_lg & 63); /* x86 shr: count mod 64 */
  if (index < num) {
    const uint32_t start = dec32(offset + index * 4);
    const uint32_t limit = dec32(offset + index * 4 + 4);
    if (start <= limit && limit <= (uint64_t)(offset - data)) {
      const uint8_t* f = data + start;
      const uint64_t flen = limit - start;
      if (policy == 0) return orc_legacy_key_may_match(f, flen, key, klen);
      const uint32_t h = orc_hash(key, klen, 1);
      for (uint64_t i = 0; i + 4 <= flen; i += 4)
        if (h == dec32(f + i)) return 1;
      return 0;
    } else if (start == limit) {
      return 0;
    }
  }
  return 1;
}
