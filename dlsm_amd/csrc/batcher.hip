// dlsm_amd/csrc/batcher.hip -- a per-device submission queue that gathers
// concurrent FullFilterBlockBuilder::Finish calls into batched builds.
//
// dLSM finishes one filter per TableBuilder, from up to 4 flush + 12
// compaction + 12 subcompaction threads at once (include/TimberSaw/
// options.h:73-78, table/table_builder_computeside.cc:389-432).  One context
// per thread issues one H2D + build + D2H per table and pays the per-call
// launch and synchronisation latency every time.  Here a caller's Finish
// enqueues its job and blocks; E executor threads (each with its own context
// and stream) take every job queued so far -- optionally waiting up to
// `window_us` for more -- and run them as ONE batched call (one set of
// kernels over all the batch's SSTables, copies on one stream).  While one
// executor's batch is in flight the next gathers the calls that arrive
// meanwhile, so batching adapts to the arrival rate.  Results are those of
// the per-table call (same kernels, same bytes).
// Host code only (no HIP calls of its own: every device call goes through
// the C ABI), so tests/cpp/batcher_cpu_test.cc compiles it with g++ against
// a stubbed ABI under ThreadSanitizer.
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/dlsm_bloom.h"

namespace {
struct Request {
  const dlsm_build_job* job;
  int bpk;
  int flags;  // DLSM_BATCH_HASHED | DLSM_BATCH_EXACT
  uint64_t out_len = 0;
  int status = DLSM_OK;
  bool done = false;
};
}  // namespace

struct dlsm_batcher {
  int device = 0;
  uint32_t window_us = 0, max_jobs = 64;
  std::mutex m;
  std::condition_variable cv_work, cv_done;
  std::deque<Request*> q;
  bool stop = false;
  std::vector<std::thread> execs;
  std::vector<dlsm_ctx*> ctxs;
  uint64_t batches = 0, jobs = 0, max_batch = 0;

  static int build(dlsm_ctx* ctx, const dlsm_build_job* jv, int n, int bpk, int flags, uint64_t* lens) {
    // the executor's context counts the line number exactly first when the
    // batch's builders saw repeated keys (their filters would otherwise take
    // the slice pass's re-hash fallback for a lowered line count)
    dlsm_ctx_set_option(ctx, DLSM_OPT_BUILD_EXACT, (flags & DLSM_BATCH_EXACT) ? 1 : 0);
    return (flags & DLSM_BATCH_HASHED) ? dlsm_bloom_full_build_hashed(ctx, jv, n, bpk, lens)
                                       : dlsm_bloom_full_build(ctx, jv, n, bpk, lens);
  }

  void run(dlsm_ctx* ctx) {
    std::vector<Request*> batch;
    std::vector<dlsm_build_job> jv;
    std::vector<uint64_t> lens;
    for (;;) {
      std::unique_lock<std::mutex> lk(m);
      cv_work.wait(lk, [&] { return stop || !q.empty(); });
      if (q.empty()) return;  // stop, nothing left
      if (window_us && q.size() < max_jobs && !stop) {
        cv_work.wait_for(lk, std::chrono::microseconds(window_us), [&] { return stop || q.size() >= max_jobs; });
        // another executor may have taken every queued job while this one
        // waited in its window
        if (q.empty()) {
          if (stop) return;
          continue;
        }
      }
      // every queued job with the front's (bits_per_key, flags): one call
      batch.clear();
      const int bpk = q.front()->bpk;
      const int flags = q.front()->flags;
      for (auto it = q.begin(); it != q.end() && batch.size() < max_jobs;) {
        if ((*it)->bpk == bpk && (*it)->flags == flags) {
          batch.push_back(*it);
          it = q.erase(it);
        } else {
          ++it;
        }
      }
      if (!q.empty()) cv_work.notify_one();  // leftovers for another executor
      batches++;
      jobs += batch.size();
      if (batch.size() > max_batch) max_batch = batch.size();
      lk.unlock();
      const int n = static_cast<int>(batch.size());
      jv.resize(n);
      lens.assign(n, 0);
      std::vector<int> status(n, DLSM_OK);
      for (int i = 0; i < n; i++) jv[i] = *batch[i]->job;
      const int st = build(ctx, jv.data(), n, bpk, flags, lens.data());
      if (st == DLSM_OK || st == DLSM_E_CAPACITY) {
        // a batch's only per-job failure is a too-small slot (its length 0)
        for (int i = 0; i < n; i++) status[i] = lens[i] ? DLSM_OK : (st == DLSM_OK ? DLSM_OK : DLSM_E_CAPACITY);
      } else if (n == 1) {
        status[0] = st;
      } else {
        // one job's invalid keyset (or a device error) failed the batched call:
        // run the jobs one at a time so every caller gets its own status
        for (int i = 0; i < n; i++) status[i] = build(ctx, &jv[i], 1, bpk, flags, &lens[i]);
      }
      lk.lock();
      for (int i = 0; i < n; i++) {
        Request* r = batch[i];
        r->out_len = status[i] == DLSM_OK ? lens[i] : 0;
        r->status = status[i];
        r->done = true;
      }
      cv_done.notify_all();
    }
  }
};

extern "C" {

int dlsm_batcher_create(int device, int executors, uint32_t window_us, uint32_t max_jobs, dlsm_batcher** out) {
  if (!out || executors < 1 || executors > 8 || max_jobs < 1) return DLSM_E_ARG;
  *out = nullptr;
  dlsm_batcher* b = new (std::nothrow) dlsm_batcher();
  if (!b) return DLSM_E_NOMEM;
  b->device = device;
  b->window_us = window_us;
  b->max_jobs = max_jobs;
  for (int e = 0; e < executors; e++) {
    dlsm_ctx* c = nullptr;
    const int st = dlsm_ctx_create(device, &c);
    if (st != DLSM_OK) {
      for (dlsm_ctx* x : b->ctxs) dlsm_ctx_destroy(x);
      delete b;
      return st;
    }
    b->ctxs.push_back(c);
  }
  for (dlsm_ctx* c : b->ctxs) b->execs.emplace_back([b, c] { b->run(c); });
  *out = b;
  return DLSM_OK;
}

int dlsm_batcher_destroy(dlsm_batcher* b) {
  if (!b) return DLSM_OK;
  {
    std::lock_guard<std::mutex> lk(b->m);
    b->stop = true;
  }
  b->cv_work.notify_all();
  for (auto& t : b->execs) t.join();
  for (dlsm_ctx* c : b->ctxs) dlsm_ctx_destroy(c);
  delete b;
  return DLSM_OK;
}

int dlsm_batcher_submit(dlsm_batcher* b, const dlsm_build_job* job, int bits_per_key, int flags, uint64_t* out_len) {
  if (!b || !job || !out_len || (flags & ~(DLSM_BATCH_HASHED | DLSM_BATCH_EXACT))) return DLSM_E_ARG;
  Request r{job, bits_per_key, flags};
  std::unique_lock<std::mutex> lk(b->m);
  if (b->stop) return DLSM_E_ARG;
  b->q.push_back(&r);
  b->cv_work.notify_one();
  b->cv_done.wait(lk, [&] { return r.done; });
  *out_len = r.out_len;
  return r.status;
}

int dlsm_batcher_full_build(dlsm_batcher* b, const dlsm_build_job* job, int bits_per_key, uint64_t* out_len) {
  return dlsm_batcher_submit(b, job, bits_per_key, 0, out_len);
}

int dlsm_batcher_full_build_hashed(dlsm_batcher* b, const dlsm_build_job* job, int bits_per_key,
                                   uint64_t* out_len) {
  return dlsm_batcher_submit(b, job, bits_per_key, DLSM_BATCH_HASHED, out_len);
}

int dlsm_batcher_stats(dlsm_batcher* b, uint64_t* batches, uint64_t* jobs, uint64_t* max_batch) {
  if (!b) return DLSM_E_ARG;
  std::lock_guard<std::mutex> lk(b->m);
  if (batches) *batches = b->batches;
  if (jobs) *jobs = b->jobs;
  if (max_batch) *max_batch = b->max_batch;
  return DLSM_OK;
}

}  // extern "C"
