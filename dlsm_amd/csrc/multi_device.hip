// dlsm_amd/csrc/multi_device.hip -- one process driving several GPUs, one
// host thread per GPU (dLSM's builders are threads of
// one process: db/db_impl.cc:3373-3386, include/TimberSaw/options.h:73-78).
//
// dlsm_multi_device_run: every device runs the same step -- its SSTables'
// filter build, then its lookup shard's probe -- on its own contexts and
// streams, from its own std::thread, with no cross-device traffic.  The timed
// region is bracketed by two host barriers with every device drained on both
// sides, so the wall time is the slowest device's.  Built only on the public
// ABI (dlsm_bloom.h): the same calls a dLSM node would make.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/dlsm_bloom.h"

namespace {

// Reusable counting barrier (C++17: no std::barrier).
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    const uint64_t gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      cv_.notify_all();
      return;
    }
    cv_.wait(lk, [&] { return gen_ != gen; });
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  uint64_t gen_ = 0;
};

int step(const dlsm_device_work& w, int bpk) {
  if (w.n_jobs > 0) {
    const int s = dlsm_bloom_full_build_dev(w.build_ctx, w.jobs, w.n_jobs, bpk, w.out_len_dev);
    if (s != DLSM_OK) return s;
  }
  if (w.fs && w.keys.n > 0) return dlsm_bloom_full_probe_dev(w.probe_ctx, w.fs, &w.keys, w.mask_dev);
  return DLSM_OK;
}

int drain(const dlsm_device_work& w) {
  int s = dlsm_ctx_sync(w.build_ctx);
  if (s == DLSM_OK && w.probe_ctx != w.build_ctx) s = dlsm_ctx_sync(w.probe_ctx);
  return s;
}

// instrument_all: every device records its pass events (dlsm_multi_device_run_timed);
// else only entry 0 does (dlsm_multi_device_run[_sampled], whose header promises
// entry 0's passes): the other devices' steps keep their build / probe overlap.
int run_impl(const dlsm_device_work* work, int n, int bits_per_key, int steps, int warmup, int event_every,
             double* wall_seconds, float* pass_ms, double* device_seconds, bool instrument_all) {
  if (!work || n < 1 || steps < 1 || warmup < 0 || !wall_seconds || event_every < 1) return DLSM_E_ARG;
  for (int d = 0; d < n; d++) {
    const dlsm_device_work& w = work[d];
    if (!w.probe_ctx || !w.build_ctx || (w.n_jobs > 0 && (!w.jobs || !w.out_len_dev))) return DLSM_E_ARG;
    if (dlsm_ctx_device(w.probe_ctx) != dlsm_ctx_device(w.build_ctx)) return DLSM_E_ARG;
  }
  Barrier start(n + 1), end(n + 1);
  std::vector<int> status(n, DLSM_OK);
  std::vector<std::thread> threads;
  threads.reserve(n);
  for (int d = 0; d < n; d++) {
    threads.emplace_back([&, d] {
      const dlsm_device_work& w = work[d];
      int& st = status[d];
      if (hipSetDevice(dlsm_ctx_device(w.probe_ctx)) != hipSuccess) st = DLSM_E_DEVICE;
      for (int i = 0; i < warmup && st == DLSM_OK; i++) st = step(w, bits_per_key);
      if (st == DLSM_OK) st = drain(w);
      // Every device brackets each pass of every event_every-th step with
      // events on the stream it runs on (an event pair at a call boundary
      // leaves the GPU idle for several microseconds:
      // profiles/r03_o_pass_events_ab.txt).  With the build on a stream of
      // its own, a sampled step runs its passes alone -- its build after the
      // probes before it, its probe after its build, the next build after its
      // probe -- so the events time each pass by itself (the roofline's
      // kernel time), not beside the other.
      const bool events = pass_ms && st == DLSM_OK && (instrument_all || d == 0);
      std::vector<hipEvent_t> ev;
      hipEvent_t gate = nullptr;
      if (events) {
        ev.resize(4 * static_cast<size_t>(steps));
        for (auto& e : ev)
          if (hipEventCreate(&e) != hipSuccess) st = DLSM_E_DEVICE;
        if (hipEventCreateWithFlags(&gate, hipEventDisableTiming) != hipSuccess) st = DLSM_E_DEVICE;
      }
      auto sampled = [&](int i) { return events && i % event_every == event_every - 1; };
      hipStream_t bs = static_cast<hipStream_t>(dlsm_ctx_stream(w.build_ctx));
      hipStream_t ps = static_cast<hipStream_t>(dlsm_ctx_stream(w.probe_ctx));
      const bool two = bs != ps;
      start.wait();  // every device idle; the host clock starts
      const auto td = std::chrono::steady_clock::now();
      for (int i = 0; i < steps && st == DLSM_OK; i++) {
        const bool e = sampled(i);
        if (e) {
          if (two) {
            (void)hipEventRecord(gate, ps);
            (void)hipStreamWaitEvent(bs, gate, 0);
          }
          (void)hipEventRecord(ev[4 * i + 0], bs);
        }
        if (w.n_jobs > 0) st = dlsm_bloom_full_build_dev(w.build_ctx, w.jobs, w.n_jobs, bits_per_key, w.out_len_dev);
        if (e) {
          (void)hipEventRecord(ev[4 * i + 1], bs);
          if (two) (void)hipStreamWaitEvent(ps, ev[4 * i + 1], 0);
          (void)hipEventRecord(ev[4 * i + 2], ps);
        }
        if (st == DLSM_OK && w.fs && w.keys.n > 0) st = dlsm_bloom_full_probe_dev(w.probe_ctx, w.fs, &w.keys, w.mask_dev);
        if (e) {
          (void)hipEventRecord(ev[4 * i + 3], ps);
          if (two) (void)hipStreamWaitEvent(bs, ev[4 * i + 3], 0);
        }
      }
      if (st == DLSM_OK) st = drain(w);
      // this device's own time: from the start barrier to its drain
      if (device_seconds)
        device_seconds[d] = std::chrono::duration<double>(std::chrono::steady_clock::now() - td).count();
      end.wait();  // every device drained; the host clock stops
      if (events) {
        float* pm = pass_ms + 2 * static_cast<size_t>(steps) * d;
        for (int i = 0; i < steps; i++) {
          float b = -1.f, p = -1.f;  // not sampled
          if (sampled(i) && st == DLSM_OK &&
              (hipEventElapsedTime(&b, ev[4 * i + 0], ev[4 * i + 1]) != hipSuccess ||
               hipEventElapsedTime(&p, ev[4 * i + 2], ev[4 * i + 3]) != hipSuccess))
            st = DLSM_E_DEVICE;
          pm[2 * i] = b;
          pm[2 * i + 1] = p;
        }
        for (auto& e : ev) (void)hipEventDestroy(e);
        if (gate) (void)hipEventDestroy(gate);
      }
    });
  }
  start.wait();
  const auto t0 = std::chrono::steady_clock::now();
  end.wait();
  const auto t1 = std::chrono::steady_clock::now();
  for (auto& t : threads) t.join();
  *wall_seconds = std::chrono::duration<double>(t1 - t0).count();
  for (int s : status)
    if (s != DLSM_OK) return s;
  return DLSM_OK;
}

}  // namespace

extern "C" int dlsm_multi_device_run_timed(const dlsm_device_work* work, int n, int bits_per_key, int steps,
                                           int warmup, int event_every, double* wall_seconds, float* pass_ms,
                                           double* device_seconds) {
  if (pass_ms && n > 0 && steps > 0)
    for (size_t i = 0; i < 2 * static_cast<size_t>(steps) * n; i++) pass_ms[i] = -1.f;
  return run_impl(work, n, bits_per_key, steps, warmup, event_every, wall_seconds, pass_ms, device_seconds, true);
}

extern "C" int dlsm_multi_device_run_sampled(const dlsm_device_work* work, int n, int bits_per_key, int steps,
                                             int warmup, int event_every, double* wall_seconds, float* pass_ms) {
  if (n < 1 || steps < 1) return DLSM_E_ARG;
  std::vector<float> all(pass_ms ? 2 * static_cast<size_t>(steps) * n : 0);
  const int st = run_impl(work, n, bits_per_key, steps, warmup, event_every, wall_seconds,
                          pass_ms ? all.data() : nullptr, nullptr, false);
  if (pass_ms && st == DLSM_OK)
    for (int i = 0; i < 2 * steps; i++) pass_ms[i] = all[i];  // device 0's
  return st;
}

extern "C" int dlsm_multi_device_run(const dlsm_device_work* work, int n, int bits_per_key, int steps, int warmup,
                                     double* wall_seconds, float* pass_ms) {
  return dlsm_multi_device_run_sampled(work, n, bits_per_key, steps, warmup, 1, wall_seconds, pass_ms);
}
