"""The C++ adapter (include/dlsm_bloom_adapter.hpp) compiled as a reference-side
caller would compile it, run on the GPU, checked against the oracle: the
single-thread class surface (adapter_test.cc) and the reference's concurrent
call shape, 16 builder threads with one context each (concurrent_builders.cc)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compile(tmp_path, name, extra=()):
    exe = tmp_path / name
    cmd = ["g++", "-std=c++17", "-O2", "-fno-rtti", "-fno-exceptions", "-pthread",
           "-I", os.path.join(ROOT, "include"), *extra,
           os.path.join(ROOT, "tests", "cpp", name + ".cc"),
           "-L", os.path.join(ROOT, "dlsm_amd", "lib"), "-ldlsm_bloom",
           "-L", os.path.join(ROOT, "oracle"), "-loracle",
           "-Wl,-rpath," + os.path.join(ROOT, "dlsm_amd", "lib"),
           "-Wl,-rpath," + os.path.join(ROOT, "oracle"),
           "-Wl,-rpath,/opt/rocm/lib", "-L/opt/rocm/lib", "-o", str(exe)]
    subprocess.run(cmd, check=True)
    return exe


def test_adapter_compiles_without_hip_headers(tmp_path):
    """A reference-side C++ caller needs only the C header (no HIP, no torch),
    and builds with the reference's -fno-rtti -fno-exceptions."""
    _compile(tmp_path, "adapter_test")
    _compile(tmp_path, "concurrent_builders")


def test_adapter_derives_from_host_filter_policy(tmp_path):
    """With DLSM_ADAPTER_HOST_NAMESPACE the adapter classes derive from the
    host's own FilterPolicy and use its Slice (what Options::filter_policy
    holds), checked here against a host namespace shaped like TimberSaw's."""
    src = tmp_path / "host_ns.cc"
    src.write_text(
        "#include <cstddef>\n#include <cstring>\n#include <string>\n"
        "namespace hostdb {\n"
        "class Slice { public: Slice():d_(\"\"),n_(0){} Slice(const char* d,size_t n):d_(d),n_(n){}\n"
        "  Slice(const std::string& s):d_(s.data()),n_(s.size()){}\n"
        "  const char* data() const {return d_;} size_t size() const {return n_;}\n"
        "  void Reset(const char* d,size_t n){d_=d;n_=n;} private: const char* d_; size_t n_; };\n"
        "class FilterPolicy { public: virtual ~FilterPolicy() {}\n"
        "  virtual const char* Name() const = 0;\n"
        "  virtual void CreateFilter(const Slice* keys, int n, Slice* dst) const = 0;\n"
        "  virtual bool KeyMayMatch(const Slice& key, const Slice& filter) const = 0; };\n"
        "struct Options { const FilterPolicy* filter_policy = nullptr; };\n"
        "}\n"
        "#define DLSM_ADAPTER_HOST_NAMESPACE hostdb\n"
        "#include \"dlsm_bloom_adapter.hpp\"\n"
        "int main() { hostdb::Options o; o.filter_policy = dlsm_adapter::NewBloomFilterPolicy(10, nullptr);\n"
        "  dlsm_adapter::InternalFilterPolicy ip(o.filter_policy); const hostdb::FilterPolicy* p = &ip;\n"
        "  int r = std::strcmp(p->Name(), \"TimberSaw.BuiltinBloomFilter2\"); delete o.filter_policy; return r; }\n")
    exe = tmp_path / "host_ns"
    subprocess.run(["g++", "-std=c++17", "-fno-rtti", "-fno-exceptions", "-I", os.path.join(ROOT, "include"),
                    str(src), "-L", os.path.join(ROOT, "dlsm_amd", "lib"), "-ldlsm_bloom",
                    "-Wl,-rpath," + os.path.join(ROOT, "dlsm_amd", "lib"), "-Wl,-rpath,/opt/rocm/lib",
                    "-L/opt/rocm/lib", "-o", str(exe)], check=True)
    assert subprocess.run([str(exe)], timeout=60).returncode == 0


def test_adapter_output_capacity_on_cpu(tmp_path):
    """Move_buffer: Finish writes at most the rest of the slot, or the size a
    buffer outside the slot came with -- 0 (refused, DLSM_E_CAPACITY) when it
    came without one (table/full_filter_block.cc:103,144-146).
    Host logic only: runs without a GPU."""
    exe = _compile(tmp_path, "adapter_host_test")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "OK adapter host" in out.stdout, out.stdout + out.stderr


def test_adapter_addkey_hashing_on_cpu(tmp_path):
    """hash_in_addkey: the hashes a builder hands to the library are BloomHash
    of every key minus consecutive repeats (full_filter_block.cc:39-49), over
    the 20-byte fast path, AVX-512 block hashing + compress-store dedup and the
    scalar paths, across block boundaries and key-length changes.  The C ABI
    calls are stubbed in the test (host memory), so it runs without a GPU."""
    exe = tmp_path / "adapter_addkey_cpu_test"
    subprocess.run(["g++", "-std=c++17", "-O2", "-fno-rtti", "-fno-exceptions", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "adapter_addkey_cpu_test.cc"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "OK adapter addkey cpu" in out.stdout, out.stdout + out.stderr


def test_adapter_fallback_without_device(tmp_path):
    """With no device visible (this CPU suite) the reference-signature builder,
    reader, policy and legacy filter block still produce the oracle's bytes
    and answers: every GPU call fails and the host loops (product code in the
    adapter) answer instead, each counted by dlsm_fallback_stats.  On a box
    with a GPU the same program runs its GPU form (test below)."""
    exe = _compile(tmp_path, "adapter_fallback_test")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "OK adapter fallback" in out.stdout, out.stdout + out.stderr


@pytest.mark.gpu
def test_adapter_fallback_and_reference_signatures_on_gpu(tmp_path):
    """The drop-in's failure path and reference signatures on the GPU:
    FullFilterBlockBuilder(ibv_mr*, int) with injected DLSM_E_DEVICE /
    DLSM_E_NOMEM at 0, 1, 7 and 153,846 keys emits the oracle's filter (host
    re-run, counted), never a 0-byte one; FullFilterBlockReader(Slice,
    shared_ptr<Manager>, FilterSide) and NewBloomFilterPolicy(int) answer
    single keys on the host with no device copy until the first batch, batches
    on the GPU; single-key latency is reported in ns."""
    exe = _compile(tmp_path, "adapter_fallback_test")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "OK adapter fallback" in out.stdout, out.stdout + out.stderr
    rec = json.loads(out.stdout.splitlines()[0])
    assert rec["device"] is True
    print(json.dumps(rec))


@pytest.mark.gpu
def test_adapter_on_gpu(tmp_path):
    exe = _compile(tmp_path, "adapter_test")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "OK adapter" in out.stdout, out.stdout + out.stderr


@pytest.mark.gpu
def test_sixteen_concurrent_builder_threads(tmp_path):
    """16 std::threads, one dlsm_ctx each, RestartBlock / AddKey x 153,846 /
    Finish per table: every filter equals the oracle's and no context
    allocates device memory after its first table."""
    exe = _compile(tmp_path, "concurrent_builders")
    out = subprocess.run([str(exe), "16", "4", "153846"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and "OK concurrent builders" in out.stdout, out.stdout + out.stderr
    rec = json.loads(out.stdout.splitlines()[0])
    assert rec["failures"] == 0 and rec["no_device_alloc_after_warmup"]
    print(json.dumps(rec))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["batch", "hash", "batch-hash"])
def test_concurrent_builders_batched_and_hashed(tmp_path, mode):
    """The same 16-thread call shape with Finish through the device's batcher
    (concurrent calls -> batched builds) and/or AddKey hashing on the host (4 B
    per key over PCIe): every filter equals the oracle's."""
    exe = _compile(tmp_path, "concurrent_builders")
    out = subprocess.run([str(exe), "16", "3", "153846", mode], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and "OK concurrent builders" in out.stdout, out.stdout + out.stderr
    rec = json.loads(out.stdout.splitlines()[0])
    assert rec["failures"] == 0 and rec["mode"] == mode
    if mode.startswith("batch"):
        assert rec["batches"] >= 1 and rec["max_batch"] >= 1
    print(json.dumps(rec))


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [16, 28])
def test_reference_signature_builders(tmp_path, threads):
    """The reference's own builder signature, FullFilterBlockBuilder(ibv_mr*,
    bits_per_key), with its own AddKey (BloomHash into hash_entries_) and the
    thread's context, from 16 and from 28 threads at once (dLSM's 4 flush + 12
    compaction + 12 subcompaction builders, options.h:73,77-78): every filter
    equals the oracle's, and no context allocates after its first table."""
    exe = _compile(tmp_path, "concurrent_builders")
    out = subprocess.run([str(exe), str(threads), "3", "153846", "ref"], capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0 and "OK concurrent builders" in out.stdout, out.stdout + out.stderr
    rec = json.loads(out.stdout.splitlines()[0])
    assert rec["failures"] == 0 and rec["mode"] == "ref" and rec["threads"] == threads
    print(json.dumps(rec))
