"""CPU-side checks of the C ABI library: it loads, exports every symbol that
include/dlsm_bloom.h declares, and its host-only helpers (hash, sizing, filter
metadata parse) agree with the oracle.  No compute call touches a device."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "dlsm_bloom.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dlsm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    import dlsm_amd._lib as L

    lib = L._lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    bound = {name for name, _, _ in L.SIGNATURES}
    assert set(syms) == bound, set(syms) ^ bound
    assert lib.dlsm_abi_version() == 1


def test_library_is_gfx950():
    so = os.path.join(ROOT, "dlsm_amd", "lib", "libdlsm_bloom.so")
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z0-9:+]*", open(so, "rb").read()))
    assert targets == {b"amdgcn-amd-amdhsa--gfx950"}, targets


def test_host_hash_matches_oracle(orc, golden):
    import dlsm_amd

    for c in golden["hash"]["cases"]:
        if c["seed"] != 0xBC9F1D34:
            continue
        k = bytes.fromhex(c["key"])
        assert dlsm_amd.bloom_hash(k) == c["hash"]


def test_sizes_match_oracle(orc):
    import dlsm_amd

    for n in list(range(0, 2000)) + [153_846, 1_600_000, 3_000_000, 2**31 - 1, 2**32 + 5]:
        for bpk in (1, 5, 10, 16):
            assert dlsm_amd.full_size(n, bpk) == orc.full_filter_bytes(n, bpk), (n, bpk)
    for n in [0, 1, 6, 7, 100, 1_600_000]:
        assert dlsm_amd.legacy_size(n, 10) == len(orc.legacy_build(orc.dbbench_keys(0, 1, n), n))


def test_parse_matches_oracle(orc):
    import dlsm_amd

    good = orc.full_build(orc.dbbench_keys(0, 1, 1000), 1000)
    cases = [good, good[:-1], b"", b"\x06\0\0\0\0", bytes([6, 1, 0, 0, 0]),
             bytes(64) + bytes([0, 1, 0, 0, 0]), bytes(64) + bytes([0xFF, 1, 0, 0, 0]),
             bytes(128) + bytes([6, 1, 0, 0, 0]),   # L*64 != len, len % L == 0 -> lg 0
             bytes(128) + bytes([6, 3, 0, 0, 0]),   # no solution -> corrupt
             bytes(64) + bytes([127, 1, 0, 0, 0])]
    for f in cases:
        st, k, L, lg = dlsm_amd.full_parse(f)
        ost, ok, oL, olg = orc.full_reader_parse(f)
        assert (st == 0) == (ost == 0), f[-5:]
        if st == 0:
            assert (k, L, lg) == (ok, oL, olg)


def test_fastmod_and_sizing_host_unit(tmp_path):
    exe = tmp_path / "test_math"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "test_math.cc"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout


def test_ctx_create_without_gpu_fails_cleanly():
    import dlsm_amd

    if dlsm_amd.device_available():
        pytest.skip("a device is present")
    with pytest.raises(dlsm_amd.DlsmError):
        dlsm_amd.Context(0)


def test_no_cpu_fallback_in_product_path():
    """The product package must not import the oracle."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "dlsm_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp", ".hpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f
                assert "liboracle" not in src, f


def test_host_crc32c_helper(orc, golden):
    import dlsm_amd

    for c in golden["full"]["crc32c"]:
        assert dlsm_amd.crc32c(bytes.fromhex(c["data"])) == c["crc"]
    assert dlsm_amd.crc32c_mask(dlsm_amd.crc32c(b"foo")) == orc.crc32c_mask(orc.crc32c(b"foo"))


def test_slice_kernels_use_no_scratch(tmp_path):
    """No slice kernel spills to scratch.  The sliced-probe corruption of
    commit 1c7c4c6 needed a scratch spill (a forced 64-VGPR bound) together
    with two 1,024-thread workgroups per CU (tests/diag/run_old_slice.py);
    keeping the slice passes spill-free rules that combination out."""
    src = os.path.join(ROOT, "dlsm_amd", "csrc", "bloom_kernels.hip")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "--offload-device-only", "-c", src, "-o", str(tmp_path / "k.o"),
                        "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    usage, name = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"remark:\s+ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            usage[name] = int(m.group(1))
    slices = {k: v for k, v in usage.items() if "slice_kernel" in k}
    assert len(slices) >= 6, sorted(usage)
    assert all(v == 0 for v in slices.values()), slices
    # the version probe's LDS kernel (one 1,024-thread workgroup per CU) too:
    # a spill there would put a scratch reload on every probe round
    vl = {k: v for k, v in usage.items() if "version_lds_kernel" in k}
    assert len(vl) >= 8, sorted(usage)
    assert all(v == 0 for v in vl.values()), vl


def test_cu_subset_is_balanced_under_both_numberings():
    """CU-masked streams (bench --cosched) take the same CUs from every XCD
    whichever way the mask numbers them."""
    import dlsm_amd

    for per in (1, 2, 4):
        s = dlsm_amd.cu_subset(per)
        assert len(s) == 8 * per and len(set(s)) == len(s)
        assert all(sum(1 for i in s if i // 32 == x) == per for x in range(8))
        assert all(sum(1 for i in s if i % 8 == x) == per for x in range(8))


def test_keys_guard_checks_data_against_host_offsets():
    """Variable-length Keys with host offsets: a data buffer shorter than
    offsets[n] is refused before any pointer reaches the library."""
    import dlsm_amd

    offs = np.array([0, 5, 12], dtype=np.uint64)
    ok = dlsm_amd.Keys(np.zeros(12, dtype=np.uint8), 2, 0, offs)
    ok.c()
    with pytest.raises(ValueError):
        dlsm_amd.Keys(np.zeros(11, dtype=np.uint8), 2, 0, offs).c()
    with pytest.raises(ValueError):
        dlsm_amd.Keys(np.zeros(12, dtype=np.uint8), 2, 0, offs[:2]).c()


def test_host_read_bytes_folds_every_word():
    """dlsm_host_read_bytes (the host read ceiling bench.py's e2e_hashed is
    measured against) reads every 64-bit word once, on any thread count."""
    import numpy as np

    import dlsm_amd

    x = np.random.default_rng(5).integers(0, 2**63, size=(1 << 20) + 3, dtype=np.uint64)
    want = int(np.bitwise_xor.reduce(x))
    for th in (0, 1, 3):
        assert dlsm_amd.host_read_bytes(x, th) == want
    assert dlsm_amd.host_read_bytes(x[:0]) == 0
