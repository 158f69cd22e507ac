"""Legacy block-based filter block:
FilterBlockBuilder / FilterBlockReader, table/filter_block.cc:14-142.

The oracle restates the builder / reader; with filter_block_test.cc's own
TestHashFilter policy (oracle policy 1) the reference test's expectations
(table/filter_block_test.cc:44-121) apply verbatim and pin the framing.  The
GPU path builds the same framing with the legacy Bloom policy and is checked
byte for byte against the oracle.
"""
import numpy as np
import pytest

import oracle


def pack_var(keys):
    offs = np.zeros(len(keys) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(k) for k in keys])
    return np.frombuffer(b"".join(keys) + b"\0" * 16, dtype=np.uint8).copy(), offs


def build(seq, policy=1):
    """seq: the reference call sequence, ("start", offset) / ("add", key)."""
    keys, ke, eo = [], [], []
    for op, arg in seq:
        if op == "add":
            keys.append(arg)
        else:
            ke.append(len(keys))
            eo.append(arg)
    data, offs = pack_var(keys)
    return oracle.filter_block_build(data, len(keys), ke, eo, offsets=offs, policy=policy)


def match(block, off, key, policy=1):
    return oracle.filter_block_key_may_match(block, off, key, policy)


def test_reference_empty_builder():  # filter_block_test.cc:44-51
    block = build([])
    assert block == b"\x00\x00\x00\x00\x0b"
    assert match(block, 0, b"foo") and match(block, 100000, b"foo")


def test_reference_single_chunk():  # filter_block_test.cc:53-72
    block = build([("start", 100), ("add", b"foo"), ("add", b"bar"), ("add", b"box"),
                   ("start", 200), ("add", b"box"), ("start", 300), ("add", b"hello")])
    for k in (b"foo", b"bar", b"box", b"hello", b"foo"):
        assert match(block, 100, k)
    assert not match(block, 100, b"missing")
    assert not match(block, 100, b"other")


def test_reference_multi_chunk():  # filter_block_test.cc:74-121
    block = build([("start", 0), ("add", b"foo"), ("start", 2000), ("add", b"bar"),
                   ("start", 3100), ("add", b"box"), ("start", 9000), ("add", b"box"),
                   ("add", b"hello")])
    assert match(block, 0, b"foo") and match(block, 2000, b"bar")
    assert not match(block, 0, b"box") and not match(block, 0, b"hello")
    assert match(block, 3100, b"box")
    for k in (b"foo", b"bar", b"hello"):
        assert not match(block, 3100, k)
    for k in (b"foo", b"bar", b"box", b"hello"):
        assert not match(block, 4100, k)
    assert match(block, 9000, b"box") and match(block, 9000, b"hello")
    assert not match(block, 9000, b"foo") and not match(block, 9000, b"bar")


def test_reader_edge_cases():
    assert match(b"\x01\x02", 0, b"k", 0) == 1                     # n < 5
    assert match(b"\x09\x00\x00\x00\x0b", 0, b"k", 0) == 1         # last_word > n - 5
    block = build([("add", b"a"), ("start", 5000)], policy=0)     # filters 0 (keys), 1 (empty)
    assert match(block, 2048, b"a", 0) == 0                        # empty filter
    assert match(block, 1 << 40, b"a", 0) == 1                     # index >= num


def table_blocks(seed, n, var=False):
    """Keys of one table split into data blocks of random byte sizes (like
    TableBuilder's 4 KiB blocks); block b ends at key ke[b] and offset eo[b]."""
    rng = np.random.default_rng(seed)
    v = np.sort(rng.choice(1 << 30, n, replace=False)).astype(np.uint64)
    keys = [bytes(k) for k in oracle.keys_from_values(v).reshape(n, 20)]
    if var:
        keys = [k[: int(rng.integers(1, 21))] for k in keys]
    ke, eo, i, off = [], [], 0, 0
    while i < n:
        i = min(n, i + int(rng.integers(0, 40)))
        off += int(rng.integers(100, 7000))
        ke.append(i)
        eo.append(off)
    if rng.random() < 0.5 and ke:
        ke[-1] = max(ke[-2] if len(ke) > 1 else 0, n - 3)  # a few keys left for Finish's filter
    return keys, ke, eo


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_bloom_block_no_false_negatives(seed):
    """Data blocks that start on a 2 KiB boundary: every key matches the filter
    the reader picks for its block (block_offset >> 11)."""
    rng = np.random.default_rng(seed)
    n = 3000
    v = np.sort(rng.choice(1 << 30, n, replace=False)).astype(np.uint64)
    keys = [bytes(k) for k in oracle.keys_from_values(v).reshape(n, 20)]
    ke, eo, i, off = [], [], 0, 0
    while i < n:
        i = min(n, i + int(rng.integers(1, 40)))
        off += 2048 * int(rng.integers(1, 4))
        ke.append(i)
        eo.append(off)
    data, offs = pack_var(keys)
    block = oracle.filter_block_build(data, n, ke, eo, offsets=offs)
    starts, bstart = [0] + ke, [0] + eo
    for b in range(len(ke)):
        for k in keys[starts[b]:ke[b]]:
            assert match(block, bstart[b], k, 0) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed,var", [(0, False), (1, True), (2, False), (3, True)])
def test_gpu_filter_block_build_and_probe(gpu, seed, var):
    import torch

    import dlsm_amd

    n = 20_000
    keys, ke, eo = table_blocks(seed, n, var)
    data, offs = pack_var(keys)
    want = oracle.filter_block_build(data, n, ke, eo, offsets=offs)
    if var:
        ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 0, torch.from_numpy(offs).cuda())
    else:
        ks = dlsm_amd.Keys(torch.from_numpy(data).cuda(), n, 20)
    block = gpu.filter_block_build_dev(ks, ke, eo, 10)
    assert block.cpu().numpy().tobytes() == want
    # probe: every key at a few block offsets
    rng = np.random.default_rng(seed + 10)
    qo = rng.integers(0, max(eo) + 5000, n).astype(np.uint64)
    out = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    gpu.filter_block_probe_dev(block, ks, torch.from_numpy(qo).cuda(), out)
    gpu.sync()
    exp = np.array([match(want, int(qo[i]), keys[i], 0) for i in range(n)], dtype=np.uint8)
    assert np.array_equal(out.cpu().numpy(), exp)


@pytest.mark.gpu
def test_gpu_filter_block_empty_and_malformed(gpu):
    import torch

    import dlsm_amd

    ks = dlsm_amd.Keys(torch.zeros(32, dtype=torch.uint8, device="cuda"), 0, 20)
    block = gpu.filter_block_build_dev(ks, [], [], 10)
    assert block.cpu().numpy().tobytes() == b"\x00\x00\x00\x00\x0b"
    q = dlsm_amd.Keys(torch.zeros(40, dtype=torch.uint8, device="cuda"), 2, 20)
    for bad in (b"\x01\x02", b"\x09\x00\x00\x00\x0b", b"\x00\x00\x00\x00\x0b"):
        out = torch.zeros(2, dtype=torch.uint8, device="cuda")
        bt = torch.frombuffer(bytearray(bad), dtype=torch.uint8).cuda()
        gpu.filter_block_probe_dev(bt, q, torch.zeros(2, dtype=torch.uint64, device="cuda"), out)
        gpu.sync()
        assert out.cpu().numpy().tolist() == [1, 1]
    with pytest.raises(dlsm_amd.DlsmError):  # StartBlock offsets must not go backwards
        gpu.filter_block_build_dev(q, [1, 2], [5000, 100], 10)
