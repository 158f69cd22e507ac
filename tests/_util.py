"""Shared helpers for the parity tests (materialise golden-fixture key sets)."""
from __future__ import annotations

import numpy as np

import oracle


def case_keys(case):
    """Return (bytes u8 array, offsets u64 array | None, stride, n) for a fixture."""
    if case.get("kind", "dbbench") == "dbbench":
        n = case["n"]
        return oracle.dbbench_keys(case["first"], case["step"], n, 20), None, 20, n
    keys = [bytes.fromhex(k) for k in case["keys"]]
    data, offs = oracle.pack_var(keys)
    return data, offs, 0, len(keys)


def key_list(data, offs, stride, n):
    if offs is None:
        return [data[i * stride:(i + 1) * stride].tobytes() for i in range(n)]
    return [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)]
