"""Host-side diagnostic for e2e_hashed's host hashing rate (no GPU work
besides page-locked allocation): where the process may run (NUMA nodes, CPU
affinity, cgroup quota), which node a page-locked key buffer's pages live
on, and the BloomHash batch rate (dlsm_bloom_hash_batch) and a plain
streaming read rate over that buffer, with the process's threads confined to
one node or spread over all of them.

    python3 scripts/diag_host_numa.py            # driver: one child per placement
    python3 scripts/diag_host_numa.py --child CPUS LABEL
"""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def nodes():
    base = "/sys/devices/system/node"
    out = {}
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            with open(os.path.join(base, d, "cpulist")) as f:
                out[int(d[4:])] = parse_list(f.read().strip())
    return out


def parse_list(s):
    cpus = []
    for part in s.split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def page_nodes(addr, nbytes, samples=64):
    """Node of `samples` pages spread over [addr, addr + nbytes) (move_pages
    with nodes=NULL reports each page's node)."""
    libc = ctypes.CDLL(None, use_errno=True)
    page = os.sysconf("SC_PAGE_SIZE")
    ptrs = (ctypes.c_void_p * samples)(*[addr + (nbytes * i // samples) // page * page for i in range(samples)])
    status = (ctypes.c_int * samples)()
    SYS_move_pages = 279  # x86_64
    r = libc.syscall(SYS_move_pages, 0, samples, ptrs, None, status, 0)
    if r != 0:
        return {"error": ctypes.get_errno()}
    hist = {}
    for s in status:
        hist[int(s)] = hist.get(int(s), 0) + 1
    return hist


def child(cpus, label):
    import numpy as np
    import torch

    import dlsm_amd
    from dlsm_amd import workload as W

    os.sched_setaffinity(0, cpus)  # before the hash pool starts: its threads inherit it
    n = int(os.environ.get("DIAG_KEYS", 100_000_000))
    keys_np = W.dbbench_keys_np(np.arange(n, dtype=np.uint64))
    rec = {"label": label, "cpus": len(cpus)}
    kinds = ("pinned", "pageable") if torch.cuda.is_available() else ("pageable",)
    for kind in kinds:
        t = torch.from_numpy(keys_np.reshape(-1))
        buf = t.pin_memory() if kind == "pinned" else t.clone()
        addr = buf.data_ptr()
        rec[f"{kind}_page_nodes"] = page_nodes(addr, buf.numel())
        out = np.empty(n, dtype=np.uint32)
        arr = buf.numpy()
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            dlsm_amd.hash_batch(dlsm_amd.Keys(arr, n, 20), out=out)
            best = max(best, n / (time.perf_counter() - t0) / 1e9)
        rec[f"{kind}_hash_gkeys_s"] = round(best, 2)
        torch.set_num_threads(len(cpus))
        x = buf.view(torch.int64)
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            _ = int(x.sum())
            best = max(best, x.numel() * 8 / (time.perf_counter() - t0) / 1e9)
        rec[f"{kind}_sum_GBs"] = round(best, 1)
        del buf, x
    print(json.dumps(rec), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(parse_list(sys.argv[2]), sys.argv[3])
        return
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota = f.read().strip()
    except OSError:
        pass
    nd = nodes()
    print(json.dumps({"affinity_cpus": len(aff), "cpu_max": quota,
                      "nodes": {k: len(v) for k, v in nd.items()},
                      "affinity_per_node": {k: len(set(v) & set(aff)) for k, v in nd.items()}}), flush=True)
    import dlsm_amd  # noqa: F401  (the library's own core count)
    share = min(len(aff), 16)
    placements = [("spread", aff[:: max(1, len(aff) // share)][:share])]
    for k, v in nd.items():
        mine = [c for c in v if c in set(aff)]
        if mine:
            placements.append((f"node{k}", mine[:share]))
    for label, cpus in placements:
        subprocess.run([sys.executable, os.path.abspath(__file__), "--child", ",".join(map(str, cpus)), label],
                       check=True, timeout=300)


if __name__ == "__main__":
    main()
