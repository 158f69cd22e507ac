"""Per-launch HBM traffic of the bench's build and probe passes from rocprofv3
PMC passes (FETCH_SIZE pass and WRITE_SIZE pass, each its own run, as
scripts/gpu_pmc.sh collects them).

MI355X_MICROARCH.md §HBM/rocprofv3: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads,
so it is doubled here; WRITE_SIZE is exact for 16-B-per-lane stores.  Both
count Infinity-Cache hits as well (memory-side counters), so the figure is
fabric traffic, an upper bound on HBM traffic.

    python scripts/pmc_traffic.py PMC_DIR BENCH_JSON OUT_JSON [VERSION_PMC_DIR] [NAME=SHAPE_PMC_DIR ...]

VERSION_PMC_DIR: FETCH/WRITE passes of scripts/bench_version_probe.py (its
version set-up builds 426 filters, so its launches are kept apart from the
bench's build pass).  NAME=SHAPE_PMC_DIR: FETCH/WRITE passes of
scripts/bench_probe_shapes.py --paths auto over one of bench.py's SHAPE_LEGS
(mixed_set, dedup_shifted): the one-pass probe's three kernels, one launch
each per call (one slice launch per image-width class: one class in both);
block=DIR: passes of scripts/bench_block.py --only-block.
"""
import csv
import glob
import json
import re
import statistics
import sys
from collections import defaultdict

PASSES = {"probe": ("probe_partition_kernel", "probe_slice_kernel", "probe_unpermute_kernel"),
          "build": ("full_partition_kernel", "full_slice_kernel"),
          "legacy": ("legacy_partition_kernel", "legacy_slice_kernel"),
          "version": ("version_lds_kernel",)}
SHAPE_KERNELS = ("probe_mpartition_kernel", "probe_slice_kernel", "probe_munpermute_kernel")
# block=DIR: FETCH/WRITE passes of scripts/bench_block.py --only-block (the
# sealed build: partition, slice pass with the crc fused, seal kernel if any)
NAMED_KERNELS = {"block": ("full_partition_kernel", "full_slice_kernel", "full_block_seal_kernel")}


def per_kernel(pmc_dir):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{pmc_dir}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            m = re.search(r"::([a-z_]+_kernel)", r["Kernel_Name"])
            if m and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
                vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    pmc_dir, bench_json, out_json = sys.argv[1:4]
    bench = json.load(open(bench_json))
    vals = per_kernel(pmc_dir)
    shapes = {}
    for a in sys.argv[4:]:
        if "=" in a:  # a probe-shape leg's own passes
            name, d = a.split("=", 1)
            shapes[name] = per_kernel(d)
            continue
        vv = per_kernel(a)  # the version probe's own passes
        if "version_lds_kernel" in vv:
            vals["version_lds_kernel"] = vv["version_lds_kernel"]
    out = {"source": pmc_dir, "config": {k: bench.get("config", bench).get(k) for k in
                                          ("tables", "keys_per_table", "lookups", "filters",
                                           "probe_chunk_lg", "probe_slice_lg", "keys")},
           "note": "per launch of the pass; FETCH_SIZE x2 (gfx950), KiB -> bytes; "
                   "fabric traffic incl. Infinity-Cache hits"}
    for name, kernels in PASSES.items():
        fetch = write = 0.0
        detail = {}
        for k in kernels:
            if k not in vals:
                continue
            # median over launches: every bench launch of a kernel has the same shape
            fb = statistics.median(vals[k]["FETCH_SIZE"]) * 1024 * 2 if vals[k]["FETCH_SIZE"] else 0.0
            wb = statistics.median(vals[k]["WRITE_SIZE"]) * 1024 if vals[k]["WRITE_SIZE"] else 0.0
            detail[k] = {"fetch_bytes": round(fb), "write_bytes": round(wb)}
            fetch += fb
            write += wb
        if not detail:
            continue
        out[name] = {"fetch_bytes": round(fetch), "write_bytes": round(write),
                     "traffic_bytes": round(fetch + write), "kernels": detail}
    for name, sv in shapes.items():
        detail = {}
        for k in NAMED_KERNELS.get(name, SHAPE_KERNELS):
            if not sv.get(k):
                continue
            detail[k] = {"fetch_bytes": round(statistics.median(sv[k]["FETCH_SIZE"]) * 1024 * 2),
                         "write_bytes": round(statistics.median(sv[k]["WRITE_SIZE"]) * 1024)}
        if detail:
            fetch = sum(d["fetch_bytes"] for d in detail.values())
            write = sum(d["write_bytes"] for d in detail.values())
            out[name] = {"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                         "kernels": detail}
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
