"""Summarise rocprofv3 PMC passes over the C5 bench for the sparse product kernel (spmv_blk_kernel)
into the JSON bench.py reads for roofline.traffic at --config c5.  Corrections as tools/pmc_summary.py:
read bytes = 2 * FETCH_SIZE * 1024 (gfx950, MI355X_MICROARCH.md §HBM), write bytes = WRITE_SIZE * 1024.

    python tools/pmc_summary_spmv.py gpurun_out/pmc_c5 profiles/r02_c5_spmv_pmc_f64.json --bytes 6939738384

The recorded kernel name is the instantiation seen in the trace (e.g. spmv_blk_kernel<double, 4>);
bench.py uses the file only when it equals the kernel it launched.
"""
import re
import argparse
import collections
import csv
import json
import os

KERNEL = "spmv_blk_kernel"


def kernel_label(full):
    m = re.search(r"(spmv_blk_kernel(<[^>]*>)?)", full)
    return m.group(1) if m else KERNEL


def per_dispatch(d, name):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(d, name, f"{name}_counter_collection.csv"))):
        if KERNEL in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {r["Dispatch_Id"]: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
           for r in csv.DictReader(open(os.path.join(d, name, f"{name}_kernel_trace.csv")))
           if KERNEL in r["Kernel_Name"]}
    return vals, dur


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--bytes", type=float, required=True, help="algorithmic bytes per launch (bench.py)")
    ap.add_argument("--values", default="fp64")
    a = ap.parse_args()
    fetch, dur = per_dispatch(a.pmc_dir, "fetch")
    write, _ = per_dispatch(a.pmc_dir, "write")
    tcc, _ = per_dispatch(a.pmc_dir, "tcc")
    label = KERNEL
    for r in csv.DictReader(open(os.path.join(a.pmc_dir, "fetch", "fetch_kernel_trace.csv"))):
        if KERNEL in r["Kernel_Name"]:
            label = kernel_label(r["Kernel_Name"])
            break
    rd = mean(2.0 * v["FETCH_SIZE"] * 1024.0 for v in fetch.values())
    wr = mean(v["WRITE_SIZE"] * 1024.0 for v in write.values())
    hit = mean(v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]) for v in tcc.values())
    out = {
        "kernel": label, "config": f"c5 (N = 2^20, m = 2^16, rho = 0.01, {a.values} values)",
        "command": "rocprofv3 --pmc <counter> --kernel-trace --output-format csv -- python3 bench.py --config c5 "
                   "[--f32] --steps 1 --warmup 0 --no-cpu-baseline (one pass each: FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum "
                   "TCC_MISS_sum; summary by tools/pmc_summary_spmv.py)",
        "launches": len(fetch),
        "duration_ms_under_pmc": mean(dur[k] for k in fetch) * 1e3,
        "hbm_bytes_per_launch": rd + wr,
        "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
        "algorithmic_bytes_per_launch": a.bytes,
        "traffic_over_algorithmic": (rd + wr) / a.bytes,
        "tcc_hit_rate": hit,
        "traffic_note": "read bytes = 2 * FETCH_SIZE * 1024 (gfx950 correction); FETCH_SIZE counts L2 misses to "
                        "the fabric with Infinity-Cache hits included, so this is an upper bound on HBM bytes",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
