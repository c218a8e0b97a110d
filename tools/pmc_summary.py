"""Summarise rocprofv3 PMC passes (tools/gpu_gram_pmc.sh) for the main Gram kernel into the JSON
bench.py reads for roofline.traffic.  Corrections per MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE
reports half of a 16-B/lane streaming read -> read bytes = 2 * FETCH_SIZE * 1024; FETCH_SIZE counts
L2 misses to the fabric (Infinity Cache hits included), so the total is an upper bound on HBM bytes.

    python tools/pmc_summary.py gpurun_out/pmc_c3 profiles/r01_gram_pmc.json --N 1048576 --m 16384
"""
import argparse
import collections
import csv
import json
import os

# the main-Gram kernels (their rocprofv3 names: every template argument, defaults included)
KERNELS = ("gram_sia_kernel<1, 4, false, true, false>", "gram_sia_kernel<1, 2, false, true, false>",
           "gram_sia_kernel<1, 4, false, false, false>", "gram_sia_kernel<1, 2, false, false, false>",
           "gram_sia_kernel<1, 4, false, true>", "gram_sia_kernel<1, 4>", "gram_sia_kernel<1, 2>",
           "gram_sia_kernel<1, 2, false, false>", "gram_sia_kernel<1, 4, false, false>", "gram_glds_kernel",
           "gram_f64_kernel<false, 4, true", "gram_f64_kernel<false, 2, true")


def load(d, name):
    rows = list(csv.DictReader(open(os.path.join(d, name, f"{name}_counter_collection.csv"))))
    vals = collections.defaultdict(float)
    kname = None
    disp = None
    for r in rows:
        if any(k in r["Kernel_Name"] for k in KERNELS):
            if disp is None:
                disp = r["Dispatch_Id"]
                kname = r["Kernel_Name"].split("(")[0]
            if r["Dispatch_Id"] == disp:
                vals[r["Counter_Name"]] += float(r["Counter_Value"])
    tr = list(csv.DictReader(open(os.path.join(d, name, f"{name}_kernel_trace.csv"))))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr if r["Dispatch_Id"] == disp]
    return kname, vals, (dur[0] * 1e-9 if dur else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--N", type=int, required=True)
    ap.add_argument("--m", type=int, required=True)
    a = ap.parse_args()
    k, clk, t_clk = load(a.pmc_dir, "clk")
    _, fetch, t_fetch = load(a.pmc_dir, "fetch")
    _, write, _ = load(a.pmc_dir, "write")
    _, tcc, _ = load(a.pmc_dir, "tcc")
    _, sq, _ = load(a.pmc_dir, "sq")
    N, m = a.N, a.m
    cyc = clk["GRBM_GUI_ACTIVE"] / 8.0
    rd = 2.0 * fetch["FETCH_SIZE"] * 1024.0
    wr = write["WRITE_SIZE"] * 1024.0
    flops = float(N) * m * (m + 1)
    out = {
        "kernel": k, "N": N, "m": m,
        "command": "rocprofv3 --pmc <group> --kernel-trace --output-format csv -- python3 bench.py --steps 1 "
                   "--warmup 0 --no-cpu-baseline (one pass per counter group, tools/gpu_gram_pmc.sh; "
                   "summary by tools/pmc_summary.py)",
        "duration_ms_under_pmc": t_fetch * 1e3,
        "FETCH_SIZE_KB": fetch["FETCH_SIZE"], "WRITE_SIZE_KB": write["WRITE_SIZE"],
        "hbm_bytes_per_launch": rd + wr,
        "traffic_note": "read bytes = 2 * FETCH_SIZE * 1024 (gfx950 correction, MI355X_MICROARCH.md §HBM); FETCH_SIZE "
                        "counts L2 misses to the fabric with Infinity-Cache hits included, so this is an upper bound "
                        "on HBM bytes",
        "algorithmic_bytes_per_launch": 8.0 * N * m,
        "tcc_hit_rate": tcc["TCC_HIT_sum"] / (tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]),
        "clock_ghz_effective": cyc / t_clk / 1e9,
        "mfma_cycles_per_instruction": clk["SQ_VALU_MFMA_BUSY_CYCLES"] / sq["SQ_INSTS_VALU_MFMA_F64"],
        "mfma_pipe_busy_frac": clk["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0),
        "lds_bank_conflict_cycles": sq["SQ_LDS_BANK_CONFLICT"],
        "algorithmic_tflops_under_pmc": flops / t_fetch / 1e12,
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
