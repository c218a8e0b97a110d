"""Summarise the PMC passes of tools/gpu_pmc_sgram.sh for the sparse Gram kernel (the first dispatch whose
name starts with sparse_gram): bytes beyond L2 against the algorithmic bytes of bench.py's hbm line.
usage: pmc_summary_sgram.py <pmc_dir> <out.json>"""
import collections
import csv
import json
import os
import sys


def load(d, name):
    rows = list(csv.DictReader(open(os.path.join(d, name, f"{name}_counter_collection.csv"))))
    vals, kname, disp = collections.defaultdict(float), None, None
    for r in rows:
        if r["Kernel_Name"].lstrip("void ").startswith("scs::sparse_gram") or "sparse_gram_" in r["Kernel_Name"]:
            if disp is None:
                disp, kname = r["Dispatch_Id"], r["Kernel_Name"].split("(")[0]
            if r["Dispatch_Id"] == disp:
                vals[r["Counter_Name"]] += float(r["Counter_Value"])
    tr = list(csv.DictReader(open(os.path.join(d, name, f"{name}_kernel_trace.csv"))))
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr if r["Dispatch_Id"] == disp]
    return kname, vals, (dur[0] * 1e-9 if dur else None)


def main():
    d, out = sys.argv[1], sys.argv[2]
    k, clk, t_clk = load(d, "clk")
    _, fetch, t_fetch = load(d, "fetch")
    _, write, _ = load(d, "write")
    _, tcc, _ = load(d, "tcc")
    _, sq, _ = load(d, "sq")
    rd = fetch["FETCH_SIZE"] * 1024.0
    wr = write["WRITE_SIZE"] * 1024.0
    res = {
        "kernel": k,
        "command": "rocprofv3 --pmc <group> --kernel-trace -- python3 bench.py --config c5ggn --steps 1 --warmup 0 "
                   "--no-cpu-baseline (one pass per counter group, tools/gpu_pmc_sgram.sh)",
        "duration_ms_under_pmc": t_fetch * 1e3 if t_fetch else None,
        "FETCH_SIZE_KB": fetch["FETCH_SIZE"], "WRITE_SIZE_KB": write["WRITE_SIZE"],
        "read_bytes_raw": rd, "read_bytes_x2": 2.0 * rd, "write_bytes": wr,
        "traffic_note": "FETCH_SIZE counts L2 misses to the fabric (Infinity-Cache hits included); the gfx950 x2 "
                        "correction of MI355X_MICROARCH.md is calibrated for 16-B/lane streaming reads only -- this "
                        "kernel's reads are 2-8 B/lane gathers, so both the raw and the x2 figure are listed",
        "tcc_hit_rate": tcc["TCC_HIT_sum"] / max(1.0, tcc["TCC_HIT_sum"] + tcc["TCC_MISS_sum"]),
        "clock_ghz_effective": (clk["GRBM_GUI_ACTIVE"] / 8.0) / t_clk / 1e9 if t_clk else None,
        "sq": dict(sq),
        "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / max(1.0, sq["SQ_WAVES"]),
        "lds_insts_per_wave": sq["SQ_INSTS_LDS"] / max(1.0, sq["SQ_WAVES"]),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
