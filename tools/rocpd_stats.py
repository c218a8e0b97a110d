"""Kernel statistics (name, calls, total / average / min / max us) from a rocprofv3 rocpd database
(the default output of `rocprofv3 --kernel-trace --stats -d DIR -o run`), the same table as the
CSV kernel_stats, optionally restricted to kernels whose name contains --match.

    python tools/rocpd_stats.py gpurun_out/.../run_results.db [--match chol] [--csv out.csv]
"""
import argparse
import sqlite3


def kernel_rows(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    q = f"select {name}, start, end from kernels"
    return [(n, s, e) for n, s, e in cur.execute(q)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--csv", default="")
    args = ap.parse_args()
    agg = {}
    for n, s, e in kernel_rows(args.db):
        if args.match and args.match not in n:
            continue
        d = (e - s) / 1000.0
        a = agg.setdefault(n, [0, 0.0, float("inf"), 0.0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = ["Name,Calls,TotalDurationUs,AverageUs,MinUs,MaxUs"]
    for n, (c, t, lo, hi) in rows:
        lines.append(f"\"{n}\",{c},{t:.1f},{t / c:.2f},{lo:.2f},{hi:.2f}")
    out = "\n".join(lines)
    if args.csv:
        with open(args.csv, "w") as f:
            f.write(out + "\n")
    print(out)


if __name__ == "__main__":
    main()
