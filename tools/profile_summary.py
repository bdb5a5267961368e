#!/usr/bin/env python3
"""Summarise one tools/gpu_profile.sh session into profiles/<tag>_summary.json (+ .md).

Inputs (under gpurun_out/<tag>/): bench.json (the default bench line), kt/run_kernel_stats.csv
(rocprofv3 --kernel-trace --stats), pmc_fetch/ and pmc_write/ run_counter_collection.csv (one
--pmc pass each).  Per query kernel: calls, average duration, FETCH_SIZE and WRITE_SIZE per
launch.  FETCH_SIZE is doubled for the gfx950 wide-read under-count (MI355X_MICROARCH.md, HBM
section) and reported raw as well.

    python tools/profile_summary.py r01b [--out profiles]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

BUILD = ("k_gen_rmat", "rocprim", "k_edge_keys", "k_dedup", "k_kept_src", "k_gather", "k_tr_col", "k_edge_src",
         "k_flip", "k_rowptr", "k_ht_insert", "k_narrow", "k_scatter", "k_iota", "k_fill", "k_bswap", "k_unflip",
         "k_row_part", "k_hub_key", "k_build_slab", "k_out_deg", "k_sorted_bounds", "k_src_global", "k_sub_lo",
         "k_count_deg", "k_row_counts", "k_not_u32", "k_col_vid", "k_pack_col", "k_minmax_w", "k_last_live",
         "k_build_pair", "k_build_slab", "k_gen_", "k_rmat_", "k_old_version", "k_ov_edges", "k_iota_off",
         "k_count_unknown", "k_hash_part", "k_odeg8", "k_live_bounds", "k_class_key")


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").strip()


def pmc(path: Path, counter: str):
    d = defaultdict(list)
    if not path.exists():
        return d
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return d


def main():
    tag = sys.argv[1]
    outdir = Path(sys.argv[sys.argv.index("--out") + 1]) if "--out" in sys.argv else Path("profiles")
    src = Path("gpurun_out") / tag
    stats = list(csv.DictReader(open(src / "kt" / "run_kernel_stats.csv")))
    fetch = pmc(src / "pmc_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    write = pmc(src / "pmc_write" / "run_counter_collection.csv", "WRITE_SIZE")
    bench = None
    for f in ("bench.json", "kt_bench.json"):
        p = src / f
        if p.exists() and p.read_text().strip():
            bench = json.loads(p.read_text().strip().splitlines()[-1])
            break
    kernels = []
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"])):
        name = short(r["Name"])
        if any(b in r["Name"] for b in BUILD) and "fillBuffer" not in name and "copyBuffer" not in name:
            continue
        f = fetch.get(name, [])
        w = write.get(name, [])
        kernels.append({
            "kernel": name,
            "calls": int(r["Calls"]),
            "avg_us": float(r["AverageNs"]) / 1e3,
            "total_ms": float(r["TotalDurationNs"]) / 1e6,
            "fetch_bytes_raw": (sum(f) / len(f) * 1024) if f else None,  # FETCH_SIZE is in KiB
            "fetch_bytes_x2": (2 * sum(f) / len(f) * 1024) if f else None,
            "write_bytes": (sum(w) / len(w) * 1024) if w else None,
        })
    out = {"tag": tag, "bench": bench, "query_kernels": kernels,
           "note": "kernel stats from rocprofv3 --kernel-trace --stats of bench.py --no-cpu --steps 5 --warmup 1; "
                   "FETCH_SIZE/WRITE_SIZE from separate --pmc passes (bench.py --steps 2 --warmup 1), per launch; "
                   "fetch_bytes_x2 applies the gfx950 wide-read correction"}
    outdir.mkdir(exist_ok=True)
    (outdir / f"{tag}_summary.json").write_text(json.dumps(out, indent=1) + "\n")
    lines = [f"# rocprof summary {tag}", ""]
    if bench:
        lines.append(f"bench: {bench['value']:.1f} {bench['unit']}, {bench['ms_per_step']:.3f} ms/query; "
                     f"roofline {json.dumps(bench.get('roofline'))}")
        lines.append("")
    lines.append("| kernel | calls | avg us | total ms | FETCH_SIZE x2 (MB/launch) | WRITE_SIZE (MB/launch) |")
    lines.append("|---|---|---|---|---|---|")
    for k in kernels:
        fb = f"{k['fetch_bytes_x2'] / 1e6:.1f}" if k["fetch_bytes_x2"] is not None else "-"
        wb = f"{k['write_bytes'] / 1e6:.1f}" if k["write_bytes"] is not None else "-"
        lines.append(f"| `{k['kernel'][:60]}` | {k['calls']} | {k['avg_us']:.1f} | {k['total_ms']:.2f} | {fb} | {wb} |")
    (outdir / f"{tag}_summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
