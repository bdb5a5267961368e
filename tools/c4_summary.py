#!/usr/bin/env python3
"""Committed summary of a C4 (FIND SHORTEST PATH, 1024 pairs, RMAT-26) profiling session
(tools/c4_counters.sh <tag>): the bench line, per-query kernel times from the rocprofv3 kernel
statistics, and the PMC traffic of every scan launch of one query next to its byte model.

    python tools/c4_summary.py gpurun_out/<tag> profiles/<tag>_c4   -> <out>.md + <out>.json

Traffic = FETCH_SIZE x 2 (the gfx950 correction calibrated in profiles/r02c_calibration.md) +
WRITE_SIZE, per dispatch.  Byte models (paths.hip timing.expand_bytes): meet probe 24 B per X
tuple + 5 B per entry examined; BFS expansion 32 B per X tuple + 5 B per entry + 26 B per claim;
sweep 32 B per X tuple + 6 B per entry + 18 B per claim."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

MODEL = {"probe": lambda l: l["x"] * 24 + l["entries"] * 5,
         "expand": lambda l: l["x"] * 32 + l["entries"] * 5 + l["claims"] * 26,
         "sweep": lambda l: l["x"] * 32 + l["entries"] * 6 + l["claims"] * 18,
         "walk": lambda l: l["x"] * 24 + l["entries"] * 5}
KIND = {"k_dv_probe": "probe", "k_dv_expand": "expand", "k_dv_sweep": "sweep", "k_dv_walk_scan": "walk",
        "k_sp_probe": "probe", "k_sp_expand": "expand", "k_sp_sweep": "sweep"}


def kname(raw):
    return raw.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def last_json(p):
    return json.loads(Path(p).read_text().strip().splitlines()[-1])


def main():
    src, out = Path(sys.argv[1]), Path(sys.argv[2])
    bench = last_json(src / "kt_bench.json")
    queries = bench["steps"] * 2 + bench["warmup"] + 1  # timed + statistics loops, warm-up, parity
    stats = []
    for r in csv.DictReader(open(src / "c4_kernel_stats.csv")):
        n = kname(r["Name"])
        if "k_dv_" in n or "k_sp_" in n or "k_publish" in n:
            stats.append({"kernel": n, "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                          "us_per_query": float(r["TotalDurationNs"]) / 1e3 / queries})
    stats.sort(key=lambda s: -s["us_per_query"])
    # PMC: every dispatch of the scan kernels, grouped per query (the passes ran --steps 1 --warmup 1)
    per = defaultdict(dict)
    for f in sorted(src.glob("pmc/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            n = kname(r["Kernel_Name"])
            k = KIND.get(n.split("<")[0].replace("nbg::", ""))
            if not k:
                continue
            d = per[(f.parent.name, int(r["Dispatch_Id"]))]
            d["kernel"], d["kind"] = n, k
            d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    by_pass = defaultdict(list)
    for (pas, did), d in sorted(per.items()):
        by_pass[pas].append(d)
    launches = [l for l in bench["config"]["launches"]]

    def last_query(ds):
        # a query's scan dispatches: probe / expansion per BFS iteration (the speculative one too),
        # then the sweep steps; a probe after a sweep starts the next query
        qs, cur = [], []
        for d in ds:
            if d["kind"] == "probe" and cur and cur[-1]["kind"] in ("sweep", "walk"):
                qs.append(cur)
                cur = []
            cur.append(d)
        if cur:
            qs.append(cur)
        q = qs[-1] if qs else []
        out, seen = {}, defaultdict(int)
        for d in q:  # the n-th dispatch of a kind is iteration / step n
            seen[d["kind"]] += 1
            out[(d["kind"], seen[d["kind"]] - (1 if d["kind"] == "walk" else 0))] = d
        return out

    fetch, write = last_query(by_pass.get("p0", [])), last_query(by_pass.get("p1", []))
    rows = []
    for l in launches:
        m = MODEL[l["kind"]](l)
        key = (l["kind"], l["iter"])
        fb = fetch[key].get("FETCH_SIZE", 0.0) * 1024 * 2 if key in fetch else None
        wb = write[key].get("WRITE_SIZE", 0.0) * 1024 if key in write else None
        rows.append({**l, "model_bytes": m, "fetch_bytes_x2": fb, "write_bytes": wb,
                     "traffic_over_model": (fb + wb) / m if fb is not None and wb is not None and m else None})
    # per-query PMC bytes of each scan kind (every launch of the kind in the profiled query): what
    # bench.py reports as the dominant kind's measured traffic
    kinds = {}
    for r in rows:
        k = kinds.setdefault(r["kind"], {"launches": 0, "fetch_bytes_x2": 0.0, "write_bytes": 0.0,
                                          "model_bytes": 0.0, "complete": True})
        k["launches"] += 1
        k["model_bytes"] += r["model_bytes"]
        if r["fetch_bytes_x2"] is None or r["write_bytes"] is None:
            k["complete"] = False
        else:
            k["fetch_bytes_x2"] += r["fetch_bytes_x2"]
            k["write_bytes"] += r["write_bytes"]
    summary = {"bench": {**{k: bench[k] for k in ("metric", "value", "unit", "ms_per_step", "parity")},
                         "config": {"workload": bench["config"]["workload"]}},
               "query_kinds": kinds,
               "device_ms_per_query": bench["roofline"]["device_ms_per_query"],
               "kernels": stats, "launches": rows, "source": str(src)}
    out.with_suffix(".json").write_text(json.dumps(summary, indent=1))
    md = [f"# C4 profile `{src.name}` (FIND SHORTEST PATH, 1024 pairs, RMAT-26, 1 MI355X)", "",
          f"bench (rocprofv3 run): {bench['ms_per_step']:.3f} ms/query, {bench['value']:.0f} pairs/s, "
          f"parity {bench['parity']['status']}; device {summary['device_ms_per_query']:.3f} ms/query", "",
          "## kernel time per query (rocprofv3 --kernel-trace --stats)", "",
          "| kernel | calls | avg us | us / query |", "|---|---|---|---|"]
    md += [f"| `{s['kernel']}` | {s['calls']} | {s['avg_us']:.1f} | {s['us_per_query']:.1f} |" for s in stats]
    md += ["", f"sum of listed kernels: {sum(s['us_per_query'] for s in stats):.1f} us / query", "",
           "## scan launches of one query: PMC traffic vs byte model", "",
           "| launch | iter | X | entries | claims | HIP-event ms | model MB | FETCH x2 MB | WRITE MB | traffic / model |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        tf = "-" if r["traffic_over_model"] is None else f"{r['traffic_over_model']:.2f}"
        fb = "-" if r["fetch_bytes_x2"] is None else f"{r['fetch_bytes_x2'] / 1e6:.1f}"
        wb = "-" if r["write_bytes"] is None else f"{r['write_bytes'] / 1e6:.1f}"
        md.append(f"| {r['kind']} | {r['iter']} | {r['x']} | {r['entries']} | {r['claims']} | {r['ms']:.3f} | "
                  f"{r['model_bytes'] / 1e6:.1f} | {fb} | {wb} | {tf} |")
    out.with_suffix(".md").write_text("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main()
