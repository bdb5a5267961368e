#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv (query kernels only, or all with --all)."""
import csv
import sys

BUILD = ("k_gen_rmat", "rocprim", "k_edge_keys", "k_dedup", "k_kept_src", "k_gather", "k_tr_col", "k_edge_src",
         "k_flip", "k_rowptr", "k_ht_insert", "k_narrow", "k_scatter", "k_iota", "k_fill", "k_bswap", "k_unflip",
         "k_row_part", "k_hub_key", "k_build_slab", "k_out_deg", "k_sorted_bounds", "k_src_global", "k_sub_lo")
rows = list(csv.DictReader(open(sys.argv[1])))
show_all = "--all" in sys.argv
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if not show_all and any(b in r["Name"] for b in BUILD):
        continue
    print(f"{name[-58:]:58s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs']) / 1e3:10.1f} "
          f"tot_ms={float(r['TotalDurationNs']) / 1e6:9.2f}")
