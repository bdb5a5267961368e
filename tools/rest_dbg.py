#!/usr/bin/env python3
"""Summarise the per-wave records of the bottom-up rest pass (option bu_rest_dbg=1, records
appended to $NBG_DBG_FILE): wall_clock64 ticks (100 MHz) of each wave's start, hub copy end and
finish, pending rows handled, batches << 16 | chunk steps, rows handed to bu_rest_scan, entries
read, ticks spent in bu_rest_scan.   python3 tools/rest_dbg.py <file>"""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
i = 0
while i < len(raw):
    pk, nw = int(raw[i]), int(raw[i + 1])
    rec = raw[i + 2:i + 2 + nw * 8].reshape(nw, 8).astype(np.int64)
    i += 2 + nw * 8
    rec = rec[rec[:, 0] > 0]
    batches, rec[:, 4] = rec[:, 4] >> 16, rec[:, 4] & 0xffff
    t0 = rec[:, 0].min()
    start, hub, end = (rec[:, 0] - t0) / 100, (rec[:, 1] - rec[:, 0]) / 100, (rec[:, 2] - t0) / 100
    dur = (rec[:, 2] - rec[:, 1]) / 100
    print(f"pk={pk} waves={len(rec)} span_us={end.max():.1f} start_us p50={np.median(start):.1f} max={start.max():.1f} "
          f"hub_us p50={np.median(hub):.2f} max={hub.max():.2f}")
    print(f"  work_us p50={np.median(dur):.1f} p90={np.percentile(dur, 90):.1f} max={dur.max():.1f}; rows sum={rec[:, 3].sum()} "
          f"max={rec[:, 3].max()}; batches max={batches.max()} steps max={rec[:, 4].max()}; scan rows sum={rec[:, 5].sum()} max={rec[:, 5].max()}; "
          f"entries sum={rec[:, 6].sum()} max={rec[:, 6].max()}; scan_us p50={np.median(rec[:, 7]) / 100:.1f} max={rec[:, 7].max() / 100:.1f}")
    for k in np.argsort(-dur)[:8]:
        r = rec[k]
        print(f"    slow wave {k}: start {start[k]:.1f} work {dur[k]:.1f} us rows {r[3]} batches {batches[k]} steps {r[4]} scan_rows {r[5]} "
              f"entries {r[6]} scan_us {r[7] / 100:.1f}")
