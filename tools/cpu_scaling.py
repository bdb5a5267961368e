#!/usr/bin/env python3
"""CPU baseline vs graph size: the oracle (tests/oracle.py over oracle/refcpu.cpp, the KV-store
restatement of storaged + graphd) running the bench query's shape -- GO 3 STEPS FROM 64 seeds
OVER follow WHERE follow.weight > 499 YIELD DISTINCT follow._dst -- on RMAT-16 .. RMAT-22 in the
faithful mode bench.py reports (1 storaged host x 10 bucket threads, min 3 vertices per bucket,
one graphd thread) and with one bucket thread per usable core.  One JSON line per scale; the
largest scales run once after no warm-up (their single query takes tens of seconds).

    python3 tools/cpu_scaling.py 16 18 20 22 > gpurun_out/<tag>/cpu_scaling.jsonl
"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import bench
    import oracle as O
    from nebula_amd import expr as X
    from nebula_amd import synth

    usable, machine, model = bench.host_cpu()
    golden = json.loads((ROOT / "tests" / "golden" / "rmat_digests.json").read_text())
    w = (X.AliasProp("follow", "weight") > 499).encode()
    y = [X.EdgeDst("follow").encode()]
    for scale in [int(a) for a in sys.argv[1:]] or [16, 18, 20]:
        st = O.Store(64)
        st.set_edge_schema(1, [("weight", O.INT)], name="follow")
        t0 = time.perf_counter()
        st.load_rmat(scale, 16, 1, 1, versions=1, threads=min(16, usable))
        load_s = time.perf_counter() - t0
        starts = synth.seeds(scale, 16, 1, 64)
        row = {"scale": scale, "load_s": round(load_s, 2), "host_cores": usable, "machine_cores": machine,
               "cpu_model": model}
        for mode, handlers in (("faithful", 10), ("all_cores", usable)):
            reps = 3 if scale <= 18 else 1
            best = None
            r = None
            for _ in range(reps):
                t1 = time.perf_counter()
                r = st.go(starts, 3, 1, where=w, yields=y, distinct=True, hosts=1, handlers=handlers, min_per_bucket=3)
                dt = time.perf_counter() - t1
                best = dt if best is None else min(best, dt)
            row[mode] = {"seconds": round(best, 3), "gteps": r.edges_scanned / best / 1e9, "reps": reps,
                         "threads": min(handlers, usable) + 1}
            row["edges_scanned"] = r.edges_scanned
            row["rows"] = r.nrows
            g = golden.get(f"go3_where499_distinct_s{scale}")
            row["parity"] = ("no golden" if g is None else
                             "digest ok" if O.digest(r.int_col(0)) == g["sha256"] and r.nrows == g["n_rows"]
                             else "mismatch")
        print(json.dumps(row), flush=True)
        del st


if __name__ == "__main__":
    main()
