"""Repeat test_rmat_bottom_up_packed_predicate's queries and print the hop counters of every query
whose edges_scanned differs from the oracle's (a nondeterministic undercount seen in round 6)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import numpy as np  # noqa: E402

from test_gpu_parity import FOLLOW, OPS, oracle_rmat, seeds_from, SEED  # noqa: E402
from nebula_amd import GraphSpace  # noqa: E402
from nebula_amd import expr as X  # noqa: E402
import oracle as O  # noqa: E402

sp = GraphSpace(64)
sp.set_edge_schema(FOLLOW, [("weight", O.INT)])
sp.gen_rmat(12, 16, SEED, FOLLOW)
sp.finalize()
st = oracle_rmat(12)
starts = sorted(set(seeds_from(12, 48, seed=29)))
wcol = X.AliasProp("follow", "weight")
bad = tot = 0
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for hub_cap in (36 * 1024, 16):
        for fin in (0, 1):
            for k, v in {"bu_force": 1, "bu_qpred": 1, "bu_hub_cap": hub_cap, "bu_fin": fin}.items():
                sp.set_option(k, v)
            for k in (-5, 0, 499, 1000):
                for op, mk in OPS.items():
                    w = mk(wcol, k)
                    g = sp.go(starts, 2, FOLLOW, where=w, yields=[X.EdgeDst("follow")], distinct=True)
                    r_ = st.go(starts, 2, FOLLOW, where=w.encode(), yields=[X.EdgeDst("follow").encode()], distinct=True)
                    tot += 1
                    rows_ok = np.array_equal(np.sort(g.columns[0]), np.sort(r_.int_col(0)))
                    if g.edges_scanned != r_.edges_scanned or not rows_ok:
                        bad += 1
                        hops = [(h["mode"], h["c"][:6], h.get("kernels")) for h in sp.last_timing()["hops"]]
                        print(f"rep {rep} hub {hub_cap} fin {fin} k {k} op {op}: scanned {g.edges_scanned} "
                              f"oracle {r_.edges_scanned} rows_ok {rows_ok} hops {hops}", flush=True)
print(f"{bad} of {tot} queries off", flush=True)
