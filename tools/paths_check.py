#!/usr/bin/env python3
"""Debug aid: FIND SHORTEST PATH with the meet probe on / off against the oracle at one scale."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
    npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    import oracle as O
    from nebula_amd import GraphSpace, synth
    sp = GraphSpace(64)
    sp.set_edge_schema(1, [("weight", 2)])
    sp.gen_rmat(scale, 16, 1, 1)
    sp.finalize()
    s, t = synth.pairs(scale, 16, 1, npairs)
    res = {}
    for probe in (0, 1):
        sp.set_option("sp_probe", probe)
        try:
            r = sp.shortest_path(s, t, 1, 8)
            res[probe] = r.rows()
            print(f"probe={probe}: ok, edges={r.edges_scanned}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"probe={probe}: {e}", flush=True)
    if scale <= 20:
        st = O.Store(64)
        st.set_edge_schema(1, [("weight", O.INT)], name="follow")
        st.load_rmat(scale, 16, 1, 1)
        want = st.shortest_path(s, t, 1, 8)
        print("oracle rows", len(want.rows()) if hasattr(want, "rows") else "?", flush=True)
    if 0 in res and 1 in res:
        bad = [i for i, (a, b) in enumerate(zip(res[0], res[1])) if a != b]
        print("mismatches probe on/off:", len(bad), [(res[0][i], res[1][i]) for i in bad[:5]], flush=True)
        for i in bad[:3]:
            for probe in (1, 0):
                sp.set_option("sp_probe", probe)
                one = sp.shortest_path(s[i:i + 1], t[i:i + 1], 1, 8)
                print("  pair", i, "probe", probe, "alone:", one.rows(), sp.last_timing()["steps_run"], flush=True)
            sp.set_option("sp_probe", 1)
            sub = sp.shortest_path(s[:i + 1], t[:i + 1], 1, 8).rows()
            print("  prefix batch", i + 1, "last row:", sub[-1], flush=True)
    else:
        # bisect the failing pairs with probe on
        sp.set_option("sp_probe", 1)
        for i in range(npairs):
            try:
                sp.shortest_path(s[i:i + 1], t[i:i + 1], 1, 8)
            except Exception as e:  # noqa: BLE001
                sp.set_option("sp_probe", 0)
                r0 = sp.shortest_path(s[i:i + 1], t[i:i + 1], 1, 8).rows()
                sp.set_option("sp_probe", 1)
                print("single pair fails:", i, int(s[i]), int(t[i]), r0, e, flush=True)
                break
        else:
            print("no single pair fails alone", flush=True)
    sp.close()


if __name__ == "__main__":
    main()
