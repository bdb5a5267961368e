"""Per-kernel stats and an averaged query timeline from a rocprofv3 SQLite database (rocpd).
usage: python tools/db_timeline.py run_results.db [first_kernel_of_query [skip [take]]]
Queries are cut at each launch of `first_kernel_of_query`; `skip` of them are dropped (warmup) and
the next `take` (default 10) are averaged launch by launch when they share one kernel sequence."""
import re
import sqlite3
import sys


def short(n):
    n = re.sub(r"\(.*$", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))
    return n if len(n) < 70 else n[:67] + "..."


db = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else None
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
take = int(sys.argv[4]) if len(sys.argv) > 4 else 10
c = sqlite3.connect(db)
rows = [(short(n), s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
stats = {}
for k, s, e in rows:
    st = stats.setdefault(k, [0, 0.0, 1e18])
    st[0] += 1
    st[1] += (e - s) / 1000.0
    st[2] = min(st[2], (e - s) / 1000.0)
print("| kernel | calls | avg us | min us |\n|---|---|---|---|")
for k, (n, t, m) in sorted(stats.items(), key=lambda x: -x[1][1])[:30]:
    print(f"| `{k}` | {n} | {t / n:.1f} | {m:.1f} |")
if first:
    cuts = [i for i, r in enumerate(rows) if r[0].startswith(first)] + [len(rows)]
    qs = [rows[cuts[i]:cuts[i + 1]] for i in range(len(cuts) - 1)][skip:skip + take]
    # the last launch of a cut may be followed by unrelated work: keep the common sequence
    seqs = {}
    for q in qs:
        seqs.setdefault(tuple(k for k, _, _ in q), []).append(q)
    seq, group = max(seqs.items(), key=lambda x: len(x[1]))
    print(f"\n# {len(group)} of {len(qs)} queries share this sequence (averaged)")
    n = len(seq)
    off = [0.0] * n
    dur = [0.0] * n
    gap = [0.0] * n
    for q in group:
        t0 = q[0][1]
        prev = t0
        for i, (k, s, e) in enumerate(q):
            off[i] += (s - t0) / 1000.0
            dur[i] += (e - s) / 1000.0
            gap[i] += (s - prev) / 1000.0
            prev = e
    g = len(group)
    for i, k in enumerate(seq):
        print(f"{off[i] / g:9.1f} gap {gap[i] / g:7.1f} dur {dur[i] / g:8.1f}  {k}")
    busy = sum(dur) / g
    span = (off[-1] + dur[-1]) / g
    print(f"# busy {busy:.1f} us, idle {span - busy:.1f} us, span {span:.1f} us (first launch start to last launch end)")
