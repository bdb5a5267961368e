"""ctypes wrapper around oracle/librefcpu.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference path (oracle/refcpu.cpp).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg load it, and only as the checker.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "oracle" / "librefcpu.so"

# cpp2::SupportedType
BOOL, INT, VID, FLOAT, DOUBLE, STRING, TIMESTAMP = 1, 2, 3, 4, 5, 6, 21
SOURCE, DEST, EDGE = 1, 2, 3


def build() -> Path:
    srcs = [ROOT / "oracle" / f for f in ("refcpu.cpp", "rmat_graph.cpp", "refcpu.h", "rmat_def.h")]
    if not LIB.exists() or any(LIB.stat().st_mtime < s.stat().st_mtime for s in srcs):
        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB))
        vp, i32, i64, u64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_size_t
        P = C.POINTER
        sig = {
            "ora_store_new": (vp, [i32]),
            "ora_store_free": (None, [vp]),
            "ora_store_put_batch": (None, [vp, i32, vp, vp, vp, vp, sz]),
            "ora_store_finalize": (None, [vp]),
            "ora_store_num_keys": (sz, [vp]),
            "ora_store_part_size": (sz, [vp, i32, P(sz), P(sz)]),
            "ora_store_dump_part": (None, [vp, i32, vp, vp, vp, vp]),
            "ora_schema_set_edge": (None, [vp, i32, i32, i32, P(C.c_char_p), P(i32)]),
            "ora_schema_set_tag": (None, [vp, i32, C.c_char_p, i32, i32, P(C.c_char_p), P(i32)]),
            "ora_schema_set_edge_name": (None, [vp, i32, C.c_char_p]),
            "ora_encode_row": (sz, [P(i32), P(i64), P(C.c_double), P(C.c_char_p), i32, vp, sz]),
            "ora_encode_varint": (sz, [u64, vp]),
            "ora_edge_key": (sz, [i32, i64, i32, i64, i64, i64, vp]),
            "ora_rmat_edges": (None, [i32, i32, u64, vp, vp, vp]),
            "ora_rmat_vid": (i64, [u64, u64]),
            "ora_rmat_load": (None, [vp, i32, i32, u64, i32, i32, i32]),
            "ora_get_bound": (vp, [vp, i32, i32, vp, vp, sz, vp, sz, vp, sz, i32, i32]),
            "ora_bound_stats": (vp, [vp, i32, i32, vp, vp, sz, vp, sz, vp, vp, sz, i32, i32]),
            "ora_gen_buckets": (i32, [vp, vp, sz, i32, i32, vp]),
            "ora_go": (vp, [vp, vp, sz, i32, i32, vp, sz, vp, vp, sz, i32, i32, i32, i32, P(u64)]),
            "ora_go_set_inputs": (None, [vp, sz, sz, P(C.c_char_p), P(i32), P(vp), P(vp)]),
            "ora_shortest_path": (vp, [vp, vp, vp, sz, i32, i32]),
            "ora_res_code": (i32, [vp]),
            "ora_res_error": (C.c_char_p, [vp]),
            "ora_res_nrows": (sz, [vp]),
            "ora_res_ncols": (i32, [vp]),
            "ora_res_type": (i32, [vp, sz, i32]),
            "ora_res_int": (i64, [vp, sz, i32]),
            "ora_res_double": (C.c_double, [vp, sz, i32]),
            "ora_res_str": (C.c_void_p, [vp, sz, i32, P(sz)]),
            "ora_res_int_col": (None, [vp, i32, vp]),
            "ora_res_nfailed": (sz, [vp]),
            "ora_res_failed": (None, [vp, sz, P(i32), P(i32)]),
            "ora_res_row_vertex": (i64, [vp, sz]),
            "ora_res_nvertices": (sz, [vp]),
            "ora_res_vertex_id": (i64, [vp, sz]),
            "ora_res_vertex_nrows": (sz, [vp, sz]),
            "ora_res_vertex_ncols": (i32, [vp]),
            "ora_res_vertex_type": (i32, [vp, sz, i32]),
            "ora_res_vertex_int": (i64, [vp, sz, i32]),
            "ora_res_vertex_str": (C.c_void_p, [vp, sz, i32, P(sz)]),
            "ora_res_vertex_bytes": (C.c_void_p, [vp, sz, P(sz)]),
            "ora_res_edge_bytes": (C.c_void_p, [vp, sz, P(sz)]),
            "ora_res_schema_ncols": (i32, [vp, i32]),
            "ora_res_schema_name": (C.c_char_p, [vp, i32, i32]),
            "ora_res_schema_type": (i32, [vp, i32, i32]),
            "ora_res_free": (None, [vp]),
            "ora_rmat_graph_new": (vp, [i32, i32, u64, i32]),
            "ora_rmat_graph_free": (None, [vp]),
            "ora_rmat_graph_info": (None, [vp, P(i64), P(i64)]),
            "ora_rmat_graph_out_degree": (i64, [vp, i64]),
            "ora_rmat_graph_go": (i64, [vp, vp, sz, i32, i32, i64, i32, i32, P(P(i64)), P(u64)]),
            "ora_rmat_graph_go_msum": (None, [vp, vp, sz, i32, i32, P(u64), P(u64)]),
            "ora_rmat_graph_shortest_path": (None, [vp, vp, vp, sz, i32, i32, vp, vp, P(P(i64))]),
            "ora_free": (None, [vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def edge_key(part, src, etype, rank, dst, ver) -> bytes:
    buf = C.create_string_buffer(40)
    n = lib().ora_edge_key(part, src, etype, rank, dst, ver, buf)
    return buf.raw[:n]


def vertex_key(part, vid, tag, ver) -> bytes:
    import struct
    return struct.pack("<iqiq", part, vid, tag, ver)


def encode_row(values) -> bytes:
    """Schemaless RowWriter encoding of python values (int->INT, float->DOUBLE, numpy.float32->FLOAT,
    bool, str)."""
    n = len(values)
    tags = (C.c_int32 * max(n, 1))()
    iv = (C.c_int64 * max(n, 1))()
    dv = (C.c_double * max(n, 1))()
    sv = (C.c_char_p * max(n, 1))()
    for i, v in enumerate(values):
        if isinstance(v, np.float32):  # a FLOAT column (4 bytes)
            tags[i], dv[i] = FLOAT, float(v)
        elif isinstance(v, bool):
            tags[i], iv[i] = BOOL, int(v)
        elif isinstance(v, int):
            tags[i], iv[i] = INT, v
        elif isinstance(v, float):
            tags[i], dv[i] = DOUBLE, v
        else:
            tags[i], sv[i] = STRING, v.encode()
    cap = 64 + sum(len(str(v)) + 10 for v in values)
    buf = C.create_string_buffer(cap)
    m = lib().ora_encode_row(tags, iv, dv, sv, n, buf, cap)
    return buf.raw[:m]


def encode_varint(v: int) -> bytes:
    buf = C.create_string_buffer(10)
    n = lib().ora_encode_varint(v, buf)
    return buf.raw[:n]


def pack_kv(pairs):
    """[(key, val)] -> (kbytes, koff, vbytes, voff) numpy arrays (the C-ABI blob layout)."""
    ks = [k for k, _ in pairs]
    vs = [v for _, v in pairs]
    koff = np.zeros(len(ks) + 1, dtype=np.uint64)
    voff = np.zeros(len(vs) + 1, dtype=np.uint64)
    koff[1:] = np.cumsum([len(k) for k in ks]) if ks else []
    voff[1:] = np.cumsum([len(v) for v in vs]) if vs else []
    kb = np.frombuffer(b"".join(ks) + b"\0", dtype=np.uint8)
    vb = np.frombuffer(b"".join(vs) + b"\0", dtype=np.uint8)
    return kb, koff, vb, voff


def _cstrs(xs):
    arr = (C.c_char_p * max(len(xs), 1))()
    for i, x in enumerate(xs):
        arr[i] = x.encode()
    return arr


class Result:
    def __init__(self, h):
        self.h = h
        L = lib()
        self.code = L.ora_res_code(h)
        self.error = L.ora_res_error(h).decode()

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_res_free(self.h)
            self.h = None

    @property
    def nrows(self):
        return lib().ora_res_nrows(self.h)

    def cell(self, r, c):
        L = lib()
        t = L.ora_res_type(self.h, r, c)
        if t == 0:
            return L.ora_res_int(self.h, r, c)
        if t == 1:
            return L.ora_res_double(self.h, r, c)
        if t == 2:
            return bool(L.ora_res_int(self.h, r, c))
        if t == 3:
            n = C.c_size_t()
            p = L.ora_res_str(self.h, r, c, C.byref(n))
            return C.string_at(p, n.value).decode()
        return None

    def rows(self):
        nc = lib().ora_res_ncols(self.h)
        return [tuple(self.cell(r, c) for c in range(nc)) for r in range(self.nrows)]

    def int_col(self, c=0) -> np.ndarray:
        out = np.empty(self.nrows, dtype=np.int64)
        if self.nrows:
            lib().ora_res_int_col(self.h, c, _ptr(out))
        return out

    def failed(self):
        L = lib()
        out = []
        for i in range(L.ora_res_nfailed(self.h)):
            p, c = C.c_int32(), C.c_int32()
            L.ora_res_failed(self.h, i, C.byref(p), C.byref(c))
            out.append((p.value, c.value))
        return out

    def row_vertex(self, r):
        return lib().ora_res_row_vertex(self.h, r)

    def vertices(self):
        L = lib()
        out = []
        nc = L.ora_res_vertex_ncols(self.h)
        for i in range(L.ora_res_nvertices(self.h)):
            vals = []
            for c in range(nc):
                t = L.ora_res_vertex_type(self.h, i, c)
                if t == 0:
                    vals.append(L.ora_res_vertex_int(self.h, i, c))
                elif t == 3:
                    n = C.c_size_t()
                    p = L.ora_res_vertex_str(self.h, i, c, C.byref(n))
                    vals.append(C.string_at(p, n.value).decode())
                else:
                    vals.append(None)
            out.append((L.ora_res_vertex_id(self.h, i), vals))
        return out

    def vertex_nrows(self, i) -> int:
        return lib().ora_res_vertex_nrows(self.h, i)

    def edge_bytes(self, i) -> bytes:
        n = C.c_size_t()
        p = lib().ora_res_edge_bytes(self.h, i, C.byref(n))
        return C.string_at(p, n.value)

    def schema(self, which=0):
        L = lib()
        return [(L.ora_res_schema_name(self.h, which, c).decode(), L.ora_res_schema_type(self.h, which, c))
                for c in range(L.ora_res_schema_ncols(self.h, which))]


class Store:
    def __init__(self, num_parts: int):
        self.num_parts = num_parts
        self.h = lib().ora_store_new(num_parts)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_store_free(self.h)
            self.h = None

    def put(self, part: int, pairs):
        kb, koff, vb, voff = pack_kv(pairs)
        lib().ora_store_put_batch(self.h, part, _ptr(kb), _ptr(koff), _ptr(vb), _ptr(voff), len(pairs))

    def finalize(self):
        lib().ora_store_finalize(self.h)

    def num_keys(self):
        return lib().ora_store_num_keys(self.h)

    def dump_part(self, part):
        """(kbytes, koff, vbytes, voff) numpy blobs of one finalized part (the C-ABI layout)."""
        kbn, vbn = C.c_size_t(), C.c_size_t()
        n = lib().ora_store_part_size(self.h, part, C.byref(kbn), C.byref(vbn))
        kb = np.zeros(kbn.value + 8, dtype=np.uint8)
        vb = np.zeros(vbn.value + 8, dtype=np.uint8)
        koff = np.zeros(n + 1, dtype=np.uint64)
        voff = np.zeros(n + 1, dtype=np.uint64)
        lib().ora_store_dump_part(self.h, part, _ptr(kb), _ptr(koff), _ptr(vb), _ptr(voff))
        return kb, koff, vb, voff

    def set_edge_schema(self, etype, fields, ver=0, name=None):
        names = _cstrs([f for f, _ in fields])
        types = (C.c_int32 * max(len(fields), 1))(*[t for _, t in fields])
        lib().ora_schema_set_edge(self.h, etype, ver, len(fields), names, types)
        if name:
            lib().ora_schema_set_edge_name(self.h, etype, name.encode())

    def set_tag_schema(self, tag, fields, ver=0, name=None):
        names = _cstrs([f for f, _ in fields])
        types = (C.c_int32 * max(len(fields), 1))(*[t for _, t in fields])
        lib().ora_schema_set_tag(self.h, tag, (name or str(tag)).encode(), ver, len(fields), names, types)

    def load_rmat(self, scale, edge_factor, seed, etype, versions=1, threads=8):
        lib().ora_rmat_load(self.h, scale, edge_factor, seed, etype, versions, threads)

    def get_bound(self, etype, parts, vids, cols, filt=b"", in_bound=False, handlers=10, min_per_bucket=3):
        parts = np.ascontiguousarray(parts, dtype=np.int32)
        vids = np.ascontiguousarray(vids, dtype=np.int64)
        arr = (PropDef * max(len(cols), 1))()
        keep = []
        for i, (name, owner, tag) in enumerate(cols):
            b = name.encode()
            keep.append(b)
            arr[i] = PropDef(b, owner, tag)
        fb = np.frombuffer(filt + b"\0", dtype=np.uint8)
        h = lib().ora_get_bound(self.h, etype, int(in_bound), _ptr(parts), _ptr(vids), len(vids),
                                _ptr(fb), len(filt), arr, len(cols), handlers, min_per_bucket)
        return Result(h)

    def bound_stats(self, etype, parts, vids, cols, stats, filt=b"", in_bound=False, handlers=10,
                    min_per_bucket=3):
        """QueryStatsProcessor (outBoundStats / inBoundStats): stats[i] = SUM 1 / COUNT 2 / AVG 3"""
        parts = np.ascontiguousarray(parts, dtype=np.int32)
        vids = np.ascontiguousarray(vids, dtype=np.int64)
        arr = (PropDef * max(len(cols), 1))()
        keep = []
        for i, (name, owner, tag) in enumerate(cols):
            b = name.encode()
            keep.append(b)
            arr[i] = PropDef(b, owner, tag)
        st = np.ascontiguousarray(list(stats) + [0], dtype=np.int32)
        fb = np.frombuffer(filt + b"\0", dtype=np.uint8)
        h = lib().ora_bound_stats(self.h, etype, int(in_bound), _ptr(parts), _ptr(vids), len(vids), _ptr(fb),
                                  len(filt), arr, _ptr(st), len(cols), handlers, min_per_bucket)
        return Result(h)

    def go(self, starts, steps, etype, where=b"", yields=(), distinct=False, hosts=1,
           handlers=10, min_per_bucket=3, inputs=None):
        """inputs: the $- / $var rows, one per start, as [(name, type, values)]."""
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        keep = []
        if inputs:
            n = len(starts)
            names = _cstrs([nm for nm, _, _ in inputs])
            types = (C.c_int32 * len(inputs))(*[t for _, t, _ in inputs])
            cols = (C.c_void_p * len(inputs))()
            offs = (C.c_void_p * len(inputs))()
            for i, (nm, t, vals) in enumerate(inputs):
                if t == STRING:
                    bs = [v.encode() for v in vals]
                    o = np.zeros(n + 1, dtype=np.int64)
                    o[1:] = np.cumsum([len(b) for b in bs]) if bs else []
                    blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
                    cols[i], offs[i] = blob.ctypes.data, o.ctypes.data
                    keep += [blob, o]
                else:
                    dt = np.float64 if t == DOUBLE else np.uint8 if t == BOOL else np.int64
                    a = np.ascontiguousarray(list(vals) or [0], dtype=dt)
                    cols[i] = a.ctypes.data
                    keep.append(a)
            keep += [names, types, cols, offs]
            lib().ora_go_set_inputs(self.h, n, len(inputs), names, types, cols, offs)
        ys = [bytes(y) for y in yields]
        yb = (C.c_void_p * max(len(ys), 1))()
        ylen = (C.c_size_t * max(len(ys), 1))()
        bufs = []
        for i, y in enumerate(ys):
            b = C.create_string_buffer(y, len(y) + 1)
            bufs.append(b)
            yb[i] = C.cast(b, C.c_void_p)
            ylen[i] = len(y)
        wb = np.frombuffer(where + b"\0", dtype=np.uint8)
        scanned = C.c_uint64()
        h = lib().ora_go(self.h, _ptr(starts), len(starts), steps, etype, _ptr(wb), len(where),
                         yb, ylen, len(ys), int(distinct), hosts, handlers, min_per_bucket,
                         C.byref(scanned))
        r = Result(h)
        r.edges_scanned = scanned.value
        return r

    def shortest_path(self, src, dst, etype, max_steps):
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        return Result(lib().ora_shortest_path(self.h, _ptr(src), _ptr(dst), len(src), etype, max_steps))


class PropDef(C.Structure):
    _fields_ = [("name", C.c_char_p), ("owner", C.c_int32), ("tag_id", C.c_int32)]


class RmatGraph:
    """Index-space restatement of GO / FIND SHORTEST PATH on the synthetic RMAT graph
    (oracle/rmat_graph.cpp) -- the checker at the configured sizes (RMAT-18..26)."""

    def __init__(self, scale, edge_factor=16, seed=1, threads=None):
        self.scale = scale
        self.threads = threads or min(16, os.cpu_count() or 1)
        self.h = lib().ora_rmat_graph_new(scale, edge_factor, seed, self.threads)
        if not self.h:
            raise ValueError("bad RMAT parameters")

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_rmat_graph_free(self.h)
            self.h = None

    def info(self):
        nv, ne = C.c_int64(), C.c_int64()
        lib().ora_rmat_graph_info(self.h, C.byref(nv), C.byref(ne))
        return {"num_vertices": nv.value, "num_edges": ne.value}

    OPS = {">": 1, ">=": 2, "<": 3, "<=": 4, "==": 5, "!=": 6}

    def go(self, starts, steps, where_gt=None, distinct=False, where=None):
        """sorted int64 result vids of GO steps [WHERE weight > where_gt | WHERE weight <op> k for
        where=(op, k)] YIELD _dst [DISTINCT] and the edges scanned (rows the storage returned
        over all hops)"""
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        out = C.POINTER(C.c_int64)()
        scanned = C.c_uint64()
        op, k = (0, 0) if where_gt is None else (1, where_gt)
        if where is not None:
            op, k = self.OPS[where[0]], where[1]
        n = lib().ora_rmat_graph_go(self.h, _ptr(starts), len(starts), steps, op, int(k), int(distinct),
                                    self.threads, C.byref(out), C.byref(scanned))
        try:
            res = np.ctypeslib.as_array(out, shape=(n,)).copy() if n > 0 else np.zeros(0, dtype=np.int64)
        finally:
            lib().ora_free(C.cast(out, C.c_void_p))
        return res, scanned.value

    def go_msum(self, starts, steps):
        """order-independent digest of a plain GO's rows (YIELD _dst): (rows, sum of
        splitmix64(vid) mod 2^64, xor of the same), and the edges scanned -- see msum()"""
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        out = (C.c_uint64 * 3)()
        scanned = C.c_uint64()
        lib().ora_rmat_graph_go_msum(self.h, _ptr(starts), len(starts), steps, self.threads, out, C.byref(scanned))
        return (int(out[0]), int(out[1]), int(out[2])), scanned.value

    def out_degree(self, idx):
        return int(lib().ora_rmat_graph_out_degree(self.h, int(idx)))

    def shortest_path(self, src, dst, max_steps):
        """(hops int64[n], [path vids per pair]) -- ora_shortest_path's definition"""
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        n = len(src)
        hops = np.empty(max(n, 1), dtype=np.int64)
        off = np.empty(n + 1, dtype=np.int64)
        pv = C.POINTER(C.c_int64)()
        lib().ora_rmat_graph_shortest_path(self.h, _ptr(src), _ptr(dst), n, max_steps, self.threads, _ptr(hops),
                                           _ptr(off), C.byref(pv))
        try:
            flat = np.ctypeslib.as_array(pv, shape=(max(int(off[-1]), 1),))[:int(off[-1])].copy()
        finally:
            lib().ora_free(C.cast(pv, C.c_void_p))
        return hops[:n], [flat[off[i]:off[i + 1]] for i in range(n)]


def digest(vids) -> str:
    """SHA-256 of a result column as sorted little-endian int64 (the committed golden form)."""
    import hashlib
    a = np.sort(np.asarray(vids, dtype=np.int64)).astype("<i8")
    return hashlib.sha256(a.tobytes()).hexdigest()


def rmat_edges(scale, edge_factor, seed):
    E = edge_factor << scale
    s = np.empty(E, dtype=np.int64)
    d = np.empty(E, dtype=np.int64)
    w = np.empty(E, dtype=np.int64)
    lib().ora_rmat_edges(scale, edge_factor, seed, _ptr(s), _ptr(d), _ptr(w))
    return s, d, w


def rmat_vid(idx, seed):
    return lib().ora_rmat_vid(idx, seed)


def part_of(vid: int, num_parts: int) -> int:
    return (vid % (1 << 64)) % num_parts + 1


os.environ.setdefault("OMP_NUM_THREADS", "8")


def msum(vids, chunk=1 << 26):
    """(rows, sum of splitmix64(vid) mod 2^64, xor of the same) of a result column: the
    order-independent digest of ora_rmat_graph_go_msum, for result sets too large to sort"""
    v = np.asarray(vids, dtype=np.int64).view(np.uint64)
    s = 0
    x = np.uint64(0)
    with np.errstate(over="ignore"):
        for i in range(0, len(v), chunk):
            z = v[i:i + chunk] + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            s = (s + int(z.sum(dtype=np.uint64))) & ((1 << 64) - 1)
            x ^= np.bitwise_xor.reduce(z) if len(z) else np.uint64(0)
    return len(v), s, int(x)
