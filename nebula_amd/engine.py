"""Host-side mirror of the reference's operator interfaces over the C ABI.

* ``GraphSpace``        -- one space on one GPU rank (the storaged's KVStore + schemas, and
                           graphd's StorageClient for that space).
* ``QueryBoundProcessor`` -- ``instance(space, bound_type)`` + ``process(GetNeighborsRequest)``
                           -> ``QueryResponse``, the shape of
                           src/storage/QueryBoundProcessor.h:23-28 / QueryBaseProcessor.h:47.
* ``GoExecutor``        -- GO N STEPS FROM ... OVER ... [WHERE] [YIELD [DISTINCT]], the
                           device-resident replacement of src/graph/GoExecutor.cpp:80-782.
* ``FindPathExecutor``  -- FIND SHORTEST PATH FROM ... TO ... OVER ... UPTO N STEPS (the
                           reference's FindExecutor is a stub, src/graph/FindExecutor.cpp:20-22;
                           semantics in include/nebula_amd.h), batched bidirectional BFS.

Everything executes in libnebula_amd.so on the GPU; there is no Python or CPU compute path.
"""
from __future__ import annotations

import ctypes as C
import struct
import time
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from . import expr as X
from ._lib import NbgError

OUT_BOUND, IN_BOUND = 0, 1


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def pack_kv(pairs):
    """[(key bytes, value bytes)] -> the C-ABI blob layout (bytes + n+1 offsets)."""
    ks = [bytes(k) for k, _ in pairs]
    vs = [bytes(v) for _, v in pairs]
    koff = np.zeros(len(ks) + 1, dtype=np.uint64)
    voff = np.zeros(len(vs) + 1, dtype=np.uint64)
    if ks:
        koff[1:] = np.cumsum([len(k) for k in ks])
        voff[1:] = np.cumsum([len(v) for v in vs])
    kb = np.frombuffer(b"".join(ks) + b"\0" * 8, dtype=np.uint8)
    vb = np.frombuffer(b"".join(vs) + b"\0" * 8, dtype=np.uint8)
    return kb, koff, vb, voff


class _RowsHandle:
    """Owns an nbg_rows until the last array viewing its host columns is gone (nbg_rows_free then
    returns the pinned blocks to the context's cache)."""

    def __init__(self, L, rows: _lib.Rows):
        self.L, self.rows = L, rows

    def __del__(self):
        rows, self.rows = self.rows, None
        if rows is not None:
            self.L.nbg_rows_free(C.byref(rows))


def _view(ptr, n, ctype, dtype, holder):
    """numpy view of n host values at ptr (no copy), keeping `holder` alive with it"""
    ct = (ctype * n).from_address(ptr)
    ct._holder = holder
    return np.frombuffer(ct, dtype=dtype)


_EMPTY_I64 = np.zeros(0, dtype=np.int64)
_ZERO1_I64 = np.zeros(1, dtype=np.int64)
_EMPTY_I64.flags.writeable = False
_ZERO1_I64.flags.writeable = False


class RowSet:
    """Typed columnar result (copied to host unless ``on_device``).  With ``holder`` (nbg_go) the
    INT / VID / DOUBLE columns are views of the engine's pinned result blocks, not copies; the
    rows are freed when the RowSet and every such column are gone."""

    def __init__(self, rows: _lib.Rows, keep_device: bool = False, holder: _RowsHandle | None = None):
        self.n_rows = int(rows.n_rows)
        self.types = [rows.col_types[i] for i in range(rows.n_cols)]
        self.edges_scanned = int(rows.edges_scanned)
        self.on_device = bool(rows.on_device)
        self.columns = []
        self.device_ptrs = []
        if self.on_device and not rows.row_vertex and not rows.n_vertices and not rows.n_failed \
                and not rows.n_vertex_cols:
            # a GO result left in HBM: column pointers only (the per-call cost of the bench loop)
            self.device_ptrs = [rows.cols[c] for c in range(len(self.types))]
            self.columns = [None] * len(self.types)
            self.row_vertex = _EMPTY_I64
            self.vertex_ids = _EMPTY_I64
            self.vertex_row_offsets = _ZERO1_I64
            self.failed = []
            self.vertex_columns = []
            return
        for c, t in enumerate(self.types):
            ptr = rows.cols[c]
            if self.on_device:
                self.device_ptrs.append(ptr)
                self.columns.append(None)
                continue
            if t == _lib.T_STRING and (self.n_rows == 0 or not rows.str_offsets[c]):
                self.columns.append([])
            elif t == _lib.T_STRING:
                offs = np.ctypeslib.as_array(rows.str_offsets[c], shape=(self.n_rows + 1,)).copy()
                raw = C.string_at(ptr, int(offs[-1])) if self.n_rows else b""
                self.columns.append([raw[offs[i]:offs[i + 1]].decode() for i in range(self.n_rows)])
            elif self.n_rows == 0:
                self.columns.append(np.zeros(0, dtype=np.uint8 if t == _lib.T_BOOL else
                                             (np.float64 if t == _lib.T_DOUBLE else np.int64)))
            elif t == _lib.T_BOOL:
                self.columns.append(np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(self.n_rows,)).astype(bool))
            elif t == _lib.T_DOUBLE:
                self.columns.append(_view(ptr, self.n_rows, C.c_double, np.float64, holder) if holder else
                                    np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_double)), shape=(self.n_rows,)).copy())
            else:
                self.columns.append(_view(ptr, self.n_rows, C.c_int64, np.int64, holder) if holder else
                                    np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_int64)), shape=(self.n_rows,)).copy())
        self.row_vertex = (np.ctypeslib.as_array(rows.row_vertex, shape=(self.n_rows,)).copy()
                           if rows.row_vertex and self.n_rows else np.zeros(0, dtype=np.int64))
        nv = int(rows.n_vertices)
        self.vertex_ids = (np.ctypeslib.as_array(rows.vertex_ids, shape=(nv,)).copy() if nv else np.zeros(0, np.int64))
        self.vertex_row_offsets = (np.ctypeslib.as_array(rows.vertex_row_offsets, shape=(nv + 1,)).copy()
                                   if nv else np.zeros(1, np.int64))
        self.failed = [(rows.failed_parts[i], rows.failed_codes[i]) for i in range(rows.n_failed)]
        # getBound tag props: vertex_columns[c][i] for vertex_ids[i] (None: no row of that tag)
        self.vertex_columns = []
        for c in range(rows.n_vertex_cols):
            t = rows.vertex_col_types[c]
            pres = rows.vertex_col_present[c]
            ptr = rows.vertex_cols[c]
            col = []
            for i in range(nv):
                if not pres[i]:
                    col.append(None)
                elif t == _lib.T_STRING:
                    o = rows.vertex_str_offsets[c]
                    col.append(C.string_at(ptr + o[i], o[i + 1] - o[i]).decode() if o[i + 1] > o[i] else "")
                elif t == _lib.T_BOOL:
                    col.append(bool(C.cast(ptr, C.POINTER(C.c_uint8))[i]))
                elif t == _lib.T_DOUBLE:
                    col.append(float(C.cast(ptr, C.POINTER(C.c_double))[i]))
                else:
                    col.append(int(C.cast(ptr, C.POINTER(C.c_int64))[i]))
            self.vertex_columns.append(col)

    def rows(self):
        out = []
        for r in range(self.n_rows):
            row = []
            for c, t in enumerate(self.types):
                v = self.columns[c][r]
                if t == _lib.T_BOOL:
                    row.append(bool(v))
                elif t == _lib.T_DOUBLE:
                    row.append(float(v))
                elif t == _lib.T_STRING:
                    row.append(v)
                else:
                    row.append(int(v))
            out.append(tuple(row))
        return out


class GraphSpace:
    def __init__(self, num_parts: int, device: int = 0, rank: int = 0, world_size: int = 1):
        self.L = _lib.load()
        self.num_parts, self.rank, self.world_size = num_parts, rank, world_size
        self._options: set[str] = set()
        self._plan_views: dict = {}  # (WHERE bytes, YIELD bytes) -> their C views (go())
        self._last_spec = None  # (argument key, GoSpec, start array) of the last go() call
        self.h = self.L.nbg_ctx_create(device, num_parts, rank, world_size)
        if not self.h:
            raise RuntimeError("nbg_ctx_create failed: no MI355X visible or bad arguments "
                               "(the engine has no CPU path)")

    def part_of(self, vid: int) -> int:
        """StorageClient partition rule: vid % num_parts + 1 over the unsigned bits (nbg_part_of)."""
        return int(self.L.nbg_part_of(vid, self.num_parts))

    # ---- lifecycle -------------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.L.nbg_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != _lib.NBG_OK:
            raise NbgError(rc, self.L.nbg_last_error(self.h).decode())

    def comm_init(self, unique_id: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        self._check(self.L.nbg_comm_init(self.h, buf))

    def comm_info(self) -> dict:
        """{"ranks": the communicator's own rank count (ncclCommCount for RCCL), "transport":
        "none" | "rccl" | "local"}"""
        r, t = C.c_int32(), C.c_int32()
        self._check(self.L.nbg_comm_info(self.h, C.byref(r), C.byref(t)))
        return {"ranks": r.value, "transport": {0: "none", 1: "rccl", 2: "local"}.get(t.value, t.value)}

    def comm_init_local(self, group_key: int):
        """In-process rank group on one device (tests of the sharded path)."""
        self._check(self.L.nbg_comm_init_local(self.h, int(group_key)))

    @staticmethod
    def comm_unique_id() -> bytes:
        L = _lib.load()
        buf = (C.c_uint8 * 128)()
        rc = L.nbg_comm_unique_id(buf)
        if rc != 0:
            raise NbgError(rc, "ncclGetUniqueId failed")
        return bytes(buf)

    def set_option(self, key: str, value: int):
        self._check(self.L.nbg_set_option(self.h, key.encode(), int(value)))
        self._options.add(key)

    def unset_option(self, key: str):
        """back to the engine's default for key"""
        self._check(self.L.nbg_set_option(self.h, key.encode(), -(1 << 63)))
        self._options.discard(key)

    def reset_options(self):
        """every option set through this handle back to the engine default"""
        for k in list(self._options):
            self.unset_option(k)

    # ---- schema + snapshot -----------------------------------------------------------
    def set_edge_schema(self, edge_type: int, fields: Sequence[tuple[str, int]], ver: int = 0):
        names = (C.c_char_p * max(len(fields), 1))(*[f.encode() for f, _ in fields])
        types = (C.c_int32 * max(len(fields), 1))(*[t for _, t in fields])
        self._check(self.L.nbg_schema_set_edge(self.h, edge_type, ver, len(fields), names, types))

    def set_tag_schema(self, tag_id: int, name: str, fields: Sequence[tuple[str, int]], ver: int = 0):
        """Tag schema + name (SchemaManager::getTagSchema / toTagID): enables $^.name.prop and
        $$.name.prop in GO WHERE / YIELD."""
        names = (C.c_char_p * max(len(fields), 1))(*[f.encode() for f, _ in fields])
        types = (C.c_int32 * max(len(fields), 1))(*[t for _, t in fields])
        self._check(self.L.nbg_schema_set_tag(self.h, tag_id, name.encode(), ver, len(fields), names, types))

    def load_part(self, part: int, pairs):
        kb, koff, vb, voff = pairs if isinstance(pairs, tuple) else pack_kv(pairs)
        n = len(koff) - 1
        self._check(self.L.nbg_snapshot_load_part(self.h, part, _p(kb), _p(koff), _p(vb), _p(voff), n))

    def gen_rmat(self, scale: int, edge_factor: int, seed: int, edge_type: int):
        self._check(self.L.nbg_snapshot_gen_rmat(self.h, scale, edge_factor, seed, edge_type))

    def finalize(self):
        self._check(self.L.nbg_snapshot_finalize(self.h))

    def write_part(self, part: int, pairs):
        """One part's batch of AddEdges / AddVertices KV puts (AddEdgesProcessor.cpp:15-31,
        AddVerticesProcessor.cpp:16-38); visible to queries after commit().  Needs
        set_option("writable", 1) before finalize()."""
        kb, koff, vb, voff = pairs if isinstance(pairs, tuple) else pack_kv(pairs)
        n = len(koff) - 1
        self._check(self.L.nbg_snapshot_write_part(self.h, part, _p(kb), _p(koff), _p(vb), _p(voff), n))

    def commit(self):
        """Rebuild the device snapshot from the written log (collective when world_size > 1)."""
        self._check(self.L.nbg_snapshot_commit(self.h))

    def info(self, edge_type: int) -> dict:
        si = _lib.SnapshotInfo()
        self._check(self.L.nbg_snapshot_info_get(self.h, edge_type, C.byref(si)))
        return {k: getattr(si, k) for k, _ in si._fields_}

    def out_degree(self, edge_type: int, vid: int) -> int:
        return int(self.L.nbg_snapshot_out_degree(self.h, edge_type, vid))

    def last_timing(self) -> dict:
        t = _lib.Timing()
        self._check(self.L.nbg_last_timing(self.h, C.byref(t)))
        d = {k: getattr(t, k) for k, _ in t._fields_ if k not in ("hops", "n_hops")}
        modes = {0: "top-down", 1: "bottom-up", 2: "sp-expand", 3: "sp-probe", 4: "sp-sweep", 5: "sp-walk"}
        d["hops"] = [{"mode": modes.get(h.mode, h.mode), "mode_id": h.mode, "final": bool(h.final_hop), "ms": h.ms,
                      "bytes": int(h.bytes), "c": list(h.c), "kernel_ms": h.kernel_ms,
                      "kernel_bytes": int(h.kernel_bytes),
                      "kernels": [k for k in h.kernels.decode().split("; ") if k] or ["nbg::k_expand"]}
                     for h in t.hops[:t.n_hops]]
        return d

    # ---- queries ---------------------------------------------------------------------
    def get_bound(self, edge_type: int, parts, vids, return_columns, filter: bytes | X.Expr | None = b"") -> RowSet:
        parts = np.ascontiguousarray(parts, dtype=np.int32)
        vids = np.ascontiguousarray(vids, dtype=np.int64)
        f = X.encode(filter)
        fb = np.frombuffer(f + b"\0", dtype=np.uint8)
        arr = (_lib.PropDef * max(len(return_columns), 1))()
        keep = []
        for i, col in enumerate(return_columns):
            name, owner, tag = (col if isinstance(col, tuple) else (col, _lib.OWNER_EDGE, 0))
            b = name.encode()
            keep.append(b)
            arr[i] = _lib.PropDef(b, owner, tag)
        rows = _lib.Rows()
        self._check(self.L.nbg_get_bound(self.h, edge_type, _p(parts), _p(vids), len(vids), _p(fb), len(f),
                                         arr, len(return_columns), C.byref(rows)))
        try:
            return RowSet(rows)
        finally:
            self.L.nbg_rows_free(C.byref(rows))

    def bound_stats(self, edge_type: int, parts, vids, return_columns, stats,
                    filter: bytes | X.Expr | None = b"") -> RowSet:
        """outBoundStats / inBoundStats: one row, stats[i] = SUM 1 / COUNT 2 / AVG 3 of column i."""
        parts = np.ascontiguousarray(parts, dtype=np.int32)
        vids = np.ascontiguousarray(vids, dtype=np.int64)
        f = X.encode(filter)
        fb = np.frombuffer(f + b"\0", dtype=np.uint8)
        arr = (_lib.PropDef * max(len(return_columns), 1))()
        keep = []
        for i, col in enumerate(return_columns):
            name, owner, tag = (col if isinstance(col, tuple) else (col, _lib.OWNER_EDGE, 0))
            b = name.encode()
            keep.append(b)
            arr[i] = _lib.PropDef(b, owner, tag)
        st = np.ascontiguousarray(list(stats) + [0], dtype=np.int32)
        if len(st) - 1 != len(return_columns):
            raise ValueError("one stat type per return column")
        rows = _lib.Rows()
        self._check(self.L.nbg_bound_stats(self.h, edge_type, _p(parts), _p(vids), len(vids), _p(fb), len(f),
                                           arr, _p(st), len(return_columns), C.byref(rows)))
        try:
            return RowSet(rows)
        finally:
            self.L.nbg_rows_free(C.byref(rows))

    @staticmethod
    def _input_table(inputs, n):
        """[(name, NBG_T_*, values)] -> ctypes arrays of the nbg_go_spec input table (+ keepalive)."""
        names = (C.c_char_p * len(inputs))(*[nm.encode() for nm, _, _ in inputs])
        types = (C.c_int32 * len(inputs))(*[t for _, t, _ in inputs])
        cols = (C.c_void_p * len(inputs))()
        offs = (C.c_void_p * len(inputs))()
        keep = [names, types, cols, offs]
        for i, (nm, t, vals) in enumerate(inputs):
            if len(vals) != n:
                raise ValueError(f"input column {nm} has {len(vals)} rows, starts has {n}")
            if t == _lib.T_STRING:
                bs = [v.encode() if isinstance(v, str) else bytes(v) for v in vals]
                o = np.zeros(n + 1, dtype=np.int64)
                o[1:] = np.cumsum([len(b) for b in bs]) if bs else []
                blob = np.frombuffer(b"".join(bs) + b"\0", dtype=np.uint8)
                cols[i], offs[i] = blob.ctypes.data, o.ctypes.data
                keep += [blob, o]
            else:
                dt = np.float64 if t == _lib.T_DOUBLE else np.uint8 if t == _lib.T_BOOL else np.int64
                a = np.ascontiguousarray(vals, dtype=dt)
                if a.size == 0:
                    a = np.zeros(1, dtype=dt)
                cols[i] = a.ctypes.data
                keep.append(a)
        return names, types, cols, offs, keep

    def go(self, starts, steps: int, edge_type: int, where=None, yields: Iterable = (), distinct: bool = False,
           keep_on_device: bool = False, inputs=None) -> RowSet:
        """GO ... FROM starts. `inputs`: the piped / variable rows ($-.prop / $var.prop), one per start,
        as [(name, NBG_T_*, values)] (GoExecutor::getPropFromInterim)."""
        starts = np.ascontiguousarray(starts, dtype=np.int64)
        w = X.encode(where)
        ys = tuple(X.encode(y) for y in yields)
        # a call repeating the previous one's arguments (the same start array object, plan and
        # flags) re-uses its prepared spec: building it cost ~15 us of Python per call (numpy's
        # ctypes pointer views), time the device sat idle between two queries.  The spec points at
        # the array's data, so values changed in place are read as they are at the call.
        ckey = (id(starts), len(starts), w, ys, steps, edge_type, bool(distinct), bool(keep_on_device))
        if not inputs and self._last_spec is not None and self._last_spec[0] == ckey:
            spec = self._last_spec[1]
            rows = _lib.Rows()
            self._check(self.L.nbg_go(self.h, C.byref(spec), C.byref(rows)))
            return self._go_rows(rows, keep_on_device)
        # the C views of the encoded WHERE / YIELD bytes, built once per distinct plan (a GO
        # repeated with the same plan re-uses them; they live as long as the space)
        key = (w, ys)
        views = self._plan_views.get(key)
        if views is None:
            wb = np.frombuffer(w + b"\0", dtype=np.uint8)
            ybufs = [C.create_string_buffer(y, len(y) + 1) for y in ys]
            yp = (C.c_void_p * max(len(ys), 1))(*[C.cast(b, C.c_void_p) for b in ybufs])
            yl = (C.c_size_t * max(len(ys), 1))(*[len(y) for y in ys])
            views = (wb, ybufs, yp, yl)
            if len(self._plan_views) >= 64:
                self._plan_views.clear()
            self._plan_views[key] = views
        wb, _, yp, yl = views
        spec = _lib.GoSpec(edge_type, steps, _p(starts), len(starts), _p(wb), len(w), yp, yl, len(ys),
                           int(distinct), int(keep_on_device))
        if inputs:
            names, types, cols, offs, _keep = self._input_table(inputs, len(starts))
            spec.n_inputs = len(inputs)
            spec.input_names, spec.input_types = names, types
            spec.input_cols, spec.input_str_offsets = cols, offs
        if not inputs:
            self._last_spec = (ckey, spec, starts)  # (the array is held while the spec points at it)
        rows = _lib.Rows()
        self._check(self.L.nbg_go(self.h, C.byref(spec), C.byref(rows)))
        return self._go_rows(rows, keep_on_device)

    def _go_rows(self, rows, keep_on_device: bool) -> RowSet:
        if keep_on_device:
            try:
                return RowSet(rows)
            finally:
                self.L.nbg_rows_free(C.byref(rows))
        # host result: zero-copy views of the pinned blocks, held until the columns are dropped
        return RowSet(rows, holder=_RowsHandle(self.L, rows))


    def shortest_path(self, src, dst, edge_type: int, max_steps: int = 5) -> "PathResult":
        """Pairwise shortest paths (src[i] -> dst[i]) over edge_type out-edges."""
        src = np.ascontiguousarray(src, dtype=np.int64)
        dst = np.ascontiguousarray(dst, dtype=np.int64)
        if src.shape != dst.shape:
            raise ValueError("src and dst must have the same length")
        rows = _lib.Rows()
        self._check(self.L.nbg_shortest_path(self.h, edge_type, _p(src), _p(dst), len(src), max_steps,
                                             C.byref(rows)))
        try:
            n = int(rows.n_rows)
            hops = (np.ctypeslib.as_array(C.cast(rows.cols[2], C.POINTER(C.c_int64)), shape=(n,)).copy()
                    if n else np.zeros(0, np.int64))
            off = np.ctypeslib.as_array(rows.path_offsets, shape=(n + 1,)).copy() if n else np.zeros(1, np.int64)
            tot = int(off[-1])
            vids = (np.ctypeslib.as_array(rows.path_vids, shape=(tot,)).copy() if tot else np.zeros(0, np.int64))
            # with world_size > 1 this rank answers pairs rank, rank + world, ... (columns 0 / 1)
            rs = np.ctypeslib.as_array(C.cast(rows.cols[0], C.POINTER(C.c_int64)), shape=(n,)).copy() if n else src[:0]
            rd = np.ctypeslib.as_array(C.cast(rows.cols[1], C.POINTER(C.c_int64)), shape=(n,)).copy() if n else dst[:0]
            return PathResult(rs, rd, hops, vids, off, int(rows.edges_scanned))
        finally:
            self.L.nbg_rows_free(C.byref(rows))


@dataclass
class PathResult:
    """FIND SHORTEST PATH result: per pair the hop count (-1 = unreachable) and the path (pair
    i's vids are path_vids[path_offsets[i]:path_offsets[i + 1]]; `paths` slices them on first use)."""
    src: np.ndarray
    dst: np.ndarray
    hops: np.ndarray
    path_vids: np.ndarray
    path_offsets: np.ndarray
    edges_scanned: int = 0

    @property
    def paths(self):
        if not hasattr(self, "_paths"):
            v, o = self.path_vids, self.path_offsets
            self._paths = [v[o[i]:o[i + 1]] for i in range(len(self.hops))]
        return self._paths

    def rows(self):
        return [(int(s), int(d), int(h), tuple(int(v) for v in p))
                for s, d, h, p in zip(self.src, self.dst, self.hops, self.paths)]


# ---- reference-shaped operator wrappers ---------------------------------------------------
@dataclass
class PropDef:
    """storage::cpp2::PropDef (src/interface/storage.thrift:43-49)."""
    owner: int
    name: str
    tag_id: int = 0


@dataclass
class GetNeighborsRequest:
    """storage::cpp2::GetNeighborsRequest (storage.thrift:125-133)."""
    space_id: int
    parts: dict
    edge_type: int
    filter: bytes = b""
    return_columns: list = field(default_factory=list)


@dataclass
class VertexData:
    vertex_id: int
    edge_rows: list


@dataclass
class QueryResponse:
    failed_codes: list
    edge_schema: list
    vertices: list


class QueryBoundProcessor:
    """QueryBoundProcessor::instance(...) / process(req) (QueryBoundProcessor.h:23-28)."""

    def __init__(self, space: GraphSpace, bound_type: int = OUT_BOUND):
        self.space, self.bound_type = space, bound_type

    @classmethod
    def instance(cls, space: GraphSpace, bound_type: int = OUT_BOUND):
        return cls(space, bound_type)

    def process(self, req: GetNeighborsRequest) -> QueryResponse:
        parts, vids = [], []
        for p, vs in req.parts.items():
            parts += [p] * len(vs)
            vids += list(vs)
        cols = [(c.name, c.owner, c.tag_id) for c in req.return_columns]
        # scanned as given for both bound types (QueryBaseProcessor.inl:39-40; the client negates for
        # in-bound, StorageClient.cpp:116) -- INTEGRATION.md's GpuBoundProcessor stub does the same
        et = req.edge_type
        rs = self.space.get_bound(et, parts, vids, cols, req.filter)
        rows = rs.rows()
        verts = []
        for i, vid in enumerate(rs.vertex_ids):
            a, b = rs.vertex_row_offsets[i], rs.vertex_row_offsets[i + 1]
            verts.append(VertexData(int(vid), rows[a:b]))
        names = [c.name for c in req.return_columns if c.owner == _lib.OWNER_EDGE]
        return QueryResponse([{"part_id": p, "code": c} for p, c in rs.failed], list(zip(names, rs.types)), verts)


SUM, COUNT, AVG = 1, 2, 3  # storage::cpp2::StatType (storage.thrift:51-55)


@dataclass
class QueryStatsResponse:
    """storage::cpp2::QueryStatsResponse (storage.thrift:95-99): schema + one row of stats."""
    failed_codes: list
    schema: list
    row: tuple | None


class QueryStatsProcessor:
    """QueryStatsProcessor::instance(...) / process(req) (QueryStatsProcessor.h, StorageServiceHandler.cpp:40-53).
    The request's PropDefs carry their stat (storage.thrift:43-49): pass them as (PropDef, stat)."""

    def __init__(self, space: GraphSpace, bound_type: int = OUT_BOUND):
        self.space, self.bound_type = space, bound_type

    @classmethod
    def instance(cls, space: GraphSpace, bound_type: int = OUT_BOUND):
        return cls(space, bound_type)

    def process(self, req: GetNeighborsRequest) -> QueryStatsResponse:
        parts, vids = [], []
        for p, vs in req.parts.items():
            parts += [p] * len(vs)
            vids += list(vs)
        cols = [(c.name, c.owner, c.tag_id) for c, _ in req.return_columns]
        stats = [st for _, st in req.return_columns]
        # the client already sends -edge_type for an in-bound request (StorageClient.cpp:116) and the
        # processor scans req.edge_type as is (QueryBaseProcessor.inl:39-40), as QueryBoundProcessor
        rs = self.space.bound_stats(req.edge_type, parts, vids, cols, stats, req.filter)
        kept = [c.name for c, _ in req.return_columns
                if self.bound_type == OUT_BOUND or c.owner != _lib.OWNER_EDGE or c.name.startswith("_")]
        failed = [{"part_id": p, "code": c} for p, c in rs.failed]
        if rs.n_rows == 0:
            return QueryStatsResponse(failed, [], None)
        return QueryStatsResponse(failed, list(zip(kept, rs.types)), rs.rows()[0])


# ---- write path ----------------------------------------------------------------
INT64_MAX = (1 << 63) - 1
_EDGE_KEY = struct.Struct("<iqiqqq")    # NebulaKeyUtils::edgeKey (NebulaKeyUtils.h:14-21)
_VERTEX_KEY = struct.Struct("<iqiq")    # NebulaKeyUtils::vertexKey


@dataclass
class EdgeKey:
    """storage::cpp2::EdgeKey (storage.thrift:111-118); edge_type < 0 is the in-edge."""
    src: int
    edge_type: int
    ranking: int
    dst: int


@dataclass
class Edge:
    key: EdgeKey
    props: bytes = b""   # RowWriter-encoded row (empty for in-edges)


@dataclass
class AddEdgesRequest:
    """storage::cpp2::AddEdgesRequest (storage.thrift:158-164): part -> edges."""
    parts: dict
    overwritable: bool = True

    @classmethod
    def insert(cls, space: "GraphSpace", edge_type: int, edges) -> "AddEdgesRequest":
        """INSERT EDGE as graphd sends it (InsertEdgeExecutor.cpp:143-162): per (src, dst, rank,
        props) an out-edge under src's part and an in-edge (-type, empty props) under dst's."""
        parts: dict = {}
        for src, dst, rank, props in edges:
            parts.setdefault(space.part_of(src), []).append(Edge(EdgeKey(src, edge_type, rank, dst), props))
            parts.setdefault(space.part_of(dst), []).append(Edge(EdgeKey(dst, -edge_type, rank, src), b""))
        return cls(parts)


@dataclass
class Tag:
    tag_id: int
    props: bytes


@dataclass
class Vertex:
    id: int
    tags: list


@dataclass
class AddVerticesRequest:
    """storage::cpp2::AddVerticesRequest (storage.thrift:150-156): part -> vertices."""
    parts: dict
    overwritable: bool = True


@dataclass
class ExecResponse:
    failed_codes: list


def _now_version() -> int:
    return INT64_MAX - time.time_ns() // 1000   # INT64_MAX - WallClock::fastNowInMicroSec()


class _WriteProcessor:
    def __init__(self, space: "GraphSpace", commit: bool = True, version: int | None = None):
        self.space, self.commit, self.version = space, commit, version

    @classmethod
    def instance(cls, space: "GraphSpace", commit: bool = True, version: int | None = None):
        return cls(space, commit, version)

    def _put(self, per_part) -> ExecResponse:
        failed = []
        for part, pairs in per_part.items():
            try:
                self.space.write_part(part, pairs)
            except NbgError as e:   # doPut's per-part result (BaseProcessor.h:47-73)
                failed.append({"part_id": part, "code": e.code})
        if self.commit:
            self.space.commit()
        return ExecResponse(failed)


class AddEdgesProcessor(_WriteProcessor):
    """AddEdgesProcessor::process (AddEdgesProcessor.cpp:15-31): one version INT64_MAX - now_us
    per request, key edgeKey(part, src, type, rank, dst, version), value = the edge's props.
    The puts become visible to queries at the space's next commit (commit=True: at once)."""

    def process(self, req: AddEdgesRequest) -> ExecResponse:
        ver = self.version if self.version is not None else _now_version()
        return self._put({part: [(_EDGE_KEY.pack(part, e.key.src, e.key.edge_type, e.key.ranking, e.key.dst, ver),
                                  e.props) for e in edges]
                          for part, edges in req.parts.items() if edges})


class AddVerticesProcessor(_WriteProcessor):
    """AddVerticesProcessor::process (AddVerticesProcessor.cpp:16-38): key vertexKey(part, vid,
    tag, INT64_MAX - now_us) per (vertex, tag), value = the tag's props."""

    def process(self, req: AddVerticesRequest) -> ExecResponse:
        ver = self.version if self.version is not None else _now_version()
        return self._put({part: [(_VERTEX_KEY.pack(part, v.id, t.tag_id, ver), t.props) for v in vs for t in v.tags]
                          for part, vs in req.parts.items() if vs})


class GoExecutor:
    """GO [N STEPS] FROM starts OVER edge [WHERE f] [YIELD [DISTINCT] cols]."""

    def __init__(self, space: GraphSpace, starts, edge_type: int, steps: int = 1, where=None, yields=(),
                 distinct: bool = False):
        self.space, self.starts, self.edge_type = space, starts, edge_type
        self.steps, self.where, self.yields, self.distinct = steps, where, list(yields), distinct

    def execute(self, keep_on_device: bool = False) -> RowSet:
        return self.space.go(self.starts, self.steps, self.edge_type, self.where, self.yields, self.distinct,
                             keep_on_device)


class FindPathExecutor:
    """FIND SHORTEST PATH FROM froms TO tos OVER edge UPTO n STEPS: every (from, to) combination,
    in from-major order (the reference only declares the executor, FindExecutor.cpp:20-22)."""

    def __init__(self, space: GraphSpace, froms, tos, edge_type: int, upto: int = 5):
        self.space, self.froms, self.tos = space, list(froms), list(tos)
        self.edge_type, self.upto = edge_type, upto

    def execute(self) -> PathResult:
        src = np.repeat(np.asarray(self.froms, dtype=np.int64), len(self.tos))
        dst = np.tile(np.asarray(self.tos, dtype=np.int64), len(self.froms))
        return self.space.shortest_path(src, dst, self.edge_type, self.upto)
