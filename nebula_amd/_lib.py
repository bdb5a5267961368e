"""ctypes binding of libnebula_amd.so (the C ABI in include/nebula_amd.h).

There is no CPU fallback: importing works anywhere (so the CPU test suite can check the
exported symbols), but creating a context needs the HIP library and an MI355X and raises
otherwise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = PKG / "libnebula_amd.so"

NBG_OK = 0
ERRORS = {
    -11: "E_LEADER_CHANGED", -13: "E_SPACE_NOT_FOUND", -14: "E_PART_NOT_FOUND",
    -21: "E_EDGE_PROP_NOT_FOUND", -22: "E_TAG_PROP_NOT_FOUND", -23: "E_IMPROPER_DATA_TYPE",
    -31: "E_INVALID_FILTER", -100: "E_UNKNOWN", -1000: "E_DEVICE", -1001: "E_INVALID_ARG",
    -1002: "E_STATE", -1003: "E_UNSUPPORTED", -1004: "E_EVAL", -1005: "E_COMM", -1006: "E_NOMEM",
}
T_BOOL, T_INT, T_VID, T_FLOAT, T_DOUBLE, T_STRING, T_TIMESTAMP = 1, 2, 3, 4, 5, 6, 21
OWNER_SOURCE, OWNER_DEST, OWNER_EDGE = 1, 2, 3
ABI_VERSION = 6  # NBG_ABI_VERSION of include/nebula_amd.h

# every symbol the header declares (tests/test_capi.py checks the .so exports them all)
EXPORTS = [
    "nbg_abi_version", "nbg_struct_size",
    "nbg_ctx_create", "nbg_ctx_destroy", "nbg_last_error", "nbg_comm_unique_id", "nbg_comm_init",
    "nbg_comm_init_local", "nbg_comm_info",
    "nbg_part_of", "nbg_rank_of_part", "nbg_schema_set_edge", "nbg_schema_set_tag", "nbg_snapshot_load_part",
    "nbg_snapshot_gen_rmat", "nbg_snapshot_finalize", "nbg_snapshot_write_part", "nbg_snapshot_commit",
    "nbg_snapshot_info_get",
    "nbg_snapshot_out_degree", "nbg_rows_free", "nbg_get_bound", "nbg_bound_stats", "nbg_go", "nbg_shortest_path",
    "nbg_last_timing", "nbg_set_option",
]


class NbgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)} ({code}): {msg}")
        self.code = code


class SnapshotInfo(C.Structure):
    _fields_ = [("num_vertices", C.c_int64), ("local_vertices", C.c_int64),
                ("local_out_edges", C.c_int64), ("local_in_edges", C.c_int64),
                ("device_bytes", C.c_int64), ("build_seconds", C.c_double),
                ("commits", C.c_int64), ("merge_commits", C.c_int64)]


class Rows(C.Structure):
    _fields_ = [("n_rows", C.c_int64), ("n_cols", C.c_int32), ("on_device", C.c_int32),
                ("col_types", C.POINTER(C.c_int32)), ("cols", C.POINTER(C.c_void_p)),
                ("str_offsets", C.POINTER(C.POINTER(C.c_int64))), ("row_vertex", C.POINTER(C.c_int64)),
                ("n_vertices", C.c_int64), ("vertex_ids", C.POINTER(C.c_int64)),
                ("vertex_row_offsets", C.POINTER(C.c_int64)), ("n_failed", C.c_int32),
                ("failed_parts", C.POINTER(C.c_int32)), ("failed_codes", C.POINTER(C.c_int32)),
                ("edges_scanned", C.c_uint64), ("path_offsets", C.POINTER(C.c_int64)),
                ("path_vids", C.POINTER(C.c_int64)), ("_impl", C.c_void_p),
                ("n_vertex_cols", C.c_int32), ("vertex_col_types", C.POINTER(C.c_int32)),
                ("vertex_cols", C.POINTER(C.c_void_p)), ("vertex_str_offsets", C.POINTER(C.POINTER(C.c_int64))),
                ("vertex_col_present", C.POINTER(C.POINTER(C.c_uint8)))]


class PropDef(C.Structure):
    _fields_ = [("name", C.c_char_p), ("owner", C.c_int32), ("tag_id", C.c_int32)]


class GoSpec(C.Structure):
    _fields_ = [("edge_type", C.c_int32), ("steps", C.c_int32), ("starts", C.c_void_p),
                ("n_starts", C.c_size_t), ("where", C.c_void_p), ("where_len", C.c_size_t),
                ("yields", C.POINTER(C.c_void_p)), ("yield_lens", C.POINTER(C.c_size_t)),
                ("n_yields", C.c_size_t), ("distinct", C.c_int32), ("keep_on_device", C.c_int32),
                ("n_inputs", C.c_size_t), ("input_names", C.POINTER(C.c_char_p)),
                ("input_types", C.POINTER(C.c_int32)), ("input_cols", C.POINTER(C.c_void_p)),
                ("input_str_offsets", C.POINTER(C.c_void_p))]


class HopStat(C.Structure):
    _fields_ = [("mode", C.c_int32), ("final_hop", C.c_int32), ("ms", C.c_double), ("bytes", C.c_uint64),
                ("c", C.c_uint64 * 8), ("kernel_ms", C.c_double), ("kernel_bytes", C.c_uint64),
                ("kernels", C.c_char * 160)]


MAX_HOP_STATS = 16


class Timing(C.Structure):
    _fields_ = [("total_ms", C.c_double), ("expand_ms", C.c_double), ("expand_launches", C.c_int64),
                ("edges_scanned", C.c_uint64), ("expand_bytes", C.c_uint64), ("steps_run", C.c_int32),
                ("bu_steps", C.c_int32), ("comm_ms", C.c_double), ("comm_bytes", C.c_uint64),
                ("n_hops", C.c_int32), ("hops", HopStat * MAX_HOP_STATS), ("host_waits", C.c_int32),
                ("spec_hops", C.c_int32), ("launches", C.c_int32),
                ("comm_calls", C.c_int32)]


_lib = None


def load(path: str | os.PathLike | None = None):
    """Load libnebula_amd.so (raises if it is missing: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise ImportError(f"{p} not built: run `make -C nebula_amd` (or __graft_entry__.build())")
    L = C.CDLL(str(p))
    vp, i32, i64, u64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_size_t
    sig = {
        "nbg_abi_version": (i32, []),
        "nbg_struct_size": (i64, [i32]),
        "nbg_ctx_create": (vp, [i32, i32, i32, i32]),
        "nbg_ctx_destroy": (None, [vp]),
        "nbg_last_error": (C.c_char_p, [vp]),
        "nbg_comm_unique_id": (i32, [vp]),
        "nbg_comm_init": (i32, [vp, vp]),
        "nbg_comm_init_local": (i32, [vp, i64]),
        "nbg_comm_info": (i32, [vp, vp, vp]),
        "nbg_part_of": (i32, [i64, i32]),
        "nbg_rank_of_part": (i32, [i32, i32]),
        "nbg_schema_set_edge": (i32, [vp, i32, i32, i32, C.POINTER(C.c_char_p), C.POINTER(i32)]),
        "nbg_schema_set_tag": (i32, [vp, i32, C.c_char_p, i32, i32, C.POINTER(C.c_char_p), C.POINTER(i32)]),
        "nbg_snapshot_load_part": (i32, [vp, i32, vp, vp, vp, vp, sz]),
        "nbg_snapshot_gen_rmat": (i32, [vp, i32, i32, u64, i32]),
        "nbg_snapshot_finalize": (i32, [vp]),
        "nbg_snapshot_write_part": (i32, [vp, i32, vp, vp, vp, vp, sz]),
        "nbg_snapshot_commit": (i32, [vp]),
        "nbg_snapshot_info_get": (i32, [vp, i32, C.POINTER(SnapshotInfo)]),
        "nbg_snapshot_out_degree": (i64, [vp, i32, i64]),
        "nbg_rows_free": (None, [C.POINTER(Rows)]),
        "nbg_get_bound": (i32, [vp, i32, vp, vp, sz, vp, sz, C.POINTER(PropDef), sz, C.POINTER(Rows)]),
        "nbg_bound_stats": (i32, [vp, i32, vp, vp, sz, vp, sz, C.POINTER(PropDef), vp, sz, C.POINTER(Rows)]),
        "nbg_go": (i32, [vp, C.POINTER(GoSpec), C.POINTER(Rows)]),
        "nbg_shortest_path": (i32, [vp, i32, vp, vp, sz, i32, C.POINTER(Rows)]),
        "nbg_last_timing": (i32, [vp, C.POINTER(Timing)]),
        "nbg_set_option": (i32, [vp, C.c_char_p, i64]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    # the ctypes mirrors below must match the library's struct layouts (include/nebula_amd.h)
    if L.nbg_abi_version() != ABI_VERSION:
        raise ImportError(f"{p}: ABI version {L.nbg_abi_version()}, this binding expects {ABI_VERSION}")
    for which, st in enumerate((Timing, HopStat, SnapshotInfo, GoSpec, Rows, PropDef)):
        if L.nbg_struct_size(which) != C.sizeof(st):
            raise ImportError(f"{p}: sizeof({st.__name__}) {C.sizeof(st)} != the library's {L.nbg_struct_size(which)}")
    _lib = L
    return L
