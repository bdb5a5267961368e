"""nebula_amd -- MI355X-native engine for Nebula Graph's neighbour-expansion hot path.

getOutBound / QueryBoundProcessor edge-prefix scan + WHERE filtering and the GoExecutor
multi-step frontier loop, as hand-written HIP kernels for gfx950 behind a C ABI
(include/nebula_amd.h).  See DESIGN.md.
"""
from . import expr  # noqa: F401
from ._lib import NbgError, load  # noqa: F401
from .engine import (FindPathExecutor, GetNeighborsRequest, GoExecutor, GraphSpace, PathResult,  # noqa: F401
                     PropDef, QueryBoundProcessor, QueryResponse, RowSet, pack_kv)

__all__ = ["GraphSpace", "QueryBoundProcessor", "GoExecutor", "FindPathExecutor", "PathResult",
           "GetNeighborsRequest", "PropDef",
           "QueryResponse", "RowSet", "NbgError", "expr", "load", "pack_kv"]
