"""nebula_amd -- MI355X-native engine for Nebula Graph's neighbour-expansion hot path.

getOutBound / QueryBoundProcessor edge-prefix scan + WHERE filtering, outBoundStats, the
GoExecutor multi-step frontier loop and FIND SHORTEST PATH, as hand-written HIP kernels for
gfx950 behind a C ABI (include/nebula_amd.h).  See DESIGN.md.
"""
from . import expr  # noqa: F401
from ._lib import NbgError, load  # noqa: F401
from .engine import (AVG, COUNT, SUM, AddEdgesProcessor, AddEdgesRequest, AddVerticesProcessor,  # noqa: F401
                     AddVerticesRequest, Edge, EdgeKey, ExecResponse, Tag, Vertex, FindPathExecutor, GetNeighborsRequest, GoExecutor,  # noqa: F401
                     GraphSpace, PathResult, PropDef, QueryBoundProcessor, QueryResponse, QueryStatsProcessor,
                     QueryStatsResponse, RowSet, pack_kv)

__all__ = ["GraphSpace", "QueryBoundProcessor", "QueryStatsProcessor", "GoExecutor", "FindPathExecutor",
           "PathResult", "GetNeighborsRequest", "PropDef", "QueryResponse", "QueryStatsResponse", "RowSet",
           "NbgError", "expr", "load", "pack_kv", "SUM", "COUNT", "AVG", "AddEdgesProcessor", "AddEdgesRequest",
           "AddVerticesProcessor", "AddVerticesRequest", "Edge", "EdgeKey", "Tag", "Vertex", "ExecResponse"]
