/*
 * nebula_amd.h -- C ABI of the MI355X neighbour-expansion engine.
 *
 * This is the drop-in boundary for the reference's getBound / GO hot path (Nebula Graph
 * v1.0.0-beta).  Every entry point is plain C (pointers + sizes, no C++/torch types), so a
 * storaged/graphd built from the reference can bind it directly (see INTEGRATION.md for the
 * C++ operator shapes that wrap it).  Each function names the reference interface it replaces.
 *
 * Error convention: functions return 0 on success or a negative code.  Codes -1..-100 are the
 * reference's storage::cpp2::ErrorCode values (src/interface/storage.thrift:13-35); codes
 * <= -1000 are engine errors.  nbg_last_error() gives the message for the calling context.
 * All calls on one context are serialised internally (the reference's processors may call
 * from many RPC worker threads: QueryBaseProcessor.inl:407-423).
 */
#ifndef NEBULA_AMD_H_
#define NEBULA_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (storage.thrift:13-35 + engine range) -------------------------------- */
#define NBG_OK 0
#define NBG_E_LEADER_CHANGED (-11)
#define NBG_E_SPACE_NOT_FOUND (-13)
#define NBG_E_PART_NOT_FOUND (-14)
#define NBG_E_EDGE_PROP_NOT_FOUND (-21)
#define NBG_E_TAG_PROP_NOT_FOUND (-22)
#define NBG_E_IMPROPER_DATA_TYPE (-23)
#define NBG_E_INVALID_FILTER (-31)
#define NBG_E_UNKNOWN (-100)
#define NBG_E_DEVICE (-1000)      /* HIP runtime / kernel failure                          */
#define NBG_E_INVALID_ARG (-1001) /* bad argument (null pointer, unknown edge type, ...)   */
#define NBG_E_STATE (-1002)       /* call out of order (query before snapshot finalize)   */
#define NBG_E_UNSUPPORTED (-1003) /* expression / column shape the engine does not run    */
#define NBG_E_EVAL (-1004)        /* expression evaluation error at the final GO step
                                     (GoExecutor.cpp:754-758 fails the whole query)       */
#define NBG_E_COMM (-1005)        /* RCCL failure                                          */
#define NBG_E_NOMEM (-1006)       /* device allocation failed                              */

/* cpp2::SupportedType values (src/interface/common.thrift:30-46) */
#define NBG_T_BOOL 1
#define NBG_T_INT 2
#define NBG_T_VID 3
#define NBG_T_FLOAT 4
#define NBG_T_DOUBLE 5
#define NBG_T_STRING 6
#define NBG_T_TIMESTAMP 21

/* cpp2::PropOwner (storage.thrift:37-41) */
#define NBG_OWNER_SOURCE 1
#define NBG_OWNER_DEST 2
#define NBG_OWNER_EDGE 3

typedef struct nbg_ctx nbg_ctx;

/* ---- context ------------------------------------------------------------------------------
 * One context = one space on one GPU (one rank of `world_size`).  Replaces the storaged's
 * KVStore* + SchemaManager* pair handed to QueryBoundProcessor::instance
 * (src/storage/QueryBoundProcessor.h:23-28) and graphd's StorageClient for that space.
 * num_parts: the space's partition count (CreateSpaceProcessor.cpp:10-11); a vid lives in part
 * (uint64)vid % num_parts + 1 (StorageClient.cpp:10-11) and part p on rank p % world_size
 * (pickHosts, CreateSpaceProcessor.cpp:77-90).                                              */
nbg_ctx* nbg_ctx_create(int32_t device, int32_t num_parts, int32_t rank, int32_t world_size);
void nbg_ctx_destroy(nbg_ctx* ctx);
const char* nbg_last_error(const nbg_ctx* ctx);

/* Multi-GPU: RCCL communicator over xGMI.  Rank 0 calls nbg_comm_unique_id and the launcher
 * broadcasts the 128 bytes (e.g. via torch.distributed's store); every rank then calls
 * nbg_comm_init.  Replaces StorageClient::collectResponse's RPC scatter/gather
 * (src/storage/client/StorageClient.inl:74-159) with a per-step all-to-all.                 */
int32_t nbg_comm_unique_id(uint8_t out[128]);
int32_t nbg_comm_init(nbg_ctx* ctx, const uint8_t unique_id[128]);
/* Test transport: contexts of ONE process (one per rank, any device) with the same group_key
 * form a group whose collectives are device-to-device copies; the sharded algorithm then runs
 * unchanged with world_size ranks on a single GPU.  Each rank must call from its own thread. */
int32_t nbg_comm_init_local(nbg_ctx* ctx, int64_t group_key);
/* The context's communicator as the transport itself reports it: *ranks = ncclCommCount of
 * the RCCL communicator (the LocalComm group size; 1 without one), *transport = 0 none,
 * 1 RCCL, 2 LocalComm.  Lets a multi-GPU bench line show the rank count RCCL really formed.  */
int32_t nbg_comm_info(nbg_ctx* ctx, int32_t* ranks, int32_t* transport);

/* ABI version of this header's structs and signatures.  Caller-allocated structs (nbg_timing,
 * nbg_hop_stat, nbg_snapshot_info, nbg_go_spec, nbg_rows) change layout between versions: an
 * integration compares nbg_abi_version() with the NBG_ABI_VERSION it was built against and
 * refuses to run on a mismatch (INTEGRATION.md "ABI versioning").                          */
#define NBG_ABI_VERSION 6
int32_t nbg_abi_version(void);
/* sizeof of the caller-allocated structs as the library was built: 0 nbg_timing, 1
 * nbg_hop_stat, 2 nbg_snapshot_info, 3 nbg_go_spec, 4 nbg_rows, 5 nbg_prop_def; -1 otherwise */
int64_t nbg_struct_size(int32_t which);

/* pure arithmetic helpers (host, no GPU needed) */
int32_t nbg_part_of(int64_t vid, int32_t num_parts);          /* StorageClient.cpp:238-243 */
int32_t nbg_rank_of_part(int32_t part, int32_t world_size);   /* CreateSpaceProcessor.cpp:77-90 */

/* ---- schema (meta SchemaManager::getEdgeSchema, src/meta/SchemaManager.h:38) ------------ */
int32_t nbg_schema_set_edge(nbg_ctx* ctx, int32_t edge_type, int32_t schema_ver,
                            int32_t nfields, const char* const* names, const int32_t* types);

/* Vertex tag schema (SchemaManager::getTagSchema, src/meta/SchemaManager.h:32-36) plus the tag's
 * name, which graphd resolves $^.tag.prop / $$.tag.prop with (SchemaManager::toTagID,
 * GoExecutor.cpp:475-478).  Vertex keys of registered tags (NebulaKeyUtils.h:14-17, 24 bytes) are
 * decoded by nbg_snapshot_load_part into per-vertex columns used by GO's $^ / $$ props.       */
int32_t nbg_schema_set_tag(nbg_ctx* ctx, int32_t tag_id, const char* tag_name, int32_t schema_ver,
                           int32_t nfields, const char* const* names, const int32_t* types);

/* ---- snapshot builder --------------------------------------------------------------------
 * Consumes a partition's KV pairs in the reference byte layout (NebulaKeyUtils.h:14-21 keys,
 * dataman RowWriter rows) -- what RocksEngine::prefix iterates (RocksEngine.cpp:191-200) --
 * and builds the GPU-resident CSR + SoA property columns.  Keys/values are concatenated blobs
 * with n+1 offsets.  Keys of unregistered tags / edge types are ignored.  Call once per part (any
 * order), then nbg_snapshot_finalize.                                                       */
int32_t nbg_snapshot_load_part(nbg_ctx* ctx, int32_t part, const uint8_t* key_bytes,
                               const uint64_t* key_offsets, const uint8_t* val_bytes,
                               const uint64_t* val_offsets, size_t n);
/* Synthetic RMAT graph generated on the device (definition in DESIGN.md): the KV the
 * reference's INSERT EDGE path would write (out-edge + empty in-edge, rank 0, one version),
 * produced directly in the decoded-tuple stage of the same builder.                        */
int32_t nbg_snapshot_gen_rmat(nbg_ctx* ctx, int32_t scale, int32_t edge_factor, uint64_t seed,
                              int32_t edge_type);
int32_t nbg_snapshot_finalize(nbg_ctx* ctx);
/* Write path.  nbg_snapshot_write_part takes one part's batch of the KV puts
 * AddEdgesProcessor::process / AddVerticesProcessor::process hand to doPut
 * (AddEdgesProcessor.cpp:15-31, AddVerticesProcessor.cpp:16-38: keys carry version
 * INT64_MAX - now_us; an identical key overwrites) in the same blob layout as load_part.
 * Before the first finalize it is load_part.  After it the snapshot must have been finalized
 * with option "writable" = 1 (which keeps the decoded tuples on the device); the batch is
 * decoded behind them and becomes visible at nbg_snapshot_commit, which rebuilds the CSRs from
 * the device-resident tuples (queries in between read the previous commit).  Commit is
 * collective when world > 1.  Errors: NBG_E_STATE (not writable), NBG_E_PART_NOT_FOUND.     */
int32_t nbg_snapshot_write_part(nbg_ctx* ctx, int32_t part, const uint8_t* key_bytes,
                                const uint64_t* key_offsets, const uint8_t* val_bytes,
                                const uint64_t* val_offsets, size_t n);
int32_t nbg_snapshot_commit(nbg_ctx* ctx);

typedef struct {
  int64_t num_vertices;     /* global vertex count (vertices appearing in any edge)          */
  int64_t local_vertices;   /* vertices owned by this rank                                    */
  int64_t local_out_edges;  /* out-edges (after version / multi-edge collapse) on this rank   */
  int64_t local_in_edges;
  int64_t device_bytes;     /* HBM held by the snapshot on this rank                          */
  double build_seconds;
  int64_t commits;          /* commits applied since finalize                                 */
  int64_t merge_commits;    /* of them, merged into the committed order (no full rebuild)     */
} nbg_snapshot_info;
int32_t nbg_snapshot_info_get(nbg_ctx* ctx, int32_t edge_type, nbg_snapshot_info* out);
/* CSR export for tests: out-degree of vid (-1 if unknown) */
int64_t nbg_snapshot_out_degree(nbg_ctx* ctx, int32_t edge_type, int64_t vid);

/* ---- result rows ------------------------------------------------------------------------
 * Column-major, typed.  col_types: NBG_T_VID (int64; every integer of a GO result is a VID,
 * GoExecutor.cpp:596-600), NBG_T_INT (int64, storage rows), NBG_T_DOUBLE, NBG_T_BOOL (1 byte),
 * NBG_T_STRING (int64 offsets n+1 + bytes).  Memory is owned by the engine until
 * nbg_rows_free.  `on_device` = 1: column pointers are device pointers.                    */
typedef struct {
  int64_t n_rows;
  int32_t n_cols;
  int32_t on_device;
  int32_t* col_types;
  void** cols;            /* per column: int64_t* / double* / uint8_t* / uint8_t* bytes    */
  int64_t** str_offsets;  /* per column: n_rows+1 offsets for STRING columns, else NULL     */
  int64_t* row_vertex;    /* get_bound: vid of the vertex a row belongs to (else NULL)      */
  /* get_bound response parts (QueryResponse, storage.thrift:207-228) */
  int64_t n_vertices;     /* vertices returned (only those with >= 1 edge row, QBP.cpp:61-67) */
  int64_t* vertex_ids;
  int64_t* vertex_row_offsets; /* n_vertices+1 */
  int32_t n_failed;       /* ResultCode list (BaseProcessor.h:64-71) */
  int32_t* failed_parts;
  int32_t* failed_codes;
  uint64_t edges_scanned; /* adjacency entries read (TEPS numerator)            */
  /* nbg_shortest_path: path of row i = path_vids[path_offsets[i] .. path_offsets[i+1])
   * (empty when the pair is unreachable); host memory.  NULL for other calls.              */
  int64_t* path_offsets;  /* n_rows+1 */
  int64_t* path_vids;
  void* _impl;
  /* get_bound SOURCE/DEST tag props (VertexData.vertex_data, QueryBoundProcessor.cpp:19-31): one
   * value per vertex_ids entry and requested tag prop, in request order; host memory.  Types as
   * for the edge columns (STRING: vertex_str_offsets[c] has n_vertices+1 offsets).
   * vertex_col_present[c][i] = 0 when the vertex has no row of that tag in the request's part
   * (the reference then leaves the prop out of the vertex row).                              */
  int32_t n_vertex_cols;
  int32_t* vertex_col_types;
  void** vertex_cols;
  int64_t** vertex_str_offsets;
  uint8_t** vertex_col_present;
} nbg_rows;
void nbg_rows_free(nbg_rows* rows);

/* ---- getBound ------------------------------------------------------------------------------
 * Replaces QueryBoundProcessor::process(GetNeighborsRequest) for OUT_BOUND / IN_BOUND
 * (src/storage/QueryBaseProcessor.inl:462-505, QueryBoundProcessor.cpp:16-106).
 * parts/vids: the request's parts map flattened (pair i = (parts[i], vids[i])).
 * edge_type < 0: in-bound scan (StorageClient.cpp:118).  filter: Expression::encode bytes or
 * empty.  Return columns are EDGE-owned props (key props _src/_dst/_rank/_type or schema props)
 * and SOURCE/DEST tag props (tag_id + name; returned per vertex in vertex_cols; unknown tag ->
 * E_TAG_PROP_NOT_FOUND, unknown prop -> E_IMPROPER_DATA_TYPE on every part).  $^ tag props in
 * the push-down filter read the request part's vertex row ($$ -> E_INVALID_FILTER, as checkExp,
 * QueryBaseProcessor.inl:160-238).  Request-level errors are
 * reported per part in failed_codes (QueryBaseProcessor.inl:470-477), not as the return.    */
typedef struct {
  const char* name;
  int32_t owner;
  int32_t tag_id;
} nbg_prop_def;
int32_t nbg_get_bound(nbg_ctx* ctx, int32_t edge_type, const int32_t* parts,
                      const int64_t* vids, size_t n, const uint8_t* filter, size_t filter_len,
                      const nbg_prop_def* cols, size_t ncols, nbg_rows* out);

/* ---- outBoundStats / inBoundStats ---------------------------------------------------------
 * Replaces QueryStatsProcessor::process (src/storage/QueryStatsProcessor.cpp:16-125,
 * StorageServiceHandler.cpp:40-53): the getBound scan with the same filter push-down, reduced
 * on the device to one row.  stat_types[i] = cpp2::StatType of cols[i] (SUM 1, COUNT 2, AVG 3,
 * storage.thrift:51-55).  Columns in request order: SUM -> INT (int64 sum), COUNT -> INT,
 * AVG -> DOUBLE (sum / count, NaN without rows); in-bound requests skip edge props.  SUM / AVG
 * over BOOL / STRING fail every part with E_IMPROPER_DATA_TYPE (validOperation,
 * QueryBaseProcessor.inl:18-35); SUM / AVG over DOUBLE values return NBG_E_UNSUPPORTED (the
 * reference's int64-initialised sum throws boost::bad_get).  SOURCE / DEST tag props
 * (tag_id + name) reduce over the request entries of owned parts whose vertex row sits in the
 * entry's part (collectVertexProps, QueryBaseProcessor.inl:309-333; QueryStatsProcessor.cpp:
 * 69-82), duplicates counted per entry; unknown tag -> E_TAG_PROP_NOT_FOUND, unknown prop or
 * SUM / AVG over BOOL / STRING -> E_IMPROPER_DATA_TYPE on every part.                        */
int32_t nbg_bound_stats(nbg_ctx* ctx, int32_t edge_type, const int32_t* parts, const int64_t* vids,
                        size_t n, const uint8_t* filter, size_t filter_len, const nbg_prop_def* cols,
                        const int32_t* stat_types, size_t ncols, nbg_rows* out);

/* ---- GO N STEPS ---------------------------------------------------------------------------
 * Replaces GoExecutor's stepOut -> getNeighbors -> onStepOutResponse -> getDstIdsFromResp loop
 * and its final processFinalResult / setupInterimResult (src/graph/GoExecutor.cpp:80-106,
 * 334-431, 585-782) with one device-resident call.  starts: literal or piped vids (duplicates
 * kept unless distinct, GoExecutor.cpp:98-104).  where/yields: Expression::encode bytes as the
 * graphd AST would encode them.  n_yields = 0 means the default YIELD e._dst AS id.
 * With world_size > 1 every rank passes the same spec; rows come back sharded by owner.     */
typedef struct {
  int32_t edge_type;
  int32_t steps;
  const int64_t* starts;
  size_t n_starts;
  const uint8_t* where;
  size_t where_len;
  const uint8_t* const* yields;
  const size_t* yield_lens;
  size_t n_yields;
  int32_t distinct;
  int32_t keep_on_device; /* 1: leave result columns in HBM (bench / chained queries)        */
  /* $-.prop / $var.prop (GoExecutor::getPropFromInterim, GoExecutor.cpp:831-838): the piped or
   * variable input rows, one per starts[i] (the FROM column).  A start vid's props come from its
   * LAST row (InterimResult::buildIndex, InterimResult.cpp:146-160).  Column types NBG_T_VID /
   * NBG_T_INT / NBG_T_DOUBLE (int64 / double arrays), NBG_T_BOOL (uint8) or NBG_T_STRING (bytes
   * + n_starts+1 int64 offsets).  With steps > 1 the final step reads the input row of each
   * dst's root start, as graphd's VertexBackTracker (GoExecutor.h:174-193) does; a dst reached
   * from several starts takes the smallest root vid among its in-edge srcs (the reference's
   * answer there depends on RPC response order; DESIGN.md divergence 6).
   * n_inputs = 0: no input table (zero-initialised specs stay valid).                        */
  size_t n_inputs;
  const char* const* input_names;
  const int32_t* input_types;
  const void* const* input_cols;
  const int64_t* const* input_str_offsets;
} nbg_go_spec;
int32_t nbg_go(nbg_ctx* ctx, const nbg_go_spec* spec, nbg_rows* out);

/* ---- FIND SHORTEST PATH (no reference implementation: FindExecutor.cpp:20-22) ------------
 * Definition (owned by this build): the unweighted hop distance from src to
 * dst over edge_type out-edges, -1 when dst is not reached within max_steps hops; the path is
 * the lexicographically smallest vid sequence among the shortest paths.  Distances toward dst
 * follow the -edge_type in-edge keys (P5: INSERT EDGE writes both), so parity with the oracle
 * assumes the in-edge keys mirror the out-edge keys, as the write path guarantees.
 * Runs as batched bidirectional BFS (pairs in batches, option "sp_batch").
 * out: 3 VID columns [src, dst, hops] per pair, in input order; paths in path_offsets /
 * path_vids (src ... dst, hops+1 vids).  src == dst gives hops 0 and the path [src].        */
int32_t nbg_shortest_path(nbg_ctx* ctx, int32_t edge_type, const int64_t* src,
                          const int64_t* dst, size_t npairs, int32_t max_steps, nbg_rows* out);

/* ---- timing of the last call (HIP events on the engine stream) --------------------------- */
/* one hop of the last nbg_go: mode 0 = top-down expansion of a frontier list, 1 = bottom-up
 * over the transposed CSR.  c[]: top-down {frontier, entries, next frontier, 0, 0, 0};
 * bottom-up {found, next-hop out-degree sum, slab words read, rows scanned past the slab,
 * entries read past the slab, predicate values read past the slab, first-pass frontier probes
 * answered by L2, first-pass probes answered from the LDS hub copy}.
 * nbg_shortest_path records one entry per launch instead: mode 2 = BFS expansion, 3 = meet
 * probe, 4 = sweep; c[] = {tuples, adjacency entries, claims, meets so far, iteration,
 * active pairs, 0, 0}; 5 = walk scan (device-driven batches), c[] = {chunks, adjacency
 * entries, 0, meets, walk step, 0, 0, 0}.                                                   */
typedef struct {
  int32_t mode;
  int32_t final_hop;
  double ms;         /* HIP-event time of the hop's expansion kernels                      */
  uint64_t bytes;    /* their algorithmic bytes                       */
  uint64_t c[8];
  double kernel_ms;      /* the hop's dominant kernel alone (first pass of a bottom-up hop)  */
  uint64_t kernel_bytes; /* that kernel's algorithmic bytes                                  */
  char kernels[160];     /* rocprof names of the hop's kernels, dominant first, "; "-separated
                            (empty: a top-down hop, nbg::k_expand)                          */
} nbg_hop_stat;
#define NBG_MAX_HOP_STATS 16
typedef struct {
  double total_ms;        /* device time of the last nbg_go / nbg_get_bound (events around the
                             whole call; 0 for nbg_go with option hop_timing = 0, which records
                             no event at all)                                                  */
  double expand_ms;       /* summed time of the expansion kernels                            */
  int64_t expand_launches;
  uint64_t edges_scanned;
  uint64_t expand_bytes;  /* algorithmic bytes of the expansion kernels          */
  int32_t steps_run;
  int32_t bu_steps;       /* steps that ran bottom-up over the transposed CSR               */
  double comm_ms;         /* time in frontier exchanges / reductions between ranks          */
  uint64_t comm_bytes;    /* bytes this rank sent to other ranks                            */
  int32_t n_hops;         /* entries of hops[] filled (nbg_go, nbg_shortest_path)            */
  nbg_hop_stat hops[NBG_MAX_HOP_STATS];
  int32_t host_waits;     /* times the engine waited on the host for the device in the last
                             call (counter fetches, stream synchronisations; waits inside the
                             LocalComm / RCCL transport not included)                          */
  int32_t spec_hops;      /* nbg_go: hops that ran speculatively behind a device gate;
                             nbg_shortest_path: batches that ran device-driven (the others ran
                             host-driven: option sp_dev = 0, or a list overflow re-ran them)   */
  int32_t launches;       /* nbg_shortest_path: kernel launches of its device-driven batches
                             (ABI 5; 0 for other calls)                                         */
  int32_t comm_calls;     /* collectives this rank issued through its communicator in the last
                             call (ABI 6; comm_ms / comm_calls = the mean time of one on the
                             engine stream, enqueue to completion)                              */
} nbg_timing;
int32_t nbg_last_timing(nbg_ctx* ctx, nbg_timing* out);
/* engine option key = value (tuning knobs); value INT64_MIN removes the key, so the
 * engine default applies again                                                              */
int32_t nbg_set_option(nbg_ctx* ctx, const char* key, int64_t value);

#ifdef __cplusplus
}
#endif
#endif /* NEBULA_AMD_H_ */
