// oracle/refcpu.h -- TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement of the reference (Nebula Graph v1.0.0-beta) neighbour-expansion
// path, used as the parity checker and as the CPU baseline.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
// product (nebula_amd/) never links or calls anything in this directory.
//
// Pinning: the restatement is checked against the reference's own known-answer
// tests (QueryBoundTest fixture/expectations, RowReader/RowWriter byte layouts,
// ExpressionTest literals, the NBA GoTest expectations) by tests/test_oracle_*.py.
// The reference itself cannot be compiled here (folly/fbthrift/rocksdb/boost are
// absent), so there is no oracle/_ref build; see DESIGN.md "Oracle".
#pragma once
#include <cstddef>
#include <cstdint>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_store ora_store;   // per-space KV store + schemas (+ graphd config)
typedef struct ora_result ora_result; // decoded result (rows / responses / paths)

// ---- store ---------------------------------------------------------------------------------
ora_store* ora_store_new(int32_t num_parts);
void ora_store_free(ora_store* st);
// One WriteBatch for one part: keys/vals are concatenated blobs with n+1 offsets.
// Identical keys inside and across batches: last write wins (RocksEngine.cpp:216-230).
void ora_store_put_batch(ora_store* st, int32_t part, const uint8_t* kbytes, const uint64_t* koff,
                         const uint8_t* vbytes, const uint64_t* voff, size_t n);
void ora_store_finalize(ora_store* st);  // sort each part bytewise (RocksEngine prefix order)
size_t ora_store_num_keys(const ora_store* st);
// dump one part's sorted KV (after finalize): sizes first, then the blobs (n+1 offsets)
size_t ora_store_part_size(const ora_store* st, int32_t part, size_t* kbytes, size_t* vbytes);
void ora_store_dump_part(const ora_store* st, int32_t part, uint8_t* kb, uint64_t* koff,
                         uint8_t* vb, uint64_t* voff);
// schema registry (meta SchemaManager stand-in).  types = cpp2::SupportedType values.
void ora_schema_set_edge(ora_store* st, int32_t edge_type, int32_t ver, int32_t nfields,
                         const char* const* names, const int32_t* types);
void ora_schema_set_tag(ora_store* st, int32_t tag_id, const char* tag_name, int32_t ver,
                        int32_t nfields, const char* const* names, const int32_t* types);
void ora_schema_set_edge_name(ora_store* st, int32_t edge_type, const char* name);

// ---- codec helpers (dataman restatement), exposed for the byte-level tests ----------------
// schemaless RowWriter: vals typed by tags (2=INT,5=DOUBLE,1=BOOL,6=STRING)
size_t ora_encode_row(const int32_t* tags, const int64_t* ivals, const double* dvals,
                      const char* const* svals, int32_t ncols, uint8_t* out, size_t cap);
size_t ora_encode_varint(uint64_t v, uint8_t* out);
size_t ora_edge_key(int32_t part, int64_t src, int32_t type, int64_t rank, int64_t dst,
                    int64_t ver, uint8_t* out);

// ---- synthetic RMAT graph (same definition as the product generator) -----------
void ora_rmat_edges(int32_t scale, int32_t edge_factor, uint64_t seed, int64_t* src_vid,
                    int64_t* dst_vid, int64_t* weight);
int64_t ora_rmat_vid(uint64_t idx, uint64_t seed);
// writes out-edges (type, weight row) and in-edges (-type, empty) into the store
void ora_rmat_load(ora_store* st, int32_t scale, int32_t edge_factor, uint64_t seed,
                   int32_t edge_type, int32_t versions, int32_t threads);

// ---- storage processor (QueryBoundProcessor restatement) -----------------------------------
typedef struct {
  const char* name;
  int32_t owner;   // cpp2::PropOwner SOURCE=1 DEST=2 EDGE=3
  int32_t tag_id;
} ora_prop_def;
ora_result* ora_get_bound(ora_store* st, int32_t edge_type, int32_t in_bound,
                          const int32_t* parts, const int64_t* vids, size_t n,
                          const uint8_t* filter, size_t filter_len,
                          const ora_prop_def* cols, size_t ncols,
                          int32_t max_handlers, int32_t min_per_bucket);
// QueryStatsProcessor restatement (outBoundStats / inBoundStats, QueryStatsProcessor.cpp:16-125):
// stat_types[i] = cpp2::StatType (SUM 1, COUNT 2, AVG 3) of cols[i].  One result row.
ora_result* ora_bound_stats(ora_store* st, int32_t edge_type, int32_t in_bound,
                            const int32_t* parts, const int64_t* vids, size_t n,
                            const uint8_t* filter, size_t filter_len,
                            const ora_prop_def* cols, const int32_t* stat_types, size_t ncols,
                            int32_t max_handlers, int32_t min_per_bucket);
// GenBuckets restatement (QueryBaseProcessor.inl:425-460): writes bucket sizes, returns count.
int32_t ora_gen_buckets(const int32_t* parts, const int64_t* vids, size_t n,
                        int32_t max_handlers, int32_t min_per_bucket, int32_t* sizes_out);

// ---- graphd GO (GoExecutor + StorageClient restatement) ------------------------------------
/* $- / $var input rows for the NEXT ora_go call only (one row per start; types 3 VID, 2 INT,
 * 5 DOUBLE, 1 BOOL as int64 / double / uint8 arrays, 6 STRING as bytes + n+1 offsets) */
void ora_go_set_inputs(ora_store* st, size_t n_rows, size_t n_cols, const char* const* names,
                       const int32_t* types, const void* const* cols, const int64_t* const* str_offsets);
ora_result* ora_go(ora_store* st, const int64_t* starts, size_t n_starts, int32_t steps,
                   int32_t edge_type, const uint8_t* where, size_t where_len,
                   const uint8_t* const* yields, const size_t* yield_lens, size_t n_yields,
                   int32_t distinct, int32_t num_hosts, int32_t max_handlers,
                   int32_t min_per_bucket, uint64_t* edges_scanned);

// ---- FIND SHORTEST PATH (A10; definition owned by this build) ------------------
ora_result* ora_shortest_path(ora_store* st, const int64_t* src, const int64_t* dst,
                              size_t npairs, int32_t edge_type, int32_t max_steps);

// ---- index-space restatement of GO / FIND SHORTEST PATH on the synthetic RMAT graph -----
// (oracle/rmat_graph.cpp): for parity at the configured sizes, where the KV store above does
// not fit.  Checked against the KV-store restatement at small scales (tests).
typedef struct ora_rmat_graph ora_rmat_graph;
ora_rmat_graph* ora_rmat_graph_new(int32_t scale, int32_t edge_factor, uint64_t seed, int32_t threads);
void ora_rmat_graph_free(ora_rmat_graph* g);
void ora_rmat_graph_info(const ora_rmat_graph* g, int64_t* n_vertices, int64_t* n_edges);
int64_t ora_rmat_graph_out_degree(const ora_rmat_graph* g, int64_t idx);
// GO steps [WHERE weight > where_gt] YIELD _dst [DISTINCT]: sorted result vids in *out
int64_t ora_rmat_graph_go(const ora_rmat_graph* g, const int64_t* starts, size_t n_starts, int32_t steps,
                          int32_t has_where, int64_t where_gt, int32_t distinct, int32_t threads,
                          int64_t** out, uint64_t* edges_scanned);
void ora_rmat_graph_shortest_path(ora_rmat_graph* g, const int64_t* src, const int64_t* dst, size_t n,
                                  int32_t max_steps, int32_t threads, int64_t* hops, int64_t* path_off,
                                  int64_t** path_vids);
void ora_free(void* p);

// ---- results --------------------------------------------------------------------------------
int32_t ora_res_code(const ora_result* r);          // 0 ok, else error code
const char* ora_res_error(const ora_result* r);
size_t ora_res_nrows(const ora_result* r);
int32_t ora_res_ncols(const ora_result* r);
// cell accessors: type 0=int64 1=double 2=bool 3=string, -1 = absent
int32_t ora_res_type(const ora_result* r, size_t row, int32_t col);
int64_t ora_res_int(const ora_result* r, size_t row, int32_t col);
double ora_res_double(const ora_result* r, size_t row, int32_t col);
const char* ora_res_str(const ora_result* r, size_t row, int32_t col, size_t* len);
// bulk int64 column extraction (rows x col), cells of other type become INT64_MIN
void ora_res_int_col(const ora_result* r, int32_t col, int64_t* out);
// get_bound extras: failed parts, per-row owning vertex, vertex tag cols
size_t ora_res_nfailed(const ora_result* r);
void ora_res_failed(const ora_result* r, size_t i, int32_t* part, int32_t* code);
int64_t ora_res_row_vertex(const ora_result* r, size_t row);
size_t ora_res_nvertices(const ora_result* r);
int64_t ora_res_vertex_id(const ora_result* r, size_t i);
size_t ora_res_vertex_nrows(const ora_result* r, size_t i);
int32_t ora_res_vertex_ncols(const ora_result* r);
int32_t ora_res_vertex_type(const ora_result* r, size_t i, int32_t col);
int64_t ora_res_vertex_int(const ora_result* r, size_t i, int32_t col);
const char* ora_res_vertex_str(const ora_result* r, size_t i, int32_t col, size_t* len);
const char* ora_res_vertex_bytes(const ora_result* r, size_t i, size_t* len);  // vertex_data
const char* ora_res_edge_bytes(const ora_result* r, size_t i, size_t* len);    // edge_data
int32_t ora_res_schema_ncols(const ora_result* r, int32_t which);  // 0 = edge, 1 = vertex
const char* ora_res_schema_name(const ora_result* r, int32_t which, int32_t col);
int32_t ora_res_schema_type(const ora_result* r, int32_t which, int32_t col);
void ora_res_free(ora_result* r);

#ifdef __cplusplus
}
#endif
