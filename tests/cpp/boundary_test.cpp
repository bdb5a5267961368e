// boundary_test.cpp -- TEST PROGRAM: a compiled C++ caller of the drop-in boundary.
//
// Includes include/nebula_amd.h, links libnebula_amd.so and runs the reference's
// QueryBoundTest OutBoundSimpleTest request (src/storage/test/QueryBoundTest.cpp:181-201:
// mockData, buildRequest, process, checkResponse) through nbg_get_bound exactly in the shape
// INTEGRATION.md section 3 gives GpuBoundProcessor::process (QueryBaseProcessor.h:47): the
// request's parts map flattened to (part, vid) pairs, the return columns as nbg_prop_def,
// per-part result codes from failed_parts / failed_codes, rows grouped per vertex by
// vertex_row_offsets.  The KV bytes of mockData come from a fixture file written by
// tests/test_capi_boundary.py (keys + RowWriter values, the oracle's encoders).
//
//   boundary_test --sizes            struct layout vs the library (no GPU needed)
//   boundary_test <fixture.bin>      the OutBoundSimpleTest request on device 0
//
// Exit status 0 and a last line "OK" on success.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/nebula_amd.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "CHECK failed (%s:%d): ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      g_fail++;                                            \
    }                                                      \
  } while (0)

static int check_sizes() {
  CHECK(nbg_abi_version() == NBG_ABI_VERSION, "ABI %d vs header %d", nbg_abi_version(), NBG_ABI_VERSION);
  const int64_t want[6] = {int64_t(sizeof(nbg_timing)),   int64_t(sizeof(nbg_hop_stat)), int64_t(sizeof(nbg_snapshot_info)),
                           int64_t(sizeof(nbg_go_spec)),  int64_t(sizeof(nbg_rows)),     int64_t(sizeof(nbg_prop_def))};
  for (int i = 0; i < 6; i++)
    CHECK(nbg_struct_size(i) == want[i], "struct %d: library %lld, header %lld", i, (long long)nbg_struct_size(i),
          (long long)want[i]);
  CHECK(nbg_struct_size(6) == -1, "unknown struct index");
  // pure helpers: StorageClient.cpp:238-243, CreateSpaceProcessor.cpp:77-90
  CHECK(nbg_part_of(7, 6) == 2, "part_of");
  CHECK(nbg_part_of(-1, 6) == int32_t(uint64_t(-1) % 6 + 1), "part_of negative vid");
  CHECK(nbg_rank_of_part(5, 4) == 1, "rank_of_part");
  return g_fail;
}

// ---- fixture file ---------------------------------------------------------------------------
struct Reader {
  std::vector<uint8_t> b;
  size_t p = 0;
  bool ok = true;
  template <typename T>
  T get() {
    T v{};
    if (p + sizeof(T) > b.size()) {
      ok = false;
      return v;
    }
    memcpy(&v, b.data() + p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    const uint32_t n = get<uint32_t>();
    if (p + n > b.size()) {
      ok = false;
      return "";
    }
    std::string s(reinterpret_cast<const char*>(b.data() + p), n);
    p += n;
    return s;
  }
  template <typename T>
  std::vector<T> vec(size_t n) {
    std::vector<T> v(n);
    if (p + n * sizeof(T) > b.size()) {
      ok = false;
      return v;
    }
    memcpy(v.data(), b.data() + p, n * sizeof(T));
    p += n * sizeof(T);
    return v;
  }
};

struct Schema {
  std::vector<std::string> names;
  std::vector<int32_t> types;
  void read(Reader& r) {
    const uint32_t n = r.get<uint32_t>();
    for (uint32_t i = 0; i < n; i++) {
      names.push_back(r.str());
      types.push_back(r.get<int32_t>());
    }
  }
  std::vector<const char*> cnames() const {
    std::vector<const char*> v;
    for (auto& s : names) v.push_back(s.c_str());
    return v;
  }
};

// ---- GpuBoundProcessor::process as INTEGRATION.md section 3 writes it -------------------------
struct PropDef {  // cpp2::PropDef (storage.thrift)
  std::string name;
  int32_t owner, tag_id;
};
struct GetNeighborsRequest {  // cpp2::GetNeighborsRequest (storage.thrift:57-63)
  int32_t space_id = 0;
  std::map<int32_t, std::vector<int64_t>> parts;
  int32_t edge_type = 0;
  std::string filter;
  std::vector<PropDef> return_columns;
};
struct VertexRows {
  int64_t vid;
  std::vector<std::vector<std::string>> rows;  // each value rendered as text
  std::vector<std::string> tag_values;
};
struct QueryResponse {
  std::map<int32_t, int32_t> failed;  // part -> ErrorCode
  std::vector<VertexRows> vertices;
  int32_t engine_rc = NBG_OK;
};

static std::string render(int32_t type, const void* col, const int64_t* soff, int64_t i) {
  char buf[64];
  switch (type) {
    case NBG_T_BOOL: return static_cast<const uint8_t*>(col)[i] ? "true" : "false";
    case NBG_T_DOUBLE: snprintf(buf, sizeof buf, "%.17g", static_cast<const double*>(col)[i]); return buf;
    case NBG_T_STRING: {
      const char* bytes = static_cast<const char*>(col);
      return std::string(bytes + soff[i], size_t(soff[i + 1] - soff[i]));
    }
    default: snprintf(buf, sizeof buf, "%lld", (long long)static_cast<const int64_t*>(col)[i]); return buf;
  }
}

static QueryResponse process(nbg_ctx* ctx, const GetNeighborsRequest& req) {
  QueryResponse resp;
  std::vector<int32_t> parts;
  std::vector<int64_t> vids;
  for (auto& kv : req.parts)
    for (auto v : kv.second) {
      parts.push_back(kv.first);
      vids.push_back(v);
    }
  std::vector<nbg_prop_def> cols;
  for (auto& pd : req.return_columns) cols.push_back({pd.name.c_str(), pd.owner, pd.tag_id});
  nbg_rows rows;
  memset(&rows, 0, sizeof rows);
  const int32_t rc = nbg_get_bound(ctx, req.edge_type, parts.data(), vids.data(), vids.size(),
                                   reinterpret_cast<const uint8_t*>(req.filter.data()), req.filter.size(), cols.data(),
                                   cols.size(), &rows);
  resp.engine_rc = rc;
  if (rc != NBG_OK) {
    for (auto& kv : req.parts) resp.failed[kv.first] = NBG_E_UNKNOWN;
    return resp;
  }
  for (int32_t i = 0; i < rows.n_failed; i++) resp.failed[rows.failed_parts[i]] = rows.failed_codes[i];
  // encodeVertices: per vertex, rows [vertex_row_offsets[i], vertex_row_offsets[i + 1])
  for (int64_t v = 0; v < rows.n_vertices; v++) {
    VertexRows vr;
    vr.vid = rows.vertex_ids[v];
    for (int64_t r = rows.vertex_row_offsets[v]; r < rows.vertex_row_offsets[v + 1]; r++) {
      std::vector<std::string> row;
      for (int32_t c = 0; c < rows.n_cols; c++) row.push_back(render(rows.col_types[c], rows.cols[c], rows.str_offsets[c], r));
      vr.rows.push_back(row);
    }
    for (int32_t c = 0; c < rows.n_vertex_cols; c++)
      vr.tag_values.push_back(rows.vertex_col_present[c][v]
                                  ? render(rows.vertex_col_types[c], rows.vertex_cols[c], rows.vertex_str_offsets
                                                                                          ? rows.vertex_str_offsets[c]
                                                                                          : nullptr, v)
                                  : "<none>");
    resp.vertices.push_back(vr);
  }
  nbg_rows_free(&rows);
  return resp;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s --sizes | <fixture.bin>\n", argv[0]);
    return 2;
  }
  if (check_sizes()) return 1;
  if (!strcmp(argv[1], "--sizes")) {
    printf("OK\n");
    return 0;
  }
  Reader rd;
  {
    FILE* f = fopen(argv[1], "rb");
    if (!f) {
      perror(argv[1]);
      return 2;
    }
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) rd.b.insert(rd.b.end(), buf, buf + n);
    fclose(f);
  }
  CHECK(rd.str() == "NBGFIX1", "fixture magic");
  const int32_t num_parts = rd.get<int32_t>();
  const int32_t edge_type = rd.get<int32_t>();
  Schema es;
  es.read(rd);
  const uint32_t ntags = rd.get<uint32_t>();
  nbg_ctx* ctx = nbg_ctx_create(0, num_parts, 0, 1);
  if (!ctx) {
    fprintf(stderr, "nbg_ctx_create failed (no MI355X visible)\n");
    return 3;
  }
  auto must = [&](int32_t rc, const char* what) {
    if (rc != NBG_OK) {
      fprintf(stderr, "%s: %d %s\n", what, rc, nbg_last_error(ctx));
      g_fail++;
    }
  };
  {
    auto nm = es.cnames();
    must(nbg_schema_set_edge(ctx, edge_type, 0, int32_t(nm.size()), nm.data(), es.types.data()), "schema_set_edge");
  }
  for (uint32_t t = 0; t < ntags; t++) {
    const int32_t id = rd.get<int32_t>();
    const std::string name = rd.str();
    Schema ts;
    ts.read(rd);
    auto nm = ts.cnames();
    must(nbg_schema_set_tag(ctx, id, name.c_str(), 0, int32_t(nm.size()), nm.data(), ts.types.data()), "schema_set_tag");
  }
  const uint32_t nparts = rd.get<uint32_t>();
  for (uint32_t i = 0; i < nparts && rd.ok; i++) {
    const int32_t part = rd.get<int32_t>();
    const uint64_t n = rd.get<uint64_t>();
    const auto kb = rd.vec<uint8_t>(rd.get<uint64_t>());
    const auto koff = rd.vec<uint64_t>(n + 1);
    const auto vb = rd.vec<uint8_t>(rd.get<uint64_t>());
    const auto voff = rd.vec<uint64_t>(n + 1);
    if (rd.ok) must(nbg_snapshot_load_part(ctx, part, kb.data(), koff.data(), vb.data(), voff.data(), n), "load_part");
  }
  CHECK(rd.ok, "fixture truncated");
  must(nbg_snapshot_finalize(ctx), "finalize");

  // buildRequest (QueryBoundTest.cpp:82-109)
  GetNeighborsRequest req;
  req.space_id = 0;
  for (int32_t part = 0; part < 3; part++)
    for (int64_t vid = part * 10; vid < (part + 1) * 10; vid++) req.parts[part].push_back(vid);
  req.edge_type = edge_type;
  for (int i = 0; i < 3; i++) {
    const int32_t tag = 3001 + i * 2;
    req.return_columns.push_back({"tag_" + std::to_string(tag) + "_col_" + std::to_string(i * 2), NBG_OWNER_SOURCE, tag});
  }
  req.return_columns.push_back({"_dst", NBG_OWNER_EDGE, 0});
  req.return_columns.push_back({"_rank", NBG_OWNER_EDGE, 0});
  for (int i = 0; i < 10; i++) req.return_columns.push_back({"col_" + std::to_string(i * 2), NBG_OWNER_EDGE, 0});

  const QueryResponse resp = process(ctx, req);
  // checkResponse (QueryBoundTest.cpp:111-178)
  CHECK(resp.engine_rc == NBG_OK, "nbg_get_bound returned %d: %s", resp.engine_rc, nbg_last_error(ctx));
  CHECK(resp.failed.empty(), "failed parts: %zu", resp.failed.size());
  CHECK(resp.vertices.size() == 30, "vertices %zu != 30", resp.vertices.size());
  for (const auto& vr : resp.vertices) {
    CHECK(vr.tag_values.size() == 3, "vertex %lld: %zu tag props", (long long)vr.vid, vr.tag_values.size());
    if (vr.tag_values.size() == 3) {
      CHECK(vr.tag_values[0] == std::to_string(vr.vid + 3001), "vertex %lld tag col 0: %s", (long long)vr.vid,
            vr.tag_values[0].c_str());
      CHECK(vr.tag_values[1] == std::to_string(vr.vid + 3003 + 2), "vertex %lld tag col 1: %s", (long long)vr.vid,
            vr.tag_values[1].c_str());
      CHECK(vr.tag_values[2] == "tag_string_col_4", "vertex %lld tag col 2: %s", (long long)vr.vid,
            vr.tag_values[2].c_str());
    }
    CHECK(vr.rows.size() == 7, "vertex %lld: %zu rows != 7", (long long)vr.vid, vr.rows.size());
    int64_t dst = 10001;
    for (const auto& row : vr.rows) {
      CHECK(row.size() == 12, "row width %zu", row.size());
      if (row.size() != 12) break;
      CHECK(row[0] == std::to_string(dst), "vertex %lld: _dst %s != %lld", (long long)vr.vid, row[0].c_str(),
            (long long)dst);
      CHECK(row[1] == "0", "_rank %s", row[1].c_str());
      for (int i = 0; i < 5; i++)  // col_{2i}: the newest version's dst + 2i (ver 0 is the latest write)
        CHECK(row[2 + i] == std::to_string(dst + 2 * i), "vertex %lld dst %lld col_%d: %s", (long long)vr.vid,
              (long long)dst, 2 * i, row[2 + i].c_str());
      for (int i = 0; i < 5; i++)
        CHECK(row[7 + i] == "string_col_" + std::to_string((i + 5) * 2) + "_2", "col_%d: %s", (i + 5) * 2,
              row[7 + i].c_str());
      dst++;
    }
  }
  nbg_ctx_destroy(ctx);
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  printf("OutBoundSimpleTest: 30 vertices x 7 rows, 3 tag props each\nOK\n");
  return 0;
}
