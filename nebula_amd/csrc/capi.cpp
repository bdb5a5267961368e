// capi.cpp -- extern "C" entry points declared in include/nebula_amd.h.
#include <unistd.h>
#include <map>
#include <mutex>
#include <algorithm>
#include <cstring>

#include "engine.h"

namespace nbg {
thread_local std::shared_ptr<BufPool> tl_pool;
AllocClock g_alloc_clock;
namespace {
std::mutex g_pools_mu;
std::vector<BufPool*> g_pools;
}  // namespace
void pool_register(BufPool* p, bool add) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  if (add) g_pools.push_back(p);
  else g_pools.erase(std::remove(g_pools.begin(), g_pools.end(), p), g_pools.end());
}
size_t pool_trim_all() {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  size_t freed = 0;
  for (BufPool* p : g_pools) freed += p->trim();
  return freed;
}
int32_t comm_unique_id(uint8_t out[128]);
void comm_init(Ctx& c, const uint8_t id[128]);
void free_rows_impl(void* impl);
}  // namespace nbg

using nbg::Ctx;
using nbg::Error;

struct nbg_ctx {
  Ctx c;
};

template <typename F>
static int32_t guarded(nbg_ctx* ctx, F f) {
  if (!ctx) return NBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lg(ctx->c.mu);
  try {
    (void)hipSetDevice(ctx->c.device);
    int32_t rc = f(ctx->c);
    if (rc == NBG_OK) ctx->c.last_error.clear();
    return rc;
  } catch (const Error& e) {
    ctx->c.last_error = e.what();
    return e.code;
  } catch (const std::exception& e) {
    ctx->c.last_error = e.what();
    return NBG_E_UNKNOWN;
  }
}

namespace nbg {
static std::mutex g_dev_mu;
static std::map<int, int> g_dev_ctx;
int ctx_count_on_device(int device) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto it = g_dev_ctx.find(device);
  return it == g_dev_ctx.end() ? 0 : it->second;
}
size_t host_ram_bytes() {
  const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
  return pages > 0 && psz > 0 ? size_t(pages) * size_t(psz) : 0;
}
static void ctx_count_add(int device, int d) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  g_dev_ctx[device] += d;
}
}  // namespace nbg

extern "C" {


nbg_ctx* nbg_ctx_create(int32_t device, int32_t num_parts, int32_t rank, int32_t world_size) {
  if (num_parts <= 0 || world_size <= 0 || rank < 0 || rank >= world_size) return nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  auto* ctx = new nbg_ctx();
  ctx->c.device = device;
  ctx->c.num_parts = num_parts;
  ctx->c.rank = rank;
  ctx->c.world = world_size;
  ctx->c.sharded = world_size > 1;
  if (hipStreamCreateWithFlags(&ctx->c.stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return nullptr;
  }
  for (auto& e : ctx->c.ev) (void)hipEventCreate(&e);
  // coherent: the device publishes counters here and the host polls them (k_publish)
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->c.host_counters), 256 * 8 + 64, hipHostMallocCoherent) != hipSuccess) {
    (void)hipStreamDestroy(ctx->c.stream);
    delete ctx;
    return nullptr;
  }
  memset(ctx->c.host_counters, 0, 256 * 8 + 64);
  ctx->c.host_seq = ctx->c.host_counters + 256;
  // pinned staging for a query's small host->device inputs (starts, compiled programs): copies
  // from pageable memory go through a driver bounce buffer and block the calling thread
  if (hipHostMalloc(&ctx->c.host_stage, nbg::kHostStageBytes, hipHostMallocDefault) != hipSuccess)
    ctx->c.host_stage = nullptr;
  // coherent: k_starts_small reads a GO's small start set straight from here
  if (hipHostMalloc(reinterpret_cast<void**>(&ctx->c.starts_host), 4096 * 8, hipHostMallocCoherent) != hipSuccess)
    ctx->c.starts_host = nullptr;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess) ctx->c.hbm_total = tot;
  nbg::ctx_count_add(device, 1);
  return ctx;
}

void nbg_ctx_destroy(nbg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->c.device);
  nbg::ctx_count_add(ctx->c.device, -1);
  (void)hipStreamSynchronize(ctx->c.stream);
  nbg::comm_destroy(ctx->c);
  ctx->c.host_pool->trim();  // results still held return their blocks to the (then ownerless) pool
  for (auto& e : ctx->c.ev) (void)hipEventDestroy(e);
  for (auto& e : ctx->c.tev) (void)hipEventDestroy(e);
  if (ctx->c.host_counters) (void)hipHostFree(ctx->c.host_counters);
  if (ctx->c.host_stage) (void)hipHostFree(ctx->c.host_stage);
  if (ctx->c.sp_host) (void)hipHostFree(ctx->c.sp_host);
  if (ctx->c.starts_host) (void)hipHostFree(ctx->c.starts_host);
  (void)hipStreamDestroy(ctx->c.stream);
  delete ctx;
}

const char* nbg_last_error(const nbg_ctx* ctx) { return ctx ? ctx->c.last_error.c_str() : "null context"; }

int32_t nbg_comm_unique_id(uint8_t out[128]) { return nbg::comm_unique_id(out); }

int32_t nbg_comm_init(nbg_ctx* ctx, const uint8_t unique_id[128]) {
  return guarded(ctx, [&](Ctx& c) {
    nbg::comm_init(c, unique_id);
    return NBG_OK;
  });
}

int32_t nbg_comm_init_local(nbg_ctx* ctx, int64_t group_key) {
  return guarded(ctx, [&](Ctx& c) {
    nbg::comm_init_local(c, group_key);
    return NBG_OK;
  });
}

int32_t nbg_comm_info(nbg_ctx* ctx, int32_t* ranks, int32_t* transport) {
  if (!ranks || !transport) return NBG_E_INVALID_ARG;
  return guarded(ctx, [&](Ctx& c) {
    nbg::comm_info(c, ranks, transport);
    return NBG_OK;
  });
}

int32_t nbg_abi_version(void) { return NBG_ABI_VERSION; }
int64_t nbg_struct_size(int32_t which) {
  switch (which) {
    case 0: return int64_t(sizeof(nbg_timing));
    case 1: return int64_t(sizeof(nbg_hop_stat));
    case 2: return int64_t(sizeof(nbg_snapshot_info));
    case 3: return int64_t(sizeof(nbg_go_spec));
    case 4: return int64_t(sizeof(nbg_rows));
    case 5: return int64_t(sizeof(nbg_prop_def));
    default: return -1;
  }
}

int32_t nbg_part_of(int64_t vid, int32_t num_parts) {
  return num_parts > 0 ? nbg::part_of_vid(vid, num_parts) : NBG_E_INVALID_ARG;
}
int32_t nbg_rank_of_part(int32_t part, int32_t world_size) {
  return world_size > 0 ? nbg::owner_of_part(part, world_size) : NBG_E_INVALID_ARG;
}

int32_t nbg_schema_set_edge(nbg_ctx* ctx, int32_t edge_type, int32_t schema_ver, int32_t nfields,
                            const char* const* names, const int32_t* types) {
  return guarded(ctx, [&](Ctx& c) {
    if (c.finalized) throw Error(NBG_E_STATE, "snapshot already finalized");
    if (edge_type <= 0) throw Error(NBG_E_INVALID_ARG, "edge type must be > 0");
    if (nfields < 0 || (nfields > 0 && (!names || !types))) throw Error(NBG_E_INVALID_ARG, "bad fields");
    nbg::EdgeSpace& es = c.edges[edge_type];
    if (es.out_stage.n || es.in_stage.n) throw Error(NBG_E_STATE, "schema changed after data was loaded");
    es.type = edge_type;
    es.schema_ver = schema_ver;
    es.fields.clear();
    for (int32_t i = 0; i < nfields; i++) {
      int32_t t = types[i];
      if (t != NBG_T_BOOL && t != NBG_T_INT && t != NBG_T_VID && t != NBG_T_FLOAT && t != NBG_T_DOUBLE &&
          t != NBG_T_STRING && t != NBG_T_TIMESTAMP)
        throw Error(NBG_E_UNSUPPORTED, "unsupported field type");
      es.fields.push_back(nbg::Field{names[i] ? names[i] : "", t});
    }
    return NBG_OK;
  });
}

int32_t nbg_schema_set_tag(nbg_ctx* ctx, int32_t tag_id, const char* tag_name, int32_t schema_ver,
                           int32_t nfields, const char* const* names, const int32_t* types) {
  return guarded(ctx, [&](Ctx& c) {
    if (c.finalized) throw Error(NBG_E_STATE, "snapshot already finalized");
    if (tag_id <= 0 || !tag_name || !*tag_name) throw Error(NBG_E_INVALID_ARG, "tag id must be > 0 with a name");
    if (nfields < 0 || nfields > 64 || (nfields > 0 && (!names || !types))) throw Error(NBG_E_INVALID_ARG, "bad fields");
    for (auto& kv : c.tags)
      if (kv.first != tag_id && kv.second.name == tag_name) throw Error(NBG_E_INVALID_ARG, "duplicate tag name");
    nbg::TagSpace& ts = c.tags[tag_id];
    if (ts.stage.n) throw Error(NBG_E_STATE, "schema changed after data was loaded");
    ts.id = tag_id;
    ts.name = tag_name;
    ts.schema_ver = schema_ver;
    ts.fields.clear();
    for (int32_t i = 0; i < nfields; i++) {
      int32_t t = types[i];
      if (t != NBG_T_BOOL && t != NBG_T_INT && t != NBG_T_VID && t != NBG_T_FLOAT && t != NBG_T_DOUBLE &&
          t != NBG_T_STRING && t != NBG_T_TIMESTAMP)
        throw Error(NBG_E_UNSUPPORTED, "unsupported field type");
      ts.fields.push_back(nbg::Field{names[i] ? names[i] : "", t});
    }
    return NBG_OK;
  });
}

int32_t nbg_snapshot_load_part(nbg_ctx* ctx, int32_t part, const uint8_t* key_bytes, const uint64_t* key_offsets,
                               const uint8_t* val_bytes, const uint64_t* val_offsets, size_t n) {
  return guarded(ctx, [&](Ctx& c) {
    if (n && (!key_bytes || !key_offsets || !val_offsets)) throw Error(NBG_E_INVALID_ARG, "null KV arrays");
    nbg::snapshot_load_part(c, part, key_bytes, key_offsets, val_bytes, val_offsets, n);
    return NBG_OK;
  });
}

int32_t nbg_snapshot_gen_rmat(nbg_ctx* ctx, int32_t scale, int32_t edge_factor, uint64_t seed, int32_t edge_type) {
  return guarded(ctx, [&](Ctx& c) {
    nbg::snapshot_gen_rmat(c, scale, edge_factor, seed, edge_type);
    return NBG_OK;
  });
}

int32_t nbg_snapshot_finalize(nbg_ctx* ctx) {
  return guarded(ctx, [&](Ctx& c) {
    nbg::snapshot_finalize(c);
    return NBG_OK;
  });
}

int32_t nbg_snapshot_write_part(nbg_ctx* ctx, int32_t part, const uint8_t* key_bytes, const uint64_t* key_offsets,
                                const uint8_t* val_bytes, const uint64_t* val_offsets, size_t n) {
  return guarded(ctx, [&](Ctx& c) {
    if (n && (!key_bytes || !key_offsets || !val_offsets)) throw Error(NBG_E_INVALID_ARG, "null KV arrays");
    nbg::snapshot_write_part(c, part, key_bytes, key_offsets, val_bytes, val_offsets, n);
    return NBG_OK;
  });
}

int32_t nbg_snapshot_commit(nbg_ctx* ctx) {
  return guarded(ctx, [&](Ctx& c) {
    nbg::snapshot_commit(c);
    return NBG_OK;
  });
}

int32_t nbg_snapshot_info_get(nbg_ctx* ctx, int32_t edge_type, nbg_snapshot_info* out) {
  return guarded(ctx, [&](Ctx& c) {
    if (!out) throw Error(NBG_E_INVALID_ARG, "null out");
    auto it = c.edges.find(edge_type);
    if (it == c.edges.end()) throw Error(NBG_E_INVALID_ARG, "unknown edge type");
    out->num_vertices = c.n_vertices;
    out->local_vertices = c.counts.empty() ? 0 : c.counts[size_t(c.rank)];
    out->local_out_edges = it->second.out.nnz;
    out->local_in_edges = it->second.in.nnz;
    out->device_bytes = int64_t(it->second.out.bytes() + it->second.in.bytes() + c.vid_of.bytes + c.ht_keys.bytes +
                                c.ht_vals.bytes);
    out->build_seconds = c.build_seconds;
    out->commits = c.commits;
    out->merge_commits = c.merge_commits;
    return NBG_OK;
  });
}

int64_t nbg_snapshot_out_degree(nbg_ctx* ctx, int32_t edge_type, int64_t vid) {
  int64_t result = -1;
  int32_t rc = guarded(ctx, [&](Ctx& c) {
    if (!c.finalized) throw Error(NBG_E_STATE, "not finalized");
    auto it = c.edges.find(edge_type < 0 ? -edge_type : edge_type);
    if (it == c.edges.end()) throw Error(NBG_E_INVALID_ARG, "unknown edge type");
    const nbg::Csr& csr = edge_type < 0 ? it->second.in : it->second.out;
    nbg::DevBuf dv, dg;
    dv.alloc(8);
    dg.alloc(4);
    NBG_HIP(hipMemcpyAsync(dv.p, &vid, 8, hipMemcpyHostToDevice, c.stream));
    nbg::lookup_gidx(c, dv.as<int64_t>(), dg.as<int32_t>(), 1);
    int32_t g = -1;
    NBG_HIP(hipMemcpyAsync(&g, dg.p, 4, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (g < c.owned_lo() || g >= c.owned_hi()) return NBG_OK;
    int64_t rp[2];
    NBG_HIP(hipMemcpy(rp, csr.row_ptr.as<int64_t>() + (g - c.owned_lo()), 16, hipMemcpyDeviceToHost));
    result = rp[1] - rp[0];
    return NBG_OK;
  });
  return rc == NBG_OK ? result : rc;
}

void nbg_rows_free(nbg_rows* rows) {
  if (!rows) return;
  if (rows->_impl) nbg::free_rows_impl(rows->_impl);
  memset(rows, 0, sizeof(*rows));
}

int32_t nbg_get_bound(nbg_ctx* ctx, int32_t edge_type, const int32_t* parts, const int64_t* vids, size_t n,
                      const uint8_t* filter, size_t filter_len, const nbg_prop_def* cols, size_t ncols,
                      nbg_rows* out) {
  return guarded(ctx, [&](Ctx& c) {
    if (!out || (n && (!parts || !vids)) || (ncols && !cols) || (filter_len && !filter))
      throw Error(NBG_E_INVALID_ARG, "bad arguments");
    memset(out, 0, sizeof(*out));
    const int32_t rc = nbg::get_bound_run(c, edge_type, parts, vids, n, filter, filter_len, cols, ncols, out);
    nbg::timing_resolve(c);
    return rc;
  });
}

int32_t nbg_bound_stats(nbg_ctx* ctx, int32_t edge_type, const int32_t* parts, const int64_t* vids, size_t n,
                        const uint8_t* filter, size_t filter_len, const nbg_prop_def* cols,
                        const int32_t* stat_types, size_t ncols, nbg_rows* out) {
  return guarded(ctx, [&](Ctx& c) {
    if (!out || (n && (!parts || !vids)) || (ncols && (!cols || !stat_types)) || (filter_len && !filter))
      throw Error(NBG_E_INVALID_ARG, "bad arguments");
    memset(out, 0, sizeof(*out));
    const int32_t rc = nbg::get_bound_run(c, edge_type, parts, vids, n, filter, filter_len, cols, ncols, out, stat_types);
    nbg::timing_resolve(c);
    return rc;
  });
}

int32_t nbg_go(nbg_ctx* ctx, const nbg_go_spec* spec, nbg_rows* out) {
  return guarded(ctx, [&](Ctx& c) {
    if (!spec || !out || (spec->n_starts && !spec->starts) || (spec->where_len && !spec->where) ||
        (spec->n_yields && (!spec->yields || !spec->yield_lens)))
      throw Error(NBG_E_INVALID_ARG, "bad arguments");
    memset(out, 0, sizeof(*out));
    const int32_t rc = nbg::go_run(c, *spec, out);
    nbg::timing_resolve(c);
    return rc;
  });
}

int32_t nbg_shortest_path(nbg_ctx* ctx, int32_t edge_type, const int64_t* src, const int64_t* dst, size_t npairs,
                          int32_t max_steps, nbg_rows* out) {
  return guarded(ctx, [&](Ctx& c) {
    if (!out || (npairs && (!src || !dst))) throw Error(NBG_E_INVALID_ARG, "bad arguments");
    memset(out, 0, sizeof(*out));
    return nbg::shortest_path_run(c, edge_type, src, dst, npairs, max_steps, out);
  });
}

int32_t nbg_last_timing(nbg_ctx* ctx, nbg_timing* out) {
  return guarded(ctx, [&](Ctx& c) {
    if (!out) throw Error(NBG_E_INVALID_ARG, "null out");
    nbg::resolve_total(c);
    out->total_ms = c.timing.total_ms;
    out->expand_ms = c.timing.expand_ms;
    out->expand_launches = c.timing.expand_launches;
    out->edges_scanned = c.timing.edges_scanned;
    out->expand_bytes = c.timing.expand_bytes;
    out->steps_run = c.timing.steps_run;
    out->bu_steps = c.timing.bu_steps;
    out->comm_ms = c.timing.comm_ms;
    out->comm_bytes = c.timing.comm_bytes;
    out->n_hops = c.timing.n_hops;
    memcpy(out->hops, c.timing.hops, sizeof(out->hops));
    out->host_waits = c.timing.host_waits;
    out->spec_hops = c.timing.spec_hops;
    out->launches = c.timing.launches;
    out->comm_calls = c.timing.comm_calls;
    return NBG_OK;
  });
}

int32_t nbg_set_option(nbg_ctx* ctx, const char* key, int64_t value) {
  return guarded(ctx, [&](Ctx& c) {
    if (!key) throw Error(NBG_E_INVALID_ARG, "null key");
    if (value == INT64_MIN) c.options.erase(key);  // back to the engine default
    else c.options[key] = value;
    return NBG_OK;
  });
}

}  // extern "C"
