// rows.h -- host-side owner of a result handed out through nbg_rows (freed by nbg_rows_free).
#pragma once
#include <cstring>
#include <vector>

#include "engine.h"

namespace nbg {

struct HostRows {
  std::vector<int32_t> types;
  std::vector<void*> cols;
  std::vector<int64_t*> str_off;
  std::vector<DevBuf> dev;       // device column storage when on_device
  std::vector<std::vector<uint8_t>> host;
  std::vector<HostBuf> hpin;  // pinned result columns (GO rows copied to the host)
  std::vector<std::vector<int64_t>> host_off;
  std::vector<int64_t> row_vertex, vertex_ids, vertex_row_offsets;
  std::vector<int32_t> failed_parts, failed_codes;
  std::vector<int64_t> path_offsets, path_vids;  // nbg_shortest_path
  // get_bound tag props per returned vertex
  std::vector<int32_t> vertex_types;
  std::vector<std::vector<uint8_t>> vertex_host, vertex_present;
  std::vector<std::vector<int64_t>> vertex_host_off;
  std::vector<void*> vertex_cols;
  std::vector<int64_t*> vertex_str_off;
  std::vector<uint8_t*> vertex_pres;
};

inline void fill_rows(nbg_rows* out, HostRows* h, int64_t nrows, bool on_device) {
  memset(out, 0, sizeof(*out));
  out->n_rows = nrows;
  out->n_cols = int32_t(h->types.size());
  out->on_device = on_device ? 1 : 0;
  out->col_types = h->types.data();
  out->cols = h->cols.data();
  out->str_offsets = h->str_off.data();
  out->row_vertex = h->row_vertex.empty() ? nullptr : h->row_vertex.data();
  out->n_vertices = int64_t(h->vertex_ids.size());
  out->vertex_ids = h->vertex_ids.empty() ? nullptr : h->vertex_ids.data();
  out->vertex_row_offsets = h->vertex_row_offsets.empty() ? nullptr : h->vertex_row_offsets.data();
  out->n_failed = int32_t(h->failed_parts.size());
  out->failed_parts = h->failed_parts.empty() ? nullptr : h->failed_parts.data();
  out->failed_codes = h->failed_codes.empty() ? nullptr : h->failed_codes.data();
  out->path_offsets = h->path_offsets.empty() ? nullptr : h->path_offsets.data();
  out->path_vids = h->path_vids.empty() ? nullptr : h->path_vids.data();
  out->_impl = h;
  h->vertex_cols.clear();
  h->vertex_str_off.clear();
  h->vertex_pres.clear();
  for (size_t i = 0; i < h->vertex_types.size(); i++) {
    h->vertex_cols.push_back(h->vertex_host[i].data());
    h->vertex_str_off.push_back(h->vertex_host_off[i].empty() ? nullptr : h->vertex_host_off[i].data());
    h->vertex_pres.push_back(h->vertex_present[i].data());
  }
  out->n_vertex_cols = int32_t(h->vertex_types.size());
  out->vertex_col_types = h->vertex_types.empty() ? nullptr : h->vertex_types.data();
  out->vertex_cols = h->vertex_cols.empty() ? nullptr : h->vertex_cols.data();
  out->vertex_str_offsets = h->vertex_str_off.empty() ? nullptr : h->vertex_str_off.data();
  out->vertex_col_present = h->vertex_pres.empty() ? nullptr : h->vertex_pres.data();
}

}  // namespace nbg
