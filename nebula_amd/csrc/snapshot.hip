// snapshot.hip -- snapshot builder: reference KV bytes (or synthetic RMAT tuples) -> GPU CSR.
//
// Stage 1 (decode, per loaded part): one thread per KV pair parses the 40-byte edge key
//   (NebulaKeyUtils.h:14-21: part i32 | src i64 | type i32 | rank i64 | dst i64 | ver i64, LE)
//   and, for out-edges, the RowWriter row (RowWriter.cpp:49-75: header byte, schema version,
//   block offsets every 16 fields, INT = LEB128 varint, VID/TIMESTAMP 8 B, DOUBLE 8 B, FLOAT
//   4 B, BOOL 1 B, STRING varint length + bytes).  Field offsets follow RowReader::skipToField
//   (RowReader.cpp:276-368), including the stored block offsets.  Output: SoA tuples.
// Stage 2 (finalize): vertex set, vid<->gidx map, sort each rank's tuples into the reference's
//   key order, keep the bytewise-first version of every (src, rank, dst)
//   (QueryBaseProcessor.inl:349-362, P3), emit CSR + narrowed SoA property columns.
#include <climits>

#include <rocprim/device/device_merge.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <numeric>

#include "device_common.h"
#include "engine.h"

namespace nbg {

constexpr int kMaxFields = 64;
struct SchemaDev {
  int32_t nfields;
  int32_t types[kMaxFields];
};

// the context's build-time block cache (option build_pool_gb, 0 = plain hipMalloc / hipFree)
static std::shared_ptr<BufPool> build_pool(Ctx& c) {
  const int64_t gb = c.opt("build_pool_gb", 128);
  if (gb <= 0) return nullptr;
  c.build_pool->limit = size_t(gb) << 30;
  return c.build_pool;
}

// ------------------------------------------------------------------------------------------
// small generic kernels
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void k_fill(T* p, T v, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    p[i] = v;
}
__global__ void k_iota_rev_u32(uint32_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    p[i] = uint32_t(n - 1 - i);
}
__global__ void k_iota_u32(uint32_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    p[i] = uint32_t(i);
}
static int grid_for(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  return int(std::max<int64_t>(1, std::min<int64_t>(g, 2048 * 8)));
}
template <typename T>
static void fill(Ctx& c, T* p, T v, int64_t n) {
  if (n <= 0) return;
  k_fill<T><<<grid_for(n), 256, 0, c.stream>>>(p, v, n);
}

// grows b to at least `need` bytes keeping its contents: exactly `need` (the caller sized it), or
// 1.25x the old size when that is larger (amortised appends of many small batches)
static void grow_copy(Ctx& c, DevBuf& b, size_t need, bool exact = false) {
  if (need <= b.bytes) return;
  DevBuf nb;
  nb.alloc(exact ? need : std::max(need, b.bytes + b.bytes / 4));
  if (b.bytes) NBG_HIP(hipMemcpyAsync(nb.p, b.p, b.bytes, hipMemcpyDeviceToDevice, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  b = std::move(nb);
}

__global__ void k_hash_part(const int64_t* src, int32_t* part, int64_t n, int32_t parts) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    part[i] = int32_t(uint64_t(src[i]) % uint64_t(parts) + 1);
}

// A device-generated stage (snapshot_gen_rmat) keeps rank / version as constants, the key part
// implicit (hash rule), no sequence numbers and no present bytes.  Before decoded KV tuples are
// appended behind it (a write batch), spell those columns out: the generated tuples precede every
// later write (sequence 0), their part is the hash part of the key's vertex.
static void materialize_stage(Ctx& c, Staging& s, size_t nfields, bool with_props) {
  if (s.n == 0 || s.seq.p) return;
  const int64_t n = s.n;
  const size_t cap = std::max(s.cap, size_t(n));
  s.rank.alloc(cap * 8);
  s.ver.alloc(cap * 8);
  s.part.alloc(cap * 4);
  s.seq.alloc(cap * 8);
  fill<int64_t>(c, s.rank.as<int64_t>(), s.rank_value, n);
  fill<int64_t>(c, s.ver.as<int64_t>(), s.ver_value, n);
  fill<int64_t>(c, s.seq.as<int64_t>(), 0, n);
  k_hash_part<<<grid_for(n), 256, 0, c.stream>>>(s.src.as<int64_t>(), s.part.as<int32_t>(), n, c.num_parts);
  NBG_HIP(hipGetLastError());
  if (with_props) {
    s.present.resize(std::max(s.present.size(), nfields));
    for (size_t f = 0; f < nfields; f++)
      if (!s.present[f].p) {
        s.present[f].alloc(cap);
        fill<uint8_t>(c, s.present[f].as<uint8_t>(), 1, n);
      }
  }
  s.rank_const = s.ver_const = false;
  s.cap = cap;
  c.load_seq = std::max<int64_t>(c.load_seq, 1);
  NBG_HIP(hipStreamSynchronize(c.stream));
}

static void stage_reserve(Ctx& c, Staging& s, size_t nfields, size_t extra, bool with_props,
                          const std::vector<Field>& fields) {
  materialize_stage(c, s, nfields, with_props);
  size_t need = size_t(s.n) + extra;
  if (need <= s.cap) return;
  // 1.25x growth: a write batch appended behind a device-sized stage must not double it
  size_t cap = std::max(need, s.cap + s.cap / 4);
  grow_copy(c, s.src, cap * 8, true);
  grow_copy(c, s.dst, cap * 8, true);
  grow_copy(c, s.rank, cap * 8, true);
  grow_copy(c, s.ver, cap * 8, true);
  grow_copy(c, s.part, cap * 4, true);
  grow_copy(c, s.seq, cap * 8, true);
  if (with_props) {
    s.props.resize(nfields);
    s.present.resize(nfields);
    s.str_len.resize(nfields);
    for (size_t f = 0; f < nfields; f++) {
      grow_copy(c, s.props[f], cap * 8, true);
      grow_copy(c, s.present[f], cap, true);
      if (fields[f].type == NBG_T_STRING) grow_copy(c, s.str_len[f], cap * 8, true);
    }
  }
  s.cap = cap;
}

// ------------------------------------------------------------------------------------------
// Stage 1a: KV decode
// ------------------------------------------------------------------------------------------
struct StageOut {
  int32_t* part;
  int64_t* src;
  int64_t* dst;
  int64_t* rank;
  int64_t* ver;
  int64_t* seq;
  int64_t* props[kMaxFields];
  uint8_t* present[kMaxFields];
  int64_t* str_len[kMaxFields];
};

template <typename T>
__device__ inline T ld_unaligned(const uint8_t* p) {
  T v;
  __builtin_memcpy(&v, p, sizeof(T));
  return v;
}

__device__ inline int dev_varint(const uint8_t* p, int64_t avail, uint64_t& out) {
  uint64_t v = 0;
  for (int i = 0; i < 10 && i < avail; i++) {
    v |= uint64_t(p[i] & 0x7f) << (7 * i);
    if (!(p[i] & 0x80)) {
      out = v;
      return i + 1;
    }
  }
  return -1;
}

// Decodes one row into field slots.  Mirrors RowReader: header (RowReader.cpp:218-263),
// sequential skip (skipToNext :276-341), stored block offsets for fields 16k (:239-249).
__device__ void decode_row(const uint8_t* row, int64_t len, const SchemaDev& sch, int64_t heap_off,
                           const StageOut& o, int64_t slot, unsigned long long* err) {
  int nf = sch.nfields;
  if (len <= 0) {
    for (int f = 0; f < nf; f++) o.present[f][slot] = 0;
    return;
  }
  uint8_t h = row[0];
  int offBytes = (h & 7) + 1;
  int verBytes = h >> 5;
  int numOffsets = nf >> 4;
  int64_t hdr = 1 + verBytes + int64_t(offBytes) * numOffsets;
  if (hdr > len) {  // "Rowe data is too short": reader is invalid, no props
    for (int f = 0; f < nf; f++) o.present[f][slot] = 0;
    atomicAdd(err, 1ull);
    return;
  }
  const uint8_t* data = row + hdr;
  int64_t dlen = len - hdr;
  int64_t pos = 0;
  bool broken = false;
  for (int f = 0; f < nf; f++) {
    if (f > 0 && (f & 15) == 0) {
      int64_t bo = 0;
      const uint8_t* ob = row + 1 + verBytes + int64_t(offBytes) * ((f >> 4) - 1);
      for (int j = 0; j < offBytes; j++) bo |= int64_t(uint64_t(ob[j]) << (8 * j));
      pos = bo;
      broken = false;
    }
    int64_t v = 0;
    int64_t next = -1;
    if (!broken && pos >= 0 && pos <= dlen) {
      switch (sch.types[f]) {
        case NBG_T_BOOL:
          if (pos + 1 <= dlen) { v = data[pos] != 0; next = pos + 1; }
          break;
        case NBG_T_INT: {
          uint64_t u;
          int n = dev_varint(data + pos, dlen - pos, u);
          if (n > 0) { v = int64_t(u); next = pos + n; }
          break;
        }
        case NBG_T_VID:
        case NBG_T_TIMESTAMP:
          if (pos + 8 <= dlen) { v = ld_unaligned<int64_t>(data + pos); next = pos + 8; }
          break;
        case NBG_T_FLOAT:
          if (pos + 4 <= dlen) {
            double d = double(ld_unaligned<float>(data + pos));
            v = __double_as_longlong(d);
            next = pos + 4;
          }
          break;
        case NBG_T_DOUBLE:
          if (pos + 8 <= dlen) { v = ld_unaligned<int64_t>(data + pos); next = pos + 8; }
          break;
        case NBG_T_STRING: {
          uint64_t sl;
          int n = dev_varint(data + pos, dlen - pos, sl);
          if (n > 0 && pos + n + int64_t(sl) <= dlen) {
            v = heap_off + hdr + pos + n;
            o.str_len[f][slot] = int64_t(sl);
            next = pos + n + int64_t(sl);
          }
          break;
        }
        default: break;
      }
    }
    if (next < 0) {
      broken = true;
      o.present[f][slot] = 0;
      o.props[f][slot] = 0;
    } else {
      o.present[f][slot] = 1;
      o.props[f][slot] = v;
      pos = next;
    }
  }
}

__global__ void k_decode_kv(const uint8_t* __restrict__ kb, const uint64_t* __restrict__ koff,
                            const uint8_t* __restrict__ vb, const uint64_t* __restrict__ voff,
                            int64_t n, int32_t etype, int32_t sver, SchemaDev sch, int64_t heap_base,
                            int64_t seq0, StageOut outS, unsigned long long* out_cnt, StageOut inS,
                            unsigned long long* in_cnt, unsigned long long* err, int32_t req_part, int32_t parts,
                            int32_t world, int32_t my_rank) {
  int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t n_rounds = (n + stride - 1) / stride;
  for (int64_t r = 0; r < n_rounds; r++) {
    int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool is_out = false, is_in = false;
    int64_t src = 0, dst = 0, rank = 0, ver = 0;
    int32_t kpart = 0;
    if (i < n) {
      uint64_t k0 = koff[i], k1 = koff[i + 1];
      if (k1 - k0 == 40) {
        const uint8_t* k = kb + k0;
        int32_t type = ld_unaligned<int32_t>(k + 12);
        if (type == etype || type == -etype) {
          kpart = ld_unaligned<int32_t>(k);
          src = ld_unaligned<int64_t>(k + 4);
          rank = ld_unaligned<int64_t>(k + 16);
          dst = ld_unaligned<int64_t>(k + 24);
          ver = ld_unaligned<int64_t>(k + 32);
          is_out = type == etype;
          is_in = !is_out;
          // a part holds only keys of its own prefix, and with several ranks this rank can only
          // host rows of the vertices it owns (err[2]: the whole batch is refused)
          if (kpart != req_part || (world > 1 && dev_owner(src, parts, world) != my_rank)) atomicAdd(err + 2, 1ull);
        }
      }
    }
    int64_t so = wave_append(out_cnt, is_out);
    int64_t si = wave_append(in_cnt, is_in);
    if (is_out) {
      outS.part[so] = kpart;
      outS.src[so] = src;
      outS.dst[so] = dst;
      outS.rank[so] = rank;
      outS.ver[so] = ver;
      outS.seq[so] = seq0 + i;
      uint64_t v0 = voff[i], v1 = voff[i + 1];
      const uint8_t* row = vb + v0;
      int64_t len = int64_t(v1 - v0);
      if (len > 0) {
        // schema version from the row header (RowReader.cpp:173-199)
        int verBytes = row[0] >> 5;
        int32_t rv = 0;
        if (verBytes > 0 && verBytes + 1 <= len)
          for (int b = 0; b < verBytes; b++) rv |= int32_t(uint32_t(row[1 + b]) << (8 * b));
        if (rv != sver) atomicAdd(err + 1, 1ull);
      }
      decode_row(row, len, sch, heap_base + int64_t(v0), outS, so, err);
    }
    if (is_in) {
      inS.part[si] = kpart;
      inS.src[si] = src;
      inS.dst[si] = dst;
      inS.rank[si] = rank;
      inS.ver[si] = ver;
      inS.seq[si] = seq0 + i;
    }
  }
}

// Vertex keys (NebulaKeyUtils.h:14-17: part i32 | vid i64 | tag i32 | ver i64, 24 bytes) of one
// tag -> staged (vid, ver, part, load sequence) + decoded row fields.
__global__ void k_decode_vkv(const uint8_t* __restrict__ kb, const uint64_t* __restrict__ koff,
                             const uint8_t* __restrict__ vb, const uint64_t* __restrict__ voff, int64_t n,
                             int32_t tag, int32_t sver, SchemaDev sch, int64_t heap_base, int64_t seq0,
                             StageOut o, unsigned long long* cnt, unsigned long long* err, int32_t req_part) {
  int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t n_rounds = (n + stride - 1) / stride;
  for (int64_t r = 0; r < n_rounds; r++) {
    int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool hit = false;
    if (i < n && koff[i + 1] - koff[i] == 24) hit = ld_unaligned<int32_t>(kb + koff[i] + 12) == tag;
    int64_t so = wave_append(cnt, hit);
    if (!hit) continue;
    const uint8_t* k = kb + koff[i];
    if (ld_unaligned<int32_t>(k) != req_part) atomicAdd(err + 2, 1ull);
    o.part[so] = ld_unaligned<int32_t>(k);
    o.src[so] = ld_unaligned<int64_t>(k + 4);
    o.ver[so] = ld_unaligned<int64_t>(k + 16);
    o.seq[so] = seq0 + i;
    const uint8_t* row = vb + voff[i];
    int64_t len = int64_t(voff[i + 1] - voff[i]);
    if (len > 0) {
      int verBytes = row[0] >> 5;
      int32_t rv = 0;
      if (verBytes > 0 && verBytes + 1 <= len)
        for (int b = 0; b < verBytes; b++) rv |= int32_t(uint32_t(row[1 + b]) << (8 * b));
      if (rv != sver) atomicAdd(err + 1, 1ull);
    }
    decode_row(row, len, sch, heap_base + int64_t(voff[i]), o, so, err);
  }
}

static StageOut stage_ptrs(Staging& s, size_t nf) {
  StageOut o{};
  o.part = s.part.as<int32_t>();
  o.src = s.src.as<int64_t>();
  o.dst = s.dst.as<int64_t>();
  o.rank = s.rank.as<int64_t>();
  o.ver = s.ver.as<int64_t>();
  o.seq = s.seq.as<int64_t>();
  for (size_t f = 0; f < nf && f < size_t(kMaxFields); f++) {
    o.props[f] = f < s.props.size() ? s.props[f].as<int64_t>() : nullptr;
    o.present[f] = f < s.present.size() ? s.present[f].as<uint8_t>() : nullptr;
    o.str_len[f] = f < s.str_len.size() ? s.str_len[f].as<int64_t>() : nullptr;
  }
  return o;
}

static void decode_part(Ctx& c, int32_t part, const uint8_t* kb, const uint64_t* koff,
                        const uint8_t* vb, const uint64_t* voff, size_t n) {
  if (part < 0 || part > c.num_parts) throw Error(NBG_E_PART_NOT_FOUND, "part out of range");
  if (owner_of_part(part, c.world) != c.rank)
    throw Error(NBG_E_PART_NOT_FOUND, "part " + std::to_string(part) + " is not owned by this rank");
  if (c.edges.empty() && c.tags.empty()) throw Error(NBG_E_STATE, "no edge or tag schema registered");
  if (n == 0) return;
  double t0 = now_s();
  size_t kbytes = koff[n], vbytes = voff[n];
  DevBuf dk, dko, dvo;
  dk.alloc(kbytes + 8);
  dko.alloc((n + 1) * 8);
  dvo.alloc((n + 1) * 8);
  NBG_HIP(hipMemcpyAsync(dk.p, kb, kbytes, hipMemcpyHostToDevice, c.stream));
  NBG_HIP(hipMemcpyAsync(dko.p, koff, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  NBG_HIP(hipMemcpyAsync(dvo.p, voff, (n + 1) * 8, hipMemcpyHostToDevice, c.stream));
  // value bytes go to the string heap (kept until finalize for STRING props)
  int64_t heap_base = int64_t(c.heap_used);
  grow_copy(c, c.heap, c.heap_used + vbytes + 8);
  if (vbytes) NBG_HIP(hipMemcpyAsync(c.heap.as<uint8_t>() + heap_base, vb, vbytes, hipMemcpyHostToDevice, c.stream));
  c.heap_used += vbytes;
  DevBuf cnt;
  cnt.alloc(64);
  // A RocksDB write batch for one part is all or nothing: remember where every stage ended, and
  // on any refusal roll them (and the value heap) back.  The load sequence advances either way,
  // so a later batch never reuses this one's numbers (identical-key order stays unambiguous).
  struct Mark {
    Staging* s;
    int64_t n;
  };
  std::vector<Mark> marks;
  for (auto& kvp : c.edges) {
    marks.push_back(Mark{&kvp.second.out_stage, kvp.second.out_stage.n});
    marks.push_back(Mark{&kvp.second.in_stage, kvp.second.in_stage.n});
  }
  for (auto& kvp : c.tags) marks.push_back(Mark{&kvp.second.stage, kvp.second.stage.n});
  const size_t heap_mark = size_t(heap_base);
  try {
  for (auto& kvp : c.edges) {
    EdgeSpace& es = kvp.second;
    size_t nf = es.fields.size();
    if (nf > size_t(kMaxFields)) throw Error(NBG_E_UNSUPPORTED, "more than 64 edge fields");
    SchemaDev sch{};
    sch.nfields = int32_t(nf);
    for (size_t f = 0; f < nf; f++) sch.types[f] = es.fields[f].type;
    stage_reserve(c, es.out_stage, nf, n, true, es.fields);
    stage_reserve(c, es.in_stage, 0, n, false, es.fields);
    NBG_HIP(hipMemsetAsync(cnt.p, 0, 64, c.stream));
    unsigned long long* d = cnt.as<unsigned long long>();
    NBG_HIP(hipMemcpyAsync(d, &es.out_stage.n, 8, hipMemcpyHostToDevice, c.stream));
    NBG_HIP(hipMemcpyAsync(d + 1, &es.in_stage.n, 8, hipMemcpyHostToDevice, c.stream));
    StageOut so = stage_ptrs(es.out_stage, nf);
    StageOut si = stage_ptrs(es.in_stage, 0);
    k_decode_kv<<<grid_for(int64_t(n)), 256, 0, c.stream>>>(
        dk.as<uint8_t>(), dko.as<uint64_t>(), c.heap.as<uint8_t>() + heap_base, dvo.as<uint64_t>(),
        int64_t(n), es.type, es.schema_ver, sch, heap_base, c.load_seq, so, d, si, d + 1, d + 2, part, c.num_parts,
        c.world, c.rank);
    NBG_HIP(hipGetLastError());
    unsigned long long h[5];
    NBG_HIP(hipMemcpyAsync(h, d, 40, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    es.out_stage.n = int64_t(h[0]);  // the marks roll back a refused batch
    es.in_stage.n = int64_t(h[1]);
    if (h[3] != 0)
      throw Error(NBG_E_UNSUPPORTED, "row schema version differs from the registered version");
    if (h[4] != 0)
      throw Error(NBG_E_PART_NOT_FOUND, "edge key of another part, or of a vertex another rank owns");
    es.out_stage.rank_const = es.out_stage.ver_const = false;
    es.in_stage.rank_const = es.in_stage.ver_const = false;
  }
  for (auto& kvp : c.tags) {
    TagSpace& ts = kvp.second;
    size_t nf = ts.fields.size();
    SchemaDev sch{};
    sch.nfields = int32_t(nf);
    for (size_t f = 0; f < nf; f++) sch.types[f] = ts.fields[f].type;
    stage_reserve(c, ts.stage, nf, n, true, ts.fields);
    NBG_HIP(hipMemsetAsync(cnt.p, 0, 64, c.stream));
    unsigned long long* d = cnt.as<unsigned long long>();
    NBG_HIP(hipMemcpyAsync(d, &ts.stage.n, 8, hipMemcpyHostToDevice, c.stream));
    k_decode_vkv<<<grid_for(int64_t(n)), 256, 0, c.stream>>>(
        dk.as<uint8_t>(), dko.as<uint64_t>(), c.heap.as<uint8_t>() + heap_base, dvo.as<uint64_t>(), int64_t(n),
        ts.id, ts.schema_ver, sch, heap_base, c.load_seq, stage_ptrs(ts.stage, nf), d, d + 2, part);
    NBG_HIP(hipGetLastError());
    unsigned long long h[5];
    NBG_HIP(hipMemcpyAsync(h, d, 40, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    ts.stage.n = int64_t(h[0]);
    if (h[3] != 0) throw Error(NBG_E_UNSUPPORTED, "tag row schema version differs from the registered version");
    if (h[4] != 0) throw Error(NBG_E_PART_NOT_FOUND, "vertex key of another part");
  }
  } catch (...) {
    for (auto& m : marks) m.s->n = m.n;
    c.heap_used = heap_mark;
    c.load_seq += int64_t(n);
    throw;
  }
  c.load_seq += int64_t(n);
  c.build_seconds += now_s() - t0;
}

void snapshot_load_part(Ctx& c, int32_t part, const uint8_t* kb, const uint64_t* koff,
                        const uint8_t* vb, const uint64_t* voff, size_t n) {
  PoolScope build_scope(build_pool(c));  // staged tuples
  if (c.finalized) throw Error(NBG_E_STATE, "snapshot already finalized");
  decode_part(c, part, kb, koff, vb, voff, n);
}

// ------------------------------------------------------------------------------------------
// Write path.  AddEdgesProcessor / AddVerticesProcessor turn a request into one
// batch of KV puts per part (AddEdgesProcessor.cpp:15-31, AddVerticesProcessor.cpp:16-38; the
// version in the key is INT64_MAX - now_us, so a newer write of the same edge sorts first and
// an identical key overwrites).  A writable snapshot keeps the decoded tuples of everything
// loaded so far (the stages, read-only to the CSR build: the "log") next to the CSRs; a write
// batch is decoded by the same k_decode_kv /
// k_decode_vkv behind the log with later load sequence numbers, so the CSR build's version
// dedup (bytewise-first key, last write of an identical key) gives exactly what the prefix scan
// of the written RocksDB part returns.  nbg_snapshot_commit rebuilds the vertex map, CSRs,
// transposes and tag columns from the log on the device -- nothing is re-uploaded -- and until
// then queries keep reading the previous commit (a RocksDB snapshot's view).
// ------------------------------------------------------------------------------------------
// drop what build_transpose derives from the out CSRs of every rank
static void reset_transpose_derived(EdgeSpace& es) {
  es.rep_out = Csr();
  es.rep_in = Csr();
  es.has_rep = es.has_rep_out = false;
  es.rep_odeg.release();
  es.tr = Csr();
  es.t_eid.release();
  es.has_tr = es.has_t_eid = false;
  es.out_nnz_global = -1;
  es.tcol_q.release();
  es.q_field = -1;
  es.q_gbits = es.q_bits = 0;
  for (int h = 0; h < 2; h++) es.pair_col[h].release();
  es.odeg.release();
  es.odeg8.release();
  es.max_odeg = -1;
  es.max_odeg_global = -1;
  es.top_deg.clear();
  es.bu_in_tiles = es.bu_both_tiles = 0;
  es.brec.release();
  es.brec_rows = 0;
}

// drop everything snapshot_finalize derives from the staged tuples
static void reset_edge_derived(EdgeSpace& es) {
  es.out = Csr();
  es.in = Csr();
  reset_transpose_derived(es);
}

static void reset_derived(Ctx& c) {
  c.brank.release();
  for (auto& kv : c.edges)
    for (auto& o : kv.second.ord) {
      o.perm.release();
      o.skey.release();
      o.dstg.release();
      o.n = 0;
    }
  c.vid_of.release();
  c.ht_keys.release();
  c.ht_vals.release();
  c.ht_cap = 0;
  c.ht_has_min = false;
  c.ht_min_gidx = -1;
  c.tag_table.release();
  for (auto& kv : c.edges) reset_edge_derived(kv.second);
  for (auto& kv : c.tags) {
    kv.second.cols.clear();
    kv.second.part.release();
  }
  c.sp_dist[0].release();
  c.sp_dist[1].release();
  c.sp_dist_bytes = 0;
  c.sp_dirty = false;
  c.sp = Ctx::SpWork();
}

// Merge commit: each edge CSR merges its sorted batch into the committed order (build_csr merge
// mode) and the transposed CSR is rebuilt from the new out CSRs.  One rank: new vertices extend
// the numbering (appended gidx) and tag writes rebuild the tag columns.  Several ranks: batches
// of edges and tag rows merge on every rank together; a batch with a new vertex anywhere takes
// the full rebuild (appending to one rank's gidx range would move every later rank's).  Returns
// false when the batch needs the full rebuild.
static bool commit_merge(Ctx& c);

void snapshot_write_part(Ctx& c, int32_t part, const uint8_t* kb, const uint64_t* koff,
                         const uint8_t* vb, const uint64_t* voff, size_t n) {
  PoolScope build_scope(build_pool(c));  // staged tuples
  if (!c.finalized) {  // before the first commit a write batch is one more loaded batch
    decode_part(c, part, kb, koff, vb, voff, n);
    return;
  }
  if (!c.has_log) throw Error(NBG_E_STATE, "snapshot is not writable (set option writable=1 before finalize)");
  decode_part(c, part, kb, koff, vb, voff, n);  // behind the kept tuples; the CSRs are untouched
  c.pending_writes = true;
}

void snapshot_commit(Ctx& c) {
  if (!c.finalized) {
    // first finalize, or a retry after a commit whose rebuild failed half-way (e.g. E_NOMEM):
    // whatever that attempt derived is dropped before building again
    NBG_HIP(hipStreamSynchronize(c.stream));
    reset_derived(c);
    snapshot_finalize(c);
    return;
  }
  if (!c.has_log) throw Error(NBG_E_STATE, "snapshot is not writable (set option writable=1 before finalize)");
  // collective when world > 1: every rank rebuilds, with or without writes of its own
  NBG_HIP(hipStreamSynchronize(c.stream));
  if (commit_merge(c)) {
    c.pending_writes = false;
    c.commits++;
    c.merge_commits++;
    return;
  }
  reset_derived(c);
  c.pending_writes = false;
  c.finalized = false;
  snapshot_finalize(c);
  c.commits++;
}

// ------------------------------------------------------------------------------------------
// Stage 1b: synthetic RMAT (definition shared with oracle/refcpu.cpp)
// ------------------------------------------------------------------------------------------
constexpr uint32_t kTA = 2448131358u;    // floor(0.57 * 2^32)
constexpr uint32_t kTAB = 3264175144u;   // floor(0.76 * 2^32)
constexpr uint32_t kTABC = 4080218931u;  // floor(0.95 * 2^32)

__device__ inline void rmat_pick(uint32_t r, uint64_t& u, uint64_t& v) {
  uint64_t bu = (r >= kTAB) ? 1 : 0;
  uint64_t bv = ((r >= kTA && r < kTAB) || r >= kTABC) ? 1 : 0;
  u = (u << 1) | bu;
  v = (v << 1) | bv;
}
__device__ inline int64_t rmat_vid(uint64_t idx, uint64_t smix) {
  const uint64_t M = (1ull << 63) - 1;
  uint64_t x = (idx + smix) & M;
  x ^= x >> 29;
  x = (x * 0xBF58476D1CE4E5B9ull) & M;
  x ^= x >> 32;
  x = (x * 0x94D049BB133111EBull) & M;
  x ^= x >> 29;
  return int64_t(x);
}

// sample i of the generator: (u, v) in the index space [0, 2^scale)
__device__ inline void rmat_sample(uint64_t i, int32_t scale, uint64_t seed, uint64_t& u, uint64_t& v) {
  u = 0;
  v = 0;
  for (int32_t l = 0; l < scale; l += 2) {
    uint64_t h = splitmix64(seed ^ (0xD6E8FEB86659FD93ull * (i + 1)) ^ (0xA0761D6478BD642Full * uint64_t(l + 1)));
    rmat_pick(uint32_t(h >> 32), u, v);
    if (l + 1 < scale) rmat_pick(uint32_t(h), u, v);
  }
}
// the edge prop of sample (s, d): follow.weight (same value for every duplicate of the pair)
__device__ inline int64_t rmat_weight(int64_t s, int64_t d, uint64_t seed) {
  const uint64_t du = uint64_t(d);
  return int64_t(splitmix64(uint64_t(s) ^ ((du << 32) | (du >> 32)) ^ seed) % 1000);
}

__global__ void k_gen_rmat(int64_t lo, int64_t hi, int32_t scale, uint64_t seed, uint64_t smix,
                           int32_t parts, int32_t world, int32_t rank, int64_t* osrc, int64_t* odst,
                           int64_t* oweight, unsigned long long* ocnt, int64_t* isrc, int64_t* idst,
                           unsigned long long* icnt, int64_t cap) {
  int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t n = hi - lo;
  int64_t rounds = (n + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    int64_t j = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool valid = j < n;
    int64_t s = 0, d = 0;
    if (valid) {
      uint64_t u, v;
      rmat_sample(uint64_t(lo + j), scale, seed, u, v);
      s = rmat_vid(u, smix);
      d = rmat_vid(v, smix);
    }
    bool is_out = valid && (world == 1 || dev_owner(s, parts, world) == rank);
    bool is_in = valid && (world == 1 || dev_owner(d, parts, world) == rank);
    int64_t so = wave_append(ocnt, is_out);
    int64_t si = wave_append(icnt, is_in);
    if (is_out && so < cap) {  // counts keep growing past cap: the host re-runs with the exact size
      osrc[so] = s;
      odst[so] = d;
      oweight[so] = rmat_weight(s, d, seed);
    }
    if (is_in && si < cap) {  // in-edge key (dst, -type, rank, src): key src = d, key dst = s
      isrc[si] = d;
      idst[si] = s;
    }
  }
}

void snapshot_gen_rmat(Ctx& c, int32_t scale, int32_t ef, uint64_t seed, int32_t et) {
  PoolScope build_scope(build_pool(c));  // staged tuples
  if (c.finalized) throw Error(NBG_E_STATE, "snapshot already finalized");
  auto it = c.edges.find(et);
  if (it == c.edges.end()) throw Error(NBG_E_INVALID_ARG, "edge type not registered");
  EdgeSpace& es = it->second;
  if (es.fields.size() != 1 || es.fields[0].type != NBG_T_INT)
    throw Error(NBG_E_INVALID_ARG, "RMAT edge schema must be (weight int)");
  if (scale < 1 || scale > 31 || ef < 1) throw Error(NBG_E_INVALID_ARG, "bad RMAT scale");
  double t0 = now_s();
  int64_t E = int64_t(ef) << scale;
  int64_t expect = !c.sharded ? E : E / c.world + E / (4 * c.world) + (1 << 20);
  Staging& so = es.out_stage;
  Staging& si = es.in_stage;
  if (so.n != 0 || si.n != 0 || es.rmat_stream) throw Error(NBG_E_STATE, "RMAT must be the only source of this edge type");
  // streamed build: forced with rmat_stream = 1, automatic on one rank once the tuple stage
  // would pass its 2^32 cap (2^31 samples and up: two CSR directions of 40+ B tuples)
  const int64_t stream_opt = c.opt("rmat_stream", -1);
  if (!c.sharded && (stream_opt > 0 || (stream_opt < 0 && E >= (int64_t(1) << 31)))) {
    if (c.opt("writable", 0)) throw Error(NBG_E_UNSUPPORTED, "streamed RMAT snapshot is read-only (writable = 1)");
    es.rmat_stream = true;
    es.rmat_scale = scale;
    es.rmat_ef = ef;
    es.rmat_seed = seed;
    return;
  }
  auto alloc_stage = [&](Staging& s, int64_t cap, bool props) {
    s.src.alloc(size_t(cap) * 8);
    s.dst.alloc(size_t(cap) * 8);
    s.rank.release();
    s.ver.release();
    s.part.release();
    s.seq.release();
    s.rank_const = s.ver_const = true;
    s.rank_value = 0;
    s.ver_value = INT64_MAX - 1;
    if (props) {
      s.props.resize(1);
      s.present.resize(1);
      s.str_len.resize(1);
      s.props[0].alloc(size_t(cap) * 8);
      s.present[0].release();  // all present
    }
    s.cap = size_t(cap);
  };
  DevBuf cnt;
  cnt.alloc(16);
  unsigned long long* d = cnt.as<unsigned long long>();
  uint64_t smix = splitmix64(seed) & ((1ull << 63) - 1);
  const int64_t chunk = int64_t(1) << 26;
  unsigned long long h[2];
  for (int attempt = 0; attempt < 2; attempt++) {
    alloc_stage(so, expect, true);
    alloc_stage(si, expect, false);
    NBG_HIP(hipMemsetAsync(cnt.p, 0, 16, c.stream));
    for (int64_t lo = 0; lo < E; lo += chunk) {
      int64_t hi = std::min(E, lo + chunk);
      k_gen_rmat<<<grid_for(hi - lo), 256, 0, c.stream>>>(lo, hi, scale, seed, smix, c.num_parts, c.world,
                                                        c.rank, so.src.as<int64_t>(), so.dst.as<int64_t>(),
                                                        so.props[0].as<int64_t>(), d, si.src.as<int64_t>(),
                                                        si.dst.as<int64_t>(), d + 1, expect);
      NBG_HIP(hipGetLastError());
    }
    NBG_HIP(hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (int64_t(std::max(h[0], h[1])) <= expect) break;
    expect = int64_t(std::max(h[0], h[1]));  // skewed ownership: regenerate with the exact size
  }
  so.n = int64_t(h[0]);
  si.n = int64_t(h[1]);
  c.build_seconds += now_s() - t0;
}

// ------------------------------------------------------------------------------------------
// Stage 2: finalize
// ------------------------------------------------------------------------------------------
template <typename K, typename V>
static void radix_pairs(Ctx& c, K* kin, K* kout, V* vin, V* vout, int64_t n, int bits) {
  size_t tb = 0;
  NBG_HIP(rocprim::radix_sort_pairs(nullptr, tb, kin, kout, vin, vout, size_t(n), 0, bits, c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::radix_sort_pairs(c.ws_tmp.p, tb, kin, kout, vin, vout, size_t(n), 0, bits, c.stream));
}
template <typename K>
static void radix_keys(Ctx& c, K* kin, K* kout, int64_t n, int bits) {
  size_t tb = 0;
  NBG_HIP(rocprim::radix_sort_keys(nullptr, tb, kin, kout, size_t(n), 0, bits, c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::radix_sort_keys(c.ws_tmp.p, tb, kin, kout, size_t(n), 0, bits, c.stream));
}
// unique of a sorted array; returns count
template <typename T>
static int64_t unique_sorted(Ctx& c, T* in, T* out, int64_t n) {
  DevBuf cnt;
  cnt.alloc(8);
  size_t tb = 0;
  NBG_HIP(rocprim::unique(nullptr, tb, in, out, cnt.as<uint64_t>(), size_t(n), rocprim::equal_to<T>(), c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::unique(c.ws_tmp.p, tb, in, out, cnt.as<uint64_t>(), size_t(n), rocprim::equal_to<T>(), c.stream));
  uint64_t h = 0;
  NBG_HIP(hipMemcpyAsync(&h, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  return int64_t(h);
}
template <typename T>
static void exclusive_scan(Ctx& c, const T* in, T* out, int64_t n) {
  size_t tb = 0;
  NBG_HIP(rocprim::exclusive_scan(nullptr, tb, in, out, T(0), size_t(n), rocprim::plus<T>(), c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::exclusive_scan(c.ws_tmp.p, tb, in, out, T(0), size_t(n), rocprim::plus<T>(), c.stream));
}

// key transform for signed int64 sort order: flip the sign bit
__global__ void k_flip_copy(const int64_t* in, uint64_t* out, int64_t n, int world, int parts, int rank,
                            int filter_owner) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int64_t v = in[i];
    out[i] = uint64_t(v) ^ (1ull << 63);
  }
}
__global__ void k_unflip(const uint64_t* in, int64_t* out, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = int64_t(in[i] ^ (1ull << 63));
}

__global__ void k_ht_insert(int64_t* keys, int32_t* vals, uint64_t mask, const int64_t* vids, int64_t n,
                            int64_t gbase, int32_t* min_gidx) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int64_t v = vids[i];
    if (v == INT64_MIN) {
      *min_gidx = int32_t(gbase + i);
      continue;
    }
    uint64_t h = ht_hash(v) & mask;
    while (true) {
      unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(keys + h),
                                          (unsigned long long)INT64_MIN, (unsigned long long)v);
      if (prev == (unsigned long long)INT64_MIN || int64_t(prev) == v) {
        vals[h] = int32_t(gbase + i);
        break;
      }
      h = (h + 1) & mask;
    }
  }
}
__global__ void k_ht_lookup(const int64_t* keys, const int32_t* vals, uint64_t mask, bool has_min,
                            int32_t min_gidx, const int64_t* vids, int32_t* out, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = ht_lookup(keys, vals, mask, vids[i], has_min, min_gidx);
}

void lookup_gidx(Ctx& c, const int64_t* d_vids, int32_t* d_gidx, int64_t n) {
  if (n <= 0) return;
  k_ht_lookup<<<grid_for(n), 256, 0, c.stream>>>(c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(),
                                                uint64_t(c.ht_cap - 1), c.ht_has_min, c.ht_min_gidx,
                                                d_vids, d_gidx, n);
  NBG_HIP(hipGetLastError());
}

// bytewise order rank of every vertex: position of gidx in the order of bswap(vid)
__global__ void k_bswap_keys(const int64_t* vid_of, uint64_t* keys, uint32_t* idx, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    keys[i] = bswap64(uint64_t(vid_of[i]));
    idx[i] = uint32_t(i);
  }
}
__global__ void k_scatter_rank(const uint32_t* sorted_idx, uint32_t* byterank, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    byterank[sorted_idx[i]] = uint32_t(i);
}

// edge sort key (single-pass case): (src_local << 32) | byterank(dst)
__global__ void k_edge_keys(const int64_t* src, const int64_t* dst, int64_t n, const int64_t* keys_ht,
                            const int32_t* vals_ht, uint64_t mask, bool has_min, int32_t min_gidx,
                            int64_t lo, int64_t hi, const uint32_t* byterank, uint64_t* keys,
                            uint32_t* perm, int32_t* dst_g, unsigned long long* err) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int32_t sg = ht_lookup(keys_ht, vals_ht, mask, src[i], has_min, min_gidx);
    int32_t dg = ht_lookup(keys_ht, vals_ht, mask, dst[i], has_min, min_gidx);
    if (sg < lo || sg >= hi || dg < 0) {
      atomicAdd(err, 1ull);
      sg = int32_t(lo);
      dg = 0;
    }
    keys[i] = (uint64_t(uint32_t(sg - lo)) << 32) | uint64_t(byterank[dg]);
    perm[i] = uint32_t(i);
    dst_g[i] = dg;
  }
}
__global__ void k_seq_desc_keys(const int64_t* seq, int64_t n, uint64_t* keys) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    keys[i] = ~uint64_t(seq[i]);
}
// multi-pass LSD helpers: gather a 64-bit key through the current permutation
__global__ void k_gather_key_bswap(const int64_t* vals, const uint32_t* perm, uint64_t* keys, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    keys[i] = bswap64(uint64_t(vals[perm[i]]));
}
__global__ void k_gather_key_src(const uint64_t* srckey, const uint32_t* perm, uint64_t* keys, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    keys[i] = srckey[perm[i]] >> 32;
}

// keep-first flags in sorted order: (src, rank, dst) differs from predecessor
__global__ void k_dedup_flags(const uint64_t* skey, const uint32_t* perm, const int64_t* rank,
                              const int32_t* dst_g, int64_t n, uint8_t* keep) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    bool k = true;
    if (i > 0) {
      uint32_t a = perm[i - 1], b = perm[i];
      bool same = (skey[a] >> 32) == (skey[b] >> 32) && dst_g[a] == dst_g[b] &&
                  (rank == nullptr || rank[a] == rank[b]);
      k = !same;
    }
    keep[i] = k;
  }
}

// row_ptr from row keys sorted ascending (no atomics): row_ptr[v] = first i with key[i] >= v
// row_ptr[0, n] from the sorted row keys of m entries: entry i (i = m: the end) opens the rows
// (keys[i - 1], keys[i]].  A run of more than kRowRun rows (rows without entries: with the
// class-ordered numbering the in-only class of an out CSR is one run of millions) goes to a list
// filled by k_rowptr_runs, one block per run -- one thread storing it row by row took 10 ms at
// RMAT-22 and most of a merge commit at RMAT-26.
constexpr int64_t kRowRun = 64;
__global__ void k_rowptr_sorted(const uint32_t* keys, int64_t m, int64_t n, int64_t* row_ptr, int64_t* runs,
                                unsigned long long* nruns, int64_t cap) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t prev = i == 0 ? -1 : int64_t(keys[i - 1]);
    const int64_t cur = i == m ? n : int64_t(keys[i]);
    if (cur - prev > kRowRun) {
      const unsigned long long slot = atomicAdd(nruns, 1ull);
      if (int64_t(slot) < cap) {
        runs[3 * slot] = prev + 1, runs[3 * slot + 1] = cur, runs[3 * slot + 2] = i;
        continue;
      }
    }
    for (int64_t v = prev + 1; v <= cur; v++) row_ptr[v] = i;
  }
}
__global__ void k_rowptr_runs(const int64_t* runs, const unsigned long long* nruns, int64_t cap, int64_t* row_ptr) {
  const int64_t nr = int64_t(*nruns) < cap ? int64_t(*nruns) : cap;
  for (int64_t r = blockIdx.x; r < nr; r += gridDim.x) {
    const int64_t a = runs[3 * r], b = runs[3 * r + 1], val = runs[3 * r + 2];
    for (int64_t v = a + threadIdx.x; v <= b; v += blockDim.x) row_ptr[v] = val;
  }
}
static void rowptr_from_sorted(Ctx& c, const uint32_t* keys, int64_t m, int64_t n, int64_t* row_ptr) {
  // every listed run holds more than kRowRun of the n + 1 rows
  const int64_t cap = (n + 1) / kRowRun + 1;
  DevBuf runs, cnt;
  runs.alloc(size_t(cap) * 24);
  cnt.alloc(8);
  NBG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  k_rowptr_sorted<<<grid_for(m + 1), 256, 0, c.stream>>>(keys, m, n, row_ptr, runs.as<int64_t>(),
                                                        cnt.as<unsigned long long>(), cap);
  k_rowptr_runs<<<1024, 256, 0, c.stream>>>(runs.as<int64_t>(), cnt.as<unsigned long long>(), cap, row_ptr);
  NBG_HIP(hipGetLastError());
}
__global__ void k_kept_src(const uint64_t* skey, const uint32_t* kept, int64_t m, uint32_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = uint32_t(skey[kept[i]] >> 32);
}
__global__ void k_row_part_default(const int64_t* vid_of_lo, int64_t n, int32_t parts, int32_t* row_part) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    row_part[i] = dev_part_of(vid_of_lo[i], parts);
}
__global__ void k_row_part_scatter(const uint64_t* skey, const uint32_t* kept_perm, int64_t m, const int32_t* part,
                                   int32_t* row_part) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    uint32_t t = kept_perm[i];
    row_part[skey[t] >> 32] = part[t];
  }
}
__global__ void k_row_ok(const int64_t* vid_of_lo, int64_t n, int32_t parts, const int32_t* row_part, uint8_t* ok,
                         unsigned long long* bad) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    bool g = row_part[i] == dev_part_of(vid_of_lo[i], parts);
    ok[i] = g;
    if (!g) atomicAdd(bad, 1ull);
  }
}
__global__ void k_row_counts(const uint64_t* skey, const uint32_t* kept_perm, int64_t m, int64_t* counts) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    atomicAdd(reinterpret_cast<unsigned long long*>(counts + (skey[kept_perm[i]] >> 32)), 1ull);
}
__global__ void k_gather_i32(const int32_t* in, const uint32_t* perm, int32_t* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = in[perm[i]];
}
__global__ void k_gather_i64(const int64_t* in, const uint32_t* perm, int64_t* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = in[perm[i]];
}
__global__ void k_gather_u8(const uint8_t* in, const uint32_t* perm, uint8_t* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = in[perm[i]];
}
__global__ void k_col_vid(const int32_t* col, const int64_t* vid_of, int64_t m, int64_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = vid_of[col[i]];
}
template <typename T>
__global__ void k_narrow(const int64_t* in, T* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = T(in[i]);
}
__global__ void k_str_lengths(const int64_t* lens, const uint8_t* present, int64_t m, int64_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = (present == nullptr || present[i]) ? lens[i] : 0;
}
__global__ void k_str_copy(const uint8_t* heap, const int64_t* offs_src, const int64_t* dst_off, int64_t m,
                           uint8_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    int64_t len = dst_off[i + 1] - dst_off[i];
    const uint8_t* s = heap + offs_src[i];
    uint8_t* d = out + dst_off[i];
    for (int64_t j = 0; j < len; j++) d[j] = s[j];
  }
}

static void minmax_i64(Ctx& c, const int64_t* d, int64_t n, int64_t& mn, int64_t& mx) {
  DevBuf r;
  r.alloc(16);
  size_t tb = 0;
  NBG_HIP(rocprim::reduce(nullptr, tb, d, r.as<int64_t>(), INT64_MAX, size_t(n), rocprim::minimum<int64_t>(), c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::reduce(c.ws_tmp.p, tb, d, r.as<int64_t>(), INT64_MAX, size_t(n), rocprim::minimum<int64_t>(), c.stream));
  tb = 0;
  NBG_HIP(rocprim::reduce(nullptr, tb, d, r.as<int64_t>() + 1, INT64_MIN, size_t(n), rocprim::maximum<int64_t>(), c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::reduce(c.ws_tmp.p, tb, d, r.as<int64_t>() + 1, INT64_MIN, size_t(n), rocprim::maximum<int64_t>(), c.stream));
  int64_t h[2];
  NBG_HIP(hipMemcpyAsync(h, r.p, 16, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  mn = h[0];
  mx = h[1];
}

// older-version flags over the sorted tuples: not kept (a later version of a kept group) and
// not an overwritten identical key (same version as its predecessor: WriteBatch last write wins
// puts the visible write first).  escan[i] = keep[i] (inclusive-scanned by the caller -> the
// group's edge index + 1).
__global__ void k_old_version_flags(const uint32_t* perm, const uint8_t* keep, const int64_t* ver, int64_t n,
                                    uint8_t* ov, uint32_t* escan, unsigned long long* count) {
  unsigned long long c = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    escan[i] = keep[i];
    const bool o = !keep[i] && i > 0 && ver[perm[i]] != ver[perm[i - 1]];
    ov[i] = o;
    c += o;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, c);
}
// the older versions' group edge indices: inclusive keep-scan - 1, widened
__global__ void k_ov_edges(const uint32_t* e, int64_t n, int64_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = int64_t(e[i]) - 1;
}
// SoA prop columns of the staged tuples kp[0..m) (in that order): INT-like values narrowed to
// the smallest width holding [min, max] when `narrow`, DOUBLE as bits, STRING as offsets + bytes
static void gather_props(Ctx& c, Staging& s, const std::vector<Field>& fields, const uint32_t* kp, int64_t m,
                         bool narrow, std::vector<PropCol>& props_out) {
  DevBuf tmp;
  tmp.alloc(size_t(m) * 8 + 8);
  for (size_t f = 0; f < fields.size(); f++) {
    PropCol pc;
    pc.name = fields[f].name;
    pc.type = fields[f].type;
    k_gather_i64<<<grid_for(m), 256, 0, c.stream>>>(s.props[f].as<int64_t>(), kp, tmp.as<int64_t>(), m);
    bool has_present = f < s.present.size() && s.present[f].p != nullptr;
    if (has_present) {
      pc.present.alloc(size_t(m) + 1);
      k_gather_u8<<<grid_for(m), 256, 0, c.stream>>>(s.present[f].as<uint8_t>(), kp, pc.present.as<uint8_t>(), m);
    }
    if (pc.type == NBG_T_STRING) {
      DevBuf lens, offs_src;
      lens.alloc(size_t(m) * 8 + 8);
      offs_src.alloc(size_t(m) * 8 + 8);
      k_gather_i64<<<grid_for(m), 256, 0, c.stream>>>(s.str_len[f].as<int64_t>(), kp, lens.as<int64_t>(), m);
      NBG_HIP(hipMemcpyAsync(offs_src.p, tmp.p, size_t(m) * 8, hipMemcpyDeviceToDevice, c.stream));
      DevBuf l2;
      l2.alloc(size_t(m + 1) * 8);
      k_str_lengths<<<grid_for(m), 256, 0, c.stream>>>(lens.as<int64_t>(),
                                                             has_present ? pc.present.as<uint8_t>() : nullptr,
                                                             m, l2.as<int64_t>());
      NBG_HIP(hipMemsetAsync(l2.as<int64_t>() + m, 0, 8, c.stream));
      pc.str_off.alloc(size_t(m + 1) * 8);
      exclusive_scan<int64_t>(c, l2.as<int64_t>(), pc.str_off.as<int64_t>(), m + 1);
      int64_t total = 0;
      NBG_HIP(hipMemcpyAsync(&total, pc.str_off.as<int64_t>() + m, 8, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
      pc.str_bytes.alloc(size_t(total) + 8);
      k_str_copy<<<grid_for(m), 256, 0, c.stream>>>(c.heap.as<uint8_t>(), offs_src.as<int64_t>(),
                                                           pc.str_off.as<int64_t>(), m, pc.str_bytes.as<uint8_t>());
      pc.width = 0;
    } else if (pc.type == NBG_T_DOUBLE || pc.type == NBG_T_FLOAT) {
      pc.width = 8;
      pc.data.alloc(size_t(m) * 8 + 8);
      NBG_HIP(hipMemcpyAsync(pc.data.p, tmp.p, size_t(m) * 8, hipMemcpyDeviceToDevice, c.stream));
    } else {
      // INT / VID / TIMESTAMP / BOOL: narrow to the smallest width holding [min, max]
      int64_t mn = 0, mx = 0;
      if (m) minmax_i64(c, tmp.as<int64_t>(), m, mn, mx);
      pc.minv = mn;
      pc.maxv = mx;
      int w = 8;
      if (mn >= INT8_MIN && mx <= INT8_MAX) w = 1;
      else if (mn >= INT16_MIN && mx <= INT16_MAX) w = 2;
      else if (mn >= INT32_MIN && mx <= INT32_MAX) w = 4;
      if (!narrow) w = 8;
      pc.width = w;
      pc.data.alloc(size_t(m) * size_t(w) + 16);
      int g = grid_for(m);
      switch (w) {
        case 1: k_narrow<int8_t><<<g, 256, 0, c.stream>>>(tmp.as<int64_t>(), pc.data.as<int8_t>(), m); break;
        case 2: k_narrow<int16_t><<<g, 256, 0, c.stream>>>(tmp.as<int64_t>(), pc.data.as<int16_t>(), m); break;
        case 4: k_narrow<int32_t><<<g, 256, 0, c.stream>>>(tmp.as<int64_t>(), pc.data.as<int32_t>(), m); break;
        default: NBG_HIP(hipMemcpyAsync(pc.data.p, tmp.p, size_t(m) * 8, hipMemcpyDeviceToDevice, c.stream));
      }
    }
    props_out.push_back(std::move(pc));
  }
}

// Builds one CSR from a staging area.  Returns after freeing the staging buffers.
// (src, rank bytes, dst bytes, version bytes) order of two tuples: the merge commit's key (the
// sort's last key, load sequence descending, is implied: a batch is newer than every committed
// tuple and the merge puts it first among equals)
struct GroupLess {
  const uint64_t* skey;
  const int64_t* rank;  // null: constant
  const int64_t* ver;   // null: constant
  __device__ bool operator()(uint32_t a, uint32_t b) const {
    const uint64_t ka = skey[a], kb = skey[b];
    if ((ka >> 32) != (kb >> 32)) return (ka >> 32) < (kb >> 32);
    if (rank) {
      const uint64_t ra = bswap64(uint64_t(rank[a])), rb = bswap64(uint64_t(rank[b]));
      if (ra != rb) return ra < rb;
    }
    if (uint32_t(ka) != uint32_t(kb)) return uint32_t(ka) < uint32_t(kb);
    if (ver) {
      const uint64_t va = bswap64(uint64_t(ver[a])), vb = bswap64(uint64_t(ver[b]));
      if (va != vb) return va < vb;
    }
    return false;
  }
};
__global__ void k_iota_off_u32(uint32_t* p, int64_t n, int64_t off) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    p[i] = uint32_t(off + i);
}

static void build_csr(Ctx& c, Staging& s, const std::vector<Field>& fields, bool with_props, Csr& out,
                      const uint32_t* byterank, bool consume = true, EdgeSpace::Order* ord = nullptr,
                      bool merge = false) {
  out = Csr();  // a commit retried after a failed build must not extend a half-built CSR
  int64_t n = s.n;
  int64_t lo = c.owned_lo(), hi = c.owned_hi();
  out.n_rows = hi - lo;
  out.row_ptr.alloc(size_t(out.n_rows + 1) * 8);
  if (n == 0) {
    NBG_HIP(hipMemsetAsync(out.row_ptr.p, 0, size_t(out.n_rows + 1) * 8, c.stream));
    out.nnz = 0;
    for (auto& f : fields)
      if (with_props) {
        PropCol pc;
        pc.name = f.name;
        pc.type = f.type;
        out.props.push_back(std::move(pc));
      }
    return;
  }
  if (n >= (int64_t(1) << 32)) throw Error(NBG_E_UNSUPPORTED, "more than 2^32 edges on one rank");
  int srcbits = 1;
  while ((int64_t(1) << srcbits) < std::max<int64_t>(out.n_rows, 2)) srcbits++;
  DevBuf keyA, keyB, permA, permB, permM, dstg, err;
  err.alloc(8);
  NBG_HIP(hipMemsetAsync(err.p, 0, 8, c.stream));
  uint32_t* perm = nullptr;
  DevBuf* perm_owner = nullptr;
  DevBuf& skey_keep = keyA;  // (src_local << 32 | byterank(dst)) by tuple index
  // LSD passes over the tuples listed in pin (m of them, global tuple indices, already ordered by
  // load sequence descending): version bytes, dst bytes, rank bytes, then src; returns the buffer
  // holding the result (pin or pout)
  auto lsd = [&](uint32_t* pin, uint32_t* pout, int64_t m) -> uint32_t* {
    DevBuf keyC;
    keyC.alloc(size_t(m) * 8);
    auto pass_bswap = [&](const DevBuf& vals) {
      k_gather_key_bswap<<<grid_for(m), 256, 0, c.stream>>>(vals.as<int64_t>(), pin, keyC.as<uint64_t>(), m);
      radix_pairs<uint64_t, uint32_t>(c, keyC.as<uint64_t>(), keyB.as<uint64_t>(), pin, pout, m, 64);
      std::swap(pin, pout);
    };
    if (!s.ver_const) pass_bswap(s.ver);
    pass_bswap(s.dst);
    if (!s.rank_const) pass_bswap(s.rank);
    k_gather_key_src<<<grid_for(m), 256, 0, c.stream>>>(skey_keep.as<uint64_t>(), pin, keyC.as<uint64_t>(), m);
    radix_pairs<uint64_t, uint32_t>(c, keyC.as<uint64_t>(), keyB.as<uint64_t>(), pin, pout, m, srcbits);
    return pout;
  };
  const int64_t n0 = ord ? ord->n : 0;
  const bool do_merge = merge && ord && n0 > 0 && n0 < n && ord->perm.p && s.seq.bytes >= size_t(n) * 8;
  if (do_merge) {
    // merge commit: keys of the batch [n0, n) only, the batch sorted on its own (LSD, load
    // sequence descending first), then merged into the committed order -- the batch first among
    // equal groups (it is newer), which is the full sort's order
    const int64_t mb = n - n0;
    // the committed keys grow in place when their (pool-rounded) block has room for the batch
    auto grow = [&](DevBuf& dst, DevBuf& old, size_t w) {
      if (old.bytes >= size_t(n) * w) {
        dst = std::move(old);
      } else {
        dst.alloc(size_t(n) * w);
        NBG_HIP(hipMemcpyAsync(dst.p, old.p, size_t(n0) * w, hipMemcpyDeviceToDevice, c.stream));
      }
    };
    grow(keyA, ord->skey, 8);
    grow(dstg, ord->dstg, 4);
    keyB.alloc(size_t(mb) * 8);
    permA.alloc(size_t(mb) * 4);
    permB.alloc(size_t(mb) * 4);
    k_edge_keys<<<grid_for(mb), 256, 0, c.stream>>>(
        s.src.as<int64_t>() + n0, s.dst.as<int64_t>() + n0, mb, c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(),
        uint64_t(c.ht_cap - 1), c.ht_has_min, c.ht_min_gidx, lo, hi, byterank, keyA.as<uint64_t>() + n0,
        permA.as<uint32_t>(), dstg.as<int32_t>() + n0, err.as<unsigned long long>());
    {
      DevBuf keyC;
      keyC.alloc(size_t(mb) * 8);
      k_iota_off_u32<<<grid_for(mb), 256, 0, c.stream>>>(permB.as<uint32_t>(), mb, n0);
      k_seq_desc_keys<<<grid_for(mb), 256, 0, c.stream>>>(s.seq.as<int64_t>() + n0, mb, keyC.as<uint64_t>());
      radix_pairs<uint64_t, uint32_t>(c, keyC.as<uint64_t>(), keyB.as<uint64_t>(), permB.as<uint32_t>(),
                                      permA.as<uint32_t>(), mb, 64);
    }
    uint32_t* batch = lsd(permA.as<uint32_t>(), permB.as<uint32_t>(), mb);
    permM.alloc(size_t(n) * 4);
    const GroupLess less{keyA.as<uint64_t>(), s.rank_const ? nullptr : s.rank.as<int64_t>(),
                         s.ver_const ? nullptr : s.ver.as<int64_t>()};
    size_t tb = 0;
    NBG_HIP(rocprim::merge(nullptr, tb, batch, ord->perm.as<uint32_t>(), permM.as<uint32_t>(), size_t(mb), size_t(n0),
                           less, c.stream));
    c.ws_tmp.ensure(tb);
    NBG_HIP(rocprim::merge(c.ws_tmp.p, tb, batch, ord->perm.as<uint32_t>(), permM.as<uint32_t>(), size_t(mb),
                           size_t(n0), less, c.stream));
    perm = permM.as<uint32_t>();
    perm_owner = &permM;
    ord->perm.release();
    ord->skey.release();
    ord->dstg.release();
  } else {
    keyA.alloc(size_t(n) * 8);
    keyB.alloc(size_t(n) * 8);
    permA.alloc(size_t(n) * 4);
    permB.alloc(size_t(n) * 4);
    dstg.alloc(size_t(n) * 4);
    k_edge_keys<<<grid_for(n), 256, 0, c.stream>>>(s.src.as<int64_t>(), s.dst.as<int64_t>(), n, c.ht_keys.as<int64_t>(),
                                                 c.ht_vals.as<int32_t>(), uint64_t(c.ht_cap - 1), c.ht_has_min,
                                                 c.ht_min_gidx, lo, hi, byterank, keyA.as<uint64_t>(),
                                                 permA.as<uint32_t>(), dstg.as<int32_t>(), err.as<unsigned long long>());
  }
  NBG_HIP(hipGetLastError());
  uint64_t herr = 0;
  NBG_HIP(hipMemcpyAsync(&herr, err.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  if (herr) throw Error(NBG_E_PART_NOT_FOUND, "edge source not owned by this rank / unknown vertex");
  if (do_merge) {
  } else if (s.rank_const && s.ver_const) {
    // single pass on (src_local, byterank(dst)) == the reference key order
    radix_pairs<uint64_t, uint32_t>(c, skey_keep.as<uint64_t>(), keyB.as<uint64_t>(), permA.as<uint32_t>(),
                                   permB.as<uint32_t>(), n, 32 + srcbits);
    perm = permB.as<uint32_t>();
    perm_owner = &permB;
  } else {
    uint32_t* pin = permA.as<uint32_t>();
    // start from reverse load order: stable passes then put the LAST write of identical keys
    // first, so keep-first implements WriteBatch last-write-wins (RocksEngine.cpp:216-230).
    // The decode stage appends tuples in wave order, not load order, so the start permutation
    // is the staged load sequence numbers sorted descending.
    if (s.seq.bytes >= size_t(n) * 8) {
      DevBuf keyC;
      keyC.alloc(size_t(n) * 8);
      k_iota_u32<<<grid_for(n), 256, 0, c.stream>>>(permB.as<uint32_t>(), n);
      k_seq_desc_keys<<<grid_for(n), 256, 0, c.stream>>>(s.seq.as<int64_t>(), n, keyC.as<uint64_t>());
      radix_pairs<uint64_t, uint32_t>(c, keyC.as<uint64_t>(), keyB.as<uint64_t>(), permB.as<uint32_t>(), pin, n, 64);
    } else {
      k_iota_rev_u32<<<grid_for(n), 256, 0, c.stream>>>(pin, n);
    }
    perm = lsd(pin, permB.as<uint32_t>(), n);
    perm_owner = perm == permA.as<uint32_t>() ? &permA : &permB;
  }
  // dedup (keep the first = bytewise-smallest version)
  DevBuf keep;
  keep.alloc(size_t(n));
  const int64_t* rank_ptr = s.rank_const ? nullptr : s.rank.as<int64_t>();
  k_dedup_flags<<<grid_for(n), 256, 0, c.stream>>>(skey_keep.as<uint64_t>(), perm, rank_ptr, dstg.as<int32_t>(), n,
                                                 keep.as<uint8_t>());
  DevBuf kept, cnt;
  kept.alloc(size_t(n) * 4);
  cnt.alloc(8);
  size_t tb = 0;
  NBG_HIP(rocprim::select(nullptr, tb, perm, keep.as<uint8_t>(), kept.as<uint32_t>(), cnt.as<uint64_t>(), size_t(n), c.stream));
  c.ws_tmp.ensure(tb);
  NBG_HIP(rocprim::select(c.ws_tmp.p, tb, perm, keep.as<uint8_t>(), kept.as<uint32_t>(), cnt.as<uint64_t>(), size_t(n), c.stream));
  uint64_t m = 0;
  NBG_HIP(hipMemcpyAsync(&m, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  // older versions (multi-version data): tuples that are neither kept nor an overwritten
  // identical key, with the edge index of their group (the firstLoop side table, Csr::ov_*)
  out.ov_n = 0;
  out.ov_edge.release();
  out.ov_props.clear();
  DevBuf ovp;
  if (with_props && !s.ver_const && int64_t(m) < n) {
    DevBuf ovf, escan, ove, ocnt;
    ovf.alloc(size_t(n));
    escan.alloc(size_t(n) * 4);
    ocnt.alloc(8);
    NBG_HIP(hipMemsetAsync(ocnt.p, 0, 8, c.stream));
    k_old_version_flags<<<grid_for(n), 256, 0, c.stream>>>(perm, keep.as<uint8_t>(), s.ver.as<int64_t>(), n,
                                                           ovf.as<uint8_t>(), escan.as<uint32_t>(),
                                                           ocnt.as<unsigned long long>());
    uint64_t no = 0;
    NBG_HIP(hipMemcpyAsync(&no, ocnt.p, 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (no) {  // buffers sized by the older-version count (kept edges < 2^32: 32-bit scan)
      size_t tb2 = 0;
      NBG_HIP(rocprim::inclusive_scan(nullptr, tb2, escan.as<uint32_t>(), escan.as<uint32_t>(), size_t(n),
                                      rocprim::plus<uint32_t>(), c.stream));
      c.ws_tmp.ensure(tb2);
      NBG_HIP(rocprim::inclusive_scan(c.ws_tmp.p, tb2, escan.as<uint32_t>(), escan.as<uint32_t>(), size_t(n),
                                      rocprim::plus<uint32_t>(), c.stream));
      ovp.alloc(size_t(no) * 4 + 4);
      ove.alloc(size_t(no) * 4 + 4);
      tb2 = 0;
      NBG_HIP(rocprim::select(nullptr, tb2, perm, ovf.as<uint8_t>(), ovp.as<uint32_t>(), ocnt.as<uint64_t>(), size_t(n),
                              c.stream));
      c.ws_tmp.ensure(tb2);
      NBG_HIP(rocprim::select(c.ws_tmp.p, tb2, perm, ovf.as<uint8_t>(), ovp.as<uint32_t>(), ocnt.as<uint64_t>(),
                              size_t(n), c.stream));
      tb2 = 0;
      NBG_HIP(rocprim::select(nullptr, tb2, escan.as<uint32_t>(), ovf.as<uint8_t>(), ove.as<uint32_t>(),
                              ocnt.as<uint64_t>(), size_t(n), c.stream));
      c.ws_tmp.ensure(tb2);
      NBG_HIP(rocprim::select(c.ws_tmp.p, tb2, escan.as<uint32_t>(), ovf.as<uint8_t>(), ove.as<uint32_t>(),
                              ocnt.as<uint64_t>(), size_t(n), c.stream));
      out.ov_n = int64_t(no);
      out.ov_edge.alloc(size_t(no) * 8 + 8);
      k_ov_edges<<<grid_for(int64_t(no)), 256, 0, c.stream>>>(ove.as<uint32_t>(), int64_t(no), out.ov_edge.as<int64_t>());
    }
  }
  keyB.release();
  if (perm_owner != &permA) permA.release();
  if (perm_owner != &permB) permB.release();
  keep.release();
  out.nnz = int64_t(m);
  const uint32_t* kp = kept.as<uint32_t>();
  // row_ptr (kept edges are sorted by src)
  {
    DevBuf ks;
    ks.alloc(size_t(m + 1) * 4);
    k_kept_src<<<grid_for(int64_t(m)), 256, 0, c.stream>>>(skey_keep.as<uint64_t>(), kp, int64_t(m), ks.as<uint32_t>());
    rowptr_from_sorted(c, ks.as<uint32_t>(), int64_t(m), out.n_rows, out.row_ptr.as<int64_t>());
    NBG_HIP(hipStreamSynchronize(c.stream));
  }
  // row_part: hash rule by default, the key's part where the staging recorded it
  out.row_part.alloc(size_t(out.n_rows + 1) * 4);
  k_row_part_default<<<grid_for(out.n_rows), 256, 0, c.stream>>>(c.vid_of.as<int64_t>() + lo, out.n_rows,
                                                               c.num_parts, out.row_part.as<int32_t>());
  if (s.part.p) {
    DevBuf bad;
    bad.alloc(8);
    NBG_HIP(hipMemsetAsync(bad.p, 0, 8, c.stream));
    k_row_part_scatter<<<grid_for(int64_t(m)), 256, 0, c.stream>>>(skey_keep.as<uint64_t>(), kp, int64_t(m),
                                                                   s.part.as<int32_t>(), out.row_part.as<int32_t>());
    out.row_ok.alloc(size_t(out.n_rows + 1));
    k_row_ok<<<grid_for(out.n_rows), 256, 0, c.stream>>>(c.vid_of.as<int64_t>() + lo, out.n_rows, c.num_parts,
                                                         out.row_part.as<int32_t>(), out.row_ok.as<uint8_t>(),
                                                         bad.as<unsigned long long>());
    uint64_t hb = 0;
    NBG_HIP(hipMemcpyAsync(&hb, bad.p, 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (hb == 0) out.row_ok.release();
  }
  // col
  out.col.alloc(size_t(m) * 4 + 64);  // padded: aligned 16-byte loads past the last entry
  k_gather_i32<<<grid_for(int64_t(m)), 256, 0, c.stream>>>(dstg.as<int32_t>(), kp, out.col.as<int32_t>(), int64_t(m));
  // the out CSR's dst vids as a column of their own: a plain GO's rows (YIELD _dst) stream it
  // instead of gathering vid_of[col[e]] (one random line per row)
  if (with_props && c.opt("rows_vid_col", 1) && m) {
    out.col_vid.alloc(size_t(m) * 8 + 8);
    k_col_vid<<<grid_for(int64_t(m)), 256, 0, c.stream>>>(out.col.as<int32_t>(), c.vid_of.as<int64_t>(), int64_t(m),
                                                        out.col_vid.as<int64_t>());
  }
  // rank
  if (!s.rank_const) {
    out.rank.alloc(size_t(m) * 8 + 8);
    k_gather_i64<<<grid_for(int64_t(m)), 256, 0, c.stream>>>(s.rank.as<int64_t>(), kp, out.rank.as<int64_t>(), int64_t(m));
    int64_t mn, mx;
    minmax_i64(c, out.rank.as<int64_t>(), int64_t(m), mn, mx);
    if (mn == 0 && mx == 0) out.rank.release();
  } else if (s.rank_value != 0) {
    out.rank.alloc(size_t(m) * 8 + 8);
    fill<int64_t>(c, out.rank.as<int64_t>(), s.rank_value, int64_t(m));
  }
  // props
  if (with_props) gather_props(c, s, fields, kp, int64_t(m), true, out.props);
  // older versions of multi-version groups (firstLoop side table, selected above)
  if (out.ov_n) gather_props(c, s, fields, ovp.as<uint32_t>(), out.ov_n, false, out.ov_props);
  NBG_HIP(hipStreamSynchronize(c.stream));
  NBG_HIP(hipGetLastError());
  // the sorted order for a later merge commit (writable snapshots only)
  if (ord) {
    ord->perm.release();
    ord->skey.release();
    ord->dstg.release();
    ord->n = 0;
    if (!consume && perm_owner) {
      ord->perm = std::move(*perm_owner);
      ord->skey = std::move(keyA);
      ord->dstg = std::move(dstg);
      ord->n = n;
    }
  }
  // free staging
  if (consume) {  // a writable snapshot keeps its decoded tuples (the write log) for the next commit
    s.src.release();
    s.dst.release();
    s.rank.release();
    s.ver.release();
    s.part.release();
    s.props.clear();
    s.present.clear();
    s.str_len.clear();
    s.n = 0;
    s.cap = 0;
  }
}

__global__ void k_edge_src(const int64_t* row_ptr, int64_t n_rows, int32_t* esrc) {
  for (int64_t r = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; r < n_rows; r += int64_t(gridDim.x) * blockDim.x)
    for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) esrc[e] = int32_t(r);
}
__global__ void k_tr_col(const uint32_t* t_eid, const int32_t* esrc, int64_t m, int64_t lo, int32_t* tcol) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    tcol[i] = int32_t(lo) + esrc[t_eid[i]];
}
template <typename T>
__global__ void k_gather_w(const T* in, const uint32_t* perm, T* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = in[perm[i]];
}

__global__ void k_sorted_bounds(const uint32_t* keys, int64_t m, const int64_t* bounds, int nb, int64_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  int64_t lo = 0, hi = m, x = bounds[i];  // first index with key >= x
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (int64_t(keys[mid]) < x) lo = mid + 1; else hi = mid;
  }
  out[i] = lo;
}
__global__ void k_src_global(const uint32_t* perm, const int32_t* esrc, int64_t m, int64_t lo, int32_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = int32_t(lo) + esrc[perm[i]];
}
__global__ void k_sub_lo(const int32_t* in, int64_t m, int64_t lo, uint32_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = uint32_t(in[i] - lo);
}
static void gather_width(Ctx& c, const void* in, const uint32_t* perm, void* out, int64_t m, int w) {
  int g = grid_for(m);
  switch (w) {
    case 1: k_gather_w<int8_t><<<g, 256, 0, c.stream>>>(static_cast<const int8_t*>(in), perm, static_cast<int8_t*>(out), m); break;
    case 2: k_gather_w<int16_t><<<g, 256, 0, c.stream>>>(static_cast<const int16_t*>(in), perm, static_cast<int16_t*>(out), m); break;
    case 4: k_gather_w<int32_t><<<g, 256, 0, c.stream>>>(static_cast<const int32_t*>(in), perm, static_cast<int32_t*>(out), m); break;
    default: k_gather_w<int64_t><<<g, 256, 0, c.stream>>>(static_cast<const int64_t*>(in), perm, static_cast<int64_t*>(out), m);
  }
}
static bool copy_prop(const PropCol& p) {
  bool intlike = p.type == NBG_T_INT || p.type == NBG_T_VID || p.type == NBG_T_TIMESTAMP || p.type == NBG_T_BOOL;
  return intlike && !p.present.p;
}


// out[0] = 1 + the last row with an in-edge (transposed row), out[1] = 1 + the last row with
// an in-edge and an out-edge
__global__ void k_live_bounds(const int64_t* trp, const uint32_t* odeg, int64_t n, unsigned long long* out) {
  unsigned long long a = 0, b = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    if (trp[i + 1] > trp[i]) {
      a = (unsigned long long)(i + 1);
      if (odeg[i]) b = (unsigned long long)(i + 1);
    }
  for (int o = 32; o > 0; o >>= 1) {
    a = max(a, (unsigned long long)__shfl_xor((long long)a, o));
    b = max(b, (unsigned long long)__shfl_xor((long long)b, o));
  }
  if ((threadIdx.x & 63) == 0) {
    if (a) atomicMax(out, a);
    if (b) atomicMax(out + 1, b);
  }
}
__global__ void k_odeg8(const uint32_t* deg, int64_t n, uint8_t* d8) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    d8[i] = uint8_t(min(deg[i], 255u));
}
__global__ void k_out_deg(const int64_t* row_ptr, const uint8_t* row_ok, int64_t n, uint32_t* deg,
                          unsigned int* maxd) {
  unsigned int m = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    uint32_t d = uint32_t(row_ptr[i + 1] - row_ptr[i]);
    if (row_ok && !row_ok[i]) d = 0;
    deg[i] = d;
    m = d > m ? d : m;
  }
  if (maxd) atomicMax(maxd, m);
}
// hub-first key: sources with larger out-degree sort first inside a transposed row
__global__ void k_hub_key(const int32_t* tsrc, int64_t m, const uint32_t* gdeg, uint32_t maxd, uint32_t* key) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    key[i] = maxd - gdeg[tsrc[i]];
}
__global__ void k_gather_u32(const uint32_t* in, const uint32_t* perm, uint32_t* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = in[perm[i]];
}
// min / max of a narrowed INT column (width 1/2/4/8)
__global__ void k_minmax_w(const void* data, int w, int64_t m, long long* mm) {
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    long long v = w == 1 ? static_cast<const int8_t*>(data)[i]
                : w == 2 ? static_cast<const int16_t*>(data)[i]
                : w == 4 ? static_cast<const int32_t*>(data)[i]
                         : static_cast<const int64_t*>(data)[i];
    lo = v < lo ? v : lo;
    hi = v > hi ? v : hi;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const long long a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(mm, lo);
    atomicMax(mm + 1, hi);
  }
}
// the quantised bucket of v: floor((v - min) * 2^bits / range) (range 0 = 2^64)
__host__ __device__ inline uint32_t q_bucket(int64_t v, int64_t vmin, uint64_t range, int bits) {
  const unsigned __int128 d = (unsigned __int128)(uint64_t(v) - uint64_t(vmin)) << bits;
  const unsigned __int128 r = range ? (unsigned __int128)range : ((unsigned __int128)1 << 64);
  return uint32_t(d / r);
}
// packed transposed column: (bucket << gbits) | src gidx
__global__ void k_pack_col(const int32_t* col, const void* data, int w, int64_t m, int64_t vmin, uint64_t range,
                           int gbits, int qbits, int32_t* out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t v = w == 1 ? static_cast<const int8_t*>(data)[i]
                    : w == 2 ? static_cast<const int16_t*>(data)[i]
                    : w == 4 ? static_cast<const int32_t*>(data)[i]
                             : static_cast<const int64_t*>(data)[i];
    out[i] = int32_t((q_bucket(v, vmin, range, qbits) << gbits) | uint32_t(col[i]));
  }
}
// quad slab: row d's first 4 entries as two row-major halves (slots 0-1 in lo, 2-3 in hi)
template <typename T>
__global__ void k_build_pair(const int64_t* trp, const T* src, int64_t n, T* lo, T* hi, T none) {
  for (int64_t d = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; d < n; d += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = trp[d], e = trp[d + 1];
#pragma unroll
    for (int q = 0; q < 4; q++) (q < 2 ? lo : hi)[size_t(d) * 2 + (q & 1)] = b + q < e ? src[b + q] : none;
  }
}

// rest records (EdgeSpace::brec): row d's start and clamped in-degree, then its first
// kRecEntries entries of src, as one 64-byte line (four 16-byte stores)
__global__ void k_build_rec(const int64_t* trp, const int32_t* src, int64_t n, uint4* rec) {
  for (int64_t d = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; d < n; d += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = trp[d], e = trp[d + 1];
    const uint64_t deg = uint64_t(e - b) < 65535u ? uint64_t(e - b) : 65535u;
    uint32_t w[16];
    w[0] = uint32_t(uint64_t(b));
    w[1] = uint32_t(uint64_t(b) >> 32) | uint32_t(deg << 16);
#pragma unroll
    for (int k = 0; k < kRecEntries; k++) w[2 + k] = b + k < e ? uint32_t(src[b + k]) : 0xffffffffu;
#pragma unroll
    for (int j = 0; j < 4; j++) rec[size_t(d) * 4 + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
  }
}

// Transpose of the out CSR for bottom-up hops: rows = owned dst, entries = global src index,
// plus copies of the INT-like props in transpose order.  With several ranks every out-edge is
// shipped to the owner of its dst (one build-time all-to-all), so each rank can run bottom-up
// hops over its own vertices against the allgathered frontier bitmap.
//
// Inside a row the sources are ordered hub-first (descending out-degree): in a dense frontier
// the first in-neighbour checked is then almost always a frontier member, and the first K
// entries of every row are copied into a slot-major slab, so the common case of a bottom-up hop
// reads 4 coalesced bytes per row instead of one scattered cache line per row.
static void build_transpose(Ctx& c, EdgeSpace& es) {
  Csr& o = es.out;
  Csr& t = es.tr;
  const int64_t m = o.nnz;
  const int64_t lo = c.owned_lo(), hi = c.owned_hi();
  const int64_t n_own = hi - lo;
  const int G = c.world;
  auto nbits = [](int64_t x) {
    int b = 1;
    while ((int64_t(1) << b) < std::max<int64_t>(x, 2)) b++;
    return b;
  };
  // out-degrees (0 for rows outside hash(vid)'s part) of every vertex of the gidx space
  // padded to whole 128-row tiles (k_bu_lean loads two rows per lane without bounds checks)
  const int64_t n_pad = (n_own + 127) / 128 * 128;
  es.odeg.alloc(size_t(n_pad + 1) * 4);
  NBG_HIP(hipMemsetAsync(es.odeg.p, 0, size_t(n_pad + 1) * 4, c.stream));
  DevBuf gdeg, dmax;
  dmax.alloc(16);
  NBG_HIP(hipMemsetAsync(dmax.p, 0, 16, c.stream));
  k_out_deg<<<grid_for(n_own), 256, 0, c.stream>>>(o.row_ptr.as<int64_t>(), o.row_ok.as<uint8_t>(), n_own,
                                                  es.odeg.as<uint32_t>(), dmax.as<unsigned int>());
  es.odeg8.alloc(size_t(n_pad + 64));
  k_odeg8<<<grid_for(n_pad + 1), 256, 0, c.stream>>>(es.odeg.as<uint32_t>(), n_pad + 1, es.odeg8.as<uint8_t>());
  const uint32_t* gdegp = es.odeg.as<uint32_t>();
  if (G > 1) {
    gdeg.alloc(size_t(c.n_global + 1) * 4);
    std::vector<size_t> rb(static_cast<size_t>(G)), ro(static_cast<size_t>(G));
    for (int p = 0; p < G; p++) {
      rb[size_t(p)] = size_t(c.base[size_t(p) + 1] - c.base[size_t(p)]) * 4;
      ro[size_t(p)] = size_t(c.base[size_t(p)]) * 4;
    }
    comm_allgatherv_bytes(c, es.odeg.p, size_t(n_own) * 4, gdeg.p, rb.data(), ro.data());
    gdegp = gdeg.as<uint32_t>();
  }
  uint32_t maxd = 0;
  NBG_HIP(hipMemcpyAsync(&maxd, dmax.p, 4, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  es.max_odeg = int64_t(maxd);
  if (G > 1) maxd = UINT32_MAX;  // other ranks' degrees may exceed the local maximum
  // the transposed edge list: tdst (local row), tsrc (global), and the order props come in
  DevBuf tdst, tsrc;
  int64_t R = 0;
  std::vector<const PropCol*> cp;
  for (const PropCol& p : o.props) cp.push_back(copy_prop(p) ? &p : nullptr);
  std::vector<DevBuf> rprops(o.props.size());  // world > 1: received prop columns
  {
    DevBuf esrc;
    esrc.alloc(size_t(m + 1) * 4);
    if (m) k_edge_src<<<grid_for(o.n_rows), 256, 0, c.stream>>>(o.row_ptr.as<int64_t>(), o.n_rows, esrc.as<int32_t>());
    if (G == 1) {
      R = m;
      tsrc = std::move(esrc);  // lo == 0: local == global
      tdst.alloc(size_t(m + 1) * 4);
      if (m) NBG_HIP(hipMemcpyAsync(tdst.p, o.col.p, size_t(m) * 4, hipMemcpyDeviceToDevice, c.stream));
    } else {
      // ship every out-edge to its dst's owner: sort by dst gidx, cut at the owner bases
      DevBuf keysB, iota, perm;
      keysB.alloc(size_t(m + 1) * 4);
      iota.alloc(size_t(m + 1) * 4);
      perm.alloc(size_t(m + 1) * 4);
      if (m) {
        k_iota_u32<<<grid_for(m), 256, 0, c.stream>>>(iota.as<uint32_t>(), m);
        radix_pairs<uint32_t, uint32_t>(c, o.col.as<uint32_t>(), keysB.as<uint32_t>(), iota.as<uint32_t>(),
                                       perm.as<uint32_t>(), m, nbits(c.n_global));
      }
      iota.release();
      DevBuf dbase, dcut;
      dbase.alloc(size_t(G + 1) * 8);
      dcut.alloc(size_t(G + 1) * 8);
      NBG_HIP(hipMemcpyAsync(dbase.p, c.base.data(), size_t(G + 1) * 8, hipMemcpyHostToDevice, c.stream));
      k_sorted_bounds<<<1, 64, 0, c.stream>>>(keysB.as<uint32_t>(), m, dbase.as<int64_t>(), G + 1, dcut.as<int64_t>());
      std::vector<int64_t> cut(static_cast<size_t>(G + 1));
      NBG_HIP(hipMemcpyAsync(cut.data(), dcut.p, size_t(G + 1) * 8, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
      cut[size_t(G)] = m;
      DevBuf ssrc;
      ssrc.alloc(size_t(m + 1) * 4);
      if (m) k_src_global<<<grid_for(m), 256, 0, c.stream>>>(perm.as<uint32_t>(), esrc.as<int32_t>(), m, lo, ssrc.as<int32_t>());
      esrc.release();
      const size_t ng = static_cast<size_t>(G);
      std::vector<int64_t> mine(ng), all(ng * ng);
      for (size_t h = 0; h < ng; h++) mine[h] = cut[h + 1] - cut[h];
      {
        DevBuf dm, da;
        dm.alloc(ng * 8);
        da.alloc(ng * ng * 8);
        NBG_HIP(hipMemcpyAsync(dm.p, mine.data(), ng * 8, hipMemcpyHostToDevice, c.stream));
        comm_allgather_bytes(c, dm.p, ng * 8, da.p);
        NBG_HIP(hipMemcpyAsync(all.data(), da.p, ng * ng * 8, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipStreamSynchronize(c.stream));
      }
      std::vector<int64_t> roff(ng + 1, 0);
      for (size_t p = 0; p < ng; p++) roff[p + 1] = roff[p] + all[p * ng + size_t(c.rank)];
      R = roff[ng];
      auto exchange = [&](const void* send, void* recv, int w) {
        std::vector<size_t> sb(ng), so(ng), rb(ng), ro(ng);
        for (size_t p = 0; p < ng; p++) {
          sb[p] = size_t(mine[p]) * size_t(w);
          so[p] = size_t(cut[p]) * size_t(w);
          rb[p] = size_t(roff[p + 1] - roff[p]) * size_t(w);
          ro[p] = size_t(roff[p]) * size_t(w);
        }
        comm_alltoallv_bytes(c, send, sb.data(), so.data(), recv, rb.data(), ro.data());
      };
      DevBuf rdst;
      tsrc.alloc(size_t(R + 1) * 4);
      rdst.alloc(size_t(R + 1) * 4);
      exchange(ssrc.p, tsrc.p, 4);
      exchange(keysB.p, rdst.p, 4);
      tdst.alloc(size_t(R + 1) * 4);
      if (R) k_sub_lo<<<grid_for(R), 256, 0, c.stream>>>(rdst.as<int32_t>(), R, lo, tdst.as<uint32_t>());
      for (size_t f = 0; f < o.props.size(); f++) {
        if (!cp[f]) continue;
        int w = cp[f]->width;
        DevBuf sp;
        sp.alloc(size_t(m + 1) * size_t(w));
        rprops[f].alloc(size_t(R + 1) * size_t(w));
        if (m) gather_width(c, cp[f]->data.p, perm.as<uint32_t>(), sp.p, m, w);
        exchange(sp.p, rprops[f].p, w);
      }
      NBG_HIP(hipStreamSynchronize(c.stream));
    }
  }
  // order: stable sort by hub key, then stable sort by row -> rows hub-first
  t.n_rows = n_own;
  t.nnz = R;
  t.props.clear();
  for (const PropCol& p : o.props) {
    PropCol q;
    q.name = p.name;
    q.type = p.type;
    q.width = p.width;
    t.props.push_back(std::move(q));
  }
  t.row_ptr.alloc(size_t(t.n_rows + 1) * 8);
  t.col.alloc(size_t(R) * 4 + 64);  // padded: the rest passes load whole aligned 16-byte groups
  DevBuf perm;
  perm.alloc(size_t(R + 1) * 4);
  if (R) {
    DevBuf key, keyS, iota, perm1;
    key.alloc(size_t(R) * 4);
    keyS.alloc(size_t(R) * 4);
    iota.alloc(size_t(R) * 4);
    perm1.alloc(size_t(R) * 4);
    k_hub_key<<<grid_for(R), 256, 0, c.stream>>>(tsrc.as<int32_t>(), R, gdegp, maxd, key.as<uint32_t>());
    k_iota_u32<<<grid_for(R), 256, 0, c.stream>>>(iota.as<uint32_t>(), R);
    radix_pairs<uint32_t, uint32_t>(c, key.as<uint32_t>(), keyS.as<uint32_t>(), iota.as<uint32_t>(),
                                   perm1.as<uint32_t>(), R, G > 1 ? 32 : nbits(int64_t(maxd) + 1));
    iota.release();
    k_gather_u32<<<grid_for(R), 256, 0, c.stream>>>(tdst.as<uint32_t>(), perm1.as<uint32_t>(), key.as<uint32_t>(), R);
    radix_pairs<uint32_t, uint32_t>(c, key.as<uint32_t>(), keyS.as<uint32_t>(), perm1.as<uint32_t>(),
                                   perm.as<uint32_t>(), R, nbits(n_own));
    k_gather_w<int32_t><<<grid_for(R), 256, 0, c.stream>>>(tsrc.as<int32_t>(), perm.as<uint32_t>(), t.col.as<int32_t>(), R);
    rowptr_from_sorted(c, keyS.as<uint32_t>(), R, t.n_rows, t.row_ptr.as<int64_t>());
  } else {
    NBG_HIP(hipMemsetAsync(t.row_ptr.p, 0, size_t(t.n_rows + 1) * 8, c.stream));
  }
  tsrc.release();
  tdst.release();
  for (size_t f = 0; f < o.props.size(); f++) {
    if (!cp[f]) continue;
    int w = cp[f]->width;
    t.props[f].data.alloc(size_t(R) * size_t(w) + 16);
    const void* src = G == 1 ? cp[f]->data.p : rprops[f].p;
    if (R) gather_width(c, src, perm.as<uint32_t>(), t.props[f].data.p, R, w);
    rprops[f].release();
  }
  if (G == 1) {
    es.t_eid = std::move(perm);
    es.has_t_eid = true;
  } else {
    es.has_t_eid = false;
  }
  // the quad slab of the bottom-up first pass (k_bu_lean), packed with the quantised bucket of
  // the first INT-like transposed prop when the gidx leaves >= 3 spare bits below bit 31
  for (int h = 0; h < 2; h++) es.pair_col[h].release();
  es.q_field = -1;
  es.q_gbits = es.q_bits = 0;
  es.tcol_q.release();
  if (R > 0) {
    // 2^gb > n_global: an empty slot (-1) decodes to a gidx past every vertex, whose bitmap
    // probe is out of bounds (k_bu_lean relies on it)
    int gb = 1;
    while ((int64_t(1) << gb) <= c.n_global) gb++;
    const int qb = std::min(8, 31 - gb);
    int f = -1;
    for (size_t i = 0; i < t.props.size() && f < 0; i++)
      if (t.props[i].data.p) f = int(i);
    if (qb >= 3 && f >= 0) {
      const PropCol& pc = t.props[size_t(f)];
      DevBuf mm;
      mm.alloc(16);
      const long long init[2] = {LLONG_MAX, LLONG_MIN};
      NBG_HIP(hipMemcpyAsync(mm.p, init, 16, hipMemcpyHostToDevice, c.stream));
      k_minmax_w<<<grid_for(R), 256, 0, c.stream>>>(pc.data.p, pc.width, R, mm.as<long long>());
      long long h[2];
      NBG_HIP(hipMemcpyAsync(h, mm.p, 16, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
      es.q_field = f;
      es.q_gbits = gb;
      es.q_bits = qb;
      es.q_min = h[0];
      es.q_range = uint64_t(h[1]) - uint64_t(h[0]) + 1;  // 0 = the whole 2^64 range
      es.tcol_q.alloc(size_t(R) * 4 + 64);
      k_pack_col<<<grid_for(R), 256, 0, c.stream>>>(t.col.as<int32_t>(), pc.data.p, pc.width, R, es.q_min, es.q_range,
                                                   gb, qb, es.tcol_q.as<int32_t>());
      NBG_HIP(hipGetLastError());
    }
  }
  {
    // padded to whole 128-row tiles with empty slots (-1)
    const int64_t n_pad = (n_own + 127) / 128 * 128;
    for (int h = 0; h < 2; h++) {
      es.pair_col[h].alloc(size_t(n_pad) * 8 + 16);
      NBG_HIP(hipMemsetAsync(es.pair_col[h].as<uint8_t>() + size_t(n_own) * 8, 0xff, size_t(n_pad - n_own) * 8 + 16,
                             c.stream));
    }
    const int32_t* src_col = es.q_field >= 0 ? es.tcol_q.as<int32_t>() : t.col.as<int32_t>();
    if (n_own)
      k_build_pair<int32_t><<<grid_for(n_own), 256, 0, c.stream>>>(t.row_ptr.as<int64_t>(), src_col, n_own,
                                                                   es.pair_col[0].as<int32_t>(),
                                                                   es.pair_col[1].as<int32_t>(), -1);
  }
  {
    // exact row bounds of the bottom-up hops: past the last row with an in-edge nothing can be
    // found (final hop), past the last one with an in-edge and an out-edge nothing can extend
    // the next frontier (non-final hops); the class-ordered numbering makes both short prefixes
    DevBuf lb;
    lb.alloc(16);
    NBG_HIP(hipMemsetAsync(lb.p, 0, 16, c.stream));
    if (n_own)
      k_live_bounds<<<grid_for(n_own), 256, 0, c.stream>>>(t.row_ptr.as<int64_t>(), es.odeg.as<uint32_t>(), n_own,
                                                           lb.as<unsigned long long>());
    unsigned long long h[2] = {0, 0};
    NBG_HIP(hipMemcpyAsync(h, lb.p, 16, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    es.bu_in_tiles = int64_t((h[0] + 127) / 128);
    es.bu_both_tiles = int64_t((h[1] + 127) / 128);
  }
  es.brec.release();
  es.brec_rows = 0;
  {
    // rest records for the rows a bottom-up hop reads (bu_rec_mb: at most that many MiB, else
    // the rest pass reads row_ptr and the columns)
    const int64_t rows = std::min(n_own, es.bu_in_tiles * 128);
    const int64_t cap_mb = c.opt("bu_rec_mb", 8192);
    if (rows > 0 && c.opt("bu_rec", 1) != 0 && rows * 64 <= (cap_mb << 20)) {
      es.brec.alloc(size_t(rows) * 64);
      const int32_t* src_col = es.q_field >= 0 ? es.tcol_q.as<int32_t>() : t.col.as<int32_t>();
      k_build_rec<<<grid_for(rows), 256, 0, c.stream>>>(t.row_ptr.as<int64_t>(), src_col, rows, es.brec.as<uint4>());
      NBG_HIP(hipGetLastError());
      es.brec_rows = rows;
    }
  }
  NBG_HIP(hipStreamSynchronize(c.stream));
  NBG_HIP(hipGetLastError());
  es.has_tr = true;
}

__global__ void k_owned_only(const uint64_t* in, int64_t n, int parts, int world, int rank, uint8_t* flag) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    int64_t v = int64_t(in[i] ^ (1ull << 63));
    flag[i] = dev_owner(v, parts, world) == rank;
  }
}

// out-degree (pre-collapse multiplicity is fine: it only orders vertices) via a provisional table
__global__ void k_count_deg(const int64_t* src, int64_t n, const int64_t* keys, const int32_t* vals, uint64_t mask,
                            bool has_min, int32_t min_idx, unsigned int* deg) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t g = ht_lookup(keys, vals, mask, src[i], has_min, min_idx);
    if (g >= 0) atomicAdd(deg + g, 1u);
  }
}
// Vertex numbering key (sorted ascending, stable over vids ascending): the degree class above
// the complemented out-degree.  Classes: 0 both in- and out-edges, 1 in-edges only, 2 out-edges
// only, 3 none (ideg null: every vertex class 0, plain descending out-degree).  A bottom-up hop
// then works on a prefix of the rows: a non-final hop on class 0 (a row needs an in-edge to be
// found and an out-edge to matter), the final hop on classes 0-1 (snapshot: bu_both_tiles,
// bu_in_tiles, exact bounds whatever the order).  idx (streamed RMAT build): counts are indexed
// through it.
__global__ void k_class_key(const unsigned int* odeg, const unsigned int* ideg, const uint32_t* idx, int64_t n,
                            uint64_t* key) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t u = idx ? int64_t(idx[i]) : i;
    const uint32_t od = odeg[u];
    uint64_t cls = 0;
    if (ideg) {
      const uint32_t id = ideg[u];
      cls = id ? (od ? 0 : 1) : (od ? 2 : 3);
    }
    key[i] = (cls << 32) | uint64_t(~od);
  }
}

// Degree-ordered vertex numbering: a rank's owned gidx range lists its vertices by descending
// out-degree (ties by vid), one rank: within the degree classes of k_class_key.  The hubs -- the sources a bottom-up hop finds first (hub-first
// transposed rows) -- then share a few cache lines of every frontier bitmap instead of being
// scattered over all of it.  `owned` holds sign-flipped vids, sorted ascending on entry.
static void order_by_degree(Ctx& c, DevBuf& owned, int64_t n_owned) {
  if (n_owned <= 1) return;
  int64_t cap = 1024;
  while (cap < 2 * n_owned) cap <<= 1;
  DevBuf keys, vals, vids, deg, dmin;
  keys.alloc(size_t(cap) * 8);
  vals.alloc(size_t(cap) * 4);
  vids.alloc(size_t(n_owned) * 8);
  deg.alloc(size_t(n_owned) * 4);
  dmin.alloc(4);
  fill<int64_t>(c, keys.as<int64_t>(), INT64_MIN, cap);
  int32_t neg = -1;
  NBG_HIP(hipMemcpyAsync(dmin.p, &neg, 4, hipMemcpyHostToDevice, c.stream));
  NBG_HIP(hipMemsetAsync(deg.p, 0, size_t(n_owned) * 4, c.stream));
  k_unflip<<<grid_for(n_owned), 256, 0, c.stream>>>(owned.as<uint64_t>(), vids.as<int64_t>(), n_owned);
  k_ht_insert<<<grid_for(n_owned), 256, 0, c.stream>>>(keys.as<int64_t>(), vals.as<int32_t>(), uint64_t(cap - 1),
                                                       vids.as<int64_t>(), n_owned, 0, dmin.as<int32_t>());
  int32_t min_idx = -1;
  NBG_HIP(hipMemcpyAsync(&min_idx, dmin.p, 4, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  // in-degrees too, for the degree classes of class_key: one rank counts the dsts of its out-edge
  // stage (every in-edge of an owned vertex is there); several ranks count the in-edge keys
  // (dst, -type, rank, src) their parts hold -- the dst owner's, P5 -- so each rank's range is
  // class-ordered too and its bottom-up hops stop at its own bu_both_tiles / bu_in_tiles
  const bool classes = true;
  DevBuf ideg;
  if (classes) {
    ideg.alloc(size_t(n_owned) * 4);
    NBG_HIP(hipMemsetAsync(ideg.p, 0, size_t(n_owned) * 4, c.stream));
  }
  for (auto& kv : c.edges) {
    const Staging& st = kv.second.out_stage;
    if (!st.n) continue;
    k_count_deg<<<grid_for(st.n), 256, 0, c.stream>>>(st.src.as<int64_t>(), st.n, keys.as<int64_t>(),
                                                     vals.as<int32_t>(), uint64_t(cap - 1), min_idx >= 0, min_idx,
                                                     deg.as<unsigned int>());
    if (classes && !c.sharded)
      k_count_deg<<<grid_for(st.n), 256, 0, c.stream>>>(st.dst.as<int64_t>(), st.n, keys.as<int64_t>(),
                                                       vals.as<int32_t>(), uint64_t(cap - 1), min_idx >= 0, min_idx,
                                                       ideg.as<unsigned int>());
    const Staging& si = kv.second.in_stage;
    if (classes && c.sharded && si.n)
      k_count_deg<<<grid_for(si.n), 256, 0, c.stream>>>(si.src.as<int64_t>(), si.n, keys.as<int64_t>(),
                                                       vals.as<int32_t>(), uint64_t(cap - 1), min_idx >= 0, min_idx,
                                                       ideg.as<unsigned int>());
  }
  keys.release();
  vals.release();
  DevBuf key, keyS, sorted;
  key.alloc(size_t(n_owned) * 8);
  keyS.alloc(size_t(n_owned) * 8);
  sorted.alloc(size_t(n_owned) * 8);
  k_class_key<<<grid_for(n_owned), 256, 0, c.stream>>>(deg.as<unsigned int>(), classes ? ideg.as<unsigned int>() : nullptr,
                                                       nullptr, n_owned, key.as<uint64_t>());
  radix_pairs<uint64_t, uint64_t>(c, key.as<uint64_t>(), keyS.as<uint64_t>(), owned.as<uint64_t>(),
                                 sorted.as<uint64_t>(), n_owned, classes ? 34 : 32);
  NBG_HIP(hipMemcpyAsync(owned.p, sorted.p, size_t(n_owned) * 8, hipMemcpyDeviceToDevice, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  NBG_HIP(hipGetLastError());
}

// Tag columns over the gidx space.  Winner per vertex = the first key of the prefix
// (part, vid, tag) in RocksDB bytewise order: smallest LE version bytes, and among identical keys
// the last write (WriteBatch last-write-wins, RocksEngine.cpp:216-230).  Rows stored in a part
// other than the vid's own are never reached by the prefix scan (the request part is
// hash(vid), StorageClient.cpp:238-243), and vids outside every edge have no gidx: both dropped.
__global__ void k_tag_gather(const int32_t* win, const uint8_t* state, int64_t ng, const int64_t* props,
                             const uint8_t* present, int64_t* data, uint8_t* pres_out) {
  for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < ng; g += int64_t(gridDim.x) * blockDim.x) {
    int32_t w = win[g];
    bool ok = w >= 0 && present[w] != 0;
    data[g] = ok ? props[w] : 0;
    pres_out[g] = ok ? state[g] : 0;
  }
}
__global__ void k_tag_str_len(const int32_t* win, int64_t ng, const uint8_t* present, const int64_t* lens,
                              int64_t* out) {
  for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g <= ng; g += int64_t(gridDim.x) * blockDim.x) {
    int32_t w = g < ng ? win[g] : -1;
    out[g] = (w >= 0 && present[w]) ? lens[w] : 0;
  }
}
__global__ void k_tag_str_copy(const int32_t* win, int64_t ng, const uint8_t* heap, const int64_t* heap_off,
                               const int64_t* off, uint8_t* out) {
  for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < ng; g += int64_t(gridDim.x) * blockDim.x) {
    int64_t len = off[g + 1] - off[g];
    if (len <= 0) continue;
    const uint8_t* s = heap + heap_off[win[g]];
    for (int64_t j = 0; j < len; j++) out[off[g] + j] = s[j];
  }
}

// world > 1: every rank fills its owned gidx slice [base[r], base[r+1]); allgather the slices
// so each rank holds the whole column ($$ props of dsts owned elsewhere)
static void replicate_owned(Ctx& c, DevBuf& col, size_t w) {
  std::vector<size_t> rb(size_t(c.world)), ro(size_t(c.world));
  for (int r = 0; r < c.world; r++) {
    ro[size_t(r)] = size_t(c.base[size_t(r)]) * w;
    rb[size_t(r)] = size_t(c.base[size_t(r) + 1] - c.base[size_t(r)]) * w;
  }
  DevBuf send;
  send.alloc(std::max<size_t>(rb[size_t(c.rank)], 8));
  if (rb[size_t(c.rank)])
    NBG_HIP(hipMemcpyAsync(send.p, col.as<uint8_t>() + ro[size_t(c.rank)], rb[size_t(c.rank)], hipMemcpyDeviceToDevice,
                           c.stream));
  comm_allgatherv_bytes(c, send.p, rb[size_t(c.rank)], col.p, rb.data(), ro.data());
}

static void build_tag_columns(Ctx& c) {
  c.tag_refs.clear();
  const int64_t ng = c.n_global;
  for (auto& kvp : c.tags) {
    TagSpace& ts = kvp.second;
    const int64_t n = ts.stage.n;
    std::vector<int32_t> win(size_t(std::max<int64_t>(ng, 1)), -1);
    std::vector<uint8_t> wstate(size_t(std::max<int64_t>(ng, 1)), 0);  // 1 own part, 2 foreign part
    std::vector<int32_t> tpart(size_t(std::max<int64_t>(ng, 1)), 0);
    if (n > 0 && ng > 0) {
      DevBuf dg;
      dg.alloc(size_t(n) * 4);
      lookup_gidx(c, ts.stage.src.as<int64_t>(), dg.as<int32_t>(), n);
      const size_t nn = static_cast<size_t>(n);
      std::vector<int32_t> g(nn), part(nn);
      std::vector<int64_t> vid(nn), ver(nn), seq(nn);
      NBG_HIP(hipMemcpyAsync(g.data(), dg.p, size_t(n) * 4, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(part.data(), ts.stage.part.p, size_t(n) * 4, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(vid.data(), ts.stage.src.p, size_t(n) * 8, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(ver.data(), ts.stage.ver.p, size_t(n) * 8, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipMemcpyAsync(seq.data(), ts.stage.seq.p, size_t(n) * 8, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
      // candidate order: rows of the vid's own part first (GO reads those), else the smallest
      // foreign part (a getBound request naming that part reads it); then the prefix scan's
      // first key (smallest LE version bytes), identical keys by last write
      auto foreign = [&](int64_t i) { return part[size_t(i)] != part_of_vid(vid[size_t(i)], c.num_parts); };
      // world > 1: a rank keeps only its owned slice (replicate_owned gathers slices); a row in a
      // foreign part held by another rank is not visible there (getBound on that part only)
      const int64_t olo = c.owned_lo(), ohi = c.owned_hi();
      for (int64_t i = 0; i < n; i++) {
        int32_t gi = g[size_t(i)];
        if (gi < 0 || (c.sharded && (gi < olo || gi >= ohi))) continue;
        int32_t& w = win[size_t(gi)];
        if (w < 0) {
          w = int32_t(i);
          continue;
        }
        const bool fi = foreign(i), fw = foreign(w);
        if (fi != fw) {
          if (!fi) w = int32_t(i);
          continue;
        }
        if (fi && part[size_t(i)] != part[size_t(w)]) {
          if (part[size_t(i)] < part[size_t(w)]) w = int32_t(i);
          continue;
        }
        uint64_t a = __builtin_bswap64(uint64_t(ver[size_t(i)])), b = __builtin_bswap64(uint64_t(ver[size_t(w)]));
        if (a < b || (a == b && seq[size_t(i)] > seq[size_t(w)])) w = int32_t(i);
      }
      for (int64_t gi = 0; gi < ng; gi++) {
        const int32_t w = win[size_t(gi)];
        if (w < 0) continue;
        wstate[size_t(gi)] = foreign(w) ? 2 : 1;
        tpart[size_t(gi)] = part[size_t(w)];
      }
    }
    DevBuf dwin, dstate;
    dwin.alloc(size_t(std::max<int64_t>(ng, 1)) * 4);
    dstate.alloc(size_t(std::max<int64_t>(ng, 1)));
    ts.part.alloc(size_t(std::max<int64_t>(ng, 1)) * 4);
    NBG_HIP(hipMemcpyAsync(dwin.p, win.data(), size_t(std::max<int64_t>(ng, 1)) * 4, hipMemcpyHostToDevice, c.stream));
    NBG_HIP(hipMemcpyAsync(dstate.p, wstate.data(), size_t(std::max<int64_t>(ng, 1)), hipMemcpyHostToDevice, c.stream));
    NBG_HIP(hipMemcpyAsync(ts.part.p, tpart.data(), size_t(std::max<int64_t>(ng, 1)) * 4, hipMemcpyHostToDevice, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));  // host vectors are pageable
    ts.cols.clear();
    for (size_t f = 0; f < ts.fields.size(); f++) {
      PropCol pc;
      pc.name = ts.fields[f].name;
      pc.type = ts.fields[f].type;
      pc.width = 8;
      pc.data.alloc(size_t(std::max<int64_t>(ng, 1)) * 8);
      pc.present.alloc(size_t(std::max<int64_t>(ng, 1)));
      if (n == 0 || ng == 0) {
        NBG_HIP(hipMemsetAsync(pc.data.p, 0, pc.data.bytes, c.stream));
        NBG_HIP(hipMemsetAsync(pc.present.p, 0, pc.present.bytes, c.stream));
      } else {
        k_tag_gather<<<grid_for(ng), 256, 0, c.stream>>>(dwin.as<int32_t>(), dstate.as<uint8_t>(), ng,
                                                          ts.stage.props[f].as<int64_t>(),
                                                          ts.stage.present[f].as<uint8_t>(), pc.data.as<int64_t>(),
                                                          pc.present.as<uint8_t>());
      }
      if (pc.type == NBG_T_STRING) {
        DevBuf lens;
        lens.alloc(size_t(ng + 1) * 8);
        pc.str_off.alloc(size_t(ng + 1) * 8);
        if (n == 0 || ng == 0) {
          NBG_HIP(hipMemsetAsync(lens.p, 0, lens.bytes, c.stream));
        } else {
          k_tag_str_len<<<grid_for(ng + 1), 256, 0, c.stream>>>(dwin.as<int32_t>(), ng, ts.stage.present[f].as<uint8_t>(),
                                                                 ts.stage.str_len[f].as<int64_t>(), lens.as<int64_t>());
        }
        exclusive_scan<int64_t>(c, lens.as<int64_t>(), pc.str_off.as<int64_t>(), ng + 1);
        int64_t total = 0;
        NBG_HIP(hipMemcpyAsync(&total, pc.str_off.as<int64_t>() + ng, 8, hipMemcpyDeviceToHost, c.stream));
        NBG_HIP(hipStreamSynchronize(c.stream));
        pc.str_bytes.alloc(size_t(total) + 8);
        if (total > 0)
          k_tag_str_copy<<<grid_for(ng), 256, 0, c.stream>>>(dwin.as<int32_t>(), ng, c.heap.as<uint8_t>(),
                                                              ts.stage.props[f].as<int64_t>(), pc.str_off.as<int64_t>(),
                                                              pc.str_bytes.as<uint8_t>());
        if (c.sharded) {
          // lengths of every rank's owned slice -> global offsets; bytes by owner block
          replicate_owned(c, lens, 8);
          exclusive_scan<int64_t>(c, lens.as<int64_t>(), pc.str_off.as<int64_t>(), ng + 1);
          std::vector<int64_t> goff(size_t(ng) + 1);
          NBG_HIP(hipMemcpyAsync(goff.data(), pc.str_off.p, size_t(ng + 1) * 8, hipMemcpyDeviceToHost, c.stream));
          NBG_HIP(hipStreamSynchronize(c.stream));
          std::vector<size_t> rb(size_t(c.world)), ro(size_t(c.world));
          for (int r = 0; r < c.world; r++) {
            ro[size_t(r)] = size_t(goff[size_t(c.base[size_t(r)])]);
            rb[size_t(r)] = size_t(goff[size_t(c.base[size_t(r) + 1])]) - ro[size_t(r)];
          }
          DevBuf all;
          all.alloc(size_t(goff[size_t(ng)]) + 8);
          comm_allgatherv_bytes(c, pc.str_bytes.p, size_t(total), all.p, rb.data(), ro.data());
          pc.str_bytes = std::move(all);
        }
      }
      if (c.sharded) {
        replicate_owned(c, pc.data, 8);
        replicate_owned(c, pc.present, 1);
      }
      NBG_HIP(hipGetLastError());
      c.tag_refs.push_back(TagFieldRef{ts.name, pc.name, pc.type});
      ts.cols.push_back(std::move(pc));
    }
    if (c.sharded) replicate_owned(c, ts.part, 4);
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (!c.opt("writable", 0)) ts.stage = Staging{};
  }
}

__global__ void k_count_unknown(const int64_t* src, const int64_t* dst, int64_t n, const int64_t* keys_ht,
                                const int32_t* vals_ht, uint64_t mask, bool has_min, int32_t min_gidx,
                                unsigned long long* cnt) {
  unsigned long long u = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    u += (ht_lookup(keys_ht, vals_ht, mask, src[i], has_min, min_gidx) < 0) +
         (ht_lookup(keys_ht, vals_ht, mask, dst[i], has_min, min_gidx) < 0);
  for (int o = 32; o > 0; o >>= 1) u += __shfl_xor(u, o);
  if ((threadIdx.x & 63) == 0 && u) atomicAdd(cnt, u);
}

// vids of a batch's endpoints that are not in the vertex map (sign-flipped for an unsigned sort)
__global__ void k_collect_unknown(const int64_t* src, const int64_t* dst, int64_t n, const int64_t* keys_ht,
                                  const int32_t* vals_ht, uint64_t mask, bool has_min, int32_t min_gidx,
                                  uint64_t* out, unsigned long long* cnt) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (n + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    int64_t a = 0, b = 0;
    bool ua = false, ub = false;
    if (i < n) {
      a = src[i];
      b = dst[i];
      ua = ht_lookup(keys_ht, vals_ht, mask, a, has_min, min_gidx) < 0;
      ub = ht_lookup(keys_ht, vals_ht, mask, b, has_min, min_gidx) < 0;
    }
    const int64_t sa = wave_append(cnt, ua);
    if (ua) out[sa] = uint64_t(a) ^ (1ull << 63);
    const int64_t sb = wave_append(cnt, ub);
    if (ub) out[sb] = uint64_t(b) ^ (1ull << 63);
  }
}
// committed sort keys under new bytewise ranks: the src half stays, the dst rank is re-read
__global__ void k_rekey(uint64_t* skey, const int32_t* dstg, int64_t n, const uint32_t* brank) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    skey[i] = (skey[i] & 0xffffffff00000000ull) | uint64_t(brank[dstg[i]]);
}

// bytewise order rank of every gidx (RocksDB key order of the dst bytes; holes sort anywhere)
static DevBuf bytewise_ranks(Ctx& c) {
  DevBuf brank;
  const int64_t ng = std::max<int64_t>(c.n_global, 1);
  DevBuf k1, k2, i1, i2;
  k1.alloc(size_t(ng) * 8);
  k2.alloc(size_t(ng) * 8);
  i1.alloc(size_t(ng) * 4);
  i2.alloc(size_t(ng) * 4);
  brank.alloc(size_t(ng) * 4);
  if (c.n_global) {
    k_bswap_keys<<<grid_for(c.n_global), 256, 0, c.stream>>>(c.vid_of.as<int64_t>(), k1.as<uint64_t>(), i1.as<uint32_t>(),
                                                             c.n_global);
    radix_pairs<uint64_t, uint32_t>(c, k1.as<uint64_t>(), k2.as<uint64_t>(), i1.as<uint32_t>(), i2.as<uint32_t>(),
                                    c.n_global, 64);
    k_scatter_rank<<<grid_for(c.n_global), 256, 0, c.stream>>>(i2.as<uint32_t>(), brank.as<uint32_t>(), c.n_global);
  }
  return brank;
}

// Merge commit with new vertices (one rank): the batch's unknown endpoint vids, sorted, take
// the gidx after the committed ones (the padding first, then a grown range), the vertex map and
// hash table grow in place (the table is rebuilt when it would pass half full), the bytewise
// ranks are recomputed and the committed sort keys re-read their dst rank -- the committed
// order itself stays sorted, since inserting vids into the bytewise order moves no committed
// vid past another.  Existing gidx never change, so every committed tuple keeps its place.
static void extend_vertex_map(Ctx& c, int64_t unknown_bound) {
  DevBuf raw, cnt;
  raw.alloc(size_t(std::max<int64_t>(unknown_bound, 1)) * 8);
  cnt.alloc(8);
  NBG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  for (auto& kv : c.edges) {
    EdgeSpace& es = kv.second;
    for (int d = 0; d < 2; d++) {
      const Staging& st = d ? es.in_stage : es.out_stage;
      const int64_t n0 = es.ord[d].n;
      if (st.n > n0)
        k_collect_unknown<<<grid_for(st.n - n0), 256, 0, c.stream>>>(
            st.src.as<int64_t>() + n0, st.dst.as<int64_t>() + n0, st.n - n0, c.ht_keys.as<int64_t>(),
            c.ht_vals.as<int32_t>(), uint64_t(c.ht_cap - 1), c.ht_has_min, c.ht_min_gidx, raw.as<uint64_t>(),
            cnt.as<unsigned long long>());
    }
  }
  unsigned long long nraw = 0;
  NBG_HIP(hipMemcpyAsync(&nraw, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  if (int64_t(nraw) > unknown_bound) throw Error(NBG_E_UNKNOWN, "merge commit: unknown-vertex count changed");
  DevBuf sorted, uniq;
  sorted.alloc(size_t(std::max<uint64_t>(nraw, 1)) * 8);
  uniq.alloc(size_t(std::max<uint64_t>(nraw, 1)) * 8);
  radix_keys<uint64_t>(c, raw.as<uint64_t>(), sorted.as<uint64_t>(), int64_t(nraw), 64);
  const int64_t k = nraw ? unique_sorted<uint64_t>(c, sorted.as<uint64_t>(), uniq.as<uint64_t>(), int64_t(nraw)) : 0;
  const int64_t n0 = c.n_vertices, n1 = n0 + k;
  const int64_t ng1 = (n1 + 63) / 64 * 64;
  if (ng1 >= (int64_t(1) << 31)) throw Error(NBG_E_UNSUPPORTED, "more than 2^31 vertices");
  if (ng1 > c.n_global) {
    DevBuf nv;
    nv.alloc(size_t(ng1) * 8);
    fill<int64_t>(c, nv.as<int64_t>(), INT64_MIN, ng1);
    NBG_HIP(hipMemcpyAsync(nv.p, c.vid_of.p, size_t(c.n_global) * 8, hipMemcpyDeviceToDevice, c.stream));
    c.vid_of = std::move(nv);
  }
  if (k) k_unflip<<<grid_for(k), 256, 0, c.stream>>>(uniq.as<uint64_t>(), c.vid_of.as<int64_t>() + n0, k);
  DevBuf dmin;
  dmin.alloc(4);
  int32_t neg = -1;
  NBG_HIP(hipMemcpyAsync(dmin.p, &neg, 4, hipMemcpyHostToDevice, c.stream));
  if (2 * ng1 > c.ht_cap) {  // past half full: a table of the grown size, every vertex inserted
    int64_t cap = 1024;
    while (cap < 2 * ng1) cap <<= 1;
    c.ht_cap = cap;
    c.ht_keys.alloc(size_t(cap) * 8);
    c.ht_vals.alloc(size_t(cap) * 4);
    fill<int64_t>(c, c.ht_keys.as<int64_t>(), INT64_MIN, cap);
    k_ht_insert<<<grid_for(n1), 256, 0, c.stream>>>(c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(),
                                                   uint64_t(cap - 1), c.vid_of.as<int64_t>(), n1, 0, dmin.as<int32_t>());
  } else if (k) {
    k_ht_insert<<<grid_for(k), 256, 0, c.stream>>>(c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(),
                                                  uint64_t(c.ht_cap - 1), c.vid_of.as<int64_t>() + n0, k, n0,
                                                  dmin.as<int32_t>());
  }
  int32_t mg = -1;
  NBG_HIP(hipMemcpyAsync(&mg, dmin.p, 4, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  if (mg >= 0) {
    c.ht_has_min = true;
    c.ht_min_gidx = mg;
  }
  c.n_vertices = n1;
  c.counts.assign(1, n1);
  c.base.assign(2, 0);
  c.base[1] = ng1;
  c.n_global = ng1;
  c.brank = bytewise_ranks(c);
  for (auto& kv : c.edges)
    for (auto& o : kv.second.ord)
      if (o.n > 0 && o.skey.p)
        k_rekey<<<grid_for(o.n), 256, 0, c.stream>>>(o.skey.as<uint64_t>(), o.dstg.as<int32_t>(), o.n,
                                                    c.brank.as<uint32_t>());
  NBG_HIP(hipGetLastError());
}

// Merge commit with new vertices on several ranks.  Every rank sends the unknown endpoint vids
// of its batch (sorted, unique) to all; the union, sorted, is the same on every rank, and each
// owner's new vertices (vid % parts + 1 on rank part % world, pickHosts) take the next gidx of
// its growth room in vid order -- every rank computes every assignment itself, so the
// replicated vertex map and hash table stay identical without a second exchange.  Returns false
// (on every rank alike) when some owner's room is too small: the caller then rebuilds fully.
struct NewVertexPlan {
  std::vector<int64_t> vids;  // the union, sorted
  std::vector<std::vector<int64_t>> per_owner;
};
static bool plan_new_vertices_ranks(Ctx& c, int64_t unknown_bound, NewVertexPlan& plan) {
  DevBuf raw, cnt;
  raw.alloc(size_t(std::max<int64_t>(unknown_bound, 1)) * 8);
  cnt.alloc(8);
  NBG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  for (auto& kv : c.edges) {
    EdgeSpace& es = kv.second;
    for (int d = 0; d < 2; d++) {
      const Staging& st = d ? es.in_stage : es.out_stage;
      const int64_t n0 = es.ord[d].n;
      if (st.n > n0)
        k_collect_unknown<<<grid_for(st.n - n0), 256, 0, c.stream>>>(
            st.src.as<int64_t>() + n0, st.dst.as<int64_t>() + n0, st.n - n0, c.ht_keys.as<int64_t>(),
            c.ht_vals.as<int32_t>(), uint64_t(c.ht_cap - 1), c.ht_has_min, c.ht_min_gidx, raw.as<uint64_t>(),
            cnt.as<unsigned long long>());
    }
  }
  unsigned long long nraw = 0;
  NBG_HIP(hipMemcpyAsync(&nraw, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  if (int64_t(nraw) > unknown_bound) throw Error(NBG_E_UNKNOWN, "merge commit: unknown-vertex count changed");
  int64_t k = 0;
  DevBuf sorted, uniq;
  sorted.alloc(size_t(std::max<uint64_t>(nraw, 1)) * 8);
  uniq.alloc(size_t(std::max<uint64_t>(nraw, 1)) * 8);
  if (nraw) {
    radix_keys<uint64_t>(c, raw.as<uint64_t>(), sorted.as<uint64_t>(), int64_t(nraw), 64);
    k = unique_sorted<uint64_t>(c, sorted.as<uint64_t>(), uniq.as<uint64_t>(), int64_t(nraw));
  }
  // every rank's list to every rank
  const size_t G = size_t(c.world);
  DevBuf dk, dall;
  dk.alloc(8);
  dall.alloc(8 * G);
  NBG_HIP(hipMemcpyAsync(dk.p, &k, 8, hipMemcpyHostToDevice, c.stream));
  comm_allgather_bytes(c, dk.p, 8, dall.p);
  std::vector<int64_t> ks(G);
  NBG_HIP(hipMemcpyAsync(ks.data(), dall.p, 8 * G, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  std::vector<size_t> rb(G), ro(G);
  size_t tot = 0;
  for (size_t r = 0; r < G; r++) {
    rb[r] = size_t(ks[r]) * 8;
    ro[r] = tot;
    tot += rb[r];
  }
  DevBuf recv;
  recv.alloc(std::max<size_t>(tot, 8));
  comm_allgatherv_bytes(c, uniq.p, size_t(k) * 8, recv.p, rb.data(), ro.data());
  std::vector<uint64_t> flipped(tot / 8);
  if (tot) NBG_HIP(hipMemcpyAsync(flipped.data(), recv.p, tot, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  std::sort(flipped.begin(), flipped.end());
  flipped.erase(std::unique(flipped.begin(), flipped.end()), flipped.end());
  plan.vids.resize(flipped.size());
  plan.per_owner.assign(G, {});
  for (size_t i = 0; i < flipped.size(); i++) {  // sign-flipped order = signed vid order
    const int64_t v = int64_t(flipped[i] ^ (1ull << 63));
    plan.vids[i] = v;
    plan.per_owner[size_t(dev_owner(v, c.num_parts, c.world))].push_back(v);
  }
  for (size_t q = 0; q < G; q++)
    if (c.counts[q] + int64_t(plan.per_owner[q].size()) > c.base[q + 1] - c.base[q]) return false;
  return true;
}

// applies a plan: each owner's new vertices at base + counts onward, in the replicated vertex map
// and hash table; bytewise ranks recomputed and the committed sort keys re-read their dst rank
static void extend_vertex_map_ranks(Ctx& c, const NewVertexPlan& plan) {
  DevBuf dmin, dv;
  dmin.alloc(4);
  int32_t neg = -1;
  NBG_HIP(hipMemcpyAsync(dmin.p, &neg, 4, hipMemcpyHostToDevice, c.stream));
  dv.alloc(std::max<size_t>(plan.vids.size(), 1) * 8);
  size_t off = 0;
  for (size_t q = 0; q < plan.per_owner.size(); q++) {
    const auto& l = plan.per_owner[q];
    if (l.empty()) continue;
    const int64_t g0 = c.base[q] + c.counts[q];
    NBG_HIP(hipMemcpyAsync(dv.as<int64_t>() + off, l.data(), l.size() * 8, hipMemcpyHostToDevice, c.stream));
    NBG_HIP(hipMemcpyAsync(c.vid_of.as<int64_t>() + g0, dv.as<int64_t>() + off, l.size() * 8, hipMemcpyDeviceToDevice,
                           c.stream));
    k_ht_insert<<<grid_for(int64_t(l.size())), 256, 0, c.stream>>>(c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(),
                                                                   uint64_t(c.ht_cap - 1), dv.as<int64_t>() + off,
                                                                   int64_t(l.size()), g0, dmin.as<int32_t>());
    off += l.size();
  }
  int32_t mg = -1;
  NBG_HIP(hipMemcpyAsync(&mg, dmin.p, 4, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));  // (the host lists are pageable)
  if (mg >= 0) {
    c.ht_has_min = true;
    c.ht_min_gidx = mg;
  }
  for (size_t q = 0; q < plan.per_owner.size(); q++) c.counts[q] += int64_t(plan.per_owner[q].size());
  c.n_vertices += int64_t(plan.vids.size());
  c.brank = bytewise_ranks(c);
  for (auto& kv : c.edges)
    for (auto& o : kv.second.ord)
      if (o.n > 0 && o.skey.p)
        k_rekey<<<grid_for(o.n), 256, 0, c.stream>>>(o.skey.as<uint64_t>(), o.dstg.as<int32_t>(), o.n,
                                                    c.brank.as<uint32_t>());
  NBG_HIP(hipGetLastError());
}

static bool commit_merge(Ctx& c) {
  // several ranks: the choice is collective (every rank merges or every rank rebuilds), agreed by
  // one sum over the ranks' flags below; the option and c.brank (writable) agree on every rank
  if (c.opt("merge_commit", 1) == 0 || !c.brank.p) return false;
  bool tag_writes = false;
  for (auto& kv : c.tags) tag_writes |= kv.second.stage.n != kv.second.committed_n;
  bool refuse = false;
  DevBuf cnt;
  cnt.alloc(8);
  NBG_HIP(hipMemsetAsync(cnt.p, 0, 8, c.stream));
  for (auto& kv : c.edges) {
    EdgeSpace& es = kv.second;
    if (es.rmat_stream) refuse = true;
    for (int d = 0; d < 2 && !refuse; d++) {
      const Staging& st = d ? es.in_stage : es.out_stage;
      const int64_t n0 = es.ord[d].n;
      if (st.n == n0) continue;
      if (n0 <= 0 || !es.ord[d].perm.p || st.n < n0 || st.seq.bytes < size_t(st.n) * 8) {
        refuse = true;
        break;
      }
      k_count_unknown<<<grid_for(st.n - n0), 256, 0, c.stream>>>(
          st.src.as<int64_t>() + n0, st.dst.as<int64_t>() + n0, st.n - n0, c.ht_keys.as<int64_t>(),
          c.ht_vals.as<int32_t>(), uint64_t(c.ht_cap - 1), c.ht_has_min, c.ht_min_gidx, cnt.as<unsigned long long>());
    }
  }
  unsigned long long unknown = 0;
  NBG_HIP(hipMemcpyAsync(&unknown, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  if (!refuse && unknown) {
    // new vertices extend the numbering (extend_vertex_map); every CSR direction then needs
    // rows for them, which the merge builds only where the batch has tuples: other batches
    // (and the off switch) take the full rebuild
    // (several ranks: the new vertices land in rows every CSR already has, the growth room)
    for (auto& kv : c.edges)
      for (int d = 0; d < 2 && !c.sharded; d++)
        if ((d ? kv.second.in_stage.n : kv.second.out_stage.n) == kv.second.ord[d].n) refuse = true;
  }
  // per edge space: did this rank's out / in CSR change (a rank without writes of its own still
  // rebuilds its transposed rows when another rank's out-edges changed)
  const size_t ne = c.edges.size();
  std::vector<int64_t> flags(3 + 2 * ne, 0);
  {
    size_t i = 3;
    for (auto& kv : c.edges) {
      flags[i++] = kv.second.out_stage.n != kv.second.ord[0].n;
      flags[i++] = kv.second.in_stage.n != kv.second.ord[1].n;
    }
  }
  flags[0] = refuse, flags[1] = int64_t(unknown), flags[2] = tag_writes;
  if (c.sharded) {
    DevBuf f;
    f.alloc(flags.size() * 8);
    NBG_HIP(hipMemcpyAsync(f.p, flags.data(), flags.size() * 8, hipMemcpyHostToDevice, c.stream));
    comm_allreduce_sum_i64(c, f.as<int64_t>(), flags.size());
    NBG_HIP(hipMemcpyAsync(flags.data(), f.p, flags.size() * 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
  }
  // several ranks with new vertices: placed in the owners' growth rooms when they fit on every
  // rank (collective: the same union and decision everywhere), else the full rebuild
  NewVertexPlan plan;
  if (c.sharded && !flags[0] && flags[1] > 0 &&
      !plan_new_vertices_ranks(c, int64_t(unknown), plan))
    flags[0] = 1;
  if (flags[0]) return false;
  const bool any_tags = flags[2] > 0;
  PoolScope build_scope(build_pool(c));
  c.finalized = false;  // a merge that throws leaves the next commit a full rebuild
  const double t0 = now_s();
  const bool trace = c.opt("build_trace", 0) != 0;
  double tmark = t0;
  auto phase = [&](const char* name) {
    if (!trace) return;
    NBG_HIP(hipStreamSynchronize(c.stream));
    const double t = now_s();
    const int64_t an = g_alloc_clock.alloc_ns.exchange(0), fn = g_alloc_clock.free_ns.exchange(0);
    const int64_t na = g_alloc_clock.allocs.exchange(0);
    fprintf(stderr, "[nbg merge] %-22s %8.3f s  (hipMalloc %lld x %.3f s, hipFree %.3f s)\n", name, t - tmark,
            (long long)na, an * 1e-9, fn * 1e-9);
    tmark = t;
  };
  phase("checks");
  const bool new_vertices = c.sharded ? !plan.vids.empty() : unknown > 0;
  if (c.sharded && new_vertices) {
    extend_vertex_map_ranks(c, plan);
    phase("vertex map (new vertices)");
  } else if (new_vertices) {
    extend_vertex_map(c, int64_t(unknown));
    phase("vertex map (new vertices)");
  }
  if (new_vertices || any_tags) {
    // tag columns span the gidx space and pick winners over every staged row: rebuilt (on every
    // rank when any has tag writes: the owned slices are allgathered)
    c.tag_table.release();
    for (auto& kv : c.tags) {
      kv.second.cols.clear();
      kv.second.part.release();
    }
    build_tag_columns(c);
    for (auto& kv : c.tags) kv.second.committed_n = kv.second.stage.n;
    phase("tag columns");
  }
  size_t fi = 3;
  for (auto& kv : c.edges) {
    EdgeSpace& es = kv.second;
    const bool out_changed = es.out_stage.n != es.ord[0].n, in_changed = es.in_stage.n != es.ord[1].n;
    const bool out_any = flags[fi] > 0, in_any = flags[fi + 1] > 0;  // on some rank
    fi += 2;
    if (out_changed) {
      Csr keep_in = std::move(es.in);  // an unchanged in CSR survives the reset
      reset_edge_derived(es);          // out CSR and everything derived from it (transpose, slabs)
      es.in = std::move(keep_in);
      build_csr(c, es.out_stage, es.fields, true, es.out, c.brank.as<uint32_t>(), false, &es.ord[0], true);
      phase("out CSR (merge)");
    } else if (out_any) {
      reset_transpose_derived(es);  // another rank's out-edges land in this rank's transposed rows
    }
    if (in_changed) build_csr(c, es.in_stage, es.fields, false, es.in, c.brank.as<uint32_t>(), false, &es.ord[1], true);
    phase("in CSR (merge)");
    if (out_any || in_any) {
      // replicated CSRs (FIND SHORTEST PATH on several ranks) are rebuilt on first use
      es.rep_out = Csr();
      es.rep_in = Csr();
      es.has_rep = es.has_rep_out = false;
      es.rep_odeg.release();
    }
    if (out_any && c.opt("bottom_up", 1)) build_transpose(c, es);  // collective on several ranks
    phase("transpose + slabs");
  }
  c.ws_tmp.release();
  NBG_HIP(hipStreamSynchronize(c.stream));
  c.finalized = true;
  c.build_seconds += now_s() - t0;
  return true;
}

// ------------------------------------------------------------------------------------------
// Streamed RMAT build (one rank).  The tuple stage holds 40+ bytes per sample in each CSR
// direction and indexes tuples with 32-bit permutations, so RMAT-28 (2^32 samples) cannot pass
// through it.  Here the generator is re-run instead of stored: one counting pass gives the vertex
// set and the per-vertex sample counts, the vertex numbering is the staged build's (vids sorted,
// then by descending sample out-degree), and each CSR direction is built in src-gidx buckets of
// at most rmat_bucket samples: regenerate, keep the bucket's samples as 64-bit keys
// (local src << 32 | bytewise rank of dst), radix sort, unique (= the version / identical-key
// collapse of a generator that writes one version of rank 0), and emit row_ptr, col, the dst-vid
// column and the weight (a function of (src, dst), recomputed).  Same CSR as the staged build.
// ------------------------------------------------------------------------------------------
__global__ void k_rmat_count(int64_t lo, int64_t hi, int32_t scale, uint64_t seed, uint8_t* present,
                             uint32_t* odeg_u, uint32_t* ideg_u) {
  for (int64_t i = lo + blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < hi; i += int64_t(gridDim.x) * blockDim.x) {
    uint64_t u, v;
    rmat_sample(uint64_t(i), scale, seed, u, v);
    present[u] = 1;  // idempotent byte stores
    present[v] = 1;
    atomicAdd(odeg_u + u, 1u);
    atomicAdd(ideg_u + v, 1u);
  }
}
__global__ void k_rmat_vkeys(const uint32_t* idx, int64_t n, uint64_t smix, uint64_t* key) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    key[i] = uint64_t(rmat_vid(idx[i], smix)) ^ (1ull << 63);
}
// gidx g <-> index u; vid_of; per-gidx sample counts of both directions
__global__ void k_rmat_number(const uint32_t* idx, int64_t n, uint64_t smix, const uint32_t* odeg_u,
                              const uint32_t* ideg_u, int32_t* gidx_of_u, int64_t* vid_of, int64_t* ocnt,
                              int64_t* icnt) {
  for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < n; g += int64_t(gridDim.x) * blockDim.x) {
    const uint32_t u = idx[g];
    gidx_of_u[u] = int32_t(g);
    vid_of[g] = rmat_vid(u, smix);
    ocnt[g] = odeg_u[u];
    icnt[g] = ideg_u[u];
  }
}
// brank_u[u] = bytewise rank of u's vid; gidx_of_rank = its inverse over the gidx space
__global__ void k_rmat_rank_maps(const uint32_t* idx, int64_t n, const uint32_t* brank, uint32_t* brank_u,
                                 int32_t* gidx_of_rank) {
  for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < n; g += int64_t(gridDim.x) * blockDim.x) {
    brank_u[idx[g]] = brank[g];
    gidx_of_rank[brank[g]] = int32_t(g);
  }
}
// bucket starts: row g opens bucket excl[g] / cap when that differs from row g - 1's
__global__ void k_rmat_cuts(const int64_t* excl, int64_t n, int64_t cap, int64_t* cut) {
  for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < n; g += int64_t(gridDim.x) * blockDim.x) {
    const int64_t k = excl[g] / cap;
    if (g == 0 || excl[g - 1] / cap != k) cut[k] = g;
  }
}
// the samples of bucket [ga, gb) of one direction (out: key src u, in: key src v) as sort keys
__global__ void k_rmat_bucket(int64_t lo, int64_t hi, int32_t scale, uint64_t seed, int32_t dir,
                              const int32_t* gidx_of_u, const uint32_t* brank_u, int64_t ga, int64_t gb, uint64_t* keys,
                              unsigned long long* cnt, int64_t cap) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  const int64_t rounds = (hi - lo + stride - 1) / stride;
  for (int64_t r = 0; r < rounds; r++) {
    const int64_t i = lo + r * stride + blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    bool take = false;
    uint64_t key = 0;
    if (i < hi) {
      uint64_t u, v;
      rmat_sample(uint64_t(i), scale, seed, u, v);
      const uint64_t sidx = dir ? v : u, didx = dir ? u : v;
      const int64_t g = gidx_of_u[sidx];
      take = g >= ga && g < gb;
      if (take) key = (uint64_t(g - ga) << 32) | brank_u[didx];
    }
    const int64_t slot = wave_append(cnt, take);
    if (take && slot < cap) keys[slot] = key;
  }
}
// CSR rows [ga, gb) from the bucket's sorted unique keys (entries base .. base + m)
__global__ void k_rmat_emit(const uint64_t* keys, int64_t m, int64_t ga, int64_t nrows, int64_t base,
                            const int32_t* gidx_of_rank, const int64_t* vid_of, uint64_t seed, int64_t* row_ptr,
                            int32_t* col, int64_t* col_vid, int16_t* w16) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= m; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t prev = i == 0 ? -1 : int64_t(keys[i - 1] >> 32);
    const int64_t cur = i == m ? nrows : int64_t(keys[i] >> 32);
    for (int64_t r = prev + 1; r <= cur; r++) row_ptr[ga + r] = base + i;
    if (i == m) continue;
    const int32_t d = gidx_of_rank[uint32_t(keys[i])];
    col[base + i] = d;
    if (col_vid) {
      const int64_t dv = vid_of[d];
      col_vid[base + i] = dv;
      w16[base + i] = int16_t(rmat_weight(vid_of[ga + cur], dv, seed));
    }
  }
}
__global__ void k_i16_to_i8(const int16_t* in, int8_t* out, int64_t m) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = int8_t(in[i]);
}

static void finalize_rmat_stream(Ctx& c, EdgeSpace& es) {
  if (c.sharded) throw Error(NBG_E_UNSUPPORTED, "streamed RMAT build on more than one rank");
  if (c.edges.size() != 1 || !c.tags.empty())
    throw Error(NBG_E_UNSUPPORTED, "streamed RMAT must be the snapshot's only edge type, without tags");
  const int32_t scale = es.rmat_scale;
  const uint64_t seed = es.rmat_seed;
  const int64_t E = int64_t(es.rmat_ef) << scale;
  const int64_t NU = int64_t(1) << scale;
  const uint64_t smix = splitmix64(seed) & ((1ull << 63) - 1);
  const int64_t chunk = int64_t(1) << 28;
  auto sample_grid = [](int64_t n) { return int(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 64))); };
  // 1. counting pass
  DevBuf present, odeg_u, ideg_u;
  present.alloc(size_t(NU));
  odeg_u.alloc(size_t(NU) * 4);
  ideg_u.alloc(size_t(NU) * 4);
  NBG_HIP(hipMemsetAsync(present.p, 0, size_t(NU), c.stream));
  NBG_HIP(hipMemsetAsync(odeg_u.p, 0, size_t(NU) * 4, c.stream));
  NBG_HIP(hipMemsetAsync(ideg_u.p, 0, size_t(NU) * 4, c.stream));
  for (int64_t lo = 0; lo < E; lo += chunk) {
    const int64_t hi = std::min(E, lo + chunk);
    k_rmat_count<<<sample_grid(hi - lo), 256, 0, c.stream>>>(lo, hi, scale, seed, present.as<uint8_t>(),
                                                             odeg_u.as<uint32_t>(), ideg_u.as<uint32_t>());
  }
  NBG_HIP(hipGetLastError());
  // 2. vertex set in the staged build's numbering: vids ascending (signed), then stable by
  // descending sample out-degree (order_by_degree), unless degree_order = 0
  DevBuf idxA, idxB, cntb;
  idxA.alloc(size_t(NU) * 4);
  cntb.alloc(8);
  {
    size_t tb = 0;
    rocprim::counting_iterator<uint32_t> it(0);
    NBG_HIP(rocprim::select(nullptr, tb, it, present.as<uint8_t>(), idxA.as<uint32_t>(), cntb.as<uint64_t>(),
                            size_t(NU), c.stream));
    c.ws_tmp.ensure(tb);
    NBG_HIP(rocprim::select(c.ws_tmp.p, tb, it, present.as<uint8_t>(), idxA.as<uint32_t>(), cntb.as<uint64_t>(),
                            size_t(NU), c.stream));
  }
  uint64_t hn = 0;
  NBG_HIP(hipMemcpyAsync(&hn, cntb.p, 8, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  present.release();
  const int64_t n = int64_t(hn);
  if (n == 0) throw Error(NBG_E_INVALID_ARG, "empty RMAT graph");
  idxB.alloc(size_t(n) * 4);
  {
    DevBuf k1, k2;
    k1.alloc(size_t(n) * 8);
    k2.alloc(size_t(n) * 8);
    k_rmat_vkeys<<<grid_for(n), 256, 0, c.stream>>>(idxA.as<uint32_t>(), n, smix, k1.as<uint64_t>());
    radix_pairs<uint64_t, uint32_t>(c, k1.as<uint64_t>(), k2.as<uint64_t>(), idxA.as<uint32_t>(), idxB.as<uint32_t>(),
                                    n, 64);
  }
  uint32_t* order = idxB.as<uint32_t>();
  if (c.opt("degree_order", 1)) {
    // the staged build's key (k_class_key; this builder runs on one rank)
    const bool classes = true;
    DevBuf d1, d2;
    d1.alloc(size_t(n) * 8);
    d2.alloc(size_t(n) * 8);
    k_class_key<<<grid_for(n), 256, 0, c.stream>>>(odeg_u.as<unsigned int>(), classes ? ideg_u.as<unsigned int>() : nullptr,
                                                   idxB.as<uint32_t>(), n, d1.as<uint64_t>());
    radix_pairs<uint64_t, uint32_t>(c, d1.as<uint64_t>(), d2.as<uint64_t>(), idxB.as<uint32_t>(), idxA.as<uint32_t>(),
                                    n, classes ? 34 : 32);
    order = idxA.as<uint32_t>();
  }
  // 3. vertex map (one rank: base = [0, n padded to 64])
  c.counts.assign(1, n);
  c.base.assign(2, 0);
  c.base[1] = (n + 63) / 64 * 64;
  c.n_global = c.base[1];
  c.n_vertices = n;
  if (c.n_global >= (int64_t(1) << 31)) throw Error(NBG_E_UNSUPPORTED, "more than 2^31 vertices");
  c.vid_of.alloc(size_t(c.n_global) * 8);
  fill<int64_t>(c, c.vid_of.as<int64_t>(), INT64_MIN, c.n_global);
  DevBuf gidx_of_u, ocnt, icnt;
  gidx_of_u.alloc(size_t(NU) * 4);
  ocnt.alloc(size_t(c.n_global + 1) * 8);
  icnt.alloc(size_t(c.n_global + 1) * 8);
  NBG_HIP(hipMemsetAsync(ocnt.p, 0, size_t(c.n_global + 1) * 8, c.stream));
  NBG_HIP(hipMemsetAsync(icnt.p, 0, size_t(c.n_global + 1) * 8, c.stream));
  k_rmat_number<<<grid_for(n), 256, 0, c.stream>>>(order, n, smix, odeg_u.as<uint32_t>(), ideg_u.as<uint32_t>(),
                                                   gidx_of_u.as<int32_t>(), c.vid_of.as<int64_t>(), ocnt.as<int64_t>(),
                                                   icnt.as<int64_t>());
  odeg_u.release();
  ideg_u.release();
  int64_t cap = 1024;
  while (cap < 2 * c.n_global) cap <<= 1;
  c.ht_cap = cap;
  c.ht_keys.alloc(size_t(cap) * 8);
  c.ht_vals.alloc(size_t(cap) * 4);
  fill<int64_t>(c, c.ht_keys.as<int64_t>(), INT64_MIN, cap);
  DevBuf dmin;
  dmin.alloc(4);
  int32_t neg = -1;
  NBG_HIP(hipMemcpyAsync(dmin.p, &neg, 4, hipMemcpyHostToDevice, c.stream));
  k_ht_insert<<<grid_for(n), 256, 0, c.stream>>>(c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(), uint64_t(cap - 1),
                                                 c.vid_of.as<int64_t>(), n, 0, dmin.as<int32_t>());
  NBG_HIP(hipMemcpyAsync(&c.ht_min_gidx, dmin.p, 4, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  c.ht_has_min = c.ht_min_gidx >= 0;
  // 4. bytewise rank of every vertex (row order = RocksDB key order), per index and inverted
  DevBuf brank_u, gidx_of_rank;
  {
    const int64_t ng = c.n_global;
    DevBuf k1, k2, i1, i2, brank;
    k1.alloc(size_t(ng) * 8);
    k2.alloc(size_t(ng) * 8);
    i1.alloc(size_t(ng) * 4);
    i2.alloc(size_t(ng) * 4);
    brank.alloc(size_t(ng) * 4);
    k_bswap_keys<<<grid_for(ng), 256, 0, c.stream>>>(c.vid_of.as<int64_t>(), k1.as<uint64_t>(), i1.as<uint32_t>(), ng);
    radix_pairs<uint64_t, uint32_t>(c, k1.as<uint64_t>(), k2.as<uint64_t>(), i1.as<uint32_t>(), i2.as<uint32_t>(), ng, 64);
    k_scatter_rank<<<grid_for(ng), 256, 0, c.stream>>>(i2.as<uint32_t>(), brank.as<uint32_t>(), ng);
    brank_u.alloc(size_t(NU) * 4);
    gidx_of_rank.alloc(size_t(ng) * 4);
    k_rmat_rank_maps<<<grid_for(n), 256, 0, c.stream>>>(order, n, brank.as<uint32_t>(), brank_u.as<uint32_t>(),
                                                        gidx_of_rank.as<int32_t>());
  }
  idxA.release();
  idxB.release();
  // 5. the two CSR directions, bucket by bucket
  const int64_t bucket_cap = std::max<int64_t>(c.opt("rmat_bucket", int64_t(1) << 30), 1 << 16);
  const int64_t n_rows = c.n_global;
  for (int dir = 0; dir < 2; dir++) {
    Csr& out = dir ? es.in : es.out;
    out = Csr();
    out.n_rows = n_rows;
    DevBuf excl;
    excl.alloc(size_t(n_rows + 1) * 8);
    exclusive_scan<int64_t>(c, (dir ? icnt : ocnt).as<int64_t>(), excl.as<int64_t>(), n_rows + 1);
    int64_t total = 0;
    NBG_HIP(hipMemcpyAsync(&total, excl.as<int64_t>() + n_rows, 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    if (total != E) throw Error(NBG_E_UNKNOWN, "streamed RMAT: sample counts do not add up");
    const int64_t nb = (total + bucket_cap - 1) / bucket_cap;
    DevBuf dcut;
    dcut.alloc(size_t(nb + 1) * 8);
    NBG_HIP(hipMemsetAsync(dcut.p, 0xff, size_t(nb + 1) * 8, c.stream));
    k_rmat_cuts<<<grid_for(n_rows), 256, 0, c.stream>>>(excl.as<int64_t>(), n_rows, bucket_cap, dcut.as<int64_t>());
    std::vector<int64_t> cut(size_t(nb + 1));
    NBG_HIP(hipMemcpyAsync(cut.data(), dcut.p, size_t(nb) * 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    std::vector<int64_t> starts;
    for (int64_t k = 0; k < nb; k++)
      if (cut[size_t(k)] >= 0) starts.push_back(cut[size_t(k)]);
    starts.push_back(n_rows);
    // samples per bucket (upper bounds of the unique keys)
    std::vector<int64_t> sb(starts.size());
    for (size_t k = 0; k < starts.size(); k++)
      NBG_HIP(hipMemcpyAsync(&sb[k], excl.as<int64_t>() + starts[k], 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    int64_t maxb = 0;
    for (size_t k = 0; k + 1 < starts.size(); k++) maxb = std::max(maxb, sb[k + 1] - sb[k]);
    excl.release();
    // final arrays sized for every sample (trimmed nnz is known only at the end; the tail stays unused)
    out.row_ptr.alloc(size_t(n_rows + 1) * 8);
    NBG_HIP(hipMemsetAsync(out.row_ptr.p, 0, 8, c.stream));
    out.col.alloc(size_t(E) * 4 + 64);  // padded: aligned 16-byte loads past the last entry
    const bool with_props = dir == 0;
    DevBuf w16;
    if (with_props) {
      if (c.opt("rows_vid_col", 1)) out.col_vid.alloc(size_t(E) * 8 + 8);
      w16.alloc(size_t(E) * 2 + 16);
    }
    DevBuf kA, kB;
    kA.alloc(size_t(std::max<int64_t>(maxb, 1)) * 8);
    kB.alloc(size_t(std::max<int64_t>(maxb, 1)) * 8);
    DevBuf bc;
    bc.alloc(8);
    int64_t base = 0;
    for (size_t k = 0; k + 1 < starts.size(); k++) {
      const int64_t ga = starts[k], gb = starts[k + 1], want = sb[k + 1] - sb[k];
      if (want == 0) {  // rows without samples (a run of zero-degree rows)
        k_rmat_emit<<<1, 64, 0, c.stream>>>(kB.as<uint64_t>(), 0, ga, gb - ga, base, gidx_of_rank.as<int32_t>(),
                                            c.vid_of.as<int64_t>(), seed, out.row_ptr.as<int64_t>(),
                                            out.col.as<int32_t>(), nullptr, nullptr);
        continue;
      }
      NBG_HIP(hipMemsetAsync(bc.p, 0, 8, c.stream));
      for (int64_t lo = 0; lo < E; lo += chunk) {
        const int64_t hi = std::min(E, lo + chunk);
        k_rmat_bucket<<<sample_grid(hi - lo), 256, 0, c.stream>>>(lo, hi, scale, seed, dir, gidx_of_u.as<int32_t>(),
                                                                  brank_u.as<uint32_t>(), ga, gb, kA.as<uint64_t>(),
                                                                  bc.as<unsigned long long>(), want);
      }
      int bits = 33;
      while ((int64_t(1) << (bits - 32)) < gb - ga) bits++;
      radix_keys<uint64_t>(c, kA.as<uint64_t>(), kB.as<uint64_t>(), want, std::min(bits, 64));
      const int64_t m = unique_sorted<uint64_t>(c, kB.as<uint64_t>(), kA.as<uint64_t>(), want);
      k_rmat_emit<<<grid_for(m + 1), 256, 0, c.stream>>>(kA.as<uint64_t>(), m, ga, gb - ga, base,
                                                         gidx_of_rank.as<int32_t>(), c.vid_of.as<int64_t>(), seed,
                                                         out.row_ptr.as<int64_t>(), out.col.as<int32_t>(),
                                                         with_props ? out.col_vid.as<int64_t>() : nullptr,
                                                         with_props ? w16.as<int16_t>() : nullptr);
      NBG_HIP(hipGetLastError());
      base += m;
    }
    out.nnz = base;
    // row_part by the hash rule (every generated key sits in hash(vid)'s part: row_ok stays empty)
    out.row_part.alloc(size_t(n_rows + 1) * 4);
    k_row_part_default<<<grid_for(n_rows), 256, 0, c.stream>>>(c.vid_of.as<int64_t>(), n_rows, c.num_parts,
                                                               out.row_part.as<int32_t>());
    if (with_props) {  // weight: narrowed to the width its range needs, as gather_props does
      PropCol pc;
      pc.name = es.fields[0].name;
      pc.type = es.fields[0].type;
      DevBuf mm;
      mm.alloc(16);
      long long hm[2] = {LLONG_MAX, LLONG_MIN};
      NBG_HIP(hipMemcpyAsync(mm.p, hm, 16, hipMemcpyHostToDevice, c.stream));
      if (base) k_minmax_w<<<grid_for(base), 256, 0, c.stream>>>(w16.p, 2, base, mm.as<long long>());
      NBG_HIP(hipMemcpyAsync(hm, mm.p, 16, hipMemcpyDeviceToHost, c.stream));
      NBG_HIP(hipStreamSynchronize(c.stream));
      pc.minv = base ? hm[0] : 0;
      pc.maxv = base ? hm[1] : 0;
      if (pc.minv >= INT8_MIN && pc.maxv <= INT8_MAX) {
        pc.width = 1;
        pc.data.alloc(size_t(base) + 16);
        if (base) k_i16_to_i8<<<grid_for(base), 256, 0, c.stream>>>(w16.as<int16_t>(), pc.data.as<int8_t>(), base);
      } else {
        pc.width = 2;
        pc.data = std::move(w16);
      }
      out.props.push_back(std::move(pc));
    }
    NBG_HIP(hipStreamSynchronize(c.stream));
  }
  // 6. out-degrees (compaction's degree reads); no transposed CSR: GO runs top-down here
  const int64_t n_pad = (n_rows + 127) / 128 * 128;
  es.odeg.alloc(size_t(n_pad + 1) * 4);
  NBG_HIP(hipMemsetAsync(es.odeg.p, 0, size_t(n_pad + 1) * 4, c.stream));
  k_out_deg<<<grid_for(n_rows), 256, 0, c.stream>>>(es.out.row_ptr.as<int64_t>(), nullptr, n_rows,
                                                    es.odeg.as<uint32_t>(), nullptr);
  es.has_tr = false;
  NBG_HIP(hipStreamSynchronize(c.stream));
  NBG_HIP(hipGetLastError());
}

void snapshot_finalize(Ctx& c) {
  if (c.finalized) throw Error(NBG_E_STATE, "snapshot already finalized");
  PoolScope build_scope(build_pool(c));
  struct TrimAfter {  // a read-only snapshot has no further builds: give the cache back
    Ctx& c;
    ~TrimAfter() {
      if (!c.opt("writable", 0)) c.build_pool->trim();
    }
  } trim_after{c};
  double t0 = now_s();
  const bool keep = c.opt("writable", 0) != 0;
  // option build_trace: per-phase wall time on stderr (the stream drained at each mark)
  const bool trace = c.opt("build_trace", 0) != 0;
  double tmark = t0;
  if (trace) {
    g_alloc_clock.alloc_ns = 0;
    g_alloc_clock.free_ns = 0;
    g_alloc_clock.allocs = 0;
  }
  auto phase = [&](const char* name) {
    if (!trace) return;
    NBG_HIP(hipStreamSynchronize(c.stream));
    const double t = now_s();
    const int64_t an = g_alloc_clock.alloc_ns.exchange(0), fn = g_alloc_clock.free_ns.exchange(0);
    const int64_t na = g_alloc_clock.allocs.exchange(0);
    fprintf(stderr, "[nbg build] %-22s %8.3f s  (hipMalloc %lld x %.3f s, hipFree %.3f s)\n", name, t - tmark,
            (long long)na, an * 1e-9, fn * 1e-9);
    tmark = t;
  };
  for (auto& kv : c.edges)
    if (kv.second.rmat_stream) {
      finalize_rmat_stream(c, kv.second);
      c.has_log = false;
      c.ws_tmp.release();
      c.finalized = true;
      c.build_seconds += now_s() - t0;
      return;
    }
  // 1. referenced vids (src/dst of every staged tuple), sign-flipped for an unsigned sort.  One
  // staged column at a time is sorted, deduplicated and merged into the running set, so the peak
  // is 16 B per tuple of the largest column (not 16 B per vid reference of the whole snapshot:
  // 69 GB for a writable RMAT-26, whose stages stay resident beside it)
  DevBuf vA;
  int64_t nuniq = 0;
  for (auto& kv : c.edges) {
    for (Staging* s : {&kv.second.out_stage, &kv.second.in_stage}) {
      if (s->n == 0) continue;
      for (const DevBuf* colp : {&s->src, &s->dst}) {
        const int64_t n = s->n;
        DevBuf t1, t2;
        t1.alloc(size_t(n) * 8);
        t2.alloc(size_t(n) * 8);
        k_flip_copy<<<grid_for(n), 256, 0, c.stream>>>(colp->as<int64_t>(), t1.as<uint64_t>(), n, 0, 0, 0, 0);
        radix_keys<uint64_t>(c, t1.as<uint64_t>(), t2.as<uint64_t>(), n, 64);
        const int64_t m = unique_sorted<uint64_t>(c, t2.as<uint64_t>(), t1.as<uint64_t>(), n);
        t2.release();
        if (nuniq == 0) {
          vA = std::move(t1);
          nuniq = m;
          continue;
        }
        DevBuf cat, srt;
        cat.alloc(size_t(nuniq + m) * 8);
        srt.alloc(size_t(nuniq + m) * 8);
        NBG_HIP(hipMemcpyAsync(cat.p, vA.p, size_t(nuniq) * 8, hipMemcpyDeviceToDevice, c.stream));
        NBG_HIP(hipMemcpyAsync(cat.as<uint64_t>() + nuniq, t1.p, size_t(m) * 8, hipMemcpyDeviceToDevice, c.stream));
        t1.release();
        vA.release();
        radix_keys<uint64_t>(c, cat.as<uint64_t>(), srt.as<uint64_t>(), nuniq + m, 64);
        nuniq = unique_sorted<uint64_t>(c, srt.as<uint64_t>(), cat.as<uint64_t>(), nuniq + m);
        vA = std::move(cat);
      }
    }
  }
  if (!vA.p) vA.alloc(8);
  phase("vertex set");
  // 2. owned set and global table
  std::vector<int64_t> counts(size_t(c.world), 0);
  DevBuf owned;
  int64_t n_owned = nuniq;
  if (!c.sharded) {
    owned = std::move(vA);
  } else {
    // every rank sends the vids it references to their owners; owners union.  (Simple form:
    // allgather the unique referenced sets, filter by owner; fine for build-time volumes.)
    int64_t mine = nuniq;
    std::vector<int64_t> sizes(size_t(c.world));
    DevBuf dsz, dall;
    dsz.alloc(8 * size_t(c.world));
    DevBuf dmine;
    dmine.alloc(8);
    NBG_HIP(hipMemcpyAsync(dmine.p, &mine, 8, hipMemcpyHostToDevice, c.stream));
    comm_allgather_bytes(c, dmine.p, 8, dsz.p);
    NBG_HIP(hipMemcpyAsync(sizes.data(), dsz.p, 8 * size_t(c.world), hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    int64_t mx = *std::max_element(sizes.begin(), sizes.end());
    DevBuf sendb, recvb;
    sendb.alloc(size_t(std::max<int64_t>(mx, 1)) * 8);
    recvb.alloc(size_t(std::max<int64_t>(mx, 1)) * 8 * size_t(c.world));
    if (nuniq) NBG_HIP(hipMemcpyAsync(sendb.p, vA.p, size_t(nuniq) * 8, hipMemcpyDeviceToDevice, c.stream));
    comm_allgather_bytes(c, sendb.p, size_t(mx) * 8, recvb.p);
    // compact all received sets, keep owned, sort + unique
    DevBuf all;
    int64_t tot = 0;
    for (auto s : sizes) tot += s;
    all.alloc(size_t(std::max<int64_t>(tot, 1)) * 8);
    int64_t p2 = 0;
    for (int r = 0; r < c.world; r++) {
      if (sizes[size_t(r)])
        NBG_HIP(hipMemcpyAsync(all.as<uint64_t>() + p2, recvb.as<uint64_t>() + size_t(r) * size_t(mx),
                               size_t(sizes[size_t(r)]) * 8, hipMemcpyDeviceToDevice, c.stream));
      p2 += sizes[size_t(r)];
    }
    DevBuf flag, sel, cnt;
    flag.alloc(size_t(std::max<int64_t>(tot, 1)));
    sel.alloc(size_t(std::max<int64_t>(tot, 1)) * 8);
    cnt.alloc(8);
    k_owned_only<<<grid_for(tot), 256, 0, c.stream>>>(all.as<uint64_t>(), tot, c.num_parts, c.world, c.rank, flag.as<uint8_t>());
    size_t tb = 0;
    NBG_HIP(rocprim::select(nullptr, tb, all.as<uint64_t>(), flag.as<uint8_t>(), sel.as<uint64_t>(), cnt.as<uint64_t>(), size_t(tot), c.stream));
    c.ws_tmp.ensure(tb);
    NBG_HIP(rocprim::select(c.ws_tmp.p, tb, all.as<uint64_t>(), flag.as<uint8_t>(), sel.as<uint64_t>(), cnt.as<uint64_t>(), size_t(tot), c.stream));
    uint64_t ns = 0;
    NBG_HIP(hipMemcpyAsync(&ns, cnt.p, 8, hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
    DevBuf s2;
    s2.alloc(size_t(std::max<uint64_t>(ns, 1)) * 8);
    radix_keys<uint64_t>(c, sel.as<uint64_t>(), s2.as<uint64_t>(), int64_t(ns), 64);
    owned.alloc(size_t(std::max<uint64_t>(ns, 1)) * 8);
    n_owned = ns ? unique_sorted<uint64_t>(c, s2.as<uint64_t>(), owned.as<uint64_t>(), int64_t(ns)) : 0;
    vA.release();
  }
  order_by_degree(c, owned, n_owned);
  phase("degree order");
  // 3. counts -> base; allgather owned tables into vid_of (rank-major; within a rank by
  // descending out-degree, or by vid with degree_order=0)
  if (!c.sharded) {
    counts[0] = n_owned;
  } else {
    DevBuf dsz, dmine;
    dsz.alloc(8 * size_t(c.world));
    dmine.alloc(8);
    NBG_HIP(hipMemcpyAsync(dmine.p, &n_owned, 8, hipMemcpyHostToDevice, c.stream));
    comm_allgather_bytes(c, dmine.p, 8, dsz.p);
    NBG_HIP(hipMemcpyAsync(counts.data(), dsz.p, 8 * size_t(c.world), hipMemcpyDeviceToHost, c.stream));
    NBG_HIP(hipStreamSynchronize(c.stream));
  }
  // owner ranges padded to 64 vertices: every rank's slice of a frontier bitmap starts on a
  // 64-bit word, so bitmap slices are exchanged without shifting (holes have no edges)
  // A writable snapshot on several ranks also reserves growth room in every owner range (option
  // grow_room_pct of the rank's vertices, at least 1024): a merge commit places new vertices
  // there without moving any rank's range (extend_vertex_map_ranks); a batch that overflows
  // some rank's room takes the full rebuild, which reserves room again.
  const int64_t room_pct = keep && c.sharded ? std::max<int64_t>(0, c.opt("grow_room_pct", 10)) : 0;
  c.base.assign(size_t(c.world) + 1, 0);
  c.counts = counts;
  for (int r = 0; r < c.world; r++) {
    const int64_t room = room_pct ? std::max<int64_t>(1024, counts[size_t(r)] * room_pct / 100) : 0;
    c.base[size_t(r) + 1] = c.base[size_t(r)] + ((counts[size_t(r)] + room + 63) / 64) * 64;
  }
  c.n_global = c.base[size_t(c.world)];
  c.n_vertices = 0;
  for (auto x : counts) c.n_vertices += x;
  if (c.n_global >= (int64_t(1) << 31)) throw Error(NBG_E_UNSUPPORTED, "more than 2^31 vertices");
  c.vid_of.alloc(size_t(std::max<int64_t>(c.n_global, 1)) * 8);
  fill<int64_t>(c, c.vid_of.as<int64_t>(), INT64_MIN, c.n_global);
  if (!c.sharded) {
    if (n_owned) k_unflip<<<grid_for(n_owned), 256, 0, c.stream>>>(owned.as<uint64_t>(), c.vid_of.as<int64_t>(), n_owned);
  } else {
    int64_t mx = *std::max_element(counts.begin(), counts.end());
    DevBuf sendb, recvb;
    sendb.alloc(size_t(std::max<int64_t>(mx, 1)) * 8);
    recvb.alloc(size_t(std::max<int64_t>(mx, 1)) * 8 * size_t(c.world));
    if (n_owned) NBG_HIP(hipMemcpyAsync(sendb.p, owned.p, size_t(n_owned) * 8, hipMemcpyDeviceToDevice, c.stream));
    comm_allgather_bytes(c, sendb.p, size_t(mx) * 8, recvb.p);
    for (int r = 0; r < c.world; r++)
      if (counts[size_t(r)])
        k_unflip<<<grid_for(counts[size_t(r)]), 256, 0, c.stream>>>(recvb.as<uint64_t>() + size_t(r) * size_t(mx),
                                                                     c.vid_of.as<int64_t>() + c.base[size_t(r)],
                                                                     counts[size_t(r)]);
  }
  owned.release();
  // 4. hash table vid -> gidx
  int64_t cap = 1024;
  while (cap < 2 * std::max<int64_t>(c.n_global, 1)) cap <<= 1;
  c.ht_cap = cap;
  c.ht_keys.alloc(size_t(cap) * 8);
  c.ht_vals.alloc(size_t(cap) * 4);
  fill<int64_t>(c, c.ht_keys.as<int64_t>(), INT64_MIN, cap);
  DevBuf dmin;
  dmin.alloc(4);
  int32_t neg = -1;
  NBG_HIP(hipMemcpyAsync(dmin.p, &neg, 4, hipMemcpyHostToDevice, c.stream));
  for (int r = 0; r < c.world; r++)
    if (counts[size_t(r)])
      k_ht_insert<<<grid_for(counts[size_t(r)]), 256, 0, c.stream>>>(
          c.ht_keys.as<int64_t>(), c.ht_vals.as<int32_t>(), uint64_t(cap - 1), c.vid_of.as<int64_t>() + c.base[size_t(r)],
          counts[size_t(r)], c.base[size_t(r)], dmin.as<int32_t>());
  NBG_HIP(hipMemcpyAsync(&c.ht_min_gidx, dmin.p, 4, hipMemcpyDeviceToHost, c.stream));
  NBG_HIP(hipStreamSynchronize(c.stream));
  c.ht_has_min = c.ht_min_gidx >= 0;
  phase("vertex map + hash");
  build_tag_columns(c);
  phase("tag columns");
  // 5. bytewise order rank of every vertex (for CSR row order = RocksDB key order)
  DevBuf brank = bytewise_ranks(c);
  phase("bytewise ranks");
  // 6. CSRs
  for (auto& kv : c.edges) {
    EdgeSpace& es = kv.second;
    build_csr(c, es.out_stage, es.fields, true, es.out, brank.as<uint32_t>(), !keep, &es.ord[0]);
    phase("out CSR");
    build_csr(c, es.in_stage, es.fields, false, es.in, brank.as<uint32_t>(), !keep, &es.ord[1]);
    phase("in CSR");
    if (c.opt("bottom_up", 1)) build_transpose(c, es);
    phase("transpose + slabs");
  }
  if (!keep) {
    c.heap.release();
    c.heap_used = 0;
  } else {
    c.brank = std::move(brank);  // the batch keys of a merge commit
    for (auto& kv : c.tags) kv.second.committed_n = kv.second.stage.n;
  }
  c.has_log = keep;
  c.ws_tmp.release();
  NBG_HIP(hipStreamSynchronize(c.stream));
  c.finalized = true;
  c.build_seconds += now_s() - t0;
}

}  // namespace nbg
