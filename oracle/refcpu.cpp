// oracle/refcpu.cpp -- TEST INFRASTRUCTURE ONLY (see refcpu.h).
//
// CPU restatement of the reference neighbour-expansion path.  Every function names the
// reference file:line it follows (paths relative to the reference repo root).  It is a
// restatement, not a copy: the reference needs folly/fbthrift/rocksdb/boost, none of which
// exist here, so each piece is re-expressed with the C++ standard library.
#include "refcpu.h"
#include "rmat_def.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <variant>
#include <vector>

namespace refcpu {

// ------------------------------------------------------------------------------------------
// Types (src/common/base/ThriftTypes.h:21-26, src/interface/common.thrift:30-46)
// ------------------------------------------------------------------------------------------
enum SupportedType : int32_t {
  T_UNKNOWN = 0, T_BOOL = 1, T_INT = 2, T_VID = 3, T_FLOAT = 4, T_DOUBLE = 5, T_STRING = 6,
  T_TIMESTAMP = 21
};
enum ErrorCode : int32_t {
  SUCCEEDED = 0, E_LEADER_CHANGED = -11, E_SPACE_NOT_FOUND = -13, E_PART_NOT_FOUND = -14,
  E_EDGE_PROP_NOT_FOUND = -21, E_TAG_PROP_NOT_FOUND = -22, E_IMPROPER_DATA_TYPE = -23,
  E_INVALID_FILTER = -31, E_UNKNOWN = -100
};
enum PropOwner : int32_t { SOURCE = 1, DEST = 2, EDGE = 3 };

// VariantType = boost::variant<int64_t, double, bool, std::string> (src/common/base/Base.h:140)
using Val = std::variant<int64_t, double, bool, std::string>;

// boost::variant ordering: which() first, then value (used by RelationalExpression,
// src/common/filter/Expressions.cpp:891-933).  `>`/`<=`/`>=` are derived from `<`.
static bool vlt(const Val& a, const Val& b) {
  if (a.index() != b.index()) return a.index() < b.index();
  switch (a.index()) {
    case 0: return std::get<0>(a) < std::get<0>(b);
    case 1: return std::get<1>(a) < std::get<1>(b);
    case 2: return std::get<2>(a) < std::get<2>(b);
    default: return std::get<3>(a) < std::get<3>(b);
  }
}
static bool veq(const Val& a, const Val& b) {
  if (a.index() != b.index()) return false;
  switch (a.index()) {
    case 0: return std::get<0>(a) == std::get<0>(b);
    case 1: return std::get<1>(a) == std::get<1>(b);
    case 2: return std::get<2>(a) == std::get<2>(b);
    default: return std::get<3>(a) == std::get<3>(b);
  }
}

struct Status {
  bool ok = true;
  std::string msg;
  static Status Err(std::string m) { return Status{false, std::move(m)}; }
};
struct OptVal {
  Status st;
  Val v;
  bool ok() const { return st.ok; }
};
static OptVal OK(Val v) { return OptVal{Status{}, std::move(v)}; }
static OptVal ERR(std::string m) { return OptVal{Status::Err(std::move(m)), Val{int64_t(0)}}; }

// ------------------------------------------------------------------------------------------
// folly::encodeVarint / decodeVarint (LEB128 of uint64) as called from
// src/dataman/RowWriter.inl:40, RowReader.inl:66, RowSetWriter.cpp:24, RowSetReader.cpp:37
// ------------------------------------------------------------------------------------------
static size_t encodeVarint(uint64_t v, uint8_t* buf) {
  size_t n = 0;
  while (v >= 0x80) {
    buf[n++] = uint8_t(0x80 | (v & 0x7f));
    v >>= 7;
  }
  buf[n++] = uint8_t(v);
  return n;
}
// returns bytes consumed, or -1 on a truncated / over-long varint (folly throws)
static int decodeVarint(const uint8_t* p, size_t avail, uint64_t& out) {
  uint64_t v = 0;
  for (size_t i = 0; i < 10 && i < avail; i++) {
    v |= uint64_t(p[i] & 0x7f) << (7 * i);
    if (!(p[i] & 0x80)) {
      out = v;
      return int(i + 1);
    }
  }
  return -1;
}

// ------------------------------------------------------------------------------------------
// Keys (src/common/base/NebulaKeyUtils.h:14-21, NebulaKeyUtils.cpp:24-49)
// ------------------------------------------------------------------------------------------
static constexpr size_t kEdgeLen = 4 + 8 + 4 + 8 + 8 + 8;
static constexpr size_t kVertexLen = 4 + 8 + 4 + 8;
template <typename T>
static void put(std::string& s, T v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <typename T>
static T get(const char* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}
static std::string edgeKey(int32_t part, int64_t src, int32_t type, int64_t rank, int64_t dst,
                           int64_t ver) {
  std::string k;
  k.reserve(kEdgeLen);
  put(k, part); put(k, src); put(k, type); put(k, rank); put(k, dst); put(k, ver);
  return k;
}
[[maybe_unused]] static std::string vertexKey(int32_t part, int64_t vid, int32_t tag, int64_t ver) {
  std::string k;
  put(k, part); put(k, vid); put(k, tag); put(k, ver);
  return k;
}
static std::string edgePrefix(int32_t part, int64_t src, int32_t type) {
  std::string k;
  put(k, part); put(k, src); put(k, type);
  return k;
}
static std::string vertexPrefix(int32_t part, int64_t vid, int32_t tag) {
  std::string k;
  put(k, part); put(k, vid); put(k, tag);
  return k;
}
static int64_t keySrc(const char* k) { return get<int64_t>(k + 4); }
static int32_t keyType(const char* k) { return get<int32_t>(k + 12); }
static int64_t keyRank(const char* k) { return get<int64_t>(k + 16); }
static int64_t keyDst(const char* k) { return get<int64_t>(k + 24); }

// ------------------------------------------------------------------------------------------
// Schemas (meta SchemaProviderIf / SchemaWriter / ResultSchemaProvider stand-in)
// ------------------------------------------------------------------------------------------
struct Field {
  std::string name;
  int32_t type;
};
struct Schema {
  int32_t ver = 0;
  std::vector<Field> fields;
  int fieldIndex(const std::string& n) const {
    for (size_t i = 0; i < fields.size(); i++)
      if (fields[i].name == n) return int(i);
    return -1;
  }
};
using SchemaPtr = std::shared_ptr<const Schema>;

// ------------------------------------------------------------------------------------------
// RowWriter (src/dataman/RowWriter.cpp:49-75, RowWriter.inl:14-43, RowWriter.h:143-160).
// Only the paths the hot path exercises: schemaless writer (PropsCollector, storage
// responses) and schema writer with types fixed by a schema (GoExecutor setupInterimResult).
// ------------------------------------------------------------------------------------------
struct RowWriter {
  SchemaPtr schema;             // null -> schemaless, types follow the values written
  std::vector<int32_t> types;   // schemaless column types (SchemaWriter)
  std::string cord;
  int64_t colNum = 0;
  std::vector<int64_t> blockOffsets;

  explicit RowWriter(SchemaPtr s = nullptr) : schema(std::move(s)) {}
  int32_t colType(int32_t deflt) const {
    if (schema && colNum < int64_t(schema->fields.size())) return schema->fields[colNum].type;
    return deflt;
  }
  void cleanup(int32_t t) {  // RW_CLEAN_UP_WRITE (RowWriter.h:143-160)
    colNum++;
    if (colNum != 0 && (colNum >> 4 << 4) == colNum) blockOffsets.push_back(int64_t(cord.size()));
    if (!schema) types.push_back(t);
  }
  void writeInt(uint64_t v) {
    uint8_t b[10];
    size_t n = encodeVarint(v, b);
    cord.append(reinterpret_cast<char*>(b), n);
  }
  RowWriter& operator<<(int64_t v) {  // RowWriter.inl:14-33
    int32_t t = colType(T_INT);
    switch (t) {
      case T_INT: writeInt(uint64_t(v)); break;
      case T_VID:
      case T_TIMESTAMP: put(cord, uint64_t(v)); break;
      default: writeInt(0); break;  // "Incompatible value type \"int\""
    }
    cleanup(T_INT);
    return *this;
  }
  RowWriter& operator<<(double v) {  // RowWriter.cpp:153-171
    int32_t t = colType(T_DOUBLE);
    switch (t) {
      case T_FLOAT: put(cord, float(v)); break;
      case T_DOUBLE: put(cord, v); break;
      default: put(cord, 0.0); break;
    }
    cleanup(T_DOUBLE);
    return *this;
  }
  RowWriter& writeFloat(float v) {  // what operator<<(double) writes under a FLOAT column
    put(cord, v);
    cleanup(T_FLOAT);
    return *this;
  }
  RowWriter& operator<<(bool v) {  // RowWriter.cpp:115-129
    int32_t t = colType(T_BOOL);
    if (t == T_BOOL) cord.push_back(char(v)); else cord.push_back(char(0));
    cleanup(T_BOOL);
    return *this;
  }
  RowWriter& operator<<(const std::string& v) {  // RowWriter.cpp:178-195
    int32_t t = colType(T_STRING);
    if (t == T_STRING) {
      writeInt(v.size());
      cord += v;
    } else {
      writeInt(0);
    }
    cleanup(T_STRING);
    return *this;
  }
  RowWriter& operator<<(const Val& v) {
    switch (v.index()) {
      case 0: return *this << std::get<0>(v);
      case 1: return *this << std::get<1>(v);
      case 2: return *this << std::get<2>(v);
      default: return *this << std::get<3>(v);
    }
  }
  static int64_t occupied(uint64_t v) {  // calcOccupiedBytes RowWriter.cpp:85-92
    int64_t b = 0;
    do {
      b++;
      v >>= 8;
    } while (v);
    return b;
  }
  int64_t size() const {  // RowWriter.cpp:27-38
    return int64_t(cord.size()) + occupied(cord.size()) * int64_t(blockOffsets.size()) + 1 +
           ((schema && schema->ver > 0) ? occupied(uint64_t(schema->ver)) : 0);
  }
  std::string encode() const {  // RowWriter.cpp:49-75 (writers here never Skip)
    std::string out;
    int64_t offBytes = occupied(cord.size());
    char header = char(offBytes - 1);
    int32_t ver = schema ? schema->ver : 0;
    if (ver > 0) {
      int64_t vb = occupied(uint64_t(ver));
      header |= char(vb << 5);
      out.push_back(header);
      out.append(reinterpret_cast<const char*>(&ver), size_t(vb));
    } else {
      out.push_back(header);
    }
    for (auto off : blockOffsets) out.append(reinterpret_cast<const char*>(&off), size_t(offBytes));
    out += cord;
    return out;
  }
  SchemaPtr outSchema() const {  // SchemaWriter built alongside a schemaless writer
    auto s = std::make_shared<Schema>();
    for (size_t i = 0; i < types.size(); i++)
      s->fields.push_back(Field{"Column" + std::to_string(i + 1), types[i]});
    return s;
  }
};

// ------------------------------------------------------------------------------------------
// RowReader (src/dataman/RowReader.cpp:173-341, RowReader.inl:59-68, RowReader.h:92-148)
// ------------------------------------------------------------------------------------------
static int32_t rowSchemaVer(const std::string& row) {  // RowReader.cpp:173-199
  if (row.empty()) return 0;
  const uint8_t* it = reinterpret_cast<const uint8_t*>(row.data());
  size_t verBytes = size_t(*it++) >> 5;
  int32_t ver = 0;
  if (verBytes > 0) {
    if (verBytes + 1 > row.size()) return 0;
    for (size_t i = 0; i < verBytes; i++) ver |= int32_t(uint32_t(*it++) << (8 * i));
  }
  return ver;
}

struct RowReader {
  SchemaPtr schema;
  const uint8_t* data = nullptr;  // first field
  size_t len = 0;
  bool valid = false;
  std::vector<int64_t> offsets;   // offsets_[i] = start of field i (-1 unknown)

  RowReader(const char* row, size_t rowLen, SchemaPtr s) : schema(std::move(s)) {
    // processHeader (RowReader.cpp:218-263)
    if (rowLen == 0 || !schema) return;
    const uint8_t* it = reinterpret_cast<const uint8_t*>(row);
    int numBytesForOffset = (*it & 0x07) + 1;
    int verBytes = *it++ >> 5;
    it += verBytes;
    uint32_t numFields = uint32_t(schema->fields.size());
    uint32_t numOffsets = numFields >> 4;
    if (size_t(numBytesForOffset) * numOffsets + verBytes + 1 > rowLen) return;
    offsets.assign(numFields + 1, -1);
    offsets[0] = 0;
    for (uint32_t i = 0; i < numOffsets; i++) {
      int64_t off = 0;
      for (int j = 0; j < numBytesForOffset; j++) off |= int64_t(uint64_t(*it++) << (8 * j));
      offsets[16 * (i + 1)] = off;
    }
    size_t headerLen = size_t(it - reinterpret_cast<const uint8_t*>(row));
    data = it;
    len = rowLen - headerLen;
    offsets[numFields] = int64_t(len);
    valid = true;
  }
  int readInteger(int64_t off, int64_t& v) const {
    if (off < 0 || size_t(off) > len) return -1;
    uint64_t u;
    int n = decodeVarint(data + off, len - size_t(off), u);
    if (n > 0) v = int64_t(u);
    return n;
  }
  // skipToNext (RowReader.cpp:276-341); returns offset of field index+1 or -1
  int64_t skipToNext(int64_t index, int64_t off) const {
    if (offsets[index + 1] >= 0) return offsets[index + 1];
    switch (schema->fields[index].type) {
      case T_BOOL: off += 1; break;
      case T_INT: {
        int64_t v;
        int n = readInteger(off, v);
        if (n <= 0) return -1;
        off += n;
        break;
      }
      case T_FLOAT: off += 4; break;
      case T_DOUBLE: off += 8; break;
      case T_STRING: {
        int64_t sl;
        int n = readInteger(off, sl);
        if (n <= 0) return -1;
        off += n + sl;
        break;
      }
      case T_VID:
      case T_TIMESTAMP: off += 8; break;
      default: return -1;
    }
    if (off > int64_t(len)) return -1;
    const_cast<RowReader*>(this)->offsets[index + 1] = off;
    return off;
  }
  int64_t skipToField(int64_t index) const {  // RowReader.cpp:344-368 (semantics)
    if (index >= int64_t(schema->fields.size())) return -1;
    int64_t base = index & ~int64_t(15);
    int64_t off = offsets[base];
    for (int64_t i = base; i < index; i++) {
      off = skipToNext(i, off);
      if (off < 0) return -1;
    }
    return off;
  }
  // getPropByIndex (RowReader.h:150-205); getPropByName = index lookup + this.
  OptVal getByIndex(int idx) const {
    if (!valid || idx < 0 || idx >= int(schema->fields.size())) return ERR("bad index");
    int64_t off = skipToField(idx);
    if (off < 0) return ERR("data invalid");
    switch (schema->fields[idx].type) {
      case T_BOOL: {
        if (size_t(off) + 1 > len) return ERR("data invalid");
        return OK(Val{bool(data[off] != 0)});
      }
      case T_INT: {
        int64_t v;
        if (readInteger(off, v) <= 0) return ERR("data invalid");
        return OK(Val{v});
      }
      case T_VID:
      case T_TIMESTAMP: {
        if (size_t(off) + 8 > len) return ERR("data invalid");
        return OK(Val{get<int64_t>(reinterpret_cast<const char*>(data + off))});
      }
      case T_FLOAT: {
        if (size_t(off) + 4 > len) return ERR("data invalid");
        return OK(Val{double(get<float>(reinterpret_cast<const char*>(data + off)))});
      }
      case T_DOUBLE: {
        if (size_t(off) + 8 > len) return ERR("data invalid");
        return OK(Val{get<double>(reinterpret_cast<const char*>(data + off))});
      }
      case T_STRING: {
        int64_t sl;
        int n = readInteger(off, sl);
        if (n <= 0 || off + n + sl > int64_t(len)) return ERR("data invalid");
        return OK(Val{std::string(reinterpret_cast<const char*>(data + off + n), size_t(sl))});
      }
      default: return ERR("unknown type");
    }
  }
  OptVal getByName(const std::string& name) const {
    if (!schema) return ERR("no schema");
    return getByIndex(schema->fieldIndex(name));
  }
};

// RowSetWriter (src/dataman/RowSetWriter.cpp:21-37) / RowSetReader (RowSetReader.cpp:32-51)
static void rowSetAdd(std::string& rs, const std::string& row) {
  uint8_t b[10];
  size_t n = encodeVarint(uint64_t(row.size()), b);
  rs.append(reinterpret_cast<char*>(b), n);
  rs += row;
}
template <typename F>
static void rowSetForEach(const std::string& rs, const SchemaPtr& schema, F f) {
  size_t off = 0;
  while (off < rs.size()) {
    uint64_t rl;
    int n = decodeVarint(reinterpret_cast<const uint8_t*>(rs.data()) + off,
                         std::min<size_t>(10, rs.size() - off), rl);
    if (n <= 0) return;
    RowReader r(rs.data() + off + size_t(n), size_t(rl), schema);
    f(r);
    off += size_t(n) + size_t(rl);
  }
}

// ------------------------------------------------------------------------------------------
// Expressions: decode (src/common/filter/Expressions.cpp:84-107 + each ::decode) and eval
// (Expressions.cpp:762-1011, Expressions.h:151-205).
// ------------------------------------------------------------------------------------------
enum Kind : uint8_t {
  kUnknown = 0, kPrimary, kFunctionCall, kUnary, kTypeCasting, kArithmetic, kRelational,
  kLogical, kSourceProp, kEdgeRank, kEdgeDstId, kEdgeSrcId, kEdgeType, kAliasProp, kEdgeProp,
  kVariableProp, kDestProp, kInputProp, kMax
};
enum UnaryOp : uint8_t { PLUS, NEGATE, NOT };
enum ArithOp : uint8_t { ADD, SUB, MUL, DIV, MOD };
enum RelOp : uint8_t { LT, LE, GT, GE, EQ, NE };
enum LogicOp : uint8_t { AND, OR };

struct Getters {
  std::function<OptVal(const std::string&, const std::string&)> getAliasProp;
  std::function<OptVal(const std::string&, const std::string&)> getSrcTagProp;
  std::function<OptVal(const std::string&, const std::string&)> getDstTagProp;
  std::function<OptVal(const std::string&)> getInputProp;
  std::function<OptVal(const std::string&)> getVariableProp;
};

struct Expr {
  uint8_t kind = kUnknown;
  uint8_t op = 0;
  Val prim{int64_t(0)};
  bool hasProp = false;           // decoded kEdge* from storage lose prop_ (Expressions.h:449-460)
  std::string alias, prop;
  std::unique_ptr<Expr> l, r;
};
using ExprPtr = std::unique_ptr<Expr>;

struct DecodeError {};
struct Cursor {
  const char* p;
  const char* e;
  void need(size_t n) const {
    if (p + n > e) throw DecodeError{};
  }
  uint8_t u8() { need(1); return uint8_t(*p++); }
  uint16_t u16() { need(2); uint16_t v = get<uint16_t>(p); p += 2; return v; }
  std::string str() {
    uint16_t n = u16();
    need(n);
    std::string s(p, n);
    p += n;
    return s;
  }
};

// graphdSemantics: an AST built by the graphd parser carries prop_ for _dst/_src/_rank/_type;
// the storage-side decode leaves it unset (P20).
static ExprPtr decodeExpr(Cursor& c, bool graphdSemantics);
static ExprPtr makeAndDecode(uint8_t kind, Cursor& c, bool g) {
  auto x = std::make_unique<Expr>();
  x->kind = kind;
  switch (kind) {
    case kPrimary: {  // Expressions.cpp:500-530
      uint8_t which = c.u8();
      switch (which) {
        case 0: c.need(8); x->prim = get<int64_t>(c.p); c.p += 8; break;
        case 1: c.need(8); x->prim = get<double>(c.p); c.p += 8; break;
        case 2: c.need(1); x->prim = bool(*c.p++ != 0); break;
        case 3: x->prim = c.str(); break;
        default: throw DecodeError{};
      }
      break;
    }
    case kUnary: {  // Expressions.cpp:632-638 (requires 2 bytes)
      c.need(2);
      x->op = c.u8();
      x->l = makeAndDecode(c.u8(), c, g);
      break;
    }
    case kArithmetic:
    case kRelational:
    case kLogical: {  // Expressions.cpp:836-845, 945-954, 1023-1032
      c.need(2);
      x->op = c.u8();
      x->l = makeAndDecode(c.u8(), c, g);
      c.need(1);
      x->r = makeAndDecode(c.u8(), c, g);
      break;
    }
    case kSourceProp:
    case kAliasProp:
    case kVariableProp:
    case kDestProp:
      x->alias = c.str();
      x->prop = c.str();
      x->hasProp = true;
      break;
    case kInputProp:
      x->prop = c.str();
      x->hasProp = true;
      break;
    case kEdgeRank:
    case kEdgeDstId:
    case kEdgeSrcId:
    case kEdgeType:
      x->alias = c.str();
      x->hasProp = g;
      x->prop = kind == kEdgeRank ? "_rank" : kind == kEdgeDstId ? "_dst"
              : kind == kEdgeSrcId ? "_src" : "_type";
      break;
    case kFunctionCall:  // functions are rejected by checkExp (QueryBaseProcessor.inl:143-145)
    case kTypeCasting:   // TypeCastingExpression has no encoding (Expressions.cpp:749-751)
    default:
      throw DecodeError{};
  }
  return x;
}
static ExprPtr decodeExpr(Cursor& c, bool g) { return makeAndDecode(c.u8(), c, g); }
static ExprPtr decodeBuffer(const uint8_t* buf, size_t n, bool g) {  // Expression::decode :92-107
  try {
    Cursor c{reinterpret_cast<const char*>(buf), reinterpret_cast<const char*>(buf) + n};
    auto x = decodeExpr(c, g);
    if (c.p != c.e) return nullptr;
    return x;
  } catch (const DecodeError&) {
    return nullptr;
  }
}

static bool asBool(const Val& v) {  // Expressions.h:162-176 (string -> empty())
  switch (v.index()) {
    case 0: return std::get<0>(v) != 0;
    case 1: return std::get<1>(v) != 0.0;
    case 2: return std::get<2>(v);
    default: return std::get<3>(v).empty();
  }
}
static double asDouble(const Val& v) {
  return v.index() == 0 ? double(std::get<0>(v)) : std::get<1>(v);
}
static bool isArith(const Val& v) { return v.index() == 0 || v.index() == 1; }
static bool almostEqual(double a, double b) { return std::abs(a - b) < 1e-8; }

static OptVal eval(const Expr& x, const Getters& g) {
  switch (x.kind) {
    case kPrimary: return OK(x.prim);
    case kAliasProp:
    case kEdgeRank:
    case kEdgeDstId:
    case kEdgeSrcId:
      if (!x.hasProp) return ERR("edge expression without prop");  // reference: null deref
      return g.getAliasProp(x.alias, x.prop);
    case kEdgeType: return OK(Val{x.alias});  // EdgeTypeExpression::eval returns *alias_
    case kSourceProp: return g.getSrcTagProp(x.alias, x.prop);
    case kDestProp: return g.getDstTagProp(x.alias, x.prop);
    case kInputProp: return g.getInputProp(x.prop);
    case kVariableProp: return g.getVariableProp(x.prop);
    case kUnary: {  // Expressions.cpp:606-623
      auto v = eval(*x.l, g);
      if (v.ok()) {
        if (x.op == PLUS) return v;
        if (x.op == NEGATE) {
          if (v.v.index() == 0) return OK(Val{int64_t(-uint64_t(std::get<0>(v.v)))});
          if (v.v.index() == 1) return OK(Val{-std::get<1>(v.v)});
        } else {
          return OK(Val{!asBool(v.v)});
        }
      }
      return ERR("unary");
    }
    case kArithmetic: {  // Expressions.cpp:762-824
      auto lv = eval(*x.l, g);
      auto rv = eval(*x.r, g);
      if (!lv.ok()) return lv;
      if (!rv.ok()) return rv;
      const Val& l = lv.v;
      const Val& r = rv.v;
      bool dbl = l.index() == 1 || r.index() == 1;
      switch (x.op) {
        case ADD:
          if (isArith(l) && isArith(r)) {
            if (dbl) return OK(Val{asDouble(l) + asDouble(r)});
            return OK(Val{int64_t(uint64_t(std::get<0>(l)) + uint64_t(std::get<0>(r)))});
          }
          if (l.index() == 3 && r.index() == 3) return OK(Val{std::get<3>(l) + std::get<3>(r)});
          break;
        case SUB:
          if (isArith(l) && isArith(r)) {
            if (dbl) return OK(Val{asDouble(l) - asDouble(r)});
            return OK(Val{int64_t(uint64_t(std::get<0>(l)) - uint64_t(std::get<0>(r)))});
          }
          break;
        case MUL:
          if (isArith(l) && isArith(r)) {
            if (dbl) return OK(Val{asDouble(l) * asDouble(r)});
            return OK(Val{int64_t(uint64_t(std::get<0>(l)) * uint64_t(std::get<0>(r)))});
          }
          break;
        case DIV:
          if (isArith(l) && isArith(r)) {
            if (dbl) return OK(Val{asDouble(l) / asDouble(r)});
            // integer division by zero is UB in the reference (SIGFPE); surfaced as an error
            if (std::get<0>(r) == 0) return ERR("division by zero");
            if (std::get<0>(r) == -1) return OK(Val{int64_t(-uint64_t(std::get<0>(l)))});
            return OK(Val{std::get<0>(l) / std::get<0>(r)});
          }
          break;
        case MOD:
          if (l.index() == 0 && r.index() == 0) {
            if (std::get<0>(r) == 0) return ERR("modulo by zero");
            if (std::get<0>(r) == -1) return OK(Val{int64_t(0)});
            return OK(Val{std::get<0>(l) % std::get<0>(r)});
          }
          break;
      }
      return ERR("arithmetic type");
    }
    case kRelational: {  // Expressions.cpp:891-933
      auto lv = eval(*x.l, g);
      auto rv = eval(*x.r, g);
      if (!lv.ok()) return lv;
      if (!rv.ok()) return rv;
      const Val& l = lv.v;
      const Val& r = rv.v;
      switch (x.op) {
        case LT: return OK(Val{vlt(l, r)});
        case LE: return OK(Val{!vlt(r, l)});
        case GT: return OK(Val{vlt(r, l)});
        case GE: return OK(Val{!vlt(l, r)});
        case EQ:
          if (isArith(l) && isArith(r) && (l.index() == 1 || r.index() == 1))
            return OK(Val{almostEqual(asDouble(l), asDouble(r))});
          return OK(Val{veq(l, r)});
        case NE:
          if (isArith(l) && isArith(r) && (l.index() == 1 || r.index() == 1))
            return OK(Val{!almostEqual(asDouble(l), asDouble(r))});
          return OK(Val{!veq(l, r)});
      }
      return ERR("Wrong operator");
    }
    case kLogical: {  // Expressions.cpp:988-1011 (both sides evaluated)
      auto lv = eval(*x.l, g);
      auto rv = eval(*x.r, g);
      if (!lv.ok()) return lv;
      if (!rv.ok()) return rv;
      if (x.op == AND) {
        if (!asBool(lv.v)) return OK(Val{false});
        return OK(Val{asBool(rv.v)});
      }
      if (asBool(lv.v)) return OK(Val{true});
      return OK(Val{asBool(rv.v)});
    }
    default: return ERR("unsupported expression");
  }
}

// props referenced by an expression (Expression::prepare -> ExpressionContext)
struct ExprRefs {
  std::set<std::pair<std::string, std::string>> alias, srcTag, dstTag;
  bool input = false, variable = false;
};
static void collectRefs(const Expr& x, ExprRefs& refs) {
  switch (x.kind) {
    case kAliasProp:
    case kEdgeRank:
    case kEdgeDstId:
    case kEdgeSrcId:
    case kEdgeType: refs.alias.emplace(x.alias, x.prop); break;
    case kSourceProp: refs.srcTag.emplace(x.alias, x.prop); break;
    case kDestProp: refs.dstTag.emplace(x.alias, x.prop); break;
    case kInputProp: refs.input = true; break;
    case kVariableProp: refs.variable = true; break;
    default: break;
  }
  if (x.l) collectRefs(*x.l, refs);
  if (x.r) collectRefs(*x.r, refs);
}

// ------------------------------------------------------------------------------------------
// KV store (NebulaStore/RocksEngine read side: src/kvstore/RocksEngine.cpp:191-230)
// Arena-backed, one sorted run per part; prefix() = lower_bound + starts_with.
// ------------------------------------------------------------------------------------------
struct KVRef {
  uint64_t koff;
  uint32_t klen;
  uint64_t voff;
  uint32_t vlen;
  uint64_t seq;
};
struct Part {
  std::string arena;
  std::vector<KVRef> kvs;
  bool sorted = true;
  const char* key(const KVRef& r) const { return arena.data() + r.koff; }
  const char* val(const KVRef& r) const { return arena.data() + r.voff; }
};

}  // namespace refcpu

struct ora_store {
  int32_t numParts = 0;
  std::vector<refcpu::Part> parts;  // index = partId (1..numParts; 0 unused unless tests)
  std::map<std::pair<int32_t, int32_t>, refcpu::SchemaPtr> edgeSchemas;  // (type, ver)
  std::map<int32_t, int32_t> edgeLatest;
  std::map<std::pair<int32_t, int32_t>, refcpu::SchemaPtr> tagSchemas;
  std::map<int32_t, int32_t> tagLatest;
  std::map<std::string, int32_t> tagByName;
  // $- / $var input rows of the next ora_go call (InterimResult rows, column name -> values)
  std::vector<std::string> inNames;
  std::vector<std::vector<refcpu::Val>> inCols;
  size_t inRows = 0;
  std::map<int32_t, std::string> edgeNames;
  uint64_t seq = 0;
};

struct ora_result {
  int32_t code = 0;
  std::string error;
  std::vector<std::vector<refcpu::Val>> rows;
  std::vector<std::vector<bool>> present;  // cell present (columns may be skipped)
  std::vector<int64_t> rowVertex;
  // get_bound response
  std::vector<std::pair<int32_t, int32_t>> failed;  // (part, code)
  struct V {
    int64_t vid;
    std::string vertexData, edgeData;
    std::vector<refcpu::Val> tagVals;
    std::vector<bool> tagPresent;
    size_t nrows = 0;
  };
  std::vector<V> vertices;
  std::vector<refcpu::Field> edgeSchema, vertexSchema;
};

namespace refcpu {

static SchemaPtr edgeSchema(const ora_store* st, int32_t type, int32_t ver) {
  auto it = st->edgeSchemas.find({type, ver});
  return it == st->edgeSchemas.end() ? nullptr : it->second;
}
static SchemaPtr latestEdgeSchema(const ora_store* st, int32_t type) {
  auto it = st->edgeLatest.find(type);
  return it == st->edgeLatest.end() ? nullptr : edgeSchema(st, type, it->second);
}
static SchemaPtr tagSchema(const ora_store* st, int32_t tag, int32_t ver) {
  auto it = st->tagSchemas.find({tag, ver});
  return it == st->tagSchemas.end() ? nullptr : it->second;
}
static SchemaPtr latestTagSchema(const ora_store* st, int32_t tag) {
  auto it = st->tagLatest.find(tag);
  return it == st->tagLatest.end() ? nullptr : tagSchema(st, tag, it->second);
}

enum KvCode { KV_OK = 0, KV_PART_NOT_FOUND = 1 };
// Iterate keys with the given prefix in bytewise order (RocksPrefixIter, RocksEngine.h:55-86)
template <typename F>
static KvCode prefixScan(const ora_store* st, int32_t part, const std::string& prefix, F f) {
  if (part < 0 || part >= int32_t(st->parts.size())) return KV_PART_NOT_FOUND;
  const Part& p = st->parts[size_t(part)];
  auto lo = std::lower_bound(p.kvs.begin(), p.kvs.end(), prefix, [&](const KVRef& r,
                                                                     const std::string& k) {
    int c = memcmp(p.key(r), k.data(), std::min<size_t>(r.klen, k.size()));
    return c < 0 || (c == 0 && r.klen < k.size());
  });
  for (auto it = lo; it != p.kvs.end(); ++it) {
    if (it->klen < prefix.size() || memcmp(p.key(*it), prefix.data(), prefix.size()) != 0) break;
    if (!f(p.key(*it), size_t(it->klen), p.val(*it), size_t(it->vlen))) break;
  }
  return KV_OK;
}

static int32_t toErr(KvCode c) {  // BaseProcessor.inl:14-27
  return c == KV_OK ? SUCCEEDED : c == KV_PART_NOT_FOUND ? E_PART_NOT_FOUND : E_UNKNOWN;
}

// ------------------------------------------------------------------------------------------
// QueryBaseProcessor / QueryBoundProcessor restatement
// (src/storage/QueryBaseProcessor.inl:37-505, QueryBoundProcessor.cpp:16-106,
//  CommonUtils.h:18-121, Collector.h:34-63)
// ------------------------------------------------------------------------------------------
enum PropInKey { PIK_NONE = 0, PIK_SRC, PIK_DST, PIK_TYPE, PIK_RANK };
struct PropCtx {
  std::string name;
  int32_t owner = EDGE;
  int32_t type = T_UNKNOWN;
  int pik = PIK_NONE;
  bool returned = false;
  bool filtered = false;
  std::string tagOrEdgeName;
  // QueryStatsProcessor state (CommonUtils.h:50-53): the request's stat, the column's position
  // in the request, and the collector's sum / count.  sum_ is boost::variant<int64_t, double>
  // initialised to int64 0, so collectDouble's boost::get<double>(sum_) throws (bad_get): kept
  // as a flag.
  int32_t stat = 0;
  int retIndex = -1;
  mutable int64_t sum = 0;
  mutable int32_t count = 0;
  mutable bool badGet = false;
};
struct TagCtx {
  int32_t tagId = 0;
  std::vector<PropCtx> props;
  std::unordered_map<std::string, int> nameIndex;
};
struct FilterCtx {
  std::map<std::pair<std::string, std::string>, Val> tagFilters;
};

struct BoundProcessor {
  const ora_store* st;
  bool outBound;
  bool stats = false;            // QueryStatsProcessor instead of QueryBoundProcessor
  bool onlyVertexProps = false;  // QueryVertexPropsProcessor (QueryVertexPropsProcessor.cpp:16-28)
  const int32_t* statTypes = nullptr;
  int32_t edgeType = 0;
  std::vector<TagCtx> tagCtxs;
  std::vector<PropCtx> edgeProps;
  ExprPtr exp;
  std::mutex lock;  // BaseProcessor::lock_ (BaseProcessor.h:82)
  std::vector<ora_result::V> vertices;

  // checkAndBuildContexts (QueryBaseProcessor.inl:37-136)
  int32_t checkAndBuildContexts(int32_t et, const ora_prop_def* cols, size_t ncols,
                                const uint8_t* filter, size_t flen) {
    edgeType = et;
    std::unordered_map<int32_t, size_t> tagIndex;
    int index = 0;
    for (size_t i = 0; i < ncols; i++) {
      PropCtx prop;
      prop.name = cols[i].name;
      prop.owner = cols[i].owner;
      prop.stat = statTypes ? statTypes[i] : 0;
      if (cols[i].owner == SOURCE || cols[i].owner == DEST) {
        auto schema = latestTagSchema(st, cols[i].tag_id);
        if (!schema) return E_TAG_PROP_NOT_FOUND;
        int fi = schema->fieldIndex(prop.name);
        if (fi < 0) return E_IMPROPER_DATA_TYPE;
        prop.type = schema->fields[size_t(fi)].type;
        if (prop.stat && !validOperation(prop.type, prop.stat)) return E_IMPROPER_DATA_TYPE;
        prop.retIndex = index++;
        prop.returned = true;
        auto it = tagIndex.find(cols[i].tag_id);
        if (it == tagIndex.end()) {
          TagCtx tc;
          tc.tagId = cols[i].tag_id;
          tc.props.push_back(prop);
          tagCtxs.push_back(std::move(tc));
          tagIndex.emplace(cols[i].tag_id, tagCtxs.size() - 1);
        } else {
          tagCtxs[it->second].props.push_back(prop);
        }
      } else {
        static const std::map<std::string, int> kPik = {
            {"_src", PIK_SRC}, {"_dst", PIK_DST}, {"_type", PIK_TYPE}, {"_rank", PIK_RANK}};
        auto pk = kPik.find(prop.name);
        if (pk != kPik.end()) {
          prop.pik = pk->second;
          prop.type = T_INT;
        } else if (outBound) {
          auto schema = latestEdgeSchema(st, edgeType);
          if (!schema) return E_EDGE_PROP_NOT_FOUND;
          int fi = schema->fieldIndex(prop.name);
          if (fi < 0) return E_IMPROPER_DATA_TYPE;
          prop.type = schema->fields[size_t(fi)].type;
        } else {
          continue;  // "InBound has none props, skip it!"
        }
        if (prop.stat && !validOperation(prop.type, prop.stat)) return E_IMPROPER_DATA_TYPE;
        prop.retIndex = index++;
        prop.returned = true;
        edgeProps.push_back(prop);
      }
    }
    if (flen > 0) {
      exp = decodeBuffer(filter, flen, /*graphdSemantics=*/false);
      if (!exp) return E_INVALID_FILTER;
      if (!checkExp(*exp)) return E_INVALID_FILTER;
    }
    return SUCCEEDED;
  }

  // validOperation (QueryBaseProcessor.inl:18-35): SUM / AVG only over numeric types
  static bool validOperation(int32_t t, int32_t stat) {
    if (stat == 1 || stat == 3)
      return t == T_INT || t == T_VID || t == T_TIMESTAMP || t == T_FLOAT || t == T_DOUBLE;
    return true;
  }

  // StatsCollector (Collector.h:66-94), under BaseProcessor::lock_
  void statCollect(const PropCtx& prop, const Val& v) {
    std::lock_guard<std::mutex> lg(lock);
    switch (v.index()) {
      case 0: prop.sum += std::get<int64_t>(v); break;  // collectInt64
      case 1: prop.badGet = true; break;                 // collectDouble: boost::get<double> throws
      default: break;                                    // collectBool / collectString
    }
    prop.count++;
  }

  // checkExp (QueryBaseProcessor.inl:138-245)
  bool checkExp(const Expr& x) {
    switch (x.kind) {
      case kPrimary: return true;
      case kFunctionCall: return false;
      case kUnary:
      case kTypeCasting: return checkExp(*x.l);
      case kArithmetic:
      case kRelational:
      case kLogical: return checkExp(*x.l) && checkExp(*x.r);
      case kSourceProp: {
        auto tn = st->tagByName.find(x.alias);
        if (tn == st->tagByName.end()) return false;
        int32_t tagId = tn->second;
        auto schema = latestTagSchema(st, tagId);
        if (!schema) return false;
        int fi = schema->fieldIndex(x.prop);
        if (fi < 0) return false;
        for (auto& tc : tagCtxs) {
          if (tc.tagId == tagId) {
            PropCtx* found = nullptr;
            auto ni = tc.nameIndex.find(x.prop);
            if (ni != tc.nameIndex.end()) found = &tc.props[size_t(ni->second)];
            if (found == nullptr) {
              pushFilterProp(tc, x.alias, x.prop, schema->fields[size_t(fi)].type);
            } else if (!found->filtered) {
              found->filtered = true;
              found->tagOrEdgeName = x.alias;
            }
            return true;
          }
        }
        TagCtx tc;
        tc.tagId = tagId;
        pushFilterProp(tc, x.alias, x.prop, schema->fields[size_t(fi)].type);
        tagCtxs.push_back(std::move(tc));
        return true;
      }
      case kEdgeRank:
      case kEdgeDstId:
      case kEdgeSrcId:
      case kEdgeType: return true;
      case kAliasProp:
      case kEdgeProp: {
        if (!outBound) return false;
        if (edgeType == -1) return false;
        auto schema = latestEdgeSchema(st, edgeType);
        if (!schema) return false;
        return schema->fieldIndex(x.prop) >= 0;
      }
      default: return false;
    }
  }
  static void pushFilterProp(TagCtx& tc, const std::string& tag, const std::string& prop,
                             int32_t type) {  // CommonUtils.h:98-110
    PropCtx pc;
    pc.name = prop;
    pc.type = type;
    pc.owner = SOURCE;
    pc.filtered = true;
    pc.tagOrEdgeName = tag;
    tc.props.push_back(pc);
    tc.nameIndex.emplace(prop, int(tc.props.size()) - 1);
  }

  // collectProps (QueryBaseProcessor.inl:247-306) into a schemaless RowWriter
  void collectProps(const RowReader* reader, const char* key, const std::vector<PropCtx>& props,
                    FilterCtx* fctx, RowWriter& w) {
    for (auto& prop : props) {
      Val kv{int64_t(0)};
      switch (prop.pik) {
        case PIK_SRC: kv = keySrc(key); break;
        case PIK_DST: kv = keyDst(key); break;
        case PIK_TYPE: kv = int64_t(keyType(key)); break;
        case PIK_RANK: kv = keyRank(key); break;
        default: break;
      }
      if (prop.pik != PIK_NONE) {
        if (stats) statCollect(prop, kv);
        else w << kv;
        continue;
      }
      if (reader != nullptr) {
        auto res = reader->getByName(prop.name);
        if (!res.ok()) continue;  // "Skip the bad value for prop"
        if ((prop.owner == SOURCE || prop.owner == DEST) && prop.filtered)
          fctx->tagFilters.emplace(std::make_pair(prop.tagOrEdgeName, prop.name), res.v);
        if (prop.returned) {
          if (stats) statCollect(prop, res.v);
          else w << res.v;
        }
      }
    }
  }

  // collectVertexProps (QueryBaseProcessor.inl:309-333)
  KvCode collectVertexProps(int32_t part, int64_t vid, int32_t tagId,
                            const std::vector<PropCtx>& props, FilterCtx* fctx, RowWriter& w) {
    bool first = true;
    auto code = prefixScan(st, part, vertexPrefix(part, vid, tagId),
                           [&](const char* k, size_t, const char* v, size_t vl) {
      if (!first) return false;
      first = false;
      std::string row(v, vl);
      auto schema = tagSchema(st, tagId, rowSchemaVer(row));
      RowReader reader(row.data(), row.size(), schema);
      collectProps(&reader, k, props, fctx, w);
      return false;
    });
    return code;
  }

  // collectEdgeProps (QueryBaseProcessor.inl:335-405), including the firstLoop quirk:
  // firstLoop only clears after an edge is emitted, so versions of a filtered-out edge are
  // re-examined until the first emit.
  template <typename Proc>
  KvCode collectEdgeProps(int32_t part, int64_t vid, int32_t et, FilterCtx* fctx, Proc proc) {
    int64_t lastRank = -1, lastDst = 0;
    bool firstLoop = true;
    return prefixScan(st, part, edgePrefix(part, vid, et),
                      [&](const char* k, size_t, const char* v, size_t vl) {
      int64_t rank = keyRank(k), dst = keyDst(k);
      if (!firstLoop && rank == lastRank && lastDst == dst) return true;
      lastRank = rank;
      lastDst = dst;
      std::unique_ptr<RowReader> reader;
      std::string row;
      if (outBound && vl != 0) {
        row.assign(v, vl);
        auto schema = edgeSchema(st, et, rowSchemaVer(row));
        reader = std::make_unique<RowReader>(row.data(), row.size(), schema);
        if (exp) {
          std::lock_guard<std::mutex> lg(lock);
          Getters g;
          g.getAliasProp = [&](const std::string&, const std::string& prop) -> OptVal {
            auto res = reader->getByName(prop);
            if (!res.ok()) return ERR("Invalid Prop");
            return res;
          };
          g.getSrcTagProp = [&](const std::string& tag, const std::string& prop) -> OptVal {
            auto it = fctx->tagFilters.find({tag, prop});
            if (it == fctx->tagFilters.end()) return ERR("Invalid Tag Filter");
            return OK(it->second);
          };
          g.getDstTagProp = [&](const std::string&, const std::string&) -> OptVal {
            return OK(Val{false});
          };
          g.getInputProp = [&](const std::string&) -> OptVal { return OK(Val{false}); };
          g.getVariableProp = [&](const std::string&) -> OptVal { return OK(Val{false}); };
          auto value = eval(*exp, g);
          if (value.ok() && !asBool(value.v)) return true;  // filtered out
        }
      }
      proc(reader.get(), k);
      firstLoop = false;
      return true;
    });
  }

  // processVertex (QueryBoundProcessor.cpp:16-72; QueryStatsProcessor.cpp:69-99 for stats)
  KvCode processVertex(int32_t part, int64_t vid) {
    FilterCtx fctx;
    if (stats) {
      RowWriter unused;
      for (auto& tc : tagCtxs) {
        auto code = collectVertexProps(part, vid, tc.tagId, tc.props, &fctx, unused);
        if (code != KV_OK) return code;
      }
      if (!edgeProps.empty())
        return collectEdgeProps(part, vid, edgeType, &fctx, [&](const RowReader* reader, const char* key) {
          RowWriter w;
          collectProps(reader, key, edgeProps, &fctx, w);
        });
      return KV_OK;
    }
    ora_result::V vresp;
    vresp.vid = vid;
    if (!tagCtxs.empty()) {
      RowWriter w;
      for (auto& tc : tagCtxs) {
        auto code = collectVertexProps(part, vid, tc.tagId, tc.props, &fctx, w);
        if (code != KV_OK) return code;
      }
      if (w.size() > 1) vresp.vertexData = w.encode();
    }
    if (onlyVertexProps) {  // QueryBoundProcessor.cpp:33-37
      std::lock_guard<std::mutex> lg(lock);
      vertices.push_back(std::move(vresp));
      return KV_OK;
    }
    if (!edgeProps.empty()) {
      std::string rs;
      auto code = collectEdgeProps(part, vid, edgeType, &fctx,
                                   [&](const RowReader* reader, const char* key) {
        RowWriter w;
        collectProps(reader, key, edgeProps, &fctx, w);
        rowSetAdd(rs, w.encode());
      });
      if (code != KV_OK) return code;
      if (!rs.empty()) {
        vresp.edgeData = std::move(rs);
        std::lock_guard<std::mutex> lg(lock);
        vertices.push_back(std::move(vresp));
      }
    }
    return KV_OK;
  }
};

// getBucketsNum + genBuckets (QueryBaseProcessor.inl:425-460)
static std::vector<std::vector<std::pair<int32_t, int64_t>>> genBuckets(
    const std::vector<std::pair<int32_t, std::vector<int64_t>>>& parts, int32_t maxHandlers,
    int32_t minPerBucket) {
  int32_t n = 0;
  for (auto& pv : parts) n += int32_t(pv.second.size());
  int32_t nb = std::min(std::max(1, n / minPerBucket), maxHandlers);
  std::vector<std::vector<std::pair<int32_t, int64_t>>> buckets;
  buckets.resize(size_t(nb));
  int32_t per = n / nb, left = n % nb;
  int32_t bi = -1;
  size_t thres = size_t(per);
  for (auto& pv : parts) {
    for (auto vid : pv.second) {
      if (bi < 0 || buckets[size_t(bi)].size() >= thres) {
        ++bi;
        thres = size_t(bi < left ? per + 1 : per);
      }
      buckets[size_t(bi)].emplace_back(pv.first, vid);
    }
  }
  return buckets;
}

// QueryBaseProcessor::process (QueryBaseProcessor.inl:462-505) + onProcessFinished
// (QueryBoundProcessor.cpp:75-106).  Buckets run concurrently, one thread each.
static int32_t processRequest(BoundProcessor& proc,
                           const std::vector<std::pair<int32_t, std::vector<int64_t>>>& parts,
                           const ora_prop_def* cols, size_t ncols, const uint8_t* filter,
                           size_t flen, int32_t maxHandlers, int32_t minPerBucket,
                           ora_result* out) {
  int32_t rc = proc.checkAndBuildContexts(proc.edgeType, cols, ncols, filter, flen);
  if (rc != SUCCEEDED) {
    for (auto& p : parts) out->failed.emplace_back(p.first, rc);
    return rc;
  }
  auto buckets = genBuckets(parts, maxHandlers, minPerBucket);
  std::vector<std::vector<std::pair<int32_t, KvCode>>> codes(buckets.size());
  std::vector<std::thread> threads;
  for (size_t b = 0; b < buckets.size(); b++) {
    threads.emplace_back([&, b] {
      for (auto& pv : buckets[b]) codes[b].emplace_back(pv.first, proc.processVertex(pv.first, pv.second));
    });
  }
  for (auto& t : threads) t.join();
  std::set<int32_t> failedParts;
  for (auto& bc : codes)
    for (auto& pc : bc)
      if (pc.second != KV_OK && failedParts.insert(pc.first).second)
        out->failed.emplace_back(pc.first, toErr(pc.second));
  for (auto& tc : proc.tagCtxs)
    for (auto& p : tc.props)
      if (p.returned) out->vertexSchema.push_back(Field{p.name, p.type});
  for (auto& p : proc.edgeProps) out->edgeSchema.push_back(Field{p.name, p.type});
  out->vertices = std::move(proc.vertices);
  return SUCCEEDED;
}

static SchemaPtr toSchema(const std::vector<Field>& f) {
  auto s = std::make_shared<Schema>();
  s->fields = f;
  return s;
}

// Partition of a vid (StorageClient.cpp:10-11, 238-243)
static int32_t partOf(int64_t vid, int32_t numParts) {
  return int32_t(uint64_t(vid) % uint64_t(numParts) + 1);
}

// StorageClient::getNeighbors (StorageClient.cpp:94-131) + clusterIdsToHosts
// (StorageClient.h:182-196): one processor per host (host = part % H, pickHosts
// CreateSpaceProcessor.cpp:77-90), hosts served concurrently.
static std::vector<ora_result> getNeighbors(const ora_store* st, const std::vector<int64_t>& vids,
                                            int32_t edgeType, const std::vector<ora_prop_def>& cols,
                                            int32_t numHosts, int32_t maxHandlers,
                                            int32_t minPerBucket, bool onlyVertexProps = false) {
  std::map<int32_t, std::map<int32_t, std::vector<int64_t>>> clusters;  // host -> part -> ids
  for (auto v : vids) {
    int32_t part = partOf(v, st->numParts);
    clusters[part % numHosts][part].push_back(v);
  }
  std::vector<ora_result> resps(clusters.size());
  std::vector<std::thread> threads;
  size_t i = 0;
  for (auto& c : clusters) {
    threads.emplace_back([&, i, hostParts = &c.second] {
      std::vector<std::pair<int32_t, std::vector<int64_t>>> parts(hostParts->begin(),
                                                                 hostParts->end());
      BoundProcessor proc;
      proc.st = st;
      proc.outBound = edgeType > 0;
      proc.edgeType = edgeType;
      proc.onlyVertexProps = onlyVertexProps;
      processRequest(proc, parts, cols.data(), cols.size(), nullptr, 0, maxHandlers,
                     minPerBucket, &resps[i]);
    });
    i++;
  }
  for (auto& t : threads) t.join();
  return resps;
}

}  // namespace refcpu

using namespace refcpu;

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

void ora_go_set_inputs(ora_store* st, size_t nRows, size_t nCols, const char* const* names,
                       const int32_t* types, const void* const* cols, const int64_t* const* strOffsets) {
  st->inNames.clear();
  st->inCols.clear();
  st->inRows = nRows;
  for (size_t c = 0; c < nCols; c++) {
    st->inNames.push_back(names[c]);
    std::vector<Val> vals;
    for (size_t r = 0; r < nRows; r++) {
      switch (types[c]) {
        case T_DOUBLE: vals.push_back(Val{static_cast<const double*>(cols[c])[r]}); break;
        case T_BOOL: vals.push_back(Val{static_cast<const uint8_t*>(cols[c])[r] != 0}); break;
        case T_STRING: {
          const int64_t* o = strOffsets[c];
          vals.push_back(Val{std::string(static_cast<const char*>(cols[c]) + o[r], size_t(o[r + 1] - o[r]))});
          break;
        }
        default: vals.push_back(Val{static_cast<const int64_t*>(cols[c])[r]});
      }
    }
    st->inCols.push_back(std::move(vals));
  }
}

ora_store* ora_store_new(int32_t numParts) {
  auto* st = new ora_store();
  st->numParts = numParts;
  st->parts.resize(size_t(numParts) + 1);
  return st;
}
void ora_store_free(ora_store* st) { delete st; }

void ora_store_put_batch(ora_store* st, int32_t part, const uint8_t* kb, const uint64_t* koff,
                         const uint8_t* vb, const uint64_t* voff, size_t n) {
  if (part < 0) return;
  if (size_t(part) >= st->parts.size()) st->parts.resize(size_t(part) + 1);
  Part& p = st->parts[size_t(part)];
  for (size_t i = 0; i < n; i++) {
    KVRef r;
    r.koff = p.arena.size();
    r.klen = uint32_t(koff[i + 1] - koff[i]);
    p.arena.append(reinterpret_cast<const char*>(kb + koff[i]), r.klen);
    r.voff = p.arena.size();
    r.vlen = uint32_t(voff[i + 1] - voff[i]);
    p.arena.append(reinterpret_cast<const char*>(vb + voff[i]), r.vlen);
    r.seq = st->seq++;
    p.kvs.push_back(r);
  }
  p.sorted = false;
}

static void finalizePart(Part& p) {
  if (p.sorted) return;
  std::sort(p.kvs.begin(), p.kvs.end(), [&](const KVRef& a, const KVRef& b) {
    int c = memcmp(p.key(a), p.key(b), std::min(a.klen, b.klen));
    if (c != 0) return c < 0;
    if (a.klen != b.klen) return a.klen < b.klen;
    return a.seq < b.seq;
  });
  // identical keys: keep the last write (largest seq)
  std::vector<KVRef> out;
  out.reserve(p.kvs.size());
  for (size_t i = 0; i < p.kvs.size(); i++) {
    if (i + 1 < p.kvs.size() && p.kvs[i].klen == p.kvs[i + 1].klen &&
        memcmp(p.key(p.kvs[i]), p.key(p.kvs[i + 1]), p.kvs[i].klen) == 0)
      continue;
    out.push_back(p.kvs[i]);
  }
  p.kvs.swap(out);
  p.sorted = true;
}

void ora_store_finalize(ora_store* st) {
  std::atomic<size_t> next{0};
  unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  std::vector<std::thread> ts;
  for (unsigned t = 0; t < nt; t++)
    ts.emplace_back([&] {
      for (size_t i = next++; i < st->parts.size(); i = next++) finalizePart(st->parts[i]);
    });
  for (auto& t : ts) t.join();
}

size_t ora_store_num_keys(const ora_store* st) {
  size_t n = 0;
  for (auto& p : st->parts) n += p.kvs.size();
  return n;
}

size_t ora_store_part_size(const ora_store* st, int32_t part, size_t* kbytes, size_t* vbytes) {
  *kbytes = *vbytes = 0;
  if (part < 0 || size_t(part) >= st->parts.size()) return 0;
  const Part& p = st->parts[size_t(part)];
  for (auto& r : p.kvs) {
    *kbytes += r.klen;
    *vbytes += r.vlen;
  }
  return p.kvs.size();
}
void ora_store_dump_part(const ora_store* st, int32_t part, uint8_t* kb, uint64_t* koff, uint8_t* vb,
                         uint64_t* voff) {
  const Part& p = st->parts[size_t(part)];
  uint64_t ko = 0, vo = 0;
  size_t i = 0;
  for (auto& r : p.kvs) {
    koff[i] = ko;
    voff[i] = vo;
    memcpy(kb + ko, p.key(r), r.klen);
    memcpy(vb + vo, p.val(r), r.vlen);
    ko += r.klen;
    vo += r.vlen;
    i++;
  }
  koff[i] = ko;
  voff[i] = vo;
}

void ora_schema_set_edge(ora_store* st, int32_t et, int32_t ver, int32_t nf,
                         const char* const* names, const int32_t* types) {
  auto s = std::make_shared<Schema>();
  s->ver = ver;
  for (int32_t i = 0; i < nf; i++) s->fields.push_back(Field{names[i], types[i]});
  st->edgeSchemas[{et, ver}] = s;
  auto it = st->edgeLatest.find(et);
  if (it == st->edgeLatest.end() || it->second < ver) st->edgeLatest[et] = ver;
}
void ora_schema_set_edge_name(ora_store* st, int32_t et, const char* name) {
  st->edgeNames[et] = name;
}
void ora_schema_set_tag(ora_store* st, int32_t tag, const char* tagName, int32_t ver, int32_t nf,
                        const char* const* names, const int32_t* types) {
  auto s = std::make_shared<Schema>();
  s->ver = ver;
  for (int32_t i = 0; i < nf; i++) s->fields.push_back(Field{names[i], types[i]});
  st->tagSchemas[{tag, ver}] = s;
  auto it = st->tagLatest.find(tag);
  if (it == st->tagLatest.end() || it->second < ver) st->tagLatest[tag] = ver;
  if (tagName) st->tagByName[tagName] = tag;
}

size_t ora_encode_row(const int32_t* tags, const int64_t* iv, const double* dv,
                      const char* const* sv, int32_t ncols, uint8_t* out, size_t cap) {
  RowWriter w;
  for (int32_t i = 0; i < ncols; i++) {
    switch (tags[i]) {
      case T_INT: w << iv[i]; break;
      case T_DOUBLE: w << dv[i]; break;
      case T_FLOAT: w.writeFloat(float(dv[i])); break;  // a FLOAT schema column: 4 bytes
      case T_BOOL: w << bool(iv[i] != 0); break;
      default: w << std::string(sv[i]); break;
    }
  }
  std::string e = w.encode();
  if (e.size() <= cap) memcpy(out, e.data(), e.size());
  return e.size();
}
size_t ora_encode_varint(uint64_t v, uint8_t* out) { return encodeVarint(v, out); }
size_t ora_edge_key(int32_t part, int64_t src, int32_t type, int64_t rank, int64_t dst,
                    int64_t ver, uint8_t* out) {
  auto k = edgeKey(part, src, type, rank, dst, ver);
  memcpy(out, k.data(), k.size());
  return k.size();
}

int64_t ora_rmat_vid(uint64_t idx, uint64_t seed) { return rmatVid(idx, seed); }

void ora_rmat_edges(int32_t scale, int32_t ef, uint64_t seed, int64_t* src, int64_t* dst,
                    int64_t* weight) {
  uint64_t E = uint64_t(ef) << scale;
  for (uint64_t i = 0; i < E; i++) {
    uint64_t u, v;
    rmatEdge(seed, scale, i, u, v);
    src[i] = rmatVid(u, seed);
    dst[i] = rmatVid(v, seed);
    if (weight) weight[i] = rmatWeight(src[i], dst[i], seed);
  }
}

// Write the RMAT graph the way INSERT EDGE does (InsertEdgeExecutor.cpp:143-162 +
// AddEdgesProcessor.cpp:15-31): out-edge (type, rank 0, row{weight}) and in-edge
// (-type, empty value).  `versions` > 1 writes extra versions whose weights differ, with the
// bytewise-first version carrying the canonical weight (the multi-version stress variant).
void ora_rmat_load(ora_store* st, int32_t scale, int32_t ef, uint64_t seed, int32_t et,
                   int32_t versions, int32_t threads) {
  uint64_t E = uint64_t(ef) << scale;
  int32_t P = st->numParts;
  if (threads <= 0) threads = 1;
  // per-thread, per-part staging to keep put order deterministic per thread
  std::vector<std::vector<std::string>> keys(size_t(threads) * size_t(P + 1)),
      vals(size_t(threads) * size_t(P + 1));
  std::vector<std::thread> ts;
  for (int32_t t = 0; t < threads; t++) {
    ts.emplace_back([&, t] {
      uint64_t lo = E * uint64_t(t) / uint64_t(threads), hi = E * uint64_t(t + 1) / uint64_t(threads);
      for (uint64_t i = lo; i < hi; i++) {
        uint64_t u, v;
        rmatEdge(seed, scale, i, u, v);
        int64_t s = rmatVid(u, seed), d = rmatVid(v, seed);
        int64_t w = rmatWeight(s, d, seed);
        int32_t ps = partOf(s, P), pd = partOf(d, P);
        for (int32_t ver = 0; ver < versions; ver++) {
          // bytewise-first version = smallest LE bytes: INT64_MAX - 1 - ver has LE low byte
          // decreasing with ver, so ver = versions-1 is first; it carries the weight.
          int64_t version = INT64_MAX - 1 - ver;
          RowWriter rw;
          rw << int64_t(ver == versions - 1 ? w : (w + 1 + ver) % 1000);
          size_t slot = size_t(t) * size_t(P + 1);
          keys[slot + size_t(ps)].push_back(edgeKey(ps, s, et, 0, d, version));
          vals[slot + size_t(ps)].push_back(rw.encode());
          keys[slot + size_t(pd)].push_back(edgeKey(pd, d, -et, 0, s, version));
          vals[slot + size_t(pd)].push_back(std::string());
        }
      }
    });
  }
  for (auto& t : ts) t.join();
  for (int32_t t = 0; t < threads; t++) {
    for (int32_t p = 1; p <= P; p++) {
      auto& K = keys[size_t(t) * size_t(P + 1) + size_t(p)];
      auto& V = vals[size_t(t) * size_t(P + 1) + size_t(p)];
      Part& part = st->parts[size_t(p)];
      for (size_t i = 0; i < K.size(); i++) {
        KVRef r;
        r.koff = part.arena.size();
        r.klen = uint32_t(K[i].size());
        part.arena += K[i];
        r.voff = part.arena.size();
        r.vlen = uint32_t(V[i].size());
        part.arena += V[i];
        r.seq = st->seq++;
        part.kvs.push_back(r);
      }
      part.sorted = false;
      std::vector<std::string>().swap(K);
      std::vector<std::string>().swap(V);
    }
  }
  ora_store_finalize(st);
}

int32_t ora_gen_buckets(const int32_t* parts, const int64_t* vids, size_t n, int32_t maxH,
                        int32_t minPer, int32_t* sizes) {
  std::vector<std::pair<int32_t, std::vector<int64_t>>> pv;
  for (size_t i = 0; i < n; i++) {
    if (pv.empty() || pv.back().first != parts[i]) pv.push_back({parts[i], {}});
    pv.back().second.push_back(vids[i]);
  }
  auto b = genBuckets(pv, maxH, minPer);
  for (size_t i = 0; i < b.size(); i++) sizes[i] = int32_t(b[i].size());
  return int32_t(b.size());
}

ora_result* ora_get_bound(ora_store* st, int32_t et, int32_t inBound, const int32_t* parts,
                          const int64_t* vids, size_t n, const uint8_t* filter, size_t flen,
                          const ora_prop_def* cols, size_t ncols, int32_t maxH, int32_t minPer) {
  auto* out = new ora_result();
  // request.parts: map<part, list<vid>> in first-appearance order of parts
  std::vector<std::pair<int32_t, std::vector<int64_t>>> pv;
  std::map<int32_t, size_t> idx;
  for (size_t i = 0; i < n; i++) {
    auto it = idx.find(parts[i]);
    if (it == idx.end()) {
      idx[parts[i]] = pv.size();
      pv.push_back({parts[i], {}});
      it = idx.find(parts[i]);
    }
    pv[it->second].second.push_back(vids[i]);
  }
  BoundProcessor proc;
  proc.st = st;
  proc.outBound = !inBound;
  proc.edgeType = et;
  processRequest(proc, pv, cols, ncols, filter, flen, maxH, minPer, out);
  // decode rows for the accessors
  auto es = toSchema(out->edgeSchema);
  auto vs = toSchema(out->vertexSchema);
  for (auto& v : out->vertices) {
    if (!v.vertexData.empty()) {
      RowReader r(v.vertexData.data(), v.vertexData.size(), vs);
      for (size_t c = 0; c < out->vertexSchema.size(); c++) {
        auto x = r.getByIndex(int(c));
        v.tagVals.push_back(x.v);
        v.tagPresent.push_back(x.ok());
      }
    }
    rowSetForEach(v.edgeData, es, [&](const RowReader& r) {
      std::vector<Val> row;
      std::vector<bool> pres;
      for (size_t c = 0; c < out->edgeSchema.size(); c++) {
        auto x = r.getByIndex(int(c));
        row.push_back(x.v);
        pres.push_back(x.ok());
      }
      out->rows.push_back(std::move(row));
      out->present.push_back(std::move(pres));
      out->rowVertex.push_back(v.vid);
      v.nrows++;
    });
  }
  return out;
}

// QueryStatsProcessor (src/storage/QueryStatsProcessor.cpp:16-125): one row, one column per
// returned prop in request order (retIndex): SUM -> INT (int64 sum), COUNT -> INT, AVG -> DOUBLE
// (sum / count, NaN for no rows).  A double value reaching the int64-initialised sum variant
// throws in the reference (boost::bad_get): reported as code -1003 (E_UNSUPPORTED).
ora_result* ora_bound_stats(ora_store* st, int32_t et, int32_t inBound, const int32_t* parts,
                            const int64_t* vids, size_t n, const uint8_t* filter, size_t flen,
                            const ora_prop_def* cols, const int32_t* statTypes, size_t ncols,
                            int32_t maxH, int32_t minPer) {
  auto* out = new ora_result();
  std::vector<std::pair<int32_t, std::vector<int64_t>>> pv;
  std::map<int32_t, size_t> idx;
  for (size_t i = 0; i < n; i++) {
    auto it = idx.find(parts[i]);
    if (it == idx.end()) {
      idx[parts[i]] = pv.size();
      pv.push_back({parts[i], {}});
      it = idx.find(parts[i]);
    }
    pv[it->second].second.push_back(vids[i]);
  }
  BoundProcessor proc;
  proc.st = st;
  proc.outBound = !inBound;
  proc.edgeType = et;
  proc.stats = true;
  proc.statTypes = statTypes;
  if (processRequest(proc, pv, cols, ncols, filter, flen, maxH, minPer, out) != SUCCEEDED)
    return out;  // request-level validation error: every part failed, no stats row
  std::vector<const PropCtx*> props;
  for (auto& tc : proc.tagCtxs)
    for (auto& p : tc.props)
      if (p.returned) props.push_back(&p);
  for (auto& p : proc.edgeProps) props.push_back(&p);
  std::sort(props.begin(), props.end(), [](const PropCtx* a, const PropCtx* b) { return a->retIndex < b->retIndex; });
  out->edgeSchema.clear();
  std::vector<Val> row;
  std::vector<bool> pres;
  for (auto* p : props) {
    if (p->badGet && p->stat != 2) {
      out->code = -1003;
      out->error = "SUM/AVG over a double value (boost::bad_get in the reference)";
      return out;
    }
    if (p->stat == 3) {
      row.push_back(Val{double(p->sum) / double(p->count)});
      out->edgeSchema.push_back(Field{p->name, T_DOUBLE});
    } else {
      row.push_back(Val{p->stat == 2 ? int64_t(p->count) : p->sum});
      out->edgeSchema.push_back(Field{p->name, T_INT});
    }
    pres.push_back(true);
  }
  out->rows.push_back(std::move(row));
  out->present.push_back(std::move(pres));
  out->rowVertex.push_back(0);
  return out;
}

// GoExecutor restatement (src/graph/GoExecutor.cpp:80-106, 334-431, 454-499, 585-782).
// Supports literal/pipe starts, N steps, one edge type, WHERE/YIELD over edge props and
// literals, DISTINCT.  $^ / $$ / $- / $var references are reported as unsupported.
ora_result* ora_go(ora_store* st, const int64_t* starts, size_t nStarts, int32_t steps,
                   int32_t et, const uint8_t* where, size_t whereLen,
                   const uint8_t* const* yields, const size_t* ylens, size_t ny,
                   int32_t distinct, int32_t numHosts, int32_t maxH, int32_t minPer,
                   uint64_t* edgesScanned) {
  auto* out = new ora_result();
  uint64_t scanned = 0;
  ExprPtr filter;
  if (whereLen) {
    filter = decodeBuffer(where, whereLen, /*graphdSemantics=*/true);
    if (!filter) {
      out->code = -1;
      out->error = "bad WHERE encoding";
      return out;
    }
  }
  std::vector<ExprPtr> ycols;
  for (size_t i = 0; i < ny; i++) {
    ycols.push_back(decodeBuffer(yields[i], ylens[i], true));
    if (!ycols.back()) {
      out->code = -1;
      out->error = "bad YIELD encoding";
      return out;
    }
  }
  if (ny == 0) {  // default YIELD e._dst AS id (parser.yy:437-446)
    auto x = std::make_unique<Expr>();
    x->kind = kEdgeDstId;
    x->alias = "";
    x->prop = "_dst";
    x->hasProp = true;
    ycols.push_back(std::move(x));
  }
  ExprRefs refs;
  if (filter) collectRefs(*filter, refs);
  for (auto& y : ycols) collectRefs(*y, refs);
  // InterimResult::buildIndex (InterimResult.cpp:125-195): vid of the FROM column (= starts[i]
  // for row i) -> row, the last row of a vid winning; getPropFromInterim (GoExecutor.cpp:831-838)
  std::vector<std::string> inNames = std::move(st->inNames);
  std::vector<std::vector<Val>> inCols = std::move(st->inCols);
  const size_t inRows = st->inRows;
  st->inNames.clear();
  st->inCols.clear();
  st->inRows = 0;
  std::unordered_map<int64_t, size_t> inIndex;
  if (refs.input || refs.variable) {
    if (inNames.empty() || inRows != nStarts) {
      out->code = -2;
      out->error = "unsupported reference ($-/$var without an input table)";
      return out;
    }
    for (size_t i = 0; i < nStarts; i++) inIndex[starts[i]] = i;
  }
  // STEPS > 1: VertexBackTracker (GoExecutor.h:174-193) maps every dst of a non-final step to a
  // start (GoExecutor.cpp:420-424), in RPC response order with the last write winning, so the
  // reference's answer depends on that order whenever a vertex is reached from several starts.
  // Restated with the build's order-free rule: a step reads the previous step's
  // roots and a dst takes the smallest root vid among the srcs of its in-edges -- the
  // reference's own answer whenever the root is unique.
  const bool backTrack = (refs.input || refs.variable) && steps != 1;
  std::unordered_map<int64_t, int64_t> rootOf;
  if (backTrack)
    for (size_t i = 0; i < nStarts; i++) rootOf[starts[i]] = starts[i];
  auto inputProp = [&](int64_t vid0, const std::string& prop) -> OptVal {
    int64_t vid = vid0;
    if (backTrack) {
      auto rt = rootOf.find(vid0);
      if (rt == rootOf.end()) return ERR("vid not traced back to a start");
      vid = rt->second;
    }
    auto r = inIndex.find(vid);
    if (r == inIndex.end()) return ERR("vid not in the input index");
    for (size_t c = 0; c < inNames.size(); c++)
      if (inNames[c] == prop) return OK(inCols[c][r->second]);
    return ERR("unknown input column " + prop);
  };
  // getStepOutProps / getDstProps (GoExecutor.cpp:454-527): tag props grouped per tag name,
  // index = position in the vertex row; unknown tag -> "No schema found"
  std::vector<std::string> tagPropNames;  // stable storage for the PropDef names
  tagPropNames.reserve(refs.srcTag.size() + refs.dstTag.size());
  std::vector<ora_prop_def> srcCols, dstCols;
  std::map<std::pair<std::string, std::string>, int> srcIndex, dstIndex;
  auto tagCols = [&](const std::set<std::pair<std::string, std::string>>& refsSet,
                     std::vector<ora_prop_def>& colsOut,
                     std::map<std::pair<std::string, std::string>, int>& index) {
    std::map<std::string, std::vector<std::string>> byTag;
    for (auto& tp : refsSet) byTag[tp.first].push_back(tp.second);
    int i = -1;
    for (auto& t : byTag) {
      auto id = st->tagByName.find(t.first);
      if (id == st->tagByName.end()) return false;
      for (auto& prop : t.second) {
        tagPropNames.push_back(prop);
        colsOut.push_back(ora_prop_def{tagPropNames.back().c_str(), DEST, id->second});
        index[{t.first, prop}] = ++i;
      }
    }
    return true;
  };
  if (!tagCols(refs.srcTag, srcCols, srcIndex) || !tagCols(refs.dstTag, dstCols, dstIndex)) {
    out->code = -5;
    out->error = "No schema found";
    return out;
  }
  std::vector<int64_t> cur(starts, starts + nStarts);
  if (distinct) {  // GoExecutor.cpp:98-104
    std::unordered_set<int64_t> u(cur.begin(), cur.end());
    cur.assign(u.begin(), u.end());
  }
  if (cur.empty()) return out;
  for (int32_t step = 1;; step++) {
    bool final = step == steps;
    // getStepOutProps (GoExecutor.cpp:454-499): _dst, then alias props on the final step
    std::vector<std::string> names{"_dst"};
    if (final)
      for (auto& ap : refs.alias) names.push_back(ap.second);
    std::vector<ora_prop_def> cols;
    cols.push_back(ora_prop_def{names[0].c_str(), EDGE, 0});
    if (final) cols.insert(cols.end(), srcCols.begin(), srcCols.end());
    for (size_t ni = 1; ni < names.size(); ni++) cols.push_back(ora_prop_def{names[ni].c_str(), EDGE, 0});
    auto resps = getNeighbors(st, cur, et, cols, numHosts, maxH, minPer);
    size_t ok = 0;
    for (auto& r : resps) ok += r.failed.empty() ? 1 : 0;
    if (!resps.empty() && ok == 0) {  // completeness 0 -> "Get neighbors failed"
      out->code = -3;
      out->error = "Get neighbors failed";
      return out;
    }
    if (!final) {
      // getDstIdsFromResp (GoExecutor.cpp:407-431)
      std::unordered_set<int64_t> set;
      std::unordered_map<int64_t, int64_t> nextRoot;
      for (auto& r : resps) {
        auto es = toSchema(r.edgeSchema);
        for (auto& v : r.vertices)
          rowSetForEach(v.edgeData, es, [&](const RowReader& row) {
            scanned++;
            auto d = row.getByName("_dst");
            const int64_t dst = std::get<0>(d.v);
            set.insert(dst);
            if (backTrack) {
              const int64_t rt = rootOf.at(v.vid);
              auto it = nextRoot.find(dst);
              if (it == nextRoot.end() || rt < it->second) nextRoot[dst] = rt;
            }
          });
      }
      if (backTrack) rootOf.swap(nextRoot);
      cur.assign(set.begin(), set.end());
      if (cur.empty()) break;  // onEmptyInputs
      continue;
    }
    // onStepOutResponse final step with $$ props: fetchVertexProps over the response's dst ids
    // (GoExecutor.cpp:377-386, 531-566), kept in a VertexHolder (:785-828)
    std::unordered_map<int64_t, std::string> holder;
    SchemaPtr holderSchema;
    if (!dstCols.empty()) {
      std::unordered_set<int64_t> set;
      for (auto& r : resps) {
        auto es = toSchema(r.edgeSchema);
        for (auto& v : r.vertices)
          rowSetForEach(v.edgeData, es, [&](const RowReader& row) { set.insert(std::get<0>(row.getByName("_dst").v)); });
      }
      if (set.empty()) break;  // onEmptyInputs
      std::vector<int64_t> dstids(set.begin(), set.end());
      auto vr = getNeighbors(st, dstids, 0, dstCols, numHosts, maxH, minPer, /*onlyVertexProps=*/true);
      size_t vok = 0;
      for (auto& r : vr) vok += r.failed.empty() ? 1 : 0;
      if (!vr.empty() && vok == 0) {
        out->code = -3;
        out->error = "Get dest props failed";
        return out;
      }
      for (auto& r : vr) {
        if (r.vertices.empty()) continue;
        if (!holderSchema) holderSchema = toSchema(r.vertexSchema);
        for (auto& v : r.vertices)
          if (!v.vertexData.empty()) holder[v.vid] = v.vertexData;
      }
    }
    // processFinalResult + setupInterimResult (GoExecutor.cpp:585-656, 669-782)
    SchemaPtr outSchema;
    std::unordered_set<std::string> uniq;
    for (auto& r : resps) {
      auto es = toSchema(r.edgeSchema);
      auto vs = toSchema(r.vertexSchema);
      for (auto& v : r.vertices) {
        bool failed = false;
        // a vertex without any requested tag has no vertex_data: the reference builds a
        // RowReader over the empty row and aborts (RowReader.cpp:207-214); reported as an error
        std::unique_ptr<RowReader> vreader;
        if (!srcCols.empty() && !v.vertexData.empty())
          vreader = std::make_unique<RowReader>(v.vertexData.data(), v.vertexData.size(), vs);
        rowSetForEach(v.edgeData, es, [&](const RowReader& row) {
          if (failed) return;
          scanned++;
          Getters g;
          g.getAliasProp = [&](const std::string&, const std::string& prop) -> OptVal {
            auto res = row.getByName(prop);
            if (res.ok()) return res;
            return ERR("get edge prop failed");
          };
          g.getSrcTagProp = [&](const std::string& tag, const std::string& prop) -> OptVal {
            auto it = srcIndex.find({tag, prop});
            if (it == srcIndex.end() || !vreader) return ERR("src tag prop missing");
            auto res = vreader->getByIndex(it->second);
            if (res.ok()) return res;
            return ERR(tag + "." + prop + " was not exist");
          };
          g.getDstTagProp = [&](const std::string& tag, const std::string& prop) -> OptVal {
            auto it = dstIndex.find({tag, prop});
            if (it == dstIndex.end()) return ERR("dst tag prop missing");
            int64_t dst = std::get<0>(row.getByName("_dst").v);
            auto h = holder.find(dst);
            if (h == holder.end()) return ERR("vertex was not found");
            RowReader rr(h->second.data(), h->second.size(), holderSchema);
            auto res = rr.getByIndex(it->second);
            if (res.ok()) return res;
            return ERR("get prop failed");
          };
          g.getInputProp = [&](const std::string& prop) -> OptVal { return inputProp(v.vid, prop); };
          g.getVariableProp = [&](const std::string& prop) -> OptVal { return inputProp(v.vid, prop); };
          if (filter) {
            auto fv = eval(*filter, g);
            if (!fv.ok()) {
              failed = true;
              out->code = -4;
              out->error = fv.st.msg;
              return;
            }
            if (!asBool(fv.v)) return;
          }
          std::vector<Val> rec;
          for (auto& y : ycols) {
            auto yv = eval(*y, g);
            if (!yv.ok()) {
              failed = true;
              out->code = -4;
              out->error = yv.st.msg;
              return;
            }
            rec.push_back(yv.v);
          }
          if (!outSchema) {  // schema from the first record; ints are VID (GoExecutor.cpp:596-600)
            auto s = std::make_shared<Schema>();
            for (auto& c : rec) {
              int32_t t = c.index() == 0 ? T_VID : c.index() == 1 ? T_DOUBLE
                        : c.index() == 2 ? T_BOOL : T_STRING;
              s->fields.push_back(Field{"", t});
            }
            outSchema = s;
          }
          RowWriter w(outSchema);
          for (auto& c : rec) w << c;
          std::string enc = w.encode();
          if (distinct && !uniq.insert(enc).second) return;
          // value as the client reads it back under outSchema
          RowReader rr(enc.data(), enc.size(), outSchema);
          std::vector<Val> row2;
          std::vector<bool> pres;
          for (size_t c = 0; c < rec.size(); c++) {
            auto x = rr.getByIndex(int(c));
            row2.push_back(x.v);
            pres.push_back(x.ok());
          }
          out->rows.push_back(std::move(row2));
          out->present.push_back(std::move(pres));
          out->rowVertex.push_back(v.vid);
        });
        if (failed) {
          out->rows.clear();
          out->present.clear();
          out->rowVertex.clear();
          if (edgesScanned) *edgesScanned = scanned;
          return out;
        }
      }
    }
    break;
  }
  if (edgesScanned) *edgesScanned = scanned;
  return out;
}

// ---------------------------------------------------------------------------------------------
// FIND SHORTEST PATH (A10, no reference implementation).  Definition owned by this build:
// unweighted hop distance from src to dst over out-edges of `edge_type` (collected with the
// getOutBound scan semantics), -1 if no path within max_steps; path = the lexicographically
// smallest vid sequence among the shortest paths.  Row: [src, dst, hops, v0, v1, ..., vL].
// ---------------------------------------------------------------------------------------------
ora_result* ora_shortest_path(ora_store* st, const int64_t* src, const int64_t* dst,
                              size_t npairs, int32_t et, int32_t maxSteps) {
  auto* out = new ora_result();
  auto neighbors = [&](int64_t v, int32_t type) {
    std::vector<int64_t> ns;
    int32_t part = partOf(v, st->numParts);
    int64_t lastRank = -1, lastDst = 0;
    bool first = true;
    prefixScan(st, part, edgePrefix(part, v, type), [&](const char* k, size_t, const char*, size_t) {
      int64_t rank = keyRank(k), d = keyDst(k);
      if (!first && rank == lastRank && d == lastDst) return true;
      first = false;
      lastRank = rank;
      lastDst = d;
      ns.push_back(d);
      return true;
    });
    return ns;
  };
  for (size_t p = 0; p < npairs; p++) {
    int64_t s = src[p], t = dst[p];
    // backward BFS distances to t over in-edges (-type), up to maxSteps
    std::unordered_map<int64_t, int32_t> dt;
    dt[t] = 0;
    std::vector<int64_t> fr{t};
    for (int32_t lvl = 1; lvl <= maxSteps && !fr.empty() && !dt.count(s); lvl++) {
      std::vector<int64_t> nx;
      for (auto v : fr)
        for (auto u : neighbors(v, -et))
          if (!dt.count(u)) {
            dt[u] = lvl;
            nx.push_back(u);
          }
      fr.swap(nx);
    }
    std::vector<Val> row{Val{s}, Val{t}};
    auto it = dt.find(s);
    if (it == dt.end()) {
      row.push_back(Val{int64_t(-1)});
    } else {
      int32_t L = it->second;
      row.push_back(Val{int64_t(L)});
      int64_t v = s;
      row.push_back(Val{v});
      for (int32_t k = L; k > 0; k--) {
        int64_t best = 0;
        bool found = false;
        for (auto w : neighbors(v, et)) {
          auto jt = dt.find(w);
          if (jt != dt.end() && jt->second == k - 1 && (!found || w < best)) {
            best = w;
            found = true;
          }
        }
        v = best;
        row.push_back(Val{v});
      }
    }
    out->present.push_back(std::vector<bool>(row.size(), true));
    out->rows.push_back(std::move(row));
  }
  return out;
}

int32_t ora_res_code(const ora_result* r) { return r->code; }
const char* ora_res_error(const ora_result* r) { return r->error.c_str(); }
size_t ora_res_nrows(const ora_result* r) { return r->rows.size(); }
int32_t ora_res_ncols(const ora_result* r) {
  size_t m = 0;
  for (auto& row : r->rows) m = std::max(m, row.size());
  return int32_t(m);
}
int32_t ora_res_type(const ora_result* r, size_t row, int32_t col) {
  if (row >= r->rows.size() || size_t(col) >= r->rows[row].size() || !r->present[row][size_t(col)])
    return -1;
  return int32_t(r->rows[row][size_t(col)].index());
}
int64_t ora_res_int(const ora_result* r, size_t row, int32_t col) {
  auto& v = r->rows[row][size_t(col)];
  return v.index() == 0 ? std::get<0>(v) : v.index() == 2 ? int64_t(std::get<2>(v)) : 0;
}
double ora_res_double(const ora_result* r, size_t row, int32_t col) {
  auto& v = r->rows[row][size_t(col)];
  return v.index() == 1 ? std::get<1>(v) : 0.0;
}
const char* ora_res_str(const ora_result* r, size_t row, int32_t col, size_t* len) {
  auto& v = r->rows[row][size_t(col)];
  if (v.index() != 3) {
    *len = 0;
    return "";
  }
  *len = std::get<3>(v).size();
  return std::get<3>(v).data();
}
void ora_res_int_col(const ora_result* r, int32_t col, int64_t* out) {
  for (size_t i = 0; i < r->rows.size(); i++) {
    const auto& row = r->rows[i];
    out[i] = (size_t(col) < row.size() && r->present[i][size_t(col)] && row[size_t(col)].index() == 0)
                 ? std::get<0>(row[size_t(col)]) : INT64_MIN;
  }
}
size_t ora_res_nfailed(const ora_result* r) { return r->failed.size(); }
void ora_res_failed(const ora_result* r, size_t i, int32_t* part, int32_t* code) {
  *part = r->failed[i].first;
  *code = r->failed[i].second;
}
int64_t ora_res_row_vertex(const ora_result* r, size_t row) { return r->rowVertex[row]; }
size_t ora_res_nvertices(const ora_result* r) { return r->vertices.size(); }
int64_t ora_res_vertex_id(const ora_result* r, size_t i) { return r->vertices[i].vid; }
size_t ora_res_vertex_nrows(const ora_result* r, size_t i) { return r->vertices[i].nrows; }
int32_t ora_res_vertex_ncols(const ora_result* r) { return int32_t(r->vertexSchema.size()); }
int32_t ora_res_vertex_type(const ora_result* r, size_t i, int32_t col) {
  auto& v = r->vertices[i];
  if (size_t(col) >= v.tagVals.size() || !v.tagPresent[size_t(col)]) return -1;
  return int32_t(v.tagVals[size_t(col)].index());
}
int64_t ora_res_vertex_int(const ora_result* r, size_t i, int32_t col) {
  auto& v = r->vertices[i].tagVals[size_t(col)];
  return v.index() == 0 ? std::get<0>(v) : 0;
}
const char* ora_res_vertex_str(const ora_result* r, size_t i, int32_t col, size_t* len) {
  auto& v = r->vertices[i].tagVals[size_t(col)];
  if (v.index() != 3) {
    *len = 0;
    return "";
  }
  *len = std::get<3>(v).size();
  return std::get<3>(v).data();
}
const char* ora_res_vertex_bytes(const ora_result* r, size_t i, size_t* len) {
  *len = r->vertices[i].vertexData.size();
  return r->vertices[i].vertexData.data();
}
const char* ora_res_edge_bytes(const ora_result* r, size_t i, size_t* len) {
  *len = r->vertices[i].edgeData.size();
  return r->vertices[i].edgeData.data();
}
int32_t ora_res_schema_ncols(const ora_result* r, int32_t which) {
  return int32_t(which == 0 ? r->edgeSchema.size() : r->vertexSchema.size());
}
const char* ora_res_schema_name(const ora_result* r, int32_t which, int32_t col) {
  return (which == 0 ? r->edgeSchema : r->vertexSchema)[size_t(col)].name.c_str();
}
int32_t ora_res_schema_type(const ora_result* r, int32_t which, int32_t col) {
  return (which == 0 ? r->edgeSchema : r->vertexSchema)[size_t(col)].type;
}
void ora_res_free(ora_result* r) { delete r; }

}  // extern "C"
