// expr.cpp -- decode Expression::encode bytes and compile them to a device Program.
//
// Decoder follows Expression::decode and each *Expression::decode
// (src/common/filter/Expressions.cpp:92-107, 128-146, 366-384, 488-530, 632-638, 836-845,
//  945-954, 1023-1032).  Validation follows QueryBaseProcessor::checkExp
// (src/storage/QueryBaseProcessor.inl:138-245) for storage filters.
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "engine.h"
#include "program.h"

namespace nbg {

namespace {

enum Kind : uint8_t {
  kUnknown = 0, kPrimary, kFunctionCall, kUnary, kTypeCasting, kArithmetic, kRelational,
  kLogical, kSourceProp, kEdgeRank, kEdgeDstId, kEdgeSrcId, kEdgeType, kAliasProp, kEdgeProp,
  kVariableProp, kDestProp, kInputProp
};

struct Node {
  uint8_t kind = 0, op = 0;
  int32_t ptype = 0;  // primary: 0 int 1 double 2 bool 3 string
  int64_t ibits = 0;
  std::string str, alias, prop;
  std::unique_ptr<Node> l, r;
};

struct Bad {};

struct Cur {
  const uint8_t* p;
  const uint8_t* e;
  void need(size_t n) {
    if (size_t(e - p) < n) throw Bad{};
  }
  uint8_t u8() {
    need(1);
    return *p++;
  }
  uint16_t u16() {
    need(2);
    uint16_t v;
    memcpy(&v, p, 2);
    p += 2;
    return v;
  }
  std::string s() {
    uint16_t n = u16();
    need(n);
    std::string r(reinterpret_cast<const char*>(p), n);
    p += n;
    return r;
  }
};

std::unique_ptr<Node> dec(uint8_t kind, Cur& c) {
  auto x = std::make_unique<Node>();
  x->kind = kind;
  switch (kind) {
    case kPrimary: {
      uint8_t w = c.u8();
      x->ptype = w;
      if (w == 0 || w == 1) {
        c.need(8);
        memcpy(&x->ibits, c.p, 8);
        c.p += 8;
      } else if (w == 2) {
        c.need(1);
        x->ibits = *c.p++ != 0;
      } else if (w == 3) {
        x->str = c.s();
      } else {
        throw Bad{};
      }
      break;
    }
    case kUnary:
      c.need(2);
      x->op = c.u8();
      x->l = dec(c.u8(), c);
      break;
    case kArithmetic:
    case kRelational:
    case kLogical:
      c.need(2);
      x->op = c.u8();
      x->l = dec(c.u8(), c);
      c.need(1);
      x->r = dec(c.u8(), c);
      break;
    case kSourceProp:
    case kAliasProp:
    case kVariableProp:
    case kDestProp:
      x->alias = c.s();
      x->prop = c.s();
      break;
    case kInputProp:
      x->prop = c.s();
      break;
    case kEdgeRank:
    case kEdgeDstId:
    case kEdgeSrcId:
    case kEdgeType:
      x->alias = c.s();
      break;
    default:
      throw Bad{};  // FunctionCall/TypeCasting/unknown: not decodable or rejected by checkExp
  }
  return x;
}

struct Compiler {
  const std::vector<Field>& fields;
  const std::vector<TagFieldRef>* tags = nullptr;
  const std::vector<Field>* inputs = nullptr;  // $- / $var input columns (graphd)
  bool graphd;     // graphd AST semantics (GoExecutor) vs storage-decoded filter
  bool out_bound;
  Program prog;
  int32_t code = NBG_OK;
  std::string msg;
  int depth = 0, maxdepth = 0;
  size_t strpos = 0;

  Compiler(const std::vector<Field>& f, bool g, bool ob) : fields(f), graphd(g), out_bound(ob) {}

  void fail(int32_t c, const std::string& m) {
    if (code == NBG_OK) {
      code = c;
      msg = m;
    }
  }
  void emit(uint8_t op, uint8_t sub, int16_t arg) {
    if (prog.n >= kMaxIns) {
      fail(NBG_E_UNSUPPORTED, "expression too long");
      return;
    }
    prog.ins[prog.n++] = Ins{op, sub, arg};
  }
  void push() {
    depth++;
    if (depth > maxdepth) maxdepth = depth;
    if (depth > kMaxStack) fail(NBG_E_UNSUPPORTED, "expression too deep");
  }
  int16_t add_const(int32_t t, int64_t bits, const std::string& s = std::string()) {
    for (int i = 0; i < prog.n && false; i++) {
    }
    static_assert(kMaxConsts <= 32767, "");
    int idx = 0;
    for (; idx < kMaxConsts; idx++)
      if (prog.ctype[idx] < 0) break;
    if (idx >= kMaxConsts) {
      fail(NBG_E_UNSUPPORTED, "too many constants");
      return 0;
    }
    prog.ctype[idx] = t;
    prog.cbits[idx] = bits;
    prog.clen[idx] = 0;
    if (t == VT_STR) {
      if (strpos + s.size() > size_t(kMaxStrConst)) {
        fail(NBG_E_UNSUPPORTED, "string constants too long");
        return 0;
      }
      memcpy(prog.cstr + strpos, s.data(), s.size());
      prog.cbits[idx] = int64_t(strpos);
      prog.clen[idx] = int32_t(s.size());
      strpos += s.size();
    }
    return int16_t(idx);
  }
  // returns static type of the pushed value
  int32_t key_prop(int which) {
    emit(uint8_t(which), 0, 0);
    push();
    return VT_INT;
  }
  int32_t gen(const Node& x) {
    switch (x.kind) {
      case kPrimary: {
        static const int32_t map[4] = {VT_INT, VT_DOUBLE, VT_BOOL, VT_STR};
        int32_t t = map[x.ptype];
        emit(P_CONST, 0, add_const(t, x.ibits, x.str));
        push();
        return t;
      }
      case kEdgeDstId:
      case kEdgeSrcId:
      case kEdgeRank: {
        if (!graphd) {  // storage-side decode leaves prop_ null (Expressions.h:449-460): unusable
          fail(NBG_E_INVALID_FILTER, "_dst/_src/_rank in a storage filter (reference dereferences a null prop)");
          return VT_ERR;
        }
        return key_prop(x.kind == kEdgeDstId ? P_DST : x.kind == kEdgeSrcId ? P_SRC : P_RANK);
      }
      case kEdgeType: {
        if (!graphd) {
          fail(NBG_E_INVALID_FILTER, "_type in a storage filter");
          return VT_ERR;
        }
        // EdgeTypeExpression::eval returns *alias_ (Expressions.cpp:241-243)
        emit(P_CONST, 0, add_const(VT_STR, 0, x.alias));
        push();
        return VT_STR;
      }
      case kAliasProp:
      case kEdgeProp: {
        if (x.prop == "_dst") return key_prop(P_DST);
        if (x.prop == "_src") return key_prop(P_SRC);
        if (x.prop == "_rank") return key_prop(P_RANK);
        if (x.prop == "_type") return key_prop(P_TYPE);
        if (!out_bound) {
          fail(graphd ? NBG_E_IMPROPER_DATA_TYPE : NBG_E_INVALID_FILTER, "in-bound edges have no props");
          return VT_ERR;
        }
        for (size_t i = 0; i < fields.size(); i++) {
          if (fields[i].name == x.prop) {
            emit(P_PROP, 0, int16_t(i));
            push();
            int32_t t = fields[i].type;
            if (t == NBG_T_DOUBLE || t == NBG_T_FLOAT) return VT_DOUBLE;
            if (t == NBG_T_BOOL) return VT_BOOL;
            if (t == NBG_T_STRING) return VT_STR;
            return VT_INT;
          }
        }
        // storage: checkExp -> E_INVALID_FILTER; graphd: the prop is a return column ->
        // checkAndBuildContexts -> E_IMPROPER_DATA_TYPE (QueryBaseProcessor.inl:93-96)
        fail(graphd ? NBG_E_IMPROPER_DATA_TYPE : NBG_E_INVALID_FILTER, "unknown edge prop " + x.prop);
        return VT_ERR;
      }
      case kSourceProp:
      case kDestProp: {
        // graphd: getStepOutProps / getDstProps resolve the tag name (GoExecutor.cpp:470-527);
        // storage filters: checkExp accepts $^ of a known tag prop and rejects $$
        // (QueryBaseProcessor.inl:190-238 -> E_INVALID_FILTER)
        if (!graphd && x.kind == kDestProp) {
          fail(NBG_E_INVALID_FILTER, "$$ in a storage filter");
          return VT_ERR;
        }
        if (!tags) {
          fail(NBG_E_UNSUPPORTED, "$^ / $$ tag props without tag schemas");
          return VT_ERR;
        }
        bool known_tag = false;
        for (size_t i = 0; i < tags->size(); i++) {
          const TagFieldRef& t = (*tags)[i];
          if (t.tag != x.alias) continue;
          known_tag = true;
          if (t.prop != x.prop) continue;
          emit(x.kind == kSourceProp ? P_SRCTAG : P_DSTTAG, 0, int16_t(i));
          push();
          if (t.type == NBG_T_DOUBLE || t.type == NBG_T_FLOAT) return VT_DOUBLE;
          if (t.type == NBG_T_BOOL) return VT_BOOL;
          if (t.type == NBG_T_STRING) return VT_STR;
          return VT_INT;
        }
        // unknown tag: "No schema found" (GoExecutor.cpp:475-478); unknown prop of a known tag:
        // checkAndBuildContexts -> E_IMPROPER_DATA_TYPE on every part (QueryBaseProcessor.inl:56-66)
        if (!graphd) fail(NBG_E_INVALID_FILTER, "unknown tag prop in a storage filter");
        else if (known_tag) fail(NBG_E_IMPROPER_DATA_TYPE, "unknown tag prop " + x.alias + "." + x.prop);
        else fail(NBG_E_TAG_PROP_NOT_FOUND, "no schema found for tag " + x.alias);
        return VT_ERR;
      }
      case kInputProp:
      case kVariableProp: {
        // checkExp rejects these in storage filters (QueryBaseProcessor.inl:235-238)
        if (!graphd) {
          fail(NBG_E_INVALID_FILTER, "$- / $var props in a storage filter");
          return VT_ERR;
        }
        if (!inputs) {
          fail(NBG_E_UNSUPPORTED, "$- / $var props without an input table");
          return VT_ERR;
        }
        for (size_t i = 0; i < inputs->size(); i++) {
          if ((*inputs)[i].name != x.prop) continue;
          emit(P_INPUT, 0, int16_t(i));
          push();
          const int32_t t = (*inputs)[i].type;
          if (t == NBG_T_DOUBLE || t == NBG_T_FLOAT) return VT_DOUBLE;
          if (t == NBG_T_BOOL) return VT_BOOL;
          if (t == NBG_T_STRING) return VT_STR;
          return VT_INT;
        }
        fail(NBG_E_INVALID_ARG, "unknown input column " + x.prop);
        return VT_ERR;
      }
      case kUnary: {
        int32_t t = gen(*x.l);
        emit(P_UNARY, x.op, 0);
        if (x.op == 2) return VT_BOOL;
        if (x.op == 1) return (t == VT_INT || t == VT_DOUBLE) ? t : VT_ERR;
        return t;
      }
      case kArithmetic: {
        int32_t a = gen(*x.l);
        int32_t b = gen(*x.r);
        emit(P_ARITH, x.op, 0);
        depth--;
        bool arith = (a == VT_INT || a == VT_DOUBLE) && (b == VT_INT || b == VT_DOUBLE);
        if (x.op == 0 && a == VT_STR && b == VT_STR) {
          fail(NBG_E_UNSUPPORTED, "string concatenation on the device");
          return VT_ERR;
        }
        if (x.op == 4) return (a == VT_INT && b == VT_INT) ? VT_INT : VT_ERR;
        if (!arith) return VT_ERR;
        return (a == VT_DOUBLE || b == VT_DOUBLE) ? VT_DOUBLE : VT_INT;
      }
      case kRelational:
      case kLogical: {
        gen(*x.l);
        gen(*x.r);
        emit(x.kind == kRelational ? P_REL : P_LOGIC, x.op, 0);
        depth--;
        return VT_BOOL;
      }
      default:
        fail(graphd ? NBG_E_UNSUPPORTED : NBG_E_INVALID_FILTER, "unsupported expression kind");
        return VT_ERR;
    }
  }
};

}  // namespace

// Compiles an encoded expression.  Returns NBG_OK or an error code (msg filled).
int32_t compile_expr(const uint8_t* buf, size_t len, const std::vector<Field>& fields, bool graphd,
                     bool out_bound, Program* out, std::string* msg, const std::vector<TagFieldRef>* tags,
                     const std::vector<Field>* inputs) {
  std::unique_ptr<Node> root;
  try {
    Cur c{buf, buf + len};
    root = dec(c.u8(), c);
    if (c.p != c.e) throw Bad{};
  } catch (const Bad&) {
    if (msg) *msg = "expression decode failed";
    return graphd ? NBG_E_INVALID_ARG : NBG_E_INVALID_FILTER;  // Expression::decode -> E_INVALID_FILTER
  }
  Compiler cc(fields, graphd, out_bound);
  cc.tags = tags;
  cc.inputs = inputs;
  for (int i = 0; i < kMaxConsts; i++) cc.prog.ctype[i] = -1;
  cc.prog.result_type = cc.gen(*root);
  if (cc.code != NBG_OK) {
    if (msg) *msg = cc.msg;
    return cc.code;
  }
  *out = cc.prog;
  return NBG_OK;
}

// Program for the default YIELD e._dst AS id (parser.yy:437-446)
Program program_dst() {
  Program p;
  for (int i = 0; i < kMaxConsts; i++) p.ctype[i] = -1;
  p.n = 1;
  p.ins[0] = Ins{P_DST, 0, 0};
  p.result_type = VT_INT;
  return p;
}

FastPred classify_pred(const Program& p, const std::vector<Field>& fields) {
  FastPred f;
  if (p.n == 0) return f;
  f.kind = 2;
  if (p.n == 3 && p.ins[2].op == P_REL) {
    const Ins& a = p.ins[0];
    const Ins& b = p.ins[1];
    auto is_int_prop = [&](const Ins& i) {
      if (i.op != P_PROP) return false;
      int32_t t = fields[size_t(i.arg)].type;
      return t == NBG_T_INT || t == NBG_T_VID || t == NBG_T_TIMESTAMP;
    };
    auto is_int_const = [&](const Ins& i) { return i.op == P_CONST && p.ctype[i.arg] == VT_INT; };
    static const int swap_op[6] = {3 /*LT->GT*/, 2 /*LE->GE*/, 1 /*GT->LT*/, 0 /*GE->LE*/, 4, 5};
    // LT=0 LE=1 GT=2 GE=3 EQ=4 NE=5; a<b == b>a
    static const int mirror[6] = {2, 3, 0, 1, 4, 5};
    (void)swap_op;
    if (is_int_prop(a) && is_int_const(b)) {
      f.kind = 1;
      f.col = a.arg;
      f.op = p.ins[2].sub;
      f.k = p.cbits[b.arg];
    } else if (is_int_const(a) && is_int_prop(b)) {
      f.kind = 1;
      f.col = b.arg;
      f.op = mirror[p.ins[2].sub];
      f.k = p.cbits[a.arg];
    }
  }
  return f;
}

}  // namespace nbg
