// program.h -- compiled WHERE / YIELD / filter expressions for the device.
//
// The reference evaluates an Expression AST per row with boost::variant values
// (src/common/filter/Expressions.cpp:762-1011).  Here the AST (decoded from its
// Expression::encode bytes) is flattened to a postfix program evaluated per edge on a small
// typed value stack.  Semantics kept bit-exact with the reference:
//   * relational < <= > >= compare the variant index first (int < double < bool < string),
//     values only within one type (boost::variant::operator<), `>`/`<=`/`>=` derived from `<`;
//   * == / != between int and double use |a-b| < 1e-8 (Expressions.h:202-205);
//   * arithmetic int op int stays int64 (wrapping), any double -> double, % ints only;
//   * asBool: int != 0, double != 0.0, bool, string -> empty() (Expressions.h:162-176);
//   * && / || evaluate both sides; an error on either side is the result.
#pragma once
#include <cstdint>

namespace nbg {

enum VType : int32_t { VT_INT = 0, VT_DOUBLE = 1, VT_BOOL = 2, VT_STR = 3, VT_ERR = 4 };

enum POp : uint8_t {
  P_CONST = 0,   // push consts[arg]
  P_PROP = 1,    // push edge prop column arg
  P_DST = 2,     // push vid of the edge's dst (the key's dst)
  P_SRC = 3,     // push vid of the key's src
  P_RANK = 4,    // push the edge rank
  P_TYPE = 5,    // push the edge type (int, the key's type)
  P_UNARY = 6,   // sub = PLUS/NEGATE/NOT
  P_ARITH = 7,   // sub = ADD/SUB/MUL/DIV/MOD
  P_REL = 8,     // sub = LT/LE/GT/GE/EQ/NE
  P_LOGIC = 9,   // sub = AND/OR
  P_SRCTAG = 10, // push $^.tag.prop: tag column arg (Ctx::tag_refs) at the edge's src vertex
  P_DSTTAG = 11, // push $$.tag.prop: tag column arg at the edge's dst vertex
  P_INPUT = 12,  // push $-.prop / $var.prop: input column arg at the row of the edge's src vid
};

constexpr int kMaxIns = 48;
constexpr int kMaxConsts = 16;
constexpr int kMaxStack = 12;
constexpr int kMaxStrConst = 256;  // bytes of string constants

struct Ins {
  uint8_t op;
  uint8_t sub;
  int16_t arg;
};

struct Program {
  int32_t n = 0;
  int32_t result_type = VT_BOOL;  // static result type
  Ins ins[kMaxIns];
  int32_t ctype[kMaxConsts];
  int64_t cbits[kMaxConsts];      // int64 / double bits / bool / string offset
  int32_t clen[kMaxConsts];       // string length
  char cstr[kMaxStrConst];
};

// Fast-path classification of a predicate program.
struct FastPred {
  int32_t kind = 0;   // 0 none (always true), 1 int-prop REL int-const, 2 general VM
  int32_t col = -1;
  int32_t op = 0;     // REL op with the prop on the left
  int64_t k = 0;
};

}  // namespace nbg
