"""Filter / YIELD expressions in the reference's binary encoding.

The drop-in boundary takes WHERE / YIELD / filter expressions as the bytes the reference's
``Expression::encode`` produces (src/common/filter/Expressions.cpp:84-90 and each
``*Expression::encode``), because that is what ``GetNeighborsRequest.filter`` carries
(src/interface/storage.thrift:125-133).  This module builds those bytes from Python.

Layout (native little-endian, as the reference assumes "the same byte order on both sides"):
  kind:u8, then per kind
  Primary      which:u8 + int64 | double | u8 | (u16 len + bytes)      (Expressions.cpp:478-498)
  AliasProp    u16+alias, u16+prop    (SourceProp, DestProp, VariableProp the same)
  InputProp    u16+prop
  EdgeRank/EdgeDstId/EdgeSrcId/EdgeType   u16+alias
  Unary        op:u8, operand         Arithmetic/Relational/Logical  op:u8, left, right
"""
from __future__ import annotations

import struct

# Expression::Kind (src/common/filter/Expressions.h:209-228)
K_PRIMARY, K_FUNCTION_CALL, K_UNARY, K_TYPE_CASTING, K_ARITHMETIC, K_RELATIONAL, K_LOGICAL = 1, 2, 3, 4, 5, 6, 7
K_SOURCE_PROP, K_EDGE_RANK, K_EDGE_DST_ID, K_EDGE_SRC_ID, K_EDGE_TYPE = 8, 9, 10, 11, 12
K_ALIAS_PROP, K_EDGE_PROP, K_VARIABLE_PROP, K_DEST_PROP, K_INPUT_PROP = 13, 14, 15, 16, 17

# operator enums (Expressions.h:624, 711, 762, 814)
PLUS, NEGATE, NOT = 0, 1, 2
ADD, SUB, MUL, DIV, MOD = 0, 1, 2, 3, 4
LT, LE, GT, GE, EQ, NE = 0, 1, 2, 3, 4, 5
AND, OR = 0, 1


def _s(x: str) -> bytes:
    b = x.encode()
    return struct.pack("<H", len(b)) + b


class Expr:
    def encode(self) -> bytes:  # pragma: no cover - abstract
        raise NotImplementedError

    # builder sugar -------------------------------------------------------------------
    def _bin(self, cls, op, other):
        return cls(op, self, other if isinstance(other, Expr) else Primary(other))

    def __lt__(self, o): return self._bin(Relational, LT, o)
    def __le__(self, o): return self._bin(Relational, LE, o)
    def __gt__(self, o): return self._bin(Relational, GT, o)
    def __ge__(self, o): return self._bin(Relational, GE, o)
    def eq(self, o): return self._bin(Relational, EQ, o)
    def ne(self, o): return self._bin(Relational, NE, o)
    def __add__(self, o): return self._bin(Arithmetic, ADD, o)
    def __sub__(self, o): return self._bin(Arithmetic, SUB, o)
    def __mul__(self, o): return self._bin(Arithmetic, MUL, o)
    def __truediv__(self, o): return self._bin(Arithmetic, DIV, o)
    def __mod__(self, o): return self._bin(Arithmetic, MOD, o)
    def __and__(self, o): return self._bin(Logical, AND, o)
    def __or__(self, o): return self._bin(Logical, OR, o)
    def __neg__(self): return Unary(NEGATE, self)
    def __invert__(self): return Unary(NOT, self)


class Primary(Expr):
    def __init__(self, v):
        self.v = v

    def encode(self) -> bytes:
        v = self.v
        if isinstance(v, bool):
            return bytes([K_PRIMARY, 2, 1 if v else 0])
        if isinstance(v, int):
            return bytes([K_PRIMARY, 0]) + struct.pack("<q", v)
        if isinstance(v, float):
            return bytes([K_PRIMARY, 1]) + struct.pack("<d", v)
        if isinstance(v, str):
            return bytes([K_PRIMARY, 3]) + _s(v)
        raise TypeError(f"unsupported literal {v!r}")


class AliasProp(Expr):
    """`edge.prop` (AliasPropertyExpression)."""

    kind = K_ALIAS_PROP

    def __init__(self, alias: str, prop: str):
        self.alias, self.prop = alias, prop

    def encode(self) -> bytes:
        return bytes([self.kind]) + _s(self.alias) + _s(self.prop)


class SourceProp(AliasProp):
    kind = K_SOURCE_PROP


class DestProp(AliasProp):
    kind = K_DEST_PROP


class VariableProp(AliasProp):
    kind = K_VARIABLE_PROP


class InputProp(Expr):
    def __init__(self, prop: str):
        self.prop = prop

    def encode(self) -> bytes:
        return bytes([K_INPUT_PROP]) + _s(self.prop)


class _EdgeKey(Expr):
    kind = 0

    def __init__(self, alias: str = ""):
        self.alias = alias

    def encode(self) -> bytes:
        return bytes([self.kind]) + _s(self.alias)


class EdgeRank(_EdgeKey):
    kind = K_EDGE_RANK


class EdgeDst(_EdgeKey):
    kind = K_EDGE_DST_ID


class EdgeSrc(_EdgeKey):
    kind = K_EDGE_SRC_ID


class EdgeType(_EdgeKey):
    kind = K_EDGE_TYPE


class Unary(Expr):
    def __init__(self, op: int, e: Expr):
        self.op, self.e = op, e

    def encode(self) -> bytes:
        return bytes([K_UNARY, self.op]) + self.e.encode()


class _Binary(Expr):
    kind = 0

    def __init__(self, op: int, l: Expr, r: Expr):
        self.op, self.l, self.r = op, l, r

    def encode(self) -> bytes:
        return bytes([self.kind, self.op]) + self.l.encode() + self.r.encode()


class Arithmetic(_Binary):
    kind = K_ARITHMETIC


class Relational(_Binary):
    kind = K_RELATIONAL


class Logical(_Binary):
    kind = K_LOGICAL


def prop(name: str, alias: str = "") -> AliasProp:
    return AliasProp(alias, name)


def encode(e: Expr | bytes | None) -> bytes:
    """Expression::encode bytes of a tree (or bytes passed through).  Not cached on the tree: Expr
    nodes are mutable, and a child changed after a first encode must change the bytes sent (the
    engine caches the C views per encoded bytes instead, GraphSpace._plan_views)."""
    if e is None:
        return b""
    if isinstance(e, (bytes, bytearray)):
        return bytes(e)
    return e.encode()
