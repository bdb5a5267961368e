"""The drop-in boundary from a compiled C++ caller (tests/cpp/boundary_test.cpp): it includes
include/nebula_amd.h, links libnebula_amd.so and runs QueryBoundTest's OutBoundSimpleTest
(src/storage/test/QueryBoundTest.cpp:181-201) through nbg_get_bound in the shape INTEGRATION.md
section 3 gives GpuBoundProcessor::process, checking checkResponse's expectations
(QueryBoundTest.cpp:111-178) in C++.  The mockData KV bytes (QueryBoundTest.cpp:24-79) are
written to a fixture file here with the oracle's key / RowWriter encoders."""
import struct
import subprocess
from pathlib import Path

import pytest

import fixtures as F

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "tests" / "cpp" / "boundary_test"


def _binary():
    if not BIN.exists():  # built by __graft_entry__.build() (make -C tests/cpp)
        subprocess.run(["make", "-C", str(BIN.parent)], check=True, capture_output=True)
    return str(BIN)


def _s(x: str) -> bytes:
    b = x.encode()
    return struct.pack("<I", len(b)) + b


def _schema(fields) -> bytes:
    return struct.pack("<I", len(fields)) + b"".join(_s(n) + struct.pack("<i", t) for n, t in fields)


def write_fixture(path: Path):
    out = [_s("NBGFIX1"), struct.pack("<ii", 6, F.EDGE_TYPE), _schema(F.qb_edge_schema())]
    tags = list(range(3001, 3010))
    out.append(struct.pack("<I", len(tags)))
    for tag in tags:
        out += [struct.pack("<i", tag), _s(str(tag)), _schema(F.qb_tag_schema(tag))]
    parts = F.qb_kv_parts()
    out.append(struct.pack("<I", len(parts)))
    for part, data in parts.items():
        ks = [k for k, _ in data]
        vs = [v for _, v in data]
        koff, voff = [0], [0]
        for k in ks:
            koff.append(koff[-1] + len(k))
        for v in vs:
            voff.append(voff[-1] + len(v))
        kb, vb = b"".join(ks), b"".join(vs)
        out += [struct.pack("<iQ", part, len(data)), struct.pack("<Q", len(kb)), kb,
                struct.pack(f"<{len(koff)}Q", *koff), struct.pack("<Q", len(vb)), vb,
                struct.pack(f"<{len(voff)}Q", *voff)]
    path.write_bytes(b"".join(out))


def test_boundary_struct_layout():
    """the C++ caller's view of every caller-allocated struct matches the library's (no GPU)"""
    r = subprocess.run([_binary(), "--sizes"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith("OK")


@pytest.mark.gpu
def test_boundary_out_bound_simple(tmp_path):
    fx = tmp_path / "qb_fixture.bin"
    write_fixture(fx)
    r = subprocess.run([_binary(), str(fx)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
