"""Host sanitizer coverage.

* ``test_gateway_fuzz_malformed_frames``: hostile bytes against the native HiveServer2 gateway
  (server/csrc/hs2_gateway.cpp): random frames, lying length prefixes, oversize list/string
  counts, deep nesting, truncated SASL.  The gateway must drop the connection and keep serving.
  In the normal suite this checks robustness; under ``tools/asan_host.py`` the same test runs
  against the ASan/UBSan build, so any out-of-bounds read or UB in the codec aborts the run.
* ``test_asan_host_run``: builds the instrumented gateway (g++ -fsanitize=address,undefined) and
  the instrumented HIP bindings (hipcc -Xarch_host -fsanitize=address) and runs both drivers.
"""
import os
import random
import socket
import struct
import subprocess
import sys

import pytest

from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models import tpch
from spark_druid_olap_amd.server.hive_client import connect
from spark_druid_olap_amd.session import Session

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def native_server(ds_small, df_small):
    from spark_druid_olap_amd.server.gateway import NativeHiveServer

    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    s.register_table("orderLineItemPartSupplierBase", df_small, schema=tpch.FLAT_SCHEMA)
    s.sql(tpch.druid_ddl(with_column_mapping=False))
    srv = NativeHiveServer(s, port=0).start()
    yield srv
    srv.stop()


def _tstr(s: bytes) -> bytes:
    return struct.pack(">i", len(s)) + s


def _msg(name: bytes, body: bytes) -> bytes:
    return struct.pack(">I", 0x80010001) + _tstr(name) + struct.pack(">i", 1) + body


def _framed(b: bytes) -> bytes:
    return struct.pack(">i", len(b)) + b


def _hostile_payloads(rng: random.Random):
    yield b""
    yield b"\x00"
    yield struct.pack(">i", 0x7FFFFFFF) + b"\x80\x01"             # frame length far beyond what follows
    yield struct.pack(">i", -5) + b"abc"                            # negative frame length
    yield b"\x01" + struct.pack(">i", 5) + b"PLA"                   # truncated SASL start
    yield b"\x01" + struct.pack(">i", 0x7FFFFFF0) + b"PLAIN"       # SASL length lie
    yield _framed(_msg(b"OpenSession", b"\x0d\x00\x01" + b"\x0b\x0b" + struct.pack(">i", 0x7FFFFFFF)))  # huge map
    yield _framed(_msg(b"ExecuteStatement", b"\x0b\x00\x02" + struct.pack(">i", 0x7FFFFFFF) + b"sel"))  # str lie
    yield _framed(_msg(b"FetchResults", b"\x0f\x00\x01\x0c" + struct.pack(">i", 0x40000000)))  # list lie
    yield _framed(_msg(b"ExecuteStatement", b"\x0c\x00\x01" * 5000 + b"\x00" * 10))  # deep nesting
    yield _framed(_msg(b"NoSuchMethod", b"\x00"))
    yield _framed(struct.pack(">I", 0x80010001) + _tstr(b"\xff" * 40))  # truncated after the name
    yield _framed(b"\x80\x01\x00\x01" + struct.pack(">i", -1))      # negative name length
    for _ in range(60):
        n = rng.randrange(1, 300)
        body = bytes(rng.randrange(256) for _ in range(n))
        yield _framed(body) if rng.random() < 0.7 else body
        # well-formed header, random body
        yield _framed(_msg(rng.choice([b"ExecuteStatement", b"OpenSession", b"FetchResults", b"GetTables"]),
                           bytes(rng.randrange(256) for _ in range(rng.randrange(0, 120)))))


def _send(port: int, payload: bytes) -> None:
    with socket.create_connection(("127.0.0.1", port), timeout=2.0) as c:
        try:
            c.sendall(payload)
            c.shutdown(socket.SHUT_WR)
            c.settimeout(0.5)
            while c.recv(65536):
                pass
        except OSError:
            pass  # the gateway dropping the connection is the expected outcome


def test_gateway_fuzz_malformed_frames(native_server, df_small):
    rng = random.Random(1234)
    for p in _hostile_payloads(rng):
        _send(native_server.port, p)
    # still serving, with and without SASL
    for sasl in (True, False):
        with connect(port=native_server.port, sasl=sasl) as c:
            rows = c.cursor().execute("select count(*) from orderLineItemPartSupplier").fetchall()
            assert rows == [(len(df_small),)]


@pytest.mark.skipif(bool(os.environ.get("SDO_ASAN_CHILD")), reason="already inside the sanitized run")
def test_asan_host_run(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan_host.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "asan: compiled" in r.stdout, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error:" not in tail, tail
