"""Smile binary-JSON codec (the reference's ``useSmile`` wire format, sd/client/DruidClient.scala:183-189,
244-251, 304-314) and the Druid HTTP endpoint / client speaking it."""
import math

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from spark_druid_olap_amd.client import smile
from spark_druid_olap_amd.client.druid_client import DruidQueryServerClient
from spark_druid_olap_amd.engine.executor import Engine
from spark_druid_olap_amd.models.bench_queries import DRUID_JSON
from spark_druid_olap_amd.server.druid_http import DruidHTTPServer
from spark_druid_olap_amd.session import Session


def test_known_encodings():
    # header + shared-names flag, then the token values from the Smile format specification
    assert smile.dumps(None) == b":)\n\x01\x21"
    assert smile.dumps(True)[4:] == b"\x23" and smile.dumps(False)[4:] == b"\x22"
    assert smile.dumps(0)[4:] == b"\xc0" and smile.dumps(-1)[4:] == b"\xc1" and smile.dumps(15)[4:] == b"\xde"
    assert smile.dumps(16)[4:] == b"\x24\xa0"            # zigzag 32, VInt last byte 0x80|32
    assert smile.dumps(1000)[4:] == b"\x24\x1f\x90"      # zigzag 2000 = 31<<6 | 16
    assert smile.dumps("")[4:] == b"\x20"
    assert smile.dumps("a")[4:] == b"\x40a"
    assert smile.dumps({"a": 1})[4:] == b"\xfa\x80a\xc2\xfb"
    assert smile.dumps([1, 2])[4:] == b"\xf8\xc2\xc4\xf9"
    # second occurrence of a key is a short shared-name reference
    assert smile.dumps([{"ab": 1}, {"ab": 2}])[4:] == b"\xf8\xfa\x81ab\xc2\xfb\xfa\x40\xc4\xfb\xf9"


json_values = st.recursive(
    st.none() | st.booleans() | st.integers(min_value=-(1 << 70), max_value=1 << 70) |
    st.floats(allow_nan=False) | st.text(max_size=80),
    lambda ch: st.lists(ch, max_size=6) | st.dictionaries(st.text(max_size=70), ch, max_size=6),
    max_leaves=30)


@settings(max_examples=300, deadline=None)
@given(json_values, st.booleans(), st.booleans())
def test_roundtrip(v, shared_names, shared_values):
    assert smile.loads(smile.dumps(v, shared_names=shared_names, shared_values=shared_values)) == v


def test_many_shared_names_and_values_reset():
    doc = [{f"k{i}": f"value-{i % 1500}", "druid": i} for i in range(3000)]
    for sv in (False, True):
        assert smile.loads(smile.dumps(doc, shared_values=sv)) == doc


def test_binary_and_special_floats():
    for b in (b"", b"\x00", b"abcdefg", bytes(range(256))):
        assert smile.loads(smile.dumps(b)) == b
    assert math.isinf(smile.loads(smile.dumps(float("inf"))))
    assert math.isnan(smile.loads(smile.dumps(float("nan"))))


def test_rejects_garbage():
    with pytest.raises(smile.SmileError):
        smile.loads(b'{"a": 1}')
    with pytest.raises(smile.SmileError):
        smile.loads(b":)\n\x01\xfa\x80a")


def test_druid_endpoint_speaks_smile(ds_small):
    s = Session(engine=Engine(use_native=False))
    s.register_datasource(ds_small)
    h = DruidHTTPServer(s, port=0).start()
    try:
        js = DruidQueryServerClient("127.0.0.1", h.port)
        sm = DruidQueryServerClient("127.0.0.1", h.port, use_smile=True)
        for name in ("TPCH Q1", "TPCH Q7"):
            a, b = js.execute_query(DRUID_JSON[name]), sm.execute_query(DRUID_JSON[name])
            assert a == b, name
        assert sm.time_boundary("tpch") == js.time_boundary("tpch")
    finally:
        h.stop()
