"""Serving processes set the caching allocator's garbage-collection threshold unless the user set
an allocator configuration of their own (utils/memory.py serving_allocator_conf)."""
from spark_druid_olap_amd.utils import memory as M


def test_sets_conf_when_unset(monkeypatch):
    monkeypatch.delenv("PYTORCH_HIP_ALLOC_CONF", raising=False)
    monkeypatch.delenv("PYTORCH_CUDA_ALLOC_CONF", raising=False)
    assert M.serving_allocator_conf()
    import os

    assert os.environ["PYTORCH_HIP_ALLOC_CONF"] == M.SERVING_ALLOC_CONF


def test_user_conf_wins(monkeypatch):
    import os

    monkeypatch.delenv("PYTORCH_HIP_ALLOC_CONF", raising=False)
    monkeypatch.setenv("PYTORCH_CUDA_ALLOC_CONF", "expandable_segments:True")
    assert not M.serving_allocator_conf()
    assert "PYTORCH_HIP_ALLOC_CONF" not in os.environ
    monkeypatch.setenv("PYTORCH_HIP_ALLOC_CONF", "max_split_size_mb:512")
    assert not M.serving_allocator_conf()
    assert os.environ["PYTORCH_HIP_ALLOC_CONF"] == "max_split_size_mb:512"
