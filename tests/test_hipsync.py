"""utils/hipsync.py: the server's GPU wait mode (no GPU here: the call must fail soft)."""
import pytest

from spark_druid_olap_amd.utils import hipsync


def test_unknown_mode_is_rejected():
    with pytest.raises(ValueError):
        hipsync.set_wait_mode("busy")


def test_without_a_device_the_flag_is_not_claimed(monkeypatch):
    import ctypes

    class _Hip:
        def hipSetDevice(self, d):
            return 100  # hipErrorNoDevice

        def hipSetDeviceFlags(self, f):
            return 100

    monkeypatch.setattr(ctypes, "CDLL", lambda name: _Hip())
    assert hipsync.set_wait_mode("blocking") is False
    assert hipsync.set_wait_mode("blocking", 0) is False


def test_applied_mode_is_recorded(monkeypatch):
    import ctypes

    seen = []

    class _Hip:
        def hipSetDevice(self, d):
            seen.append(("dev", d.value))
            return 0

        def hipSetDeviceFlags(self, f):
            seen.append(("flags", f.value))
            return 0

    monkeypatch.setattr(ctypes, "CDLL", lambda name: _Hip())
    assert hipsync.set_wait_mode("blocking", 3)
    assert seen == [("dev", 3), ("flags", hipsync.HIP_DEVICE_SCHEDULE_BLOCKING_SYNC)]
    assert hipsync.wait_mode()[3] == "blocking"
