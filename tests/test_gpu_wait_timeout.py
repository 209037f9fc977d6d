"""Bounded host waits on a real stream (VERDICT r5 Weak #1: a stalled stream
must end in GG_ERR_TIMEOUT, not a blocked prover).  The CPU side of the same
deadline is test_capi.py::test_bounded_wait_times_out_instead_of_blocking."""
import time

import pytest

import coracle
from helpers import random_fr_mont, random_g1_points

pytestmark = pytest.mark.gpu


def test_stream_wait_deadline_returns_timeout_then_device_works():
    from gnark_amd import _lib, msm
    L = _lib.lib
    # one wave sleeping ~0.2 s against a 50-ms deadline: the library's stream
    # wait gives up with GG_ERR_TIMEOUT naming the wait (the wave drains after)
    t = time.time()
    rc = L.gg_wait_selftest_device(60000, 0.05)
    el = time.time() - t
    msg = L.gg_last_error().decode()
    assert rc == _lib.GG_ERR_TIMEOUT, (rc, msg)
    assert "timed out" in msg and "device selftest" in msg and "waiting for st" in msg, msg
    assert el < 30
    # the same wait under a generous deadline returns GG_OK
    assert L.gg_wait_selftest_device(1000, 30.0) == 0, L.gg_last_error()
    # the process-wide deadline is back to its value and the device still proves
    assert L.gg_get_wait_timeout() > 1
    n = 1 << 12
    pts = random_g1_points(n, 901)
    sc = random_fr_mont(n, 902)
    base = msm.MsmBase(msm.G1, pts, n)
    assert base.msm(sc, n) == coracle.msm_g1(pts.tobytes(), sc.tobytes(), n)
