"""GPU NTT / computeH parity through the C ABI (gg_ntt, gg_groth16_compute_h)."""
import numpy as np
import pytest

import coracle
from helpers import b, golden, random_fr_mont

pytestmark = pytest.mark.gpu

VARIANTS = [(inv, dif, cos) for inv in (0, 1) for dif in (0, 1) for cos in (0, 1)]


def gpu_fft(data, log_n, inverse, dif, coset, dom=None):
    from gnark_amd import ntt
    dec = ntt.DIF if dif else ntt.DIT
    return ntt.fft_host(data, log_n, bool(inverse), dec, bool(coset), dom)


def test_ntt_golden():
    for c in golden()["ntt"]:
        got = gpu_fft(b(c["input"]), c["log_n"], c["inverse"], c["dif"], c["coset"])
        assert got.hex() == c["expected"], c


@pytest.mark.parametrize("log_n", [2, 8, 11, 12, 13, 16, 19, 20])
def test_ntt_vs_oracle(log_n):
    from gnark_amd import ntt
    dom = ntt.Domain(log_n)
    v = random_fr_mont(1 << log_n, 100 + log_n).tobytes()
    for inv, dif, cos in VARIANTS:
        exp = coracle.ntt(v, log_n, inv, dif, cos)
        got = gpu_fft(v, log_n, inv, dif, cos, dom)
        assert got == exp, (log_n, inv, dif, cos)


def test_ntt_roundtrip_2p24():
    """BASELINE config 3: 2^24 forward then inverse is the identity (bit-exact)."""
    from gnark_amd import ntt, DeviceBuffer
    from gnark_amd._lib import check, lib
    log_n = 24
    dom = ntt.Domain(log_n)
    v = random_fr_mont(1 << log_n, 7).tobytes()
    buf = DeviceBuffer.from_host(v)
    dom.fft(buf, ntt.DIF, coset=True)          # natural -> bit-reversed evals on coset
    dom.fft_inverse(buf, ntt.DIT, coset=True)  # bit-reversed -> natural coefficients
    check(lib.gg_synchronize())
    assert buf.to_host() == v
    dom.fft(buf, ntt.DIT)                      # treat as bit-reversed input
    dom.fft_inverse(buf, ntt.DIF)
    check(lib.gg_synchronize())
    assert buf.to_host() == v


@pytest.mark.parametrize("inv,dif,cos", [(0, 1, 0), (0, 0, 1), (1, 1, 1)])
def test_ntt_2p24_vs_oracle(inv, dif, cos):
    """BASELINE configs[2] at its size: 2^24 transforms compared element for
    element with the C oracle (the computeH forms: DIF iFFT, coset DIT FFT,
    coset DIF iFFT)."""
    log_n = 24
    v = random_fr_mont(1 << log_n, 24 + 2 * inv + dif).tobytes()
    assert gpu_fft(v, log_n, inv, dif, cos) == coracle.ntt(v, log_n, inv, dif, cos)


def test_ntt_2p22_vs_oracle_single_variant():
    log_n = 22
    v = random_fr_mont(1 << log_n, 8).tobytes()
    assert gpu_fft(v, log_n, 1, 1, 0) == coracle.ntt(v, log_n, 1, 1, 0)


def test_compute_h_golden():
    from gnark_amd import ntt, DeviceBuffer
    for g in golden()["groth16"]:
        dom = ntt.Domain(g["log_n"])
        a, bb, c = b(g["solA"]), b(g["solB"]), b(g["solC"])
        h = DeviceBuffer(32 << g["log_n"])
        dom.compute_h(a, bb, c, len(a) // 32, h)
        assert h.to_host().hex() == g["h"]


@pytest.mark.parametrize("log_n,fill", [(4, 13), (10, 1000), (16, 60000), (20, (1 << 20) - 5)])
def test_compute_h_vs_oracle(log_n, fill):
    from gnark_amd import ntt, DeviceBuffer
    dom = ntt.Domain(log_n)
    a = random_fr_mont(fill, 1).tobytes()
    bb = random_fr_mont(fill, 2).tobytes()
    c = random_fr_mont(fill, 3).tobytes()
    exp = coracle.compute_h(a, bb, c, fill, log_n)
    h = DeviceBuffer(32 << log_n)
    dom.compute_h(a, bb, c, fill, h)
    assert h.to_host() == exp
    # inputs already resident on the device
    da, db, dc = (DeviceBuffer.from_host(x) for x in (a, bb, c))
    h2 = DeviceBuffer(32 << log_n)
    dom.compute_h(da, db, dc, fill, h2, inputs_on_device=True)
    assert h2.to_host() == exp
