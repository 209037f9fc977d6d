"""NTT domain + transforms (replaces iciclegnark GenerateTwiddleFactors /
INttOnDevice / NttOnDevice / ReverseScalars, icicle.go:68-76, 489-510, and
gnark-crypto fft.Domain.FFT / FFTInverse at prove.go:369-393)."""
from __future__ import annotations

import ctypes

from . import fr
from ._lib import GG_CURVE_BLS12_381, GG_CURVE_BN254, GG_DIF, GG_DIT, DeviceBuffer, check, lib, ptr

DIF, DIT = GG_DIF, GG_DIT


class Domain:
    """Device-resident radix-2 domain of size 2^log_n.

    omega / coset_gen default to gnark-crypto's fft.NewDomain choice; pass
    pk.Domain.Generator / FrMultiplicativeGen (Montgomery bytes) to mirror a key."""

    def __init__(self, log_n: int, omega_mont: bytes = None, coset_gen_mont: bytes = None,
                 curve: int = GG_CURVE_BN254):
        if curve == GG_CURVE_BN254:
            if omega_mont is None:
                omega_mont = fr.fr_mont(fr.domain_generator(log_n))
            if coset_gen_mont is None:
                coset_gen_mont = fr.fr_mont(fr.FR_MULTIPLICATIVE_GEN)
        elif omega_mont is None or coset_gen_mont is None:
            # BLS12-381: take Generator / FrMultiplicativeGen from pk.Domain
            raise ValueError("BLS12-381 domains need omega and the coset generator (pk.Domain)")
        h = ctypes.c_void_p()
        check(lib.gg_domain_create_ex(curve, log_n, ptr(omega_mont), ptr(coset_gen_mont),
                                      ctypes.byref(h)))
        self.curve = curve
        self.handle = h
        self.log_n = log_n
        self.cardinality = 1 << log_n

    def fft(self, data_dev, decimation=DIF, coset=False, stream=None):
        """domain.FFT(a, decimation, [OnCoset()]) in place on device data."""
        check(lib.gg_ntt(self.handle, ptr(data_dev), 0, decimation, int(coset), ptr(stream)))

    def fft_inverse(self, data_dev, decimation=DIF, coset=False, stream=None):
        """domain.FFTInverse(a, decimation, [OnCoset()]) in place on device data."""
        check(lib.gg_ntt(self.handle, ptr(data_dev), 1, decimation, int(coset), ptr(stream)))

    def compute_h(self, a, b, c, length: int, h_dev, inputs_on_device=False, stream=None):
        """Fused Groth16 computeH (prove.go:353-396): h (bit-reversed) into h_dev."""
        check(lib.gg_groth16_compute_h(self.handle, ptr(a), ptr(b), ptr(c), length,
                                       int(inputs_on_device), ptr(h_dev), ptr(stream)))

    def close(self):
        if self.handle:
            lib.gg_domain_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fft_host(data: bytes, log_n: int, inverse: bool, decimation: int, coset: bool,
             domain: Domain = None) -> bytes:
    """Convenience: upload, transform on the GPU, download."""
    d = domain or Domain(log_n)
    buf = DeviceBuffer.from_host(data)
    if inverse:
        d.fft_inverse(buf, decimation, coset)
    else:
        d.fft(buf, decimation, coset)
    check(lib.gg_synchronize())
    return buf.to_host()
