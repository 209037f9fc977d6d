"""Pins the CPU oracle against every fixture the reference itself holds for
this path.  No reference run is possible (no Go toolchain)."""
import bn254_oracle as o


def test_moduli_match_reference_solidity():
    # backend/groth16/bn254/solidity.go:41-42
    assert o.P == 0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47
    assert o.R == 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001


def test_domain_generator_pinned_by_fri_test():
    # std/commitments/fri/fri_test.go:35: inverse of the generator of the size-256 domain
    g_inv = 14607982016670611764231825270871087984049314771307170893064215224383340934614
    d = o.Domain(256)
    assert d.generator_inv == g_inv
    assert d.generator == pow(g_inv, -1, o.R)
    # consistent with the 2^28 root used for every size
    d28 = o.Domain(1 << 28)
    assert pow(d28.generator, 1 << 20, o.R) == d.generator


def test_witness_encoding_kat():
    # backend/witness/witness.go:33-36 (Y=35 public, X=3, Z=2 secret)
    kat = ("00000001000000020000000300000000000000000000000000000000000000000000000000000000000000"
           "2300000000000000000000000000000000000000000000000000000000000000030000000000000000000000"
           "000000000000000000000000000000000000000002")
    assert o.witness_encode([35], [3, 2]).hex() == kat


def test_filter_heap_kats():
    # backend/groth16/bn254/utils_test.go:17-38
    e = [0, 1, 2, 3]
    assert o.filter_heap(e, 0, [1, 2]) == [0, 3]
    assert o.filter_heap(e[1:], 1, [1, 2]) == [3]
    assert o.filter_heap(e, 0, [1, 1, 2]) == [0, 3]
    assert o.filter_heap(e[1:], 1, [1, 1, 2]) == [3]


def test_cubic_circuit_satisfied():
    # examples/cubic: x**3 + x + 5 == y with X=3, Y=35 (cubic_test.go)
    rcs = o.cubic_r1cs()
    A, B, C = rcs.solution(o.cubic_witness(3, 35))
    assert A == [3, 9, 1] and B == [3, 3, 35] and C == [9, 27, 35]


def test_generators_and_subgroups():
    assert o.on_curve_g1(o.G1_GEN) and o.on_curve_g2(o.G2_GEN)
    assert o.g1_mul(o.G1_GEN, o.R) is None
    assert o.g2_mul(o.G2_GEN, o.R) is None


def test_groth16_cubic_verifies_with_pairing():
    """The reference's own correctness signal is Verify (verify.go:43-140);
    the oracle's prover output passes it and a wrong public input fails."""
    rcs = o.cubic_r1cs()
    tw = o.ToxicWaste(1234567, 891011, 121314, 151617, 181920)
    pk, vk = o.setup(rcs, tw)
    pr = o.prove(rcs, pk, o.cubic_witness(), 4242, 5353)
    assert o.verify(pr, vk, [35])
    assert not o.verify(pr, vk, [36])


def test_groth16_trapdoor_identity():
    rcs = o.mimc_chain_r1cs(2, 2)
    w = o.mimc_chain_witness(rcs, [7, 11])
    tw = o.ToxicWaste(3, 5, 7, 11, 13)
    pk, vk = o.setup(rcs, tw)
    pr = o.prove(rcs, pk, w, 17, 19)
    a, b, c = o.expected_proof_scalars(rcs, tw, w, 17, 19)
    assert pr.Ar == o.g1_mul(o.G1_GEN, a)
    assert pr.Bs == o.g2_mul(o.G2_GEN, b)
    assert pr.Krs == o.g1_mul(o.G1_GEN, c)
    assert o.verify(pr, vk, [])


def test_ntt_roundtrips_and_definition():
    rng = o.SplitMix64(3)
    for n in (1, 2, 8, 32):
        d = o.Domain(n)
        v = [rng.fr() for _ in range(n)]
        # FFT(DIF) = evaluations in bit-reversed order
        ev = o.fft(d, list(v), o.DIF)
        for i in range(n):
            x = pow(d.generator, o.bitrev(i, d.log_n), o.R)
            assert ev[i] == sum(c * pow(x, k, o.R) for k, c in enumerate(v)) % o.R
        # inverse round trips with every decimation / coset combination
        for dec in (o.DIF, o.DIT):
            for coset in (False, True):
                a = list(v)
                if dec == o.DIF:
                    o.fft(d, a, o.DIF, coset)
                    a = [a[o.bitrev(i, d.log_n)] for i in range(n)]
                    o.fft_inverse(d, a, o.DIF, coset)
                    a = [a[o.bitrev(i, d.log_n)] for i in range(n)]
                else:
                    a = [a[o.bitrev(i, d.log_n)] for i in range(n)]
                    o.fft(d, a, o.DIT, coset)
                    a = [a[o.bitrev(i, d.log_n)] for i in range(n)]
                    o.fft_inverse(d, a, o.DIT, coset)
                assert a == v, (n, dec, coset)


def test_compute_h_divides():
    """h(X) * (X^n - 1) == A(X) B(X) - C(X) (evaluated at a random point)."""
    rcs = o.mimc_chain_r1cs(1, 3)
    w = o.mimc_chain_witness(rcs, [9])
    A, B, C = rcs.solution(w)
    d = o.Domain(len(A))
    h = o.compute_h(A, B, C, d)
    coeffs = [h[o.bitrev(i, d.log_n)] for i in range(d.cardinality)]
    x = 987654321

    def interp_eval(vals):
        vals = list(vals) + [0] * (d.cardinality - len(vals))
        c = o.fft_inverse(d, vals, o.DIF)
        c = [c[o.bitrev(i, d.log_n)] for i in range(d.cardinality)]
        return sum(ci * pow(x, k, o.R) for k, ci in enumerate(c)) % o.R

    hx = sum(ci * pow(x, k, o.R) for k, ci in enumerate(coeffs)) % o.R
    lhs = hx * (pow(x, d.cardinality, o.R) - 1) % o.R
    rhs = (interp_eval(A) * interp_eval(B) - interp_eval(C)) % o.R
    assert lhs == rhs
