"""Generates the committed golden fixtures in tests/golden/ from the pinned
Python oracle (oracle/bn254_oracle.py).  The reference itself cannot run here
(no Go toolchain, gnark-crypto absent), so these vectors are oracle outputs,
pinned by tests/test_oracle_pins.py (reference KATs + pairing Verify).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import bn254_oracle as o  # noqa: E402


def hx(b):
    return b.hex()


def msm_case(rng, n, group, edge=False):
    ks = [rng.fr() for _ in range(n)]
    ss = [rng.fr() for _ in range(n)]
    if edge and n >= 8:
        ss[0], ss[1], ss[2] = 0, 1, o.R - 1
        ks[4] = ks[3]            # repeated point (DummySetup-like P+P)
        ss[4] = ss[3]
        ks[6] = (o.R - ks[5]) % o.R  # P and -P
        ss[6] = ss[5]
    mul = o.g1_mul if group == 1 else o.g2_mul
    gen = o.G1_GEN if group == 1 else o.G2_GEN
    enc = o.g1_to_bytes if group == 1 else o.g2_to_bytes
    pts = [mul(gen, k) for k in ks]
    if edge and n >= 8:
        pts[7] = None            # infinity in the key (pk.G1.K may hold it)
    res = (o.msm_g1 if group == 1 else o.msm_g2)(pts, ss)
    return {"n": n, "group": group,
            "points": hx(b"".join(enc(p) for p in pts)),
            "scalars": hx(o.fr_vec_to_bytes(ss)),
            "expected": hx(enc(res))}


def main():
    rng = o.SplitMix64(0x67726F7468)
    out = {}
    out["msm"] = [msm_case(rng, n, 1, edge=(n == 16)) for n in (1, 3, 16, 100)]
    out["msm"] += [msm_case(rng, n, 2, edge=(n == 16)) for n in (1, 16)]
    ntt = []
    for log_n in (0, 1, 3, 5):
        n = 1 << log_n
        d = o.Domain(n)
        v = [rng.fr() for _ in range(n)]
        for inverse in (0, 1):
            for dec in (o.DIF, o.DIT):
                for coset in (0, 1):
                    f = o.fft_inverse if inverse else o.fft
                    r = f(d, list(v), dec, bool(coset))
                    ntt.append({"log_n": log_n, "inverse": inverse, "dif": int(dec == o.DIF),
                                "coset": coset, "input": hx(o.fr_vec_to_bytes(v)),
                                "expected": hx(o.fr_vec_to_bytes(r))})
    out["ntt"] = ntt

    def g16(name, rcs, w, tw, r, s, public):
        pk, vk = o.setup(rcs, tw)
        pr, h = o.prove(rcs, pk, w, r, s, return_h=True)
        assert o.verify(pr, vk, public)
        A, B, C = rcs.solution(w)
        return {
            "name": name, "log_n": pk.domain.log_n, "nb_public": rcs.nb_public,
            "g1_A": hx(b"".join(o.g1_to_bytes(p) for p in pk.g1_A)),
            "g1_B": hx(b"".join(o.g1_to_bytes(p) for p in pk.g1_B)),
            "g1_Z": hx(b"".join(o.g1_to_bytes(p) for p in pk.g1_Z)),
            "g1_K": hx(b"".join(o.g1_to_bytes(p) for p in pk.g1_K)),
            "g2_B": hx(b"".join(o.g2_to_bytes(p) for p in pk.g2_B)),
            "alpha1": hx(o.g1_to_bytes(pk.g1_alpha)), "beta1": hx(o.g1_to_bytes(pk.g1_beta)),
            "delta1": hx(o.g1_to_bytes(pk.g1_delta)), "beta2": hx(o.g2_to_bytes(pk.g2_beta)),
            "delta2": hx(o.g2_to_bytes(pk.g2_delta)),
            "infA": hx(bytes(int(x) for x in pk.infinity_A)),
            "infB": hx(bytes(int(x) for x in pk.infinity_B)),
            "wires": hx(o.fr_vec_to_bytes(w)),
            "solA": hx(o.fr_vec_to_bytes(A)), "solB": hx(o.fr_vec_to_bytes(B)),
            "solC": hx(o.fr_vec_to_bytes(C)),
            "r": hx(o.fr_to_bytes(r)), "s": hx(o.fr_to_bytes(s)),
            "h": hx(o.fr_vec_to_bytes(h)),
            "Ar": hx(o.g1_to_bytes(pr.Ar)), "Bs": hx(o.g2_to_bytes(pr.Bs)),
            "Krs": hx(o.g1_to_bytes(pr.Krs)), "raw_prefix": hx(pr.raw_bytes()),
        }

    out["groth16"] = [
        g16("cubic", o.cubic_r1cs(), o.cubic_witness(3, 35),
            o.ToxicWaste(1234567, 891011, 121314, 151617, 181920), 4242, 5353, [35]),
    ]
    rcs = o.mimc_chain_r1cs(3, 4)
    w = o.mimc_chain_witness(rcs, [5, 6, 7])
    out["groth16"].append(g16("mimc3x4", rcs, w, o.ToxicWaste(31, 37, 41, 43, 47), 53, 59, []))
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
