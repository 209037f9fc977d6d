"""Extracts the BLS12-381 pin fixtures (data only) from the reference:
  * p, r of BLS12-381 (std/math/emulated/emparams/emparams.go:145-171);
  * the compressed G1 points (48 B, Zcash/bellman encoding) of the BLS12-381
    Groth16 verifying keys and proofs in backend/groth16/bellman_test.go:19-132
    (vk alpha_g1, proof A, proof C of every case) and the compressed G2 points
    (96 B: vk beta_g2, gamma_g2, delta_g2, proof B).
Run in the build container (where /root/reference exists):
    python tests/golden/make_golden_bls.py
Writes tests/golden/bls12_381_pins.json."""
import base64
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    em = open(os.path.join(REF, "std/math/emulated/emparams/emparams.go")).read()
    i = em.index("type BLS12381Fp struct")
    fp_hex = re.findall(r"0x([0-9a-f]+) \(base 16\)", em[:i])[-1]
    j = em.index("type BLS12381Fr struct")
    fr_hex = re.findall(r"0x([0-9a-f]+) \(base 16\)", em[i:j])[-1]
    src = open(os.path.join(REF, "backend/groth16/bellman_test.go")).read()
    cases = re.findall(r'\{\s*"([A-Za-z0-9+/=]+)",\s*"([A-Za-z0-9+/=]+)",\s*"([A-Za-z0-9+/=]*)",\s*(true|false)', src)
    pts, g2 = [], []
    for vk, proof, _, _ in cases:
        v = base64.b64decode(vk)
        p = base64.b64decode(proof)
        pts += [v[:48].hex(), p[:48].hex(), p[144:192].hex()]
        # vk: [a]1 [b]1 [b]2 [g]2 [d]1 [d]2 (marshal.go:191-215); proof: Ar Bs Krs
        g2 += [v[96:192].hex(), v[192:288].hex(), v[336:432].hex(), p[48:144].hex()]
    out = {"source": ["std/math/emulated/emparams/emparams.go:145-171",
                      "backend/groth16/bellman_test.go:19-132"],
           "p_hex": fp_hex, "r_hex": fr_hex, "g1_compressed": sorted(set(pts)),
           "g2_compressed": sorted(set(g2))}
    json.dump(out, open(os.path.join(HERE, "bls12_381_pins.json"), "w"), indent=1)
    print(len(out["g1_compressed"]), "points")


if __name__ == "__main__":
    main()
