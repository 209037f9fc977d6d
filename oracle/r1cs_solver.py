"""TEST INFRASTRUCTURE ONLY (the checker of tests/test_gpu_solver.py, never the
product path): the R1CS solver of constraint/bn254/solver.go restated in Python
big-int arithmetic, for circuits without hints.

    levels_of   blueprint_r1cs.go:61-96 + core.go:405-419 (r1cs.Levels): an R1C
                sits one level above the deepest internal wire it reads; its
                still-unplaced wires are placed at that level.  Computed here
                by a memoised dependency walk (producer of each wire), a
                different route from the mirror's single pass.
    solve       solver.go:65-114 (witness at wires 1.., ONE_WIRE = 1) and
                solveR1C solver.go:535-608 (the unsolved term's wire from
                c / b - a, c / a - b or a b - c, divided by its coefficient; a
                zero divisor leaves it 0 after the a b == c check), levels in
                order; returns (W, A, B, C) or raises Unsatisfied(cid).
"""
from __future__ import annotations

from bn254_oracle import R, inv


class Unsatisfied(Exception):
    def __init__(self, cid, why):
        super().__init__("constraint #%d is not satisfied: %s" % (cid, why))
        self.cid = cid


def levels_of(nb_inputs, constraints):
    producer = {}
    for c, (L, Rr, O) in enumerate(constraints):
        for w, _ in list(L) + list(Rr) + list(O):
            if w >= nb_inputs and w not in producer:
                producer[w] = c
    lvl = {}

    def level(c):
        if c in lvl:
            return lvl[c]
        L, Rr, O = constraints[c]
        deps = [producer[w] for w, _ in list(L) + list(Rr) + list(O)
                if w >= nb_inputs and producer[w] != c]
        lvl[c] = 1 + max((level(d) for d in deps), default=-1)
        return lvl[c]

    out = []
    for c in range(len(constraints)):
        lv = level(c)
        while len(out) <= lv:
            out.append([])
        out[lv].append(c)
    return out


def solve(nb_wires, nb_inputs, constraints, witness, levels, R=R):
    """witness: the nb_inputs - 1 values after ONE_WIRE (R: the scalar field,
    BN254 by default; constraint/bls12-381/solver.go is the same code)."""
    W = [0] * nb_wires
    solved = [False] * nb_wires
    W[0], solved[0] = 1, True
    for i, v in enumerate(witness):
        W[1 + i], solved[1 + i] = v % R, True
    n = len(constraints)
    A, B, C = [0] * n, [0] * n, [0] * n
    for level in levels:
        for c in level:
            acc = [0, 0, 0]
            unknown = None
            for s, side in enumerate(constraints[c]):
                for w, k in side:
                    if solved[w]:
                        acc[s] = (acc[s] + k * W[w]) % R
                    elif unknown is not None:
                        raise Unsatisfied(c, "more than one wire to instantiate")
                    else:
                        unknown = (s, w, k % R)
            a, b, cc = acc
            if unknown is None:
                if a * b % R != cc:
                    raise Unsatisfied(c, "a b != c")
            else:
                s, w, k = unknown
                v = 0
                if s == 0:
                    if b:
                        v = (cc * inv(b, R) - a) % R
                        acc[0] = (a + v) % R
                    elif a * b % R != cc:
                        raise Unsatisfied(c, "a b != c")
                elif s == 1:
                    if a:
                        v = (cc * inv(a, R) - b) % R
                        acc[1] = (b + v) % R
                    elif a * b % R != cc:
                        raise Unsatisfied(c, "a b != c")
                else:
                    v = (a * b - cc) % R
                    acc[2] = (cc + v) % R
                W[w] = v * inv(k, R) % R
                solved[w] = True
            A[c], B[c], C[c] = acc
    if not all(solved):
        raise Unsatisfied(-1, "solver didn't assign a value to all wires")
    return W, A, B, C


def random_circuit(rng, nb_public, nb_secret, n_internal, zero_divisor=False, R=R):
    """A random R1CS the frontend could emit: every constraint introduces one new
    internal wire on a random side (L, R or O) with a random coefficient, next
    to up to two solved terms per side; with zero_divisor, some constraints
    multiply the new wire by a side that evaluates to zero (the wire is then 0)."""
    nin = nb_public + nb_secret
    cons = []
    known = list(range(nin))
    for j in range(n_internal):
        new = nin + j
        sides = [[], [], []]
        for s in range(3):
            for _ in range(rng.randrange(1, 3)):
                sides[s].append((rng.choice(known), rng.randrange(1, R)))
        tgt = rng.randrange(3)
        sides[tgt].append((new, rng.randrange(1, R)))
        zero = zero_divisor and tgt < 2 and rng.random() < 0.3
        if zero:
            sides[1 - tgt] = [(0, 0)]  # evaluates to zero: a b == c needs c == 0
            sides[2] = [(0, 0)]
        cons.append(tuple(sides))
        if not zero:  # the zero-divisor wire (0) is never read: no other side collapses
            known.append(new)
    return cons
