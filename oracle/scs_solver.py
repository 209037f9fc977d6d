"""TEST INFRASTRUCTURE ONLY (the checker of tests/test_gpu_scs_solver.py): the
sparse-R1CS (PlonK) solver restated in Python big-int arithmetic.

    levels_of  blueprint.go updateInstructionTree over (xa, xb, xc): a
               constraint sits one level above the deepest internal wire it
               reads; computed here by a memoised producer walk
    solve      BlueprintGenericSparseR1C.Solve (blueprint_scs.go:53-151): at
               most one unsolved wire among xa, xb, xc, solved from
               qL xa + qR xb + qO xc + qM xa xb + qC = 0; errDivideByZero on a
               zero denominator; commitment constraints skipped
    lro        evaluateLROSmallDomain (constraint/bls12-381/system.go:221-264)
"""
from __future__ import annotations


class Unsatisfied(Exception):
    def __init__(self, cid, why):
        super().__init__("constraint #%d: %s" % (cid, why))
        self.cid = cid


def levels_of(nb_inputs, cons):
    producer = {}
    for c, k in enumerate(cons):
        for w in k[:3]:
            if w >= nb_inputs and w not in producer:
                producer[w] = c
    lvl = {}

    def level(c):
        if c not in lvl:
            deps = [producer[w] for w in cons[c][:3] if w >= nb_inputs and producer[w] != c]
            lvl[c] = 1 + max((level(d) for d in deps), default=-1)
        return lvl[c]

    out = []
    for c in range(len(cons)):
        lv = level(c)
        while len(out) <= lv:
            out.append([])
        out[lv].append(c)
    return out


def solve(mod, n_wires, cons, witness, levels, flags=None):
    """cons[c] = (xa, xb, xc, qL, qR, qO, qM, qC); witness at wires 0.."""
    W = [0] * n_wires
    solved = [False] * n_wires
    for i, v in enumerate(witness):
        W[i], solved[i] = v % mod, True
    inv = lambda x: pow(x, mod - 2, mod)
    for level in levels:
        for c in level:
            if flags is not None and flags[c] & 1:
                continue
            xa, xb, xc, qL, qR, qO, qM, qC = cons[c]
            sa, sb, sc = solved[xa], solved[xb], solved[xc]
            if (not sa) + (not sb) + (not sc) > 1 or (not sa and xa == xb):
                raise Unsatisfied(c, "more than one unsolved wire")
            a, b, o = W[xa], W[xb], W[xc]
            if not sa or not sb:
                den = (qM * b + qL) % mod if not sa else (qM * a + qR) % mod
                if den == 0:
                    raise Unsatisfied(c, "division by zero")
                num = ((qR * b) if not sa else (qL * a)) + qO * o + qC
                w = xa if not sa else xb
                W[w] = (-num * inv(den)) % mod
                solved[w] = True
            elif not sc:
                if qO % mod == 0:
                    raise Unsatisfied(c, "division by zero")
                t = qM * a * b + qL * a + qR * b + qC
                W[xc] = (-t * inv(qO % mod)) % mod
                solved[xc] = True
            elif (qM * a * b + qL * a + qR * b + qO * o + qC) % mod:
                raise Unsatisfied(c, "not satisfied")
    if not all(solved):
        raise Unsatisfied(-1, "solver didn't assign a value to all wires")
    return W


def lro(W, cons, nb_public):
    n = len(cons) + nb_public
    s = 1
    while s < n:
        s <<= 1
    s0 = W[0]
    L, R, O = [s0] * s, [s0] * s, [s0] * s
    for i in range(nb_public):
        L[i] = W[i]
    for j, k in enumerate(cons):
        L[nb_public + j], R[nb_public + j], O[nb_public + j] = W[k[0]], W[k[1]], W[k[2]]
    return L, R, O


def random_circuit(rng, mod, nb_public, nb_secret, n_cons, commit_every=0):
    """Random SCS constraints as gnark's frontend emits them: each introduces one
    new internal wire at xa, xb or xc (qO = -1 add / mul gates and generic
    forms with random coefficients), plus assertions over solved wires and, with
    commit_every, commitment-flagged rows (flags[c] = 1, skipped by the solver)."""
    nin = nb_public + nb_secret
    cons, flags = [], []
    known = list(range(nin))
    nxt = nin
    for c in range(n_cons):
        if commit_every and c % commit_every == commit_every - 1:
            cons.append((rng.choice(known), 0, 0, mod - 1, 0, 0, 0, 0))
            flags.append(1)
            continue
        r = rng.random()
        x, y = rng.choice(known), rng.choice(known)
        if r < 0.3:      # xc = x * y (Mul blueprint: qM, qO = -1)
            cons.append((x, y, nxt, 0, 0, mod - 1, rng.randrange(1, mod), 0))
        elif r < 0.55:   # xc = qL x + qR y + qC (Add blueprint)
            cons.append((x, y, nxt, rng.randrange(mod), rng.randrange(mod), mod - 1, 0, rng.randrange(mod)))
        elif r < 0.75:   # the new wire at xa: (qL + qM y) xa + qR y + qO z + qC = 0
            cons.append((nxt, y, x, rng.randrange(1, mod), rng.randrange(mod), rng.randrange(mod),
                         rng.randrange(mod), rng.randrange(mod)))
        elif r < 0.95:   # the new wire at xb
            cons.append((x, nxt, y, rng.randrange(mod), rng.randrange(1, mod), rng.randrange(mod),
                         rng.randrange(mod), rng.randrange(mod)))
        else:            # an assertion over solved wires (fill_assertions)
            cons.append(None)
            flags.append(0)
            continue
        flags.append(0)
        known.append(nxt)
        nxt += 1
    return cons, flags, nxt


def fill_assertions(mod, cons, witness):
    """Replace the None placeholders by satisfied assertions over the first two
    witness wires: xa - xb + (w1 - w0) = 0 (qL = 1, qR = -1, qO = 0)."""
    qc = (witness[1] - witness[0]) % mod
    return [k if k is not None else (0, 1, 0, 1, mod - 1, 0, 0, qc) for k in cons]
