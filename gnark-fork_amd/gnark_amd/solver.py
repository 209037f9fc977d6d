"""R1CS solver on MI355X: mirror of cs.R1CS's Solve for BN254 circuits without
hint calls (constraint/bn254/solver.go:418-608, system.go:64-104), the system
resident in HBM and the solution left there for the prover.

    sys = R1CS.from_terms(nb_public, nb_secret, n_wires, constraints)   # once
    sol = sys.solve(witness_values)            # -> groth16.Solution (on device)
    proof = groth16.prove(pk, sol, with_amd_acceleration())

``constraints`` are (L, R, O) lists of (wire, coefficient) pairs, the terms
r1cs.GetR1Cs() yields; the coefficient table and the CSR arrays are built here
(r1cs.Coefficients), and the levels are r1cs.Levels as gnark's level builder
assigns them (constraint/blueprint_r1cs.go:61-96: an R1C sits one level above
the deepest internal wire it reads and places its unsolved wires there)."""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import fr
from ._lib import check, lib, ptr, DeviceBuffer

GG_ERR_UNSATISFIED = 6


class UnsatisfiedConstraintError(RuntimeError):
    """solver.UnsatisfiedConstraintError (solver.go:610-623)."""

    def __init__(self, cid: int, msg: str):
        super().__init__(msg)
        self.cid = cid


def _schedule(fn, handle):
    s, nl, ns = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_size_t()
    check(fn(handle, ctypes.byref(s), ctypes.byref(nl), ctypes.byref(ns)))
    return bool(s.value), nl.value, ns.value


def compute_levels(nb_inputs: int, n_wires: int, term_off, term_wire) -> list:
    """r1cs.Levels from the CSR terms (blueprint_r1cs.go:61-96, core.go:405-419):
    wires < nb_inputs are inputs (not in the instruction tree)."""
    level = np.full(n_wires, -1, dtype=np.int64)
    ncons = (len(term_off) - 1) // 3
    out = []
    for c in range(ncons):
        lo, hi = int(term_off[3 * c]), int(term_off[3 * c + 3])
        mx, outs = -1, []
        for w in term_wire[lo:hi]:
            w = int(w)
            if w < nb_inputs:
                continue
            if level[w] < 0:
                outs.append(w)
            elif level[w] > mx:
                mx = int(level[w])
        mx += 1
        for w in outs:
            level[w] = mx
        while len(out) <= mx:
            out.append([])
        out[mx].append(c)
    return out


class R1CS:
    """Device-resident R1CS (gg_r1cs_create) with its solver."""

    def __init__(self, nb_public: int, nb_secret: int, n_wires: int, term_off, term_wire, term_coeff,
                 coeffs: Sequence[int], levels: Optional[Sequence[Sequence[int]]] = None,
                 curve: str = "bn254"):
        from ._lib import GG_CURVE_BN254, GG_CURVE_BLS12_381
        self.curve = curve
        self.mod = fr.R if curve == "bn254" else fr.BLS_R
        self._mont = fr.fr_mont if curve == "bn254" else fr.bls_fr_mont
        self.nb_public, self.nb_secret, self.n_wires = nb_public, nb_secret, n_wires
        self.term_off = np.ascontiguousarray(term_off, dtype=np.uint32)
        self.term_wire = np.ascontiguousarray(term_wire, dtype=np.uint32)
        self.term_coeff = np.ascontiguousarray(term_coeff, dtype=np.uint32)
        self.n_constraints = (len(self.term_off) - 1) // 3
        if levels is None:
            levels = compute_levels(nb_public + nb_secret, n_wires, self.term_off, self.term_wire)
        self.levels = levels
        lo = np.zeros(len(levels) + 1, dtype=np.uint32)
        lo[1:] = np.cumsum([len(x) for x in levels])
        lc = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.uint32) for x in levels])
                                  if levels else np.zeros(0, dtype=np.uint32), dtype=np.uint32)
        cbytes = b"".join(self._mont(int(k) % self.mod) for k in coeffs)
        h = ctypes.c_void_p()
        check(lib.gg_r1cs_create_ex(GG_CURVE_BN254 if curve == "bn254" else GG_CURVE_BLS12_381, n_wires,
                                    self.n_constraints, ptr(self.term_off), ptr(self.term_wire),
                                    ptr(self.term_coeff), ptr(cbytes), len(coeffs), ptr(lo), ptr(lc),
                                    len(levels), ctypes.byref(h)))
        self.handle = h
        # newSolver's witness-size check, enforced by the library too (solver.go:71-76)
        check(lib.gg_r1cs_set_inputs(h, nb_public, nb_secret))

    @classmethod
    def from_terms(cls, nb_public: int, nb_secret: int, n_wires: int, constraints, levels=None,
                   curve: str = "bn254") -> "R1CS":
        """constraints: [(L, R, O)] with L = [(wire, coeff int), ...]."""
        mod = fr.R if curve == "bn254" else fr.BLS_R
        table, index = [], {}
        off, wires, cids = [0], [], []
        for L, R, O in constraints:
            for side in (L, R, O):
                for w, k in side:
                    k %= mod
                    if k not in index:
                        index[k] = len(table)
                        table.append(k)
                    wires.append(w)
                    cids.append(index[k])
                off.append(len(wires))
        if not table:
            table = [1]
        return cls(nb_public, nb_secret, n_wires, off, wires, cids, table, levels, curve)

    def info(self):
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        check(lib.gg_r1cs_info(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def schedule(self):
        """(strands, launches, segments) of the last solve (gg_r1cs_schedule)."""
        return _schedule(lib.gg_r1cs_schedule, self.handle)

    def solve(self, witness, on_device: bool = True):
        """r1cs.Solve(fullWitness): witness = public (without ONE_WIRE) then
        secret values (ints, or Montgomery bytes / a DeviceBuffer).  Returns a
        groth16.Solution whose W, A, B, C live in HBM (on_device) or on the host."""
        from .groth16 import Solution
        n_in = self.nb_public - 1 + self.nb_secret
        wdev = False
        if isinstance(witness, DeviceBuffer):
            wbuf, wdev = witness, True
        elif isinstance(witness, (bytes, bytearray)):
            wbuf = bytes(witness)
        else:
            wbuf = b"".join(self._mont(int(v) % self.mod) for v in witness)
            if len(witness) != n_in:
                raise ValueError("invalid witness size, got %d, expected %d" % (len(witness), n_in))
        if not wdev and len(wbuf) != 32 * n_in:
            raise ValueError("invalid witness size, got %d bytes, expected %d" % (len(wbuf), 32 * n_in))
        nw, nc = self.n_wires, self.n_constraints
        if on_device:
            W, A, B, C = (DeviceBuffer(max(32 * k, 32)) for k in (nw, nc, nc, nc))
        else:
            W, A, B, C = (bytearray(32 * k) for k in (nw, nc, nc, nc))
        bad = ctypes.c_int64(-1)
        rc = lib.gg_r1cs_solve(self.handle, ptr(wbuf), n_in, int(wdev), ptr(W), ptr(A), ptr(B), ptr(C),
                               int(on_device), ctypes.byref(bad))
        if rc == GG_ERR_UNSATISFIED:
            raise UnsatisfiedConstraintError(bad.value, lib.gg_last_error().decode())
        check(rc)
        return Solution(W, A, B, C, nw, nc, on_device=on_device)

    def solve_resident(self, witness: bytes):
        """solve() without copies: the returned Solution points at the handle's own
        HBM buffers (valid until the next solve or close) -- the shape a prover
        pipeline uses (witness in, proof out, the solution never leaves HBM)."""
        from .groth16 import Solution
        n_in = self.nb_public - 1 + self.nb_secret
        if len(witness) != 32 * n_in:
            raise ValueError("invalid witness size, got %d bytes, expected %d" % (len(witness), 32 * n_in))
        bad = ctypes.c_int64(-1)
        rc = lib.gg_r1cs_solve(self.handle, ptr(witness), n_in, 0, None, None, None, None, 1, ctypes.byref(bad))
        if rc == GG_ERR_UNSATISFIED:
            raise UnsatisfiedConstraintError(bad.value, lib.gg_last_error().decode())
        check(rc)
        p = [ctypes.c_void_p() for _ in range(4)]
        check(lib.gg_r1cs_solution_dev(self.handle, *(ctypes.byref(x) for x in p)))
        return Solution(p[0], p[1], p[2], p[3], self.n_wires, self.n_constraints, on_device=True)

    def close(self):
        if getattr(self, "handle", None):
            lib.gg_r1cs_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def compute_scs_levels(nb_inputs: int, n_wires: int, wires) -> list:
    """r1cs.Levels of a sparse R1CS (blueprint.go updateInstructionTree over
    xa, xb, xc): wires < nb_inputs are the witness."""
    level = np.full(n_wires, -1, dtype=np.int64)
    w = np.asarray(wires, dtype=np.int64).reshape(-1, 3)
    out = []
    for c in range(len(w)):
        mx, outs = -1, []
        for x in w[c]:
            x = int(x)
            if x < nb_inputs:
                continue
            if level[x] < 0:
                if x not in outs:
                    outs.append(x)
            elif level[x] > mx:
                mx = int(level[x])
        mx += 1
        for x in outs:
            level[x] = mx
        while len(out) <= mx:
            out.append([])
        out[mx].append(c)
    return out


class SparseR1CS:
    """Device-resident sparse R1CS (gg_scs_create) with its solver: the PlonK
    side of r1cs.Solve (constraint/blueprint_scs.go:53-151), returning the
    L, R, O columns of evaluateLROSmallDomain (system.go:221-264)."""

    def __init__(self, nb_public: int, nb_secret: int, n_wires: int, wires, qidx, coeffs: Sequence[int],
                 flags=None, levels=None, curve: str = "bls12-381"):
        from ._lib import GG_CURVE_BN254, GG_CURVE_BLS12_381
        self.curve = curve
        self.mod = fr.BLS_R if curve == "bls12-381" else fr.R
        self._mont = fr.bls_fr_mont if curve == "bls12-381" else fr.fr_mont
        cid = GG_CURVE_BLS12_381 if curve == "bls12-381" else GG_CURVE_BN254
        self.nb_public, self.nb_secret, self.n_wires = nb_public, nb_secret, n_wires
        self.wires = np.ascontiguousarray(wires, dtype=np.uint32)
        self.qidx = np.ascontiguousarray(qidx, dtype=np.uint32)
        self.n_constraints = len(self.wires) // 3
        self.flags = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        if levels is None:
            levels = compute_scs_levels(nb_public + nb_secret, n_wires, self.wires)
        self.levels = levels
        lo = np.zeros(len(levels) + 1, dtype=np.uint32)
        lo[1:] = np.cumsum([len(x) for x in levels])
        lc = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.uint32) for x in levels])
                                  if levels else np.zeros(0, dtype=np.uint32), dtype=np.uint32)
        cbytes = b"".join(self._mont(int(k) % self.mod) for k in coeffs)
        h = ctypes.c_void_p()
        check(lib.gg_scs_create(cid, n_wires, self.n_constraints, nb_public, ptr(self.wires), ptr(self.qidx),
                                ptr(self.flags), ptr(cbytes), len(coeffs), ptr(lo), ptr(lc), len(levels),
                                ctypes.byref(h)))
        self.handle = h
        check(lib.gg_scs_set_inputs(h, nb_public, nb_secret))
        d = ctypes.c_size_t()
        check(lib.gg_scs_info(h, None, None, ctypes.byref(d)))
        self.domain = d.value

    @classmethod
    def from_constraints(cls, nb_public: int, nb_secret: int, n_wires: int, constraints, flags=None,
                         levels=None, curve: str = "bls12-381") -> "SparseR1CS":
        """constraints: [(xa, xb, xc, qL, qR, qO, qM, qC)] with int coefficients."""
        mod = fr.BLS_R if curve == "bls12-381" else fr.R
        table, index = [0, 1], {0: 0, 1: 1}
        wires, qidx = [], []
        for xa, xb, xc, *qs in constraints:
            wires += [xa, xb, xc]
            for k in qs:
                k %= mod
                if k not in index:
                    index[k] = len(table)
                    table.append(k)
                qidx.append(index[k])
        return cls(nb_public, nb_secret, n_wires, wires, qidx, table, flags, levels, curve)

    def solve(self, witness, on_device: bool = True):
        """spr.Solve(fullWitness) -> (W, L, R, O): host bytes or DeviceBuffers."""
        n_in = self.nb_public + self.nb_secret
        if len(witness) != n_in:
            raise ValueError("invalid witness size, got %d, expected %d" % (len(witness), n_in))
        wbuf = b"".join(self._mont(int(v) % self.mod) for v in witness)
        nw, d = self.n_wires, self.domain
        if on_device:
            out = [DeviceBuffer(32 * nw), DeviceBuffer(32 * d), DeviceBuffer(32 * d), DeviceBuffer(32 * d)]
        else:
            out = [bytearray(32 * nw), bytearray(32 * d), bytearray(32 * d), bytearray(32 * d)]
        bad = ctypes.c_int64(-1)
        rc = lib.gg_scs_solve(self.handle, ptr(wbuf), n_in, 0, *(ptr(x) for x in out), int(on_device),
                              ctypes.byref(bad))
        if rc == GG_ERR_UNSATISFIED:
            raise UnsatisfiedConstraintError(bad.value, lib.gg_last_error().decode())
        check(rc)
        return out

    def schedule(self):
        """(strands, launches, segments) of the last solve (gg_scs_schedule)."""
        return _schedule(lib.gg_scs_schedule, self.handle)

    def close(self):
        if getattr(self, "handle", None):
            lib.gg_scs_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
