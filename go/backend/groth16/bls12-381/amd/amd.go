//go:build amd

package amd_bls12381

/*
#cgo CFLAGS: -I${SRCDIR}/../../../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../../../gnark-fork_amd/lib -lgnark_amd -Wl,-rpath,${SRCDIR}/../../../../../gnark-fork_amd/lib
#include <stdlib.h>
#include "gnark_amd.h"
*/
import "C"

import (
	"fmt"
	"math/big"
	"time"
	"unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bls12-381"
	"github.com/consensys/gnark-crypto/ecc/bls12-381/fr"
	"github.com/consensys/gnark-crypto/ecc/bls12-381/fr/hash_to_field"
	"github.com/consensys/gnark-crypto/ecc/bls12-381/fr/pedersen"
	"github.com/consensys/gnark/backend"
	groth16_bls12381 "github.com/consensys/gnark/backend/groth16/bls12-381"
	"github.com/consensys/gnark/backend/groth16/internal"
	"github.com/consensys/gnark/backend/witness"
	"github.com/consensys/gnark/constraint"
	cs "github.com/consensys/gnark/constraint/bls12-381"
	"github.com/consensys/gnark/constraint/solver"
	"github.com/consensys/gnark/logger"
	fcs "github.com/consensys/gnark/frontend/cs"
)

// HasAMD mirrors icicle_bls12381.HasIcicle (icicle.go:29).
const HasAMD = true

func lastError() error { return fmt.Errorf("gnark_amd: %s", C.GoString(C.gg_last_error())) }

func ptrOr(b bool, p unsafe.Pointer) unsafe.Pointer {
	if b {
		return p
	}
	return nil
}

// setupDevicePointers uploads pk once (replaces icicle.go:31-130).
func (pk *ProvingKey) setupDevicePointers(nbPublic int, kWireIndex []uint32) error {
	if pk.deviceInfo != nil {
		return nil
	}
	n := pk.Domain.Cardinality
	logN := 0
	for (uint64(1) << logN) < n {
		logN++
	}
	nWires := len(pk.InfinityA)
	infA := make([]byte, nWires)
	infB := make([]byte, nWires)
	for i := range pk.InfinityA {
		if pk.InfinityA[i] {
			infA[i] = 1
		}
		if pk.InfinityB[i] {
			infB[i] = 1
		}
	}
	var h C.gg_groth16_pk_t
	p := func(s unsafe.Pointer, n int) unsafe.Pointer { return ptrOr(n > 0, s) }
	rc := C.gg_groth16_pk_create_ex(C.GG_CURVE_BLS12_381, C.int(logN),
		unsafe.Pointer(&pk.Domain.Generator), unsafe.Pointer(&pk.Domain.FrMultiplicativeGen),
		p(unsafe.Pointer(unsafe.SliceData(pk.G1.A)), len(pk.G1.A)), C.size_t(len(pk.G1.A)),
		p(unsafe.Pointer(unsafe.SliceData(pk.G1.B)), len(pk.G1.B)), C.size_t(len(pk.G1.B)),
		p(unsafe.Pointer(unsafe.SliceData(pk.G1.Z)), len(pk.G1.Z)), C.size_t(len(pk.G1.Z)),
		p(unsafe.Pointer(unsafe.SliceData(pk.G1.K)), len(pk.G1.K)), C.size_t(len(pk.G1.K)),
		unsafe.Pointer(&pk.G1.Alpha), unsafe.Pointer(&pk.G1.Beta), unsafe.Pointer(&pk.G1.Delta),
		p(unsafe.Pointer(unsafe.SliceData(pk.G2.B)), len(pk.G2.B)),
		unsafe.Pointer(&pk.G2.Beta), unsafe.Pointer(&pk.G2.Delta),
		(*C.uint8_t)(unsafe.Pointer(&infA[0])), (*C.uint8_t)(unsafe.Pointer(&infB[0])),
		C.size_t(nWires), C.size_t(nbPublic),
		(*C.uint32_t)(p(unsafe.Pointer(unsafe.SliceData(kWireIndex)), len(kWireIndex))), &h)
	if rc != C.GG_OK {
		return lastError()
	}
	pk.deviceInfo = &deviceInfo{handle: unsafe.Pointer(h)}
	return nil
}

// Release frees the HBM-resident key (the icicle path never frees it).
func (pk *ProvingKey) Release() {
	if pk.deviceInfo != nil {
		pk.deviceInfo.solver.release()
		C.gg_groth16_pk_release(C.gg_groth16_pk_t(pk.deviceInfo.handle))
		pk.deviceInfo = nil
	}
}

// Prove mirrors icicle_bls12381.Prove (icicle.go:133-422): identical solver,
// commitment and randomness handling; the MSM/NTT section runs in one
// gg_groth16_prove call.
func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bls12381.Proof, error) {
	opt, err := backend.NewProverConfig(opts...)
	if err != nil {
		return nil, fmt.Errorf("new prover config: %w", err)
	}
	if opt.HashToFieldFn == nil {
		opt.HashToFieldFn = hash_to_field.New([]byte(constraint.CommitmentDst))
	}
	if opt.Accelerator != "amd" && opt.Accelerator != "icicle" {
		return groth16_bls12381.Prove(r1cs, &pk.ProvingKey, fullWitness, opts...)
	}
	log := logger.Logger().With().Str("curve", r1cs.CurveID().String()).Str("acceleration", "amd").Int("nbConstraints", r1cs.GetNbConstraints()).Str("backend", "groth16").Logger()

	commitmentInfo := r1cs.CommitmentInfo.(constraint.Groth16Commitments)
	nbPublic := r1cs.GetNbPublicVariables()
	if pk.deviceInfo == nil {
		// wire index of each pk.G1.K scalar = filterHeap(wires[nbPublic:]) (prove.go:238-248)
		toRemove := commitmentInfo.GetPrivateCommitted()
		toRemove = append(toRemove, commitmentInfo.CommitmentIndexes())
		removed := map[int]bool{}
		for _, i := range internal.ConcatAll(toRemove...) {
			removed[i] = true
		}
		nWires := len(pk.InfinityA)
		kIdx := make([]uint32, 0, len(pk.G1.K))
		for i := nbPublic; i < nWires; i++ {
			if !removed[i] {
				kIdx = append(kIdx, uint32(i))
			}
		}
		if err := pk.setupDevicePointers(nbPublic, kIdx); err != nil {
			return nil, fmt.Errorf("setup device pointers: %w", err)
		}
	}

	proof := &groth16_bls12381.Proof{Commitments: make([]curve.G1Affine, len(commitmentInfo))}
	solverOpts := opt.SolverOpts[:len(opt.SolverOpts):len(opt.SolverOpts)]
	privateCommittedValues := make([][]fr.Element, len(commitmentInfo))
	bsb22ID := solver.GetHintID(fcs.Bsb22CommitmentComputePlaceholder)
	solverOpts = append(solverOpts, solver.OverrideHint(bsb22ID, func(_ *big.Int, in []*big.Int, out []*big.Int) error {
		i := int(in[0].Int64())
		in = in[1:]
		privateCommittedValues[i] = make([]fr.Element, len(commitmentInfo[i].PrivateCommitted))
		hashed := in[:len(commitmentInfo[i].PublicAndCommitmentCommitted)]
		committed := in[len(hashed):]
		for j, inJ := range committed {
			privateCommittedValues[i][j].SetBigInt(inJ)
		}
		var err error
		if proof.Commitments[i], err = pk.CommitmentKeys[i].Commit(privateCommittedValues[i]); err != nil {
			return err
		}
		opt.HashToFieldFn.Write(constraint.SerializeCommitment(proof.Commitments[i].Marshal(), hashed, (fr.Bits-1)/8+1))
		hashBts := opt.HashToFieldFn.Sum(nil)
		opt.HashToFieldFn.Reset()
		nbBuf := fr.Bytes
		if opt.HashToFieldFn.Size() < fr.Bytes {
			nbBuf = opt.HashToFieldFn.Size()
		}
		var res fr.Element
		res.SetBytes(hashBts[:nbBuf])
		res.BigInt(out[0])
		return nil
	}))

	// GKR hints get the same override as on the CPU path (prove.go:112-117)
	if r1cs.GkrInfo.Is() {
		var gkrData cs.GkrSolvingData
		solverOpts = append(solverOpts,
			solver.OverrideHint(r1cs.GkrInfo.SolveHintID, cs.GkrSolveHint(r1cs.GkrInfo, &gkrData)),
			solver.OverrideHint(r1cs.GkrInfo.ProveHintID, cs.GkrProveHint(r1cs.GkrInfo.HashName, &gkrData)))
	}

	// hint-free systems without commitments: r1cs.Solve on the GPU over
	// BLS12-381 fr (gg_r1cs_create_ex), the solution stays in HBM (solver_amd.go)
	if len(commitmentInfo) == 0 && len(opt.SolverOpts) == 0 && !r1cs.GkrInfo.Is() {
		if !pk.deviceInfo.solverTried {
			pk.deviceInfo.solverTried = true
			if pk.deviceInfo.solver, err = newDeviceSolver(r1cs); err != nil {
				return nil, fmt.Errorf("device solver: %w", err)
			}
		}
		if ds := pk.deviceInfo.solver; ds != nil {
			w, a, b, c, err := ds.solve(fullWitness)
			if err != nil {
				return nil, err
			}
			var r, s fr.Element
			if _, err := r.SetRandom(); err != nil {
				return nil, err
			}
			if _, err := s.SetRandom(); err != nil {
				return nil, err
			}
			var ar, krs curve.G1Affine
			var bs curve.G2Affine
			if C.gg_groth16_prove(C.gg_groth16_pk_t(pk.deviceInfo.handle), w, C.size_t(ds.nbWires), a, b, c,
				C.size_t(ds.nbCons), 1, unsafe.Pointer(&r), unsafe.Pointer(&s),
				unsafe.Pointer(&ar), unsafe.Pointer(&bs), unsafe.Pointer(&krs), nil) != C.GG_OK {
				return nil, lastError()
			}
			proof.Ar, proof.Bs, proof.Krs = ar, bs, krs
			return proof, nil
		}
	}

	_solution, err := r1cs.Solve(fullWitness, solverOpts...)
	if err != nil {
		return nil, err
	}
	solution := _solution.(*cs.R1CSSolution)
	wireValues := []fr.Element(solution.W)
	start := time.Now()

	commitmentsSerialized := make([]byte, fr.Bytes*len(commitmentInfo))
	for i := range commitmentInfo {
		copy(commitmentsSerialized[fr.Bytes*i:], wireValues[commitmentInfo[i].CommitmentIndex].Marshal())
	}
	if proof.CommitmentPok, err = pedersen.BatchProve(pk.CommitmentKeys, privateCommittedValues, commitmentsSerialized); err != nil {
		return nil, err
	}

	var r, s fr.Element
	if _, err := r.SetRandom(); err != nil {
		return nil, err
	}
	if _, err := s.SetRandom(); err != nil {
		return nil, err
	}
	var ar, krs curve.G1Affine
	var bs curve.G2Affine
	rc := C.gg_groth16_prove(C.gg_groth16_pk_t(pk.deviceInfo.handle),
		unsafe.Pointer(&wireValues[0]), C.size_t(len(wireValues)),
		unsafe.Pointer(&solution.A[0]), unsafe.Pointer(&solution.B[0]), unsafe.Pointer(&solution.C[0]),
		C.size_t(len(solution.A)), 0,
		unsafe.Pointer(&r), unsafe.Pointer(&s),
		unsafe.Pointer(&ar), unsafe.Pointer(&bs), unsafe.Pointer(&krs), nil)
	if rc != C.GG_OK {
		return nil, lastError()
	}
	proof.Ar, proof.Bs, proof.Krs = ar, bs, krs
	log.Debug().Dur("took", time.Since(start)).Msg("prover done")
	return proof, nil
}
