//go:build amd

package plonk

/*
#include <stdlib.h>
#include "gnark_amd.h"
*/
import "C"

import (
	"fmt"
	"sync"
	"unsafe"

	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	"github.com/consensys/gnark/backend/witness"
	"github.com/consensys/gnark/constraint"
	cs "github.com/consensys/gnark/constraint/bn254"
)

// scsSolver is spr.Solve on the GPU for sparse-R1CS without hint calls
// (blueprint_scs.go:53-151 per level + evaluateLROSmallDomain, system.go:221-264):
// the constraints (DecompressSparseR1C of every instruction), spr.Coefficients
// and spr.Levels uploaded once (gg_scs_create); a solve leaves L, R, O in HBM
// for gg_plonk_prove (inputs on device).  nil for systems with hints.
type scsSolver struct {
	h C.gg_scs_t
}

var amdSolvers sync.Map // *ProvingKey -> *scsSolver (nil: the system has hints)

func newScsSolver(spr *cs.SparseR1CS) (*scsSolver, error) {
	n := len(spr.Instructions)
	wires := make([]uint32, 0, 3*n)
	qidx := make([]uint32, 0, 5*n)
	flags := make([]uint8, 0, n)
	var c constraint.SparseR1C
	for _, inst := range spr.Instructions {
		bc, ok := spr.Blueprints[inst.BlueprintID].(constraint.BlueprintSparseR1C)
		if !ok {
			return nil, nil // a hint (or another non-constraint instruction): keep gnark's solver
		}
		bc.DecompressSparseR1C(&c, inst.Unpack(&spr.System))
		wires = append(wires, c.XA, c.XB, c.XC)
		qidx = append(qidx, c.QL, c.QR, c.QO, c.QM, c.QC)
		var f uint8
		if c.Commitment != constraint.NOT {
			f = 1
		}
		flags = append(flags, f)
	}
	levelOff := make([]uint32, 1, len(spr.Levels)+1)
	levelCons := make([]uint32, 0, n)
	for _, l := range spr.Levels { // instruction ids == constraint ids without hints
		for _, iID := range l {
			levelCons = append(levelCons, uint32(iID))
		}
		levelOff = append(levelOff, uint32(len(levelCons)))
	}
	if n == 0 || len(spr.Coefficients) == 0 {
		return nil, nil
	}
	nbWires := spr.GetNbPublicVariables() + spr.GetNbSecretVariables() + spr.NbInternalVariables
	var h C.gg_scs_t
	if C.gg_scs_create(C.GG_CURVE_BN254, C.size_t(nbWires), C.size_t(n), C.size_t(len(spr.Public)),
		(*C.uint32_t)(unsafe.Pointer(&wires[0])), (*C.uint32_t)(unsafe.Pointer(&qidx[0])),
		(*C.uint8_t)(unsafe.Pointer(&flags[0])), unsafe.Pointer(&spr.Coefficients[0]),
		C.size_t(len(spr.Coefficients)), (*C.uint32_t)(unsafe.Pointer(&levelOff[0])),
		(*C.uint32_t)(unsafe.Pointer(&levelCons[0])), C.size_t(len(spr.Levels)), &h) != C.GG_OK {
		return nil, amdError()
	}
	// the library rejects a witness of another size too (solver.go:71-76)
	if C.gg_scs_set_inputs(h, C.size_t(spr.GetNbPublicVariables()), C.size_t(spr.GetNbSecretVariables())) != C.GG_OK {
		C.gg_scs_release(h)
		return nil, amdError()
	}
	return &scsSolver{h: h}, nil
}

func (pk *ProvingKey) amdSolver(spr *cs.SparseR1CS, h C.gg_plonk_pk_t) (*scsSolver, error) {
	if s, ok := amdSolvers.Load(pk); ok {
		return s.(*scsSolver), nil
	}
	var s *scsSolver
	// on the GPU that runs the key's prover (gg_plonk_prove reads L, R, O
	// there): the device the key was created on, not the current
	// SetAMDDevices / GNARK_AMD_DEVICES choice, which may have changed since
	dev, err := keyPrimaryDevice(h)
	if err != nil {
		return nil, err
	}
	err = onAMDDevice(dev, func() error {
		var err error
		s, err = newScsSolver(spr)
		return err
	})
	if err != nil {
		return nil, err
	}
	if old, loaded := amdSolvers.LoadOrStore(pk, s); loaded { // a concurrent first call won
		if s != nil {
			C.gg_scs_release(s.h)
		}
		return old.(*scsSolver), nil
	}
	return s, nil
}

// solve returns the device pointers of L, R, O (valid until the next solve).
func (s *scsSolver) solve(fullWitness witness.Witness) (l, r, o unsafe.Pointer, err error) {
	vec, ok := fullWitness.Vector().(fr.Vector)
	if !ok || len(vec) == 0 {
		return nil, nil, nil, witness.ErrInvalidWitness
	}
	var bad C.int64_t
	if rc := C.gg_scs_solve(s.h, unsafe.Pointer(&vec[0]), C.size_t(len(vec)), 0, nil, nil, nil, nil, 1, &bad); rc != C.GG_OK {
		if rc == C.GG_ERR_UNSATISFIED {
			return nil, nil, nil, fmt.Errorf("constraint #%d is not satisfied: %w", int64(bad), amdError())
		}
		return nil, nil, nil, amdError()
	}
	if C.gg_scs_solution_dev(s.h, nil, &l, &r, &o) != C.GG_OK {
		return nil, nil, nil, amdError()
	}
	return l, r, o, nil
}

func (pk *ProvingKey) releaseSolver() {
	if s, ok := amdSolvers.LoadAndDelete(pk); ok && s.(*scsSolver) != nil {
		C.gg_scs_release(s.(*scsSolver).h)
	}
}
