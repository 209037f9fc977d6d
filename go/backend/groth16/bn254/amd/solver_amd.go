//go:build amd

package amd_bn254

/*
#include <stdlib.h>
#include "gnark_amd.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	"github.com/consensys/gnark/backend/witness"
	"github.com/consensys/gnark/constraint"
	cs "github.com/consensys/gnark/constraint/bn254"
)

// deviceSolver is r1cs.Solve on the GPU (constraint/bn254/solver.go:418-608)
// for systems without hint calls: the R1Cs, the coefficient table and the
// levels are uploaded once (gg_r1cs_create), and a solve leaves W, A, B, C in
// HBM for gg_groth16_prove (inputs_on_device = 1) -- only the witness crosses
// PCIe.  Built lazily next to setupDevicePointers; nil for systems with hints
// (hints are Go functions: those keep gnark's solver).  A multi-GPU key has one
// solver per device, each leaving the whole solution on its GPU
// (gg_groth16_mpk_prove_ex reads shard r's copy on devices[r]).
type deviceSolver struct {
	h        C.gg_r1cs_t
	nbWires  int
	nbCons   int
	nbInputs int // witness length: nbPublic - 1 + nbSecret (solver.go:71-76)
}

// newDeviceSolvers builds the CSR form of a hint-free system once and uploads
// it to every distinct device of devs (nil map: the system has hints).
func newDeviceSolvers(sys *cs.R1CS, devs []int) (map[int]*deviceSolver, error) {
	for _, inst := range sys.Instructions {
		if _, ok := sys.Blueprints[inst.BlueprintID].(constraint.BlueprintHint); ok {
			return nil, nil
		}
	}
	rs := sys.GetR1Cs() // one R1C per instruction: instruction ids == constraint ids
	off := make([]uint32, 1, 3*len(rs)+1)
	var wires, coeffs []uint32
	for _, c := range rs {
		for _, le := range []constraint.LinearExpression{c.L, c.R, c.O} {
			for _, t := range le {
				w := uint32(t.WireID())
				if t.IsConstant() { // coeff * ONE_WIRE (term.go:35-41)
					w = 0
				}
				wires = append(wires, w)
				coeffs = append(coeffs, uint32(t.CoeffID()))
			}
			off = append(off, uint32(len(wires)))
		}
	}
	levelOff := make([]uint32, 1, len(sys.Levels)+1)
	levelCons := make([]uint32, 0, len(rs))
	for _, l := range sys.Levels {
		for _, iID := range l {
			levelCons = append(levelCons, uint32(iID))
		}
		levelOff = append(levelOff, uint32(len(levelCons)))
	}
	nbPublic, nbSecret := sys.GetNbPublicVariables(), sys.GetNbSecretVariables()
	nbWires := nbPublic + nbSecret + sys.NbInternalVariables
	if len(wires) == 0 || len(levelCons) == 0 || len(sys.Coefficients) == 0 {
		return nil, nil
	}
	out := map[int]*deviceSolver{}
	for _, dev := range devs {
		if _, ok := out[dev]; ok {
			continue
		}
		var h C.gg_r1cs_t
		err := onDevice(dev, func() error {
			if C.gg_r1cs_create(C.size_t(nbWires), C.size_t(len(rs)),
				(*C.uint32_t)(unsafe.Pointer(&off[0])), (*C.uint32_t)(unsafe.Pointer(&wires[0])),
				(*C.uint32_t)(unsafe.Pointer(&coeffs[0])), unsafe.Pointer(&sys.Coefficients[0]),
				C.size_t(len(sys.Coefficients)), (*C.uint32_t)(unsafe.Pointer(&levelOff[0])),
				(*C.uint32_t)(unsafe.Pointer(&levelCons[0])), C.size_t(len(sys.Levels)), &h) != C.GG_OK {
				return lastError()
			}
			// the library rejects a witness of another size too (a second line of defence)
			if C.gg_r1cs_set_inputs(h, C.size_t(nbPublic), C.size_t(nbSecret)) != C.GG_OK {
				C.gg_r1cs_release(h)
				return lastError()
			}
			return nil
		})
		if err != nil {
			for _, ds := range out {
				ds.release()
			}
			return nil, err
		}
		out[dev] = &deviceSolver{h: h, nbWires: nbWires, nbCons: len(rs), nbInputs: nbPublic - 1 + nbSecret}
	}
	return out, nil
}

// solve runs the levels on the GPU and returns the device pointers of W, A, B, C
// (valid until the next solve on this solver).
func (d *deviceSolver) solve(fullWitness witness.Witness) (w, a, b, c unsafe.Pointer, err error) {
	vec, ok := fullWitness.Vector().(fr.Vector)
	if !ok {
		return nil, nil, nil, nil, fmt.Errorf("gnark_amd: witness is not a bn254 fr.Vector")
	}
	if len(vec) != d.nbInputs { // newSolver (solver.go:71-76)
		return nil, nil, nil, nil, fmt.Errorf("invalid witness size, got %d, expected %d", len(vec), d.nbInputs)
	}
	var in unsafe.Pointer
	if len(vec) > 0 {
		in = unsafe.Pointer(&vec[0])
	}
	var bad C.int64_t
	if rc := C.gg_r1cs_solve(d.h, in, C.size_t(len(vec)), 0, nil, nil, nil, nil, 1, &bad); rc != C.GG_OK {
		if rc == C.GG_ERR_UNSATISFIED {
			return nil, nil, nil, nil, fmt.Errorf("constraint #%d is not satisfied: %w", int64(bad), lastError())
		}
		return nil, nil, nil, nil, lastError()
	}
	if C.gg_r1cs_solution_dev(d.h, &w, &a, &b, &c) != C.GG_OK {
		return nil, nil, nil, nil, lastError()
	}
	return w, a, b, c, nil
}

func (d *deviceSolver) release() {
	if d != nil && d.h != nil {
		C.gg_r1cs_release(d.h)
		d.h = nil
	}
}
