//go:build !amd

package amd_bls12381

import (
	"fmt"

	"github.com/consensys/gnark/backend"
	groth16_bls12381 "github.com/consensys/gnark/backend/groth16/bls12-381"
	"github.com/consensys/gnark/backend/witness"
	cs "github.com/consensys/gnark/constraint/bls12-381"
)

// HasAMD mirrors icicle_bls12381.HasIcicle (noicicle.go:16).
const HasAMD = false

func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bls12381.Proof, error) {
	return nil, fmt.Errorf("amd backend requested but program compiled without 'amd' build tag")
}

// Release frees the HBM-resident key (no-op without the build tag).
func (pk *ProvingKey) Release() {}

// deviceSolver exists only with the build tag (solver_amd.go); deviceInfo names it.
type deviceSolver struct{}
