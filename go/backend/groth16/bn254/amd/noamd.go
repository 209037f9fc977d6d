//go:build !amd

package amd_bn254

import (
	"fmt"

	"github.com/consensys/gnark/backend"
	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	"github.com/consensys/gnark/backend/witness"
	cs "github.com/consensys/gnark/constraint/bn254"
)

// HasAMD mirrors icicle_bn254.HasIcicle (noicicle.go:16).
const HasAMD = false

func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bn254.Proof, error) {
	return nil, fmt.Errorf("amd backend requested but program compiled without 'amd' build tag")
}

// Release frees the HBM-resident key (no-op without the build tag).
func (pk *ProvingKey) Release() {}

// deviceSolver exists only with the build tag (solver_amd.go); deviceInfo names it.
type deviceSolver struct{}
