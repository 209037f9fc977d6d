//go:build !amd

package plonk

import (
	"errors"

	"github.com/consensys/gnark/backend"
	"github.com/consensys/gnark/backend/witness"
	cs "github.com/consensys/gnark/constraint/bn254"
)

// HasAMD mirrors icicle's HasIcicle (noicicle.go).
const HasAMD = false

func proveAMD(spr *cs.SparseR1CS, pk *ProvingKey, fullWitness witness.Witness, opt *backend.ProverConfig) (*Proof, error) {
	return nil, errors.New("gnark built without the amd tag")
}

func (pk *ProvingKey) ReleaseAMD() {}

// SetAMDDevices is a no-op without the amd build tag.
func SetAMDDevices(ids []int) {}
