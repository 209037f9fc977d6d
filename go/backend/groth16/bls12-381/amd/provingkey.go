// Package amd_bls12381 is the gnark-side shim of the MI355X backend for
// backend/groth16/bls12-381 (gg_groth16_pk_create_ex with GG_CURVE_BLS12_381): a drop-in
// twin of backend/groth16/bn254/icicle (provingkey.go:30-48, icicle.go,
// noicicle.go) that calls libgnark_amd.so through cgo (include/gnark_amd.h).
// Source only in this repository (no Go toolchain in the build image); see
// INTEGRATION.md for how it is wired into gnark.
package amd_bls12381

import (
	"unsafe"

	groth16_bls12381 "github.com/consensys/gnark/backend/groth16/bls12-381"
	cs "github.com/consensys/gnark/constraint/bls12-381"
)

// deviceInfo holds the HBM-resident proving key (gg_groth16_pk_t).
type deviceInfo struct {
	handle      unsafe.Pointer
	solver      *deviceSolver // GPU r1cs.Solve (nil: the system has hints)
	solverTried bool
}

// ProvingKey embeds the CPU key so WriteTo/ReadFrom/... are promoted unchanged
// (same layout trick as icicle_bls12381.ProvingKey, provingkey.go:45-48).
type ProvingKey struct {
	groth16_bls12381.ProvingKey
	*deviceInfo
}

func Setup(r1cs *cs.R1CS, pk *ProvingKey, vk *groth16_bls12381.VerifyingKey) error {
	return groth16_bls12381.Setup(r1cs, &pk.ProvingKey, vk)
}

func DummySetup(r1cs *cs.R1CS, pk *ProvingKey) error {
	return groth16_bls12381.DummySetup(r1cs, &pk.ProvingKey)
}
