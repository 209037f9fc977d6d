// Package amd_bn254 is the gnark-side shim of the MI355X backend: a drop-in
// twin of backend/groth16/bn254/icicle (provingkey.go:30-48, icicle.go,
// noicicle.go) that calls libgnark_amd.so through cgo (include/gnark_amd.h).
// Source only in this repository (no Go toolchain in the build image); see
// INTEGRATION.md for how it is wired into gnark.
package amd_bn254

import (
	"os"
	"strconv"
	"strings"
	"sync"
	"unsafe"

	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	cs "github.com/consensys/gnark/constraint/bn254"
)

// deviceInfo holds the HBM-resident proving key: one gg_groth16_pk_t, or, when
// several devices are configured, one gg_groth16_mpk_t (a shard per GPU, the
// distributed computeH's exchanges done inside the library).
type deviceInfo struct {
	handle  unsafe.Pointer
	multi   bool
	devices []int // the key's GPUs (shard order; one entry for a single-GPU key)

	// GPU r1cs.Solve, one solver per distinct device of the key (empty: the
	// system has hints).  Built once; a GPU-solved proof holds mu from the solve
	// to the end of the prove, because the prove reads the solvers' resident
	// W, A, B, C, which the next solve overwrites.
	solverOnce sync.Once
	solverErr  error
	solvers    map[int]*deviceSolver
	mu         sync.Mutex
}

var (
	devicesMu  sync.Mutex
	devices    []int
	configured bool
)

// SetDevices selects the GPUs keys created afterwards are sharded over
// (the SURVEY 8(b) gg_init(ngpu) shape).  nil / empty: the default GPU; one id:
// that GPU.  An explicit call wins over GNARK_AMD_DEVICES ("0,1,2,3,4,5,6,7"),
// which is read only when SetDevices was never called.
func SetDevices(ids []int) {
	devicesMu.Lock()
	defer devicesMu.Unlock()
	devices = append([]int{}, ids...)
	configured = true
}

func configuredDevices() []int {
	devicesMu.Lock()
	defer devicesMu.Unlock()
	if !configured {
		for _, f := range strings.Split(os.Getenv("GNARK_AMD_DEVICES"), ",") {
			if id, err := strconv.Atoi(strings.TrimSpace(f)); err == nil {
				devices = append(devices, id)
			}
		}
		configured = true
	}
	return append([]int{}, devices...)
}

// ProvingKey embeds the CPU key so WriteTo/ReadFrom/... are promoted unchanged
// (same layout trick as icicle_bn254.ProvingKey, provingkey.go:45-48).
type ProvingKey struct {
	groth16_bn254.ProvingKey
	*deviceInfo
}

func Setup(r1cs *cs.R1CS, pk *ProvingKey, vk *groth16_bn254.VerifyingKey) error {
	return groth16_bn254.Setup(r1cs, &pk.ProvingKey, vk)
}

func DummySetup(r1cs *cs.R1CS, pk *ProvingKey) error {
	return groth16_bn254.DummySetup(r1cs, &pk.ProvingKey)
}
