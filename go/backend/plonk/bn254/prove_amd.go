//go:build amd

// MI355X path of plonk.Prove for BN254: a file of package plonk
// (backend/plonk/bn254) so it reads pk.trace / pk.Kzg / pk.KzgLagrange
// directly.  Prove (prove.go:116) dispatches here when the prover option
// WithAMDAcceleration() / WithIcicleAcceleration() is set (INTEGRATION.md §4).
// Hint-free systems without commitments solve on the GPU (solver_amd.go);
// otherwise the solver stays gnark's (prove.go:365-395) with the BSB22 hint
// committing on the GPU; everything after Solve -- prove.go:116-176's errgroup DAG -- is one
// gg_plonk_prove call.  Source only here (no Go toolchain in the build image).
package plonk

/*
#cgo CFLAGS: -I${SRCDIR}/../../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../../gnark-fork_amd/lib -lgnark_amd -Wl,-rpath,${SRCDIR}/../../../../gnark-fork_amd/lib
#include <stdlib.h>
#include "gnark_amd.h"
extern int ggGoHash(void *ctx, void *data, size_t len, void *out, size_t *out_len);
static int gg_go_hash(void *ctx, const void *data, size_t len, void *out, size_t *out_len) {
	return ggGoHash(ctx, (void *)data, len, out, out_len);
}
static gg_hash_fn gg_go_hash_fn(void) { return gg_go_hash; }
*/
import "C"

import (
	"errors"
	"fmt"
	"hash"
	"math/big"
	"os"
	"runtime"
	"runtime/cgo"
	"strconv"
	"strings"
	"sync"
	"unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bn254"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr/hash_to_field"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr/iop"
	"github.com/consensys/gnark/backend"
	"github.com/consensys/gnark/backend/witness"
	"github.com/consensys/gnark/constraint"
	cs "github.com/consensys/gnark/constraint/bn254"
	"github.com/consensys/gnark/constraint/solver"
	fcs "github.com/consensys/gnark/frontend/cs"
)

// HasAMD mirrors icicle's HasIcicle.
const HasAMD = true

// the C ABI's id of this package's curve
const amdCurve = C.GG_CURVE_BN254

func amdError() error { return fmt.Errorf("gnark_amd: %s", C.GoString(C.gg_last_error())) }

// device keys, one per *ProvingKey (HBM-resident; released by ReleaseAMD)
var amdKeys sync.Map

// per-key lock of the GPU-solved path: the prove reads the solver's resident
// L, R, O, which the next solve on the same key overwrites
var amdLocks sync.Map // *ProvingKey -> *sync.Mutex

func (pk *ProvingKey) amdLock() *sync.Mutex {
	m, _ := amdLocks.LoadOrStore(pk, &sync.Mutex{})
	return m.(*sync.Mutex)
}

var (
	amdDevicesMu  sync.Mutex
	amdDevices    []int
	amdConfigured bool
)

// SetAMDDevices selects the GPUs PlonK keys created afterwards are split over
// (gg_plonk_pk_create_ex with devices: KZG base slices and numerator cosets per device,
// all driven from this process; configs[4] "8xMI355X").  nil / empty: the
// default GPU; one id: that GPU.  An explicit call wins over GNARK_AMD_DEVICES.
func SetAMDDevices(ids []int) {
	amdDevicesMu.Lock()
	defer amdDevicesMu.Unlock()
	amdDevices = append([]int{}, ids...)
	amdConfigured = true
}

func amdConfiguredDevices() []int {
	amdDevicesMu.Lock()
	defer amdDevicesMu.Unlock()
	if !amdConfigured {
		for _, f := range strings.Split(os.Getenv("GNARK_AMD_DEVICES"), ",") {
			if id, err := strconv.Atoi(strings.TrimSpace(f)); err == nil {
				amdDevices = append(amdDevices, id)
			}
		}
		amdConfigured = true
	}
	return append([]int{}, amdDevices...)
}

// onAMDDevice runs fn on an OS thread bound to GPU dev (gg_set_device binds the
// calling thread; the goroutine must not migrate between the bind and the calls).
func onAMDDevice(dev int, fn func() error) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	if C.gg_set_device(C.int(dev)) != C.GG_OK {
		return amdError()
	}
	return fn()
}

// amdPrimaryDevice is the GPU a device key created now would run its prover
// on (the first configured device).  An existing key's GPU is keyPrimaryDevice.
func amdPrimaryDevice() int {
	if devs := amdConfiguredDevices(); len(devs) > 0 {
		return devs[0]
	}
	return 0
}

// keyPrimaryDevice is the GPU that runs h's prover -- where gg_plonk_prove
// reads device-resident L, R, O -- as recorded when h was created (a later
// SetAMDDevices does not move it).
func keyPrimaryDevice(h C.gg_plonk_pk_t) (int, error) {
	var nd C.int
	if C.gg_plonk_pk_devices(h, nil, 0, &nd) != C.GG_OK || nd < 1 {
		return 0, amdError()
	}
	devs := make([]C.int, int(nd))
	if C.gg_plonk_pk_devices(h, &devs[0], nd, &nd) != C.GG_OK {
		return 0, amdError()
	}
	return int(devs[0]), nil
}

func (pk *ProvingKey) amdKey() (C.gg_plonk_pk_t, error) {
	if h, ok := amdKeys.Load(pk); ok {
		return h.(C.gg_plonk_pk_t), nil
	}
	n := pk.Domain[0].Cardinality
	logN, logBig := 0, 0
	for (uint64(1) << logN) < n {
		logN++
	}
	for (uint64(1) << logBig) < pk.Domain[1].Cardinality {
		logBig++
	}
	// The arrays of polynomial pointers live in C memory (ctr, cqcp below), and
	// cgo forbids storing Go pointers there unless the objects are pinned: pin
	// every coefficient slice for the duration of gg_plonk_pk_create_ex (the
	// library copies the polynomials to HBM before it returns).
	var pin runtime.Pinner
	defer pin.Unpin()
	tr := [8]unsafe.Pointer{}
	for i, p := range []*iop.Polynomial{pk.trace.Ql, pk.trace.Qr, pk.trace.Qm, pk.trace.Qo, pk.trace.Qk,
		pk.trace.S1, pk.trace.S2, pk.trace.S3} {
		c := &p.Coefficients()[0] // canonical regular after Setup (setup.go:229-240)
		pin.Pin(c)
		tr[i] = unsafe.Pointer(c)
	}
	qcp := make([]unsafe.Pointer, len(pk.trace.Qcp)+1)
	for i, p := range pk.trace.Qcp {
		c := &p.Coefficients()[0]
		pin.Pin(c)
		qcp[i] = unsafe.Pointer(c)
	}
	idx := append(pk.Vk.CommitmentConstraintIndexes, 0)
	vk := make([]curve.G1Affine, 0, 8+len(pk.Vk.Qcp))
	vk = append(vk, pk.Vk.S[0], pk.Vk.S[1], pk.Vk.S[2], pk.Vk.Ql, pk.Vk.Qr, pk.Vk.Qm, pk.Vk.Qo, pk.Vk.Qk)
	vk = append(vk, pk.Vk.Qcp...)
	// the C side copies everything it needs before returning (cgo pointer rules)
	ctr := C.malloc(C.size_t(8 * unsafe.Sizeof(uintptr(0))))
	defer C.free(ctr)
	copy(unsafe.Slice((*unsafe.Pointer)(ctr), 8), tr[:])
	cqcp := C.malloc(C.size_t(len(qcp)) * C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(cqcp)
	copy(unsafe.Slice((*unsafe.Pointer)(cqcp), len(qcp)), qcp)
	var h C.gg_plonk_pk_t
	// one GPU (the calling thread's, bound below) or the configured device parts
	devs := amdConfiguredDevices()
	cdevs := make([]C.int, len(devs)+1)
	for i, d := range devs {
		cdevs[i] = C.int(d)
	}
	if err := onAMDDevice(amdPrimaryDevice(), func() error {
		if C.gg_plonk_pk_create_ex(amdCurve, C.int(logN), C.int(logBig),
			unsafe.Pointer(&pk.Domain[0].Generator), unsafe.Pointer(&pk.Domain[1].Generator),
			unsafe.Pointer(&pk.Domain[0].FrMultiplicativeGen),
			unsafe.Pointer(&pk.Kzg.G1[0]), C.size_t(len(pk.Kzg.G1)), unsafe.Pointer(&pk.KzgLagrange.G1[0]),
			(*unsafe.Pointer)(ctr), (*unsafe.Pointer)(cqcp), C.int(len(pk.trace.Qcp)),
			(*C.int64_t)(unsafe.Pointer(&pk.trace.S[0])), C.size_t(pk.Vk.NbPublicVariables),
			(*C.uint64_t)(unsafe.Pointer(&idx[0])), unsafe.Pointer(&vk[0]), C.int(len(devs)), &cdevs[0],
			&h) != C.GG_OK {
			return amdError()
		}
		return nil
	}); err != nil {
		return nil, err
	}
	if old, loaded := amdKeys.LoadOrStore(pk, h); loaded {
		C.gg_plonk_pk_release(h)
		return old.(C.gg_plonk_pk_t), nil
	}
	return h, nil
}

// ReleaseAMD frees the HBM-resident copy of pk.
func (pk *ProvingKey) ReleaseAMD() {
	mu := pk.amdLock()
	mu.Lock()
	defer mu.Unlock()
	pk.releaseSolver()
	if h, ok := amdKeys.LoadAndDelete(pk); ok {
		C.gg_plonk_pk_release(h.(C.gg_plonk_pk_t))
	}
}

//export ggGoHash
func ggGoHash(ctx unsafe.Pointer, data unsafe.Pointer, n C.size_t, out unsafe.Pointer, outLen *C.size_t) C.int {
	h := cgo.Handle(ctx).Value().(hash.Hash)
	h.Reset()
	h.Write(C.GoBytes(data, C.int(n)))
	d := h.Sum(nil)
	h.Reset()
	if C.size_t(len(d)) > *outLen {
		return 1
	}
	copy(unsafe.Slice((*byte)(out), len(d)), d)
	*outLen = C.size_t(len(d))
	return 0
}

// proveAMD replaces prove.go:129-176 after NewProverConfig.
func proveAMD(spr *cs.SparseR1CS, pk *ProvingKey, fullWitness witness.Witness, opt *backend.ProverConfig) (*Proof, error) {
	h, err := pk.amdKey()
	if err != nil {
		return nil, err
	}
	if opt.HashToFieldFn == nil {
		opt.HashToFieldFn = hash_to_field.New([]byte("BSB22-Plonk"))
	}
	proof := &Proof{}
	commitmentInfo := spr.CommitmentInfo.(constraint.PlonkCommitments)
	nCmt := len(commitmentInfo)
	userHints := len(opt.SolverOpts) > 0
	commitmentVal := make([]fr.Element, nCmt)
	committed := make([][]fr.Element, nCmt)
	proof.Bsb22Commitments = make([]curve.G1Affine, nCmt)
	// bsb22Hint (prove.go:316-352) with the commitment on the GPU
	bsb22ID := solver.GetHintID(fcs.Bsb22CommitmentComputePlaceholder)
	opt.SolverOpts = append(opt.SolverOpts, solver.OverrideHint(bsb22ID, func(_ *big.Int, ins, outs []*big.Int) error {
		commDepth := int(ins[0].Int64())
		ins = ins[1:]
		info := commitmentInfo[commDepth]
		vals := make([]fr.Element, pk.Domain[0].Cardinality)
		offset := spr.GetNbPublicVariables()
		for i := range ins {
			vals[offset+info.Committed[i]].SetBigInt(ins[i])
		}
		if _, err := vals[offset+info.CommitmentIndex].SetRandom(); err != nil {
			return err
		}
		if _, err := vals[offset+spr.GetNbConstraints()-1].SetRandom(); err != nil {
			return err
		}
		if C.gg_plonk_commit_lagrange(h, unsafe.Pointer(&vals[0]), 0, unsafe.Pointer(&proof.Bsb22Commitments[commDepth])) != C.GG_OK {
			return amdError()
		}
		committed[commDepth] = vals
		opt.HashToFieldFn.Write(proof.Bsb22Commitments[commDepth].Marshal())
		hashBts := opt.HashToFieldFn.Sum(nil)
		opt.HashToFieldFn.Reset()
		nbBuf := fr.Bytes
		if opt.HashToFieldFn.Size() < fr.Bytes {
			nbBuf = opt.HashToFieldFn.Size()
		}
		commitmentVal[commDepth].SetBytes(hashBts[:nbBuf])
		commitmentVal[commDepth].BigInt(outs[0])
		return nil
	}))
	if spr.GkrInfo.Is() { // setupGKRHints (prove.go:354-361)
		var gkrData cs.GkrSolvingData
		opt.SolverOpts = append(opt.SolverOpts,
			solver.OverrideHint(spr.GkrInfo.SolveHintID, cs.GkrSolveHint(spr.GkrInfo, &gkrData)),
			solver.OverrideHint(spr.GkrInfo.ProveHintID, cs.GkrProveHint(spr.GkrInfo.HashName, &gkrData)))
	}
	w, ok := fullWitness.Vector().(fr.Vector)
	if !ok {
		return nil, witness.ErrInvalidWitness
	}
	// newSolver's check (constraint/bn254/solver.go:71-76): the public
	// inputs below are read from w[:len(spr.Public)]
	if exp := spr.GetNbPublicVariables() + spr.GetNbSecretVariables(); len(w) != exp {
		return nil, fmt.Errorf("invalid witness size, got %d, expected %d", len(w), exp)
	}
	// hint-free systems without commitments: spr.Solve on the GPU, L, R, O stay
	// in HBM (solver_amd.go); everything else keeps gnark's solver
	var lro [3]unsafe.Pointer
	onDevice := 0
	if nCmt == 0 && !userHints && !spr.GkrInfo.Is() {
		ds, err := pk.amdSolver(spr, h)
		if err != nil {
			return nil, err
		}
		if ds != nil {
			// held until gg_plonk_prove has read L, R, O from the solver's buffers
			mu := pk.amdLock()
			mu.Lock()
			defer mu.Unlock()
			if lro[0], lro[1], lro[2], err = ds.solve(fullWitness); err != nil {
				return nil, err
			}
			onDevice = 1
		}
	}
	if onDevice == 0 {
		_solution, err := spr.Solve(fullWitness, opt.SolverOpts...)
		if err != nil {
			return nil, err
		}
		sol := _solution.(*cs.SparseR1CSSolution)
		lro = [3]unsafe.Pointer{unsafe.Pointer(&sol.L[0]), unsafe.Pointer(&sol.R[0]), unsafe.Pointer(&sol.O[0])}
	}
	nbPub := len(spr.Public)
	cv := C.malloc(C.size_t(nCmt+1) * C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(cv)
	cvs := unsafe.Slice((*unsafe.Pointer)(cv), nCmt+1)
	for i := range committed {
		cvs[i] = C.CBytes(unsafe.Slice((*byte)(unsafe.Pointer(&committed[i][0])), len(committed[i])*fr.Bytes))
		defer C.free(cvs[i])
	}
	hc := cgo.NewHandle(opt.ChallengeHash)
	defer hc.Delete()
	hf := cgo.NewHandle(opt.KZGFoldingHash)
	defer hf.Delete()
	size := C.gg_plonk_proof_size_ex(amdCurve, C.int(nCmt))
	out := make([]byte, size)
	var pubPtr, dgPtr, hvPtr unsafe.Pointer
	if nbPub > 0 {
		pubPtr = unsafe.Pointer(&w[0])
	}
	if nCmt > 0 {
		dgPtr = unsafe.Pointer(&proof.Bsb22Commitments[0])
		hvPtr = unsafe.Pointer(&commitmentVal[0])
	}
	rc := C.gg_plonk_prove(h, lro[0], lro[1], lro[2], C.int(onDevice),
		pubPtr, C.size_t(nbPub), (*unsafe.Pointer)(cv), dgPtr, hvPtr, C.int(nCmt), nil,
		C.gg_go_hash_fn(), unsafe.Pointer(uintptr(hc)), C.gg_go_hash_fn(), unsafe.Pointer(uintptr(hf)),
		unsafe.Pointer(&out[0]), size)
	if rc != C.GG_OK {
		return nil, amdError()
	}
	// proof layout: include/gnark_amd.h gg_plonk_prove (gnark-crypto memory layout)
	o := 0
	g1 := func(p *curve.G1Affine) { *p = *(*curve.G1Affine)(unsafe.Pointer(&out[o])); o += curve.SizeOfG1AffineUncompressed }
	frv := func(e *fr.Element) { *e = *(*fr.Element)(unsafe.Pointer(&out[o])); o += 32 }
	for i := 0; i < 3; i++ {
		g1(&proof.LRO[i])
	}
	g1(&proof.Z)
	for i := 0; i < 3; i++ {
		g1(&proof.H[i])
	}
	for i := 0; i < nCmt; i++ {
		g1(&proof.Bsb22Commitments[i])
	}
	g1(&proof.BatchedProof.H)
	proof.BatchedProof.ClaimedValues = make([]fr.Element, 7+nCmt)
	for i := range proof.BatchedProof.ClaimedValues {
		frv(&proof.BatchedProof.ClaimedValues[i])
	}
	g1(&proof.ZShiftedOpening.H)
	frv(&proof.ZShiftedOpening.ClaimedValue)
	if o != len(out) {
		return nil, errors.New("gnark_amd: proof size mismatch")
	}
	return proof, nil
}
