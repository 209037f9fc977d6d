//go:build amd

package amd_bn254

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
	"runtime"
	"sync"
	"time"
	"unsafe"

	curve "github.com/consensys/gnark-crypto/ecc/bn254"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr/hash_to_field"
	"github.com/consensys/gnark-crypto/ecc/bn254/fr/pedersen"
	"github.com/consensys/gnark/backend"
	groth16_bn254 "github.com/consensys/gnark/backend/groth16/bn254"
	"github.com/consensys/gnark/backend/groth16/internal"
	"github.com/consensys/gnark/backend/witness"
	"github.com/consensys/gnark/constraint"
	cs "github.com/consensys/gnark/constraint/bn254"
	"github.com/consensys/gnark/constraint/solver"
	"github.com/consensys/gnark/logger"
	fcs "github.com/consensys/gnark/frontend/cs"
)

// HasAMD mirrors icicle_bn254.HasIcicle (icicle.go:29).
const HasAMD = true

func lastError() error { return fmt.Errorf("gnark_amd: %s", C.GoString(C.gg_last_error())) }

func ptrOr(b bool, p unsafe.Pointer) unsafe.Pointer {
	if b {
		return p
	}
	return nil
}

var setupMu sync.Mutex // one key upload at a time (concurrent first Prove calls)

// onDevice runs fn on an OS thread bound to GPU dev (gg_set_device binds the
// calling thread; a goroutine must not migrate between the bind and the calls).
func onDevice(dev int, fn func() error) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	if C.gg_set_device(C.int(dev)) != C.GG_OK {
		return lastError()
	}
	return fn()
}

// setupDevicePointers uploads pk once (replaces icicle.go:31-130).
func (pk *ProvingKey) setupDevicePointers(nbPublic int, kWireIndex []uint32) error {
	setupMu.Lock()
	defer setupMu.Unlock()
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
	p := func(s unsafe.Pointer, n int) unsafe.Pointer { return ptrOr(n > 0, s) }
	devs := configuredDevices()
	if len(devs) > 1 {
		// one shard per GPU, driven from this process (gg_groth16_mpk_create_ex)
		cdevs := make([]C.int, len(devs))
		for i, d := range devs {
			cdevs[i] = C.int(d)
		}
		var mh C.gg_groth16_mpk_t
		rc := C.gg_groth16_mpk_create_ex(C.GG_CURVE_BN254, C.int(logN),
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
			(*C.uint32_t)(p(unsafe.Pointer(unsafe.SliceData(kWireIndex)), len(kWireIndex))),
			C.int(len(devs)), &cdevs[0], &mh)
		if rc != C.GG_OK {
			return lastError()
		}
		pk.deviceInfo = &deviceInfo{handle: unsafe.Pointer(mh), multi: true, devices: devs}
		return nil
	}
	dev := 0
	if len(devs) == 1 {
		dev = devs[0]
	}
	var h C.gg_groth16_pk_t
	err := onDevice(dev, func() error {
		if C.gg_groth16_pk_create_ex(C.GG_CURVE_BN254, C.int(logN),
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
			(*C.uint32_t)(p(unsafe.Pointer(unsafe.SliceData(kWireIndex)), len(kWireIndex))), &h) != C.GG_OK {
			return lastError()
		}
		return nil
	})
	if err != nil {
		return err
	}
	pk.deviceInfo = &deviceInfo{handle: unsafe.Pointer(h), devices: []int{dev}}
	return nil
}

// SetHBMBudget caps (bytes per device, 0 = the free HBM less a reserve) what
// the precomputed tables of keys created afterwards may take: a key that would
// not fit stores every G-th window shift instead (gg_set_hbm_budget,
// DESIGN.md §3), e.g. a 2^25-domain key, or a Groth16 and a PlonK key on one GPU.
func SetHBMBudget(bytes uint64) error {
	if C.gg_set_hbm_budget(C.size_t(bytes)) != C.GG_OK {
		return lastError()
	}
	return nil
}

// Release frees the HBM-resident key (the icicle path never frees it).
func (pk *ProvingKey) Release() {
	setupMu.Lock()
	defer setupMu.Unlock()
	if di := pk.deviceInfo; di != nil {
		di.mu.Lock()
		for _, ds := range di.solvers {
			ds.release()
		}
		if di.multi {
			C.gg_groth16_mpk_release(C.gg_groth16_mpk_t(di.handle))
		} else {
			C.gg_groth16_pk_release(C.gg_groth16_pk_t(di.handle))
		}
		di.mu.Unlock()
		pk.deviceInfo = nil
	}
}

// proveOnDeviceSolution solves a hint-free system on every GPU of the key
// (gg_r1cs_solve, the solution stays in HBM) and proves from there: the
// witness is the only per-proof PCIe traffic.  Holds di.mu from the solve to
// the end of the prove (the prove reads the solvers' resident vectors).
func (di *deviceInfo) proveOnDeviceSolution(fullWitness witness.Witness, ar *curve.G1Affine, bs *curve.G2Affine,
	krs *curve.G1Affine) error {
	var r, s fr.Element
	if _, err := r.SetRandom(); err != nil {
		return err
	}
	if _, err := s.SetRandom(); err != nil {
		return err
	}
	di.mu.Lock()
	defer di.mu.Unlock()
	type sol struct{ w, a, b, c unsafe.Pointer }
	sols := make(map[int]sol, len(di.solvers))
	errs := make(chan error, len(di.solvers))
	var smu sync.Mutex
	var wg sync.WaitGroup
	for dev, ds := range di.solvers {
		wg.Add(1)
		go func(dev int, ds *deviceSolver) {
			defer wg.Done()
			w, a, b, c, err := ds.solve(fullWitness)
			if err != nil {
				errs <- err
				return
			}
			smu.Lock()
			sols[dev] = sol{w, a, b, c}
			smu.Unlock()
		}(dev, ds)
	}
	wg.Wait()
	close(errs)
	if err := <-errs; err != nil {
		return err
	}
	var ds0 *deviceSolver
	for _, ds := range di.solvers {
		ds0 = ds
		break
	}
	if !di.multi {
		x := sols[di.devices[0]]
		if C.gg_groth16_prove(C.gg_groth16_pk_t(di.handle), x.w, C.size_t(ds0.nbWires), x.a, x.b, x.c,
			C.size_t(ds0.nbCons), 1, unsafe.Pointer(&r), unsafe.Pointer(&s),
			unsafe.Pointer(ar), unsafe.Pointer(bs), unsafe.Pointer(krs), nil) != C.GG_OK {
			return lastError()
		}
		return nil
	}
	// per-shard device pointers (C memory: device addresses, no Go pointers)
	world := len(di.devices)
	ptrs := C.malloc(C.size_t(4*world) * C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(ptrs)
	ps := unsafe.Slice((*unsafe.Pointer)(ptrs), 4*world)
	for i, dev := range di.devices {
		x := sols[dev]
		ps[i], ps[world+i], ps[2*world+i], ps[3*world+i] = x.w, x.a, x.b, x.c
	}
	if C.gg_groth16_mpk_prove_ex(C.gg_groth16_mpk_t(di.handle), 1, (*unsafe.Pointer)(&ps[0]),
		C.size_t(ds0.nbWires), (*unsafe.Pointer)(&ps[world]), (*unsafe.Pointer)(&ps[2*world]),
		(*unsafe.Pointer)(&ps[3*world]), C.size_t(ds0.nbCons), unsafe.Pointer(&r), unsafe.Pointer(&s),
		unsafe.Pointer(ar), unsafe.Pointer(bs), unsafe.Pointer(krs)) != C.GG_OK {
		return lastError()
	}
	return nil
}

// Prove mirrors icicle_bn254.Prove (icicle.go:133-422): identical solver,
// commitment and randomness handling; the MSM/NTT section runs in one
// gg_groth16_prove call.
func Prove(r1cs *cs.R1CS, pk *ProvingKey, fullWitness witness.Witness, opts ...backend.ProverOption) (*groth16_bn254.Proof, error) {
	opt, err := backend.NewProverConfig(opts...)
	if err != nil {
		return nil, fmt.Errorf("new prover config: %w", err)
	}
	if opt.HashToFieldFn == nil {
		opt.HashToFieldFn = hash_to_field.New([]byte(constraint.CommitmentDst))
	}
	if opt.Accelerator != "amd" && opt.Accelerator != "icicle" {
		return groth16_bn254.Prove(r1cs, &pk.ProvingKey, fullWitness, opts...)
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

	proof := &groth16_bn254.Proof{Commitments: make([]curve.G1Affine, len(commitmentInfo))}
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

	// hint-free systems without commitments: r1cs.Solve on the GPU(s) of the
	// key, the solution stays in HBM (solver_amd.go); everything else keeps
	// gnark's solver
	if len(commitmentInfo) == 0 && len(opt.SolverOpts) == 0 && !r1cs.GkrInfo.Is() {
		di := pk.deviceInfo
		di.solverOnce.Do(func() { di.solvers, di.solverErr = newDeviceSolvers(r1cs, di.devices) })
		if di.solverErr != nil {
			return nil, fmt.Errorf("device solver: %w", di.solverErr)
		}
		if len(di.solvers) > 0 {
			if err := di.proveOnDeviceSolution(fullWitness, &proof.Ar, &proof.Bs, &proof.Krs); err != nil {
				return nil, err
			}
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
	var rc C.int
	if pk.deviceInfo.multi {
		rc = C.gg_groth16_mpk_prove(C.gg_groth16_mpk_t(pk.deviceInfo.handle),
			unsafe.Pointer(&wireValues[0]), C.size_t(len(wireValues)),
			unsafe.Pointer(&solution.A[0]), unsafe.Pointer(&solution.B[0]), unsafe.Pointer(&solution.C[0]),
			C.size_t(len(solution.A)),
			unsafe.Pointer(&r), unsafe.Pointer(&s),
			unsafe.Pointer(&ar), unsafe.Pointer(&bs), unsafe.Pointer(&krs))
	} else {
		rc = C.gg_groth16_prove(C.gg_groth16_pk_t(pk.deviceInfo.handle),
			unsafe.Pointer(&wireValues[0]), C.size_t(len(wireValues)),
			unsafe.Pointer(&solution.A[0]), unsafe.Pointer(&solution.B[0]), unsafe.Pointer(&solution.C[0]),
			C.size_t(len(solution.A)), 0,
			unsafe.Pointer(&r), unsafe.Pointer(&s),
			unsafe.Pointer(&ar), unsafe.Pointer(&bs), unsafe.Pointer(&krs), nil)
	}
	if rc != C.GG_OK {
		return nil, lastError()
	}
	proof.Ar, proof.Bs, proof.Krs = ar, bs, krs
	log.Debug().Dur("took", time.Since(start)).Msg("prover done")
	return proof, nil
}
