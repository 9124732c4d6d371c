//go:build rsgpu

// gpu.go -- cgo binding of the MI355X hot path (include/rsgpu.h) for the reference's Go package core.
//
// Drop-in: copy this file into the reference's core/ directory, put rsgpu.h and librsgpu.so where the
// #cgo lines below point (third_party/rsgpu/{include,lib}), and build with `go build -tags rsgpu`.
// Without the tag the package builds exactly as before.  Each Fit body below is the reference's own
// setup (parameter defaults, allocations, the unseeded init draws of svd.go:80-85 / 167-168 / 335-341)
// followed by ONE library call in place of the epoch loop; the estimators' exported fields
// ([][]float64 rows) alias the buffers the library writes, so Predict (svd.go:32-51, knn.go:75-141)
// runs unchanged.  The one edit to the reference itself is a two-line dispatch at the top of each Fit:
//
//	if s.Params.GetString("device", "") == "gpu" { s.fitGPU(trainData); return }     // svd.go:63
//
// (likewise in SVDPP.Fit, NMF.Fit and, for the pair loop of knn.go:188-216, KNN.Fit).
//
// cgo pointer rules: no memory handed to C holds a Go pointer.  The rs_ratings struct and its arrays are
// C.malloc'd and freed after the call (newCRatings); outputs are []float64 backing arrays (no pointers
// inside); the rs_ctx is closed before Fit returns.  The library keeps no caller pointer after a call.
//
// This file is unverified by a Go build: neither the container nor the MI355X boxes this repository is
// tested on have a Go toolchain (DESIGN.md §1).  Every entry point it calls is exercised through the same
// C-ABI by the Python ctypes binding (tests/) and by the C++ mirror of this API (recommend-sys_amd/host/,
// tests/test_host_cpp.py), whose TestCgoRatingsShape drives rs_svd_fit with rs_ratings allocated and
// freed exactly as newCRatings does.
package core

// #cgo CFLAGS: -I${SRCDIR}/../third_party/rsgpu/include
// #cgo LDFLAGS: -L${SRCDIR}/../third_party/rsgpu/lib -lrsgpu -Wl,-rpath,${SRCDIR}/../third_party/rsgpu/lib
// #include <stdlib.h>
// #include "rsgpu.h"
import "C"

import (
	"fmt"
	"unsafe"
)

// gpuCtx is one rs_ctx: one device and one HIP stream, not thread-safe.  CrossValidate (eval.go:28-35)
// fits every fold's own estimator copy in its own goroutine, so each Fit opens its own ctx and closes it
// before returning (`defer g.close()`): the ctx holds a HIP stream and its pinned staging (owned by the ctx,
// freed by rs_close), which a finalizer would keep alive until some later GC.
//
// Goroutine migration: Go may resume a goroutine on another OS thread between two cgo calls.  Every entry
// point re-binds its ctx's device, and a ctx's error message lives in the ctx, so ctx calls are unaffected.
// The ctx-less calls (rs_open, rs_svd_fit_multi) would leave theirs in the failing OS thread's slot, so they go
// through the rs_report variants: the call itself writes its message (and rs_svd_fit_multi its refits) into a
// report the caller owns -- a Go struct with no Go pointers, legal to pass (host/tests/core_test.cpp
// TestCtxlessErrorAcrossThreads reads such a report on another thread).
type gpuCtx struct{ p *C.rs_ctx }

func openGPU(device int) *gpuCtx {
	var p *C.rs_ctx
	var rep C.rs_report
	if rc := C.rs_open_r(C.int32_t(device), &p, &rep); rc != C.RS_OK {
		panic(fmt.Sprintf("rs_open: %s", C.GoString(&rep.error[0])))
	}
	return &gpuCtx{p}
}

func (g *gpuCtx) close() {
	if g.p != nil {
		C.rs_close(g.p)
		g.p = nil
	}
}

// check panics like the reference does on bad input: its Fit has no error return.  RS_ERR_NUMERIC means
// the FAST fit diverged even after the library's own refits with shorter hot-item runs (rsgpu.h).
func (g *gpuCtx) check(rc C.int, what string) {
	if rc != C.RS_OK {
		panic(fmt.Sprintf("%s: %s", what, C.GoString(C.rs_last_error(g.p))))
	}
}

// cRatings: the TrainSet's triples in train-set order with inner ids (data.go:131-154), copied into C
// memory.  cgo's pointer-passing rule forbids handing C a Go struct that holds Go pointers (the default
// GODEBUG=cgocheck=1 panics with "cgo argument has Go pointer to unpinned Go pointer"), so the
// rs_ratings struct and its three arrays are all C.malloc'd; the caller frees them once the call has
// returned (`defer cr.free()`).  The library copies what it needs during the call and keeps no pointer.
// (tests: host/tests/core_test.cpp TestCgoRatingsShape builds and frees rs_ratings exactly this way.)
type cRatings struct{ r *C.rs_ratings }

func newCRatings(t *TrainSet) cRatings {
	n := t.Length()
	m := n
	if m == 0 {
		m = 1 // a valid pointer for an empty set
	}
	r := (*C.rs_ratings)(C.malloc(C.size_t(unsafe.Sizeof(C.rs_ratings{}))))
	users := (*C.int32_t)(C.malloc(C.size_t(m) * 4))
	items := (*C.int32_t)(C.malloc(C.size_t(m) * 4))
	vals := (*C.double)(C.malloc(C.size_t(m) * 8))
	u, i, v := unsafe.Slice(users, m), unsafe.Slice(items, m), unsafe.Slice(vals, m)
	for k := 0; k < n; k++ {
		u[k] = C.int32_t(t.ConvertUserID(t.Users[k]))
		i[k] = C.int32_t(t.ConvertItemID(t.Items[k]))
		v[k] = C.double(t.Ratings[k])
	}
	r.nnz = C.int64_t(n)
	r.n_users = C.int32_t(t.UserCount)
	r.n_items = C.int32_t(t.ItemCount)
	r.users, r.items, r.ratings = users, items, vals
	return cRatings{r}
}

func (c cRatings) free() {
	C.free(unsafe.Pointer(c.r.users))
	C.free(unsafe.Pointer(c.r.items))
	C.free(unsafe.Pointer(c.r.ratings))
	C.free(unsafe.Pointer(c.r))
}

// flat: one contiguous []float64 with the [][]float64 rows sliced out of it (the rows alias the buffer
// the library writes into, so nothing is copied back).
func flat(rows, k int) ([]float64, [][]float64) {
	buf := make([]float64, rows*k+1)
	m := make([][]float64, rows)
	for r := range m {
		m[r] = buf[r*k : (r+1)*k : (r+1)*k]
	}
	return buf, m
}

// f64: an output buffer.  Passing a pointer into a []float64 is legal cgo: the backing array holds no Go
// pointers, and the library writes it before returning and keeps nothing.  (rs_sgd_params, passed as &p,
// holds no pointers either.)
func f64(b []float64) *C.double { return (*C.double)(unsafe.Pointer(&b[0])) }

func sgdMode(p Parameters) C.int32_t {
	if p.GetString("mode", "fast") == "ordered" { // svd.go:93-129's exact visit order (1e-5 contract)
		return C.RS_SGD_ORDERED
	}
	return C.RS_SGD_FAST
}

// fitGPU is (*SVD).Fit (svd.go:63-132) with the epoch loop on the GPU.  "nGPUs" > 1 runs the sharded
// fit on that many devices of this process (rs_svd_fit_multi: the smaller factor matrix rotates).
func (s *SVD) fitGPU(trainData TrainSet) {
	nFactors := s.Params.GetInt("nFactors", 100)
	nEpochs := s.Params.GetInt("nEpochs", 20)
	lr := s.Params.GetFloat64("lr", 0.005)
	reg := s.Params.GetFloat64("reg", 0.02)
	initMean := s.Params.GetFloat64("initMean", 0)
	initStdDev := s.Params.GetFloat64("initStdDev", 0.1)
	s.Data = trainData
	pBuf, P := flat(trainData.UserCount, nFactors)
	qBuf, Q := flat(trainData.ItemCount, nFactors)
	for u := range P { // svd.go:80-85: the same draws in the same order (users, then items)
		copy(P[u], newNormalVector(nFactors, initMean, initStdDev))
	}
	for i := range Q {
		copy(Q[i], newNormalVector(nFactors, initMean, initStdDev))
	}
	s.UserFactor, s.ItemFactor = P, Q
	s.UserBias = make([]float64, trainData.UserCount+1)[:trainData.UserCount]
	s.ItemBias = make([]float64, trainData.ItemCount+1)[:trainData.ItemCount]
	s.GlobalBias = 0
	cr := newCRatings(&trainData)
	defer cr.free()
	p := C.rs_sgd_params{n_factors: C.int32_t(nFactors), n_epochs: C.int32_t(nEpochs),
		lr: C.double(lr), reg: C.double(reg), mode: sgdMode(s.Params), write_back: C.RS_SGD_WB_TILE}
	bu := (*C.double)(unsafe.Pointer(&s.UserBias[:1][0]))
	bi := (*C.double)(unsafe.Pointer(&s.ItemBias[:1][0]))
	gb := (*C.double)(unsafe.Pointer(&s.GlobalBias))
	if nGPUs := s.Params.GetInt("nGPUs", 1); nGPUs > 1 && p.mode == C.RS_SGD_FAST {
		d := make([]int32, nGPUs)
		for k := range d {
			d[k] = int32(k)
		}
		var rep C.rs_report
		rc := C.rs_svd_fit_multi((*C.int32_t)(unsafe.Pointer(&d[0])), C.int32_t(len(d)), cr.r, &p, 0,
			f64(pBuf), f64(qBuf), bu, bi, gb, &rep)
		if rc != C.RS_OK {
			panic(fmt.Sprintf("SVD.Fit (%d GPUs, %d refits): %s", nGPUs, int(rep.refits), C.GoString(&rep.error[0])))
		}
		return
	}
	g := openGPU(s.Params.GetInt("deviceID", 0))
	defer g.close()
	g.check(C.rs_svd_fit(g.p, cr.r, &p, f64(pBuf), f64(qBuf), bu, bi, gb), "SVD.Fit")
}

// fitGPU is (*SVDPP).Fit (svd.go:316-427): the same shape with the implicit factors Y.
func (pp *SVDPP) fitGPU(trainData TrainSet) {
	nFactors := pp.Params.GetInt("nFactors", 20)
	nEpochs := pp.Params.GetInt("nEpochs", 20)
	lr := pp.Params.GetFloat64("lr", 0.007)
	reg := pp.Params.GetFloat64("reg", 0.02)
	initMean := pp.Params.GetFloat64("initMean", 0)
	initStdDev := pp.Params.GetFloat64("initStdDev", 0.1)
	pp.Data = trainData
	pp.UserBias = make([]float64, trainData.UserCount+1)[:trainData.UserCount]
	pp.ItemBias = make([]float64, trainData.ItemCount+1)[:trainData.ItemCount]
	pBuf, P := flat(trainData.UserCount, nFactors)
	qBuf, Q := flat(trainData.ItemCount, nFactors)
	yBuf, Y := flat(trainData.ItemCount, nFactors)
	for u := range P { // svd.go:335-341: users, then per item q_i and y_i
		copy(P[u], newNormalVector(nFactors, initMean, initStdDev))
	}
	for i := range Q {
		copy(Q[i], newNormalVector(nFactors, initMean, initStdDev))
		copy(Y[i], newNormalVector(nFactors, initMean, initStdDev))
	}
	pp.UserFactor, pp.ItemFactor, pp.ImplFactor = P, Q, Y
	pp.GlobalBias = 0
	pp.UserRatings = trainData.UserRatings() // Predict still needs N(u) (svd.go:271-282)
	cr := newCRatings(&trainData)
	defer cr.free()
	p := C.rs_sgd_params{n_factors: C.int32_t(nFactors), n_epochs: C.int32_t(nEpochs),
		lr: C.double(lr), reg: C.double(reg), mode: sgdMode(pp.Params), write_back: C.RS_SGD_WB_TILE}
	g := openGPU(pp.Params.GetInt("deviceID", 0))
	defer g.close()
	g.check(C.rs_svdpp_fit(g.p, cr.r, &p, f64(pBuf), f64(qBuf), f64(yBuf),
		(*C.double)(unsafe.Pointer(&pp.UserBias[:1][0])), (*C.double)(unsafe.Pointer(&pp.ItemBias[:1][0])),
		(*C.double)(unsafe.Pointer(&pp.GlobalBias))), "SVDPP.Fit")
}

// fitGPU is (*NMF).Fit (svd.go:158-251).  "nmfAsWritten" (default true) keeps svd.go:243-249's item
// update as written (DESIGN.md Q5); false runs the intended multiplicative update.
func (N *NMF) fitGPU(trainSet TrainSet) {
	nFactors := N.Params.GetInt("nFactors", 15)
	nEpochs := N.Params.GetInt("nEpochs", 50)
	initLow := N.Params.GetFloat64("initLow", 0)
	initHigh := N.Params.GetFloat64("initHigh", 1)
	reg := N.Params.GetFloat64("reg", 0.06)
	N.Data = trainSet
	pBuf, P := flat(trainSet.UserCount, nFactors)
	qBuf, Q := flat(trainSet.ItemCount, nFactors)
	up, iq := newUniformMatrix(trainSet.UserCount, nFactors, initLow, initHigh),
		newUniformMatrix(trainSet.ItemCount, nFactors, initLow, initHigh) // svd.go:167-168
	for k := range P {
		copy(P[k], up[k])
	}
	for k := range Q {
		copy(Q[k], iq[k])
	}
	N.userFactor, N.itemFactor = P, Q
	asWritten := C.int32_t(1)
	if !N.Params.GetBool("nmfAsWritten", true) {
		asWritten = 0
	}
	cr := newCRatings(&trainSet)
	defer cr.free()
	g := openGPU(N.Params.GetInt("deviceID", 0))
	defer g.close()
	g.check(C.rs_nmf_fit(g.p, cr.r, C.int32_t(nFactors), C.int32_t(nEpochs), C.double(reg), asWritten,
		f64(pBuf), f64(qBuf)), "NMF.Fit")
}

// simsGPU replaces the sorts() + nJobs pair loop of (*KNN).Fit (knn.go:188-216): everything before
// knn.go:188 stays as it is (LeftRatings, RightRatings, Means, StdDevs, Bias); this fills K.Sims with the
// same float64 values, bitwise, NaN where nothing is co-rated.
func (K *KNN) simsGPU(sim Sim) {
	L, R := len(K.LeftRatings), len(K.RightRatings)
	rowptr := make([]int64, L+1)
	ids := make([]int32, 0, K.Data.Length()+1)
	vals := make([]float64, 0, K.Data.Length()+1)
	for l, row := range K.LeftRatings { // any order inside a row: the library orders by ID itself
		for _, ir := range row {
			ids = append(ids, int32(ir.ID))
			vals = append(vals, ir.Rating)
		}
		rowptr[l+1] = int64(len(ids))
	}
	ids, vals = append(ids, 0), append(vals, 0) // valid &x[0] for an empty set
	buf, S := flat(L, L)
	g := openGPU(K.Params.GetInt("deviceID", 0))
	defer g.close()
	g.check(C.rs_knn_sims(g.p, simKind(sim), C.int32_t(L), C.int32_t(R),
		(*C.int64_t)(unsafe.Pointer(&rowptr[0])), (*C.int32_t)(unsafe.Pointer(&ids[0])),
		f64(vals), f64(buf)), "KNN.Fit")
	K.Sims = S
}

// simKind maps the three exported Sim values (Go funcs are not comparable, so by pointer).
func simKind(s Sim) C.int32_t {
	switch fmt.Sprintf("%p", s) {
	case fmt.Sprintf("%p", Cosine):
		return C.RS_SIM_COSINE
	case fmt.Sprintf("%p", Pearson):
		return C.RS_SIM_PEARSON
	case fmt.Sprintf("%p", MSD):
		return C.RS_SIM_MSD
	}
	panic("KNN: only core.Cosine, core.MSD and core.Pearson run on the GPU")
}

// fitGPU is (*BaseLine).Fit (base.go:135-163), bitwise (KNNBaseLine reaches it through knn.go:179-187).
func (baseLine *BaseLine) fitGPU(trainSet TrainSet) {
	nEpochs := baseLine.Params.GetInt("nEpochs", 20)
	reg := baseLine.Params.GetFloat64("reg", 0.02)
	lr := baseLine.Params.GetFloat64("lr", 0.005)
	baseLine.trainSet = trainSet
	baseLine.userBias = make([]float64, trainSet.UserCount+1)[:trainSet.UserCount]
	baseLine.itemBias = make([]float64, trainSet.ItemCount+1)[:trainSet.ItemCount]
	baseLine.globalBias = 0 // base.go:135-163 starts it at zero (the loop learns it)
	cr := newCRatings(&trainSet)
	defer cr.free()
	g := openGPU(baseLine.Params.GetInt("deviceID", 0))
	defer g.close()
	g.check(C.rs_baseline_fit(g.p, cr.r, C.int32_t(nEpochs), C.double(lr), C.double(reg),
		(*C.double)(unsafe.Pointer(&baseLine.userBias[:1][0])), (*C.double)(unsafe.Pointer(&baseLine.itemBias[:1][0])),
		(*C.double)(unsafe.Pointer(&baseLine.globalBias))), "BaseLine.Fit")
}
