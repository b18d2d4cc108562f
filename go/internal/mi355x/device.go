//go:build mi355x

// Package mi355x holds what the htree / store / ahtree shims share: the one
// device context of the process, pinned arenas and the mapping of the C ABI's
// status codes (include/immustore_merkle.h) onto the reference's sentinel
// errors.  Uncompiled in the build image (no Go toolchain); see go/README.md.
package mi355x

/*
#cgo CFLAGS: -I${SRCDIR}/../../../third_party/immustore_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../../third_party/immustore_amd -limmustore_merkle -Wl,-rpath,${SRCDIR}/../../../third_party/immustore_amd
#include <stdlib.h>
#include "immustore_merkle.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"sync"
	"unsafe"
)

var (
	ctxOnce sync.Once
	ctx     *C.mh_ctx
	ctxErr  error
)

// Context returns the process-wide device context (device 0), created on
// first use.  MH_ERR_NO_DEVICE (no gfx950 GPU) is returned as an error and
// the callers fall back to the reference's CPU code.
func Context() (unsafe.Pointer, error) {
	ctxOnce.Do(func() {
		if st := C.mh_ctx_create(0, nil, &ctx); st != C.MH_OK {
			ctxErr = Status(int(st))
		}
	})
	return unsafe.Pointer(ctx), ctxErr
}

// Cliques for the batch paths bound by one device's PCIe link (tx-log
// validation, value checks, precommit batches, ahtree batch appends): each is
// an mh_multi over every visible GPU (one context per device and an RCCL
// clique inside the library) that splits its input over the devices, each
// part over its own link.  A clique serialises its calls, so concurrent
// committers (immudb runs up to MaxConcurrency precommits at once,
// immustore.go:1620-1632, options.go:35) each check one out of a small pool
// instead of sharing one: two handles per device by default (two builds in
// flight measured 1247 GiB/s against 1094 with one, profiles/
// cabi_inflight_r05.txt; the pool's aggregate from plain C threads,
// tests/c_client/mh_committers.c, profiles/committers_r06.txt).
var (
	poolMu   sync.Mutex
	poolCond = sync.NewCond(&poolMu)
	poolFree []*C.mh_multi
	poolMade int
	poolMax  int // 0 until first use or SetCliquePool
	poolDevs []C.int
)

// SetCliquePool sets how many cliques the batch paths may hold at once (the
// number of callers that run in parallel; the store sets it from its
// options).  Takes effect for cliques created after the call; n < 1 means
// the default of two per device.
func SetCliquePool(n int) {
	poolMu.Lock()
	defer poolMu.Unlock()
	poolMax = n
	poolCond.Broadcast()
}

func poolInit() error {
	if poolDevs != nil {
		return nil
	}
	var n C.int
	if st := C.mh_device_count(&n); st != C.MH_OK || n < 1 {
		return ErrNoDevice
	}
	poolDevs = make([]C.int, int(n))
	for i := range poolDevs {
		poolDevs[i] = C.int(i)
	}
	if poolMax < 1 {
		poolMax = 2 * int(n)
	}
	return nil
}

// AcquireClique checks out a clique over every visible GPU: a free one, a
// new one while fewer than the pool size exist, else it waits for one to be
// returned.  Every AcquireClique is paired with a ReleaseClique.
func AcquireClique() (unsafe.Pointer, error) {
	poolMu.Lock()
	defer poolMu.Unlock()
	if err := poolInit(); err != nil {
		return nil, err
	}
	for {
		if k := len(poolFree); k > 0 {
			m := poolFree[k-1]
			poolFree = poolFree[:k-1]
			return unsafe.Pointer(m), nil
		}
		if poolMade < poolMax {
			var m *C.mh_multi
			if st := C.mh_multi_create(C.int(len(poolDevs)), &poolDevs[0], &m); st != C.MH_OK {
				return nil, Status(int(st))
			}
			poolMade++
			return unsafe.Pointer(m), nil
		}
		poolCond.Wait()
	}
}

// ReleaseClique returns a clique after a call that ended with status st.  A
// clique whose call failed with MH_ERR_COLLECTIVE has aborted its
// communicators (capi_multi.hip gather_bytes) and fails every later call, so
// it is destroyed instead and the next AcquireClique creates a new one.
func ReleaseClique(m unsafe.Pointer, st int) {
	poolMu.Lock()
	defer poolMu.Unlock()
	if st == int(C.MH_ERR_COLLECTIVE) || poolMade > poolMax && poolMax > 0 {
		C.mh_multi_destroy((*C.mh_multi)(m))
		poolMade--
	} else {
		poolFree = append(poolFree, (*C.mh_multi)(m))
	}
	poolCond.Signal()
}

// StatusError is a C ABI status with no Go sentinel of its own.
type StatusError struct {
	Code int
	Msg  string
}

func (e *StatusError) Error() string { return fmt.Sprintf("mi355x: %s (%d)", e.Msg, e.Code) }

// Status maps a non-OK status to an error; packages map the codes that have
// a sentinel in their own package first (see htree.mapErr, store.mapErr).
func Status(st int) error {
	if st == int(C.MH_OK) {
		return nil
	}
	return &StatusError{Code: st, Msg: C.GoString(C.mh_status_string(C.int(st)))}
}

// Arena is C-allocated pinned host memory: Go pointers cannot be stored on
// the C side and Go 1.18 has no runtime.Pinner, so entries are packed here
// and each arena goes over PCIe as one DMA.
type Arena struct {
	p   unsafe.Pointer
	cap int
}

func (a *Arena) Ensure(n int) error {
	if n <= a.cap && a.p != nil {
		return nil
	}
	a.Free()
	var p unsafe.Pointer
	if st := C.mh_host_alloc_pinned(C.uint64_t(n), &p); st != C.MH_OK {
		return Status(int(st))
	}
	a.p, a.cap = p, n
	return nil
}

func (a *Arena) Bytes() []byte {
	if a.p == nil {
		return nil
	}
	return unsafe.Slice((*byte)(a.p), a.cap)
}

func (a *Arena) Ptr() unsafe.Pointer { return a.p }

func (a *Arena) Free() {
	if a.p != nil {
		C.mh_host_free_pinned(a.p)
		a.p, a.cap = nil, 0
	}
}

var ErrNoDevice = errors.New("mi355x: no gfx950 device")
