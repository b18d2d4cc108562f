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

var (
	multiOnce sync.Once
	multi     *C.mh_multi
	multiErr  error
)

// Multi returns the process-wide clique over every visible GPU
// (mh_multi_create: one context per device, an RCCL clique inside the
// library), created on first use: the batch paths bound by one device's PCIe
// link (tx-log validation, value checks, precommit batches, proof batches)
// split their input over it, each part over its own link.
func Multi() (unsafe.Pointer, error) {
	multiOnce.Do(func() {
		var n C.int
		if st := C.mh_device_count(&n); st != C.MH_OK || n < 1 {
			multiErr = ErrNoDevice
			return
		}
		devs := make([]C.int, int(n))
		for i := range devs {
			devs[i] = C.int(i)
		}
		if st := C.mh_multi_create(n, &devs[0], &multi); st != C.MH_OK {
			multiErr = Status(int(st))
		}
	})
	return unsafe.Pointer(multi), multiErr
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
