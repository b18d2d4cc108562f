//go:build mi355x

// The MI355X build of embedded/htree: the reference implementation
// (htree.go, its HTree renamed cpuHTree / New renamed newCPUHTree under this
// build tag) keeps narrow trees, the device builds the wide ones.  Each
// function cites the reference it replaces.  Uncompiled in the build image
// (no Go toolchain); see go/README.md.
package htree

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/immustore_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/immustore_amd -limmustore_merkle -Wl,-rpath,${SRCDIR}/../../third_party/immustore_amd
#include <stdlib.h>
#include "immustore_merkle.h"
*/
import "C"

import (
	"crypto/sha256"
	"runtime"
	"unsafe"

	"github.com/codenotary/immudb/embedded/internal/mi355x"
)

// Trees narrower than this stay on the CPU: one small tree is launch / copy
// latency bound on the device (54 us at width 16 against 10 us on one core;
// the crossover lies between 256 and 4 096, profiles/build_latency_r01.json).
const deviceMinWidth = 1024

func mapErr(st C.int) error {
	switch st {
	case C.MH_OK:
		return nil
	case C.MH_ERR_MAX_WIDTH_EXCEEDED:
		return ErrMaxWidthExceeded // htree.go:25
	case C.MH_ERR_ILLEGAL_ARGUMENTS:
		return ErrIllegalArguments // htree.go:26
	case C.MH_ERR_ILLEGAL_STATE:
		return ErrIllegalState // htree.go:27
	}
	return mi355x.Status(int(st))
}

// HTree keeps the reference tree for narrow builds and a device tree,
// created on the first wide build, for the others; each proof follows the
// tree its build used.
type HTree struct {
	cpu      *cpuHTree
	h        *C.mh_htree
	onDevice bool
	maxWidth int
	width    int
	root     [sha256.Size]byte
}

// New -- htree.go:45-66.
func New(maxWidth int) (*HTree, error) {
	cpu, err := newCPUHTree(maxWidth)
	if err != nil {
		return nil, err
	}
	return &HTree{cpu: cpu, maxWidth: maxWidth}, nil
}

// BuildWith -- htree.go:68-113.
func (t *HTree) BuildWith(digests [][sha256.Size]byte) error {
	if len(digests) < deviceMinWidth {
		if err := t.cpu.BuildWith(digests); err != nil {
			return err
		}
		t.onDevice, t.width, t.root = false, len(digests), t.cpu.Root()
		return nil
	}
	if t.h == nil {
		p, err := mi355x.Context()
		if err != nil {
			return err
		}
		if st := C.mh_htree_new((*C.mh_ctx)(p), C.uint64_t(t.maxWidth), &t.h); st != C.MH_OK {
			return mapErr(st)
		}
		runtime.SetFinalizer(t, func(t *HTree) { C.mh_htree_free(t.h) })
	}
	// [][32]byte is one contiguous Go allocation of plain bytes: it may be
	// passed to C for the duration of the call (cgo pointer rules).
	p := (*C.uint8_t)(unsafe.Pointer(&digests[0][0]))
	if st := C.mh_htree_build_with(t.h, p, C.uint64_t(len(digests))); st != C.MH_OK {
		return mapErr(st)
	}
	t.onDevice, t.width = true, len(digests)
	if st := C.mh_htree_root(t.h, (*C.uint8_t)(unsafe.Pointer(&t.root[0]))); st != C.MH_OK {
		return mapErr(st)
	}
	return nil
}

// Root -- htree.go:115-117.
func (t *HTree) Root() [sha256.Size]byte { return t.root }

// InclusionProof -- htree.go:121-164 (terms read from the device levels).
func (t *HTree) InclusionProof(i int) (*InclusionProof, error) {
	if !t.onDevice {
		return t.cpu.InclusionProof(i)
	}
	if i < 0 {
		return nil, ErrIllegalArguments
	}
	var terms [64][sha256.Size]byte
	var n C.uint32_t
	st := C.mh_htree_inclusion_proof(t.h, C.uint64_t(i), (*C.uint8_t)(unsafe.Pointer(&terms[0][0])), 64, &n)
	if st != C.MH_OK {
		return nil, mapErr(st)
	}
	p := &InclusionProof{Leaf: i, Width: t.width}
	if n > 0 {
		p.Terms = append([][sha256.Size]byte(nil), terms[:n]...)
	}
	return p, nil
}

// VerifyInclusionBatch checks many proofs at once (htree.go:166-195 per
// proof); a single proof stays the reference's VerifyInclusion (one proof is
// cheaper on a host core than a PCIe round trip).  ok[p] is the verdict; a
// nil proof is false without reaching the device, as VerifyInclusion returns
// false for it (htree.go:167-169).  digests and roots hold one entry per
// proof: anything else is ErrIllegalArguments before C reads n x 32 bytes.
func VerifyInclusionBatch(proofs []*InclusionProof, digests, roots [][sha256.Size]byte) ([]bool, error) {
	n := len(proofs)
	if len(digests) != n || len(roots) != n {
		return nil, ErrIllegalArguments
	}
	ok := make([]bool, n)
	// the non-nil proofs, packed (idx[q] = their position in proofs)
	idx := make([]int, 0, n)
	for k, pr := range proofs {
		if pr != nil {
			idx = append(idx, k)
		}
	}
	m := len(idx)
	if m == 0 {
		return ok, nil
	}
	p, err := mi355x.Context()
	if err != nil {
		return nil, err
	}
	leaf := make([]uint64, m)
	width := make([]uint64, m)
	off := make([]uint64, m+1)
	dig := make([][sha256.Size]byte, m)
	rts := make([][sha256.Size]byte, m)
	var terms [][sha256.Size]byte
	for q, k := range idx {
		pr := proofs[k]
		leaf[q], width[q] = uint64(pr.Leaf), uint64(pr.Width)
		dig[q], rts[q] = digests[k], roots[k]
		terms = append(terms, pr.Terms...)
		off[q+1] = uint64(len(terms))
	}
	if len(terms) == 0 {
		terms = make([][sha256.Size]byte, 1)
	}
	res := make([]uint8, m)
	st := C.mh_htree_verify_inclusion_batch((*C.mh_ctx)(p), C.uint64_t(m),
		(*C.uint64_t)(unsafe.Pointer(&leaf[0])), (*C.uint64_t)(unsafe.Pointer(&width[0])),
		(*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint8_t)(unsafe.Pointer(&terms[0][0])),
		(*C.uint8_t)(unsafe.Pointer(&dig[0][0])), (*C.uint8_t)(unsafe.Pointer(&rts[0][0])),
		(*C.uint8_t)(unsafe.Pointer(&res[0])))
	if st != C.MH_OK {
		return nil, mapErr(st)
	}
	for q, k := range idx {
		ok[k] = res[q] != 0
	}
	return ok, nil
}
