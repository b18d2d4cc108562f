//go:build mi355x

// The MI355X build's batch append for embedded/ahtree: syncBinaryLinking's
// replay (embedded/store/immustore.go:1198-1232, reached on every open,
// :686-693, resuming at aht.Size()+1) appends a whole range of Alh values as
// ONE device call onto the tree's current peaks instead of one Append
// (ahtree.go:246-373) per transaction -- across every GPU of the node, each
// holding only its own range of the new dLog.  Single appends on the commit
// path stay the reference's (one serial chain of ~24 compressions: 81 us
// through the device against 6.8 us on a core, DESIGN.md).  Uncompiled in the
// build image (no Go toolchain); see go/README.md.
package ahtree

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/immustore_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/immustore_amd -limmustore_merkle -Wl,-rpath,${SRCDIR}/../../third_party/immustore_amd
#include <stdlib.h>
#include "immustore_merkle.h"
*/
import "C"

import (
	"crypto/sha256"
	"encoding/binary"
	"sync"
	"unsafe"

	"github.com/codenotary/immudb/embedded/internal/mi355x"
)

// devices checks a clique over every visible GPU out of the process's pool
// (mi355x.AcquireClique); the caller returns it with mi355x.ReleaseClique.
func devices() (*C.mh_multi, error) {
	m, err := mi355x.AcquireClique()
	return (*C.mh_multi)(m), err
}

func mapErr(st C.int) error {
	switch st {
	case C.MH_OK:
		return nil
	case C.MH_ERR_ILLEGAL_ARGUMENTS:
		return ErrIllegalArguments // ahtree.go:35
	case C.MH_ERR_EMPTY_TREE:
		return ErrEmptyTree // ahtree.go:42
	case C.MH_ERR_UNEXISTENT_DATA:
		return ErrUnexistentData // ahtree.go:44
	case C.MH_ERR_CANNOT_RESET_TO_LARGER:
		return ErrCannotResetToLargerSize
	}
	return mi355x.Status(int(st))
}

// peaks are the perfect subtree roots of a tree of size n, lowest level
// first: node(n with the bits below l cleared, l) for every set bit l of n
// (the only old nodes any later append reads, ahtree.go:296-322).
func (t *AHtree) peaks(n uint64) ([]byte, error) {
	var out []byte
	for l := 0; l < 64; l++ {
		if n>>uint(l)&1 == 0 {
			continue
		}
		h, err := t.node(n&^(uint64(1)<<uint(l)-1), l)
		if err != nil {
			return nil, err
		}
		out = append(out, h[:]...)
	}
	return out, nil
}

// AppendBatch appends every payload of ds (32-byte Alh values on the replay
// path; any lengths) exactly as len(ds) calls of Append would: the same pLog
// records, dLog digests (the tree/*.sha stream) and cLog entries, and returns
// RootAt(size) after the batch.  Like Append (ahtree.go:260-263) it rejects
// only a nil payload; the C ABI takes one payload length per call, so each
// maximal run of equal-length payloads is one device batch.
//
// Partial failure: the runs are committed one after the other.  If run k
// fails, runs 0..k-1 are already in pLog, dLog and cLog (as len(ds) single
// Appends would have left them up to the failing one), so the error comes
// with n = the tree size after the last run that succeeded and root =
// RootAt(n) -- the state the caller resumes from (n = the size before the
// call and a zero root when the first run fails).
func (t *AHtree) AppendBatch(ds [][]byte) (n uint64, root [sha256.Size]byte, err error) {
	t.mutex.Lock()
	defer t.mutex.Unlock()
	if t.closed {
		return 0, root, ErrAlreadyClosed
	}
	if t.readOnly {
		return 0, root, ErrReadOnly
	}
	if len(ds) == 0 {
		return t.size(), root, ErrIllegalArguments
	}
	for _, d := range ds {
		if d == nil {
			return 0, root, ErrIllegalArguments
		}
	}
	n = t.size()
	for i := 0; i < len(ds); {
		j := i + 1
		for j < len(ds) && len(ds[j]) == len(ds[i]) {
			j++
		}
		rn, rroot, rerr := t.appendRun(ds[i:j])
		if rerr != nil {
			// n / root: what the runs before this one committed
			return n, root, rerr
		}
		n, root = rn, rroot
		i = j
	}
	return n, root, nil
}

// appendRun: one device batch of equal-length payloads (t.mutex held).
func (t *AHtree) appendRun(ds [][]byte) (n uint64, root [sha256.Size]byte, err error) {
	m := len(ds)
	plen := len(ds[0])
	mm, err := devices()
	if err != nil {
		return 0, root, err
	}
	released := false
	defer func() { // on the early returns; the call's own status releases it below
		if !released {
			mi355x.ReleaseClique(unsafe.Pointer(mm), 0)
		}
	}()
	// what earlier single Appends buffered goes to disk first, so the cLog
	// entries of the batch follow synced pLog / dLog bytes (ahtree.go:788-836)
	if err = t.sync(); err != nil {
		return 0, root, err
	}
	n0 := t.size()
	pk, err := t.peaks(n0)
	if err != nil {
		return 0, root, err
	}
	payloads := make([]byte, m*plen)
	plog := make([]byte, m*(szSize+plen))
	clog := make([]byte, m*cLogEntrySize)
	for i, d := range ds {
		copy(payloads[i*plen:], d)
		r := plog[i*(szSize+plen):]
		binary.BigEndian.PutUint32(r, uint32(plen)) // ahtree.go:271-284
		copy(r[szSize:], d)
		poff := t.pLogSize + int64(i*(szSize+plen))
		binary.BigEndian.PutUint64(clog[i*cLogEntrySize:], uint64(poff)) // ahtree.go:353-355
		binary.BigEndian.PutUint32(clog[i*cLogEntrySize+offsetSize:], uint32(plen))
	}
	nd := uint64(C.mh_ahtree_nodes_upto(C.uint64_t(n0+uint64(m)))) - uint64(C.mh_ahtree_nodes_upto(C.uint64_t(n0)))
	dlog := make([]byte, nd*sha256.Size)
	var pkp *C.uint8_t
	if len(pk) > 0 {
		pkp = (*C.uint8_t)(unsafe.Pointer(&pk[0]))
	}
	// zero-length payloads (Append accepts them, ahtree.go:279 only skips
	// the pLog bytes): no payload buffer, which the C side allows for plen 0
	var pp *C.uint8_t
	if plen > 0 {
		pp = (*C.uint8_t)(unsafe.Pointer(&payloads[0]))
	}
	st := C.mh_multi_ahtree_append_batch(mm, C.uint64_t(n0), pkp,
		pp, C.uint64_t(m), C.uint32_t(plen),
		(*C.uint8_t)(unsafe.Pointer(&dlog[0])), (*C.uint8_t)(unsafe.Pointer(&root[0])))
	mi355x.ReleaseClique(unsafe.Pointer(mm), int(st))
	released = true
	if st != C.MH_OK {
		return 0, root, mapErr(st)
	}
	// the three appendables, as Append writes them (ahtree.go:266-370)
	if err = t.pLog.SetOffset(t.pLogSize); err != nil {
		return 0, root, err
	}
	if _, _, err = t.pLog.Append(plog); err != nil {
		return 0, root, err
	}
	if err = t.dLog.SetOffset(t.dLogSize); err != nil {
		return 0, root, err
	}
	if _, _, err = t.dLog.Append(dlog); err != nil {
		return 0, root, err
	}
	for _, a := range []interface {
		Flush() error
		Sync() error
	}{t.pLog, t.dLog} {
		if err = a.Flush(); err != nil {
			return 0, root, err
		}
		if err = a.Sync(); err != nil {
			return 0, root, err
		}
	}
	if err = t.cLog.SetOffset(int64(t.latestSyncedNode) * cLogEntrySize); err != nil {
		return 0, root, err
	}
	if _, _, err = t.cLog.Append(clog); err != nil {
		return 0, root, err
	}
	if err = t.cLog.Flush(); err != nil {
		return 0, root, err
	}
	if err = t.cLog.Sync(); err != nil {
		return 0, root, err
	}
	t.latestSyncedNode += uint64(m)
	t.pLogSize += int64(len(plog))
	t.dLogSize += int64(len(dlog))
	t.cLogSize += int64(len(clog))
	return n0 + uint64(m), root, nil
}
