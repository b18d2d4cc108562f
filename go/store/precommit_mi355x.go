//go:build mi355x

// The MI355X build's batch entry points for embedded/store: the hashing of
// precommit / preCommitWith for many transactions at once
// (immustore.go:1620-1632, 2301-2313, with ReplicateTx's Eh check
// :1649-1654), readValueAt's integrity check over many values (:3235) and
// the read-path re-hash of a run of tx-log records (tx.go:388-630), each
// split over every GPU of the process (the mh_multi_* forms: one part per
// device over its own PCIe link), each call on a clique checked out of the
// process's pool (mi355x.AcquireClique), so concurrent committers run in
// parallel.  Single
// small transactions keep the reference's CPU path (a 16 KiB transaction is
// 10 us on one SHA-NI core against ~300 us through the device queue,
// DESIGN.md section 5).  Uncompiled in the build image (no Go toolchain); see
// go/README.md.
package store

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/immustore_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/immustore_amd -limmustore_merkle -Wl,-rpath,${SRCDIR}/../../third_party/immustore_amd
#include <stdlib.h>
#include "immustore_merkle.h"
*/
import "C"

import (
	"crypto/sha256"
	"fmt"
	"unsafe"

	"github.com/codenotary/immudb/embedded/internal/mi355x"
)

func mapErr(st C.int) error {
	switch st {
	case C.MH_OK:
		return nil
	case C.MH_ERR_ILLEGAL_ARGUMENTS:
		return ErrIllegalArguments
	case C.MH_ERR_METADATA_UNSUPPORTED:
		return ErrMetadataUnsupported // tx.go:692
	case C.MH_ERR_CORRUPTED_DATA:
		return ErrCorruptedData // immustore.go:77
	case C.MH_ERR_CORRUPTED_MAX_ENTRIES:
		return ErrCorruptedTxDataMaxTxEntriesExceeded
	case C.MH_ERR_CORRUPTED_MAX_KEYLEN:
		return ErrCorruptedTxDataMaxKeyLenExceeded
	case C.MH_ERR_CORRUPTED_UNKNOWN_VERSION:
		return ErrCorruptedTxDataUnknownHeaderVersion
	}
	return mi355x.Status(int(st))
}

// packed is a batch of EntrySpecs flattened into one pinned arena: keys,
// KV metadata (KVMetadata.Bytes(), kv_metadata.go:207-219) and values back to
// back with CSR offsets, the IsValueTruncated overrides beside them.
type packed struct {
	arena                  mi355x.Arena
	keyOff, mdOff, valOff  []uint64
	txOff                  []uint64
	hvOverride             [][sha256.Size]byte
	useOverride            []uint8
	keys, md, vals         uintptr // byte offsets of the three areas in the arena
}

func (p *packed) pack(txs [][]*EntrySpec) error {
	var kb, mb, vb int
	ne := 0
	for _, es := range txs {
		for _, e := range es {
			kb += len(e.Key)
			vb += len(e.Value)
			if e.Metadata != nil {
				mb += len(e.Metadata.Bytes())
			}
			ne++
		}
	}
	if err := p.arena.Ensure(kb + mb + vb + 64); err != nil {
		return err
	}
	buf := p.arena.Bytes()
	p.keys, p.md, p.vals = 0, uintptr(kb), uintptr(kb+mb)
	p.keyOff = make([]uint64, ne+1)
	p.mdOff = make([]uint64, ne+1)
	p.valOff = make([]uint64, ne+1)
	p.txOff = make([]uint64, len(txs)+1)
	p.hvOverride = make([][sha256.Size]byte, ne)
	p.useOverride = make([]uint8, ne)
	k, m, v, i := 0, kb, kb+mb, 0
	for t, es := range txs {
		for _, e := range es {
			p.keyOff[i], p.mdOff[i], p.valOff[i] = uint64(k), uint64(m), uint64(v)
			k += copy(buf[k:], e.Key)
			if e.Metadata != nil {
				m += copy(buf[m:], e.Metadata.Bytes())
			}
			v += copy(buf[v:], e.Value)
			if e.IsValueTruncated { // immustore.go:1624-1626
				p.hvOverride[i], p.useOverride[i] = e.HashValue, 1
			}
			i++
		}
		p.txOff[t+1] = uint64(i)
	}
	p.keyOff[ne], p.mdOff[ne], p.valOff[ne] = uint64(k), uint64(m), uint64(v)
	return nil
}

// PrecommitBatch hashes many transactions as precommit does one
// (immustore.go:1620-1632): hVal of every value (or its HashValue when
// truncated), the entry digests of the header version and one htree per
// transaction -> Eh.  expectEh (nil, or one per tx) is ReplicateTx's check
// (immustore.go:1649-1654): a mismatch is ErrIllegalArguments for that tx.
// The batch runs over every GPU (mh_multi_precommit_batch: whole
// transactions, parts of nearly equal value bytes, each device with its own
// commit pipe) on a clique checked out for the call: each concurrent
// committer holds its own (INTEGRATION.md, "concurrent committers").
type PrecommitBatch struct {
	p packed
}

func NewPrecommitBatch() (*PrecommitBatch, error) {
	return &PrecommitBatch{}, nil
}

func (b *PrecommitBatch) Close() {
	b.p.arena.Free()
}

func (b *PrecommitBatch) Run(version int, maxTxEntries int, txs [][]*EntrySpec,
	expectEh [][sha256.Size]byte) (hvals [][sha256.Size]byte, eh [][sha256.Size]byte, errs []error, err error) {
	if err := b.p.pack(txs); err != nil {
		return nil, nil, nil, err
	}
	ntx, ne := len(txs), len(b.p.useOverride)
	hvals = make([][sha256.Size]byte, ne+1)
	eh = make([][sha256.Size]byte, ntx+1)
	status := make([]int32, ntx+1)
	base := b.p.arena.Ptr()
	var exp *C.uint8_t
	if expectEh != nil {
		exp = (*C.uint8_t)(unsafe.Pointer(&expectEh[0][0]))
	}
	hv := make([][sha256.Size]byte, ne+1)
	copy(hv, b.p.hvOverride)
	use := append(b.p.useOverride, 0)
	mm, err := mi355x.AcquireClique()
	if err != nil {
		return nil, nil, nil, err
	}
	st := C.mh_multi_precommit_batch((*C.mh_multi)(mm), C.int(version), C.uint64_t(maxTxEntries), C.uint64_t(ntx),
		(*C.uint64_t)(unsafe.Pointer(&b.p.txOff[0])),
		(*C.uint8_t)(unsafe.Add(base, b.p.keys)), (*C.uint64_t)(unsafe.Pointer(&b.p.keyOff[0])),
		(*C.uint8_t)(unsafe.Add(base, b.p.md)), (*C.uint64_t)(unsafe.Pointer(&b.p.mdOff[0])),
		(*C.uint8_t)(unsafe.Add(base, b.p.vals)), (*C.uint64_t)(unsafe.Pointer(&b.p.valOff[0])),
		(*C.uint8_t)(unsafe.Pointer(&hv[0][0])), (*C.uint8_t)(unsafe.Pointer(&use[0])), exp,
		(*C.uint8_t)(unsafe.Pointer(&hvals[0][0])), (*C.uint8_t)(unsafe.Pointer(&eh[0][0])),
		(*C.int32_t)(unsafe.Pointer(&status[0])))
	mi355x.ReleaseClique(mm, int(st))
	if st != C.MH_OK {
		return nil, nil, nil, mapErr(st)
	}
	errs = make([]error, ntx)
	for t := 0; t < ntx; t++ {
		switch status[t] {
		case 0:
		case int32(C.MH_ERR_ILLEGAL_ARGUMENTS):
			errs[t] = fmt.Errorf("%w: entries hash (Eh) differs", ErrIllegalArguments)
		default:
			errs[t] = mapErr(C.int(status[t]))
		}
	}
	return hvals[:ne], eh[:ntx], errs, nil
}

// VerifyValues is readValueAt's integrity check (immustore.go:3235) over a
// batch: vals[i] are the bytes read for entry i, vLen[i] its stored length,
// hVal[i] its stored digest; errs[i] is ErrCorruptedData ("value length or
// digest mismatch") or nil.  For a scrub or an export of many values.
func VerifyValues(vals [][]byte, vLen []int, hVal [][sha256.Size]byte) ([]error, error) {
	n := len(vals)
	// one length and one digest per value: C reads n of each
	if len(vLen) != n || len(hVal) != n {
		return nil, ErrIllegalArguments
	}
	if n == 0 {
		return nil, nil
	}
	m, err := mi355x.AcquireClique()
	if err != nil {
		return nil, err
	}
	var arena mi355x.Arena
	defer arena.Free()
	total := 0
	for _, v := range vals {
		total += len(v)
	}
	if err := arena.Ensure(total + 16); err != nil {
		mi355x.ReleaseClique(m, 0)
		return nil, err
	}
	buf := arena.Bytes()
	off := make([]uint64, n+1)
	lens := make([]uint64, n)
	for i, v := range vals {
		off[i+1] = off[i] + uint64(copy(buf[off[i]:], v))
		lens[i] = uint64(vLen[i])
	}
	status := make([]int32, n)
	var bad C.uint64_t
	// parts of nearly equal value bytes, one per GPU (mh_multi_verify_values_batch)
	st := C.mh_multi_verify_values_batch((*C.mh_multi)(m), C.uint64_t(n), (*C.uint8_t)(arena.Ptr()),
		(*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint64_t)(unsafe.Pointer(&lens[0])),
		(*C.uint8_t)(unsafe.Pointer(&hVal[0][0])), (*C.int32_t)(unsafe.Pointer(&status[0])), &bad)
	mi355x.ReleaseClique(m, int(st))
	if st != C.MH_OK {
		return nil, mapErr(st)
	}
	errs := make([]error, n)
	if bad > 0 {
		for i, s := range status {
			if s != 0 {
				errs[i] = fmt.Errorf("%w: value length or digest mismatch", ErrCorruptedData)
			}
		}
	}
	return errs, nil
}

// ValidateTxLog re-hashes a run of tx-log records as Tx.readFrom +
// buildAndValidateHtree do one (tx.go:388-630): per record the entry
// digests, the htree, innerHash and Alh, compared with the stored Alh.  buf
// should be a pinned arena for throughput (one DMA under the host record
// hop).  Returns the Alh of every record and a per-record error
// (ErrCorruptedData on an ALH mismatch); err is the structural error of the
// record at consumed.
func ValidateTxLog(buf []byte, maxEntries, maxKeyLen, maxTxs int) (alhs [][sha256.Size]byte,
	errs []error, consumed uint64, err error) {
	m, e := mi355x.AcquireClique()
	if e != nil {
		return nil, nil, 0, e
	}
	alhs = make([][sha256.Size]byte, maxTxs+1)
	status := make([]int32, maxTxs+1)
	var ntx, used C.uint64_t
	var p *C.uint8_t
	if len(buf) > 0 {
		p = (*C.uint8_t)(unsafe.Pointer(&buf[0]))
	}
	// the records cut at record boundaries into one part per GPU, each copied
	// and validated over its own link (mh_multi_txlog_validate)
	st := C.mh_multi_txlog_validate((*C.mh_multi)(m), p, C.uint64_t(len(buf)), C.uint32_t(maxEntries),
		C.uint32_t(maxKeyLen), C.uint64_t(maxTxs), &ntx, &used, nil,
		(*C.uint8_t)(unsafe.Pointer(&alhs[0][0])), (*C.int32_t)(unsafe.Pointer(&status[0])))
	mi355x.ReleaseClique(m, int(st))
	errs = make([]error, int(ntx))
	for k := range errs {
		if status[k] != 0 {
			errs[k] = fmt.Errorf("%w: ALH mismatch", ErrCorruptedData) // tx.go:625
		}
	}
	return alhs[:ntx], errs, uint64(used), mapErr(st)
}

// ValidateTxLogFromCommitLog is ImmuStore.readTx (immustore.go:3048-3060) for
// txs 1..n located by the store's commit log, as txOffsetAndSize reads it
// (:2569-2597): cLog holds n entries of cLogEntrySize bytes (12: BE64 offset
// || BE32 size; 44: + the tx's Alh, :122-123), txLog the tx log's data.  No
// host record hop: the device checks every record's structure where its
// entry points (plus the open path's cLog checks, :458-528), then re-hashes
// it (tx.go:388-630).  txLog may be a pinned arena or any slice (copied up in
// chunks, each checked as it lands; as fast as ValidateTxLog from either,
// with no host record parse, DESIGN.md).  Returns the Alh of every tx (zero where
// the record is bad), a per-tx error (ErrCorruptedData for an ALH mismatch or
// a cLog entry that disagrees with its record, ErrCorruptedTxData for a read
// past the log, readHeader / readEntry's errors otherwise) and the index of
// the first bad tx (n when none).
func ValidateTxLogFromCommitLog(txLog, cLog []byte, cLogEntrySize, maxEntries, maxKeyLen int) (
	alhs [][sha256.Size]byte, errs []error, firstBad int, err error) {
	if cLogEntrySize != 12 && cLogEntrySize != 44 {
		return nil, nil, 0, ErrIllegalArguments
	}
	n := len(cLog) / cLogEntrySize
	if n == 0 {
		return nil, nil, 0, nil
	}
	if len(txLog) == 0 {
		return nil, nil, 0, ErrIllegalArguments
	}
	m, e := mi355x.AcquireClique()
	if e != nil {
		return nil, nil, 0, e
	}
	alhs = make([][sha256.Size]byte, n)
	status := make([]int32, n)
	var nbad, first C.uint64_t
	// one device: the call copies and checks the whole log on it (device 0 of
	// the clique)
	st := C.mh_txlog_validate_clog(C.mh_multi_ctx((*C.mh_multi)(m), 0),
		(*C.uint8_t)(unsafe.Pointer(&txLog[0])), C.uint64_t(len(txLog)),
		(*C.uint8_t)(unsafe.Pointer(&cLog[0])), C.uint64_t(n), C.uint32_t(cLogEntrySize),
		C.uint32_t(maxEntries), C.uint32_t(maxKeyLen), nil,
		(*C.uint8_t)(unsafe.Pointer(&alhs[0][0])), (*C.int32_t)(unsafe.Pointer(&status[0])),
		&nbad, &first)
	mi355x.ReleaseClique(m, int(st))
	if st != C.MH_OK {
		return nil, nil, 0, mapErr(st)
	}
	errs = make([]error, n)
	for k := range errs {
		switch status[k] {
		case 0:
		case C.MH_ERR_CORRUPTED_DATA:
			errs[k] = fmt.Errorf("%w: ALH mismatch or commit-log entry disagrees", ErrCorruptedData)
		case C.MH_ERR_TRUNCATED:
			// readTx's io.EOF (immustore.go:3054-3056)
			errs[k] = fmt.Errorf("%w: unexpected EOF while reading tx %d", ErrCorruptedTxData, k+1)
		default:
			errs[k] = mapErr(C.int(status[k]))
		}
	}
	return alhs, errs, int(first), nil
}
