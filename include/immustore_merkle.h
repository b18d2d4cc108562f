/*
 * immustore_merkle.h -- C ABI of the MI355X Merkle-hash engine for immudb.
 *
 * Drop-in boundary for ONE hot path of codenotary/immudb: the per-transaction
 * binary hash tree (embedded/htree), the entry hashing that feeds it
 * (value hash + TxEntryDigest + leaf hash), the cross-transaction append-only
 * tree (embedded/ahtree) and the proof re-hash of both.  The reference is Go;
 * it has no FFI for this path, so the replacement is a cgo shim that keeps the
 * Go signatures and forwards here (see INTEGRATION.md for the shim).
 *
 * Conventions (inherited from the Go reference):
 *  - every function returns an int status: MH_OK, a positive MH_ERR_* that
 *    mirrors one of the Go sentinel errors, or a negative HIP runtime error
 *    (-hipError_t).  Nothing aborts, throws or exits across this ABI.
 *  - digests are 32 raw bytes (Go [sha256.Size]byte); "levels" is the flat
 *    level-major copy of Go's HTree.levels: level l holds ceil(n/2^l) nodes
 *    (including the promoted odd node) starting at node mh_htree_level_offset.
 *  - mh_htree handles are not synchronised (like Go's HTree, one per pooled
 *    Tx, tx.go:70); use one per goroutine.  mh_ahtree handles ARE
 *    synchronised like Go's AHtree (t.mutex, ahtree.go:60-84): every
 *    mh_ahtree_* call holds the handle's lock, so readers (root, proofs,
 *    dLog reads) may run concurrently with appends.  A device pointer from
 *    mh_ahtree_dlog_device is valid only until the next append that grows
 *    the dLog.  An mh_ctx may be shared by many handles, and
 *    calls on different handles of one context may run concurrently from
 *    different threads (the context's scratch is locked and used on its own
 *    stream only).
 *  - mh_dev_* functions take DEVICE pointers, are asynchronous on the
 *    context's stream and never allocate; all other functions take HOST
 *    pointers and return after the result is in host memory.
 */
#ifndef IMMUSTORE_MERKLE_H
#define IMMUSTORE_MERKLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
/* the library is built with hidden visibility: only these entry points are
 * exported */
#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility push(default)
#endif

#define MH_ABI_VERSION 1

/* status codes */
#define MH_OK 0
#define MH_ERR_MAX_WIDTH_EXCEEDED 1  /* htree.ErrMaxWidthExceeded   htree.go:25 */
#define MH_ERR_ILLEGAL_ARGUMENTS 2   /* htree/ahtree.ErrIllegalArguments htree.go:26, ahtree.go:35 */
#define MH_ERR_ILLEGAL_STATE 3       /* htree.ErrIllegalState       htree.go:27 */
#define MH_ERR_EMPTY_TREE 4          /* ahtree.ErrEmptyTree         ahtree.go:42 */
#define MH_ERR_UNEXISTENT_DATA 5     /* ahtree.ErrUnexistentData    ahtree.go:44 */
#define MH_ERR_METADATA_UNSUPPORTED 6 /* store.ErrMetadataUnsupported tx.go:692 */
#define MH_ERR_CANNOT_RESET_TO_LARGER 7 /* ahtree.ErrCannotResetToLargerSize ahtree.go:45 */
#define MH_ERR_NO_DEVICE 8           /* no usable gfx950 device / library not initialised */
#define MH_ERR_OUT_OF_MEMORY 9
/* transaction layer (embedded/store) */
#define MH_ERR_SOURCE_TX_NEWER 10       /* store.ErrSourceTxNewerThanTargetTx immustore.go:101 */
#define MH_ERR_UNEXPECTED_LINKING 11    /* store.ErrUnexpectedLinkingError immustore.go:53 */
#define MH_ERR_INCLUSION_NOT_VALID 12   /* "inclusion proof does NOT validate" verification.go:349 */
#define MH_ERR_CONSISTENCY_NOT_VALID 13 /* "consistency proof does NOT validate" verification.go:368 */
#define MH_ERR_CORRUPTED_DATA 14        /* store.ErrCorruptedData immustore.go:77 (ALH mismatch, tx.go:625) */
#define MH_ERR_CORRUPTED_MAX_ENTRIES 15 /* ErrCorruptedTxDataMaxTxEntriesExceeded immustore.go:72 */
#define MH_ERR_CORRUPTED_MAX_KEYLEN 16  /* ErrCorruptedTxDataMaxKeyLenExceeded immustore.go:75 */
#define MH_ERR_CORRUPTED_UNKNOWN_VERSION 17 /* ErrCorruptedTxDataUnknownHeaderVersion immustore.go:74 */
#define MH_ERR_TRUNCATED 18             /* record cut short (io.ErrUnexpectedEOF from the reader) */
#define MH_ERR_BUFFER_TOO_SMALL 19      /* output capacity below the encoded size (wire formats) */
#define MH_ERR_INVALID_PROOF 20         /* store.ErrInvalidProof immustore.go:114 */
#define MH_ERR_UNSUPPORTED_TX_VERSION 21 /* store.ErrUnsupportedTxVersion immustore.go:90 */
#define MH_ERR_INVALID_PROOF_ENTRY 22   /* store.ErrInvalidProof from VerifyDocument's entry /
                                           hash-value check (pkg/verification/verification.go:60-76),
                                           i.e. raised BEFORE the document decode (:78-110) */
#define MH_ERR_COLLECTIVE 23            /* RCCL unavailable or a collective failed (mh_multi_*) */

#define MH_MAX_TX_METADATA_LEN 268 /* maxTxMetadataLen tx_metadata.go:36-39 */
#define MH_MAX_KV_METADATA_LEN 11  /* maxKVMetadataLen kv_metadata.go:41-43 */

/* ahtree verification kinds (embedded/ahtree/verification.go) */
#define MH_AHT_INCLUSION 0      /* VerifyInclusion      verification.go:21 */
#define MH_AHT_CONSISTENCY 1    /* VerifyConsistency    verification.go:58 */
#define MH_AHT_LAST_INCLUSION 2 /* VerifyLastInclusion  verification.go:111 */

typedef struct mh_ctx mh_ctx;

/* TxHeader (embedded/store/tx.go:103-117) as a plain C struct.  md_len bytes of
 * TxMetadata.Bytes() (version 1 only) live at md_blob + md_off, md_blob being
 * the buffer passed next to the headers.  136 bytes, 8-byte aligned. */
typedef struct mh_tx_header {
    uint64_t id;
    int64_t ts;
    uint64_t bl_tx_id;
    uint8_t bl_root[32];
    uint8_t prev_alh[32];
    uint8_t eh[32];
    uint32_t version; /* 0 or 1 (TxHeader.Version) */
    uint32_t nentries;
    uint32_t md_len;
    uint32_t md_off;
} mh_tx_header;
typedef struct mh_htree mh_htree;
typedef struct mh_ahtree mh_ahtree;

int mh_abi_version(void);
const char *mh_status_string(int status);
int mh_device_count(int *count);

/* ---------------------------------------------------------------- context */
/* device_ordinal: HIP device; hip_stream: an existing hipStream_t to run on,
 * or NULL to create a private non-blocking stream. */
int mh_ctx_create(int device_ordinal, void *hip_stream, mh_ctx **out);
int mh_ctx_destroy(mh_ctx *ctx);
int mh_ctx_synchronize(mh_ctx *ctx);
void *mh_ctx_stream(mh_ctx *ctx);
/* Per-kernel timing with HIP events recorded around every launch on the
 * stream it runs on.  mh_ctx_timing synchronises and reports the total
 * milliseconds and launch count of kernels whose name starts with `prefix`. */
int mh_ctx_set_timing(mh_ctx *ctx, int enable);
int mh_ctx_timing(mh_ctx *ctx, const char *prefix, double *total_ms, uint64_t *launches);
int mh_ctx_timing_reset(mh_ctx *ctx);

/* TEST ONLY: fault injection for error-path tests.  The next `countdown`-th
 * time (1 = the next time) the library passes fault site `site`, it fails
 * there as if the HIP / RCCL call at that point had failed.  countdown 0
 * disarms the site.  Sites: MH_FAULT_RCCL_GROUP (inside the RCCL group of a
 * multi-device all-gather, after ncclGroupStart), MH_FAULT_TXLOG_AFTER_GROUP
 * (mh_txlog_validate, after the first chunk group's kernels were queued),
 * MH_FAULT_RCCL_GROUP_LATE (the same all-gather after every device's
 * collective was queued: the clique is aborted and the handle refuses every
 * later collective).  No reference counterpart: production callers never arm
 * it. */
#define MH_FAULT_RCCL_GROUP 1
#define MH_FAULT_TXLOG_AFTER_GROUP 2
#define MH_FAULT_RCCL_GROUP_LATE 3
int mh_debug_fail_at(int site, int countdown);

/* device memory helpers, so that a cgo caller needs no HIP headers */
int mh_dev_alloc(mh_ctx *ctx, uint64_t bytes, void **dptr);
int mh_dev_free(mh_ctx *ctx, void *dptr);
int mh_host_alloc_pinned(uint64_t bytes, void **hptr); /* pinned staging arena */
int mh_host_free_pinned(void *hptr);
int mh_memcpy_h2d(mh_ctx *ctx, void *dst, const void *src, uint64_t bytes); /* async */
int mh_memcpy_d2h(mh_ctx *ctx, void *dst, const void *src, uint64_t bytes); /* async */
/* deterministic synthetic data: splitmix64 words, word w = mix(seed + (w+1)*gamma) */
int mh_dev_fill_random(mh_ctx *ctx, void *dptr, uint64_t nbytes, uint64_t seed);
/* keys[i] = BE64(first + i)  (immustore_test.go:1844-1849 key shape) */
int mh_dev_fill_keys_be64(mh_ctx *ctx, void *dptr, uint64_t n, uint64_t first);

/* ------------------------------------------------------------------ htree */
/* Flat level layout (htree.go:45-66 capacity, :85-110 used widths). */
uint64_t mh_htree_levels_len(uint64_t n);
uint64_t mh_htree_level_offset(uint64_t n, int level);

/* htree.New(maxWidth)                                 htree.go:45-66 */
int mh_htree_new(mh_ctx *ctx, uint64_t max_width, mh_htree **out);
int mh_htree_free(mh_htree *t);
/* (*HTree).BuildWith(digests)                         htree.go:68-113 */
int mh_htree_build_with(mh_htree *t, const uint8_t *digests, uint64_t n);
/* value hash loop immustore.go:1620-1630 + Tx.BuildHashTree tx.go:332-355:
 * version 0 -> TxEntryDigest_v1_1, 1 -> TxEntryDigest_v1_2 (tx.go:321-330).
 * CSR inputs: *_off arrays have n+1 entries; md/md_off may be NULL (no KV
 * metadata); hval_override (n*32) + use_override (n bytes) model
 * EntrySpec.IsValueTruncated (may be NULL); hvals_out (n*32) may be NULL. */
int mh_htree_build_entries(mh_htree *t, int version, uint64_t n, const uint8_t *keys,
                           const uint64_t *key_off, const uint8_t *md, const uint64_t *md_off,
                           const uint8_t *vals, const uint64_t *val_off,
                           const uint8_t *hval_override, const uint8_t *use_override,
                           uint8_t *hvals_out);
/* (*HTree).Root()                                      htree.go:115-117 */
int mh_htree_root(mh_htree *t, uint8_t root[32]);
int mh_htree_width(mh_htree *t, uint64_t *width);
/* (*HTree).InclusionProof(i): terms leaf-side first   htree.go:121-164 */
int mh_htree_inclusion_proof(mh_htree *t, uint64_t i, uint8_t *terms, uint32_t cap,
                             uint32_t *nterms);
/* copy of the used levels (mh_htree_levels_len(width) nodes) */
int mh_htree_levels(mh_htree *t, uint8_t *out, uint64_t cap_nodes);
/* Many (*HTree).InclusionProof calls at once (htree.go:121-164), generated on
 * the device from the tree's resident levels: proof p (leaf[p]) gets nterms[p]
 * terms at terms + p * max_terms * 32, Go order (leaf side first);
 * status[p] = MH_OK or MH_ERR_ILLEGAL_ARGUMENTS (leaf >= width, or more than
 * max_terms terms; ceil(log2 width) always suffices). */
int mh_htree_inclusion_proof_batch(mh_htree *t, uint64_t n, const uint64_t *leaf, uint8_t *terms,
                                   uint32_t max_terms, uint32_t *nterms, int32_t *status);
/* device pointer of the handle's level buffer (device-resident consumers) */
int mh_htree_levels_device(mh_htree *t, const uint8_t **dptr);

/* htree.VerifyInclusion batch (htree.go:166-195; store.VerifyInclusion
 * verification.go:28-30).  Proof p has terms [term_off[p], term_off[p+1]).
 * leaf / width are the bits of Go ints (values >= 2^63 are negative and take
 * Go's signed % and /).  ok[p] = 1 if it verifies.  Host pointers. */
int mh_htree_verify_inclusion_batch(mh_ctx *ctx, uint64_t nproofs, const uint64_t *leaf,
                                    const uint64_t *width, const uint64_t *term_off,
                                    const uint8_t *terms, const uint8_t *digests,
                                    const uint8_t *roots, uint8_t *ok);

/* ------------------------------------------------- htree, device-resident */
/* BuildWith over device digests. levels: mh_htree_levels_len(n)*32 bytes. */
int mh_dev_htree_build_digests(mh_ctx *ctx, const uint8_t *digests, uint64_t n, uint8_t *levels,
                               uint8_t *root);
/* Fused value hash + entry digest + leaf + all levels for fixed-stride
 * entries without KV metadata (BASELINE configs C1/C2/C4): key i at
 * keys + i*key_len, value i at vals + i*val_len. */
int mh_dev_htree_build_entries_fixed(mh_ctx *ctx, int version, uint64_t n, const uint8_t *keys,
                                     uint32_t key_len, const uint8_t *vals, uint32_t val_len,
                                     uint8_t *hvals_out, uint8_t *levels, uint8_t *root);
/* General CSR variant (device arrays); scratch is allocated by the context. */
int mh_dev_htree_build_entries(mh_ctx *ctx, int version, uint64_t n, const uint8_t *keys,
                               const uint64_t *key_off, const uint8_t *md, const uint64_t *md_off,
                               const uint8_t *vals, const uint64_t *val_off,
                               const uint8_t *hval_override, const uint8_t *use_override,
                               uint8_t *hvals_out, uint8_t *levels, uint8_t *root);
/* Reduce w given nodes (e.g. all-gathered per-GPU subtree roots) to a root
 * with htree's pairing rule; nodes are copied to level 0 of `levels`
 * (mh_htree_levels_len(w)*32 bytes) without leaf hashing. */
int mh_dev_htree_reduce_nodes(mh_ctx *ctx, const uint8_t *nodes, uint64_t w, uint8_t *levels,
                              uint8_t *root);
/* SHA-256 of n byte ranges buf[off[i], off[i+1]) -> out (n*32). */
int mh_dev_sha256_batch(mh_ctx *ctx, const uint8_t *buf, const uint64_t *off, uint64_t n,
                        uint8_t *out);
/* The read-side value integrity check of ImmuStore.readValueAt
 * (embedded/store/immustore.go:3183-3240, the check at :3235) over a batch:
 * value i is vals[off[i], off[i+1]) -- the n_i bytes the vLog or the value
 * cache returned for a buffer of the entry's stored length vlen[i] -- and
 * status[i] = MH_OK, or MH_ERR_CORRUPTED_DATA when n_i != vlen[i] or
 * SHA256(value) != hvals[i] (32 bytes per entry), exactly as Go rejects it
 * ("value length or digest mismatch").  vlen may be NULL (lengths not
 * checked).  Host variant: host memory in and out, synchronous; the value
 * bytes go up in ~64 MiB chunks on a copy stream while the previous chunk is
 * checked; *ncorrupted (may be NULL) = entries not MH_OK.  Device variant:
 * every pointer device memory, asynchronous on the context stream. */
int mh_verify_values_batch(mh_ctx *ctx, uint64_t n, const uint8_t *vals, const uint64_t *off,
                           const uint64_t *vlen, const uint8_t *hvals, int32_t *status,
                           uint64_t *ncorrupted);
int mh_dev_verify_values_batch(mh_ctx *ctx, uint64_t n, const uint8_t *vals, const uint64_t *off,
                               const uint64_t *vlen, const uint8_t *hvals, int32_t *status);
/* Device variants of the batch proof generators: every pointer is device
 * memory (levels of a tree of `width` leaves / a dLog of `size` appends). */
int mh_dev_htree_inclusion_proof_batch(mh_ctx *ctx, const uint8_t *levels, uint64_t width,
                                       uint64_t n, const uint64_t *leaf, uint8_t *terms,
                                       uint32_t max_terms, uint32_t *nterms, int32_t *status);
int mh_dev_ahtree_proof_batch(mh_ctx *ctx, int kind, const uint8_t *dlog, uint64_t size,
                              uint64_t n, const uint64_t *i, const uint64_t *j, uint8_t *terms,
                              uint32_t max_terms, uint32_t *nterms, int32_t *status);
int mh_dev_htree_verify_inclusion_batch(mh_ctx *ctx, uint64_t nproofs, const uint64_t *leaf,
                                        const uint64_t *width, const uint64_t *term_off,
                                        const uint8_t *terms, const uint8_t *digests,
                                        const uint8_t *roots, uint8_t *ok);

/* ----------------------------------------------------------------- ahtree */
/* In-memory append-only tree whose dLog (ahtree.go:60-84, tree/NNNNNNNN.sha) lives
 * in HBM.  No pLog/cLog files: persistence stays with the Go appendables, which
 * mh_ahtree_append_batch_logs feeds with ready-made record streams. */
int mh_ahtree_new(mh_ctx *ctx, mh_ahtree **out);
int mh_ahtree_free(mh_ahtree *t);
/* (*AHtree).Append(d)                                   ahtree.go:246-373 */
int mh_ahtree_append(mh_ahtree *t, const uint8_t *payload, uint64_t plen, uint64_t *n,
                     uint8_t h[32]);
/* m fixed-size payloads appended in order (syncBinaryLinking batch,
 * immustore.go:1198-1232). roots_out (m*32, RootAt(n0+1..n0+m)) may be NULL. */
int mh_ahtree_append_batch(mh_ahtree *t, const uint8_t *payloads, uint64_t m, uint32_t plen,
                           uint8_t *roots_out);
/* mh_ahtree_append_batch that also returns the batch's appendable records
 * (SURVEY.md 8(f) row 4), ready for the Go appendables' Append calls of
 * (*AHtree).Append: plog_out (m*(4+plen) bytes, the data/NNNNNNNN.dat
 * stream: BE32 plen || payload per append, ahtree.go:266-282) and clog_out
 * (m*12 bytes, the commit/NNNNNNNN.di stream: BE64 pLog offset || BE32 plen,
 * ahtree.go:341-351); p_off0 = the pLog size before the batch (t.pLogSize).
 * The dLog bytes of the batch are mh_ahtree_dlog(nodes_upto(n0),
 * nodes_upto(n0+m) - nodes_upto(n0)).  Either output may be NULL. */
int mh_ahtree_append_batch_logs(mh_ahtree *t, const uint8_t *payloads, uint64_t m, uint32_t plen,
                                uint64_t p_off0, uint8_t *plog_out, uint8_t *clog_out,
                                uint8_t *roots_out);
int mh_ahtree_size(mh_ahtree *t, uint64_t *size);
/* (*AHtree).Root / RootAt                                ahtree.go:727-771 */
int mh_ahtree_root(mh_ahtree *t, uint64_t *n, uint8_t root[32]);
int mh_ahtree_root_at(mh_ahtree *t, uint64_t n, uint8_t root[32]);
/* (*AHtree).InclusionProof / ConsistencyProof            ahtree.go:525-651 */
int mh_ahtree_inclusion_proof(mh_ahtree *t, uint64_t i, uint64_t j, uint8_t *terms, uint32_t cap,
                              uint32_t *nterms);
int mh_ahtree_consistency_proof(mh_ahtree *t, uint64_t i, uint64_t j, uint8_t *terms,
                                uint32_t cap, uint32_t *nterms);
/* (*AHtree).ResetSize                                     ahtree.go:375-458 */
/* Many (*AHtree).InclusionProof (kind MH_AHT_INCLUSION, ahtree.go:525-577) or
 * ConsistencyProof (MH_AHT_CONSISTENCY, :579-651) calls at once, generated on
 * the device from the resident dLog; layout as mh_htree_inclusion_proof_batch;
 * status[p]: MH_OK, MH_ERR_ILLEGAL_ARGUMENTS (i > j, or > max_terms terms),
 * MH_ERR_UNEXISTENT_DATA (j > size or j == 0).  128 terms always suffice. */
int mh_ahtree_proof_batch(mh_ahtree *t, int kind, uint64_t n, const uint64_t *i,
                          const uint64_t *j, uint8_t *terms, uint32_t max_terms, uint32_t *nterms,
                          int32_t *status);
int mh_ahtree_reset_size(mh_ahtree *t, uint64_t new_size);
/* copy dLog digests [first, first+count) (the tree/NNNNNNNN.sha byte stream) */
int mh_ahtree_dlog(mh_ahtree *t, uint64_t first, uint64_t count, uint8_t *out);
int mh_ahtree_dlog_device(mh_ahtree *t, const uint8_t **dptr);

/* Device-resident batch append: dlog holds nodesUpto(n0) digests and has
 * room for nodesUpto(n0+m); payloads m*plen bytes. */
int mh_dev_ahtree_append_batch(mh_ctx *ctx, uint8_t *dlog, uint64_t n0, const uint8_t *payloads,
                               uint64_t m, uint32_t plen, uint8_t *roots_out);
/* Device variants of the appendable records: fused into the append's leaf
 * phase (the payload is read once), or alone (e.g. per rank of a sharded
 * append: rank r passes p_off0 + r*S*(4+plen)).  plog / clog: device memory
 * of m*(4+plen) / m*12 bytes, either may be NULL. */
int mh_dev_ahtree_append_batch_logs(mh_ctx *ctx, uint8_t *dlog, uint64_t n0,
                                    const uint8_t *payloads, uint64_t m, uint32_t plen,
                                    uint64_t p_off0, uint8_t *plog, uint8_t *clog,
                                    uint8_t *roots_out);
int mh_dev_ahtree_log_records(mh_ctx *ctx, const uint8_t *payloads, uint64_t m, uint32_t plen,
                              uint64_t p_off0, uint8_t *plog, uint8_t *clog);
uint64_t mh_ahtree_nodes_upto(uint64_t n); /* ahtree.go:492-511 */
/* The appendable framing around those streams, host
 * code.  An ahtree's data/ tree/ commit/ logs are multiapps
 * (ahtree.go:106-140): file id holds logical bytes [id*file_size,
 * (id+1)*file_size) (multi_app.go:208-214, named "%08d.<dat|sha|di>") behind
 * a singleapp header BE32 len(m) || m (single_app.go:116-171), m =
 * appendable.Metadata.Bytes() (metadata.go:33-80) of { COMPRESSION_FORMAT,
 * COMPRESSION_LEVEL, PREALLOC_SIZE (omitted when prealloc_size < 0, as in
 * files written before it existed), WRAPPED_METADATA = { FILE_SIZE,
 * WRAPPED_METADATA = { VERSION: 1 } } }; Go writes each level's entries in
 * map order, any order reads back the same -- here in the order shown.
 * *len = the header size; MH_ERR_BUFFER_TOO_SMALL when out is NULL or cap is
 * below it. */
int mh_ahtree_log_header(uint64_t file_size, int64_t prealloc_size, int32_t compression_format,
                         int32_t compression_level, uint8_t *out, uint64_t cap, uint64_t *len);
/* appendable.Metadata.Bytes() of n (key, value) pairs in the given order. */
int mh_appendable_metadata(uint32_t n, const char *const *keys, const uint8_t *const *vals,
                           const uint64_t *val_len, uint8_t *out, uint64_t cap, uint64_t *len);
/* Logical log bytes [off, off+n) split at file boundaries: segment k =
 * seg[4k .. 4k+3] = (file id, byte position in that file = header_len + off
 * within the file, offset in the source range, length).  *nseg = the count
 * (seg may be NULL to ask for it); MH_ERR_BUFFER_TOO_SMALL if cap < *nseg. */
int mh_multiapp_segments(uint64_t off, uint64_t n, uint64_t file_size, uint64_t header_len,
                         uint64_t *seg, uint32_t cap, uint32_t *nseg);

/* dLog index of node(n, level) = nodesUntil(n) + level (ahtree.go:460-462). */
uint64_t mh_ahtree_node_index(uint64_t n, int level);

/* Sharded batch append.  mh_dev_ahtree_append_batch in three
 * phases so that G ranks can append one global batch together: rank r owns
 * appends (n0 + r*S, n0 + (r+1)*S], S = 2^shard_bits, n0 a multiple of S, and
 * keeps a dLog indexed like the global one (it only fills its own range and
 * the nodes above shard level).  Every perfect node of level <= shard_bits
 * and every spine node of a rank lies inside its range except the nodes
 * above shard level, which are built from the G shard roots.
 *  1. mh_dev_ahtree_append_local: leaves + perfect nodes of levels
 *     1..shard_bits ending in (n0, n0 + m];
 *  2. all-gather the 32-byte shard roots, dLog[mh_ahtree_node_index((r+1)*S
 *     + n0, shard_bits)] of every complete shard (RCCL, 32 B per rank);
 *  3. mh_dev_ahtree_put_shard_roots (count = complete shards before the
 *     global end, roots in shard order, for a batch starting at n0 = 0) writes
 *     them and the perfect nodes above them; mh_dev_ahtree_append_spine then
 *     finishes the rank's appends.  The rank's dLog range is byte-identical to
 *     a single-device append of the whole batch. */
int mh_dev_ahtree_append_local(mh_ctx *ctx, uint8_t *dlog, uint64_t n0, const uint8_t *payloads,
                               uint64_t m, uint32_t plen, int shard_bits);
int mh_dev_ahtree_put_shard_roots(mh_ctx *ctx, uint8_t *dlog, int shard_bits, uint64_t count,
                                  const uint8_t *roots);
int mh_dev_ahtree_append_spine(mh_ctx *ctx, uint8_t *dlog, uint64_t n0, uint64_t m,
                               uint8_t *roots_out);

/* One device, the dLog kept as a RANGE (the replay of syncBinaryLinking,
 * immustore.go:1198-1232, with no copy of the old dLog on the device):
 * append m payloads onto a tree of size n0 whose peaks (as for
 * mh_multi_ahtree_append_batch, host memory, NULL when n0 == 0) are given;
 * dlog_range (device, 16-byte aligned) receives the new digests
 * [nodesUpto(n0), nodesUpto(n0 + m)) from its start, roots_out (may be NULL)
 * RootAt after each append.  Asynchronous on the context stream. */
int mh_dev_ahtree_append_range(mh_ctx *ctx, uint8_t *dlog_range, uint64_t n0,
                               const uint8_t *peaks, const uint8_t *payloads, uint64_t m,
                               uint32_t plen, uint8_t *roots_out);
/* The popcount(n) peaks of a tree of size n, lowest level first, from a
 * device dLog indexed from 0 (synchronous; peaks_out in host memory). */
int mh_dev_ahtree_peaks(mh_ctx *ctx, const uint8_t *dlog, uint64_t n, uint8_t *peaks_out);

/* ahtree proof re-hash, batch (verification.go).  kind = MH_AHT_*.
 * INCLUSION:      a = leaf (leafFor(alh)), b = root of j
 * CONSISTENCY:    a = root of i, b = root of j
 * LAST_INCLUSION: a = leaf, b = root (j ignored)
 * ok[p] = Verify*(...) ; eval_out (np*32 for INCLUSION / LAST, np*64 for
 * CONSISTENCY = ci||cj) may be NULL. */
int mh_ahtree_verify_batch(mh_ctx *ctx, int kind, uint64_t nproofs, const uint64_t *i,
                           const uint64_t *j, const uint64_t *term_off, const uint8_t *terms,
                           const uint8_t *a, const uint8_t *b, uint8_t *ok, uint8_t *eval_out);
int mh_dev_ahtree_verify_batch(mh_ctx *ctx, int kind, uint64_t nproofs, const uint64_t *i,
                               const uint64_t *j, const uint64_t *term_off, const uint8_t *terms,
                               const uint8_t *a, const uint8_t *b, uint8_t *ok,
                               uint8_t *eval_out);

/* ---------------------------------------------------------------- tx layer
 * SURVEY.md 8(a) a7 (header hashes), a13 (linear / dual proofs), a14 (tx-log
 * read-path validation) and a3 for many trees at once.  Hashing runs on the
 * device; the host side parses records and combines verdicts. */

/* TxHeader.Alh for n headers (tx.go:249-319: innerHash then
 * SHA256(BE64 id || prevAlh || innerHash)).  inner_out may be NULL.
 * Replaces per-header hdr.Alh() calls (tx.go:307, verification.go:141-150,
 * 317-325).  MH_ERR_ILLEGAL_ARGUMENTS: version not 0/1, md on a v0 header or
 * md_len > MH_MAX_TX_METADATA_LEN, md outside md_blob. */
int mh_tx_alh_batch(mh_ctx *ctx, uint64_t n, const mh_tx_header *hdrs, const uint8_t *md_blob,
                    uint64_t md_blob_len, uint8_t *inner_out, uint8_t *alh_out);
/* Device variant: hdrs / md_blob / outputs in device memory; eh (nullable,
 * n x 32) replaces hdrs[k].eh (e.g. Eh just built on the device).  scratch:
 * n * 384 bytes of device memory.  Arguments are not validated. */
int mh_dev_tx_alh_batch(mh_ctx *ctx, uint64_t n, const mh_tx_header *hdrs, const uint8_t *md_blob,
                        const uint8_t *eh, uint8_t *scratch, uint8_t *inner_out, uint8_t *alh_out);

/* Many independent htrees in one pass (Tx.BuildHashTree tx.go:332-355 over
 * many txs, e.g. the MaxConcurrency concurrent commits at immustore.go:1632):
 * tree t is digests[leaf_off[t] .. leaf_off[t+1]) and gets roots[t]
 * (width 0 -> SHA256(nil), htree.go:73-77).  leaf_off has ntrees + 1 entries. */
int mh_htree_build_many(mh_ctx *ctx, uint64_t ntrees, const uint64_t *leaf_off,
                        const uint8_t *digests, uint8_t *roots);

/* VerifyLinearProof (verification.go:40-64) for n proofs: proof p has
 * SourceTxID proof_src[p], TargetTxID proof_tgt[p] and terms
 * terms[term_off[p] .. term_off[p+1]); it is checked against src[p], tgt[p],
 * src_alh[p], tgt_alh[p].  ok[p] = 1 iff it verifies. */
int mh_verify_linear_proof_batch(mh_ctx *ctx, uint64_t n, const uint64_t *proof_src,
                                 const uint64_t *proof_tgt, const uint64_t *term_off,
                                 const uint8_t *terms, const uint64_t *src, const uint64_t *tgt,
                                 const uint8_t *src_alh, const uint8_t *tgt_alh, uint8_t *ok);

/* VerifyDualProofV2 (verification.go:304-372) for n proofs.  Proof p:
 * src_hdr[p], tgt_hdr[p] (md in md_blob), InclusionProof terms
 * incl_terms[incl_off[p] .. incl_off[p+1]), ConsistencyProof terms
 * cons_terms[cons_off[p] ..), checked against src[p], tgt[p], src_alh[p],
 * tgt_alh[p].  status[p] = MH_OK or the Go error: MH_ERR_ILLEGAL_ARGUMENTS,
 * MH_ERR_SOURCE_TX_NEWER, MH_ERR_UNEXPECTED_LINKING,
 * MH_ERR_INCLUSION_NOT_VALID, MH_ERR_CONSISTENCY_NOT_VALID. */
int mh_verify_dual_proof_v2_batch(mh_ctx *ctx, uint64_t n, const mh_tx_header *src_hdr,
                                  const mh_tx_header *tgt_hdr, const uint8_t *md_blob,
                                  uint64_t md_blob_len, const uint64_t *incl_off,
                                  const uint8_t *incl_terms, const uint64_t *cons_off,
                                  const uint8_t *cons_terms, const uint64_t *src,
                                  const uint64_t *tgt, const uint8_t *src_alh,
                                  const uint8_t *tgt_alh, int32_t *status);

/* pkg/verification.VerifyDocument (pkg/verification/verification.go:37-196),
 * the hashing part, for n documents: replaces the per-document Go calls of a
 * client verifying many ProofDocumentResponses.  The caller keeps what is not
 * hashing: the document-id lookup and encodedKeyForDocument (:50-58), the
 * EncodedDocument decode and proto.Equal against the caller's document
 * (:78-110, which Go runs between the entry check and the htree) and the
 * signature check of the new state (:199-205).
 * Document d:
 *   doc[doc_off[d] .. doc_off[d+1])              proof.EncodedDocument
 *   doc_key[doc_key_off[d] .. doc_key_off[d+1])  encodedKeyForDocument(...)
 *   tx_hdr[d]                                    VerifiableTx.Tx.Header (its Eh is checked)
 *   entries ent_off[d] .. ent_off[d+1] of the flat entry arrays (offsets index
 *   ekey_off / emd_off / ehval directly): key ekeys[ekey_off[e] .. ekey_off[e+1]),
 *   KVMetadata.Bytes() emd[emd_off[e] .. emd_off[e+1]) (emd_off may be NULL:
 *   no metadata), HValue ehval[32 e]
 *   src_hdr[d], tgt_hdr[d], InclusionProof incl_terms[incl_off[d] .. incl_off[d+1]),
 *   ConsistencyProof cons_terms[cons_off[d] ..)  VerifiableTx.DualProof (V2)
 *   known_tx_id[d] (0: no known state), known_alh[32 d]  knownState
 * Tx metadata of every header lives in md_blob (mh_tx_header.md_off).
 * status[d]: MH_OK; MH_ERR_INVALID_PROOF_ENTRY (:60-76); MH_ERR_UNSUPPORTED_TX_VERSION
 * (:118-121); MH_ERR_INVALID_PROOF (Eh :137-139, headers :146-163, known state
 * :165-183); MH_ERR_ILLEGAL_ARGUMENTS for a header Go cannot hash (its
 * innerHash panics); or the VerifyDualProofV2 status.  target_alh_out[32 d]
 * (may be NULL): the new state's TxHash (the target header's Alh) when OK,
 * zeros otherwise. */
typedef struct mh_document_batch {
    uint64_t n;
    const uint8_t *doc;
    const uint64_t *doc_off;
    const uint8_t *doc_key;
    const uint64_t *doc_key_off;
    const mh_tx_header *tx_hdr;
    const uint64_t *ent_off;
    const uint8_t *ekeys;
    const uint64_t *ekey_off;
    const uint8_t *emd;
    const uint64_t *emd_off;
    const uint8_t *ehval;
    const mh_tx_header *src_hdr;
    const mh_tx_header *tgt_hdr;
    const uint8_t *md_blob;
    uint64_t md_blob_len;
    const uint64_t *incl_off;
    const uint8_t *incl_terms;
    const uint64_t *cons_off;
    const uint8_t *cons_terms;
    const uint64_t *known_tx_id;
    const uint8_t *known_alh;
} mh_document_batch;
int mh_verify_document_batch(mh_ctx *ctx, const mh_document_batch *batch, int32_t *status,
                             uint8_t *target_alh_out);

/* VerifyDualProof (verification.go:127-235: v1 proofs with linear and
 * linear-advance parts) for n proofs, all arrays host memory, term lists as
 * CSR (x_off has n + 1 entries, terms x_terms[x_off[p] .. x_off[p+1])).
 * The linear-advance inclusion proofs of proof p are nested proofs
 * advance_incl_first[p] .. advance_incl_first[p+1]) whose terms are
 * advance_incl_terms[advance_incl_off[q] .. advance_incl_off[q+1]).
 * has_linear / has_advance = 0 stand for Go's nil proofs.  ok[p] = 1 iff the
 * proof verifies (the Go function returns bool). */
typedef struct mh_dual_proof_batch {
    uint64_t n;
    const mh_tx_header *src_hdr;
    const mh_tx_header *tgt_hdr;
    const uint8_t *md_blob;
    uint64_t md_blob_len;
    const uint64_t *incl_off;
    const uint8_t *incl_terms;
    const uint64_t *cons_off;
    const uint8_t *cons_terms;
    const uint8_t *target_bl_tx_alh; /* n x 32 (DualProof.TargetBlTxAlh) */
    const uint64_t *last_off;
    const uint8_t *last_terms;
    const uint8_t *has_linear;
    const uint64_t *linear_src; /* LinearProof.SourceTxID */
    const uint64_t *linear_tgt; /* LinearProof.TargetTxID */
    const uint64_t *linear_off;
    const uint8_t *linear_terms;
    const uint8_t *has_advance;
    const uint64_t *advance_off;
    const uint8_t *advance_terms;
    const uint64_t *advance_incl_first;
    const uint64_t *advance_incl_off;
    const uint8_t *advance_incl_terms;
    const uint64_t *src;
    const uint64_t *tgt;
    const uint8_t *src_alh;
    const uint8_t *tgt_alh;
} mh_dual_proof_batch;
int mh_verify_dual_proof_batch(mh_ctx *ctx, const mh_dual_proof_batch *b, uint8_t *ok);

/* The wire side of v1: DualProofFromProto (database_protoconv.go:213-224,
 * LinearProofFromProto :264-270, LinearAdvanceProofFromProto :272-287) over n
 * DualProof messages msgs[msg_off[p] .. msg_off[p+1]), on the device, into the
 * arrays of mh_dual_proof_batch (same names and layout; tx metadata packed into
 * md_blob as for mh_dual_proof_v2_pb_decode_batch).  status[p]: MH_OK;
 * MH_ERR_CORRUPTED_DATA (not a valid encoding: zero headers, no terms);
 * MH_ERR_ILLEGAL_ARGUMENTS (a header or the linear proof missing: Go's
 * conversion dereferences them).  Capacities are in terms, advance_incl_cap in
 * nested InclusionProofs; when one is short the n + 1 offset arrays and the
 * statuses are written and MH_ERR_BUFFER_TOO_SMALL is returned (the size query;
 * nested_proofs / nested_terms report the nested totals on every return). */
typedef struct mh_dual_proof_decoded {
    mh_tx_header *src_hdr;        /* n */
    mh_tx_header *tgt_hdr;        /* n */
    uint8_t *md_blob;             /* room for 2n x MH_MAX_TX_METADATA_LEN */
    uint8_t *target_bl_tx_alh;    /* n x 32 */
    uint8_t *has_linear;          /* n */
    uint64_t *linear_src;         /* n */
    uint64_t *linear_tgt;         /* n */
    uint8_t *has_advance;         /* n */
    uint64_t *incl_off, *cons_off, *last_off, *linear_off, *advance_off; /* n + 1 each */
    uint64_t *advance_incl_first; /* n + 1 */
    uint64_t *advance_incl_off;   /* advance_incl_cap + 1 */
    uint8_t *incl_terms, *cons_terms, *last_terms, *linear_terms, *advance_terms;
    uint8_t *advance_incl_terms;
    uint64_t incl_cap, cons_cap, last_cap, linear_cap, advance_cap;
    uint64_t advance_incl_cap, advance_incl_terms_cap;
    uint64_t nested_proofs, nested_terms; /* out */
} mh_dual_proof_decoded;
int mh_dual_proof_pb_decode_batch(mh_ctx *ctx, uint64_t n, const uint8_t *msgs,
                                  const uint64_t *msg_off, mh_dual_proof_decoded *out,
                                  int32_t *status);

/* Tx-log read path (Tx.readFrom tx.go:388-630: readHeader, readEntry,
 * buildAndValidateHtree) over buf = back-to-back tx records as written by
 * immustore.go:1812-1924.  Parses up to max_txs records, stopping at id 0 (a
 * preallocated tail) or at the first structural error, which is returned
 * (MH_ERR_CORRUPTED_* / MH_ERR_TRUNCATED) with *consumed = that record's
 * offset; then, on the device, rebuilds every entry digest, every tx's htree
 * (Eh) and Alh and compares it with the stored one: status[k] = MH_OK or
 * MH_ERR_CORRUPTED_DATA ("ALH mismatch", tx.go:625).  Optional outputs
 * (capacity max_txs): hdrs (md_off relative to buf, eh = rebuilt Eh) and
 * alh (recomputed).  KV / tx metadata are parsed as the reader parses them
 * (KVMetadata.unsafeReadFrom kv_metadata.go:221-256, TxMetadata.ReadFrom
 * tx_metadata.go:159-193): unknown attribute codes, short payloads and an
 * extra running past the metadata stop the parse with MH_ERR_CORRUPTED_DATA;
 * valid metadata is hashed in its re-serialized form (Bytes(), attributes in
 * code order, a repeated attribute's last value), as Go hashes it -- records
 * whose stored metadata is not already in that form (never written by immudb)
 * are hashed from canonical copies placed after the log on the device. */
/* The record structure alone (host only, no hashing, no device): the same
 * parse as mh_txlog_validate (readHeader / readEntry limits and errors,
 * tx.go:419-603) returning the headers (eh zero) and the offset of each
 * record's stored Alh.  Long runs are parsed by several threads from
 * speculated record starts; the result is always the sequential parse's. */
int mh_txlog_scan(const uint8_t *buf, uint64_t len, uint32_t max_entries, uint32_t max_key_len,
                  uint64_t max_txs, uint64_t *ntx, uint64_t *consumed, mh_tx_header *hdrs,
                  uint64_t *alh_off);
int mh_txlog_validate(mh_ctx *ctx, const uint8_t *buf, uint64_t len, uint32_t max_entries,
                      uint32_t max_key_len, uint64_t max_txs, uint64_t *ntx, uint64_t *consumed,
                      mh_tx_header *hdrs, uint8_t *alh, int32_t *status);
/* The same check of a log that is ALREADY in device memory -- the caller
 * re-validating what it just wrote or keeps resident (a scrub of the tx log,
 * the indexer's readTx of recent txs, embedded/store/indexer.go:570, tx.go:
 * 388-630): buf is the host copy the record hop parses, dlog (device, on the
 * context's device) the same len bytes, read by the kernels in place -- no
 * host->device copy.  The device allocation holding dlog must extend at least
 * 256 bytes past dlog + len (checked: MH_ERR_ILLEGAL_ARGUMENTS).  Outputs and
 * statuses as mh_txlog_validate.  The kernels never walk a length of dlog:
 * every record's structure in dlog is checked on the device against the host
 * copy's first, and a record whose resident bytes give another structure (or
 * differ from buf, for records the fused kernels do not take) is
 * MH_ERR_CORRUPTED_DATA with its Alh zeroed -- a drifted resident log is
 * reported per record, never a fault. */
int mh_txlog_validate_resident(mh_ctx *ctx, const uint8_t *buf, const uint8_t *dlog, uint64_t len,
                               uint32_t max_entries, uint32_t max_key_len, uint64_t max_txs,
                               uint64_t *ntx, uint64_t *consumed, mh_tx_header *hdrs,
                               uint8_t *alh, int32_t *status);
/* The same check of a log already in device memory, indexed by the store's
 * commit log instead of a host copy (no host hop, no host->device copy of the
 * log): ImmuStore.readTx for txs 1..ntx of the cLog (immustore.go:3048-3060 ->
 * txOffsetAndSize :2569-2597 -> Tx.readFrom tx.go:388-630).  clog holds ntx
 * commit-log entries of clog_entry_size bytes (12: BE64 tx offset || BE32 tx
 * size, cLogEntrySizeV1; 44: + the tx's Alh, cLogEntrySizeV2,
 * immustore.go:122-123) -- the entries after the appendable header, in device
 * or host memory.  dlog: the tx-log data (after its appendable header), len
 * bytes, either on the context's device, its allocation extending 256 bytes
 * past it, or in host memory (pinned -- the cgo shim's arena -- or pageable):
 * then it is copied up in chunks (5 : 2 : 1 from 16 MiB, as
 * mh_txlog_validate) and, when the cLog entries are in log order, the records
 * ending in each chunk are checked as soon as it lands.  Record t is parsed where entry t points, on to the end of the log as Go's
 * reader does; status[t] (each output nullable; device, pinned or pageable
 * memory, capacity ntx):
 *   MH_ERR_TRUNCATED        the record runs past len / reads as an id-0 tail
 *                           (readTx's "unexpected EOF", ErrCorruptedTxData);
 *   MH_ERR_CORRUPTED_*, MH_ERR_METADATA_UNSUPPORTED  the reader's structural
 *                           errors, as mh_txlog_validate reports them;
 *   MH_ERR_CORRUPTED_DATA   ALH mismatch (tx.go:625); or the record does not
 *                           end exactly at offset + size, or a 44-byte entry's
 *                           Alh differs (the open path's cLog checks,
 *                           immustore.go:458-528);
 * with hdrs (md_off relative to dlog, eh rebuilt) and alh as mh_txlog_validate
 * for valid records, zeros for records with a structural error.  *nbad: the
 * number of non-OK records, *first_bad: the first (ntx when none).  Returns
 * MH_OK when the call ran.  Records with metadata not in Go's canonical form
 * or with more than 1024 entries (and, for a host log, records whose read runs
 * past their chunk) are re-validated on the host bytes of that record alone
 * (mh_txlog_validate). */
int mh_txlog_validate_clog(mh_ctx *ctx, const uint8_t *dlog, uint64_t len, const uint8_t *clog,
                           uint64_t ntx, uint32_t clog_entry_size, uint32_t max_entries,
                           uint32_t max_key_len, mh_tx_header *hdrs, uint8_t *alh,
                           int32_t *status, uint64_t *nbad, uint64_t *first_bad);

/* ------------------------------------------------------------ commit path */
/* the hashing of ImmuStore.precommit / preCommitWith
 * (immustore.go:1620-1632 and 2301-2313: hVal = SHA256(value), or
 * EntrySpec.HashValue when IsValueTruncated, then Tx.BuildHashTree
 * tx.go:332-355 -> header Eh) for a batch of transactions, plus the
 * replicated-tx check `tx.header.Eh != hdr.Eh` (immustore.go:1649-1654).
 * A pipe owns a copy stream, a compute stream and three slots of device /
 * pinned buffers; a batch is cut into chunks of whole transactions
 * (~chunk_bytes of keys + values each, 0 = 64 MiB) whose host->device copies
 * run back to back under the hashing of the previous chunks.  Outputs in
 * pinned memory receive the device->host copies directly.  Not synchronised:
 * one pipe per goroutine. */
typedef struct mh_commit_pipe mh_commit_pipe;
int mh_commit_pipe_new(mh_ctx *ctx, uint64_t chunk_bytes, mh_commit_pipe **out);
int mh_commit_pipe_free(mh_commit_pipe *p);
/* Transaction t owns entries [tx_off[t], tx_off[t+1]) (tx_off: ntx + 1
 * entries, ascending); entry e has key keys[key_off[e] .. key_off[e+1]), KV
 * metadata (KVMetadata.Bytes(), kv_metadata.go:207-219) md[md_off[e] ..
 * md_off[e+1]) and value vals[val_off[e] .. val_off[e+1]) -- offsets index
 * the host arrays directly; md / md_off may both be NULL (no metadata).
 * hval_override + use_override (both or neither) model IsValueTruncated.
 * Outputs, host memory: hvals_out[e - tx_off[0]] (may be NULL), eh_out[t]
 * (may be NULL) and status[t]: MH_OK; MH_ERR_MAX_WIDTH_EXCEEDED if the tx has
 * more than max_width entries (htree.go:69-71; 0 = no limit);
 * MH_ERR_METADATA_UNSUPPORTED for KV metadata under version 0 (tx.go:691-693);
 * MH_ERR_ILLEGAL_ARGUMENTS if expect_eh (ntx x 32, may be NULL) differs from
 * the built Eh ("entries hash (Eh) differs", immustore.go:1651).  eh_out is
 * zeroed for the first two.  Pinned inputs (mh_host_alloc_pinned) make the
 * copies asynchronous DMA; pageable inputs work at the runtime's staged rate. */
int mh_precommit_batch(mh_commit_pipe *p, int version, uint64_t max_width, uint64_t ntx,
                       const uint64_t *tx_off, const uint8_t *keys, const uint64_t *key_off,
                       const uint8_t *md, const uint64_t *md_off, const uint8_t *vals,
                       const uint64_t *val_off, const uint8_t *hval_override,
                       const uint8_t *use_override, const uint8_t *expect_eh, uint8_t *hvals_out,
                       uint8_t *eh_out, int32_t *status);

/* Group commit of single transactions (the concurrent committers of
 * precommit, immustore.go:1620-1632: each hashes its own tx before taking the
 * store lock at :1689, up to MaxConcurrency = 30 at once, options.go:35).
 * mh_commit_queue_submit hashes ONE transaction -- hVal per entry
 * (immustore.go:1624-1629), entry digests and the htree (tx.go:332-355) --
 * and blocks until its results are ready; a worker thread coalesces the
 * transactions submitted within wait_us (or max_txs of them) into one
 * mh_precommit_batch.  Arguments of submit are those of one tx of
 * mh_precommit_batch (offsets index the arrays directly; n + 1 of each);
 * expect_eh (32 bytes, may be NULL) is ReplicateTx's Eh (immustore.go:1649-1654).
 * Returns the tx's status (MH_OK, MH_ERR_MAX_WIDTH_EXCEEDED,
 * MH_ERR_METADATA_UNSUPPORTED, MH_ERR_ILLEGAL_ARGUMENTS for an Eh mismatch)
 * or an error of the batch.  Thread-safe: call submit from any number of
 * threads. */
typedef struct mh_commit_queue mh_commit_queue;
int mh_commit_queue_new(mh_ctx *ctx, int version, uint64_t max_width, uint32_t max_txs,
                        uint32_t wait_us, mh_commit_queue **out);
int mh_commit_queue_free(mh_commit_queue *q);
int mh_commit_queue_submit(mh_commit_queue *q, uint64_t n, const uint8_t *keys,
                           const uint64_t *key_off, const uint8_t *md, const uint64_t *md_off,
                           const uint8_t *vals, const uint64_t *val_off,
                           const uint8_t *hval_override, const uint8_t *use_override,
                           const uint8_t *expect_eh, uint8_t *hvals_out, uint8_t *eh_out);
/* batches run and transactions hashed so far */
int mh_commit_queue_stats(mh_commit_queue *q, uint64_t *batches, uint64_t *txs);

/* ------------------------------------------------------------ multi-GPU
 * one process (a cgo caller) driving K devices, one mh_ctx
 * (HIP stream) per device, an RCCL clique over them (ncclCommInitAll; RCCL is
 * loaded on first use, MH_ERR_COLLECTIVE if it is missing).  The htree leaves
 * are cut into power-of-two aligned shards of S entries (mh_multi_shard_plan:
 * S = next power of two >= ceil(n / K), shard g = [gS, min((g+1)S, n)),
 * G = ceil(n / S) <= K shards); device g builds its shard's subtree with every
 * level (exactly the global levels 0..log2 S of that range, htree.go:85-110),
 * the G subtree roots are all-gathered over RCCL (32 bytes per device) and the
 * top ceil(log2 G) levels are reduced over them.  A device may be listed more
 * than once (more shards than devices); the roots are then gathered with
 * device-to-device copies instead of RCCL. */
typedef struct mh_multi mh_multi;
int mh_multi_create(int ndev, const int *devices, mh_multi **out);
int mh_multi_destroy(mh_multi *m);
int mh_multi_size(mh_multi *m, int *ndev);
/* the context of device d (for mh_dev_alloc / fills / copies on that device) */
mh_ctx *mh_multi_ctx(mh_multi *m, int d);
int mh_multi_synchronize(mh_multi *m);
int mh_multi_shard_plan(uint64_t n, int ndev, uint64_t *shard, uint64_t *nshards);
/* Tx.BuildHashTree over n fixed-shape entries (value hash loop
 * immustore.go:1620-1630 + tx.go:332-355 + htree.go:68-113) across the K
 * devices, HOST memory in and out (as mh_htree_build_entries with fixed
 * strides): hvals_out (n x 32, may be NULL), levels_out (the flat level-major
 * layout, mh_htree_levels_len(n) x 32, may be NULL), root. */
int mh_multi_htree_build_entries_fixed(mh_multi *m, int version, uint64_t n, const uint8_t *keys,
                                       uint32_t key_len, const uint8_t *vals, uint32_t val_len,
                                       uint8_t *hvals_out, uint8_t *levels_out, uint8_t root[32]);
/* The general (CSR) form of the same build (mh_htree_build_entries' inputs:
 * ragged keys / KV metadata / values, IsValueTruncated overrides), host
 * memory in and out: each shard's byte ranges and offsets go to its device. */
int mh_multi_htree_build_entries(mh_multi *m, int version, uint64_t n, const uint8_t *keys,
                                 const uint64_t *key_off, const uint8_t *md,
                                 const uint64_t *md_off, const uint8_t *vals,
                                 const uint64_t *val_off, const uint8_t *hval_override,
                                 const uint8_t *use_override, uint8_t *hvals_out,
                                 uint8_t *levels_out, uint8_t root[32]);
/* Device-resident variant (BASELINE configs[3]): device d holds entries
 * [d n_per_dev, (d+1) n_per_dev) of a K * n_per_dev-entry tree (n_per_dev a
 * power of two when K > 1) in keys[d] / vals[d]; it writes its subtree's levels
 * to levels[d] (mh_htree_levels_len(n_per_dev) nodes), hVals to hvals_out[d]
 * (array may be NULL), the top levels over the K gathered roots to
 * top_levels[d] (mh_htree_levels_len(K) nodes) and the GLOBAL root to root[d]
 * -- every device ends with the same top levels and root.  Asynchronous on the
 * devices' context streams (mh_multi_synchronize). */
int mh_multi_dev_htree_build_entries_fixed(mh_multi *m, int version, uint64_t n_per_dev,
                                           const uint8_t *const *keys, uint32_t key_len,
                                           const uint8_t *const *vals, uint32_t val_len,
                                           uint8_t *const *hvals_out, uint8_t *const *levels,
                                           uint8_t *const *top_levels, uint8_t *const *root);
/* ahtree AppendBatch of `total` payloads (plen bytes each) onto a tree of
 * size n0 across the K devices (ahtree.go:246-373; BASELINE configs[2] at
 * scale, and the replay of syncBinaryLinking, immustore.go:1198-1232, which
 * resumes at aht.Size()+1 on every open, :686-693).  The batch
 * (n0, n0 + total] is cut at multiples of S = 2^k (S <= total / 8K) into
 * G <= K nearly equal ranges (mh_ahtree_range_plan); device d appends range
 * d and keeps ONLY that range's digests: dLog indices
 * [mh_ahtree_nodes_upto(b[d]), mh_ahtree_nodes_upto(b[d+1])).  Every node a
 * range reads outside itself is a peak of its left end (the perfect subtree
 * of a set bit of b[d]); the old tree's peaks come from the caller and the
 * others are built on the devices from the ranges' level-k piece roots,
 * all-gathered over RCCL (32 B per piece, tens of pieces per device).
 * peaks: the popcount(n0) peaks of the old tree, lowest level first, in host
 * memory -- peak l is node(n0 with the bits below l cleared, l) =
 * dLog[mh_ahtree_node_index(n0 & ~(2^l - 1), l)] for every set bit l of n0
 * (NULL when n0 == 0; mh_dev_ahtree_peaks reads them from a resident dLog).
 * Device variant: payloads[d] holds range d's b[d+1] - b[d] payloads and
 * dlog[d] the room for its digests (16-byte aligned); roots_out (may be NULL,
 * or hold NULL entries) receives RootAt after each append of range d.
 * Ranges d >= G are unused.  Asynchronous on the devices' context streams.
 * Host variant: payloads and dlog_out (the NEW digests only,
 * (nodesUpto(n0 + total) - nodesUpto(n0)) x 32 bytes = what Append writes to
 * tree/NNNNNNNN.sha, may be NULL) in host memory, root = RootAt(n0 + total);
 * total == 0 -> MH_ERR_UNEXISTENT_DATA for an empty tree (ahtree.go:727-745),
 * MH_ERR_ILLEGAL_ARGUMENTS otherwise. */
int mh_multi_dev_ahtree_append_batch(mh_multi *m, uint64_t n0, const uint8_t *peaks,
                                     uint64_t total, const uint8_t *const *payloads, uint32_t plen,
                                     uint8_t *const *dlog, uint8_t *const *roots_out);
int mh_multi_ahtree_append_batch(mh_multi *m, uint64_t n0, const uint8_t *peaks,
                                 const uint8_t *payloads, uint64_t total, uint32_t plen,
                                 uint8_t *dlog_out, uint8_t root[32]);
/* The range plan of those calls (host only): bounds[0..*nranges] (room for
 * ndev + 1 values; bounds[0] = n0, bounds[*nranges] = n0 + total, the others
 * multiples of 2^*shard_bits), range d = (bounds[d], bounds[d+1]] on device d.
 * ndev <= 64. */
int mh_ahtree_range_plan(uint64_t n0, uint64_t total, int ndev, int *shard_bits, uint64_t *bounds,
                         int *nranges);
/* The same ranged append with ONE PROCESS PER DEVICE (torch.distributed /
 * any launcher whose ranks exchange bytes themselves): rank r of `world`
 * appends range r of mh_ahtree_range_plan(n0, total, world) -- the same
 * digests mh_multi_dev_ahtree_append_batch leaves on device r -- in two calls
 * around one all-gather the caller runs (ahtree.go:246-373):
 *  1. mh_dev_ahtree_range_local: leaves + perfect nodes of the range and its
 *     pieces' level-k roots into `send` (device, send_bytes);
 *  2. the caller all-gathers send_bytes from every rank, in rank order, into
 *     `recv` (device, world x send_bytes; skipped when the plan has one range);
 *  3. mh_dev_ahtree_range_finish: the piece tree above level k, the rank's
 *     frontier and its spines; roots_out (may be NULL) gets RootAt after each
 *     append of the range.
 * send_bytes / work_bytes from mh_ahtree_range_sizes; `work` (device,
 * 16-byte aligned) is this rank's scratch and must be kept between the two
 * calls; payloads / dlog_range as for the device variant above (range r's
 * payloads, room for its new digests).  peaks (host) on EVERY rank when
 * n0 > 0.  A rank past the plan's ranges (r >= nranges) does nothing but
 * still joins the all-gather.  Asynchronous on the context stream. */
int mh_ahtree_range_sizes(uint64_t n0, uint64_t total, int ndev, uint64_t *send_bytes,
                          uint64_t *work_bytes);
int mh_dev_ahtree_range_local(mh_ctx *ctx, uint64_t n0, const uint8_t *peaks, uint64_t total,
                              int world, int rank, const uint8_t *payloads, uint32_t plen,
                              uint8_t *dlog_range, uint8_t *work, uint8_t *send);
int mh_dev_ahtree_range_finish(mh_ctx *ctx, uint64_t n0, const uint8_t *peaks, uint64_t total,
                               int world, int rank, const uint8_t *recv, uint8_t *dlog_range,
                               uint8_t *work, uint8_t *roots_out);
/* The PCIe-bound batch paths over the K devices: the batch is cut into K
 * contiguous parts -- by index for proofs, at record boundaries (nearly equal
 * bytes) for a tx log -- and part d runs the single-context call on device d
 * from its own thread, over its own PCIe link; outputs land side by side,
 * byte-equal to one single-context call over the whole batch (K = 1 IS that
 * call).  Arguments, statuses and outputs as mh_htree_verify_inclusion_batch
 * (htree.go:166-195), mh_verify_dual_proof_v2_batch (verification.go:303-372)
 * and mh_txlog_validate (tx.go:388-630; the replay of
 * immustore.go:1198-1223 and the indexer's readTx, indexer.go:570: every
 * record carries its prevAlh, so the parts are independent).  For the tx log
 * the host hop finds the record boundaries once first (mh_txlog_scan's status
 * is the call's); a header's md_off stays relative to buf. */
int mh_multi_htree_verify_inclusion_batch(mh_multi *m, uint64_t n, const uint64_t *leaf,
                                          const uint64_t *width, const uint64_t *term_off,
                                          const uint8_t *terms, const uint8_t *digests,
                                          const uint8_t *roots, uint8_t *ok);
int mh_multi_verify_dual_proof_v2_batch(mh_multi *m, uint64_t n, const mh_tx_header *src_hdr,
                                        const mh_tx_header *tgt_hdr, const uint8_t *md_blob,
                                        uint64_t md_blob_len, const uint64_t *incl_off,
                                        const uint8_t *incl_terms, const uint64_t *cons_off,
                                        const uint8_t *cons_terms, const uint64_t *src,
                                        const uint64_t *tgt, const uint8_t *src_alh,
                                        const uint8_t *tgt_alh, int32_t *status);
int mh_multi_txlog_validate(mh_multi *m, const uint8_t *buf, uint64_t len, uint32_t max_entries,
                            uint32_t max_key_len, uint64_t max_txs, uint64_t *ntx,
                            uint64_t *consumed, mh_tx_header *hdrs, uint8_t *alh,
                            int32_t *status);
/* More PCIe-bound batches over the K devices, each part on its own link, cut
 * into parts of nearly equal input bytes: readValueAt's hVal check
 * (immustore.go:3183-3240; *ncorrupted summed over the parts), the fused
 * DualProofV2 wire verify (database_protoconv.go:226-262 +
 * verification.go:303-372), and precommit's hashing (immustore.go:1620-1632;
 * whole transactions per part, each device with its own commit pipe made on
 * first use).  Arguments and outputs as mh_verify_values_batch,
 * mh_verify_dual_proof_v2_pb_batch and mh_precommit_batch. */
int mh_multi_verify_values_batch(mh_multi *m, uint64_t n, const uint8_t *vals, const uint64_t *off,
                                 const uint64_t *vlen, const uint8_t *hvals, int32_t *status,
                                 uint64_t *ncorrupted);
int mh_multi_verify_dual_proof_v2_pb_batch(mh_multi *m, uint64_t n, const uint8_t *msgs,
                                           const uint64_t *msg_off, const uint64_t *src,
                                           const uint64_t *tgt, const uint8_t *src_alh,
                                           const uint8_t *tgt_alh, int32_t *status);
/* VerifyDocument's hashing part (verification.go:37-196) over the devices:
 * parts of nearly equal entries + document bytes, as mh_verify_document_batch. */
int mh_multi_verify_document_batch(mh_multi *m, const mh_document_batch *batch, int32_t *status,
                                   uint8_t *target_alh_out);
int mh_multi_precommit_batch(mh_multi *m, int version, uint64_t max_width, uint64_t ntx,
                             const uint64_t *tx_off, const uint8_t *keys, const uint64_t *key_off,
                             const uint8_t *md, const uint64_t *md_off, const uint8_t *vals,
                             const uint64_t *val_off, const uint8_t *hval_override,
                             const uint8_t *use_override, const uint8_t *expect_eh,
                             uint8_t *hvals_out, uint8_t *eh_out, int32_t *status);

/* ------------------------------------------------------------ wire formats
 * proofs as the protobuf messages the gRPC server sends
 * (pkg/api/schema/schema.proto, Go conversion pkg/api/schema/database_protoconv.go,
 * marshalled as protobuf-go does: field-number order, proto3 zero values
 * omitted), generated AND encoded on the device from the resident tree, so a
 * batch of VerifiableGet / VerifiableTxByIdV2 answers is one device->host
 * copy of ready-to-send bytes.  Message p is out[off[p] .. off[p+1]) (off has
 * n + 1 entries, off[0] = 0); a message that fails is empty and status[p]
 * holds the Go error.  If out_cap < off[n] nothing is written to out, off and
 * status are filled and MH_ERR_BUFFER_TOO_SMALL is returned (call again with
 * a buffer of off[n] bytes). */

/* The other direction, on the device: DualProofV2FromProto
 * (database_protoconv.go:226-262, TxHeaderFromProto, TxMetadataFromProto,
 * DigestsFromProto :293-305) over n DualProofV2 messages, message p =
 * msgs[msg_off[p] .. msg_off[p+1]), read as protobuf-go's Unmarshal does
 * (any field order, last scalar wins, repeated headers merged, unknown and
 * mistyped fields skipped).  Outputs are the arguments of
 * mh_verify_dual_proof_v2_batch: src_hdr / tgt_hdr (n each), md_blob (room for
 * 2n x MH_MAX_TX_METADATA_LEN bytes; the canonical TxMetadata.Bytes() of
 * every header packed in message order, source before target, located by each
 * header's md_off / md_len), incl_off / cons_off (n + 1 each) and the
 * terms (32 bytes each, DigestFromProto: shorter terms zero-padded, longer
 * truncated).  status[p]: MH_OK, MH_ERR_CORRUPTED_DATA (not a valid encoding;
 * no terms), MH_ERR_ILLEGAL_ARGUMENTS (a header missing: Go dereferences the
 * nil header).  If incl_cap / cons_cap (terms) are below incl_off[n] /
 * cons_off[n], only the offsets and statuses are written and
 * MH_ERR_BUFFER_TOO_SMALL is returned.  n <= 8 013 008 (32-bit md_off). */
int mh_dual_proof_v2_pb_decode_batch(mh_ctx *ctx, uint64_t n, const uint8_t *msgs,
                                     const uint64_t *msg_off, mh_tx_header *src_hdr,
                                     mh_tx_header *tgt_hdr, uint8_t *md_blob, uint64_t *incl_off,
                                     uint8_t *incl_terms, uint64_t incl_cap, uint64_t *cons_off,
                                     uint8_t *cons_terms, uint64_t cons_cap, int32_t *status);
/* InclusionProofFromProto (database_protoconv.go:123-129) over n InclusionProof
 * messages (msgs / msg_off as above), on the device -> the arguments of
 * mh_htree_verify_inclusion_batch: leaf[p] / width[p] (the wire's int32 as a
 * Go int: sign-extended, stored as its 64-bit pattern; htree verification
 * takes them with Go's signed arithmetic), term_off (n + 1) and the terms (32
 * bytes each, DigestFromProto).  status[p]: MH_OK or MH_ERR_CORRUPTED_DATA
 * (no terms, leaf = width = 0).  term_cap < term_off[n]: offsets and statuses
 * only, MH_ERR_BUFFER_TOO_SMALL. */
/* What a client auditing many VerifiableTxV2 answers does per answer --
 * DualProofV2FromProto then store.VerifyDualProofV2 (verification.go:303-372)
 * -- for n DualProofV2 messages in one call, entirely on the device: the
 * messages go up once, only the statuses come back.  status[p] is
 * mh_dual_proof_v2_pb_decode_batch's failure for message p (CORRUPTED_DATA,
 * ILLEGAL_ARGUMENTS) or else mh_verify_dual_proof_v2_batch's verdict on the
 * decoded proof with (src[p], tgt[p], src_alh[32 p], tgt_alh[32 p]), except
 * that a version-0 header's metadata is ignored, as Go's innerHash ignores it
 * (tx.go:258-263; mh_verify_dual_proof_v2_batch rejects a v0 header with
 * md_len > 0, a combination the tx log cannot hold but a message can). */
int mh_verify_dual_proof_v2_pb_batch(mh_ctx *ctx, uint64_t n, const uint8_t *msgs,
                                     const uint64_t *msg_off, const uint64_t *src,
                                     const uint64_t *tgt, const uint8_t *src_alh,
                                     const uint8_t *tgt_alh, int32_t *status);

int mh_htree_inclusion_proof_pb_decode_batch(mh_ctx *ctx, uint64_t n, const uint8_t *msgs,
                                             const uint64_t *msg_off, uint64_t *leaf,
                                             uint64_t *width, uint64_t *term_off, uint8_t *terms,
                                             uint64_t term_cap, int32_t *status);

/* InclusionProof messages (schema.proto:534-540, InclusionProofToProto
 * database_protoconv.go:115-121) of (*HTree).InclusionProof(leaf[p])
 * (htree.go:121-164) over the tree's last build; status[p] MH_OK or
 * MH_ERR_ILLEGAL_ARGUMENTS (leaf >= width). */
int mh_htree_inclusion_proof_pb_batch(mh_htree *t, uint64_t n, const uint64_t *leaf, uint8_t *out,
                                      uint64_t out_cap, uint64_t *off, int32_t *status);
/* DualProofV2 messages (schema.proto:437-445; DualProofV2ToProto /
 * TxHeaderToProto / TxMetadataToProto database_protoconv.go:152-193) of
 * ImmuStore.DualProofV2(src[p], tgt[p]) (immustore.go:2356-2387: the ahtree
 * InclusionProof(src.ID, tgt.BlTxID) and ConsistencyProof(max(1,
 * src.BlTxID), tgt.BlTxID)) over t's dLog.  Header metadata (md_len bytes of
 * TxMetadata.Bytes() at md_blob + md_off) is re-encoded as the TxMetadata
 * message; md_len == 0 is Go's nil Metadata (a header read from the tx log,
 * tx.go:483-501).  status[p]: MH_OK, MH_ERR_ILLEGAL_ARGUMENTS (src.ID == 0),
 * MH_ERR_SOURCE_TX_NEWER, MH_ERR_UNEXPECTED_LINKING, MH_ERR_UNEXISTENT_DATA
 * (tgt.BlTxID beyond the tree), MH_ERR_CORRUPTED_DATA (metadata bytes). */
int mh_ahtree_dual_proof_v2_pb_batch(mh_ahtree *t, uint64_t n, const mh_tx_header *src,
                                     const mh_tx_header *tgt, const uint8_t *md_blob,
                                     uint64_t md_blob_len, uint8_t *out, uint64_t out_cap,
                                     uint64_t *off, int32_t *status);
/* Device variants (all pointers device memory, asynchronous, no allocation):
 * scratch = mh_pb_scratch_size(n) bytes; messages beyond out_cap get status
 * MH_ERR_BUFFER_TOO_SMALL.  phase: 1 = sizes + offsets only, 2 = write only
 * (after a phase-1 call with the same inputs), 3 = both. */
uint64_t mh_pb_scratch_size(uint64_t n);
int mh_dev_htree_inclusion_proof_pb_batch(mh_ctx *ctx, int phase, const uint8_t *levels,
                                          uint64_t width, uint64_t n, const uint64_t *leaf,
                                          uint8_t *out, uint64_t out_cap, uint64_t *off,
                                          int32_t *status, void *scratch);
int mh_dev_dual_proof_v2_pb_batch(mh_ctx *ctx, int phase, const uint8_t *dlog, uint64_t size,
                                  uint64_t n, const mh_tx_header *src, const mh_tx_header *tgt,
                                  const uint8_t *md_blob, uint8_t *out, uint64_t out_cap,
                                  uint64_t *off, int32_t *status, void *scratch);

#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility pop
#endif
#ifdef __cplusplus
}
#endif
#endif /* IMMUSTORE_MERKLE_H */
