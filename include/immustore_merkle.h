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
 *  - mh_htree / mh_ahtree handles are not synchronised (like Go's HTree); use
 *    one handle per goroutine.  An mh_ctx may be shared by many handles.
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

/* ahtree verification kinds (embedded/ahtree/verification.go) */
#define MH_AHT_INCLUSION 0      /* VerifyInclusion      verification.go:21 */
#define MH_AHT_CONSISTENCY 1    /* VerifyConsistency    verification.go:58 */
#define MH_AHT_LAST_INCLUSION 2 /* VerifyLastInclusion  verification.go:111 */

typedef struct mh_ctx mh_ctx;
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
/* device pointer of the handle's level buffer (device-resident consumers) */
int mh_htree_levels_device(mh_htree *t, const uint8_t **dptr);

/* htree.VerifyInclusion batch (htree.go:166-195; store.VerifyInclusion
 * verification.go:28-30).  Proof p has terms [term_off[p], term_off[p+1]).
 * ok[p] = 1 if it verifies.  Host pointers. */
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
int mh_dev_htree_verify_inclusion_batch(mh_ctx *ctx, uint64_t nproofs, const uint64_t *leaf,
                                        const uint64_t *width, const uint64_t *term_off,
                                        const uint8_t *terms, const uint8_t *digests,
                                        const uint8_t *roots, uint8_t *ok);

/* ----------------------------------------------------------------- ahtree */
/* In-memory append-only tree whose dLog (ahtree.go:60-84, tree/NNNNNNNN.sha) lives
 * in HBM.  No pLog/cLog files: persistence stays with the Go appendables. */
int mh_ahtree_new(mh_ctx *ctx, mh_ahtree **out);
int mh_ahtree_free(mh_ahtree *t);
/* (*AHtree).Append(d)                                   ahtree.go:246-373 */
int mh_ahtree_append(mh_ahtree *t, const uint8_t *payload, uint64_t plen, uint64_t *n,
                     uint8_t h[32]);
/* m fixed-size payloads appended in order (syncBinaryLinking batch,
 * immustore.go:1198-1232). roots_out (m*32, RootAt(n0+1..n0+m)) may be NULL. */
int mh_ahtree_append_batch(mh_ahtree *t, const uint8_t *payloads, uint64_t m, uint32_t plen,
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
int mh_ahtree_reset_size(mh_ahtree *t, uint64_t new_size);
/* copy dLog digests [first, first+count) (the tree/NNNNNNNN.sha byte stream) */
int mh_ahtree_dlog(mh_ahtree *t, uint64_t first, uint64_t count, uint8_t *out);
int mh_ahtree_dlog_device(mh_ahtree *t, const uint8_t **dptr);

/* Device-resident batch append: dlog holds nodesUpto(n0) digests and has
 * room for nodesUpto(n0+m); payloads m*plen bytes. */
int mh_dev_ahtree_append_batch(mh_ctx *ctx, uint8_t *dlog, uint64_t n0, const uint8_t *payloads,
                               uint64_t m, uint32_t plen, uint8_t *roots_out);
uint64_t mh_ahtree_nodes_upto(uint64_t n); /* ahtree.go:492-511 */

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

#ifdef __cplusplus
}
#endif
#endif /* IMMUSTORE_MERKLE_H */
