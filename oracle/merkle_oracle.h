/*
 * merkle_oracle.h -- CPU restatement of immudb's Merkle-hash path.
 *
 * TEST INFRASTRUCTURE.  This is the parity oracle and the timed CPU baseline
 * (bench.py `cpu_baseline`, kind "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library
 * (immustore_amd/libimmustore_merkle.so) never links or calls it.
 *
 * Pinned by: the Go-written fixtures of the reference (tests/golden/
 * immudb_fixtures.json: 36 stored Alh values, 42 stored values/hVal pairs and
 * three ahtree dLog streams) and the reference's own known-answer tables
 * (nodesUpto 1..16, empty root = SHA256(nil)).  See tests/test_oracle.py.
 *
 * Every function names the reference file:line it restates.  Status codes are
 * the same as include/immustore_merkle.h (MH_*).
 */
#ifndef IMMUSTORE_MERKLE_ORACLE_H
#define IMMUSTORE_MERKLE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FIPS 180-4 SHA-256 (Go crypto/sha256.Sum256, pinned by Go 1.18 toolchain). */
void orc_sha256(const uint8_t *msg, size_t len, uint8_t out[32]);
int orc_sha256_has_shani(void);
void orc_sha256_use_shani(int enable); /* 0 = force portable code */

/* embedded/store/tx.go:690-701 (v0, version 0) and :703-731 (v1, version 1).
 * Returns 0, or 6 (MH_ERR_METADATA_UNSUPPORTED) for v0 with non-empty md. */
int orc_entry_digest(int version, const uint8_t *key, size_t klen, const uint8_t *md,
                     size_t mdlen, const uint8_t hval[32], uint8_t out[32]);

/* Number of 32-byte nodes in the flat level-major layout: sum_l ceil(n/2^l)
 * while the width is > 1, plus the root level (htree.go:88-107). */
uint64_t orc_htree_levels_len(uint64_t n);
/* Offset (in nodes) of level l inside that flat layout. */
uint64_t orc_htree_level_offset(uint64_t n, int level);

/* embedded/htree/htree.go:68-113.  levels may be NULL. */
int orc_htree_build(const uint8_t *digests, uint64_t n, uint8_t *levels, uint8_t root[32]);
/* embedded/htree/htree.go:121-164.  terms has room for 64 terms. */
int orc_htree_inclusion_proof(const uint8_t *levels, uint64_t width, uint64_t i,
                              uint8_t *terms, uint32_t *nterms);
/* embedded/htree/htree.go:166-195.  returns 1 = verifies. */
int orc_htree_verify_inclusion(uint64_t leaf, uint64_t width, const uint8_t *terms,
                               uint32_t nterms, const uint8_t digest[32], const uint8_t root[32]);

/* n VerifyInclusion calls with a fixed term stride (BASELINE configs[4] on
 * the CPU); returns how many verify, ok[p] (may be NULL) per proof. */
uint64_t orc_htree_verify_batch(uint64_t n, const uint64_t *leaf, uint64_t width,
                                const uint8_t *terms, uint32_t nterms_each,
                                const uint8_t *digests, const uint8_t root[32], uint8_t *ok);

/* n ahtree Verify{Inclusion,Consistency,LastInclusion} calls (kind 0/1/2,
 * ahtree/verification.go:21-137) over CSR term lists (term_off[n+1], in
 * 32-byte terms), a / b = leaf / root, iroot / jroot, leaf / root per proof;
 * nthreads host threads.  Returns how many verify, ok[p] per proof. */
uint64_t orc_ahtree_verify_batch(int kind, uint64_t n, const uint64_t *i, const uint64_t *j,
                                 const uint64_t *term_off, const uint8_t *terms, const uint8_t *a,
                                 const uint8_t *b, uint8_t *ok, int nthreads);

/* Value hash loop (embedded/store/immustore.go:1620-1630) + Tx.BuildHashTree
 * (embedded/store/tx.go:332-355): CSR inputs (offsets have n+1 entries).
 * md / md_off may be NULL (no KV metadata).  hval_override / use_override
 * (IsValueTruncated) may be NULL.  hvals_out / levels may be NULL. */
int orc_build_entries(int version, uint64_t n, const uint8_t *keys, const uint64_t *key_off,
                      const uint8_t *md, const uint64_t *md_off, const uint8_t *vals,
                      const uint64_t *val_off, const uint8_t *hval_override,
                      const uint8_t *use_override, uint8_t *hvals_out, uint8_t *levels,
                      uint8_t root[32]);
/* Same with fixed-stride keys / values and no metadata (BASELINE C1/C2 layout).
 * nthreads > 1 splits the leaf range into power-of-two chunks (exact by
 * SURVEY.md finding 3). */
int orc_build_entries_fixed(int version, uint64_t n, const uint8_t *keys, uint32_t key_len,
                            const uint8_t *vals, uint32_t val_len, uint8_t *hvals_out,
                            uint8_t *levels, uint8_t root[32], int nthreads);

/* ImmuStore.precommit over ntx transactions (immustore.go:1620-1632, 2301-2313;
 * Eh check :1649-1654): same contract as mh_precommit_batch
 * (include/immustore_merkle.h); nthreads splits the txs. */
/* ImmuStore.readValueAt's integrity check (immustore.go:3235) over a batch:
 * status[i] = 0 when off[i+1]-off[i] == vlen[i] (vlen may be NULL) and
 * SHA256(vals[off[i]..off[i+1])) == hvals[i], else ERR_CORRUPTED_DATA (14);
 * entries split over nthreads threads.  Returns the number not OK. */
uint64_t orc_verify_values(uint64_t n, const uint8_t *vals, const uint64_t *off,
                           const uint64_t *vlen, const uint8_t *hvals, int32_t *status,
                           int nthreads);
int orc_precommit_batch(int version, uint64_t max_width, uint64_t ntx, const uint64_t *tx_off,
                        const uint8_t *keys, const uint64_t *key_off, const uint8_t *md,
                        const uint64_t *md_off, const uint8_t *vals, const uint64_t *val_off,
                        const uint8_t *hval_override, const uint8_t *use_override,
                        const uint8_t *expect_eh, uint8_t *hvals_out, uint8_t *eh_out,
                        int32_t *status, int nthreads);

/* TxHeader.innerHash / Alh: embedded/store/tx.go:249-319. */
int orc_tx_inner_hash(uint64_t ts, int version, const uint8_t *txmd, size_t txmdlen,
                      uint32_t nentries, const uint8_t eh[32], uint64_t bltxid,
                      const uint8_t blroot[32], uint8_t out[32]);
void orc_tx_alh(uint64_t id, const uint8_t prev_alh[32], const uint8_t inner[32], uint8_t out[32]);

/* Transaction header (embedded/store/tx.go:103-117), same layout as
 * include/immustore_merkle.h mh_tx_header.  md_len bytes of TxMetadata.Bytes()
 * live at md_blob + md_off (v1 only). */
typedef struct orc_tx_header {
    uint64_t id;
    int64_t ts;
    uint64_t bl_tx_id;
    uint8_t bl_root[32];
    uint8_t prev_alh[32];
    uint8_t eh[32];
    uint32_t version;
    uint32_t nentries;
    uint32_t md_len;
    uint32_t md_off;
} orc_tx_header;

/* tx.go:249-319 on a header struct; inner may be NULL. */
int orc_tx_header_alh(const orc_tx_header *h, const uint8_t *md_blob, uint8_t inner[32],
                      uint8_t alh[32]);
/* store/verification.go:40-64 (VerifyLinearProof); returns 1 = verifies. */
int orc_verify_linear_proof(uint64_t p_src, uint64_t p_tgt, const uint8_t *terms, uint32_t nterms,
                            uint64_t src, uint64_t tgt, const uint8_t src_alh[32],
                            const uint8_t tgt_alh[32]);
/* store/verification.go:66-125 (VerifyLinearAdvanceProof); incl_off has
 * nincl + 1 entries (term offsets of each nested inclusion proof). */
int orc_verify_linear_advance_proof(int has_proof, const uint8_t *lin_terms, uint32_t nlin,
                                    const uint8_t *incl_terms, const uint32_t *incl_off,
                                    uint32_t nincl, uint64_t start, uint64_t end,
                                    const uint8_t end_alh[32], const uint8_t root[32],
                                    uint64_t size);
/* store/verification.go:304-372 (VerifyDualProofV2): MH_OK or the status of
 * the Go error (2 ErrIllegalArguments, 10 ErrSourceTxNewerThanTargetTx,
 * 11 ErrUnexpectedLinkingError, 12 inclusion / 13 consistency not valid). */
int orc_verify_dual_proof_v2(const orc_tx_header *sh, const orc_tx_header *th,
                             const uint8_t *md_blob, const uint8_t *incl, uint32_t nincl,
                             const uint8_t *cons, uint32_t ncons, uint64_t src, uint64_t tgt,
                             const uint8_t src_alh[32], const uint8_t tgt_alh[32]);
/* store/verification.go:127-235 (VerifyDualProof, v1 proofs with linear and
 * linear-advance parts); returns 1 = verifies. */
int orc_verify_dual_proof(const orc_tx_header *sh, const orc_tx_header *th,
                          const uint8_t *md_blob, const uint8_t *incl, uint32_t nincl,
                          const uint8_t *cons, uint32_t ncons, const uint8_t tbl_alh[32],
                          const uint8_t *last, uint32_t nlast, int has_lin, uint64_t lin_src,
                          uint64_t lin_tgt, const uint8_t *lin, uint32_t nlin, int has_lap,
                          const uint8_t *lap_terms, uint32_t nlap, const uint8_t *lap_incl,
                          const uint32_t *lap_incl_off, uint32_t nlap_incl, uint64_t src,
                          uint64_t tgt, const uint8_t src_alh[32], const uint8_t tgt_alh[32]);
/* Tx log read path (tx.go:388-630: readHeader, readEntry, buildAndValidateHtree)
 * over a buffer of back-to-back tx records (immustore.go:1812-1924).  Stops at
 * id 0 (preallocated tail), at max_txs, or at the first structural error
 * (returned; *consumed_out = offset of the failing record).  Per parsed tx:
 * the recomputed Alh and status 0 / 14 (ALH mismatch, ErrCorruptedData). */
int orc_txlog_validate(const uint8_t *buf, uint64_t len, uint32_t max_entries,
                       uint32_t max_key_len, uint64_t max_txs, uint64_t *ntx_out,
                       uint64_t *consumed_out, uint8_t *alh_out, int32_t *status_out);

/* ahtree: embedded/ahtree/ahtree.go. The dLog is a flat array of digests. */
uint64_t orc_ahtree_nodes_upto(uint64_t n);  /* ahtree.go:492-511 */
uint64_t orc_ahtree_nodes_until(uint64_t n); /* ahtree.go:485-490 */
/* ahtree.go:246-373: append one payload to a tree of size n_before; dlog has
 * room for nodesUpto(n_before+1) digests. Writes the new root to root (opt). */
int orc_ahtree_append(uint8_t *dlog, uint64_t n_before, const uint8_t *payload, size_t plen,
                      uint8_t root[32]);
/* Fixed-size payload batch (syncBinaryLinking analog, immustore.go:1198-1232). */
int orc_ahtree_append_batch(uint8_t *dlog, uint64_t n_before, const uint8_t *payloads,
                            uint64_t m, size_t plen);
/* pLog records (BE32 len || payload, ahtree.go:266-282) and cLog entries
 * (BE64 poff || BE32 len, ahtree.go:341-351) of m appends; p_off0 = pLog size
 * before the batch.  plog / clog may be NULL. */
void orc_ahtree_log_records(const uint8_t *payloads, uint64_t m, size_t plen, uint64_t p_off0,
                            uint8_t *plog, uint8_t *clog);
int orc_ahtree_root_at(const uint8_t *dlog, uint64_t size, uint64_t n, uint8_t out[32]);
int orc_ahtree_inclusion_proof(const uint8_t *dlog, uint64_t size, uint64_t i, uint64_t j,
                               uint8_t *terms, uint32_t *nterms);
int orc_ahtree_consistency_proof(const uint8_t *dlog, uint64_t size, uint64_t i, uint64_t j,
                                 uint8_t *terms, uint32_t *nterms);
/* embedded/ahtree/verification.go */
void orc_ahtree_eval_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                               const uint8_t leaf[32], uint8_t out[32]);
int orc_ahtree_verify_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                                const uint8_t leaf[32], const uint8_t root[32]);
int orc_ahtree_eval_consistency(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                                uint8_t ci[32], uint8_t cj[32]);
int orc_ahtree_verify_consistency(const uint8_t *terms, uint32_t nterms, uint64_t i, uint64_t j,
                                  const uint8_t iroot[32], const uint8_t jroot[32]);
void orc_ahtree_eval_last_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i,
                                    const uint8_t leaf[32], uint8_t out[32]);
int orc_ahtree_verify_last_inclusion(const uint8_t *terms, uint32_t nterms, uint64_t i,
                                     const uint8_t leaf[32], const uint8_t root[32]);

/* Deterministic synthetic input used by tests and bench (splitmix64 stream,
 * little-endian words): identical to immustore_amd's device generator. */
void orc_fill_random(uint8_t *dst, uint64_t nbytes, uint64_t seed);

/* n InclusionProof (kind 0) / ConsistencyProof (kind 1) calls, proof p at
 * terms + p * cap * 32 (ahtree.go:525-651). */
void orc_ahtree_proof_batch(const uint8_t *dlog, uint64_t size, int kind, uint64_t n,
                            const uint64_t *i, const uint64_t *j, uint8_t *terms, uint32_t cap,
                            uint32_t *nterms, int32_t *st);

/* ahtree appends (n_start, n_end] of orc_fill_random(seed) payloads kept as
 * the 64 peaks only (no dLog): the dLog digests of sampled appends and the
 * peaks of n_end.  See merkle_oracle.c. */
int orc_ahtree_stream(uint64_t seed, uint32_t plen, uint64_t pay0, uint64_t n_start,
                      const uint8_t *peaks_in, uint64_t n_end, const uint64_t *samples,
                      uint64_t ns, uint8_t *out, uint32_t *cnt, uint8_t *peaks_out);

#ifdef __cplusplus
}
#endif
#endif
