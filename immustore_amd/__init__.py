"""MI355X-native Merkle-hash engine for immudb's commit path.

The hot path of codenotary/immudb -- embedded/htree (per-transaction tree and
the entry hashing feeding it), embedded/ahtree (append-only tree over Alh) and
the proof re-hash of both -- as hand-written CDNA4 HIP kernels behind a C ABI
(include/immustore_merkle.h, libimmustore_merkle.so).  This Python package is
a thin ctypes mirror of the reference's Go API used by tests and bench.py.
"""
from . import _native
from ._native import (MerkleError, ErrMaxWidthExceeded, ErrIllegalArguments, ErrIllegalState,
                      ErrEmptyTree, ErrUnexistentData, ErrMetadataUnsupported,
                      ErrCannotResetToLargerSize, ErrNoDevice, ErrOutOfMemory, HipError)
from .merkle import (Context, default_context, device_count, HTree, InclusionProof,
                     decode_inclusion_proof_pb,
                     verify_inclusion, verify_inclusion_batch, VerifyInclusion, AHtree,
                     nodes_upto, levels_len, level_offset, ahtree_verify_inclusion,
                     ahtree_eval_inclusion, ahtree_verify_consistency, ahtree_eval_consistency,
                     ahtree_verify_last_inclusion, ahtree_verify_batch, build_hash_tree,
                     verify_values)
from . import txlayer
from .txlayer import (TX_HEADER, tx_alh_batch, htree_build_many, verify_linear_proof_batch,
                      verify_dual_proof_v2_batch, VerifyDualProofV2, verify_dual_proof_batch,
                      txlog_validate)
from . import commit
from .commit import CommitPipe, EntrySpec

__all__ = [n for n in dir() if not n.startswith("_")]
