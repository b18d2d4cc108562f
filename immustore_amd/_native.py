"""ctypes binding of libimmustore_merkle.so (the C ABI in include/immustore_merkle.h).

The library is built in-tree by `__graft_entry__.build()` (hipcc, gfx950 only).
There is no fallback: if the library or a gfx950 device is missing, every
call raises instead of silently hashing on the CPU.
"""
import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MH_LIB_PATH") or os.path.join(_HERE, "libimmustore_merkle.so")

MH_OK = 0
# test-only fault sites of mh_debug_fail_at
MH_FAULT_RCCL_GROUP = 1
MH_FAULT_RCCL_GROUP_LATE = 3
MH_FAULT_TXLOG_AFTER_GROUP = 2
MH_ERR_MAX_WIDTH_EXCEEDED = 1
MH_ERR_ILLEGAL_ARGUMENTS = 2
MH_ERR_ILLEGAL_STATE = 3
MH_ERR_EMPTY_TREE = 4
MH_ERR_UNEXISTENT_DATA = 5
MH_ERR_METADATA_UNSUPPORTED = 6
MH_ERR_CANNOT_RESET_TO_LARGER = 7
MH_ERR_NO_DEVICE = 8
MH_ERR_OUT_OF_MEMORY = 9
MH_ERR_SOURCE_TX_NEWER = 10
MH_ERR_UNEXPECTED_LINKING = 11
MH_ERR_INCLUSION_NOT_VALID = 12
MH_ERR_CONSISTENCY_NOT_VALID = 13
MH_ERR_CORRUPTED_DATA = 14
MH_ERR_CORRUPTED_MAX_ENTRIES = 15
MH_ERR_CORRUPTED_MAX_KEYLEN = 16
MH_ERR_CORRUPTED_UNKNOWN_VERSION = 17
MH_ERR_TRUNCATED = 18
MH_ERR_BUFFER_TOO_SMALL = 19
MH_ERR_INVALID_PROOF = 20
MH_ERR_UNSUPPORTED_TX_VERSION = 21
MH_ERR_INVALID_PROOF_ENTRY = 22
MH_ERR_COLLECTIVE = 23

MH_AHT_INCLUSION = 0
MH_AHT_CONSISTENCY = 1
MH_AHT_LAST_INCLUSION = 2


class MerkleError(Exception):
    """Base class; `.status` holds the C status code."""

    status = None

    def __init__(self, status, msg=None):
        self.status = status
        super().__init__(msg or "status %d" % status)


class ErrMaxWidthExceeded(MerkleError):
    pass


class ErrIllegalArguments(MerkleError):
    pass


class ErrIllegalState(MerkleError):
    pass


class ErrEmptyTree(MerkleError):
    pass


class ErrUnexistentData(MerkleError):
    pass


class ErrMetadataUnsupported(MerkleError):
    pass


class ErrCannotResetToLargerSize(MerkleError):
    pass


class ErrNoDevice(MerkleError):
    pass


class ErrOutOfMemory(MerkleError):
    pass


class ErrSourceTxNewerThanTargetTx(ErrIllegalArguments):
    pass


class ErrUnexpectedLinkingError(MerkleError):
    pass


class ErrInclusionProofNotValid(MerkleError):
    pass


class ErrConsistencyProofNotValid(MerkleError):
    pass


class ErrCorruptedData(MerkleError):
    pass


class ErrCorruptedTxData(MerkleError):
    pass


class ErrCorruptedTxDataMaxTxEntriesExceeded(ErrCorruptedTxData):
    pass


class ErrCorruptedTxDataMaxKeyLenExceeded(ErrCorruptedTxData):
    pass


class ErrCorruptedTxDataUnknownHeaderVersion(ErrCorruptedTxData):
    pass


class ErrUnexpectedEOF(MerkleError):
    pass


class ErrBufferTooSmall(MerkleError):
    pass


class ErrInvalidProof(MerkleError):
    """store.ErrInvalidProof (immustore.go:114)"""


class ErrInvalidProofEntry(ErrInvalidProof):
    """store.ErrInvalidProof from VerifyDocument's entry check (verification.go:60-76)"""


class ErrUnsupportedTxVersion(MerkleError):
    """store.ErrUnsupportedTxVersion (immustore.go:90)"""


class ErrCollective(MerkleError):
    """RCCL unavailable or a collective failed (mh_multi_*)"""


class HipError(MerkleError):
    pass


_ERRORS = {
    MH_ERR_MAX_WIDTH_EXCEEDED: ErrMaxWidthExceeded,
    MH_ERR_ILLEGAL_ARGUMENTS: ErrIllegalArguments,
    MH_ERR_ILLEGAL_STATE: ErrIllegalState,
    MH_ERR_EMPTY_TREE: ErrEmptyTree,
    MH_ERR_UNEXISTENT_DATA: ErrUnexistentData,
    MH_ERR_METADATA_UNSUPPORTED: ErrMetadataUnsupported,
    MH_ERR_CANNOT_RESET_TO_LARGER: ErrCannotResetToLargerSize,
    MH_ERR_NO_DEVICE: ErrNoDevice,
    MH_ERR_OUT_OF_MEMORY: ErrOutOfMemory,
    MH_ERR_SOURCE_TX_NEWER: ErrSourceTxNewerThanTargetTx,
    MH_ERR_UNEXPECTED_LINKING: ErrUnexpectedLinkingError,
    MH_ERR_INCLUSION_NOT_VALID: ErrInclusionProofNotValid,
    MH_ERR_CONSISTENCY_NOT_VALID: ErrConsistencyProofNotValid,
    MH_ERR_CORRUPTED_DATA: ErrCorruptedData,
    MH_ERR_CORRUPTED_MAX_ENTRIES: ErrCorruptedTxDataMaxTxEntriesExceeded,
    MH_ERR_CORRUPTED_MAX_KEYLEN: ErrCorruptedTxDataMaxKeyLenExceeded,
    MH_ERR_CORRUPTED_UNKNOWN_VERSION: ErrCorruptedTxDataUnknownHeaderVersion,
    MH_ERR_TRUNCATED: ErrUnexpectedEOF,
    MH_ERR_BUFFER_TOO_SMALL: ErrBufferTooSmall,
    MH_ERR_INVALID_PROOF: ErrInvalidProof,
    MH_ERR_UNSUPPORTED_TX_VERSION: ErrUnsupportedTxVersion,
    MH_ERR_INVALID_PROOF_ENTRY: ErrInvalidProofEntry,
    MH_ERR_COLLECTIVE: ErrCollective,
}

vp = C.c_void_p
u8p = C.c_void_p  # raw addresses (host or device) are passed as integers
u64 = C.c_uint64
u32 = C.c_uint32
i32 = C.c_int

# name -> (restype, argtypes); mirrors include/immustore_merkle.h exactly.
SIGNATURES = {
    "mh_abi_version": (i32, []),
    "mh_status_string": (C.c_char_p, [i32]),
    "mh_device_count": (i32, [C.POINTER(i32)]),
    "mh_ctx_create": (i32, [i32, vp, C.POINTER(vp)]),
    "mh_ctx_destroy": (i32, [vp]),
    "mh_ctx_synchronize": (i32, [vp]),
    "mh_ctx_stream": (vp, [vp]),
    "mh_ctx_set_timing": (i32, [vp, i32]),
    "mh_ctx_timing": (i32, [vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(u64)]),
    "mh_ctx_timing_reset": (i32, [vp]),
    "mh_debug_fail_at": (i32, [i32, i32]),
    "mh_dev_alloc": (i32, [vp, u64, C.POINTER(vp)]),
    "mh_dev_free": (i32, [vp, vp]),
    "mh_host_alloc_pinned": (i32, [u64, C.POINTER(vp)]),
    "mh_host_free_pinned": (i32, [vp]),
    "mh_memcpy_h2d": (i32, [vp, vp, vp, u64]),
    "mh_memcpy_d2h": (i32, [vp, vp, vp, u64]),
    "mh_dev_fill_random": (i32, [vp, vp, u64, u64]),
    "mh_dev_fill_keys_be64": (i32, [vp, vp, u64, u64]),
    "mh_htree_levels_len": (u64, [u64]),
    "mh_htree_level_offset": (u64, [u64, i32]),
    "mh_htree_new": (i32, [vp, u64, C.POINTER(vp)]),
    "mh_htree_free": (i32, [vp]),
    "mh_htree_build_with": (i32, [vp, u8p, u64]),
    "mh_htree_build_entries": (i32, [vp, i32, u64, u8p, vp, u8p, vp, u8p, vp, u8p, u8p, u8p]),
    "mh_htree_root": (i32, [vp, u8p]),
    "mh_htree_width": (i32, [vp, C.POINTER(u64)]),
    "mh_htree_inclusion_proof": (i32, [vp, u64, u8p, u32, C.POINTER(u32)]),
    "mh_htree_levels": (i32, [vp, u8p, u64]),
    "mh_htree_levels_device": (i32, [vp, C.POINTER(vp)]),
    "mh_htree_verify_inclusion_batch": (i32, [vp, u64, vp, vp, vp, u8p, u8p, u8p, u8p]),
    "mh_dev_htree_build_digests": (i32, [vp, u8p, u64, u8p, u8p]),
    "mh_dev_htree_build_entries_fixed": (i32, [vp, i32, u64, u8p, u32, u8p, u32, u8p, u8p, u8p]),
    "mh_dev_htree_build_entries": (i32, [vp, i32, u64, u8p, vp, u8p, vp, u8p, vp, u8p, u8p, u8p,
                                         u8p, u8p]),
    "mh_dev_htree_reduce_nodes": (i32, [vp, u8p, u64, u8p, u8p]),
    "mh_dev_sha256_batch": (i32, [vp, u8p, vp, u64, u8p]),
    "mh_verify_values_batch": (i32, [vp, u64, u8p, vp, vp, u8p, vp, C.POINTER(u64)]),
    "mh_dev_verify_values_batch": (i32, [vp, u64, u8p, vp, vp, u8p, vp]),
    "mh_dev_htree_verify_inclusion_batch": (i32, [vp, u64, vp, vp, vp, u8p, u8p, u8p, u8p]),
    "mh_ahtree_new": (i32, [vp, C.POINTER(vp)]),
    "mh_ahtree_free": (i32, [vp]),
    "mh_ahtree_append": (i32, [vp, u8p, u64, C.POINTER(u64), u8p]),
    "mh_ahtree_append_batch": (i32, [vp, u8p, u64, u32, u8p]),
    "mh_ahtree_size": (i32, [vp, C.POINTER(u64)]),
    "mh_ahtree_root": (i32, [vp, C.POINTER(u64), u8p]),
    "mh_ahtree_root_at": (i32, [vp, u64, u8p]),
    "mh_ahtree_inclusion_proof": (i32, [vp, u64, u64, u8p, u32, C.POINTER(u32)]),
    "mh_ahtree_consistency_proof": (i32, [vp, u64, u64, u8p, u32, C.POINTER(u32)]),
    "mh_ahtree_reset_size": (i32, [vp, u64]),
    "mh_ahtree_dlog": (i32, [vp, u64, u64, u8p]),
    "mh_ahtree_dlog_device": (i32, [vp, C.POINTER(vp)]),
    "mh_dev_ahtree_append_batch": (i32, [vp, u8p, u64, u8p, u64, u32, u8p]),
    "mh_pb_scratch_size": (u64, [u64]),
    "mh_txlog_scan": (i32, [u8p, u64, u32, u32, u64, vp, vp, vp, vp]),
    "mh_htree_inclusion_proof_pb_batch": (i32, [vp, u64, vp, u8p, u64, vp, vp]),
    "mh_ahtree_dual_proof_v2_pb_batch": (i32, [vp, u64, vp, vp, u8p, u64, u8p, u64, vp, vp]),
    "mh_dev_htree_inclusion_proof_pb_batch": (i32, [vp, i32, u8p, u64, u64, vp, u8p, u64, vp, vp, vp]),
    "mh_dev_dual_proof_v2_pb_batch": (i32, [vp, i32, u8p, u64, u64, vp, vp, u8p, u8p, u64, vp, vp, vp]),
    "mh_ahtree_append_batch_logs": (i32, [vp, u8p, u64, u32, u64, u8p, u8p, u8p]),
    "mh_dev_ahtree_append_batch_logs": (i32, [vp, u8p, u64, u8p, u64, u32, u64, u8p, u8p, u8p]),
    "mh_dev_ahtree_log_records": (i32, [vp, u8p, u64, u32, u64, u8p, u8p]),
    "mh_ahtree_nodes_upto": (u64, [u64]),
    "mh_htree_inclusion_proof_batch": (i32, [vp, u64, vp, u8p, u32, vp, vp]),
    "mh_dev_htree_inclusion_proof_batch": (i32, [vp, u8p, u64, u64, vp, u8p, u32, vp, vp]),
    "mh_ahtree_proof_batch": (i32, [vp, i32, u64, vp, vp, u8p, u32, vp, vp]),
    "mh_dev_ahtree_proof_batch": (i32, [vp, i32, u8p, u64, u64, vp, vp, u8p, u32, vp, vp]),
    "mh_ahtree_node_index": (u64, [u64, i32]),
    "mh_ahtree_log_header": (i32, [u64, C.c_int64, i32, i32, u8p, u64, C.POINTER(u64)]),
    "mh_appendable_metadata": (i32, [u32, vp, vp, vp, u8p, u64, C.POINTER(u64)]),
    "mh_multiapp_segments": (i32, [u64, u64, u64, u64, vp, u32, C.POINTER(u32)]),
    "mh_dev_ahtree_append_local": (i32, [vp, u8p, u64, u8p, u64, u32, i32]),
    "mh_dev_ahtree_put_shard_roots": (i32, [vp, u8p, i32, u64, u8p]),
    "mh_dev_ahtree_append_spine": (i32, [vp, u8p, u64, u64, u8p]),
    "mh_ahtree_verify_batch": (i32, [vp, i32, u64, vp, vp, vp, u8p, u8p, u8p, u8p, u8p]),
    "mh_dev_ahtree_verify_batch": (i32, [vp, i32, u64, vp, vp, vp, u8p, u8p, u8p, u8p, u8p]),
    "mh_tx_alh_batch": (i32, [vp, u64, vp, u8p, u64, u8p, u8p]),
    "mh_dev_tx_alh_batch": (i32, [vp, u64, vp, u8p, u8p, u8p, u8p, u8p]),
    "mh_htree_build_many": (i32, [vp, u64, vp, u8p, u8p]),
    "mh_verify_linear_proof_batch": (i32, [vp, u64, vp, vp, vp, u8p, vp, vp, u8p, u8p, u8p]),
    "mh_verify_dual_proof_v2_batch": (i32, [vp, u64, vp, vp, u8p, u64, vp, u8p, vp, u8p, vp, vp,
                                            u8p, u8p, vp]),
    "mh_verify_dual_proof_batch": (i32, [vp, vp, u8p]),
    "mh_dual_proof_pb_decode_batch": (i32, [vp, u64, u8p, vp, vp, vp]),
    "mh_verify_dual_proof_v2_pb_batch": (i32, [vp, u64, u8p, vp, vp, vp, u8p, u8p, vp]),
    "mh_verify_document_batch": (i32, [vp, vp, vp, u8p]),
    "mh_commit_queue_new": (i32, [vp, i32, u64, u32, u32, C.POINTER(vp)]),
    "mh_commit_queue_free": (i32, [vp]),
    "mh_commit_queue_submit": (i32, [vp, u64, u8p, vp, u8p, vp, u8p, vp, u8p, u8p, u8p, u8p,
                                     u8p]),
    "mh_commit_queue_stats": (i32, [vp, C.POINTER(u64), C.POINTER(u64)]),
    "mh_dual_proof_v2_pb_decode_batch": (i32, [vp, u64, u8p, vp, vp, vp, u8p, vp, u8p, u64, vp,
                                               u8p, u64, vp]),
    "mh_htree_inclusion_proof_pb_decode_batch": (i32, [vp, u64, u8p, vp, vp, vp, vp, u8p, u64, vp]),
    "mh_multi_create": (i32, [i32, vp, C.POINTER(vp)]),
    "mh_multi_destroy": (i32, [vp]),
    "mh_multi_size": (i32, [vp, C.POINTER(i32)]),
    "mh_multi_ctx": (vp, [vp, i32]),
    "mh_multi_synchronize": (i32, [vp]),
    "mh_multi_shard_plan": (i32, [u64, i32, C.POINTER(u64), C.POINTER(u64)]),
    "mh_multi_htree_build_entries_fixed": (i32, [vp, i32, u64, u8p, u32, u8p, u32, u8p, u8p,
                                                 u8p]),
    "mh_multi_dev_htree_build_entries_fixed": (i32, [vp, i32, u64, vp, u32, vp, u32, vp, vp, vp,
                                                     vp]),
    "mh_multi_htree_build_entries": (i32, [vp, i32, u64, u8p, vp, u8p, vp, u8p, vp, u8p,
                                           u8p, u8p, u8p, u8p]),
    "mh_multi_dev_ahtree_append_batch": (i32, [vp, u64, u8p, u64, vp, u32, vp, vp]),
    "mh_multi_ahtree_append_batch": (i32, [vp, u64, u8p, u8p, u64, u32, u8p, u8p]),
    "mh_ahtree_range_plan": (i32, [u64, u64, i32, C.POINTER(i32), vp, C.POINTER(i32)]),
    "mh_ahtree_range_sizes": (i32, [u64, u64, i32, C.POINTER(u64), C.POINTER(u64)]),
    "mh_multi_htree_verify_inclusion_batch": (i32, [vp, u64, u8p, u8p, u8p, u8p, u8p, u8p, u8p]),
    "mh_multi_verify_dual_proof_v2_batch": (i32, [vp, u64, vp, vp, u8p, u64, u8p, u8p, u8p, u8p,
                                                  u8p, u8p, u8p, u8p, vp]),
    "mh_multi_txlog_validate": (i32, [vp, u8p, u64, u32, u32, u64, C.POINTER(u64),
                                      C.POINTER(u64), vp, u8p, vp]),
    "mh_multi_verify_values_batch": (i32, [vp, u64, u8p, vp, vp, u8p, vp, C.POINTER(u64)]),
    "mh_multi_verify_document_batch": (i32, [vp, vp, vp, u8p]),
    "mh_multi_verify_dual_proof_v2_pb_batch": (i32, [vp, u64, u8p, vp, vp, vp, u8p, u8p, vp]),
    "mh_multi_precommit_batch": (i32, [vp, i32, u64, u64, vp, u8p, vp, u8p, vp, u8p, vp, u8p,
                                       u8p, u8p, u8p, u8p, vp]),
    "mh_dev_ahtree_range_local": (i32, [vp, u64, u8p, u64, i32, i32, u8p, u32, u8p, u8p, u8p]),
    "mh_dev_ahtree_range_finish": (i32, [vp, u64, u8p, u64, i32, i32, u8p, u8p, u8p, u8p]),
    "mh_dev_ahtree_append_range": (i32, [vp, u8p, u64, u8p, u8p, u64, u32, u8p]),
    "mh_dev_ahtree_peaks": (i32, [vp, u8p, u64, u8p]),
    "mh_txlog_validate": (i32, [vp, u8p, u64, u32, u32, u64, C.POINTER(u64), C.POINTER(u64), vp,
                                u8p, vp]),
    "mh_txlog_validate_resident": (i32, [vp, u8p, u8p, u64, u32, u32, u64, C.POINTER(u64),
                                         C.POINTER(u64), vp, u8p, vp]),
    "mh_txlog_validate_clog": (i32, [vp, vp, u64, vp, u64, u32, u32, u32, vp, vp, vp,
                                     C.POINTER(u64), C.POINTER(u64)]),
    "mh_commit_pipe_new": (i32, [vp, u64, C.POINTER(vp)]),
    "mh_commit_pipe_free": (i32, [vp]),
    "mh_precommit_batch": (i32, [vp, i32, u64, u64, vp, u8p, vp, u8p, vp, u8p, vp, u8p, u8p, u8p,
                                 u8p, u8p, vp]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load the library (no device access).  Raises if it was not built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ErrNoDevice(MH_ERR_NO_DEVICE,
                                  "libimmustore_merkle.so not built: run __graft_entry__.build()")
            L = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def check(status):
    if status == MH_OK:
        return
    msg = load().mh_status_string(status)
    msg = msg.decode() if msg else "status %d" % status
    if status < 0:
        raise HipError(status, msg)
    raise _ERRORS.get(status, MerkleError)(status, msg)
