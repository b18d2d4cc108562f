"""The appendable file framing of the ahtree logs: the
singleapp header and the multiapp file addressing, through the C ABI
(capi_app.hip: mh_ahtree_log_header, mh_appendable_metadata,
mh_multiapp_segments).  With the record streams the device produces
(AHtree.append_batch_logs, the dLog) these give the bytes of every
data/ tree/ commit/ file and where they go (ahtree.go:106-140,
multi_app.go:120-214, single_app.go:116-171)."""
import ctypes as C
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import _native as N

# multiapp.DefaultOptions (multiapp/options.go:52-66) as ahtree.Open uses them
DEFAULT_FILE_SIZE = 1 << 26  # multiapp DefaultFileSize
NO_COMPRESSION, BEST_SPEED = 0, 1  # appendable.go:25-39
EXT = {"data": "dat", "tree": "sha", "commit": "di"}  # ahtree.go:127-139


def _sized(call) -> bytes:
    n = C.c_uint64(0)
    st = call(None, 0, C.byref(n))
    if st not in (0, 19):  # MH_OK / MH_ERR_BUFFER_TOO_SMALL (size query)
        N.check(st)
    buf = np.zeros(max(n.value, 1), np.uint8)
    N.check(call(buf.ctypes.data, n.value, C.byref(n)))
    return buf[:n.value].tobytes()


def ahtree_log_header(file_size: int = DEFAULT_FILE_SIZE, prealloc_size: int = 0,
                      compression_format: int = NO_COMPRESSION,
                      compression_level: int = BEST_SPEED) -> bytes:
    """Header of every file of an ahtree log (prealloc_size < 0: without the
    PREALLOC_SIZE entry, as in files written before it existed)."""
    L = N.load()
    return _sized(lambda o, c, n: L.mh_ahtree_log_header(file_size, prealloc_size,
                                                         compression_format, compression_level,
                                                         o, c, n))


def metadata_bytes(pairs: Sequence[Tuple[str, bytes]]) -> bytes:
    """appendable.Metadata.Bytes() of the pairs, in the given order."""
    L = N.load()
    k = len(pairs)
    keys = (C.c_char_p * max(k, 1))(*[p[0].encode() for p in pairs])
    bufs = [np.frombuffer(bytes(p[1]) + b"\0", np.uint8) for p in pairs]
    vals = (C.c_void_p * max(k, 1))(*[b.ctypes.data for b in bufs])
    lens = (C.c_uint64 * max(k, 1))(*[len(p[1]) for p in pairs])
    return _sized(lambda o, c, n: L.mh_appendable_metadata(k, keys, vals, lens, o, c, n))


def multiapp_segments(off: int, n: int, file_size: int, header_len: int) -> List[Tuple[int, ...]]:
    """[(file id, position in the file, offset in the range, length)] of the
    logical log bytes [off, off + n)."""
    L = N.load()
    k = C.c_uint32(0)
    N.check(L.mh_multiapp_segments(off, n, file_size, header_len, None, 0, C.byref(k)))
    seg = np.zeros((max(k.value, 1), 4), np.uint64)
    N.check(L.mh_multiapp_segments(off, n, file_size, header_len, seg.ctypes.data, k.value,
                                   C.byref(k)))
    return [tuple(int(x) for x in r) for r in seg[:k.value]]


def write_range(files: Dict[int, bytearray], off: int, data: bytes, file_size: int,
                header: bytes) -> None:
    """Place log bytes [off, off + len(data)) into in-memory file images
    (file id -> bytes, each starting with `header`), as the multiapp would."""
    for fid, pos, src, ln in multiapp_segments(off, len(data), file_size, len(header)):
        f = files.setdefault(fid, bytearray(header))
        if len(f) < pos:
            f.extend(bytes(pos - len(f)))
        f[pos:pos + ln] = data[src:src + ln]


def file_name(kind: str, fid: int) -> str:
    """multiapp appendableName (multi_app.go:204-206) under the ahtree dir."""
    return "%s/%08d.%s" % (kind, fid, EXT[kind])
