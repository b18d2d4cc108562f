#!/bin/bash
# Host code under AddressSanitizer (no GPU needed): the C-ABI library built
# with -Xarch_host -fsanitize=address, the host-only entry points exercised by
# the CPU tests (mh_txlog_scan's multi-threaded hop, ABI exports) and random
# garbage logs of up to 9 MiB.
set -e
cd "$(dirname "$0")/../immustore_amd/csrc"
make -s -j8 EXTRA_FLAGS="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer" \
     OBJDIR=../../build/obj_asan OUT=../../build/lib_asan.so
cd ../../build/obj_asan
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -fsanitize=address -shared-libasan \
     -fno-gpu-sanitize -o ../lib_asan.so *.o
cd ../..
ASAN=$(find /opt/rocm/lib/llvm -name "libclang_rt.asan-x86_64.so" | head -1)
# the sanitizer runtime goes first; anything already preloaded stays in the list
export LD_PRELOAD="$ASAN${LD_PRELOAD:+:$LD_PRELOAD}" ASAN_OPTIONS=detect_leaks=0 MH_LIB_PATH=build/lib_asan.so
python -m pytest tests/test_txlog_scan_cpu.py tests/test_abi.py -q -p no:cacheprovider
python - <<'PY'
import sys; sys.path.insert(0, '.')
import numpy as np
from immustore_amd import txlayer
rng = np.random.default_rng(1)
for n in (0, 1, 50, 1000, 100000, 9 << 20):
    txlayer.txlog_scan(rng.integers(0, 256, n, dtype=np.uint8))
print("asan: garbage scans clean")
PY
