#!/bin/bash
# Host-code AddressSanitizer + UndefinedBehaviorSanitizer check of the library.
#
#   bash tools/asan_check.sh build      # here (CPU container): sanitized build
#   bash tools/asan_check.sh host       # the C replays on the host CRC route
#   bash tools/asan_check.sh gpu        # the same replays with every verify /
#                                       # sync on the GPU route (host pipeline)
#   bash tools/asan_check.sh tsan       # here: ThreadSanitizer build + the host
#                                       # route on the 8-thread CRC pool
#   bash tools/asan_check.sh tsan-gpu   # that build's replay on the GPU route
#
# Every host source of libchunkio_amd.so is instrumented: the C files with
# clang, and the host side of the .hip files (each -fsanitize= after
# -Xarch_host, so device code is built exactly as in the product).  The
# sanitized library goes to chunkio_amd/lib/asan/, the C callers of the public
# headers (tests/c: the reference's fs.c / metadata_update.c replayed through
# cioa_chunk.h, and the crc32.h drop-in) to tests/c/bin/asan/, linked with the
# static ASan runtime so it comes first without any preload.  Leak detection
# is on; any report fails the run.
set -euo pipefail
cd "$(dirname "$0")/.."
MODE=${1:-build}
CL=/opt/rocm/lib/llvm/bin/clang
HIPCC=/opt/rocm/bin/hipcc
OBJ=build/asan
LIBD=chunkio_amd/lib/asan
BIN=tests/c/bin/asan
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
INC="-Iinclude -Ichunkio_amd/csrc"

case "$MODE" in
build)
    mkdir -p $OBJ $LIBD $BIN
    for f in host_copy crc32_host crc32_scalar cio_verify cio_sync cioa_chunk crc_route crc_cpu_batch cio_sha1; do
        $CL -O2 -g -fPIC -Wall -std=gnu11 $SAN $INC -c -o $OBJ/$f.o chunkio_amd/csrc/$f.c
    done
    for f in crc32_gpu host_pipeline sha1_gpu; do
        $HIPCC -O3 -g -fPIC --offload-arch=gfx950 -std=c++17 $INC -munsafe-fp-atomics \
            -mllvm -amdgpu-atomic-optimizer-strategy=None -mllvm -amdgpu-kernarg-preload-count=9 \
            $HSAN -c -o $OBJ/$f.o chunkio_amd/csrc/$f.hip
    done
    $HIPCC -shared -fPIC --offload-arch=gfx950 -o $LIBD/libchunkio_amd.so $OBJ/*.o -lpthread
    for t in test_chunk_api test_crc32_dropin test_multi test_sha1; do
        $CL -O1 -g -Wall -std=gnu11 $SAN -Iinclude -o $BIN/$t tests/c/$t.c \
            -L$LIBD -lchunkio_amd -Wl,-rpath,'$ORIGIN/../../../../chunkio_amd/lib/asan' -lpthread
    done
    echo "built $LIBD/libchunkio_amd.so, $BIN/{test_chunk_api,test_crc32_dropin,test_multi,test_sha1}"
    ;;
host|gpu)
    DATA=tests/golden/400kb.txt
    W=$(mktemp -d /tmp/cioa-asan-XXXXXX)
    trap 'rm -rf "$W"' EXIT
    export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1
    export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
    timeout -k 10 300 $BIN/test_crc32_dropin $DATA
    timeout -k 10 300 $BIN/test_sha1 $DATA 0:0 3:1,63,64,65,1000 7:55,56,57,409000 > /dev/null
    if [ "$MODE" = host ]; then
        for th in 1 8; do
            for m in immediate deferred; do   # deferred compares with immediate's files
                CIOA_CPU_CRC_MAX=$((1 << 62)) CIOA_HOST_CRC_THREADS=$th \
                    timeout -k 10 900 $BIN/test_chunk_api $DATA "$W" $m | tail -1
            done
        done
    else
        # Memory errors and UB only: leak checking stays in the host mode (the
        # ROCm runtime's init-time allocations are not freed at exit, and the
        # library's per-device pipelines are process-lifetime pools).  No
        # quarantine: ROCm's ASan runtime tracks HSA pool allocations, and one
        # still quarantined when libamdhip64's destructors unload the runtime
        # trips its "device runtime unloaded" CHECK at exit (seen in r04ao).
        export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:quarantine_size_mb=0
        # CIOA_CPU_CRC_MAX=0: every batch on the GPU alone; =1 with
        # CIOA_SPLIT_ROUTE=2: every batch of two or more chunks on the split
        # route (GPU helper thread + host, learned rates)
        for cm in 0 1; do
            for m in immediate deferred; do
                CIOA_CPU_CRC_MAX=$cm CIOA_SPLIT_ROUTE=$((cm * 2)) timeout -k 10 300 $BIN/test_chunk_api $DATA "$W" $m
            done
        done
        timeout -k 10 300 $BIN/test_multi "$W"
    fi
    echo "asan $MODE: clean"
    ;;
tsan|tsan-gpu)
    # Same sources with -fsanitize=thread (host code only): objects in
    # build/tsan, library and replay in chunkio_amd/lib/tsan, tests/c/bin/tsan
    # (so a GPU box gets them).  tsan builds and runs the host route on the
    # 8-thread CRC pool; tsan-gpu runs the prebuilt replay on the GPU route.
    T=build/tsan
    TL=chunkio_amd/lib/tsan
    TB=tests/c/bin/tsan
    if [ "$MODE" = tsan ]; then
        mkdir -p $T $TL $TB
        for f in host_copy crc32_host crc32_scalar cio_verify cio_sync cioa_chunk crc_route crc_cpu_batch cio_sha1; do
            $CL -O1 -g -fPIC -std=gnu11 -fsanitize=thread $INC -c -o $T/$f.o chunkio_amd/csrc/$f.c
        done
        for f in crc32_gpu host_pipeline sha1_gpu; do
            $HIPCC -O3 -g -fPIC --offload-arch=gfx950 -std=c++17 $INC -munsafe-fp-atomics \
                -mllvm -amdgpu-atomic-optimizer-strategy=None -mllvm -amdgpu-kernarg-preload-count=9 \
                -Xarch_host -fsanitize=thread -c -o $T/$f.o chunkio_amd/csrc/$f.hip
        done
        $HIPCC -shared -fPIC --offload-arch=gfx950 -o $TL/libchunkio_amd.so $T/*.o -lpthread
        for t in test_chunk_api test_multi; do
            $CL -O1 -g -std=gnu11 -fsanitize=thread -Iinclude -o $TB/$t tests/c/$t.c \
                -L$TL -lchunkio_amd -Wl,-rpath,'$ORIGIN/../../../../chunkio_amd/lib/tsan' -lpthread
        done
    fi
    W=$(mktemp -d /tmp/cioa-tsan-XXXXXX)
    trap 'rm -rf "$W"' EXIT
    export TSAN_OPTIONS=halt_on_error=1
    for m in immediate deferred; do
        if [ "$MODE" = tsan ]; then
            CIOA_CPU_CRC_MAX=$((1 << 62)) CIOA_HOST_CRC_THREADS=8 \
                timeout -k 10 900 $TB/test_chunk_api tests/golden/400kb.txt "$W" $m | tail -1
        else
            for cm in 0 1; do
                TSAN_OPTIONS=halt_on_error=1:suppressions=$PWD/tools/tsan_rocm.supp CIOA_CPU_CRC_MAX=$cm \
                    CIOA_SPLIT_ROUTE=$((cm * 2)) timeout -k 10 300 $TB/test_chunk_api tests/golden/400kb.txt "$W" $m
            done
        fi
    done
    if [ "$MODE" = tsan-gpu ]; then
        TSAN_OPTIONS=halt_on_error=1:suppressions=$PWD/tools/tsan_rocm.supp \
            timeout -k 10 300 $TB/test_multi "$W"
    fi
    echo "$MODE: clean"
    ;;
*)
    echo "usage: $0 build|host|gpu|tsan|tsan-gpu" >&2
    exit 2
    ;;
esac
