#!/usr/bin/env bash
# SURVEY.md §8(b) drop-in proof: the UNMODIFIED chunkio library, tests and
# tools/cio, built by their own CMake from a /tmp copy of /root/reference,
# once as shipped and once with cio-crc32 (deps/crc32) replaced by
# libchunkio_amd.so; the reference's ctest must pass 5/5 in both, the second
# once per host CRC path (CIOA_HOST_CRC=table|clmul|auto).
#
# Boundary and harness evidence only: the oracle is oracle/_ref (deps/crc32
# compiled by gcc), never this build.  Nothing under /root/reference is
# written; the copy and both build trees live under $WORK.
#
# The only edits to the copy (all reported in the log as a diff):
#   src/CMakeLists.txt:16   set(libs cio-crc32) -> set(libs <repo>/chunkio_amd/lib/libchunkio_amd.so)
#   src/CMakeLists.txt:13   cio_sha1.c added to the source list (the reference leaves it out;
#                           it compiles unmodified against include/sha1/sha1.h)
#   CMakeLists.txt          include_directories(BEFORE <repo>/include) ahead of deps/,
#                           so <crc32/crc32.h> resolves to include/crc32/crc32.h
#
# Usage: tools/ref_dropin_ctest.sh [WORK=/tmp/cioa_ref_dropin]
# Prints "DROPIN_CTEST_OK" last on success.  Leaves the reference binary
# $WORK/stock/build{,-release}/tools/cio (Debug as CIO_DEV builds it, and
# -O3) for tools/ref_perf_timing.py.
set -euo pipefail

REF=${REF:-/root/reference}
REPO=$(cd "$(dirname "$0")/.." && pwd)
WORK=${1:-/tmp/cioa_ref_dropin}
SHIM=$REPO/chunkio_amd/lib/libchunkio_amd.so
JOBS=${JOBS:-8}

[ -f "$REF/CMakeLists.txt" ] || { echo "no reference tree at $REF"; exit 3; }
[ -f "$SHIM" ] || { echo "build $SHIM first (make)"; exit 3; }

rm -rf "$WORK"
mkdir -p "$WORK"

copy_ref() {
    mkdir -p "$1"
    (cd "$REF" && tar --exclude=./build -cf - .) | (cd "$1" && tar -xf -)
}

build() {   # $1 = tree, $2 = build dir name, then cmake options
    local tree=$1 bdir=$2
    shift 2
    cmake -S "$tree" -B "$tree/$bdir" "$@" >"$tree/$bdir.cmake.log" 2>&1 ||
        { cat "$tree/$bdir.cmake.log"; exit 1; }
    cmake --build "$tree/$bdir" -j "$JOBS" >"$tree/$bdir.build.log" 2>&1 || { tail -50 "$tree/$bdir.build.log"; exit 1; }
}

echo "== reference: $REF ($(cd "$REF" && git rev-parse --short HEAD 2>/dev/null || echo no-git))"
echo "== cmake: $(cmake --version | head -1), cc: $(cc --version | head -1)"

# 1. as shipped (CIO_DEV forces a Debug build with the tests); plus an
#    optimised build of tools/cio alone for tools/ref_perf_timing.py
copy_ref "$WORK/stock"
build "$WORK/stock" build -DCIO_DEV=On
build "$WORK/stock" build-release -DCMAKE_BUILD_TYPE=Release
check5() {   # ctest summary line: "100% tests passed[, 0 tests failed] out of 5"
    echo "$1" | grep -Eq "^100% tests passed(, 0 tests failed)? out of 5\$" || { echo "$1"; echo "not 5/5"; exit 1; }
}
echo "== stock build: ctest"
out=$(cd "$WORK/stock/build" && ctest --output-on-failure 2>&1) || { echo "$out"; exit 1; }
echo "$out" | tail -12
check5 "$out"

# 2. cio-crc32 replaced by the shim
copy_ref "$WORK/shim"
sed -i "16s|^set(libs cio-crc32)\$|set(libs $SHIM)|" "$WORK/shim/src/CMakeLists.txt"
grep -q "^set(libs $SHIM)\$" "$WORK/shim/src/CMakeLists.txt" || { echo "src/CMakeLists.txt:16 not as expected"; exit 1; }
# the SHA-1 wrapper, which the reference's CMake leaves out: compiled unmodified
# against include/sha1/sha1.h (round 6), into the same library
sed -i "13s|^  chunkio.c\$|  chunkio.c\n  cio_sha1.c|" "$WORK/shim/src/CMakeLists.txt"
grep -q "^  cio_sha1.c\$" "$WORK/shim/src/CMakeLists.txt" || { echo "src/CMakeLists.txt:13 not as expected"; exit 1; }
awk -v inc="$REPO/include" '
    /^include_directories\($/ && !done { print "include_directories(BEFORE " inc ")"; done = 1 }
    { print }' "$WORK/shim/CMakeLists.txt" >"$WORK/shim/CMakeLists.txt.new"
mv "$WORK/shim/CMakeLists.txt.new" "$WORK/shim/CMakeLists.txt"
echo "== edits to the copy:"
(cd "$WORK" && diff -u "$REF/src/CMakeLists.txt" shim/src/CMakeLists.txt;
               diff -u "$REF/CMakeLists.txt" shim/CMakeLists.txt) | grep '^[-+][^-+]' || true
build "$WORK/shim" build -DCIO_DEV=On

# The link really takes crc_update from the shim: the test binaries need
# libchunkio_amd.so, the static library leaves crc_update undefined, no
# cio-crc32 archive is on any link line, and the compile saw our header.
B=$WORK/shim/build
echo "== link evidence"
for t in "$B"/tests/cio-test-* "$B"/tools/cio; do
    [ -x "$t" ] || continue
    printf '%-28s %s\n' "$(basename "$t")" "$(ldd "$t" | grep -o 'libchunkio_amd.so => [^ ]*' || echo 'NOT LINKED')"
    ldd "$t" | grep -q "libchunkio_amd.so => $SHIM" || { echo "$t does not load the shim"; exit 1; }
done
nm "$B"/src/libchunkio-static.a 2>/dev/null | grep -E ' [UT] crc_update$' | sort | uniq -c
if nm "$B"/src/libchunkio-static.a | grep -q ' T crc_update$'; then echo "crc_update defined inside chunkio"; exit 1; fi
if grep -rl "libcio-crc32.a" "$B" --include=link.txt --include=*.make --include=build.ninja 2>/dev/null | grep -v deps/crc32; then
    echo "cio-crc32 still on a link line"; exit 1
fi
grep -h -o "$REPO/include/crc32/crc32.h" "$B"/src/CMakeFiles/chunkio-static.dir/*.d 2>/dev/null | sort -u |
    sed 's/^/header seen by src\/: /' || true

# cio_sha1.c from the reference's own source list: defined in chunkio's static
# library, its SHA1_* calls resolved by the shim (cioa_SHA1_*); a C caller of
# the reference's cio_sha1.h linked against both gets OpenSSL's digest
echo "== cio_sha1 (src/cio_sha1.c compiled by the reference's CMake against include/sha1/sha1.h)"
nm "$B"/src/libchunkio-static.a | grep -E ' [TU] (cio_sha1_hash|cioa_SHA1_Init)$' | sort -u
nm "$B"/src/libchunkio-static.a | grep -q ' T cio_sha1_hash$' || { echo "cio_sha1.c not in chunkio"; exit 1; }
nm "$B"/src/libchunkio-static.a | grep -q ' U cioa_SHA1_Init$' || { echo "SHA1_Init not taken from the shim"; exit 1; }
cc -O2 -std=gnu11 -DCIOA_REF_BOUNDARY -I"$REPO/include" -I"$REF/include" -o "$WORK/test_sha1_cmake" \
    "$REPO/tests/c/test_sha1.c" "$B"/src/libchunkio-static.a "$SHIM" -Wl,-rpath,"$(dirname "$SHIM")"
got=$("$WORK/test_sha1_cmake" "$REPO/tests/golden/400kb.txt" 0:409600 | awk '/^hash /{print $2}')
want=$(python3 -c "import hashlib,sys; print(hashlib.sha1(open(sys.argv[1],'rb').read()).hexdigest())" "$REPO/tests/golden/400kb.txt")
echo "cio_sha1_hash(400kb.txt) = $got (hashlib $want)"
[ "$got" = "$want" ] || { echo "cio_sha1 digest differs"; exit 1; }

for mode in table clmul auto; do
    echo "== shim build: ctest, CIOA_HOST_CRC=$mode"
    out=$(cd "$B" && CIO_GPU_DIAG=1 CIOA_HOST_CRC=$mode ctest --output-on-failure 2>&1) || { echo "$out"; exit 1; }
    echo "$out" | tail -9
    check5 "$out"
done
echo "DROPIN_CTEST_OK"
