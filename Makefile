# Build libchunkio_amd.so (HIP kernels for gfx950 + C ABI) and the oracle.
# `python -c "import __graft_entry__ as g; g.build()"` drives this file.

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
OUT     := chunkio_amd/lib
LIB     := $(OUT)/libchunkio_amd.so
SRC     := chunkio_amd/csrc
BLD     := build
INC     := -Iinclude -I$(SRC)

CFLAGS   := -O3 -fPIC -Wall -Wextra -std=gnu11 $(INC)
HIPFLAGS := -O3 -fPIC --offload-arch=$(ARCH) -std=c++17 -Wall $(INC) -munsafe-fp-atomics \
            -mllvm -amdgpu-atomic-optimizer-strategy=None -mllvm -amdgpu-kernarg-preload-count=9

COBJS   := $(BLD)/host_copy.o $(BLD)/crc32_host.o $(BLD)/crc32_scalar.o $(BLD)/cio_verify.o $(BLD)/cio_sync.o $(BLD)/cioa_chunk.o $(BLD)/crc_route.o $(BLD)/crc_cpu_batch.o $(BLD)/cio_sha1.o
HOBJS   := $(BLD)/crc32_gpu.o $(BLD)/host_pipeline.o $(BLD)/sha1_gpu.o

CTEST   := tests/c/bin
REF_INC := /root/reference/include/chunkio/cio_crc32.h
REF_SHA1 := /root/reference/src/cio_sha1.c
CTESTS  := $(CTEST)/test_crc32_dropin $(CTEST)/test_chunk_api $(CTEST)/test_multi $(CTEST)/test_sha1 \
           $(if $(wildcard $(REF_INC)),$(CTEST)/test_crc32_dropin_ref) $(if $(wildcard $(REF_SHA1)),$(CTEST)/test_sha1_ref)
CLINK   := -Lchunkio_amd/lib -lchunkio_amd -Wl,-rpath,'$$ORIGIN/../../../chunkio_amd/lib'

all: $(LIB) oracle ctests

# C callers of the public headers (tests/test_c_api.py runs them).  The _ref
# variant compiles the reference's own include/chunkio/cio_crc32.h, unmodified,
# against include/crc32/crc32.h (only where /root/reference exists).
ctests: $(CTESTS)

$(CTEST)/test_crc32_dropin: tests/c/test_crc32_dropin.c $(LIB) include/crc32/crc32.h
	@mkdir -p $(CTEST)
	$(CC) -O2 -Wall -Wextra -std=gnu11 -Iinclude -o $@ $< $(CLINK)

$(CTEST)/test_crc32_dropin_ref: tests/c/test_crc32_dropin.c $(LIB) include/crc32/crc32.h
	@mkdir -p $(CTEST)
	$(CC) -O2 -Wall -Wextra -std=gnu11 -DCIOA_REF_BOUNDARY -Iinclude -I/root/reference/include -o $@ $< $(CLINK)

# chunkio's cio_sha1 API: the library's exports, and the reference's own
# cio_sha1.h + cio_sha1.c (unmodified, compiled where they lie) over
# include/sha1/sha1.h -- include/ ahead of the reference's include/.
$(CTEST)/test_sha1: tests/c/test_sha1.c $(LIB) include/sha1/sha1.h include/chunkio_amd/cio_sha1.h
	@mkdir -p $(CTEST)
	$(CC) -O2 -Wall -Wextra -std=gnu11 -Iinclude -o $@ $< $(CLINK)

$(CTEST)/test_sha1_ref: tests/c/test_sha1.c $(REF_SHA1) $(LIB) include/sha1/sha1.h
	@mkdir -p $(CTEST)
	$(CC) -O2 -Wall -std=gnu11 -DCIOA_REF_BOUNDARY -Iinclude -I/root/reference/include -o $@ $< $(REF_SHA1) $(CLINK)

$(CTEST)/test_chunk_api: tests/c/test_chunk_api.c $(LIB) $(wildcard include/*/*.h)
	@mkdir -p $(CTEST)
	$(CC) -O2 -Wall -Wextra -std=gnu11 -Iinclude -o $@ $< $(CLINK)

$(CTEST)/test_multi: tests/c/test_multi.c $(LIB) include/chunkio_amd/cio_crc32_gpu.h
	@mkdir -p $(CTEST)
	$(CC) -O2 -Wall -Wextra -std=gnu11 -Iinclude -o $@ $< $(CLINK) -lpthread

$(BLD)/%.o: $(SRC)/%.c $(wildcard $(SRC)/*.h) $(wildcard include/*/*.h)
	@mkdir -p $(BLD)
	$(CC) $(CFLAGS) -c -o $@ $<

$(BLD)/%.o: $(SRC)/%.hip $(wildcard $(SRC)/*.h) $(wildcard include/*/*.h)
	@mkdir -p $(BLD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(COBJS) $(HOBJS)
	@mkdir -p $(OUT)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread

oracle:
	$(MAKE) -C oracle

# A/B variant of the library: make ablib VAR=name DEFS="-DFOO" -> chunkio_amd/lib/ab/name.so
ablib:
	@mkdir -p $(OUT)/ab $(BLD)/ab
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c -o $(BLD)/ab/crc32_gpu_$(VAR).o $(SRC)/crc32_gpu.hip
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(OUT)/ab/$(VAR).so $(COBJS) $(BLD)/ab/crc32_gpu_$(VAR).o $(BLD)/host_pipeline.o $(BLD)/sha1_gpu.o -lpthread

# Same for the SHA-1 kernel: make ablib_sha1 VAR=name DEFS="-DCIO_SHA1_CHAINS=32"
ablib_sha1:
	@mkdir -p $(OUT)/ab $(BLD)/ab
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c -o $(BLD)/ab/sha1_gpu_$(VAR).o $(SRC)/sha1_gpu.hip
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $(OUT)/ab/$(VAR).so $(COBJS) $(BLD)/crc32_gpu.o $(BLD)/host_pipeline.o $(BLD)/ab/sha1_gpu_$(VAR).o -lpthread

asm: $(SRC)/crc32_gpu.hip
	@mkdir -p $(BLD)/asm
	$(HIPCC) $(HIPFLAGS) --offload-device-only -S -o $(BLD)/asm/crc32_gpu.s $<

# make install PREFIX=/usr/local: the library, the public headers (crc32/crc32.h,
# sha1/sha1.h, chunkio_amd/*.h) and a pkg-config file, for a chunkio build to
# link against.
PREFIX ?= /usr/local
install: $(LIB)
	install -d $(DESTDIR)$(PREFIX)/lib/pkgconfig $(DESTDIR)$(PREFIX)/include/crc32 \
	    $(DESTDIR)$(PREFIX)/include/sha1 $(DESTDIR)$(PREFIX)/include/chunkio_amd
	install -m 755 $(LIB) $(DESTDIR)$(PREFIX)/lib/
	install -m 644 include/crc32/crc32.h $(DESTDIR)$(PREFIX)/include/crc32/
	install -m 644 include/sha1/sha1.h $(DESTDIR)$(PREFIX)/include/sha1/
	install -m 644 include/chunkio_amd/*.h $(DESTDIR)$(PREFIX)/include/chunkio_amd/
	printf 'prefix=%s\nlibdir=$${prefix}/lib\nincludedir=$${prefix}/include\n\nName: chunkio_amd\nDescription: MI355X-native CRC-32 / SHA-1 path of fluent/chunkio (drop-in crc32.h, batched GPU calls)\nVersion: 0.5.0\nLibs: -L$${libdir} -lchunkio_amd\nCflags: -I$${includedir}\n' \
	    "$(PREFIX)" > $(DESTDIR)$(PREFIX)/lib/pkgconfig/chunkio_amd.pc

clean:
	rm -rf $(BLD) $(LIB) $(CTEST)
	$(MAKE) -C oracle clean

.PHONY: all oracle asm clean ctests ablib ablib_sha1 install
