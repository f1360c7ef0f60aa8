# Build recipe (no cmake needed).  `python -c "import __graft_entry__ as g; g.build()"`
# runs the same commands.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CC ?= gcc

LIB := rusty_enet_amd/lib/libenet_crc_amd.so
ORACLE := oracle/liboracle_crc32.so
ORACLE_RANGE := oracle/liboracle_range.so
HIP_SRC := rusty_enet_amd/csrc/crc32_kernels.hip rusty_enet_amd/csrc/crc32_mailbox.hip rusty_enet_amd/csrc/crc32_slot.hip rusty_enet_amd/csrc/enet_crc_abi.hip rusty_enet_amd/csrc/range_coder.hip
HIP_DEP := $(HIP_SRC) $(wildcard rusty_enet_amd/csrc/*.hpp) include/enet_crc_amd.h include/enet_range_amd.h
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++20 -fPIC -fvisibility=hidden -Wall

# The same sources with compile-time test hooks (a failing staging chunk, a server that
# never answers a 4095-byte request, a 200-ms call timeout): loaded only by
# tests/test_gpu_hooks.py through ENET_CRC_AMD_LIB, never by the product.
TESTLIB := rusty_enet_amd/lib/variants/libenet_crc_amd_testhooks.so

# Same-process HBM read ceiling (bench.py's roofline.read_ceiling_gbs; tooling, not product).
CEILING := tools/lib/libenet_read_ceiling.so

all: $(LIB) $(TESTLIB) $(ORACLE) $(ORACLE_RANGE) $(CEILING)

$(CEILING): tools/ceiling/read_ceiling.hip
	mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

$(LIB): $(HIP_DEP)
	mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_SRC)

$(TESTLIB): $(HIP_DEP)
	mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DENET_CRC_TEST_HOOKS -shared -o $@ $(HIP_SRC)

$(ORACLE): oracle/crc32_oracle.c
	$(CC) -O2 -fPIC -shared -pthread -Wall -o $@ $<

clean:
	rm -f $(LIB) $(TESTLIB) $(ORACLE) $(ORACLE_RANGE) $(CEILING)

.PHONY: all clean

$(ORACLE_RANGE): oracle/range_coder_oracle.c
	$(CC) -O2 -fPIC -shared -Wall -o $@ $<

# A/B builds of the library with compile-time variant switches (never the product):
#   make variant NAME=nolines DEFS=-DENET_CRC_NO_LINES
#   -> rusty_enet_amd/lib/variants/libenet_crc_amd_nolines.so, loaded with ENET_CRC_AMD_LIB.
variant: $(HIP_DEP)
	mkdir -p rusty_enet_amd/lib/variants
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o rusty_enet_amd/lib/variants/libenet_crc_amd_$(NAME).so $(HIP_SRC)

.PHONY: variant

# Host code under AddressSanitizer + UBSan: crc32_host.hpp (shard split,
# slot correction, merge, staging chunks) and the C oracle, built with g++/gcc and run.
ASAN_FLAGS := -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all
asan: tests/cpp/bin/host_asan
	ASAN_OPTIONS=detect_leaks=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1 tests/cpp/bin/host_asan

tests/cpp/bin/host_asan: tests/cpp/host_asan.cpp oracle/crc32_oracle.c oracle/range_coder_oracle.c rusty_enet_amd/csrc/crc32_host.hpp rusty_enet_amd/csrc/crc32_slot.hpp rusty_enet_amd/csrc/crc32_ops.hpp
	mkdir -p tests/cpp/bin
	$(CC) $(ASAN_FLAGS) -c -o tests/cpp/bin/crc32_oracle_asan.o oracle/crc32_oracle.c
	$(CC) $(ASAN_FLAGS) -c -o tests/cpp/bin/range_oracle_asan.o oracle/range_coder_oracle.c
	g++ -std=c++20 $(ASAN_FLAGS) -fconstexpr-ops-limit=1000000000 -o $@ tests/cpp/host_asan.cpp \
	  tests/cpp/bin/crc32_oracle_asan.o tests/cpp/bin/range_oracle_asan.o -lpthread

.PHONY: asan

# Measurement probes (tooling, not product): tools/dma_probe, and round 6's
# load-shape probes tools/dma_shape, tools/shape_arith, tools/lines_probe.
probes: tools/dma_probe tools/dma_shape tools/shape_arith tools/lines_probe
tools/dma_probe: tools/dma_probe.hip rusty_enet_amd/csrc/crc32_layout.hpp rusty_enet_amd/csrc/crc32_ops.hpp
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++20 -o $@ tools/dma_probe.hip
tools/dma_shape: tools/dma_shape.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -o $@ tools/dma_shape.hip
tools/shape_arith tools/lines_probe: tools/%: tools/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++20 -o $@ $<

.PHONY: probes
