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

all: $(LIB) $(TESTLIB) $(ORACLE) $(ORACLE_RANGE)

$(LIB): $(HIP_DEP)
	mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_SRC)

$(TESTLIB): $(HIP_DEP)
	mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DENET_CRC_TEST_HOOKS -shared -o $@ $(HIP_SRC)

$(ORACLE): oracle/crc32_oracle.c
	$(CC) -O2 -fPIC -shared -pthread -Wall -o $@ $<

clean:
	rm -f $(LIB) $(TESTLIB) $(ORACLE) $(ORACLE_RANGE)

.PHONY: all clean

$(ORACLE_RANGE): oracle/range_coder_oracle.c
	$(CC) -O2 -fPIC -shared -Wall -o $@ $<

# A/B builds of the library with compile-time variant switches (never the product):
#   make variant NAME=region DEFS=-DENET_CRC_REGION_RAGGED
#   -> rusty_enet_amd/lib/variants/libenet_crc_amd_region.so, loaded with ENET_CRC_AMD_LIB.
variant: $(HIP_DEP)
	mkdir -p rusty_enet_amd/lib/variants
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o rusty_enet_amd/lib/variants/libenet_crc_amd_$(NAME).so $(HIP_SRC)

.PHONY: variant
