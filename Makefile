# Build recipe (no cmake needed).  `python -c "import __graft_entry__ as g; g.build()"`
# runs the same commands.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CC ?= gcc

LIB := rusty_enet_amd/lib/libenet_crc_amd.so
ORACLE := oracle/liboracle_crc32.so
HIP_SRC := rusty_enet_amd/csrc/crc32_kernels.hip rusty_enet_amd/csrc/crc32_slot.hip rusty_enet_amd/csrc/enet_crc_abi.hip
HIP_DEP := $(HIP_SRC) $(wildcard rusty_enet_amd/csrc/*.hpp) include/enet_crc_amd.h
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++20 -fPIC -fvisibility=hidden -Wall

all: $(LIB) $(ORACLE)

$(LIB): $(HIP_DEP)
	mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_SRC)

$(ORACLE): oracle/crc32_oracle.c
	$(CC) -O2 -fPIC -shared -pthread -Wall -o $@ $<

clean:
	rm -f $(LIB) $(ORACLE)

.PHONY: all clean
