# Builds the product library (gfx950) and the oracle/CPU-baseline library.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -pthread
SRC := pfs_amd/csrc/cdc_kernels.hip pfs_amd/csrc/pfscdc.cpp pfs_amd/csrc/writer.cpp pfs_amd/csrc/fileset.cpp pfs_amd/csrc/group.cpp pfs_amd/csrc/gorand.cpp pfs_amd/csrc/knobs.cpp
HDR := include/pfscdc.h pfs_amd/csrc/pfscdc_internal.h

all: pfs_amd/libpfscdc.so oracle/_build/liboracle.so

pfs_amd/libpfscdc.so: $(SRC) $(HDR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -x hip $(filter %.hip %.cpp,$(SRC)) -o $@

oracle/_build/liboracle.so: oracle/cdc_oracle.c oracle/Makefile
	$(MAKE) -C oracle

clean:
	rm -f pfs_amd/libpfscdc.so oracle/_build/liboracle.so

.PHONY: all clean
