# Build libpps_hip.so (gfx950): the HIP kernels + the C ABI (include/pps_abi.h).
# `python -c "import __graft_entry__ as g; g.build()"` drives the same recipe.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRCS := $(wildcard pps_amd/csrc/*.hip)
OBJS := $(patsubst pps_amd/csrc/%.hip,build/%.o,$(SRCS))
LIB := pps_amd/libpps_hip.so

all: $(LIB)

# the GEMM kernels interleave their f32 split arithmetic with MFMAs: keep it
# scalar (SLP-packed v_pk_add_f32 issues at half rate beside MFMAs)
build/gemm_x3p.o: HIPFLAGS += -fno-slp-vectorize

build/%.o: pps_amd/csrc/%.hip pps_amd/csrc/pps_internal.hpp pps_amd/csrc/gemm_common.hpp pps_amd/csrc/gemm_x3_common.hpp pps_amd/csrc/gemm_x3p_common.hpp include/pps_abi.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# relink when a source file is added or removed (not only when one changes)
build/srcs.list: FORCE
	@mkdir -p build
	@echo '$(SRCS)' | cmp -s - $@ || echo '$(SRCS)' > $@

$(LIB): $(OBJS) build/srcs.list
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean FORCE
FORCE:
