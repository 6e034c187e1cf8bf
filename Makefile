# vccl-mi355x build: hand-written HIP for gfx950 + host C++ into one C-ABI
# shared library (vccl_amd/lib/libvccl.so), plus the CPU oracle (test-only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS := -std=c++20 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
            --offload-arch=$(ARCH) -I include $(DEFS)
# Experiment builds: `make VARIANT=_x DEFS=-DVCCL_RING_SRC_POL=2` builds
# vccl_amd/lib/libvccl_x.so (selected at run time with VCCL_LIB=...).
VARIANT ?=
OBJ := build/obj$(VARIANT)
LIB := vccl_amd/lib/libvccl$(VARIANT).so
DEV := vccl_amd/csrc/device
HOST := vccl_amd/csrc/host
KTS := 0 1 2 3 4 5 6 7 8
HDRS := $(wildcard $(DEV)/*.hpp) $(wildcard $(HOST)/*.h) $(wildcard include/*.h)

RC_OBJS := $(foreach k,$(KTS),$(OBJ)/rc_kernels_$(k).o)
RING_OBJS := $(foreach k,$(KTS),$(OBJ)/ring_kernels_$(k).o)
API_OBJS := $(OBJ)/rc_api.o
HOST_OBJS := $(patsubst $(HOST)/%.cc,$(OBJ)/host_%.o,$(wildcard $(HOST)/*.cc))

PERF := vccl_amd/lib/coll_perf

all: $(LIB) $(PERF) oracle

# nccl-tests-style driver linked against the C API only (tools/coll_perf.hip)
$(PERF): tools/coll_perf.hip include/nccl.h $(LIB)
	$(HIPCC) -std=c++20 -O2 --offload-arch=$(ARCH) -I include $< -o $@ -L vccl_amd/lib -lvccl \
	  -Wl,-rpath,'$$ORIGIN'

$(LIB): $(RC_OBJS) $(RING_OBJS) $(API_OBJS) $(HOST_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -lpthread

$(OBJ)/rc_kernels_%.o: $(DEV)/rc_kernels.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -DVCCL_KT=$* -c $< -o $@

$(OBJ)/ring_kernels_%.o: $(DEV)/ring_kernels.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -DVCCL_KT=$* -c $< -o $@

$(OBJ)/rc_api.o: $(DEV)/rc_api.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(OBJ)/host_%.o: $(HOST)/%.cc $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -x hip --offload-host-only -c $< -o $@

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) $(PERF)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
