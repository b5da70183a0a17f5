# Build for MI355X (gfx950).  `make` builds the product library and the CPU
# oracle; __graft_entry__.build() runs it.  Outputs stay in-tree (git-ignored)
# so they travel to the GPU box with the snapshot.
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
CXX       ?= g++
CC        ?= gcc
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-result
CXXFLAGS  := -O3 -mpopcnt -std=c++17 -fPIC -fopenmp -Iinclude -Wall
CFLAGS    := -O2 -std=c11 -fPIC -fopenmp -Wall -D_GNU_SOURCE

PKG       := dag_rider_amd
LIB       := $(PKG)/libdagrider_gpu.so
# profiling build (per-query sweep phase timings, tools/sweep_timing.py); never loaded by tests or the bench
LIBT      := $(PKG)/libdagrider_gpu_timing.so
ORACLE    := oracle/liboracle.so
BUILD     := build

.PHONY: all lib oracle clean tests-cpp timing FORCE
all: lib oracle tests-cpp timing
timing: $(LIBT)

lib: $(LIB)
oracle: $(ORACLE)

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/dag_gen.o: $(PKG)/csrc/dag_gen.cpp include/dagrider_gen.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/wire.o: $(PKG)/csrc/wire.cpp include/dagrider_wire.h include/dagrider_gpu.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/host_rounds.o: $(PKG)/csrc/host_rounds.cpp $(PKG)/csrc/host_rounds.hpp include/dagrider_gpu.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

ENGINE_DEPS := $(PKG)/csrc/engine.hip $(PKG)/csrc/kernels.hpp $(PKG)/csrc/wave_ops.hpp $(PKG)/csrc/replay_plan.hpp $(PKG)/csrc/batch.hpp $(PKG)/csrc/batch1w.hpp $(PKG)/csrc/general.hpp $(PKG)/csrc/host_rounds.hpp include/dagrider_gpu.h
SHARD_DEPS  := $(PKG)/csrc/shard.hip $(PKG)/csrc/shard_memo.hpp $(PKG)/csrc/shard_fused.hpp $(PKG)/csrc/shard_step.hpp $(PKG)/csrc/wave_ops.hpp include/dagrider_shard.h include/dagrider_gpu.h

$(BUILD)/engine.o: $(ENGINE_DEPS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/engine_timing.o: $(ENGINE_DEPS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DDR_SWEEP_TIMING -DDR_TUNING -c $< -o $@

$(BUILD)/shard_timing.o: $(SHARD_DEPS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DDR_SWEEP_TIMING -c $< -o $@

$(LIBT): $(BUILD)/engine_timing.o $(BUILD)/shard_timing.o $(BUILD)/dag_gen.o $(BUILD)/wire.o $(BUILD)/host_rounds.o $(BUILD)/build_id.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lgomp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdagrider_gpu_timing.so

$(BUILD)/shard.o: $(SHARD_DEPS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# provenance: dr_build_id() returns the sha256 (first 16 hex digits) of every source
# the library is built from, in byte order of their paths -- the same hash
# dag_rider_amd/_lib.py source_hash() computes from a tree, so a prebuilt library can be
# matched to the sources it claims.  build_id.c is rewritten only when the hash changes.
ID_SRCS  := $(sort $(wildcard $(PKG)/csrc/*.hip $(PKG)/csrc/*.hpp $(PKG)/csrc/*.cpp include/*.h))
BUILD_ID := $(shell cat $(ID_SRCS) | sha256sum | cut -c1-16)
$(BUILD)/build_id.c: FORCE | $(BUILD)
	@echo 'const char *dr_build_id(void) { return "$(BUILD_ID)"; }' > $@.tmp
	@if cmp -s $@.tmp $@; then rm -f $@.tmp; else mv $@.tmp $@; fi
$(BUILD)/build_id.o: $(BUILD)/build_id.c
	$(CC) -O2 -fPIC -c $< -o $@
FORCE:

$(LIB): $(BUILD)/engine.o $(BUILD)/shard.o $(BUILD)/dag_gen.o $(BUILD)/wire.o $(BUILD)/host_rounds.o $(BUILD)/build_id.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lgomp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-soname,libdagrider_gpu.so

$(ORACLE): oracle/ref_literal.c oracle/ref_bitset.c oracle/oracle.h
	$(CC) $(CFLAGS) -shared -o $@ oracle/ref_literal.c oracle/ref_bitset.c

# C++ host mirror of process.Process over the C ABI + its TestPath port
tests-cpp: $(BUILD)/process_internal_test
$(BUILD)/process_internal_test: tests/cpp/process_internal_test.cpp $(PKG)/host/process.hpp include/dagrider_gpu.h $(LIB) | $(BUILD)
	$(CXX) -O2 -std=c++17 -Iinclude -I$(PKG)/host $< -o $@ -L$(PKG) -ldagrider_gpu -Wl,-rpath,'$$ORIGIN/../$(PKG)'

clean:
	rm -rf $(BUILD) $(LIB) $(LIBT) $(ORACLE)
