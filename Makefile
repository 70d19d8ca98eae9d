# Build of the MI355X (gfx950) Viterbi engine, its oracle and the C++ parity tests.
# `make -j16` (the GPU box allows at most -j16).  __graft_entry__.build() runs this.
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
CC       ?= gcc
ARCH     ?= gfx950
REF      ?= /root/reference

CSRC     := spec_viterbi_amd/csrc
BUILD    := build
LIB      := spec_viterbi_amd/libspec_viterbi_hip.so
ORACLE   := oracle/liboracle.so

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) \
            -fno-honor-nans -mllvm -amdgpu-atomic-optimizer-strategy=None -Wall -Wno-unused-parameter \
            $(EXTRA_HIPFLAGS)
HOSTFLAGS := --offload-arch=$(ARCH) -O2 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall

HIP_SRCS  := $(wildcard $(CSRC)/fused_*.hip) $(CSRC)/misc.hip $(CSRC)/band.hip $(wildcard $(CSRC)/chain_*.hip) $(CSRC)/timepar.hip $(CSRC)/pipe.hip \
             $(CSRC)/pipe_tm1.hip $(CSRC)/pipe_tm1p.hip $(CSRC)/pipe_wide.hip $(CSRC)/pipe_wide_paths.hip $(CSRC)/pipe_paths.hip \
             $(CSRC)/spec2.hip $(CSRC)/pipe_l2.hip $(CSRC)/diag.hip
HOST_SRCS := $(CSRC)/runtime.cpp $(CSRC)/svh_api.cpp $(CSRC)/HIP_impl.cpp $(CSRC)/data_reader.cpp $(CSRC)/stream.cpp \
             $(CSRC)/seqreader.cpp $(CSRC)/chunker.cpp
OBJS := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(HIP_SRCS)) $(patsubst $(CSRC)/%.cpp,$(BUILD)/%.o,$(HOST_SRCS))
HDRS := $(wildcard $(CSRC)/*.h) $(wildcard include/*.h)

CPP_TESTS := tests/cpp/test_HIP_impl tests/cpp/test_HIP_spec_impl tests/cpp/test_semantic_equality \
             tests/cpp/test_readers_asan tests/cpp/test_host_asan

.PHONY: all lib oracle ref tests tools clean
all: lib oracle tests tools ref

lib: $(LIB)
oracle: $(ORACLE)
tests: $(CPP_TESTS)
tools: tools/bench_harness

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(HDRS) | $(BUILD)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(OBJS) $(BUILD)/pipe.hazards
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# The pipelined kernel's inline-asm DPP reads rely on the schedule for one of their two wait
# states: every build checks all of them in the gfx950 code objects (tools/dpp_hazards.py).  Its
# asm granule prefetches must not be read (copied, spilled) before their wait: every build checks
# them in the compiler's assembly output, where inline asm is marked (tools/check_prefetch.py).
PIPE_OBJS := pipe pipe_tm1 pipe_tm1p pipe_l2
$(BUILD)/%.dev.s: $(CSRC)/%.hip $(HDRS) | $(BUILD)
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $< -o $@
$(BUILD)/pipe.hazards: $(foreach o,$(PIPE_OBJS),$(BUILD)/$(o).o $(BUILD)/$(o).dev.s) tools/dpp_hazards.py tools/check_prefetch.py
	set -e; for o in $(PIPE_OBJS); do \
	  (cd $(BUILD) && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading $$o.o > /dev/null); \
	  co=$(BUILD)/$$o.o.0.hipv4-amdgcn-amd-amdhsa--gfx950; [ -f $$co ] || continue; \
	  /opt/rocm/lib/llvm/bin/llvm-objdump -d $$co > $(BUILD)/$$o.s; \
	  python3 tools/dpp_hazards.py $(BUILD)/$$o.s pipe_viterbi_kernel; \
	  python3 tools/check_prefetch.py $(BUILD)/$$o.dev.s; done > $@.tmp
	mv $@.tmp $@

# Oracle: plain C, every add rounded on its own (test infrastructure only).
$(ORACLE): oracle/viterbi_oracle.c oracle/viterbi_oracle.h
	$(CC) -O2 -ffp-contract=off -fno-fast-math -fopenmp -fPIC -shared -o $@ oracle/viterbi_oracle.c

# Host readers (the code that parses untrusted input) under AddressSanitizer + UBSan, without HIP:
# the counterpart of the reference's valgrind memcheck run (run_tests.sh:4-7).
tests/cpp/test_readers_asan: tests/cpp/test_readers_asan.cpp $(CSRC)/data_reader.cpp $(CSRC)/seqreader.cpp \
		$(CSRC)/seqreader.h $(CSRC)/error.h include/data_reader.h include/HMM.h
	$(CXX) -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -Iinclude -I$(CSRC) \
		-o $@ tests/cpp/test_readers_asan.cpp $(CSRC)/data_reader.cpp $(CSRC)/seqreader.cpp

# The rest of the host code under AddressSanitizer + UBSan (host side only: -fno-gpu-sanitize): the
# host CSR and every plan builder of runtime.cpp and the file decoder's chunk hand-off
# (chunker.cpp), linked with the uninstrumented kernel objects; the test touches no GPU.
ASAN_HOST := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-gpu-sanitize
ASAN_OBJS := $(patsubst $(CSRC)/%.cpp,$(BUILD)/asan/%.o,$(HOST_SRCS))
$(BUILD)/asan/%.o: $(CSRC)/%.cpp $(HDRS) | $(BUILD)
	mkdir -p $(BUILD)/asan
	$(HIPCC) $(HOSTFLAGS) $(ASAN_HOST) -c $< -o $@
$(BUILD)/asan/test_host_asan.o: tests/cpp/test_host_asan.cpp $(HDRS) | $(BUILD)
	mkdir -p $(BUILD)/asan
	$(HIPCC) $(HOSTFLAGS) $(ASAN_HOST) -c $< -o $@
tests/cpp/test_host_asan: $(BUILD)/asan/test_host_asan.o $(ASAN_OBJS) $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(HIP_SRCS))
	$(HIPCC) --offload-arch=$(ARCH) $(ASAN_HOST) -o $@ $^

# The reference benchmark harness's per-sequence call loop over HIP_impl / HIP_spec_impl.
tools/bench_harness: tools/bench_harness.cpp $(LIB) include/HIP_impl.h include/HIP_spec_impl.h
	$(HIPCC) $(HOSTFLAGS) -o $@ $< -L$(dir $(LIB)) -lspec_viterbi_hip -Wl,-rpath,'$$ORIGIN/../spec_viterbi_amd'

# C++ tests written against the reference's interfaces (tests/cpp/*.cpp).
tests/cpp/%: tests/cpp/%.cpp tests/cpp/test_helper.h $(LIB)
	$(HIPCC) $(HOSTFLAGS) -o $@ $< -L$(dir $(LIB)) -lspec_viterbi_hip -Wl,-rpath,'$$ORIGIN/../../spec_viterbi_amd'

# The reference's own reader, compiled from its sources where they lie (oracle/_ref only).
ref:
	@if [ -f $(REF)/Viterbi_impl/data_reader.cpp ]; then $(MAKE) -C oracle -f ref.mk REF=$(REF); \
	else echo "reference checkout not present: skipping oracle/_ref"; fi

clean:
	rm -rf $(BUILD) $(LIB) $(ORACLE) $(CPP_TESTS) tools/bench_harness oracle/_ref
