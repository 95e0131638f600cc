# Builds the MI355X scan library, the `speq` CLI and the oracle (test-only) for gfx950.
#   make            -> speq_amd/libspeq_scan.so, bin/speq, oracle/build/libkmer_oracle.so
# No cmake/ninja: plain hipcc/gcc lines.
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
CC       ?= gcc
ARCH     ?= gfx950
JOBS     ?= 8

INC      := -Iinclude -Ispeq_amd/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wextra -munsafe-fp-atomics $(INC)
HOSTFLAGS:= -O3 -std=c++17 -fPIC -Wall -Wextra $(INC)

LIB      := speq_amd/libspeq_scan.so
CLI      := bin/speq
OBJDIR   := build/obj

LIB_HIP  := speq_amd/csrc/scan_kernels.hip speq_amd/csrc/ax_scan.hip speq_amd/csrc/build_gpu.hip speq_amd/csrc/fastq_gpu.hip
LIB_CPP  := speq_amd/csrc/sais.cpp speq_amd/csrc/fm_index.cpp speq_amd/csrc/capi.cpp speq_amd/csrc/comm.cpp \
            speq_amd/csrc/host_io.cpp speq_amd/csrc/em.cpp speq_amd/csrc/pipeline.cpp \
            speq_amd/csrc/fastq_stream.cpp
CLI_CPP  := speq_amd/cli/speq_main.cpp

LIB_OBJS := $(patsubst speq_amd/csrc/%.hip,$(OBJDIR)/%.o,$(LIB_HIP)) \
            $(patsubst speq_amd/csrc/%.cpp,$(OBJDIR)/%.o,$(LIB_CPP))
HDRS     := include/speq_scan.h $(wildcard speq_amd/csrc/*.hpp)

SYNTH    := tools/build/libsynth_gen.so

all: $(LIB) $(CLI) oracle $(SYNTH)

# synthetic-input generator for bench.py / tests (makes inputs, computes no counts)
$(SYNTH): tools/synth_gen.c
	@mkdir -p tools/build
	$(CC) -O2 -fopenmp -fPIC -shared -Wall -Wextra -o $@ $< -lm

$(OBJDIR)/%.o: speq_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only translation units that call the HIP runtime / RCCL API (no kernels): g++ with the ROCm headers
$(OBJDIR)/comm.o $(OBJDIR)/pipeline.o: $(OBJDIR)/%.o: speq_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(CXX) $(HOSTFLAGS) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJDIR)/%.o: speq_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(LIB_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lamdhip64 -lz -lpthread -ldl \
	    -Wl,-rpath,/opt/rocm/lib

$(CLI): $(CLI_CPP) $(LIB) $(HDRS) speq_amd/cli/*.hpp
	@mkdir -p bin
	$(CXX) $(HOSTFLAGS) -Ispeq_amd/cli -o $@ $(CLI_CPP) -Lspeq_amd -lspeq_scan -Wl,-rpath,'$$ORIGIN/../speq_amd' -lpthread

oracle:
	$(MAKE) -C oracle

# A/B kernel variants for scripts/sweep.py (SPEQ_LIB_PATH=build/variants/<NAME>/libspeq_scan.so):
#   make variant NAME=hibranch VFLAGS=-DSPEQ_HI_BRANCH=1
variant: $(filter-out $(OBJDIR)/scan_kernels.o,$(LIB_OBJS))
	@mkdir -p build/variants/$(NAME)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c speq_amd/csrc/scan_kernels.hip -o build/variants/$(NAME)/scan_kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/variants/$(NAME)/libspeq_scan.so \
	    build/variants/$(NAME)/scan_kernels.o $^ -L/opt/rocm/lib -lamdhip64 -lz -lpthread -ldl -Wl,-rpath,/opt/rocm/lib

clean:
	rm -rf build bin $(LIB) tools/build
	$(MAKE) -C oracle clean

# A/B variants of the anchor-and-extend kernel: make axvariant NAME=w3 VFLAGS=-DSPEQ_AX_MIN_WAVES=3
axvariant: $(filter-out $(OBJDIR)/ax_scan.o,$(LIB_OBJS))
	@mkdir -p build/variants/$(NAME)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c speq_amd/csrc/ax_scan.hip -o build/variants/$(NAME)/ax_scan.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/variants/$(NAME)/libspeq_scan.so \
	    build/variants/$(NAME)/ax_scan.o $^ -L/opt/rocm/lib -lamdhip64 -lz -lpthread -ldl -Wl,-rpath,/opt/rocm/lib

# Every compile-time knob of k_scan_ax forced off its default, three builds (tests/test_gpu_ax_knobs.py runs the
# parity suite tests/ax_knob_suite.py against each): make axknobs -> build/axknobs/<name>/libspeq_scan.so
AXKNOB_kv1 := -DSPEQ_AX_SU=1 -DSPEQ_AX_SU_LOCAL=2 -DSPEQ_AX_REFILL=8 -DSPEQ_AX_BLOCKED=32 -DSPEQ_AX_P2_MARGIN=64 -DSPEQ_AX_PRIO_MIN=0 -DSPEQ_AX_WL=64 -DSPEQ_AX_MTILES=0
AXKNOB_kv2 := -DSPEQ_AX_WPB=2 -DSPEQ_AX_MIN_WAVES=4 -DSPEQ_AX_MIN_WAVES_LOCAL=3 -DSPEQ_AX_DEF_GLOBAL=192 -DSPEQ_AX_DEF_LOCAL=128
AXKNOB_kv3 := -DSPEQ_AX_SPEC_HW=1 -DSPEQ_AX_PRIO=0 -DSPEQ_AX_MPROOF=0
AXKNOBS    := kv1 kv2 kv3
AXKNOB_OTHER := $(filter-out $(OBJDIR)/ax_scan.o,$(LIB_OBJS))

axknobs: $(foreach v,$(AXKNOBS),build/axknobs/$(v)/libspeq_scan.so)

build/axknobs/%/ax_scan.o: speq_amd/csrc/ax_scan.hip $(HDRS) Makefile
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(AXKNOB_$*) -c $< -o $@

build/axknobs/%/libspeq_scan.so: build/axknobs/%/ax_scan.o $(AXKNOB_OTHER)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L/opt/rocm/lib -lamdhip64 -lz -lpthread -ldl \
	    -Wl,-rpath,/opt/rocm/lib

.PHONY: all oracle clean variant axvariant axknobs
