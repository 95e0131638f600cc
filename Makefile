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

.PHONY: all oracle clean variant axvariant
