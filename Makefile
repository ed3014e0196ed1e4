# Build recipe for the product library (libesgd.so, gfx950) and the CPU oracle.
#   make            -> both
#   make lib        -> eager-sgd_amd/esgd/libesgd.so
#   make oracle     -> oracle/libffref.so
#   make sweeps     -> tools/bin/libesgd_sweeps.so (measurement-only kernel variants,
#                      tools/sweep_reduce.py; never linked into the product)
# No -ffast-math anywhere: parity with fflib2 is bitwise (SURVEY.md §7 "Hard parts").

ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
PKG       := eager-sgd_amd
CSRC      := $(PKG)/csrc
OUTLIB    := $(PKG)/esgd/libesgd.so
BUILD     := build/obj

HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off \
             -Iinclude -I$(CSRC) -Wall -Wno-unused-result
# host-only sources (-x c++) include hip_runtime.h, which asks the platform of a non-HIP
# translation unit (hipcc sets it for .hip files itself)
CXXFLAGS  := -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -I$(CSRC) \
             -I$(ROCM)/include -D__HIP_PLATFORM_AMD__ -Wall
LDFLAGS   := -shared -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -lpthread -lrt \
             -Wl,--no-undefined -Wl,-soname,libesgd.so \
             -Wl,--version-script=$(CSRC)/exports.map

HIP_SRCS  := $(wildcard $(CSRC)/*.hip)
CPP_SRCS  := $(wildcard $(CSRC)/*.cpp)
OBJS      := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.hip.o,$(HIP_SRCS)) \
             $(patsubst $(CSRC)/%.cpp,$(BUILD)/%.cpp.o,$(CPP_SRCS))
HDRS      := $(wildcard include/*.h) $(wildcard $(CSRC)/*.h)

.PHONY: all lib oracle sweeps clean tsan
all: lib oracle

lib: $(OUTLIB)

$(BUILD)/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(CXXFLAGS) -x c++ -c $< -o $@

$(OUTLIB): $(OBJS) $(CSRC)/exports.map
	$(HIPCC) --offload-arch=$(ARCH) $(OBJS) $(LDFLAGS) -o $@

# ---- sweep variants of the tree kernel (tools only) ----
SWEEPS    := tools/bin/libesgd_sweeps.so

sweeps: $(SWEEPS)

$(SWEEPS): tools/sweeps/reduce_sweeps.hip $(CSRC)/reduce_core.h $(HDRS)
	@mkdir -p tools/bin
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $< -L$(ROCM)/lib -lamdhip64

# ---- CPU oracle (test infrastructure only) ----
oracle: oracle/libffref.so

oracle/libffref.so: oracle/ffref.c oracle/ffref.h
	gcc -O3 -ftree-vectorize -ffp-contract=off -fno-fast-math -fPIC -shared -std=c11 \
	    -Wall -o $@ oracle/ffref.c -lpthread

clean:
	rm -rf $(BUILD) $(OUTLIB) oracle/libffref.so $(SWEEPS)

# ---- ThreadSanitizer build of the host side (CPU control-plane tests only) ----
# make tsan -> build/tsan/libesgd.so; run e.g.
#   LD_PRELOAD=$(TSAN_RT) ESGD_LIB=build/tsan/libesgd.so TSAN_OPTIONS=report_signal_unsafe=0 \
#   python -m pytest tests/test_control_plane.py -m "not gpu"
TSAN_RT   := $(ROCM)/lib/llvm/lib/clang/22/lib/linux/libclang_rt.tsan-x86_64.so
TSAN_DIR  := build/tsan
TSAN_OBJS := $(patsubst $(CSRC)/%.hip,$(TSAN_DIR)/%.hip.o,$(HIP_SRCS)) \
             $(patsubst $(CSRC)/%.cpp,$(TSAN_DIR)/%.cpp.o,$(CPP_SRCS))

tsan: $(TSAN_DIR)/libesgd.so

$(TSAN_DIR)/%.hip.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(TSAN_DIR)
	$(HIPCC) $(HIPFLAGS) -O1 -g -Xarch_host -fsanitize=thread -c $< -o $@

$(TSAN_DIR)/%.cpp.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(TSAN_DIR)
	$(HIPCC) $(CXXFLAGS) -O1 -g -fsanitize=thread -x c++ -c $< -o $@

$(TSAN_DIR)/libesgd.so: $(TSAN_OBJS) $(CSRC)/exports.map
	$(HIPCC) --offload-arch=$(ARCH) $(TSAN_OBJS) $(LDFLAGS) $(TSAN_RT) -Wl,-rpath,$(dir $(TSAN_RT)) -o $@
