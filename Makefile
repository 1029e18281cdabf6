# Build of the MI355X block-hash path (gfx950 only) and of the CPU oracle.
#   make            -> ciruela_amd/libciruela_amd.so, bin/ciruela-index, the two
#                      load drivers under build/, oracle
#   make oracle     -> oracle/build/liboracle_blake2b.so (test infrastructure)
#   make asan/tsan  -> build/host_{asan,tsan}_driver (host code under the
#                      sanitizers; `make sanitizers` = both; not in `all`)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
CC ?= gcc
ARCH ?= gfx950
# COV5 keeps the code object loadable by the ROCm 7.0 runtime that ships
# inside the PyTorch wheel as well as by /opt/rocm (7.2).
COMMON := -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude -Iciruela_amd/csrc
HIPFLAGS ?= $(COMMON) --offload-arch=$(ARCH) -mcode-object-version=5
HOSTFLAGS ?= $(COMMON) -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include
CSRC := ciruela_amd/csrc
OBJDIR := build/obj
LIB := ciruela_amd/libciruela_amd.so
CLI := bin/ciruela-index

SRCS_HIP := $(CSRC)/kernels.hip $(CSRC)/order.hip
SRCS_CPP := $(CSRC)/runtime.cpp $(CSRC)/dirsig.cpp $(CSRC)/scan.cpp $(CSRC)/registry.cpp \
            $(CSRC)/blake2b_host.cpp $(CSRC)/sha512_host.cpp
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS_HIP)) \
        $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(SRCS_CPP))
HDRS := $(wildcard $(CSRC)/*.hpp) include/ciruela_blockhash.h

all: $(LIB) $(CLI) build/hash_bytes_conc build/verify_daemon_sim oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only translation units: compiled by hipcc as C++ (HIP headers, no device code)
$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HOSTFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS) -lpthread

$(CLI): $(CSRC)/cli.cpp $(LIB) $(HDRS)
	@mkdir -p bin
	$(HIPCC) $(HOSTFLAGS) $< -o $@ -Lciruela_amd -lciruela_amd \
	    -Wl,-rpath,'$$ORIGIN/../ciruela_amd'

# concurrent hash_bytes callers from C threads (tools/hash_bytes_conc.cpp)
build/hash_bytes_conc: tools/hash_bytes_conc.cpp $(LIB) include/ciruela_blockhash.h
	@mkdir -p build
	$(HIPCC) $(HOSTFLAGS) $< -o $@ -Lciruela_amd -lciruela_amd \
	    -Wl,-rpath,'$$ORIGIN/../ciruela_amd' -lpthread

# the daemon's per-block verify under load (tools/verify_daemon_sim.cpp)
build/verify_daemon_sim: tools/verify_daemon_sim.cpp $(LIB) include/ciruela_blockhash.h
	@mkdir -p build
	$(HIPCC) $(HOSTFLAGS) $< -o $@ -Lciruela_amd -lciruela_amd \
	    -Wl,-rpath,'$$ORIGIN/../ciruela_amd' -lpthread

# the library's host code under ASan + UBSan against the production device
# code (tools/host_asan_driver.cpp; sanitizers on the host side only)
ASAN_HOST := -O1 -g -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
             -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer
ASAN_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS_HIP)) \
             $(patsubst $(CSRC)/%.cpp,build/asan/%.o,$(SRCS_CPP)) build/asan/host_asan_driver.o
build/asan/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build/asan
	$(HIPCC) $(HOSTFLAGS) $(ASAN_HOST) -c $< -o $@
build/asan/host_asan_driver.o: tools/host_asan_driver.cpp include/ciruela_blockhash.h
	@mkdir -p build/asan
	$(HIPCC) $(HOSTFLAGS) $(ASAN_HOST) -c $< -o $@
build/host_asan_driver: $(ASAN_OBJS)
	$(HIPCC) $(HIPFLAGS) $(ASAN_HOST) -o $@ $(ASAN_OBJS) -lpthread
asan: build/host_asan_driver

# the same driver with the host code under ThreadSanitizer
# (TSAN_OPTIONS=suppressions=tools/tsan_hip.supp)
TSAN_HOST := -O1 -g -Xarch_host -fsanitize=thread
TSAN_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS_HIP)) \
             $(patsubst $(CSRC)/%.cpp,build/tsan/%.o,$(SRCS_CPP)) build/tsan/host_asan_driver.o
build/tsan/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p build/tsan
	$(HIPCC) $(HOSTFLAGS) $(TSAN_HOST) -c $< -o $@
build/tsan/host_asan_driver.o: tools/host_asan_driver.cpp include/ciruela_blockhash.h
	@mkdir -p build/tsan
	$(HIPCC) $(HOSTFLAGS) $(TSAN_HOST) -c $< -o $@
build/host_tsan_driver: $(TSAN_OBJS)
	$(HIPCC) $(HIPFLAGS) $(TSAN_HOST) -o $@ $(TSAN_OBJS) -lpthread
tsan: build/host_tsan_driver

sanitizers: asan tsan

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(CLI)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean asan tsan sanitizers
