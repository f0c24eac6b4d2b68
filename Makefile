# libpanman_amd.so: HIP kernels + C-ABI for gfx950 (MI355X).  No CPU fallback inside.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -mllvm -amdgpu-atomic-optimizer-strategy=None
SRC := $(wildcard panman_amd/csrc/*.cpp) $(wildcard panman_amd/csrc/*.hip)
HDR := $(wildcard panman_amd/csrc/*.h) include/panman_gpu.h
OBJ := $(patsubst panman_amd/csrc/%,build/%.o,$(SRC)) build/pm_build_id.o
# build id = hash of every library source and header and of the compile flags:
# profiles/traffic_fitch.json entries carry the id they were measured on, and bench.py reports
# no PMC traffic for a different build
BUILD_ID := $(shell (cat $(sort $(SRC) $(HDR)); echo '$(HIPCC) $(HIPFLAGS)') | sha256sum | cut -c1-16)
LIB := panman_amd/libpanman_amd.so
CLI := bin/panmanUtils
DEMO := bin/facade_demo

all: $(LIB) $(CLI) $(DEMO) oracle

# the compile line, rewritten only when it changes: a flag-only change (make HIPFLAGS=...)
# rebuilds every object and the build id without a clean
FLAGS_LINE := $(HIPCC) $(HIPFLAGS)
build/flags.stamp: FORCE
	@mkdir -p build
	@echo '$(FLAGS_LINE)' | cmp -s - $@ || echo '$(FLAGS_LINE)' > $@

# the _nt copies compile their base file with PM_NT_LOADS
build/pm_fitch_nt.hip.o: panman_amd/csrc/pm_fitch.hip
build/pm_sankoff_nt.hip.o: panman_amd/csrc/pm_sankoff.hip

build/%.o: panman_amd/csrc/% $(HDR) build/flags.stamp
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

build/pm_build_id.o: $(SRC) $(HDR) Makefile build/flags.stamp
	@mkdir -p build
	@printf 'extern "C" const char* pm_build_id(void) { return "%s"; }\n' $(BUILD_ID) > build/pm_build_id.cpp
	g++ -O2 -fPIC -c build/pm_build_id.cpp -o $@

# (linked to a temporary name and renamed: a snapshot of the tree never holds half a library)
$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@.tmp $(OBJ) -l:liblzma.so.5 && mv -f $@.tmp $@

# panmanUtils-compatible CLI (host C++ over the C-ABI; finds the library next to the package)
$(CLI): panman_amd/csrc/cli/panmanUtils.cpp include/panman_gpu.h $(LIB)
	@mkdir -p bin
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ $< -Lpanman_amd -l:libpanman_amd.so \
	    -Wl,-rpath,'$$ORIGIN/../panman_amd'

# the C++ facade (include/panman_tree.hpp) driven like the reference's Tree / TreeGroup
$(DEMO): panman_amd/csrc/cli/facade_demo.cpp include/panman_tree.hpp include/panman_gpu.h $(LIB)
	@mkdir -p bin
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ $< -Lpanman_amd -l:libpanman_amd.so \
	    -Wl,-rpath,'$$ORIGIN/../panman_amd'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build bin $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean FORCE
FORCE:
