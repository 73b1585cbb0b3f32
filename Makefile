# Builds the product library helyim_amd/libhec.so (gfx950) and the test
# oracle oracle/build/liboracle.so. `make -j8`.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC := $(wildcard helyim_amd/csrc/*.cpp) $(wildcard helyim_amd/csrc/*.hip)
HDR := $(wildcard helyim_amd/csrc/*.hpp) $(wildcard helyim_amd/csrc/*.inc) include/hec.h
OBJ := $(patsubst helyim_amd/csrc/%,build/obj/%.o,$(SRC))

all: helyim_amd/libhec.so oracle build/cabi_bench build/membench_calib

helyim_amd/libhec.so: $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ) -lpthread

build/obj/%.hip.o: helyim_amd/csrc/%.hip $(HDR)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/obj/%.cpp.o: helyim_amd/csrc/%.cpp $(HDR)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

oracle:
	$(MAKE) -C oracle

# The BASELINE workload through the C ABI alone (no Python / PyTorch).
build/cabi_bench: tools/cabi_bench.cpp include/hec.h helyim_amd/libhec.so
	@mkdir -p build
	$(HIPCC) -O2 -std=c++17 -Wall -o $@ $< -Lhelyim_amd -lhec -Wl,-rpath,'$$ORIGIN/../helyim_amd'

# FETCH_SIZE / WRITE_SIZE calibration streams + the shipped kernels in one
# process (tools/membench.hip calib; profiles/pmc_traffic.json "calibration").
build/membench_calib: tools/membench.hip include/hec.h helyim_amd/libhec.so
	@mkdir -p build
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -DMEMBENCH_WITH_HEC -o $@ $< -Lhelyim_amd -lhec \
	    -Wl,-rpath,'$$ORIGIN/../helyim_amd'

# A/B method check: a byte-identical rebuild of the kernel file as a separate
# library (HEC_LIB_PATH=build/variants/libhec_null.so), to measure the spread
# of alternating-process A/Bs between two library builds (tools/tune.py).
VARIANTS := null
variants: $(foreach v,$(VARIANTS),build/variants/libhec_$(v).so)
build/variants/libhec_%.so: $(SRC) $(HDR)
	@mkdir -p build/variants/$*
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c helyim_amd/csrc/rs_kernels.hip -o build/variants/$*/rs_kernels.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ build/variants/$*/rs_kernels.o \
	    $(filter-out build/obj/rs_kernels.hip.o,$(OBJ)) -lpthread
VFLAGS_null := -DHEC_NULL_VARIANT=1  # identical code: measures the A/B method itself

clean:
	rm -rf build helyim_amd/libhec.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean variants
