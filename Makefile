# Builds the product library helyim_amd/libhec.so (gfx950) and the test
# oracle oracle/build/liboracle.so. `make -j8`.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC := $(wildcard helyim_amd/csrc/*.cpp) $(wildcard helyim_amd/csrc/*.hip)
HDR := $(wildcard helyim_amd/csrc/*.hpp) include/hec.h
OBJ := $(patsubst helyim_amd/csrc/%,build/obj/%.o,$(SRC))

all: helyim_amd/libhec.so oracle

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

clean:
	rm -rf build helyim_amd/libhec.so
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
