# Build libpgx.so (HIP for gfx950) and the C oracle twin.  `make -j8`
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-variable
SRC = pinot_amd/csrc/pgx_host.cpp pinot_amd/csrc/pgx_kernels.hip
HDR = include/pgx.h pinot_amd/csrc/pgx_internal.h

all: pinot_amd/libpgx.so

build/pgx_host.o: pinot_amd/csrc/pgx_host.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_kernels.o: pinot_amd/csrc/pgx_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

pinot_amd/libpgx.so: build/pgx_host.o build/pgx_kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

clean:
	rm -rf build pinot_amd/libpgx.so

.PHONY: all clean
