# Build libpgx.so (HIP for gfx950) and the C oracle twin.  `make -j8`
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-variable
CSRC = pinot_amd/csrc
HDR = include/pgx.h $(CSRC)/pgx_internal.h $(CSRC)/pgx_jit_abi.h
HOST_HDR = $(HDR) $(CSRC)/pgx_host.h

all: pinot_amd/libpgx.so

# The query compiler pastes these headers in front of every generated kernel: embed them as raw string literals.
build/%.inc: $(CSRC)/%.h
	@mkdir -p build
	@(echo 'R"PGXSRC('; cat $<; echo ')PGXSRC"') > $@

build/pgx_host.o: $(CSRC)/pgx_host.cpp $(HOST_HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_part.o build/pgx_multi.o build/pgx_realtime.o build/pgx_fixtures.o build/pgx_stage.o build/pgx_mv.o build/pgx_plan_cache.o build/pgx_plan.o: build/%.o: $(CSRC)/%.cpp $(HOST_HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_jit.o: $(CSRC)/pgx_jit.cpp $(HDR) build/pgx_jit_abi.inc build/pgx_jit_device.inc
	$(HIPCC) $(HIPFLAGS) -Ibuild -c $< -o $@

build/pgx_kernels.o: $(CSRC)/pgx_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_stats.o: $(CSRC)/pgx_stats.cpp $(CSRC)/pgx_internal.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_trim.o: $(CSRC)/pgx_trim.hip
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_merge.o: $(CSRC)/pgx_merge.hip
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/pgx_narrow.o: $(CSRC)/pgx_narrow.hip $(CSRC)/pgx_internal.h $(CSRC)/pgx_jit_abi.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

pinot_amd/libpgx.so: build/pgx_host.o build/pgx_part.o build/pgx_multi.o build/pgx_realtime.o build/pgx_fixtures.o build/pgx_stage.o build/pgx_mv.o build/pgx_plan_cache.o build/pgx_plan.o build/pgx_jit.o build/pgx_kernels.o build/pgx_trim.o build/pgx_stats.o build/pgx_merge.o build/pgx_narrow.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@ -L/opt/rocm/lib -lhiprtc -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined

clean:
	rm -rf build pinot_amd/libpgx.so

.PHONY: all clean
