# Build the MI355X (gfx950) Bloom-filter library and the CPU oracle.
#   make            -> dlsm_amd/lib/libdlsm_bloom.so + oracle/liboracle.so
#   make oracle-ref -> oracle/_ref/libref.so (build container only)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-result
SRC := dlsm_amd/csrc/bloom_kernels.hip dlsm_amd/csrc/bloom_capi.hip dlsm_amd/csrc/block_crc.hip \
       dlsm_amd/csrc/key_select.hip dlsm_amd/csrc/stream_probe.hip \
       dlsm_amd/csrc/multi_device.hip dlsm_amd/csrc/batcher.hip dlsm_amd/csrc/host_hash.hip
HDR := dlsm_amd/csrc/bloom_math.h dlsm_amd/csrc/bloom_internal.h include/dlsm_bloom.h
LIB := dlsm_amd/lib/libdlsm_bloom.so
OBJ := $(patsubst dlsm_amd/csrc/%.hip,build/%.o,$(SRC))

all: $(LIB) oracle

build/%.o: dlsm_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p dlsm_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

oracle:
	$(MAKE) -C oracle liboracle.so

oracle-ref:
	$(MAKE) -C oracle ref

asm: dlsm_amd/csrc/bloom_kernels.hip $(HDR)
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) --offload-device-only -S $< -o build/asm/bloom_kernels.s \
	  -Rpass-analysis=kernel-resource-usage 2> build/asm/resource_usage.txt || true

# A/B build with extra defines: make variant TAG=u4 VFLAGS="-DDLSM_PROBE_U=4"
# -> dlsm_amd/lib/variants/libdlsm_bloom_u4.so (loaded with DLSM_LIB_VARIANT=u4)
variant: $(SRC) $(HDR)
	@mkdir -p build/variants/$(TAG) dlsm_amd/lib/variants
	for f in $(SRC); do $(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $$f -o build/variants/$(TAG)/$$(basename $$f .hip).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC build/variants/$(TAG)/*.o -o dlsm_amd/lib/variants/libdlsm_bloom_$(TAG).so

clean:
	rm -rf build dlsm_amd/lib
	$(MAKE) -C oracle clean

.PHONY: all oracle oracle-ref asm variant clean
