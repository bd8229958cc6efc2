# libsamplers_hip.so — MI355X (gfx950) hot path.  `make` builds in-tree so the
# .so travels to the GPU box with the repo snapshot.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
SRC := samplers_amd/csrc/sp_dps.hip samplers_amd/csrc/sp_blur.hip samplers_amd/csrc/sp_latent.hip \
       samplers_amd/csrc/sp_groupnorm.hip samplers_amd/csrc/sp_conv.hip \
       samplers_amd/csrc/sp_wino.hip samplers_amd/csrc/sp_conv_thin.hip \
       samplers_amd/csrc/sp_conv_s2.hip samplers_amd/csrc/sp_upsample.hip \
       samplers_amd/csrc/sp_attention.hip samplers_amd/csrc/sp_attention6.hip \
       samplers_amd/csrc/sp_gemm_x6.hip samplers_amd/csrc/sp_transformer.hip \
       samplers_amd/csrc/sp_bf16.hip
OBJ := $(patsubst samplers_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := samplers_amd/lib/libsamplers_hip.so
# bounds-checked debug build (SP_DCHECK index / range invariants counted on the device,
# sp_debug_violations): same sources, -DSP_DEBUG=1, its own objects and library
DOBJ := $(patsubst samplers_amd/csrc/%.hip,build/debug/%.o,$(SRC))
DLIB := samplers_amd/lib/debug/libsamplers_hip.so

all: $(LIB) $(DLIB)

debug: $(DLIB)

# the Winograd tile's transforms stay scalar: packed f32 ops cost more than two scalar
# ones beside MFMAs (MI355X_MICROARCH price list)
build/sp_wino.o build/debug/sp_wino.o: EXTRA := -fno-slp-vectorize
# the attention kernels keep their accumulators in VGPRs: in the AGPR form the compiler copied
# every score / output block between the two register files around each MFMA
build/sp_attention.o build/debug/sp_attention.o build/sp_attention6.o build/debug/sp_attention6.o build/sp_bf16.o build/debug/sp_bf16.o: EXTRA := -mllvm -amdgpu-mfma-vgpr-form=1

build/%.o: samplers_amd/csrc/%.hip samplers_amd/csrc/sp_common.h include/samplers_hip.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) $(EXTRA) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p samplers_amd/lib
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

build/debug/%.o: samplers_amd/csrc/%.hip samplers_amd/csrc/sp_common.h include/samplers_hip.h
	@mkdir -p build/debug
	$(HIPCC) $(CXXFLAGS) $(EXTRA) -DSP_DEBUG=1 -c $< -o $@

$(DLIB): $(DOBJ)
	@mkdir -p samplers_amd/lib/debug
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(DOBJ)

clean:
	rm -rf build $(LIB) $(DLIB)

.PHONY: all debug clean
