# Build recipes (no cmake needed).  `make` builds the product library and the CPU oracle.
#   dirt_amd/libdirt_mi355x.so  -- HIP kernels + C ABI (include/dirt_mi355x.h), gfx950 only
#   oracle/libdirt_oracle.so    -- CPU oracle (test infrastructure only)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CC ?= gcc

# -ffp-contract=off + correctly rounded divide: the raster rules are stated as
# single IEEE operations so that the HIP path and the oracle agree bit-exactly on coverage and depth.
# -amdgpu-set-wave-priority: waves raise their priority (s_setprio) while issuing their loads, so the
# latency-bound setup/raster/grad waves get their memory requests out before VALU-heavy neighbours.
# A/B on one box, three interleaved rounds (profiles/r02/ab_waveprio_*): without 16.06 / 16.10 / 15.96,
# with 16.59 / 16.49 / 16.40 Gpixels/s (+2.8 %).  `make WAVEPRIO=` builds without it.
# -Wno-pass-failed: the generic-C backward paths ask for 6 waves / SIMD although LDS caps them at 5
WAVEPRIO ?= -mllvm -amdgpu-set-wave-priority
# -fno-slp-vectorize: the SLP vectoriser packs pairs of fp32 operations into v_pk_* instructions whose operands
# need even-aligned register pairs; in the backward that costs registers the 64-VGPR / 8-wave budget does not
# have (the vertex-only instantiation spilled 30 VGPRs).  Without it, A/B in one call, three rounds
# (profiles/r04/ab_no_slp/): c3 18.06-18.25 -> 18.28-18.50, c4 7.33-7.47 -> 7.82-7.91, c5 28.17-28.26 ->
# 28.44-28.70 Gpixels/s (bench_configs, 10-step graphs).  `make SLP=` builds with it.
SLP ?= -fno-slp-vectorize
# SCHED: extra scheduler options for A/B builds (`make variant NAME=x SCHED=...`).  -amdgpu-use-amdgpu-trackers
# measured within noise in round 4 (profiles/r04/ab_sched/) and again in round 6 (+0.3 % over six paired rounds in
# two calls, -0.5 % in a third; profiles/r06/ab_sched_trackers/); the max-ILP strategy spilled the raster and lost
# 7 %.  The product builds without any.
SCHED ?=
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
           -fhip-fp32-correctly-rounded-divide-sqrt $(WAVEPRIO) $(SLP) $(SCHED) -Wall -Wno-unused-function \
           -Wno-pass-failed
ORACLE_CFLAGS = -O3 -std=c99 -ffp-contract=off -fno-fast-math -fopenmp -fPIC -Wall

LIB = dirt_amd/libdirt_mi355x.so
ORACLE = oracle/libdirt_oracle.so
HIP_SRC = dirt_amd/csrc/dirt_raster.hip
HIP_DEPS = $(HIP_SRC) dirt_amd/csrc/lighting_kernels.h dirt_amd/csrc/setup_kernel.h dirt_amd/csrc/raster_kernel.h dirt_amd/csrc/grad_kernel.h dirt_amd/csrc/raster_rules.h dirt_amd/csrc/oceanic.h dirt_amd/csrc/hill.h include/dirt_mi355x.h Makefile

# the public op's C++ autograd function (PyTorch extension over the C ABI; dirt_amd/csrc/torch_op.cpp)
PY ?= python3
TORCH_DIR := $(shell $(PY) -c "import os, torch; print(os.path.dirname(torch.__file__))" 2>/dev/null)
PY_INC := $(shell $(PY) -c "import sysconfig; print(sysconfig.get_paths()['include'])" 2>/dev/null)
EXT_SUFFIX := $(shell $(PY) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))" 2>/dev/null)
CXX11ABI := $(shell $(PY) -c "import torch; print(int(torch._C._GLIBCXX_USE_CXX11_ABI))" 2>/dev/null)
TORCH_EXT = dirt_amd/_dirt_torch$(EXT_SUFFIX)
EXT_CXXFLAGS = -O2 -std=c++17 -fPIC -shared -Wall -Wno-unused-function -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 \
               -DTORCH_EXTENSION_NAME=_dirt_torch -DTORCH_API_INCLUDE_EXTENSION_H -D_GLIBCXX_USE_CXX11_ABI=$(CXX11ABI) \
               -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include -I/opt/rocm/include -I$(PY_INC)
EXT_LDFLAGS = -L$(TORCH_DIR)/lib -ltorch -ltorch_cpu -ltorch_python -lc10 -lc10_hip -Wl,-rpath,$(TORCH_DIR)/lib -ldl

# the C library and the oracle never need torch; the extension is built only where torch imports
ifeq ($(TORCH_DIR),)
all: $(LIB) $(ORACLE)
	@echo "torch not importable: skipping the optional $(TORCH_EXT)"
else
all: $(LIB) $(ORACLE) $(TORCH_EXT)
endif

$(TORCH_EXT): dirt_amd/csrc/torch_op.cpp include/dirt_mi355x.h
	g++ $(EXT_CXXFLAGS) -o $@ $< $(EXT_LDFLAGS)

$(LIB): $(HIP_DEPS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_SRC)

$(ORACLE): oracle/dirt_oracle.c
	$(CC) $(ORACLE_CFLAGS) -shared -o $@ $< -lm

# experiment builds: make variant NAME=w5 DEFS=-DDIRT_GRAD_WAVES=5  -> build/variants/w5.so
variant: $(HIP_DEPS)
	mkdir -p build/variants && $(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o build/variants/$(NAME).so $(HIP_SRC)

asm: $(HIP_DEPS)
	mkdir -p build/asm && cd build/asm && $(HIPCC) $(HIPFLAGS) $(DEFS) --cuda-device-only -S -o $(or $(NAME),dirt_raster).s ../../$(HIP_SRC)

clean:
	rm -f $(LIB) $(ORACLE) $(TORCH_EXT)

.PHONY: all clean asm
