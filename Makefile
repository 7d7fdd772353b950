# vame -- MI355X affine-ME engine.  `make` builds everything in-tree:
#   vvc-affine-gpu_amd/lib/libvame.so   HIP kernels (gfx950) + C ABI (include/vame.h)
#   vvc-affine-gpu_amd/bin/vame         C++ CLI, drop-in for the reference's ./main
#   oracle/libvame_oracle.so            CPU restatement (tests / CPU baseline only)
#   oracle/_ref/*                       reference kernels + harness (only where /root/reference exists)

HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := vvc-affine-gpu_amd
CSRC    := $(PKG)/csrc
LIBDIR  := $(PKG)/lib
BINDIR  := $(PKG)/bin
# -ffp-contract=off: the FP64 solve must round exactly like the reference
# (explicit fma where OpenCL's FP_CONTRACT fuses); integer paths are unaffected.
# -disable-machine-licm: the quadrant kernel's task loop (several tasks per
# workgroup) made MachineLICM hoist constants and lane addresses out of it and
# spill registers for them (16-48 B/lane, their writes reaching HBM); without
# it every kernel runs at zero scratch.
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
            -mllvm -disable-machine-licm
# SimplifyCFG's sinking (and, for the 2-CP-only kernels, hoisting) of code
# common to both sides of a branch stretched live ranges across the kernels'
# per-item and per-kind branches into spill slots: without it the kernels of
# the engine's unit drop to 0-32 B of scratch per lane and the 2-CP-only ones
# (vame_kernels_2cp.hip) from 76-84 B to 0-40 B; c2 -2.3 %, c3 / c4 -0.8 %
# (profiles/r06_quad2_ab.txt, seventh and eighth A/B).
# Uniform branches left unstructurized (the per-item and per-kind branches
# are wave-uniform): scratch 0 in the quadrant kernels, c2 -1.1 %, c4 -0.6 %
# (ninth A/B).
KFLAGS     := -mllvm -simplifycfg-sink-common=false -mllvm -structurizecfg-skip-uniform-regions=true
KFLAGS_2CP := -mllvm -simplifycfg-sink-common=false -mllvm -simplifycfg-hoist-common=false \
              -mllvm -structurizecfg-skip-uniform-regions=true

LIB_SRCS := $(CSRC)/vame_engine.hip $(CSRC)/vame_kernels_2cp.hip $(CSRC)/vame_hostlogic.cpp $(CSRC)/vame_io.cpp
LIB_HDRS := $(CSRC)/vame_kernel.h $(CSRC)/vame_tables.h include/vame.h
OBJDIR   := $(PKG)/build
# $(call build_lib,<output .so>,<extra flags>): every unit with its own flags, then one link
define build_lib
	@mkdir -p $(LIBDIR) $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) $(2) -c -o $(OBJDIR)/$(notdir $(1)).engine.o $(CSRC)/vame_engine.hip
	$(HIPCC) $(HIPFLAGS) $(KFLAGS_2CP) $(2) -c -o $(OBJDIR)/$(notdir $(1)).2cp.o $(CSRC)/vame_kernels_2cp.hip
	$(HIPCC) $(HIPFLAGS) $(2) -c -o $(OBJDIR)/$(notdir $(1)).hostlogic.o $(CSRC)/vame_hostlogic.cpp
	$(HIPCC) $(HIPFLAGS) $(2) -c -o $(OBJDIR)/$(notdir $(1)).io.o $(CSRC)/vame_io.cpp
	$(HIPCC) --offload-arch=$(ARCH) -fPIC -shared -o $(1) $(OBJDIR)/$(notdir $(1)).engine.o \
	    $(OBJDIR)/$(notdir $(1)).2cp.o $(OBJDIR)/$(notdir $(1)).hostlogic.o $(OBJDIR)/$(notdir $(1)).io.o
endef

all: lib cli synth oracle probe

lib: $(LIBDIR)/libvame.so

# synthetic test-sequence generator (bench / tests only; vame/synth.py is its spec)
synth: $(LIBDIR)/libvame_synth.so
$(LIBDIR)/libvame_synth.so: $(CSRC)/vame_synth.c
	@mkdir -p $(LIBDIR)
	gcc -O2 -fopenmp -ffp-contract=off -fPIC -shared -Wall -o $@ $<

# timing-only ablation builds (results are wrong): make ablate [ABLATE_SET="..."]
ABLATE_SET ?= 1 2 4 6 7 8 11 13 14 15 16 32
ablate:
	@mkdir -p $(LIBDIR)
	for a in $(ABLATE_SET); do $(MAKE) -s variant NAME=ablate$$a DEFS=-DVAME_ABLATE=$$a || exit 1; done
# experiment builds: make variant NAME=x DEFS="-DFOO=1" -> lib/libvame_x.so
variant:
	$(call build_lib,$(LIBDIR)/libvame_$(NAME).so,$(DEFS))
# instrumentation build counting the sub-block predictions run: make count
count:
	$(call build_lib,$(LIBDIR)/libvame_count.so,-DVAME_COUNT_PRED=1)
# profiling-only build with per-phase shader-clock counters: make phase
phase:
	$(call build_lib,$(LIBDIR)/libvame_phase.so,-DVAME_PHASE_TIMING=1)

cli: $(BINDIR)/vame

# does an event after a call wait for its any-order kernels? (tests/test_gpu_parity.py)
probe: tests/native/anyorder_probe
tests/native/anyorder_probe: tests/native/anyorder_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Wall -o $@ $<

$(LIBDIR)/libvame.so: $(LIB_SRCS) $(LIB_HDRS)
	$(call build_lib,$@,)

$(BINDIR)/vame: $(PKG)/host/vame_main.cpp include/vame.h $(LIBDIR)/libvame.so
	@mkdir -p $(BINDIR)
	$(HIPCC) -O2 -std=c++17 -Wall -o $@ $(PKG)/host/vame_main.cpp \
	    -L$(LIBDIR) -lvame -Wl,-rpath,'$$ORIGIN/../lib' -lpthread

oracle:
	$(MAKE) -s -C oracle libvame_oracle.so
	@if [ -d /root/reference ]; then $(MAKE) -s -C oracle ref; fi

resource-usage:
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -Rpass-analysis=kernel-resource-usage -c -o /dev/null $(CSRC)/vame_engine.hip
	$(HIPCC) $(HIPFLAGS) $(KFLAGS_2CP) -Rpass-analysis=kernel-resource-usage -c -o /dev/null $(CSRC)/vame_kernels_2cp.hip

clean:
	rm -rf $(LIBDIR) $(BINDIR) $(OBJDIR)
	$(MAKE) -s -C oracle clean

.PHONY: all lib cli synth oracle probe clean resource-usage ablate phase variant count
