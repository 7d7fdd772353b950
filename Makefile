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

LIB_SRCS := $(CSRC)/vame_engine.hip $(CSRC)/vame_hostlogic.cpp $(CSRC)/vame_io.cpp
LIB_HDRS := $(CSRC)/vame_kernel.h $(CSRC)/vame_tables.h include/vame.h

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
	for a in $(ABLATE_SET); do $(HIPCC) $(HIPFLAGS) -DVAME_ABLATE=$$a -shared -o $(LIBDIR)/libvame_ablate$$a.so $(LIB_SRCS) || exit 1; done
# experiment builds: make variant NAME=x DEFS="-DFOO=1" -> lib/libvame_x.so
variant:
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o $(LIBDIR)/libvame_$(NAME).so $(LIB_SRCS)
# instrumentation build counting the sub-block predictions run: make count
count:
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DVAME_COUNT_PRED=1 -shared -o $(LIBDIR)/libvame_count.so $(LIB_SRCS)
# profiling-only build with per-phase shader-clock counters: make phase
phase:
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DVAME_PHASE_TIMING=1 -shared -o $(LIBDIR)/libvame_phase.so $(LIB_SRCS)

cli: $(BINDIR)/vame

# does an event after a call wait for its any-order kernels? (tests/test_gpu_parity.py)
probe: tests/native/anyorder_probe
tests/native/anyorder_probe: tests/native/anyorder_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Wall -o $@ $<

$(LIBDIR)/libvame.so: $(LIB_SRCS) $(LIB_HDRS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(LIB_SRCS)

$(BINDIR)/vame: $(PKG)/host/vame_main.cpp include/vame.h $(LIBDIR)/libvame.so
	@mkdir -p $(BINDIR)
	$(HIPCC) -O2 -std=c++17 -Wall -o $@ $(PKG)/host/vame_main.cpp \
	    -L$(LIBDIR) -lvame -Wl,-rpath,'$$ORIGIN/../lib' -lpthread

oracle:
	$(MAKE) -s -C oracle libvame_oracle.so
	@if [ -d /root/reference ]; then $(MAKE) -s -C oracle ref; fi

resource-usage:
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -c -o /dev/null $(CSRC)/vame_engine.hip

clean:
	rm -rf $(LIBDIR) $(BINDIR)
	$(MAKE) -s -C oracle clean

.PHONY: all lib cli synth oracle probe clean resource-usage ablate phase variant count
