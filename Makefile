# Builds the gfx950 HIP C-ABI library in-tree (travels to the GPU box with the
# snapshot) and the H pass's ISA for the static hazard check.  Usage: make -j8
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := image_processor_pipeline_amd
CSRC := $(PKG)/csrc
SRCS := $(CSRC)/ipp_gather.hip $(CSRC)/ipp_hsv.hip $(CSRC)/ipp_resample.hip $(CSRC)/ipp_pipe.hip \
        $(CSRC)/ipp_ccl.hip $(CSRC)/ipp_util.hip $(CSRC)/ipp_bilinear.hip \
        $(CSRC)/ipp_enhance.hip $(CSRC)/ipp_taps.hip
HOST_SRCS := $(CSRC)/ipp_host.cpp $(CSRC)/ipp_plan.cpp
HDRS := include/ipp.h $(wildcard $(CSRC)/*.h)
OBJDIR := build/obj
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS)) $(OBJDIR)/ipp_host.o $(OBJDIR)/ipp_plan.o
LIB := $(PKG)/libipp.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall -Wno-unused-function
HOSTFLAGS := -O2 -std=c++17 -fPIC -Iinclude

all: $(LIB) $(OBJDIR)/ipp_pipe.s

# The H pass's ISA, for the static check of its hand-waited gathers
# (tools/asm_hazard.py, tests/test_asm_gather_hazard.py).
$(OBJDIR)/ipp_pipe.s: $(CSRC)/ipp_pipe.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -S --cuda-device-only $< -o $@

# Pillow's BILINEAR (double), Blend (float) and LANCZOS tap (double)
# arithmetic is plain mul/add (x86-64 baseline, no FMA): these files must not
# contract a*b+c into fma, inlined HIP header helpers included.
FPEXACT := ipp_bilinear.hip ipp_enhance.hip ipp_taps.hip
$(OBJDIR)/ipp_bilinear.o $(OBJDIR)/ipp_enhance.o $(OBJDIR)/ipp_taps.o: HIPFLAGS += -ffp-contract=off

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS) | $(OBJDIR)
	g++ $(HOSTFLAGS) -c $< -o $@

$(OBJDIR):
	mkdir -p $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lpthread

asm: | $(OBJDIR)
	for f in $(SRCS); do $(HIPCC) $(HIPFLAGS) -S --cuda-device-only $$f -o $(OBJDIR)/$$(basename $$f .hip).s; done

# Experiment builds (A/B on the GPU box through IPP_LIB_PATH): one in-tree
# library per variant, variants/<name>/libipp.so, built with VFLAGS.
#   make variant NAME=wpe6 VFLAGS=-DIPP_CCL_WPE=6
variant:
	mkdir -p variants/$(NAME)/obj
	for f in $(SRCS); do $(HIPCC) $(HIPFLAGS) $(VFLAGS) $$(echo " $(FPEXACT) " | grep -q " $$(basename $$f) " && echo -ffp-contract=off) -c $$f -o variants/$(NAME)/obj/$$(basename $$f .hip).o || exit 1; done
	for f in $(HOST_SRCS); do g++ $(HOSTFLAGS) -c $$f -o variants/$(NAME)/obj/$$(basename $$f .cpp).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o variants/$(NAME)/libipp.so variants/$(NAME)/obj/*.o -lpthread

# A variant that differs only in one kernel file (F, default ipp_pipe): that
# file rebuilt with VFLAGS, linked with the in-tree objects of the others.
#   make kvariant NAME=kb2 VFLAGS=-DIPP_HP_BANDS=2 [F=ipp_ccl]
F ?= ipp_pipe
kvariant: $(OBJS)
	mkdir -p variants/$(NAME)/obj
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) $$(echo " $(FPEXACT) " | grep -q " $(F).hip " && echo -ffp-contract=off) -c $(CSRC)/$(F).hip -o variants/$(NAME)/obj/$(F).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o variants/$(NAME)/libipp.so variants/$(NAME)/obj/$(F).o $(filter-out $(OBJDIR)/$(F).o,$(OBJS)) -lpthread

clean:
	rm -rf build $(LIB)

.PHONY: all clean asm variant kvariant
