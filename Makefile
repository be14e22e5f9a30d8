# Build of the MI355X (gfx950) hot-path library and the CPU oracle.
#   make            -> sp-slam_amd/libspslam_gpu.so  and  oracle/liboracle.so
# hipcc cross-compiles for gfx950 in the build container (no GPU needed).
# One object per source (parallel with make -j), linked into one shared library.
HIPCC ?= /opt/rocm/bin/hipcc
OFFLOAD_ARCH ?= gfx950
HIPFLAGS ?= --offload-arch=$(OFFLOAD_ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -Wall -Wno-unused-result

PKG := sp-slam_amd
CSRC := $(PKG)/csrc
OBJDIR := build/obj
KERNELS := orb_kernels pose_kernels plane_kernels plane_segment supposed_kernels frame_kernels lba_kernels lba_g2o lba_g2o_wide \
           assoc_kernels match_kernels track_kernels grab_kernels bow_kernels
OBJS := $(addprefix $(OBJDIR)/,$(addsuffix .o,$(KERNELS) spslam_capi spslam_step))
GPU_HDRS := $(wildcard $(CSRC)/*.h) include/spslam_gpu.h include/spslam_brief_pattern.inc

all: $(PKG)/libspslam_gpu.so oracle/liboracle.so tests/shim/libreference_shim.so

$(OBJDIR)/%.o: $(CSRC)/%.hip $(GPU_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJDIR)/spslam_capi.o: $(CSRC)/spslam_capi.cpp $(GPU_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -x hip -o $@ $<

$(OBJDIR)/spslam_step.o: $(CSRC)/spslam_step.cpp $(GPU_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -x hip -o $@ $<

# the wide LocalBundleAdjustment instance is lba_g2o.hip compiled again
$(OBJDIR)/lba_g2o_wide.o $(PROFDIR)/lba_g2o_wide.o $(VARDIR)/lba_g2o_wide.o: $(CSRC)/lba_g2o.hip

$(PKG)/libspslam_gpu.so: $(OBJS)
	$(HIPCC) --offload-arch=$(OFFLOAD_ARCH) -shared -fPIC -o $@ $(OBJS)
	@python3 tools/build_info.py $@ > $(PKG)/build_info.json

# Diagnostic build: PoseOptimization phase timers (tools/pose_phases.py loads it via SPSLAM_GPU_LIB).
PROFDIR := build/prof
PROF_OBJS := $(addprefix $(PROFDIR)/,$(addsuffix .o,$(KERNELS) spslam_capi spslam_step))
prof: $(PKG)/libspslam_gpu_prof.so

$(PROFDIR)/%.o: $(CSRC)/%.hip $(GPU_HDRS)
	@mkdir -p $(PROFDIR)
	$(HIPCC) $(HIPFLAGS) -DSPSLAM_POSE_PROF -c -o $@ $<

$(PROFDIR)/spslam_capi.o: $(CSRC)/spslam_capi.cpp $(GPU_HDRS)
	@mkdir -p $(PROFDIR)
	$(HIPCC) $(HIPFLAGS) -DSPSLAM_POSE_PROF -c -x hip -o $@ $<

$(PROFDIR)/spslam_step.o: $(CSRC)/spslam_step.cpp $(GPU_HDRS)
	@mkdir -p $(PROFDIR)
	$(HIPCC) $(HIPFLAGS) -DSPSLAM_POSE_PROF -c -x hip -o $@ $<

$(PKG)/libspslam_gpu_prof.so: $(PROF_OBJS)
	$(HIPCC) --offload-arch=$(OFFLOAD_ARCH) -shared -fPIC -o $@ $(PROF_OBJS)

# Measurement variants: make variant VARIANT=<name> VAR_FLAGS="-D..." -> sp-slam_amd/libspslam_gpu_<name>.so
# (loaded via SPSLAM_GPU_LIB by tools/gpu_r02_variants.sh).
VARIANT ?= var
VAR_FLAGS ?=
VARDIR := build/var_$(VARIANT)
VAR_OBJS := $(addprefix $(VARDIR)/,$(addsuffix .o,$(KERNELS) spslam_capi spslam_step))
variant: $(PKG)/libspslam_gpu_$(VARIANT).so

$(VARDIR)/%.o: $(CSRC)/%.hip $(GPU_HDRS)
	@mkdir -p $(VARDIR)
	$(HIPCC) $(HIPFLAGS) $(VAR_FLAGS) -c -o $@ $<

$(VARDIR)/spslam_capi.o: $(CSRC)/spslam_capi.cpp $(GPU_HDRS)
	@mkdir -p $(VARDIR)
	$(HIPCC) $(HIPFLAGS) $(VAR_FLAGS) -c -x hip -o $@ $<

$(VARDIR)/spslam_step.o: $(CSRC)/spslam_step.cpp $(GPU_HDRS)
	@mkdir -p $(VARDIR)
	$(HIPCC) $(HIPFLAGS) $(VAR_FLAGS) -c -x hip -o $@ $<

$(PKG)/libspslam_gpu_$(VARIANT).so: $(VAR_OBJS)
	$(HIPCC) --offload-arch=$(OFFLOAD_ARCH) -shared -fPIC -o $@ $(VAR_OBJS)

# Reference-side shim (test infrastructure, INTEGRATION.md 1-7 compiled): plain g++ against the C ABI.
tests/shim/libreference_shim.so: tests/shim/reference_shim.cpp tests/shim/cv_lite.h include/spslam_gpu.h $(PKG)/libspslam_gpu.so
	g++ -O2 -std=c++17 -fPIC -shared -Wall -Wextra -o $@ tests/shim/reference_shim.cpp \
	    -L$(PKG) -l:libspslam_gpu.so -Wl,-rpath,'$$ORIGIN/../../$(PKG)'

oracle/liboracle.so:
	$(MAKE) -C oracle liboracle.so

clean:
	rm -rf $(PKG)/libspslam_gpu*.so build/var_* tests/shim/libreference_shim.so $(OBJDIR) $(PROFDIR)
	$(MAKE) -C oracle clean

.PHONY: all clean prof variant oracle/liboracle.so
