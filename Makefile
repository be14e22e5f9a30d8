# Build of the MI355X (gfx950) hot-path library and the CPU oracle.
#   make            -> sp-slam_amd/libspslam_gpu.so  and  oracle/liboracle.so
# hipcc cross-compiles for gfx950 in the build container (no GPU needed).
HIPCC ?= /opt/rocm/bin/hipcc
OFFLOAD_ARCH ?= gfx950
HIPFLAGS ?= --offload-arch=$(OFFLOAD_ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -Wall -Wno-unused-result

PKG := sp-slam_amd
CSRC := $(PKG)/csrc
GPU_SRCS := $(CSRC)/orb_kernels.hip $(CSRC)/pose_kernels.hip $(CSRC)/plane_kernels.hip $(CSRC)/plane_segment.hip $(CSRC)/supposed_kernels.hip $(CSRC)/frame_kernels.hip $(CSRC)/lba_kernels.hip $(CSRC)/assoc_kernels.hip $(CSRC)/match_kernels.hip $(CSRC)/track_kernels.hip $(CSRC)/grab_kernels.hip $(CSRC)/spslam_capi.cpp
GPU_HDRS := $(CSRC)/wave_priority.h $(CSRC)/orb_geom.h $(CSRC)/orb_launch.h $(CSRC)/pose_launch.h $(CSRC)/plane_launch.h $(CSRC)/supposed_launch.h $(CSRC)/frame_launch.h $(CSRC)/libm_restated.h $(CSRC)/g2o_device.h $(CSRC)/lba_launch.h $(CSRC)/assoc_launch.h $(CSRC)/match_launch.h $(CSRC)/track_launch.h $(CSRC)/grab_launch.h $(CSRC)/plane_not_seen.h include/spslam_gpu.h include/spslam_brief_pattern.inc

all: $(PKG)/libspslam_gpu.so oracle/liboracle.so

$(PKG)/libspslam_gpu.so: $(GPU_SRCS) $(GPU_HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/orb_kernels.hip $(CSRC)/pose_kernels.hip $(CSRC)/plane_kernels.hip $(CSRC)/plane_segment.hip $(CSRC)/supposed_kernels.hip $(CSRC)/frame_kernels.hip $(CSRC)/lba_kernels.hip $(CSRC)/assoc_kernels.hip $(CSRC)/match_kernels.hip $(CSRC)/track_kernels.hip $(CSRC)/grab_kernels.hip \
	    -x hip $(CSRC)/spslam_capi.cpp

oracle/liboracle.so:
	$(MAKE) -C oracle liboracle.so

clean:
	rm -f $(PKG)/libspslam_gpu.so
	$(MAKE) -C oracle clean

.PHONY: all clean oracle/liboracle.so
