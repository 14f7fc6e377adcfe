# Native build for gpumon (MI355X / gfx950).
#   make            -> python extension gpumon/_core*.so + bin/gpumon-exporter + HIP library
#   make core       -> C++ core only (no hipcc needed)
#   make hip        -> gpumon/_hip*.so (HIP kernels: probe + synthetic load, gfx950)
#   make plugins    -> lib/libgpumon_pmc.so + lib/libgpumon_probe.so (dlopen'd on-device plugins)
#   make asan       -> bin/gpumon-exporter-asan (host-only sanitizers)
#   make tools      -> test / experiment binaries (nodev, perf_snapshot_probe, hsa_stages); not in `all`
# `all` is the product only: deploy/Dockerfile's build stage copies Makefile, csrc and gpumon and
# runs `make all` -- nothing under tools/ or tests/ may become a prerequisite of it
# (tests/test_deploy.py::test_image_build_stage_makes_all_from_its_copy_set).
# Everything builds IN-TREE so the .so files travel with the repo snapshot to the GPU box.

PY        ?= python3
CXX       ?= g++
HIPCC     ?= /opt/rocm/bin/hipcc
ROCM      ?= /opt/rocm
GPUMON_ARCH ?= gfx950
PYINC     := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND    := $(shell $(PY) -c "import pybind11;print(pybind11.get_include())")
EXT       := $(shell $(PY) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

CXXFLAGS  ?= -O2 -g0 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -Wno-missing-field-initializers
INC       := -I$(ROCM)/include -Icsrc
LIBS      := -ldl -lpthread -lz

CORE_SRC  := $(wildcard csrc/core/*.cpp)
CORE_OBJ  := $(patsubst csrc/%.cpp,build/obj/%.o,$(CORE_SRC))
CORE_HDR  := $(wildcard csrc/core/*.h) csrc/plugins/ondevice_abi.h csrc/plugins/ondevice_helper_proto.h

PYEXT     := gpumon/_core$(EXT)
HIPEXT    := gpumon/_hip$(EXT)
BIN       := bin/gpumon-exporter
HIP_SRC   := $(wildcard csrc/hip/*.hip)
HIP_HDR   := $(wildcard csrc/hip/*.h)

.PHONY: all core hip pmc plugins clean asan tsan fakes nodev snapshot tools
all: core hip plugins pmc
tools: nodev snapshot
core: $(PYEXT) $(BIN)
hip: $(HIPEXT)

build/obj/%.o: csrc/%.cpp $(CORE_HDR)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) $(INC) -c $< -o $@

build/obj/bindings/core_module.o: csrc/bindings/core_module.cpp $(CORE_HDR)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -fvisibility=hidden $(INC) -I$(PYINC) -I$(PYBIND) -c $< -o $@

$(PYEXT): $(CORE_OBJ) build/obj/bindings/core_module.o
	$(CXX) -shared -o $@ $^ $(LIBS)

$(BIN): $(CORE_OBJ) build/obj/exporter_main.o
	@mkdir -p bin
	$(CXX) -o $@ $^ $(LIBS)

# HIP kernels + their pybind11 wrapper in one hipcc-built extension (gfx950 only).
HIPFLAGS  := --offload-arch=$(GPUMON_ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden -Icsrc
build/obj/hip/kernels.o: csrc/hip/kernels.hip $(HIP_HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# 16x16x32 burn: MFMA accumulators in VGPRs. With AGPR accumulators LLVM rotates the 4-register
# chains through v_accvgpr_read/write/mov inside the loop (checked with --cuda-device-only -S);
# the 32x32x16 burn stays in AGPR form (the VGPR form cost it 94 -> 82 % MFMA busy).
BURN16_FLAGS := -mllvm -amdgpu-mfma-vgpr-form
build/obj/hip/burn16.o: csrc/hip/burn16.hip $(HIP_HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(BURN16_FLAGS) -c $< -o $@

build/obj/bindings/hip_module.o: csrc/bindings/hip_module.cpp $(HIP_HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -I$(PYINC) -I$(PYBIND) -c $< -o $@

build/obj/hip/burn_dtypes.o: csrc/hip/burn_dtypes.hip $(HIP_HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(BURN16_FLAGS) -c $< -o $@

$(HIPEXT): build/obj/hip/kernels.o build/obj/hip/burn16.o build/obj/hip/burn_dtypes.o build/obj/bindings/hip_module.o
	$(HIPCC) --offload-arch=$(GPUMON_ARCH) -shared -fPIC $^ -o $@

# Sanitizer builds, one object per source so `make -j` compiles them in parallel.
ASAN_FLAGS := -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer
TSAN_FLAGS := -O1 -g -std=c++17 -fsanitize=thread
ASAN_OBJ := $(patsubst csrc/%.cpp,build/asan/%.o,$(CORE_SRC) csrc/exporter_main.cpp)
TSAN_OBJ := $(patsubst csrc/%.cpp,build/tsan/%.o,$(CORE_SRC) csrc/exporter_main.cpp)
build/asan/%.o: csrc/%.cpp $(CORE_HDR)
	@mkdir -p $(dir $@)
	$(CXX) $(ASAN_FLAGS) $(INC) -c $< -o $@
build/tsan/%.o: csrc/%.cpp $(CORE_HDR)
	@mkdir -p $(dir $@)
	$(CXX) $(TSAN_FLAGS) $(INC) -c $< -o $@

asan: bin/gpumon-exporter-asan
bin/gpumon-exporter-asan: $(ASAN_OBJ)
	@mkdir -p bin
	$(CXX) -fsanitize=address,undefined $^ -o $@ $(LIBS)

tsan: bin/gpumon-exporter-tsan
bin/gpumon-exporter-tsan: $(TSAN_OBJ)
	@mkdir -p bin
	$(CXX) -fsanitize=thread $^ -o $@ $(LIBS)

# Test tool: the exporter with /dev/kfd and /dev/dri opens refused (csrc/testtools/nodev_interpose.cpp,
# tools/no_device_check.sh): what an unprivileged pod without device access still exports.
nodev: bin/gpumon-exporter-nodev
bin/gpumon-exporter-nodev: $(CORE_OBJ) build/obj/exporter_main.o csrc/testtools/nodev_interpose.cpp
	@mkdir -p bin build/obj/testtools
	$(CXX) $(CXXFLAGS) -c csrc/testtools/nodev_interpose.cpp -o build/obj/testtools/nodev_interpose.o
	$(CXX) -rdynamic -o $@ $(CORE_OBJ) build/obj/exporter_main.o build/obj/testtools/nodev_interpose.o $(LIBS)

# Experiment tools: can a shader read the SQ's perf-snapshot registers (tools/perf_snapshot_probe.hip)?
# Which raw-HSA step pins the per-queue host blocks (tools/hsa_stages.cpp)?
snapshot: bin/perf_snapshot_probe bin/hsa_stages
bin/hsa_stages: tools/hsa_stages.cpp
	@mkdir -p bin
	$(CXX) -O2 -std=c++17 -Wall -I$(ROCM)/include $< -L$(ROCM)/lib -lhsa-runtime64 -Wl,-rpath,$(ROCM)/lib -o $@
bin/perf_snapshot_probe: tools/perf_snapshot_probe.hip
	@mkdir -p bin
	$(HIPCC) --offload-arch=$(GPUMON_ARCH) -O2 $< -o $@

clean:
	rm -rf build bin lib gpumon/_core*.so gpumon/_hip*.so gpumon/_pmc*.so

# On-device plugins (csrc/plugins/ondevice_abi.h). The exporter binary and gpumon._core dlopen()
# them from lib/ only when PMC / probe sampling is enabled, so neither links HIP or rocprofiler.
PMCLIB   := lib/libgpumon_pmc.so
PROBELIB := lib/libgpumon_probe.so
ONDHELPER := lib/gpumon-ondevice-helper
plugins: $(PMCLIB) $(PROBELIB) $(ONDHELPER)
# The process that runs the on-device samplers' GPU-runtime side (device counting contexts + K1
# probe, csrc/plugins/ondevice_helper_proto.h), frozen by the exporter between requests.
$(ONDHELPER): csrc/plugins/ondevice_helper_main.cpp csrc/plugins/ondevice_helper_proto.h csrc/plugins/ondevice_abi.h $(PMCLIB)
	$(CXX) -O2 -std=c++17 $< -Llib -lgpumon_pmc -ldl -Wl,-rpath,'$$ORIGIN' -o $@
$(PMCLIB): csrc/plugins/pmc_plugin.cpp csrc/plugins/ondevice_abi.h
	@mkdir -p lib
	$(HIPCC) -O2 -std=c++17 -fPIC -shared -fvisibility=hidden -I$(ROCM)/include $< -Wl,-soname,libgpumon_pmc.so \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lrocprofiler-sdk -lhsa-runtime64 -o $@
build/obj/plugins/probe_plugin.o: csrc/plugins/probe_plugin.cpp csrc/plugins/ondevice_abi.h csrc/plugins/probe_hsa.h $(HIP_HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
# The K1 probe as an unbundled gfx950 code object, embedded (.incbin) in the raw-HSA launch path.
PROBECO := build/obj/hip/probe_$(GPUMON_ARCH).hsaco
$(PROBECO): csrc/hip/probe_co.hip $(HIP_HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(GPUMON_ARCH) --offload-device-only --no-gpu-bundle-output -O3 -std=c++17 -Icsrc $< -o $@
build/obj/plugins/probe_hsa.o: csrc/plugins/probe_hsa.cpp csrc/plugins/probe_hsa.h $(HIP_HDR) $(PROBECO)
	@mkdir -p $(dir $@)
	$(CXX) -O2 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wextra -I$(ROCM)/include \
	  -DGPUMON_PROBE_HSACO='"$(abspath $(PROBECO))"' -c $< -o $@
$(PROBELIB): build/obj/plugins/probe_plugin.o build/obj/plugins/probe_hsa.o build/obj/hip/kernels.o build/obj/hip/burn16.o \
             build/obj/hip/burn_dtypes.o
	@mkdir -p lib
	$(HIPCC) --offload-arch=$(GPUMON_ARCH) -shared -fPIC $^ -Wl,-soname,libgpumon_probe.so \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lhsa-runtime64 -o $@

# gpumon._pmc: Python view of the PMC plugin (linked, rpath $ORIGIN/../lib).
PMCEXT := gpumon/_pmc$(EXT)
pmc: $(PMCEXT)
$(PMCEXT): csrc/pmc/pmc_module.cpp csrc/plugins/ondevice_abi.h $(PMCLIB)
	$(CXX) -O2 -std=c++17 -fPIC -shared -fvisibility=hidden -I$(PYINC) -I$(PYBIND) $< \
	  -Llib -lgpumon_pmc -Wl,-rpath,'$$ORIGIN/../lib' -o $@

# Fake libamd_smi (CPU tests of the real amdsmi backend through the dlopen table).
FAKESMI := build/fakes/libfake_amd_smi.so
FAKERSMI := build/fakes/libfake_rocm_smi.so
FAKEOND := build/fakes/ondevice/libgpumon_pmc.so build/fakes/ondevice/libgpumon_probe.so \
           build/fakes/ondevice/gpumon-ondevice-helper
fakes: $(FAKESMI) $(FAKERSMI) $(FAKEOND)
build/fakes/ondevice/gpumon-ondevice-helper: csrc/plugins/ondevice_helper_main.cpp csrc/plugins/ondevice_helper_proto.h \
                                        build/fakes/ondevice/libgpumon_pmc.so
	$(CXX) -O1 -std=c++17 $< -Lbuild/fakes/ondevice -lgpumon_pmc -ldl -Wl,-rpath,'$$ORIGIN' -o $@
build/fakes/ondevice/%.so: csrc/fakes/fake_ondevice.cpp csrc/plugins/ondevice_abi.h
	@mkdir -p $(dir $@)
	$(CXX) -O1 -std=c++17 -fPIC -shared $< -o $@ -lpthread
$(FAKESMI): csrc/fakes/fake_amd_smi.cpp csrc/fakes/fake_metrics.h
	@mkdir -p $(dir $@)
	$(CXX) -O1 -std=c++17 -fPIC -shared -I$(ROCM)/include $< -o $@
$(FAKERSMI): csrc/fakes/fake_rocm_smi.cpp csrc/fakes/fake_metrics.h
	@mkdir -p $(dir $@)
	$(CXX) -O1 -std=c++17 -fPIC -shared -I$(ROCM)/include $< -o $@
