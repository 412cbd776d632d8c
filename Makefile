# Build of the native core for gfx950 (MI355X).
#   make -j8            -> bin/bfs  and  distributed_cuda_bfs_amd/_dbfs_native*.so
# Device code: hipcc --offload-arch=gfx950.  Host code: g++ against the ROCm
# 7.2 HIP runtime headers.  Artefacts are in-tree (git-ignored) so they travel
# with the repo snapshot to the GPU box.

ROCM      ?= /opt/rocm
ARCH      ?= gfx950
PYTHON    ?= python3
HIPCC     := $(ROCM)/bin/hipcc
CXX       := g++
BUILD     := build
PKG       := distributed_cuda_bfs_amd

PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
EXT_SUFFIX:= $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

COMMON    := -O3 -std=c++17 -fPIC -Icsrc/include -Wall -Wno-unused-result
HOSTFLAGS := $(COMMON) -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include $(EXTRA_HIPFLAGS)
HIPFLAGS  := $(COMMON) --offload-arch=$(ARCH) -munsafe-fp-atomics $(EXTRA_HIPFLAGS)
LDLIBS    := -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib -lpthread

HOST_SRC  := csrc/graph/io.cpp csrc/graph/csr.cpp csrc/backend/cpu_backend.cpp \
             csrc/backend/hip_backend.cpp csrc/comm/comm.cpp csrc/comm/nccl_comm.cpp \
             csrc/comm/tcp_bootstrap.cpp csrc/comm/peer_comm.cpp csrc/comm/replay_comm.cpp csrc/engine/engine.cpp csrc/engine/device_loop.cpp csrc/graph/shard_reader.cpp
HIP_SRC   := csrc/kernels/bfs_kernels.hip csrc/kernels/td_kernels.hip csrc/kernels/bu_kernels.hip csrc/kernels/graph_kernels.hip csrc/kernels/ref_kernels.hip \
             csrc/kernels/graph_sort.hip csrc/kernels/peer_kernels.hip

HOST_OBJ  := $(patsubst csrc/%.cpp,$(BUILD)/%.o,$(HOST_SRC))
HIP_OBJ   := $(patsubst csrc/%.hip,$(BUILD)/%.o,$(HIP_SRC))
CORE_LIB  := $(BUILD)/libdbfs_core.a
PYMOD     := $(PKG)/_dbfs_native$(EXT_SUFFIX)
CLI       := bin/bfs

HEADERS   := $(wildcard csrc/include/dbfs/*.hpp) $(wildcard csrc/kernels/*.hpp) $(wildcard csrc/engine/*.hpp)

.PHONY: all clean lib asan checked
all: $(CLI) $(PYMOD) bin/bfs_checked
lib: $(CORE_LIB)

# Device-checked build: bin/bfs_checked, the traversal kernels
# built with -DDBFS_CHECKED (work-list, owner-list and vertex-id bounds
# verified on the device; the first violation fails the run on the host,
# HipBackend::take_device_check).  Host code and the other kernels unchanged.
CHECKED_BUILD := build-checked
CHECKED_SRC   := csrc/kernels/bfs_kernels.hip csrc/kernels/td_kernels.hip csrc/kernels/bu_kernels.hip
CHECKED_OBJ   := $(patsubst csrc/%.hip,$(CHECKED_BUILD)/%.o,$(CHECKED_SRC))
checked: bin/bfs_checked
$(CHECKED_BUILD)/%.o: csrc/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DDBFS_CHECKED -c $< -o $@
bin/bfs_checked: $(BUILD)/cli/main.o $(HOST_OBJ) $(CHECKED_OBJ) $(filter-out $(patsubst csrc/%.hip,$(BUILD)/%.o,$(CHECKED_SRC)),$(HIP_OBJ))
	@mkdir -p bin
	$(HIPCC) --offload-arch=$(ARCH) $^ -o $@ $(LDLIBS)

# Host sanitizers: bin/bfs_asan, every host translation unit
# built with AddressSanitizer + UBSan (g++), device code unchanged.  GPU
# sanitizers are not available on this pool: run it with --cpu.
ASAN_BUILD := build-asan
ASANFLAGS  := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
              -std=c++17 -Icsrc/include -Wall -Wno-unused-result -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
ASAN_OBJ   := $(patsubst csrc/%.cpp,$(ASAN_BUILD)/%.o,$(HOST_SRC) csrc/cli/main.cpp)
asan: bin/bfs_asan
$(ASAN_BUILD)/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(ASANFLAGS) -c $< -o $@
bin/bfs_asan: $(ASAN_OBJ) $(HIP_OBJ)
	@mkdir -p bin
	$(CXX) -fsanitize=address,undefined $^ -o $@ $(LDLIBS)

$(BUILD)/%.o: csrc/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(BUILD)/%.o: csrc/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(CORE_LIB): $(HOST_OBJ) $(HIP_OBJ)
	@rm -f $@
	ar rcs $@ $^

$(BUILD)/cli/main.o: csrc/cli/main.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(CLI): $(BUILD)/cli/main.o $(CORE_LIB)
	@mkdir -p bin
	$(HIPCC) --offload-arch=$(ARCH) $^ -o $@ $(LDLIBS)

$(BUILD)/python/module.o: csrc/python/module.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -fvisibility=hidden -I$(PY_INC) -I$(PYBIND_INC) -c $< -o $@

$(PYMOD): $(BUILD)/python/module.o $(CORE_LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared $^ -o $@ $(LDLIBS)

clean:
	rm -rf $(BUILD) $(ASAN_BUILD) $(CHECKED_BUILD) bin $(PKG)/_dbfs_native*.so
