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
HOSTFLAGS := $(COMMON) -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include
HIPFLAGS  := $(COMMON) --offload-arch=$(ARCH) -munsafe-fp-atomics
LDLIBS    := -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -Wl,-rpath,$(ROCM)/lib -lpthread

HOST_SRC  := csrc/graph/io.cpp csrc/graph/csr.cpp csrc/backend/cpu_backend.cpp \
             csrc/backend/hip_backend.cpp csrc/comm/comm.cpp csrc/comm/nccl_comm.cpp \
             csrc/comm/tcp_bootstrap.cpp csrc/engine/engine.cpp
HIP_SRC   := csrc/kernels/bfs_kernels.hip csrc/kernels/graph_kernels.hip csrc/kernels/ref_kernels.hip \
             csrc/kernels/graph_sort.hip

HOST_OBJ  := $(patsubst csrc/%.cpp,$(BUILD)/%.o,$(HOST_SRC))
HIP_OBJ   := $(patsubst csrc/%.hip,$(BUILD)/%.o,$(HIP_SRC))
CORE_LIB  := $(BUILD)/libdbfs_core.a
PYMOD     := $(PKG)/_dbfs_native$(EXT_SUFFIX)
CLI       := bin/bfs

HEADERS   := $(wildcard csrc/include/dbfs/*.hpp) $(wildcard csrc/kernels/*.hpp)

.PHONY: all clean lib
all: $(CLI) $(PYMOD)
lib: $(CORE_LIB)

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
	rm -rf $(BUILD) bin $(PKG)/_dbfs_native*.so
