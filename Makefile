# Build for the MI355X (gfx950) framework.
#   make -j8            -> slate_d35_amd/libslate_amd.so + slate_d35_amd/_slate*.so
# Device code: hipcc --offload-arch=gfx950 (only target).  Host code: g++ + OpenMP.
ROCM      ?= /opt/rocm
ARCH      ?= gfx950
PYTHON    ?= python3
BUILD     := build/obj
PKG       := slate_d35_amd

HIPCC     := $(ROCM)/bin/hipcc
CXX       := g++
PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
PY_EXT    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")

INC       := -Icsrc/include -Icsrc/kernels -I$(ROCM)/include
DEFS      := -D__HIP_PLATFORM_AMD__ -DSLATE_AMD_VERSION=\"2026.10.0\"
CXXFLAGS  := -std=c++17 -O3 -fPIC -fopenmp -march=x86-64-v3 -fcx-fortran-rules -Wall -Wno-unused-function -Wno-sign-compare $(INC) $(DEFS)
HIPFLAGS  := -std=c++17 -O3 -fPIC --offload-arch=$(ARCH) -Wno-unused-result $(INC) $(DEFS)
LDLIBS    := -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lrccl -fopenmp

HIP_SRC   := $(wildcard csrc/kernels/*.hip)
CC_SRC    := $(wildcard csrc/src/*.cc)
HIP_OBJ   := $(patsubst csrc/kernels/%.hip,$(BUILD)/k_%.o,$(HIP_SRC))
CC_OBJ    := $(patsubst csrc/src/%.cc,$(BUILD)/s_%.o,$(CC_SRC))
HDRS      := $(wildcard csrc/include/slate_amd/*.hh) $(wildcard csrc/kernels/*.hh) $(wildcard csrc/src/*.hh) $(wildcard csrc/python/*.hh)

LIB       := $(PKG)/libslate_amd.so
PYMOD     := $(PKG)/_slate$(PY_EXT)
TESTER    := bin/slate_tester
LAPACK_API    := $(PKG)/libslate_lapack_api.so
SCALAPACK_API := $(PKG)/libslate_scalapack_api.so

all: $(LIB) $(PYMOD) $(LAPACK_API) $(SCALAPACK_API)

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/k_%.o: csrc/kernels/%.hip csrc/kernels/*.hh | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/s_%.o: csrc/src/%.cc $(HDRS) | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJ) $(CC_OBJ)
	$(CXX) -shared -o $@ $^ $(LDLIBS)

$(BUILD)/bind.o: csrc/python/bind.cc $(HDRS) | $(BUILD)
	$(CXX) $(CXXFLAGS) -I$(PY_INC) -I$(PYBIND_INC) -fvisibility=hidden -c $< -o $@

$(PYMOD): $(BUILD)/bind.o $(LIB)
	$(CXX) -shared -o $@ $(BUILD)/bind.o -L$(PKG) -lslate_amd -Wl,-rpath,'$$ORIGIN' $(LDLIBS)

$(BUILD)/api_%.o: csrc/api/%.cc $(HDRS) | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LAPACK_API): $(BUILD)/api_lapack_api.o $(LIB)
	$(CXX) -shared -o $@ $(BUILD)/api_lapack_api.o -L$(PKG) -lslate_amd -Wl,-rpath,'$$ORIGIN' $(LDLIBS)

$(SCALAPACK_API): $(BUILD)/api_scalapack_api.o $(LIB)
	$(CXX) -shared -o $@ $(BUILD)/api_scalapack_api.o -L$(PKG) -lslate_amd -Wl,-rpath,'$$ORIGIN' $(LDLIBS)

tester: $(TESTER)
# native tester (reference test/tester); like the examples it only depends on
# its source, so a tree without build/obj does not rebuild the library
$(TESTER): csrc/tools/tester.cc $(wildcard csrc/include/slate_amd/*.hh)
	@mkdir -p bin
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(PKG) -lslate_amd -Wl,-rpath,'$$ORIGIN/../$(PKG)' $(LDLIBS)

# C++ examples (reference examples/ex01-ex15), linked against the library
EX_SRC    := $(wildcard examples/cpp/ex*.cc)
# Binaries go to examples/bin (shipped to GPU boxes with the tree); they only
# depend on their sources and the public headers (inline classes such as
# MatrixStorage) so a tree without build/obj does not rebuild the library.
EX_BIN    := $(patsubst examples/cpp/%.cc,examples/bin/%,$(EX_SRC))
examples: $(EX_BIN)
PUB_HDR   := $(wildcard csrc/include/slate_amd/*.hh)
examples/bin/%: examples/cpp/%.cc examples/cpp/util.hh $(PUB_HDR)
	@mkdir -p examples/bin
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(PKG) -lslate_amd -Wl,-rpath,'$$ORIGIN/../../$(PKG)' $(LDLIBS)

# ThreadSanitizer CPU build of the threaded runtime (in-process ranks,
# ThreadComm, scheduler lanes): every host source instrumented, the device
# objects linked unchanged; bin/tsan_check runs on the host target.
#   make tsan && TSAN_OPTIONS=halt_on_error=1 OMP_NUM_THREADS=1 bin/tsan_check
TSAN_BUILD := build/tsan
TSAN_FLAGS := -std=c++17 -O1 -g -fPIC -fsanitize=thread -fno-omit-frame-pointer -fopenmp -march=x86-64-v3 \
              -fcx-fortran-rules -Wno-unused-function -Wno-sign-compare $(INC) $(DEFS)
TSAN_OBJ  := $(patsubst csrc/src/%.cc,$(TSAN_BUILD)/s_%.o,$(CC_SRC))
$(TSAN_BUILD)/s_%.o: csrc/src/%.cc $(HDRS)
	@mkdir -p $(TSAN_BUILD)
	$(CXX) $(TSAN_FLAGS) -c $< -o $@
bin/tsan_check: csrc/tools/tsan_check.cc $(TSAN_OBJ) $(HIP_OBJ)
	@mkdir -p bin
	$(CXX) $(TSAN_FLAGS) $< $(TSAN_OBJ) $(HIP_OBJ) -o $@ $(LDLIBS)
tsan: bin/tsan_check

clean:
	rm -rf build $(LIB) $(PYMOD) $(LAPACK_API) $(SCALAPACK_API)

.PHONY: all clean tester examples tsan
