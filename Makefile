# kdl build / test / deploy entry points (the reference's Makefile:16-69 has
# test, manager, manifests, docker-build; same verbs here).
PY ?= python
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: all build native native-asan test test-gpu bench manifests docker-build clean

all: build

build:            ## compile every HIP kernel for gfx950 + the native runtime, in-tree
	$(PY) -m kubedl_amd.ops.build

native:           ## only the C++ runtime (spawner, GPU best-fit) -> kubedl_amd/_native.so
	$(PY) -m kubedl_amd.ops.build --native-only

native-asan:      ## C++ runtime with -fsanitize=address,undefined + its stress run (host only)
	$(PY) -m kubedl_amd.ops.build --native-asan
	KDL_NATIVE_SO=build/kdl_ext/asan/_native.so KDL_ZYGOTE=0 \
	LD_PRELOAD=$$(gcc -print-file-name=libasan.so) \
	ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1 \
	UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
	$(PY) scripts/native_stress.py

test:             ## CPU suite (what CI runs)
	$(PY) -m pytest tests -q -m "not gpu" --timeout=300

test-gpu:         ## GPU suite on an MI355X
	$(PY) -m pytest tests -q -m gpu --timeout=600

bench:            ## headline ResNet-50 bf16 DDP bench, 1 GPU
	$(PY) bench.py

manifests:        ## CRDs generated from kubedl_amd/api/kinds.py
	$(PY) -m kubedl_amd.api.crd config/crd/bases

docker-build:
	docker build -t kdl:latest .

clean:
	rm -rf build kubedl_amd/_C.so kubedl_amd/_native.so
