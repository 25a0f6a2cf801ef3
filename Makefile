# nos-amd developer targets.  Everything runs without a cluster: the control plane is
# exercised against the in-process API server / kubelet simulator (nos_amd.sim).
PY      ?= python
ARCH    ?= gfx950
JOBS    ?= 8
IMG_TAG ?= 0.1.0
REG     ?= ghcr.io/nos-amd

.PHONY: all build build-cmake test test-gpu test-sanitizers lint manifests bench smoke docker-build clean help

all: build test

help:
	@grep -E '^[a-z-]+:.*##' $(MAKEFILE_LIST) | sed 's/:.*##/\t/'

build: ## compile libnos_hip.so (gfx950) and libnos_amdsmi.so in-tree
	NOS_AMD_ARCH=$(ARCH) $(PY) -m nos_amd._native.build -j $(JOBS)

build-cmake: ## same libraries through CMake + Ninja
	cmake -S . -B build/cmake -G Ninja -DNOS_GPU_ARCH=$(ARCH) -DCMAKE_HIP_COMPILER=/opt/rocm/llvm/bin/clang++
	cmake --build build/cmake -j $(JOBS)

test: build ## CPU test suite (simulator, scheduler, planner, agents, gloo collectives)
	$(PY) -m pytest tests/ -x -q -m "not gpu"

test-gpu: build ## kernel numerics + CU-mask tests on an MI355X
	$(PY) -m pytest tests/ -x -q -m gpu

test-sanitizers: ## ThreadSanitizer and ASan/UBSan stress of the amd-smi library
	$(PY) -m pytest tests/test_native_sanitizers.py -q

lint: ## byte-compile everything; ruff when installed
	$(PY) -m compileall -q nos_amd tests tools bench.py __graft_entry__.py
	@if command -v ruff >/dev/null; then ruff check nos_amd tests; else echo "ruff not installed: skipped"; fi

manifests: ## regenerate config/ (CRDs, RBAC, deployments, daemonsets, configs)
	$(PY) -m nos_amd.cmd.manifests --out config

bench: build ## flagship benchmark on 1 GPU
	$(PY) bench.py

smoke: build
	$(PY) -c "import __graft_entry__ as g; g.build(); g.smoke()"

docker-build: ## control-plane and node-agent images
	docker build -f docker/controlplane.Dockerfile -t $(REG)/nos-amd:$(IMG_TAG) .
	docker build -f docker/agent.Dockerfile -t $(REG)/nos-amd-rocm:$(IMG_TAG) .

clean:
	rm -rf build nos_amd/_native/*.so
