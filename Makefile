# Developer task runner (the reference's Justfile targets, Justfile:5-61,
# mapped onto the CMake/pytest tree of this repository).
#
#   make build            native tree: tunnel, tunnel-signal, tunnel-mock, tunnel-loadgen, _native
#   make build-ops        HIP kernels for gfx950 (p2p_llm_tunnel_amd/ops/_hip_ops.so)
#   make test             CPU test-suite (pytest -m "not gpu") + native unit tests
#   make test-unit        native C++ unit tests only
#   make test-local       curl end-to-end through a local signal server
#   make test-public      same through the public signal server
#   make test-gpu         GPU tests (needs a HIP device)
#   make sanitize         ASan/UBSan build of the host tree + native tests
#   make tsan             ThreadSanitizer build + native tests
#   make bench            headline benchmark (bench.py) on this host
#   make serve ROOM=r UPSTREAM=http://127.0.0.1:11434
#   make proxy ROOM=r [LISTEN=127.0.0.1:8000]
#   make signal [PORT=8787]
#   make docker-signal    container image for the signal server (deploy/)
#   make deploy-signal    deploy the signal server to Fly.io (deploy/fly.toml; needs flyctl)
#   make signal-status    Fly.io status of the signal server app
#   make signal-logs      Fly.io logs of the signal server app
#   make clean

BUILD ?= build
JOBS ?= 8
PY ?= python3
PORT ?= 8787
LISTEN ?= 127.0.0.1:8000
SIGNAL_FLAG := $(if $(SIGNAL),--signal $(SIGNAL),)

.PHONY: build build-tunnel build-signal build-ops test test-unit test-local test-public test-gpu \
        sanitize tsan bench serve proxy signal docker-signal deploy-signal signal-status signal-logs clean

build:
	cmake -S . -B $(BUILD) -G Ninja -DCMAKE_BUILD_TYPE=Release
	cmake --build $(BUILD) -j $(JOBS)

build-tunnel: build
build-signal: build

build-ops:
	$(PY) -m p2p_llm_tunnel_amd.ops.build

test: build
	$(BUILD)/bin/native_tests
	$(PY) -m pytest tests -x -q -m "not gpu"

test-unit: build
	$(BUILD)/bin/native_tests

test-local: build
	scripts/e2e.sh

test-public: build
	scripts/e2e.sh --public

test-gpu: build build-ops
	$(PY) -m pytest tests -x -q -m gpu

sanitize:
	cmake -S . -B $(BUILD)-asan -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DP2PT_SANITIZE=ON
	cmake --build $(BUILD)-asan -j $(JOBS)
	$(BUILD)-asan/bin/native_tests

tsan:
	cmake -S . -B $(BUILD)-tsan -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DP2PT_TSAN=ON
	cmake --build $(BUILD)-tsan -j $(JOBS)
	$(BUILD)-tsan/bin/native_tests

bench: build
	$(PY) bench.py

serve: build
	@test -n "$(ROOM)" -a -n "$(UPSTREAM)" || (echo "usage: make serve ROOM=<room> UPSTREAM=<url>"; exit 2)
	$(BUILD)/bin/tunnel serve $(SIGNAL_FLAG) --room $(ROOM) --upstream $(UPSTREAM)

proxy: build
	@test -n "$(ROOM)" || (echo "usage: make proxy ROOM=<room> [LISTEN=host:port]"; exit 2)
	$(BUILD)/bin/tunnel proxy $(SIGNAL_FLAG) --room $(ROOM) --listen $(LISTEN)

signal: build
	$(BUILD)/bin/tunnel-signal --port $(PORT)

docker-signal:
	docker build -f deploy/Dockerfile.signal -t p2pt-signal .

FLY ?= fly
FLY_CONFIG := deploy/fly.toml

deploy-signal:
	$(FLY) deploy --config $(FLY_CONFIG) --dockerfile deploy/Dockerfile.signal .

signal-status:
	$(FLY) status --config $(FLY_CONFIG)

signal-logs:
	$(FLY) logs --config $(FLY_CONFIG)

clean:
	rm -rf $(BUILD) $(BUILD)-asan $(BUILD)-tsan
	rm -f p2p_llm_tunnel_amd/_native*.so p2p_llm_tunnel_amd/ops/_hip_ops.so
