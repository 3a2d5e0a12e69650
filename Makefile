# gpupool — developer entry points. Mirrors the reference's kubebuilder workflow
# (`make manifests generate`, `install`, `run`, `docker-build docker-push`, `deploy`;
# /root/reference/README.md:159, :256, :261, :300-301) for an MI355X-native operator.
PY      ?= python3
GPUCTL  := bin/gpuctl
IMG     ?= gpupool:dev
JOBS    ?= 8

.PHONY: all manifests generate native build test test-gpu sanitize install run run-manager bench smoke \
        docker-build docker-push deploy undeploy fixtures clean

all: manifests native

## manifests / generate: CRDs, RBAC and the C++ constants header from gpupool/api/schema.py
manifests generate:
	$(PY) scripts/gen_manifests.py

fixtures:
	$(PY) scripts/gen_fake_fixture.py

## native / build: C++17 control plane + gfx950 HIP probe (hipcc --offload-arch=gfx950)
native build:
	$(MAKE) -C native all -j$(JOBS)

## test: CPU suite (apiserver-sim, C++ unit tests incl. ASan/TSan, integration, property)
test: native
	$(PY) -m pytest tests -q -m "not gpu"

## test-gpu: hardware tier (needs an MI355X)
test-gpu: native
	$(PY) -m pytest tests -q -m gpu

sanitize:
	$(MAKE) -C native SAN=asan host -j$(JOBS) && build/native-asan/gpupool_tests
	$(MAKE) -C native SAN=tsan host -j$(JOBS) && build/native-tsan/gpupool_tests

## install: CRDs into the apiserver selected by the current gpuctl context
install:
	$(GPUCTL) install

## run: local control plane in the foreground (BACKEND=fake|amdsmi NODES=1)
BACKEND ?= fake
NODES   ?= 1
run: native
	$(PY) scripts/run_local.py --backend $(BACKEND) --nodes $(NODES)

## run-manager: only the operator, against the cluster of the current kubeconfig / in-cluster
## config (the reference's `make run`, README.md:259-263). CLOUD=fake|azure-arm selects the
## AzureVmPool backend; KINDS the reconcilers.
CLOUD ?= fake
KINDS ?= mi355x,azure,job
run-manager: native
	build/native/gpupool-manager --cloud $(CLOUD) --kinds $(KINDS)

## bench: headline metric (p50 reconcile-to-Ready + readyReplicas accuracy)
GPUS ?= 1
bench: native
	$(PY) bench.py --gpus $(GPUS) --steps 10 --warmup 2

smoke: native
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

## docker-build / docker-push / deploy: in-cluster deployment (no docker or cluster here)
docker-build:
	@command -v docker >/dev/null || { echo "docker not available; Dockerfiles: deploy/docker/"; exit 1; }
	docker build -f deploy/docker/Dockerfile.manager -t $(IMG)-manager .
	docker build -f deploy/docker/Dockerfile.agent -t $(IMG)-agent .

docker-push:
	docker push $(IMG)-manager && docker push $(IMG)-agent

deploy: manifests
	$(GPUCTL) apply -f config/crd
	$(GPUCTL) apply -f config/manager   # creates the gpupool-system namespace first
	$(GPUCTL) apply -f config/rbac
	$(GPUCTL) apply -f config/agent

undeploy:
	$(GPUCTL) delete -f config/agent; $(GPUCTL) delete -f config/rbac; $(GPUCTL) delete -f config/manager

clean:
	rm -rf build
