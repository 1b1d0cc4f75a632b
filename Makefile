# nos-mi355x developer targets. CPU-only targets run anywhere; *-gpu targets need an MI355X.
PYTHON ?= python3
IMG ?= ghcr.io/walkai/nos-mi355x:0.1.0
CLIENT_IMG ?= ghcr.io/walkai/nos-mi355x-client:0.1.0
NAMESPACE ?= nos-system

.PHONY: all native test test-gpu lint sanitize helm-docs bench bench-8 smoke simulate devcluster kbench docker-build docker-push \
        deploy undeploy install-crds helm-install helm-uninstall kind-up clean

all: native test

native:            ## compile every HIP/C++ library for gfx950 into walkai_nos_amd/_native
	$(PYTHON) -m walkai_nos_amd.ops.build

test: native       ## CPU test suite (multi-process parts use gloo)
	$(PYTHON) -m pytest tests/ -x -q -m "not gpu"

test-gpu: native   ## GPU test suite (MI355X)
	$(PYTHON) -m pytest tests/ -x -q -m gpu

lint:
	$(PYTHON) hack/lint.py

sanitize:          ## host-code sanitizers (ASan+UBSan, TSan) over the HBM-limit shim's self-test
	$(PYTHON) -m pytest tests/test_native_sanitizers.py -q

bench: native      ## flagship benchmark, 1 GPU
	$(PYTHON) bench.py

bench-8: native    ## flagship benchmark, 8 GPUs of one node (one rank per GPU over RCCL)
	$(PYTHON) -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
	  --master-port 29511 bench.py --gpus 8

smoke: native
	$(PYTHON) -c "import __graft_entry__ as g; g.build(); g.smoke()"

kbench: native     ## per-slice kernel microbenchmark (attention / GEMM / LayerNorm on 256..32 CUs)
	$(PYTHON) tools/kbench.py

simulate:          ## in-memory cluster simulation of the control plane (no GPU)
	$(PYTHON) -m walkai_nos_amd.cmd.simulate --gpus 8 --epochs 50

devcluster:        ## the partitioner and partition agents as local processes over a REST API server (no Kubernetes)
	$(PYTHON) -m walkai_nos_amd.cmd.devcluster --nodes 2 --gpus 1 --demo

docker-build:
	docker build -f docker/Dockerfile -t $(IMG) .
	docker build -f docker/Dockerfile.client -t $(CLIENT_IMG) .

docker-push:
	docker push $(IMG)
	docker push $(CLIENT_IMG)

install-crds:
	kubectl apply -k config/crd

deploy:            ## plain manifests (kustomize)
	kubectl apply -k config/default

undeploy:
	kubectl delete -k config/default --ignore-not-found

helm-install:
	helm upgrade --install nos helm-charts/nos -n $(NAMESPACE) --create-namespace

helm-uninstall:
	helm uninstall nos -n $(NAMESPACE)

helm-docs:         ## regenerate helm-charts/nos/README.md from values.yaml's `# --` comments
	$(PYTHON) hack/helm_docs.py

kind-up:
	kind create cluster --config hack/kind/cluster.yaml

clean:
	rm -rf walkai_nos_amd/_native/*.so .pytest_cache
