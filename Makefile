# Convenience targets (everything also works with plain python/pytest commands).
PY ?= python3
.PHONY: build native kernels test test-gpu bench sd15-bench lint-manifests images clean
build:            ## every HIP kernel (gfx950) + native tool, in-tree
	$(PY) -c "import __graft_entry__ as g; g.build()"
kernels:
	$(PY) -m k8s_nvidia_gpus_amd.ops.build kernels
native:
	$(PY) -m k8s_nvidia_gpus_amd.ops.build native
test:             ## CPU suite (static checks, fakes, gloo, sanitizers)
	$(PY) -m pytest tests -m "not gpu" -q
test-gpu:         ## on an MI355X
	$(PY) -m pytest tests -m gpu -q
bench:            ## headline benchmark on all local GPUs (one rank per GPU)
	n=$$($(PY) -c "import torch; print(torch.cuda.device_count())"); \
	if [ $$n -gt 1 ]; then $(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $$n \
	  --master-addr 127.0.0.1 bench.py --gpus $$n; else $(PY) bench.py; fi
lint-manifests:
	$(PY) -m pytest tests/test_static_manifests.py -q
sd15-bench:       ## SD1.5 UNet pass / 512x512 30-step latency on one MI355X
	$(PY) tools/sd15_bench.py
images:
	docker build -f images/operator/Dockerfile -t ghcr.io/example-org/amd-gpu-operator:0.1.0 .
	docker build -f images/bench/Dockerfile -t ghcr.io/example-org/amd-gpu-bench:0.1.0 .
clean:
	rm -rf build native/bin k8s_nvidia_gpus_amd/ops/_lib
