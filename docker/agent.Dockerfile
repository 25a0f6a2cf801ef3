# Node image (partition agent, gpuagent + slice prober, device plugin).
# ROCm + PyTorch base: the gpuagent runs the gfx950 probe kernels, the partition
# agent dlopens libamd_smi through libnos_amdsmi.  Referenced by config/ as
# ghcr.io/nos-amd/nos-amd-rocm.  Runs privileged with /dev/kfd, /dev/dri, the
# kubelet pod-resources socket and the device-plugin socket directory mounted.
ARG BASE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${BASE}
ENV PYTORCH_ROCM_ARCH=gfx950 NOS_AMD_ARCH=gfx950 HSA_ENABLE_IPC_MODE_LEGACY=0
WORKDIR /opt/nos-amd
COPY pyproject.toml README.md CMakeLists.txt ./
COPY csrc ./csrc
COPY nos_amd ./nos_amd
# in-tree native build (hipcc cross-compiles gfx950 without a GPU)
RUN python -m nos_amd._native.build -j 16 && \
    pip install --no-cache-dir --no-deps . && \
    pip install --no-cache-dir "pydantic>=2" pyyaml grpcio protobuf prometheus_client
ENTRYPOINT ["python", "-m"]
CMD ["nos_amd.cmd.gpuagent", "--help"]
