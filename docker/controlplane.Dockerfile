# Control plane image (operator, scheduler, gpupartitioner, webhooks, metricsexporter).
# Pure Python: no ROCm, no torch.  Referenced by config/ as ghcr.io/nos-amd/nos-amd.
FROM python:3.10-slim AS build
WORKDIR /src
COPY pyproject.toml README.md ./
COPY nos_amd ./nos_amd
RUN pip wheel --no-deps -w /wheels . && \
    pip wheel -w /wheels "pydantic>=2" pyyaml grpcio protobuf prometheus_client

FROM python:3.10-slim
RUN useradd -u 65532 -M nonroot
COPY --from=build /wheels /wheels
RUN pip install --no-cache-dir /wheels/*.whl && rm -rf /wheels
USER 65532:65532
ENTRYPOINT ["python", "-m"]
CMD ["nos_amd.cmd.operator", "--help"]
