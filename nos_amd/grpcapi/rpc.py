"""Minimal generic gRPC plumbing over the descriptor-built APIs of
:mod:`nos_amd.grpcapi.protos` (no generated stubs)."""
from __future__ import annotations

import os
from pathlib import Path

import grpc


def handler(api, service: str, impl) -> grpc.GenericRpcHandler:
    """Route ``/<pkg>.<service>/<Method>`` to ``impl.<Method>(request, context)``."""
    methods = {}
    for name, inp, out, streaming in api.services[service]:
        fn = getattr(impl, name)
        req_cls, resp_cls = getattr(api, inp), getattr(api, out)
        make = grpc.unary_stream_rpc_method_handler if streaming else grpc.unary_unary_rpc_method_handler
        methods[name] = make(fn, request_deserializer=req_cls.FromString,
                             response_serializer=resp_cls.SerializeToString)
    return grpc.method_handlers_generic_handler(f"{api.package}.{service}", methods)


class Stub:
    """``stub.Method(request, timeout=...)`` for every method of a service."""

    def __init__(self, channel: grpc.Channel, api, service: str):
        for name, inp, out, streaming in api.services[service]:
            factory = channel.unary_stream if streaming else channel.unary_unary
            setattr(self, name, factory(api.method_path(service, name),
                                        request_serializer=getattr(api, inp).SerializeToString,
                                        response_deserializer=getattr(api, out).FromString))


def unix_target(path: str | Path) -> str:
    return f"unix://{os.path.abspath(str(path))}"


def serve_unix(path: str | Path, handlers: list[grpc.GenericRpcHandler], max_workers: int = 8) -> grpc.Server:
    from concurrent import futures

    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    if p.exists():
        p.unlink()
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
    for h in handlers:
        server.add_generic_rpc_handlers((h,))
    server.add_insecure_port(unix_target(p))
    server.start()
    return server
