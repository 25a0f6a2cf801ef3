"""Kubernetes REST path conventions shared by the HTTP front end of the
in-process API server (:mod:`nos_amd.sim.http`) and the REST client
(:mod:`nos_amd.kube.client`).

``/api/v1[/namespaces/<ns>]/<plural>[/<name>[/<subresource>]]`` for the core
group, ``/apis/<group>/<version>/...`` for the others.
"""
from __future__ import annotations

from dataclasses import dataclass
from urllib.parse import quote


@dataclass(frozen=True)
class Route:
    api_version: str
    plural: str
    namespace: str | None
    name: str | None
    subresource: str | None


def base_path(api_version: str) -> str:
    return "/api/v1" if api_version == "v1" else f"/apis/{api_version}"


def path_for(api_version: str, plural: str, namespaced: bool, namespace: str | None = None,
             name: str | None = None, subresource: str | None = None) -> str:
    p = base_path(api_version)
    if namespaced and namespace:
        p += f"/namespaces/{quote(namespace)}"
    p += f"/{plural}"
    if name:
        p += f"/{quote(name)}"
        if subresource:
            p += f"/{subresource}"
    return p


def parse_path(path: str, known_plurals: set[str]) -> Route | None:
    parts = [p for p in path.split("?")[0].split("/") if p]
    if not parts:
        return None
    if parts[0] == "api" and len(parts) >= 2:
        api_version, rest = parts[1], parts[2:]
    elif parts[0] == "apis" and len(parts) >= 3:
        api_version, rest = f"{parts[1]}/{parts[2]}", parts[3:]
    else:
        return None
    ns = None
    if len(rest) >= 3 and rest[0] == "namespaces" and rest[2] in known_plurals:
        ns, rest = rest[1], rest[2:]
    if not rest:
        return None
    plural = rest[0]
    name = rest[1] if len(rest) > 1 else None
    sub = rest[2] if len(rest) > 2 else None
    return Route(api_version, plural, ns, name, sub)


def status_body(code: int, reason: str, message: str) -> dict:
    return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "message": message,
            "reason": reason, "code": code}
