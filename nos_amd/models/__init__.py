"""Tenant workloads run inside GPU slices."""
from .yolos import YolosConfig, YolosDetector, GraphedTenant, make_demo_input  # noqa: F401
