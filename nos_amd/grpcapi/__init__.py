"""gRPC APIs of the kubelet (device plugin v1beta1, PodResources v1)."""
