"""nos_amd.kube."""
