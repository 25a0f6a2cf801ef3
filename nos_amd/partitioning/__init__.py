"""nos_amd.partitioning."""
