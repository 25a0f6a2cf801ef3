"""nos_amd.parallel."""
