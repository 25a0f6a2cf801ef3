"""nos_amd.scheduler."""
