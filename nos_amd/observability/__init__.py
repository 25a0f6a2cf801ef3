"""nos_amd.observability."""
